"""bench.py's launch contract on CPU: `python bench.py --gpus 2` (no WORLD_SIZE) starts
torch.distributed.run with 2 ranks as a child process and relays rank 0's JSON line; every rank
checks that the launch's WORLD_SIZE equals --gpus.  The engines come from the --engine-factory test
hook (the CPU oracle, tests/bench_hooks.py), so the ranks rendezvous over gloo on 127.0.0.1 and time
the same schedule without a GPU."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, env_extra=None, timeout=300):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], cwd=REPO, env=env,
                          capture_output=True, text=True, timeout=timeout)


HOOK = ["--engine-factory", os.path.join(REPO, "tests", "bench_hooks.py") + ":oracle_lib", "--members", "64",
        "--steps", "3", "--warmup", "2", "--no-cpu-baseline"]


def test_gpus_2_spawns_two_ranks():
    p = _bench("--gpus", "2", *HOOK)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 only
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["ranks"]["processes"] == 2
    assert line["steps"] == 3 and line["warmup"] == 2 and line["value"] > 0
    assert "TEST HOOK" in line["engine"]
    # counters are the timed window's deltas: every member pings once per period (x 2 ranks, each
    # running the whole cluster through the hook)
    assert line["stats"]["pings"] == 2 * 64 * 3


def test_world_size_must_match_gpus():
    p = _bench("--gpus", "2", *HOOK, env_extra={"WORLD_SIZE": "1"})
    assert p.returncode != 0 and "WORLD_SIZE=1" in (p.stderr + p.stdout)


def test_window_traffic_only_from_the_same_window(tmp_path, monkeypatch):
    """roofline.traffic is taken from the newest committed PMC profile of the SAME window (same
    --steps / --warmup), never borrowed from a window of another length."""
    sys.path.insert(0, REPO)
    import bench
    prof = tmp_path / "profiles"
    prof.mkdir()
    for name, steps, warm, b in (("r01_quiet64k_pmc.json", 40, 10, 100.0), ("r02_quiet64k_pmc.json", 20, 5, 7.0),
                                 ("r03_quiet64k_pmc.json", 20, 5, 9.0)):
        (prof / name).write_text(json.dumps({"bench_args": {"steps": steps, "warmup": warm},
                                             "kernels": {"k_quiet_apply": {"last_launch_hbm_bytes": b},
                                                         "k_quiet_scan": {"last_launch_hbm_bytes": 1.0}}}))
    monkeypatch.setattr(bench, "REPO", str(tmp_path))
    assert bench.window_pmc_traffic("quiet", 65536, 20, 5, scanned=False) == (9.0, "profiles/r03_quiet64k_pmc.json")
    assert bench.window_pmc_traffic("quiet", 65536, 40, 10, scanned=True) == (101.0, "profiles/r01_quiet64k_pmc.json")
    t, why = bench.window_pmc_traffic("quiet", 65536, 7, 3)
    assert t is None and "not this window" in why
    # with per-launch bytes the timed window's own launch is taken, not the last (a side run's)
    (prof / "r04_quiet64k_pmc.json").write_text(json.dumps({
        "bench_args": {"steps": 20, "warmup": 5},
        "kernels": {"k_quiet_apply": {"last_launch_hbm_bytes": 50.0, "launch_hbm_bytes": [20.0, 31.0, 19.0, 50.0]}}}))
    first = {"k_quiet_apply": 1, "k_quiet_scan": 1}
    assert bench.window_pmc_traffic("quiet", 65536, 20, 5, scanned=False, first=first) == \
        (31.0, "profiles/r04_quiet64k_pmc.json")
    t, why = bench.window_pmc_traffic("quiet", 65536, 20, 5, scanned=False, first={"k_quiet_apply": 9})
    assert t is None and "the timed one is #9" in why
