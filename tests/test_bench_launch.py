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


def _profile(path, key, build, created, apply_bytes, emit_bytes=None):
    eng0 = {"k_quiet_apply": {"hbm_bytes": apply_bytes, "fetch_bytes": apply_bytes, "write_bytes": [0.0] * len(apply_bytes),
                              "us": [1.0] * len(apply_bytes)}}
    engines = [eng0, {}]
    if emit_bytes is not None:
        engines.append({"k_gossip_emit": {"hbm_bytes": emit_bytes, "fetch_bytes": emit_bytes,
                                          "write_bytes": [0.0] * len(emit_bytes), "us": [2.0] * len(emit_bytes)}})
    path.write_text(json.dumps({"bench_key": key, "build": build, "created": created, "engines": engines}))


def test_traffic_only_from_this_command_and_build(tmp_path, monkeypatch):
    """roofline.traffic comes from the per-launch PMC profile of the SAME command (bench_key) and the
    SAME build (the lib's source hash), newest by its own timestamp — never by file name order, never
    from another window, command or build — and from the timed window's own launch."""
    sys.path.insert(0, REPO)
    import bench
    prof = tmp_path / "profiles"
    prof.mkdir()
    key = {"gpus": 1, "steps": 20, "warmup": 5}
    other = {"gpus": 1, "steps": 40, "warmup": 10}
    # lexically last, but another build; a newer one of another command; the right one in the middle
    _profile(prof / "r09_quiet64k_pmc.json", key, "oldbuild", "2026-01-03T00:00:00", [5.0, 6.0, 7.0])
    _profile(prof / "r01_quiet64k_pmc.json", key, "thisbuild", "2026-01-01T00:00:00", [1.0, 2.0, 3.0])
    _profile(prof / "r02_quiet64k_pmc.json", key, "thisbuild", "2026-01-02T00:00:00", [20.0, 31.0, 19.0],
             emit_bytes=[1.0, 2.0, 4.0, 6.0])
    _profile(prof / "r03_quiet64k_pmc.json", other, "thisbuild", "2026-01-05T00:00:00", [8.0, 8.0])
    monkeypatch.setattr(bench, "REPO", str(tmp_path))
    monkeypatch.setattr(bench, "build_hash", lambda: "thisbuild")
    monkeypatch.setattr(bench, "_PROFILE", {})
    t, src, us = bench.window_pmc_traffic(key, scanned=False, first={"k_quiet_apply": 1})
    assert (t, src, us) == (31.0, "profiles/r02_quiet64k_pmc.json", 1.0)
    # the timed launch is past the profile's list: no traffic, and a reason
    t, why, _ = bench.window_pmc_traffic(key, scanned=False, first={"k_quiet_apply": 9})
    assert t is None and "no launch #9" in why
    # a scanned window needs the scan's launch too
    t, why, _ = bench.window_pmc_traffic(key, scanned=True, first={"k_quiet_apply": 1, "k_quiet_scan": 1})
    assert t is None and "k_quiet_scan" in why
    # a command nobody profiled on this build
    t, why, _ = bench.window_pmc_traffic({"gpus": 1, "steps": 7, "warmup": 3}, scanned=False, first={"k_quiet_apply": 0})
    assert t is None and "measured this command on this build" in why
    # the storm window: the mean of the last launches of the side run's engine (#2)
    w, src, n = bench.window_traffic(key, 2, ("k_gossip_emit",), 2)
    assert w["hbm"] == 5.0 and w["us"] == 2.0 and src == "profiles/r02_quiet64k_pmc.json"
    w, why, _ = bench.window_traffic(key, 2, ("k_gossip_emit",), 9)
    assert w is None and "fewer than 9 launches" in why


def test_headline_launch_index_counts_attempts():
    """k_quiet_apply is launched on every window attempt (also one that advances no tick) and once per
    local shard: the timed launch's index counts attempts x shards, not windows"""
    sys.path.insert(0, REPO)
    import bench
    # a warm-up with a failed attempt (attempts > windows) and one precomputed window
    qs0 = {"windows": 2, "attempts": 3, "precomputed": 1}
    assert bench.timed_launch_index(qs0) == {"k_quiet_apply": 3, "k_quiet_scan": 2}
    assert bench.timed_launch_index(qs0, 4) == {"k_quiet_apply": 12, "k_quiet_scan": 8}
