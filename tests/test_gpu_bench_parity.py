"""bench.py's own workloads at their own size, GPU against the threaded CPU oracle, bit-exact —
unsharded and over 8 in-process shards (BASELINE config 4's deployment plan on one GPU).

The headline (config4-lan-quiet: N = 65,536, LAN defaults, aligned timers, staggered periodic SYNC)
and the failures workload through its first kill's failure detection are run on libswimgpu.so and
on the oracle from the same schedule (bench.Schedule), and compared at checkpoints: the full member
state of sampled rows — the witness-block boundaries 1,023 / 1,024 / 2,047 / 2,048 ..., the victim
and its neighbours — (view cells, scalars, ping and remote lists in order, live gossips, collectors),
the whole canonical event stream and every counter.  The quiet run is 12 periods (120 ticks: seven
16-tick witness rebases, MembershipProtocolImpl.java:339-357,394-415 SYNCs every tick, the
exactness of the witness skip); the failures run crosses the kill at period 10 (FD SUSPECT, the
SUSPECT gossip storm, FailureDetectorImpl.java:126-171, GossipProtocolImpl.java:141-184).
"""
import os

import pytest

import bench
import oracle
import parity

pytestmark = pytest.mark.gpu

THREADS = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1)))
N = 65536
BOUNDARY_ROWS = [0, 1, 1023, 1024, 2047, 2048, 4095, 4096, 32767, 32768, 65534, 65535]


def _engines(glib, workload, periods, local_shards=1, rccl=False):
    from swimgpu import abi
    out = {}
    for k, lib in (("gpu", glib), ("oracle", oracle.lib())):
        sch = bench.Schedule(workload, N, periods)
        cfg = bench.make_config(lib)
        if k == "gpu":
            cfg.local_shards = local_shards
        if k == "gpu" and rccl:  # an RCCL engine of one rank (swim_create_shard, world 1 with an id)
            e = abi.Engine(lib, cfg, sch.capacity, N, 1, rank=0, world=1, comm_id=abi.comm_unique_id(lib))
        else:
            e = abi.Engine(lib, cfg, sch.capacity, N, 1)
        sch.setup(e)
        out[k] = (e, sch)
    oracle.set_threads(out["oracle"][0], THREADS)
    if local_shards > 1:
        assert out["gpu"][0].shard_info()["world"] == local_shards
    return out


def _run_steps(eng, members, steps, p=0):
    """advance both engines by e.step(k) for each k of `steps` (one swim_step call each, exactly as
    bench.py times them), comparing after every call; returns the last counters"""
    st = None
    for k in steps:
        for key in ("gpu", "oracle"):
            e, _ = eng[key]
            e.step(k)
        p += k
        _, st = _compare(eng, members, f"period {p} (after step({k}))")
    return st


def _compare(eng, members, where):
    g, o = eng["gpu"][0], eng["oracle"][0]
    d = parity.diff_states(parity.state_digest(o, members), parity.state_digest(g, members))
    assert not d, f"diverged by {where}:\n" + "\n".join(d)
    ea, eb = o.drain_events(), g.drain_events()
    assert not parity.diff_events(ea, eb), (where, parity.diff_events(ea, eb))
    sa, sb = o.stats(), g.stats()
    assert not parity.diff_stats(sa, sb), (where, parity.diff_stats(sa, sb))
    assert sb["capacity_errors"] == 0
    return ea, sb


@pytest.fixture(scope="module")
def glib():
    import swimgpu
    return swimgpu.load_library()


def test_headline_quiet_65536_matches_oracle(glib):
    """config4-lan-quiet exactly as bench.py runs it, 12 periods, checked after periods 1, 4, 8, 12."""
    eng = _engines(glib, "quiet", 12)
    members = BOUNDARY_ROWS + list(range(517, N, 2311))[:28]
    p = 0
    try:
        for upto in (1, 4, 8, 12):
            for k in ("gpu", "oracle"):
                e, sch = eng[k]
                sch.run(e, p, upto)
            p = upto
            _, st = _compare(eng, members, f"period {p}")
        assert st["syncs"] > 0 and st["sync_records"] > 0 and st["pings"] == N * 12
    finally:
        for e, _ in eng.values():
            e.close()


def test_failures_first_kill_65536_matches_oracle(glib):
    """The failures workload (bench.py --workload failures) through its first kill (member 17 at
    period 10) and the failure detection that follows, checked after periods 10, 11, 12, 14."""
    eng = _engines(glib, "failures", 14)
    victim = 17
    members = BOUNDARY_ROWS + [16, victim, 18] + list(range(733, N, 2729))[:24]
    p = 0
    try:
        for upto in (10, 11, 12, 14):
            for k in ("gpu", "oracle"):
                e, sch = eng[k]
                sch.run(e, p, upto)
            p = upto
            _, st = _compare(eng, members, f"period {p}")
        assert st["gossips_created"] > 0 and st["gossip_messages"] > 0  # the SUSPECT storm started
    finally:
        for e, _ in eng.values():
            e.close()


def test_headline_quiet_65536_stepped_like_bench(glib):
    """config4-lan-quiet stepped exactly as the driver's bench command times it (`bench.py --steps 20
    --warmup 5`: step(5), then ONE step(20), a 200-tick quiet window) and as the default command
    does (`--steps 40`: one 400-tick window): sampled full state, every event, every counter against
    the oracle after each call, and the windows really ran on the GPU."""
    eng = _engines(glib, "quiet", 65)
    members = BOUNDARY_ROWS + list(range(517, N, 2311))[:28]
    try:
        g = eng["gpu"][0]
        q0 = g.quiet_stats()
        st = _run_steps(eng, members, (5, 20, 40))
        q1 = g.quiet_stats()
        assert st["pings"] == N * 65 and st["syncs"] > 0
        assert q1["ticks"] - q0["ticks"] >= 600, q1  # the 200- and 400-tick calls ran as windows
    finally:
        for e, _ in eng.values():
            e.close()


@pytest.mark.parametrize("pull", [False, True], ids=["local", "pull"])
def test_config4_sharded8_65536_quiet_matches_oracle(glib, monkeypatch, pull):
    """BASELINE config 4 at its stated N = 65,536 over 8 in-process shards (the RCCL plan's exchange
    kernels; `pull`: content rows through k_pull_rows' copies as over RCCL, SWIM_EXCHANGE_PULL=1)
    against the UNSHARDED oracle, 14 periods with quiet windows on: step(2) on the per-tick chain
    (cross-shard SYNC / SYNC_ACK exchange every tick), then windows of 2 / 5 / 5 periods, each of
    which needs every shard's witness ref to agree.  Sampled full state incl. the
    shard boundaries, all events, all counters."""
    if pull:
        monkeypatch.setenv("SWIM_EXCHANGE_PULL", "1")
    eng = _engines(glib, "quiet", 14, local_shards=8)
    sz = N // 8
    members = sorted(set(BOUNDARY_ROWS + [sz - 1, sz, 3 * sz - 1, 3 * sz, 7 * sz - 1, 7 * sz] +
                         list(range(211, N, 3001))[:20]))
    try:
        g = eng["gpu"][0]
        g.set_quiet_path(False)
        st = _run_steps(eng, members, (2,))
        g.set_quiet_path(True)
        q0 = g.quiet_stats()
        st = _run_steps(eng, members, (2, 5, 5), p=2)
        q1 = g.quiet_stats()
        assert st["pings"] == N * 14 and st["syncs"] > 0
        assert q1["windows"] > q0["windows"] and q1["ticks"] - q0["ticks"] >= 100, (q0, q1)
    finally:
        for e, _ in eng.values():
            e.close()


def test_failures_sharded8_65536_first_kill_matches_oracle(glib):
    """The failures workload at N = 65,536 over 8 in-process shards through its first kill (member 17
    at period 10) and the SUSPECT storm that follows: every GOSSIP_REQ to a member of another shard
    crosses E1 (k_recv_msgs), SYNCs E2 / E3; against the unsharded oracle after periods 10, 11, 12,
    14."""
    eng = _engines(glib, "failures", 14, local_shards=8)
    sz = N // 8
    victim = 17
    members = sorted(set(BOUNDARY_ROWS + [16, victim, 18, sz - 1, sz, 5 * sz - 1, 5 * sz] +
                         list(range(733, N, 2729))[:20]))
    p = 0
    try:
        for upto in (10, 11, 12, 14):
            for k in ("gpu", "oracle"):
                e, sch = eng[k]
                sch.run(e, p, upto)
            p = upto
            _, st = _compare(eng, members, f"period {p}")
        assert st["gossips_created"] > 0 and st["gossip_messages"] > 0
    finally:
        for e, _ in eng.values():
            e.close()


def _rccl_info(g):
    """which branch of the RCCL setup ran (an IPC handle of the uncached region, or the cached
    fallback), also written to gpurun_out/rccl_exchange_info.json on the GPU box"""
    import json
    info = g.exchange_info()
    print("RCCL exchange on one GPU:", info, flush=True)
    out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
    if os.path.isdir(out):
        with open(os.path.join(out, "rccl_exchange_info.json"), "w") as f:
            json.dump(info, f)
    assert info["exchange"] and info["rccl"] and info["ipc"], info
    return info


def test_rccl_world1_quiet_65536_stepped_like_bench(glib):
    """The RCCL transport executed on hardware with one rank: swim_create_shard with a
    comm id at world 1 runs the whole exchange machinery — the IPC handle of the exchange region
    (uncached, or the cached fallback: exchange_info says which) and its ncclAllGather, a count
    ncclAllToAll per exchange, k_recv_msgs / k_pack_rows / k_recv_sync / k_pull_rows every tick, and
    the quiet windows' collectives — the refs' and the window end's allreduces of a scanned window,
    the precomputed end's 8-byte allreduce of the windows after it — on the headline workload stepped
    as bench.py times it, bit-exact against the unsharded oracle."""
    eng = _engines(glib, "quiet", 30, rccl=True)
    members = BOUNDARY_ROWS + list(range(517, N, 2311))[:28]
    try:
        g = eng["gpu"][0]
        _rccl_info(g)
        g.set_quiet_path(False)
        st = _run_steps(eng, members, (2,))  # the per-tick chain with its exchange kernels
        g.set_quiet_path(True)
        q0 = g.quiet_stats()
        st = _run_steps(eng, members, (3, 20, 5), p=2)
        q1 = g.quiet_stats()
        assert st["pings"] == N * 30 and st["syncs"] > 0
        assert q1["ticks"] - q0["ticks"] >= 250 and q1["precomputed"] - q0["precomputed"] >= 2, (q0, q1)
    finally:
        for e, _ in eng.values():
            e.close()


def test_rccl_world1_failures_first_kill_65536_matches_oracle(glib):
    """The failures workload through its first kill on the one-rank RCCL engine: the SUSPECT storm's
    gossip rounds each run E1's count all-to-all and stop all-gather, the SYNC sub-phases E2 / E3's;
    against the unsharded oracle after periods 10, 11, 12, 14."""
    eng = _engines(glib, "failures", 14, rccl=True)
    victim = 17
    members = BOUNDARY_ROWS + [16, victim, 18] + list(range(733, N, 2729))[:24]
    p = 0
    try:
        _rccl_info(eng["gpu"][0])
        for upto in (10, 11, 12, 14):
            for k in ("gpu", "oracle"):
                e, sch = eng[k]
                sch.run(e, p, upto)
            p = upto
            _, st = _compare(eng, members, f"period {p}")
        assert st["gossips_created"] > 0 and st["gossip_messages"] > 0
    finally:
        for e, _ in eng.values():
            e.close()
