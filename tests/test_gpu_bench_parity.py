"""bench.py's own workloads at their own size, GPU against the threaded CPU oracle, bit-exact.

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


def _engines(glib, workload, periods):
    from swimgpu import abi
    out = {}
    for k, lib in (("gpu", glib), ("oracle", oracle.lib())):
        sch = bench.Schedule(workload, N, periods)
        e = abi.Engine(lib, bench.make_config(lib), sch.capacity, N, 1)
        sch.setup(e)
        out[k] = (e, sch)
    oracle.set_threads(out["oracle"][0], THREADS)
    return out


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
