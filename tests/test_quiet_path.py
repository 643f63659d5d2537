"""Quiet windows (swim_quiet.h): while the cluster is provably quiet the GPU engine
advances a window of ticks with two launches instead of the per-tick kernel chain.  The windows
must be invisible: every scenario here runs on libswimgpu.so with quiet windows ON and is compared
bit-exactly against the CPU oracle (full state of every member, events, counters) at every
checkpoint — across the transitions into and out of the windows: a kill (the window ends at the
first ping of the stopped member: FailureDetectorImpl.doPing :126-171 -> ping-req), the suspicion
timers falling due (a non-empty wheel bucket ends a window), a graceful leave and a user gossip (live
gossips: GossipProtocolImpl.doSpreadGossip :141-184), an inbound block (an ack that cannot arrive),
loss switched on and off (a host-side setting), joins (control operations), the KS timing mode
(10 ms ticks, staggered timers) and a ping list reaching its end (Collections.shuffle on wrap,
:352-361).  A larger run compares quiet ON against quiet OFF on the GPU itself, every row."""
import numpy as np
import pytest

import oracle
import parity
import scenarios
from swimgpu import abi

pytestmark = pytest.mark.gpu

ALL = abi.ALL_MEMBERS
S = scenarios.Scenario
QUIET_SCENARIOS = [
    # kills, their suspicion timeouts (5 x ceilLog2(256) periods), then quiet again
    S("quiet_kill_256", 256, 256, 1300, seed=31, ops=[(300, "kill", 77), (301, "kill", 78)], check_every=100),
    # a graceful leave, a user gossip, an inbound block (pings to member 3 are never acknowledged)
    S("quiet_leave_spread_inbound_128", 128, 128, 1100, seed=32, seeds=(0,),
      ops=[(100, "leave", 5, 1), (400, "spread", 9, 42), (700, "default_in", 0, 3), (760, "default_in", 1, 3)],
      check_every=100),
    # loss on, then off again (host-side eligibility), a kill while lossy
    S("quiet_loss_toggle_96", 96, 96, 900, seed=33, ops=[(200, "loss", 3, ALL), (250, "kill", 40), (330, "loss", 0, ALL)],
      check_every=100),
    # joins through a seed (control operations; the joiners' initial SYNCs, ADDED storms)
    S("quiet_join_80", 80, 64, 800, seed=34, seeds=(0,), ops=[(150, "join", 64), (150, "join", 65), (420, "join", 66)],
      check_every=100),
    # small cluster: ping lists wrap every few periods (the window ends at the reshuffle)
    S("quiet_wrap_6", 6, 6, 600, seed=35, ops=[(300, "kill", 4)], check_every=50),
    # the KS timing mode: 10 ms ticks, staggered timer phases (100 ticks per period)
    S("quiet_ks_mode_64", 64, 64, 6000, seed=36, cfg=dict(timer_stagger=1, tick_ms=10), ops=[(2500, "kill", 9)],
      check_every=500),
]


@pytest.fixture(scope="module")
def glib():
    import swimgpu
    return swimgpu.load_library()


@pytest.mark.parametrize("sc", QUIET_SCENARIOS, ids=lambda s: s.name)
def test_quiet_windows_match_oracle(glib, sc):
    ge, oe = scenarios.make_engine(glib, sc), scenarios.make_engine(oracle.lib(), sc)
    ge.set_quiet_path(True)
    ops = sorted(sc.ops, key=lambda x: x[0])
    t, oi = 0, 0
    while t < sc.ticks:
        while oi < len(ops) and ops[oi][0] <= t:
            for e in (ge, oe):
                scenarios.apply_op(e, ops[oi][1], ops[oi][2:])
            oi += 1
        nxt = min(sc.ticks, t + sc.check_every)
        if oi < len(ops):
            nxt = min(nxt, max(ops[oi][0], t + 1))
        ge.step_ticks(nxt - t)
        oe.step_ticks(nxt - t)
        t = nxt
        d = parity.diff_states(parity.state_digest(oe), parity.state_digest(ge))
        assert not d, f"{sc.name} diverged by tick {t}:\n" + "\n".join(d)
    ea, eb = oe.drain_events(), ge.drain_events()
    assert not parity.diff_events(ea, eb), parity.diff_events(ea, eb)
    sa, sb = oe.stats(), ge.stats()
    assert not parity.diff_stats(sa, sb), parity.diff_stats(sa, sb)
    q = ge.quiet_stats()
    # the windows ran, and some ended early at a tick the per-tick chain had to take
    assert q["windows"] > 0 and q["ticks"] > 0 and q["cut_short"] > 0, q
    assert q["ticks"] < sc.ticks, q


def test_quiet_on_equals_quiet_off_4096(glib):
    """N = 4,096, LAN defaults: 30 quiet periods, a kill, its detection and removal everywhere
    (suspicion timeout 65 periods), quiet again; quiet windows ON vs OFF on the GPU, every row and
    every member's scalars and lists, the events and counters."""
    n = 4096
    sc = S("quiet_ab_4096", n, n, 1200, seed=37, ops=[(300, "kill", 1234)])
    eng = {}
    for on in (True, False):
        e = scenarios.make_engine(glib, sc)
        e.set_quiet_path(on)
        e.step_ticks(300)
        e.kill(1234)
        e.step_ticks(900)
        eng[on] = e
    assert eng[True].quiet_stats()["ticks"] > 300 and eng[False].quiet_stats()["ticks"] == 0
    members = list(range(0, n, 7)) + [1233, 1234, 1235, n - 1]
    d = parity.diff_states(parity.state_digest(eng[False], members, False), parity.state_digest(eng[True], members, False))
    assert not d, "\n".join(d)
    for v in range(n):  # every row
        assert np.array_equal(eng[False].read_view(v), eng[True].read_view(v)), v
    ea, eb = eng[False].drain_events(), eng[True].drain_events()
    assert not parity.diff_events(ea, eb), parity.diff_events(ea, eb)
    assert (ea["type"] == abi.EV_REMOVED).sum() == n - 1
    sa, sb = eng[False].stats(), eng[True].stats()
    assert not parity.diff_stats(sa, sb), parity.diff_stats(sa, sb)


def test_precomputed_windows_match_oracle(glib):
    """A pristine cluster (no member ever stopped or filtered) lets a window's apply find the next
    window's end, so consecutive windows launch no scan (swim_quiet.h QuietPre).  Calls of varying
    length with reads between them (which keep the precompute), ping lists wrapping every few
    periods (N = 12: the reshuffle ends windows), and then a metadata update and a join (control
    operations: the next window scans); compared with the oracle after every call, then the
    precomputed windows are checked to have run (they cover the longest window a call may ask
    for, kQuietMax ticks, so a longer call after a shorter one needs no scan either)."""
    sc = S("quiet_pristine_12", 16, 12, 0, seed=38, seeds=(0,))
    ge, oe = scenarios.make_engine(glib, sc), scenarios.make_engine(oracle.lib(), sc)
    ge.set_quiet_path(True)
    steps = [50, 50, 20, 20, 80, 10, 200, 200, 7, 7, 7, 300, 33, 33]
    for i, k in enumerate(steps + ["meta", 60, 60, "join", 120, 120, 40]):
        if k == "meta":
            for e in (ge, oe):
                e.update_metadata(3)
            continue
        if k == "join":
            for e in (ge, oe):
                e.join(12)
            continue
        ge.step_ticks(k)
        oe.step_ticks(k)
        d = parity.diff_states(parity.state_digest(oe), parity.state_digest(ge))
        assert not d, f"call {i} ({k} ticks) diverged:\n" + "\n".join(d)
    ea, eb = oe.drain_events(), ge.drain_events()
    assert not parity.diff_events(ea, eb), parity.diff_events(ea, eb)
    sa, sb = oe.stats(), ge.stats()
    assert not parity.diff_stats(sa, sb), parity.diff_stats(sa, sb)
    q = ge.quiet_stats()
    assert q["precomputed"] > 0 and q["precomputed"] < q["attempts"], q
