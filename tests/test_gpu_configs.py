"""BASELINE configs 3-5 at the largest sizes one MI355X runs.

The CPU oracle (threaded, oracle.set_threads) still finishes the first periods of N = 16,384, so those
runs are compared bit-exactly; beyond that the GPU engine alone runs the configuration and the
tests check size-independent properties of the protocol's outcome (every live viewer removes a
killed member exactly once, inside the suspicion window; no capacity error; ...).
"""
import os

import numpy as np
import pytest

import oracle
import parity
import scenarios
from swimgpu import abi

pytestmark = pytest.mark.gpu

THREADS = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1)))


@pytest.fixture(scope="module")
def glib():
    import swimgpu
    return swimgpu.load_library()


def _ceil_log2(n):
    return int(n).bit_length()


def test_config4_65536_single_kill_removed_everywhere(glib):
    """Config 4 at N = 65,536 on one GPU: kill one member; every other member removes it exactly
    once, between suspicion timeout and suspicion timeout + a few periods after the kill (the SUSPECT
    spreads by gossip within a few periods), and nobody else is removed."""
    n, victim, kill_period = 65536, 40503, 2
    cfg = abi.default_config(glib, 0, sync_stagger=1, record_fd_events=0)
    e = abi.Engine(glib, cfg, n, n, 7)
    tpp = e.now()[2]
    e.step(kill_period)
    e.kill(victim)
    kill_tick = e.now()[0]
    timeout_periods = 5 * _ceil_log2(n)  # suspicionMult x ceilLog2(N) x pingInterval
    removed = np.zeros(n, dtype=np.int64)
    first, last = None, None
    for _ in range((timeout_periods + 12) // 4):
        e.step(4)
        ev = e.drain_events()
        rem = ev[ev["type"] == abi.EV_REMOVED]
        assert (rem["subject"] == victim).all(), "a live member was removed"
        np.add.at(removed, rem["viewer"].astype(np.int64), 1)
        if len(rem):
            first = int(rem["tick"].min()) if first is None else first
            last = int(rem["tick"].max())
    st = e.stats()
    assert st["capacity_errors"] == 0
    live = np.ones(n, dtype=bool)
    live[victim] = False
    assert (removed[live] == 1).all(), f"{int((removed[live] != 1).sum())} live viewers did not remove it once"
    assert removed[victim] == 0
    # the first removal: a suspicion timeout after the first SUSPECT (the first ping of the victim);
    # the last: within a few periods of gossip spread after that
    assert first >= kill_tick + timeout_periods * tpp
    assert last <= kill_tick + (timeout_periods + 10) * tpp
    assert st["gossips_created"] > 0 and st["timers_fired"] >= n - 1


def test_config4_sharded8_16384_matches_oracle(glib):
    """Config 4's sharded deployment in miniature: N = 16,384 rows over 8 in-process shards (the RCCL
    exchange plan with device copies) against the UNSHARDED oracle for the first periods, a member
    killed at tick 5: sampled full member state, the event stream and every counter bit-exact."""
    olib = oracle.lib()
    sc = scenarios.Scenario("config4_ls8_16384", 16384, 16384, 60, seed=3, ops=[(5, "kill", 777)], check_every=20)
    ge = scenarios.make_engine(glib, scenarios.Scenario(**{**sc.__dict__, "cfg": {"local_shards": 8}}))
    oe = scenarios.make_engine(olib, sc)
    oracle.set_threads(oe, THREADS)
    members = [0, 1, 776, 777, 778, 2047, 2048, 8191, 8192, 16383] + list(range(101, 16384, 1637))
    t = 0
    for tk in (5, 20, 40, 60):
        if t == 5:
            scenarios.apply_op(ge, "kill", (777,))
            scenarios.apply_op(oe, "kill", (777,))
        ge.step_ticks(tk - t)
        oe.step_ticks(tk - t)
        t = tk
        d = parity.diff_states(parity.state_digest(oe, members, False), parity.state_digest(ge, members, False))
        assert not d, f"diverged by tick {t}:\n" + "\n".join(d)
    ea, eb = oe.drain_events(), ge.drain_events()
    assert not parity.diff_events(ea, eb), parity.diff_events(ea, eb)
    sa, sb = oe.stats(), ge.stats()
    assert not parity.diff_stats(sa, sb), parity.diff_stats(sa, sb)
    assert sb["capacity_errors"] == 0
