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


def test_config3_16384_first_periods_match_oracle(glib):
    """Config 3 at its stated size, N = 16,384: 5 % uniform loss, 164 kills + 164 joins through seed 0
    per period (bench.py's churn schedule).  The first two periods (the joins' SYNC storm begins)
    are compared bit-exactly with the threaded oracle — sampled full member state (killed members,
    joiners, the seed), the event stream and every counter; the GPU then runs the third period alone
    (the SYNC-originated gossip storm: ~10^9 GOSSIP_REQs per period) with no capacity error and no
    removal (suspicion timeouts are 70 periods away).  Longer runs do not fit any memory: DESIGN.md §6."""
    import bench
    n, exact, total = 16384, 2, 3
    sch = {k: bench.Schedule("churn", n, total) for k in ("gpu", "oracle")}
    engines = {}
    for k, lib in (("gpu", glib), ("oracle", oracle.lib())):
        cfg = bench.churn_capacities(bench.make_config(lib), sch[k].capacity)
        cfg.message_capacity = 1 << 30  # the third period's gossip rounds: ~4 x 10^8 messages each
        engines[k] = abi.Engine(lib, cfg, sch[k].capacity, n, 1)
        sch[k].setup(engines[k])
    oracle.set_threads(engines["oracle"], THREADS)
    ops1 = sch["gpu"].ops(0)
    killed = [m for op, m in ops1 if op == "kill"][:6]
    joined = [m for op, m in ops1 if op == "join"][:6]
    sch["gpu"] = bench.Schedule("churn", n, total)  # ops() consumed the schedule's draws: start over
    members = [0, 1, 5000, n - 1] + killed + joined + [n + 164 + 3]
    for p in range(exact):
        for k in ("gpu", "oracle"):
            sch[k].run(engines[k], p, p + 1)
        d = parity.diff_states(parity.state_digest(engines["oracle"], members, False),
                               parity.state_digest(engines["gpu"], members, False))
        assert not d, f"diverged in period {p + 1}:\n" + "\n".join(d)
        ea, eb = engines["oracle"].drain_events(), engines["gpu"].drain_events()
        assert not parity.diff_events(ea, eb), parity.diff_events(ea, eb)
        sa, sb = engines["oracle"].stats(), engines["gpu"].stats()
        assert not parity.diff_stats(sa, sb), parity.diff_stats(sa, sb)
    engines["oracle"].close()
    e = engines["gpu"]
    for p in range(exact, total):
        sch["gpu"].run(e, p, p + 1)
        ev = e.drain_events()
        assert not (ev["type"] == abi.EV_REMOVED).any()
    st = e.stats()
    assert st["capacity_errors"] == 0
    assert st["gossip_messages"] > 10 ** 8


def _partition_cfg(lib, n, gossip_capacity):
    # a partition puts a suspicion timer for every member of the other side at every viewer (N^2 / 2
    # pending), falling due within the few ticks the SUSPECT gossip took to spread
    return dict(sync_stagger=1, record_fd_events=0, gossip_capacity=gossip_capacity,
                timer_capacity=max(64 * n, n * n // 2), timer_pool_capacity=n * n // 2 + 64 * n,
                collector_capacity=1 << (2 * n - 1).bit_length())


@pytest.mark.parametrize("n,hold,after", [(256, 52, 8), (128, 20, 10)])
def test_config5_partition_heal_matches_oracle(glib, n, hold, after):
    """Config 5 in miniature, bit-exact for the whole run: a 2-way partition [0, N/2) | [N/2, N) from
    period 2, seeds {0, N/2}; held past the suspicion timeout (each side REMOVEs the other, then the
    seeds' SYNCs re-join the halves) or healed while the other side is still SUSPECT (every FD ping
    across succeeds again: the SYNC storm of refutations).  Full state of every member every 10
    periods, the event stream and the counters against the threaded oracle."""
    g = np.zeros(n, dtype=np.uint16)
    g[n // 2:] = 1
    heal = 2 + hold
    sc = scenarios.Scenario(f"partition_{n}_{hold}", n, n, (heal + after) * 10, seed=5, seeds=(0, n // 2),
                            cfg=_partition_cfg(glib, n, 1 << 17), ops=[(20, "partition", g), (heal * 10, "partition", None)],
                            check_every=100)
    ge, oe = scenarios.make_engine(glib, sc), scenarios.make_engine(oracle.lib(), sc)
    oracle.set_threads(oe, THREADS)

    def check(t):
        d = parity.diff_states(parity.state_digest(oe, None, False), parity.state_digest(ge, None, False))
        assert not d, f"diverged by tick {t}:\n" + "\n".join(d)

    scenarios.run(ge, sc)
    scenarios.run(oe, sc, on_check=None)
    check(sc.ticks)
    ea, eb = oe.drain_events(), ge.drain_events()
    assert not parity.diff_events(ea, eb), parity.diff_events(ea, eb)
    sa, sb = oe.stats(), ge.stats()
    assert not parity.diff_stats(sa, sb), parity.diff_stats(sa, sb)
    assert sb["capacity_errors"] == 0


def _golden_run(name):
    import json
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "config_digests.json")
    runs = json.load(open(path))["runs"] if os.path.exists(path) else {}
    if name not in runs:
        pytest.skip(f"{name} not in tests/golden/config_digests.json (tests/golden/make_config_digests.py)")
    return runs[name]


def _check_checkpoints(want, got, where):
    """every checkpoint of the oracle's golden run, in order: state digest, events, counters"""
    order = sorted(want["checkpoints"], key=int)  # (the JSON file keeps its keys sorted as strings)
    assert sorted(got, key=int) == order, (list(got), order)
    for p in order:
        w = want["checkpoints"][p]
        g = got[p]
        assert g["stats"] == w["stats"], f"{where}: counters differ by period {p}: " + "; ".join(
            f"{k} {w['stats'][k]} != {g['stats'][k]}" for k in w["stats"] if w["stats"][k] != g["stats"][k])
        assert (g["events"], g["events_sha256"]) == (w["events"], w["events_sha256"]), \
            f"{where}: events of the stretch ending at period {p} differ ({g['events']} vs {w['events']})"
        assert g["state_sha256"] == w["state_sha256"], f"{where}: state differs at period {p}"


@pytest.mark.parametrize("n,shards", [(1024, 1), (1024, 8), (4096, 1), (4096, 8)])
def test_config5_partition_heal_matches_oracle_checkpoints(glib, n, shards):
    """BASELINE config 5 bit-exact over its whole run at N = 1,024 and N = 4,096, unsharded and over 8
    in-process shards: seeds {0, N/2}, a 2-way partition from period 2, held past the suspicion
    timeout (every viewer REMOVEs the other side), healed (period 82 / 92), run until every view is
    all-ALIVE again (period 122 / 152).  Every 10 periods the digest of the members' full state (all
    1,024; at N = 4,096 every 64th and the shard boundaries), the stretch's events and every counter
    must equal the threaded oracle's committed checkpoints (tests/golden/make_config_digests.py;
    MembershipProtocolTest.java:1035-1109, MembershipProtocolImpl.java:339-357,461-472).  Then the
    outcome itself: all views all-ALIVE again."""
    import make_config_digests as mk
    want = _golden_run(f"config5_partition_heal_{n}")
    heal, end = want["heal_period"], want["periods"]
    members = None if want["members"] == "all" else want["members"]
    assert members == mk.c5_members(n)
    # (sharded: every GOSSIP_REQ to another shard the receipt filter cannot prove redundant is
    # materialised — ~12 M a round in the heal's storm at N = 1,024; a shard's inbox and its
    # per-destination outgoing buffers are sized for them)
    extra = {"message_capacity": 1 << 26 if n <= 1024 else 1 << 27} if shards > 1 else {}
    e = mk.c5_engine(glib, n, local_shards=shards, **extra)
    got = {}
    try:
        if shards > 1:
            assert e.shard_info()["world"] == shards
        mk.c5_run(e, lambda p, ev: got.__setitem__(str(p), mk.checkpoint(e, ev, members, False)), n, heal, end)
        _check_checkpoints(want, got, f"config 5, N = {n}, {shards} shard(s)")
        for v in range(n):
            row = e.read_view(v)
            assert (((row >> 34) & 1) == 1).all() and (((row >> 32) & 3) == 0).all(), f"view {v} not all-ALIVE"
        st = e.stats()
        assert st["capacity_errors"] == 0 and st["orig_sync"] > 0
    finally:
        e.close()


@pytest.mark.parametrize("shards", [1, 4])
def test_config3_churn_4096_eight_periods_match_oracle(glib, shards):
    """BASELINE config 3's churn schedule (bench.py: 5 % uniform loss, 1 % kills + 1 % fresh joins
    through seed 0 per period) bit-exact for 8 periods at N = 4,096, unsharded and over 4 in-process
    shards: every period the sampled members' full state (SequenceIdCollectors included), the
    period's events and every counter against the oracle's committed checkpoints
    (tests/golden/make_config_digests.py).  Period 8 carries ~10^9 GOSSIP_REQs."""
    import make_config_digests as mk
    want = _golden_run("config3_churn_4096")
    e, sch, members = mk.c3_engine(glib, local_shards=shards)
    assert members == want["members"]
    got = {}
    try:
        for p in range(mk.C3_PERIODS):
            sch.run(e, p, p + 1)
            ev = e.drain_events(1 << 27)
            got[str(p + 1)] = mk.checkpoint(e, ev, members, True)
            if str(p + 1) in want["checkpoints"]:  # fail at the first differing period
                _check_checkpoints({"checkpoints": {k: v for k, v in want["checkpoints"].items() if int(k) <= p + 1}},
                                   got, f"config 3, N = 4,096, {shards} shard(s)")
        _check_checkpoints(want, got, f"config 3, N = 4,096, {shards} shard(s)")
        assert e.stats()["capacity_errors"] == 0
    finally:
        e.close()


def test_config5_partition_heal_2048_reconverges(glib):
    """Config 5 at the largest size one MI355X holds for a heal after removal (the
    partition's SUSPECT gossips alone keep ~80 x N live gossips per member): N = 2,048, partition from
    period 2, held past the suspicion timeout, healed through seeds {0, N/2}.  Every viewer REMOVEs
    each member of the other side exactly once while partitioned and nobody of its own side; after
    the heal every viewer ADDs each of them back exactly once, and within 20 periods every viewer
    sees all N members ALIVE; no capacity error."""
    n = 2048
    cfg = abi.default_config(glib, 0, message_capacity=1 << 28, event_capacity=1 << 26,
                             **_partition_cfg(glib, n, 1 << 19))
    e = abi.Engine(glib, cfg, n, n, 5)
    e.set_seeds([0, n // 2])
    side = (np.arange(n) >= n // 2).astype(np.int64)
    # past the suspicion timeout of the last SUSPECT: a side's FD pings find the other side's members
    # over ~15 periods (one ping per member per period), and the SUSPECT gossip spreads in a few more
    hold = 5 * _ceil_log2(n) + 30
    heal = 2 + hold
    removed = np.zeros((n, n), dtype=np.int16)
    added = np.zeros((n, n), dtype=np.int16)
    converged_at = None
    for p in range(heal + 20):
        if p == 2:
            e.set_partition(side.astype(np.uint16))
        if p == heal:
            assert (removed.sum(axis=1) == n // 2).all()
            e.set_partition(None)
        e.step(1)
        ev = e.drain_events()
        for typ, acc in ((abi.EV_REMOVED, removed), (abi.EV_ADDED, added)):
            x = ev[ev["type"] == typ]
            np.add.at(acc, (x["viewer"].astype(np.int64), x["subject"].astype(np.int64)), 1)
        if p >= heal and converged_at is None:
            if all(((((row := e.read_view(v)) >> 34) & 1) == 1).all() and (((row >> 32) & 3) == 0).all()
                   for v in range(0, n, 97)):
                if all(((((row := e.read_view(v)) >> 34) & 1) == 1).all() and (((row >> 32) & 3) == 0).all()
                       for v in range(n)):
                    converged_at = p + 1
                    break
    assert e.stats()["capacity_errors"] == 0
    other = side[:, None] != side[None, :]
    assert (removed[other] == 1).all() and (removed[~other] == 0).all()
    assert converged_at is not None, "not converged within 20 periods of the heal"
    assert (added[other] == 1).all() and (added[~other] == 0).all()


def _period_log(name):
    """per-period JSON lines of a long config run, under gpurun_out/ when it exists (GPU box)"""
    import json
    d = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
    f = open(os.path.join(d, f"{name}.jsonl"), "w") if os.path.isdir(d) else None

    def log(**kw):
        if f:
            f.write(json.dumps(kw) + "\n")
            f.flush()
    return log


def _reason_delta(st, prev):
    return {r: st[f"orig_{r}"] - prev[f"orig_{r}"] for r in abi.ORIG_REASONS if st[f"orig_{r}"] != prev[f"orig_{r}"]}


def _partition_run(e, n, hold, log, stop_on_capacity=False):
    """2-way partition from period 2 held for `hold` periods: per-period origination counters to
    `log`; returns (REMOVED (viewer, subject) keys, the period a capacity error stopped the run or
    None, the errors' bits)."""
    side = (np.arange(n) >= n // 2).astype(np.int64)
    keys = []
    prev = e.stats()
    for p in range(2 + hold):
        if p == 2:
            e.set_partition(side.astype(np.uint16))
        try:
            e.step(1)
        except abi.SwimError as ex:
            if not stop_on_capacity:
                raise
            st = e.stats()
            log(period=p + 1, stopped=str(ex), by_reason=_reason_delta(st, prev), capacity_errors=st["capacity_errors"])
            return np.concatenate(keys) if keys else np.zeros(0, np.int64), p + 1, st["capacity_errors"]
        ev = e.drain_events(1 << 27)
        rem = ev[ev["type"] == abi.EV_REMOVED]
        keys.append(rem["viewer"].astype(np.int64) * n + rem["subject"].astype(np.int64))
        assert not (ev["type"] == abi.EV_ADDED).any()
        st = e.stats()
        log(period=p + 1, gossips=st["gossips_created"] - prev["gossips_created"], by_reason=_reason_delta(st, prev),
            msgs=st["gossip_messages"] - prev["gossip_messages"], removed=len(rem),
            timers_fired=st["timers_fired"] - prev["timers_fired"], max_live_gossips_sampled=max(
                e.read_member(m)["gossip_len"] for m in range(0, n, max(1, n // 16))),
            capacity_errors=st["capacity_errors"])
        prev = st
        assert st["capacity_errors"] == 0, f"capacity error in period {p + 1}"
    return np.concatenate(keys), None, 0


def test_config5_partition_8192_removes_other_side(glib):
    """BASELINE config 5's partition phase at N = 8,192 on one MI355X (the largest power of two whose
    partition-phase gossip state fits one GPU, see the N = 16,384 test): seeds {0, N/2}, a 2-way
    partition [0, N/2) | [N/2, N) from period 2, held past the suspicion timeout.  Every viewer
    REMOVEs each member of the other side exactly once and nobody of its own side; no capacity
    error; nobody refutes (no gossip crosses the cut)."""
    n = 8192
    cfg = abi.default_config(glib, 0, message_capacity=1 << 29, event_capacity=1 << 27,
                             **_partition_cfg(glib, n, 1 << 18))
    e = abi.Engine(glib, cfg, n, n, 5)
    try:
        e.set_seeds([0, n // 2])
        keys, _, _ = _partition_run(e, n, 5 * _ceil_log2(n) + 30, _period_log("config5_partition_8192"))
        side = (np.arange(n) >= n // 2).astype(np.int64)
        v, s = keys // n, keys % n
        assert (side[v] != side[s]).all(), "a member of the viewer's own side was removed"
        assert len(np.unique(keys)) == len(keys), "a member was removed twice by one viewer"
        assert len(keys) == n * (n // 2), f"{n * (n // 2) - len(keys)} (viewer, other-side member) pairs not removed"
        st = e.stats()
        assert st["orig_fd"] > 0 and st["orig_refute"] == 0
        assert st["orig_fd"] + st["orig_sync"] == st["gossips_created"]
    finally:
        e.close()


@pytest.mark.slow
def test_config5_partition_16384_storm_is_sync_regossip(glib):
    """BASELINE config 5's partition phase at N = 16,384: why it does not fit one GPU,
    measured.  SUSPECTs spread by gossip from the failure detectors, but every member whose periodic
    SYNC (N / 30 per period) reaches a same-side member first learns the suspicions from the SYNC and
    re-gossips each one (spreadMembershipGossipUnlessGossiped gossips on every reason but
    MEMBERSHIP_GOSSIP and INITIAL_SYNC, MembershipProtocolImpl.java:621-628,836-843): from period 5
    on, >= 90 % of all originated gossips come from the SYNC branch (swim_stats.gossips_by_reason)
    and a member's live gossips outgrow 2^17 slab entries (the run stops at the slab's capacity
    error rather than truncating).  With a bigger slab the phase must still remove the other side
    exactly once."""
    n = 16384
    cfg = abi.default_config(glib, 0, message_capacity=1 << 29, event_capacity=1 << 27,
                             **_partition_cfg(glib, n, 1 << 17))
    e = abi.Engine(glib, cfg, n, n, 5)
    lines = []
    log = _period_log("config5_partition_16384")

    def tee(**kw):
        lines.append(kw)
        log(**kw)
    try:
        e.set_seeds([0, n // 2])
        keys, stopped, bits = _partition_run(e, n, 5 * _ceil_log2(n) + 30, tee, stop_on_capacity=True)
        storm = [ln for ln in lines if ln["period"] >= 5 and "gossips" in ln and ln["gossips"] > 1000]
        assert storm, "no gossip storm"
        sync = sum(ln["by_reason"].get("sync", 0) for ln in storm)
        total = sum(ln["gossips"] for ln in storm)
        assert sync >= 0.9 * total, (sync, total)
        if stopped is not None:
            assert bits & 0x1, f"stopped by {bits:#x}, not by the gossip slab"
            # the storm property holds, but BASELINE config 5 at this size is NOT met on one GPU: the
            # run cannot complete, so it is reported as an expected failure, never as a pass
            pytest.xfail(f"config 5 at N={n} does not fit one MI355X: the gossip slab overflowed in period "
                         f"{stopped} (SYNC-originated share {sync / max(1, total):.3f})")
        else:
            side = (np.arange(n) >= n // 2).astype(np.int64)
            assert len(np.unique(keys)) == len(keys) == n * (n // 2)
            assert (side[keys // n] != side[keys % n]).all()
    finally:
        e.close()


def test_config5_heal_4096_reconverges_and_sync_originates_the_storm(glib):
    """Config 5's heal at N = 4,096 (twice the round-2 size): partition from period 2, held past the
    suspicion timeout (each side REMOVEs the other), healed through seeds {0, N/2}.  Every viewer
    REMOVEs each member of the other side exactly once and ADDs it back exactly once; all views are
    all-ALIVE within 120 periods of the heal; no capacity error.  (After the removal the sides meet
    again only when a periodic SYNC — N/30 per period — picks the other side's seed among the N/2
    candidates it knows: 1/15 such SYNC per period whatever N, so the first one comes ~15 periods
    after the heal on average; a 20-period window missed it in one run of this test.)  The gossips originated after the
    heal come from the SYNC branch of updateMembership (spreadMembershipGossipUnlessGossiped,
    MembershipProtocolImpl.java:627,652,836-843): a member that learns the other side through a
    SYNC / SYNC_ACK re-gossips every record it learned — swim_stats.gossips_by_reason['sync']
    carries (almost) all of them, which is the O(N^2) gossip volume DESIGN.md §6 cites."""
    n = 4096
    cfg = abi.default_config(glib, 0, message_capacity=1 << 28, event_capacity=1 << 26,
                             **_partition_cfg(glib, n, 800_000))
    e = abi.Engine(glib, cfg, n, n, 5)
    try:
        _heal_4096_body(e, n)
    finally:
        e.close()


def _heal_4096_body(e, n):
    e.set_seeds([0, n // 2])
    side = (np.arange(n) >= n // 2).astype(np.int64)
    hold = 5 * _ceil_log2(n) + 30
    heal = 2 + hold
    log = _period_log("config5_heal_4096")
    removed = np.zeros((n, n), dtype=np.int16)
    added = np.zeros((n, n), dtype=np.int16)
    converged_at = None
    prev = e.stats()
    at_heal = None
    for p in range(heal + 120):
        if p == 2:
            e.set_partition(side.astype(np.uint16))
        if p == heal:
            assert (removed.sum(axis=1) == n // 2).all()
            e.set_partition(None)
            at_heal = e.stats()
        e.step(1)
        ev = e.drain_events(1 << 26)
        for typ, acc in ((abi.EV_REMOVED, removed), (abi.EV_ADDED, added)):
            x = ev[ev["type"] == typ]
            np.add.at(acc, (x["viewer"].astype(np.int64), x["subject"].astype(np.int64)), 1)
        st = e.stats()
        glen = max(e.read_member(m)["gossip_len"] for m in range(0, n, 257))
        log(period=p + 1, gossips=st["gossips_created"] - prev["gossips_created"], by_reason=_reason_delta(st, prev),
            msgs=st["gossip_messages"] - prev["gossip_messages"], syncs=st["syncs"] - prev["syncs"],
            events=len(ev), max_live_gossips_sampled=glen, capacity_errors=st["capacity_errors"])
        prev = st
        assert st["capacity_errors"] == 0, f"capacity error in period {p + 1}"
        def all_alive(v):
            row = e.read_view(v)
            return bool((((row >> 34) & 1) == 1).all() and (((row >> 32) & 3) == 0).all())
        if p >= heal and converged_at is None and all(all_alive(v) for v in range(0, n, 61)):
            if all(all_alive(v) for v in range(n)):
                converged_at = p + 1
                break
    other = side[:, None] != side[None, :]
    assert (removed[other] == 1).all() and (removed[~other] == 0).all()
    assert converged_at is not None, "not converged within 120 periods of the heal"
    assert (added[other] == 1).all() and (added[~other] == 0).all()
    st = e.stats()
    healed = {r: st[f"orig_{r}"] - at_heal[f"orig_{r}"] for r in abi.ORIG_REASONS}
    total = sum(healed.values())
    log(heal_gossips_by_reason=healed, converged_at=converged_at)
    assert healed["sync"] >= 0.9 * total, healed
