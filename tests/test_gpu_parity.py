"""Bit-exact parity of libswimgpu.so (HIP kernels on cuda:0) against the CPU oracle.

Every scenario is run by both engines in lockstep through the same C ABI; at every checkpoint the
complete protocol state is compared: all view rows (status, incarnation, table / members /
aliveEmitted / metadata / timer bits and deadlines), per-member FD / gossip / membership scalars,
ping and remote lists in order, live gossips with infection periods and infected sets, and every
SequenceIdCollector.  Events (canonical order) and counters are compared at the end.
"""
import dataclasses

import numpy as np
import pytest

import oracle
import parity
import scenarios
import test_oracle_kat as kat
from swimgpu import abi

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def glib():
    import swimgpu
    return swimgpu.load_library()


@pytest.fixture(scope="module")
def olib():
    return oracle.lib()


def test_gpu_kat_overrides(glib):
    kat.check_overrides(glib)


def test_gpu_kat_collector(glib):
    kat.check_collector(glib)


def test_gpu_kat_collector_random(glib):
    """Every spill tier of the device collector (up to ~1,200 intervals), growth and merge-back."""
    kat.check_collector_random(glib)


def test_gpu_kat_philox(glib):
    kat.check_philox(glib)


def test_gpu_cluster_math(glib):
    kat.check_cluster_math(glib)


def _run_parity(glib, olib, sc, members=None, collectors=True, rccl=False):
    """Run both engines through `sc` in lockstep, comparing full state at every checkpoint (rccl: the
    GPU engine is an RCCL engine of one rank, swim_create_shard with a comm id at world 1)."""
    oe, ge = scenarios.make_engine(olib, sc), scenarios.make_engine(glib, sc, rccl=rccl)
    ops = sorted(sc.ops, key=lambda x: x[0])
    t, oi = 0, 0
    oev, gev = [], []
    while t < sc.ticks:
        while oi < len(ops) and ops[oi][0] <= t:
            scenarios.apply_op(oe, ops[oi][1], ops[oi][2:])
            scenarios.apply_op(ge, ops[oi][1], ops[oi][2:])
            oi += 1
        nxt = min(sc.ticks, t + sc.check_every)
        if oi < len(ops):
            nxt = min(nxt, max(ops[oi][0], t + 1))
        oe.step_ticks(nxt - t)
        ge.step_ticks(nxt - t)
        t = nxt
        oev.append(oe.drain_events())
        gev.append(ge.drain_events())
        d = parity.diff_states(parity.state_digest(oe, members, collectors),
                               parity.state_digest(ge, members, collectors))
        assert not d, f"{sc.name}: state diverged by tick {t}:\n" + "\n".join(d)
    ea, eb = np.concatenate(oev), np.concatenate(gev)
    assert not parity.diff_events(ea, eb), parity.diff_events(ea, eb)
    sa, sb = oe.stats(), ge.stats()
    assert not parity.diff_stats(sa, sb), parity.diff_stats(sa, sb)
    assert sb["capacity_errors"] == 0
    return sa, ea


@pytest.mark.parametrize("sc", scenarios.catalog(), ids=lambda s: s.name)
def test_gpu_parity_scenario(glib, olib, sc):
    _run_parity(glib, olib, sc)


def test_gpu_parity_config2_1024(glib, olib):
    sc = scenarios.config2()
    members = list(range(0, 1024, 37)) + [17, 18, 1023]
    stats, events = _run_parity(glib, olib, sc, members=members, collectors=False)
    # every live member removed member 17 exactly once
    rem = events[(events["type"] == abi.EV_REMOVED) & (events["subject"] == 17)]
    assert sorted(set(rem["viewer"].tolist())) == [v for v in range(1024) if v != 17]
    assert len(rem) == 1023


# ---- the sharded path: the cluster's rows split over 2 / 3 shards that exchange
# GOSSIP_REQ / SYNC / SYNC_ACK traffic exactly as the RCCL ranks do (cfg.local_shards), compared with
# the UNSHARDED oracle: sharding must not change a single bit.  3 shards over 4 members leaves the
# last shard empty; over 3 members every shard owns one row.
# the longest scenario (config3_rates_200, ~70 s a run) runs unsharded, with 3 shards and through
# the pull route with 3 shards in the default suite; its other variants are marked slow (run with
# SWIM_GPU_SLOW=1, tools/gpu_slow.sh) to keep `-m gpu` inside the driver's time limit
SLOW_SCENARIOS = ("config3_rates_200",)


def _cases(shard_list=None):
    out = []
    for sc in scenarios.catalog():
        for sh in (shard_list or [None]):
            slow = sc.name in SLOW_SCENARIOS and sh != 3
            args = (sc,) if sh is None else (sc, sh)
            out.append(pytest.param(*args, id=sc.name if sh is None else f"{sc.name}-{sh}",
                                    marks=[pytest.mark.slow] if slow else []))
    return out


@pytest.mark.parametrize("sc,shards", _cases([2, 3]))
def test_gpu_sharded_parity_scenario(glib, olib, sc, shards):
    if not sc.shardable:
        pytest.skip("scenario uses a single-shard-only feature")
    _run_parity(glib, olib, dataclasses.replace(sc, cfg={**sc.cfg, "local_shards": shards}))


# the RCCL route of the content rows (k_pull_rows: pulled with system-scope loads into per-shard
# copies, then classified from there) in the single-GPU rig (SWIM_EXCHANGE_PULL=1)
PULL_SCENARIOS = ("mp_joins_via_seed", "churn_48", "config3_rates_200", "partition_heal_32", "restart_same_address_40",
                  "sync_delay_24")


# (config3_rates_200 through the pull route is slow-marked at both shard counts: the other five pull
# scenarios cover the route, and the default suite stays well inside the driver's time limit)
@pytest.mark.parametrize("name,shards", [
    pytest.param(nm, sh, id=f"{nm}-{sh}", marks=[pytest.mark.slow] if nm in SLOW_SCENARIOS else [])
    for nm in PULL_SCENARIOS for sh in (2, 3)])
def test_gpu_sharded_pull_parity_scenario(glib, olib, name, shards, monkeypatch):
    sc = {s.name: s for s in scenarios.catalog()}[name]
    monkeypatch.setenv("SWIM_EXCHANGE_PULL", "1")
    _run_parity(glib, olib, dataclasses.replace(sc, cfg={**sc.cfg, "local_shards": shards}))


# row_cap (the content rows a shard sends in one SYNC / SYNC_ACK exchange) grows before a join burst
# that could exceed it (engine.hip grow_rows_for_joins): started at 16 rows (SWIM_DEBUG_ROW_CAP), the
# bursts of 80 joiners through one seed need 80 rows each way; without the growth the tick fails with
# a capacity error (ERR_REQS), with it the run stays bit-exact with the unsharded oracle
@pytest.mark.parametrize("name,shards,pull", [("join_burst_144", 2, False), ("join_burst_144", 3, True),
                                              ("mp_joins_via_seed", 2, False)])
def test_gpu_sharded_row_cap_grows_for_join_burst(glib, olib, name, shards, pull, monkeypatch):
    sc = {s.name: s for s in scenarios.catalog()}[name]
    monkeypatch.setenv("SWIM_DEBUG_ROW_CAP", "16")
    if pull:
        monkeypatch.setenv("SWIM_EXCHANGE_PULL", "1")
    _run_parity(glib, olib, dataclasses.replace(sc, cfg={**sc.cfg, "local_shards": shards}))


# ---- the RCCL transport on one GPU: an RCCL engine of ONE rank runs every exchange step of the
# sharded tick (the count ncclAllToAll / stop ncclAllGather per exchange, the IPC-mapped region,
# k_recv_* / k_pack_rows / k_pull_rows, the quiet windows' allreduces, row_cap growth agreed by
# rank_min) with nothing crossing; bit-exact against the unsharded oracle
RCCL_SCENARIOS = ("config1_kill", "mp_joins_via_seed", "churn_48", "partition_heal_32", "restart_same_address_40",
                  "sync_delay_24", "delay_fd_gossip_12", "user_gossip_10_loss25", "sync_ack_waits_24")


@pytest.mark.parametrize("name", RCCL_SCENARIOS)
def test_gpu_rccl_world1_parity_scenario(glib, olib, name):
    sc = {s.name: s for s in scenarios.catalog()}[name]
    _run_parity(glib, olib, sc, rccl=True)


def test_gpu_rccl_world1_row_cap_grows_for_join_burst(glib, olib, monkeypatch):
    sc = {s.name: s for s in scenarios.catalog()}["join_burst_144"]
    monkeypatch.setenv("SWIM_DEBUG_ROW_CAP", "16")
    _run_parity(glib, olib, sc, rccl=True)


def test_gpu_sharded_parity_config2_1024(glib, olib):
    sc = scenarios.config2()
    sc = dataclasses.replace(sc, cfg={**sc.cfg, "local_shards": 4})
    members = list(range(0, 1024, 37)) + [17, 18, 255, 256, 1023]
    _run_parity(glib, olib, sc, members=members, collectors=False)


# ---- committed regression digests (tests/golden/scenario_digests.json, made by the CPU oracle):
# the GPU engine, unsharded and with 4 in-process shards, reproduces them
@pytest.mark.parametrize("shards", [1, 4])
@pytest.mark.parametrize("sc", scenarios.catalog() + [scenarios.config2()], ids=lambda s: s.name)
def test_gpu_matches_golden_digest(glib, sc, shards):
    import json
    import os

    from make_scenario_digests import digest, event_digest
    golden = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "scenario_digests.json")))
    want = golden["scenarios"][sc.name]
    if shards > sc.capacity:
        pytest.skip("more shards than members")
    if shards > 1 and not sc.shardable:
        pytest.skip("scenario uses a single-shard-only feature")
    sc2 = dataclasses.replace(sc, cfg={**sc.cfg, "local_shards": shards})
    e = scenarios.make_engine(glib, sc2)
    scenarios.run(e, sc2)
    ev = e.drain_events()
    big = sc.name == "config2_1024"
    got_state = digest(e, scenarios.CONFIG2_MEMBERS if big else None, not big)
    st = e.stats()
    assert event_digest(ev) == want["events_sha256"] and len(ev) == want["events"]
    assert {k: int(st[k]) for k in want["stats"]} == want["stats"]
    assert got_state == want["state_sha256"]


# ---- the wave-parallel delivery path (deliver_big: stable-by-sender canonical ranking, wave-batched
# pingMembers inserts) for EVERY gossip inbox, not only the big ones of a storm
@pytest.mark.parametrize("sc", [pytest.param(sc, id=sc.name, marks=[pytest.mark.slow] if sc.name in SLOW_SCENARIOS else [])
                                for sc in scenarios.catalog()])
def test_gpu_parity_wave_delivery(glib, olib, sc):
    _run_parity(glib, olib, dataclasses.replace(sc, cfg={**sc.cfg, "deliver_wave_min": 1}))


# ---- the whole-wave delivery (deliver_coop: leader lanes per gossiper, the no-op records skipped, the
# rest in rank order) for every inbox of two or more messages, unsharded and with 3 shards
COOP_SCENARIOS = ("join_burst_144", "join_burst_seg", "churn_48", "loss5_kills_64", "user_gossip_10_loss25",
                  "delay_fd_gossip_12", "namespaces_9", "mp_leave_cluster", "restart_same_address_40",
                  "update_metadata_12", "external_sync_16", "sync_delay_24", "partition_heal_32")


@pytest.mark.parametrize("name,shards", [(nm, sh) for nm in COOP_SCENARIOS for sh in (1, 3)])
def test_gpu_parity_coop_delivery(glib, olib, name, shards, monkeypatch):
    sc = {s.name: s for s in scenarios.catalog()}[name]
    monkeypatch.setenv("SWIM_DEBUG_COOP_MIN", "2")
    cfg = {**sc.cfg, "deliver_wave_min": 1}
    if shards > 1:
        cfg["local_shards"] = shards
    _run_parity(glib, olib, dataclasses.replace(sc, cfg=cfg))
