"""KS tolerance of the lockstep engine's detection-latency and convergence distributions against the
reference-timing DES (north_star; SURVEY.md §8 "KS": two-sample KS, pass at p >= 0.01).

Lockstep runs use `timer_stagger = 1` (independent ping / gossip timer phases per member, as in a
cluster whose members started at different instants) and a 10 ms tick, the resolution at which the
lockstep order is a faithful discretisation of the asynchronous reference ("Distributional parity").  The
aligned default (every member's timers in phase, 100 ms tick) is the throughput mode; the last CPU
test pins that it is NOT distributionally equivalent (each gossip hop costs a full gossip interval
instead of a uniform fraction of one), so nobody reads the aligned mode's latencies as reference
latencies.

DES samples come from tests/golden/des_n{64,1024}.json (tests/golden/make_des_fixtures.py), which
test_des_fixture_reproduces re-derives live for a few seeds.
"""
import json
import os

import pytest

import des
import ks
import oracle
from swimgpu import abi

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FAITHFUL = dict(timer_stagger=1, tick_ms=10)


def fixture(n):
    with open(os.path.join(GOLDEN, f"des_n{n}.json")) as f:
        doc = json.load(f)
    samples = {k: [r[k] for r in doc["samples"]] for k in ks.STATS}
    return doc, samples


def check(res, label):
    lines = [f"{k}: D={v['D']:.3f} p={v['p']:.3g} missing={v['missing']} median lockstep "
             f"{v['median_lockstep']:.0f} ms / DES {v['median_des']:.0f} ms" for k, v in res.items()]
    print(f"\n[{label}]\n  " + "\n  ".join(lines))
    for k, v in res.items():
        assert v["missing"] == 0, f"{label} {k}: runs that never reached it"
        assert v["p"] >= ks.P_MIN, f"{label} {k}: KS D={v['D']:.3f} p={v['p']:.3g} < {ks.P_MIN}"


def lockstep(lib, doc, **kw):
    def one(s):
        if s % 50 == 0:
            print(f"  N={doc['n']} seed {s}/{len(doc['seeds'])}", flush=True)
        return ks.lockstep_sample(lib, doc["n"], s, doc["horizon_ms"], **kw)
    return ks.collect(one, doc["seeds"])


def test_des_config_is_the_lockstep_config():
    """The DES runs the same ClusterConfig the lockstep runs use (preset 0 = reference defaults)."""
    cfg = abi.default_config(oracle.lib(), 0)
    d = des.Des(4, 1).cfg
    assert (d["ping_interval"], d["ping_timeout"], d["ping_req"]) == (
        cfg.ping_interval, cfg.ping_timeout, cfg.ping_req_members)
    assert (d["gossip_interval"], d["fanout"], d["repeat"]) == (
        cfg.gossip_interval, cfg.gossip_fanout, cfg.gossip_repeat_mult)
    assert (d["sync_interval"], d["sync_timeout"], d["suspicion_mult"], d["metadata_timeout"]) == (
        cfg.sync_interval, cfg.sync_timeout, cfg.suspicion_mult, cfg.metadata_timeout)


@pytest.mark.parametrize("n", [64, 1024])
def test_des_fixture_reproduces(n):
    doc, _ = fixture(n)
    for i in (0, 1) if n > 64 else (0, 1, 2, 3):
        live = des.des_sample(n, doc["seeds"][i], doc["horizon_ms"])
        want = doc["samples"][i]
        for k in ks.STATS:
            assert live[k] == pytest.approx(want[k], rel=0, abs=1e-6), (n, doc["seeds"][i], k)


@pytest.mark.parametrize("n", [64, 1024])
def test_ks_oracle_vs_des(n):
    doc, des_s = fixture(n)
    check(ks.compare(lockstep(oracle.lib(), doc, **FAITHFUL), des_s), f"oracle N={n}")


def test_aligned_timers_are_not_reference_timing():
    """Characterisation of the aligned throughput mode: SUSPECT dissemination is measurably slower
    than the reference's (KS rejects at p < 0.01)."""
    doc, des_s = fixture(64)
    res = ks.compare(lockstep(oracle.lib(), doc), des_s)
    assert res["suspect"]["p"] < ks.P_MIN
    assert res["suspect"]["median_lockstep"] > res["suspect"]["median_des"]


@pytest.mark.gpu
@pytest.mark.parametrize("n", [64, 1024])
def test_ks_gpu_vs_des(n):
    import swimgpu
    doc, des_s = fixture(n)
    check(ks.compare(lockstep(swimgpu.load_library(), doc, **FAITHFUL), des_s), f"GPU N={n}")
