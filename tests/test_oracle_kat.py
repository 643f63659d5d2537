"""Pins the CPU oracle against the reference's own known-answer tests.

* MembershipRecordTest.java:34-108 — the isOverrides truth table.
* SequenceIdCollectorTest.java:19-114 — interval-set dedupe.
* ClusterMath values quoted in SURVEY.md §6 / BASELINE.md (ClusterMath.java:65-135).
* Philox4x32-10 known-answer vectors (Random123 kat_vectors), the RNG hook of DESIGN.md §4.

The same KATs run against libswimgpu.so's device code in test_gpu_parity.py.
"""
import json
import os

import pytest

import oracle
from swimgpu import abi
from swimgpu.abi import ALIVE, DEAD, LEAVING, SUSPECT

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
REFERENCE_KATS = json.load(open(os.path.join(GOLDEN, "reference_kats.json")))

# every isOverrides assertion of MembershipRecordTest (transcribed with file:line by
# tests/golden/transcribe_reference_kats.py)
OVERRIDE_CASES = [(tuple(c["r1"]), None if c["r0"] is None else tuple(c["r0"]), c["overrides"])
                  for c in REFERENCE_KATS["MembershipRecordTest"]["cases"]]
# LEAVING rows of the isOverrides logic (MembershipRecord.java:68-87), which the reference's tests
# do not cover: derived from the source, not from an assertion
OVERRIDE_CASES += [((LEAVING, 0), None, True), ((SUSPECT, 3), (LEAVING, 3), True),
                   ((ALIVE, 3), (LEAVING, 3), False), ((LEAVING, 4), (ALIVE, 3), True),
                   ((LEAVING, 3), (ALIVE, 3), False)]


def _override_inputs():
    return [(r1[0], r1[1], r0) for r1, r0, _ in OVERRIDE_CASES], [e for *_, e in OVERRIDE_CASES]


def check_overrides(lib):
    cases, expected = _override_inputs()
    assert abi.kat_overrides(lib, cases) == expected


# SequenceIdCollectorTest, one op list per @Test (expected None: the reference does not assert it)
COLLECTOR_CASES = {
    name: ([(o["op"],) + ((o["value"],) if "value" in o else ()) for o in t["ops"]], [o["expect"] for o in t["ops"]])
    for name, t in REFERENCE_KATS["SequenceIdCollectorTest"]["tests"].items()}


def check_collector(lib):
    for name, (ops, expected) in COLLECTOR_CASES.items():
        got = abi.kat_collector(lib, ops)
        assert [g for g, e in zip(got, expected) if e is not None] == [e for e in expected if e is not None], name


class TreeMapCollector:
    """SequenceIdCollector (SequenceIdCollector.java:43-72) restated over a sorted interval list: the
    model the randomized collector test checks the oracle's and the device's collectors against."""

    def __init__(self):
        self.iv = []  # [lo, hi] ascending, disjoint, non-adjacent

    def _floor(self, x):
        lo, hi, r = 0, len(self.iv) - 1, -1
        while lo <= hi:
            mid = (lo + hi) // 2
            if self.iv[mid][0] <= x:
                r, lo = mid, mid + 1
            else:
                hi = mid - 1
        return r

    def contains(self, x):
        f = self._floor(x)
        return f >= 0 and x <= self.iv[f][1]

    def add(self, x):
        f = self._floor(x)
        if f >= 0 and x <= self.iv[f][1]:
            return False
        c = f + 1
        nf = f >= 0 and x - 1 == self.iv[f][1]
        nc = c < len(self.iv) and x + 1 == self.iv[c][0]
        if nf and nc:
            self.iv[f][1] = self.iv[c][1]
            del self.iv[c]
        elif nf:
            self.iv[f][1] = x
        elif nc:
            self.iv[c][0] = x
        else:
            self.iv.insert(c, [x, x])
        return True


def random_collector_ops(seed, n_ops=6000, span=5000):
    """Random adds / contains / size over [0, span): grows one collector to ~1,200 intervals (every
    spill tier of the device collector) and merges most of them back; a clear half way.  The
    model's own answers are checked against the committed reference KATs (check_collector)."""
    import random
    rng = random.Random(seed)
    ops, model, expected = [], TreeMapCollector(), []
    for i in range(n_ops):
        if i == n_ops // 2:
            ops.append(("clear", 0))
            model.iv = []
            expected.append(0)
            continue
        k = rng.choice((0, 0, 0, 1, 2))
        x = rng.randrange(span) if i < n_ops // 2 else rng.randrange(span // 2)
        ops.append((("add", "contains", "size")[k], x))
        expected.append(int(model.add(x)) if k == 0 else int(model.contains(x)) if k == 1 else len(model.iv))
    return ops, expected


def check_collector_random(lib, seeds=(1, 2)):
    for seed in seeds:
        ops, expected = random_collector_ops(seed)
        got = abi.kat_collector(lib, ops)
        bad = [i for i, (g, e) in enumerate(zip(got, expected)) if g != e]
        assert not bad, f"seed {seed}: first mismatch at op {bad[0]}: {ops[bad[0]]} got {got[bad[0]]} want {expected[bad[0]]}"


PHILOX_KAT = [  # Random123 kat_vectors: philox4x32 10 <ctr> <key> <expected>
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


def check_philox(lib):
    for ctr, key, exp in PHILOX_KAT:
        assert tuple(abi.philox(lib, ctr, key)) == exp


# ClusterMath: N -> (spread, sweep, suspicion s, max msgs/gossip/node) for LAN
CLUSTER_MATH = {3: (6, 14, 10, 18), 1024: (33, 68, 55, 99), 16384: (45, 92, 75, 135),
                65536: (51, 104, 85, 153), 262144: (57, 116, 95, 171)}


def check_cluster_math(lib):
    for n, (spread, sweep, susp_s, msgs) in CLUSTER_MATH.items():
        assert lib.swim_gossip_periods_to_spread(3, n) == spread
        assert lib.swim_gossip_periods_to_sweep(3, n) == sweep
        assert lib.swim_suspicion_timeout(5, n, 1000) == susp_s * 1000
        assert 3 * 3 * lib.swim_ceil_log2(n) == msgs
    assert lib.swim_ceil_log2(0) == 0 and lib.swim_ceil_log2(1) == 1 and lib.swim_ceil_log2(-1) == 32


@pytest.fixture(scope="module")
def olib():
    return oracle.lib()


def test_oracle_overrides_truth_table(olib):
    check_overrides(olib)


def test_oracle_sequence_id_collector(olib):
    check_collector(olib)


def test_treemap_model_matches_reference_kats():
    """The collector model of the randomized test answers every SequenceIdCollectorTest assertion."""
    for name, (ops, expected) in COLLECTOR_CASES.items():
        m, got = TreeMapCollector(), []
        for o in ops:
            if o[0] == "add":
                got.append(int(m.add(o[1])))
            elif o[0] == "contains":
                got.append(int(m.contains(o[1])))
            elif o[0] == "size":
                got.append(len(m.iv))
            else:
                m.iv = []
                got.append(0)
        assert [g for g, e in zip(got, expected) if e is not None] == [e for e in expected if e is not None], name


def test_oracle_collector_random(olib):
    check_collector_random(olib)


def test_oracle_philox_kat(olib):
    check_philox(olib)


def test_oracle_cluster_math(olib):
    check_cluster_math(olib)


def test_oracle_config_presets(olib):
    lan = abi.default_config(olib, 0)
    assert (lan.ping_interval, lan.ping_timeout, lan.ping_req_members) == (1000, 500, 3)
    assert (lan.gossip_interval, lan.gossip_fanout, lan.gossip_repeat_mult) == (200, 3, 3)
    assert (lan.sync_interval, lan.sync_timeout, lan.suspicion_mult, lan.metadata_timeout) == (30000, 3000, 5, 3000)
    wan = abi.default_config(olib, 1)
    assert (wan.ping_interval, wan.ping_timeout, wan.gossip_fanout, wan.suspicion_mult) == (5000, 3000, 4, 6)
    assert (wan.sync_interval, wan.metadata_timeout) == (60000, 10000)
    loc = abi.default_config(olib, 2)
    assert (loc.ping_interval, loc.ping_timeout, loc.ping_req_members) == (1000, 200, 1)
    assert (loc.gossip_interval, loc.gossip_repeat_mult, loc.suspicion_mult, loc.sync_interval) == (100, 2, 3, 15000)
