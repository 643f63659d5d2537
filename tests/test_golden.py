"""Golden fixtures (tests/golden/): the reference's transcribed known-answer tests and the oracle's
per-scenario regression digests.

* reference_kats.json — every assertion of MembershipRecordTest / SequenceIdCollectorTest, with its
  source line (transcribe_reference_kats.py); test_oracle_kat.py and the GPU KAT tests run them.
* scenario_digests.json — sha256 of the final state, of the canonical event stream and the
  counters of every parity scenario as the CPU oracle produces them (make_scenario_digests.py).
  The GPU engine, sharded or not, must reproduce them (test_gpu_parity.py).
"""
import json
import os

import pytest

import oracle
import scenarios
from make_scenario_digests import run as oracle_run

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
DIGESTS = json.load(open(os.path.join(GOLDEN, "scenario_digests.json")))["scenarios"]


def test_reference_kats_cover_every_assertion():
    d = json.load(open(os.path.join(GOLDEN, "reference_kats.json")))
    assert len(d["MembershipRecordTest"]["cases"]) == 33  # 3 x 10 override tables + 3 equal records
    tests = d["SequenceIdCollectorTest"]["tests"]
    assert set(tests) == {"testEmpty", "testOneElement", "testIsHeldNotExistedElements", "testAddExistedElement",
                          "testClear", "testLowestAndHighestElementInRange", "testJoinLowerRange",
                          "testJoinUpperRange", "testJoinTwoRange"}


@pytest.mark.parametrize("sc", scenarios.catalog(), ids=lambda s: s.name)
def test_oracle_reproduces_scenario_digest(sc):
    assert oracle_run(sc) == DIGESTS[sc.name]


def test_oracle_reproduces_config2_digest():
    sc = scenarios.config2()
    assert oracle_run(sc, members=scenarios.CONFIG2_MEMBERS, collectors=False) == DIGESTS[sc.name]


# the CPU baseline's multi-threaded oracle (std::thread workers over member ranges in every phase)
# must reproduce the same digests as the sequential loops
@pytest.mark.parametrize("name", ["loss5_kills_64", "churn_48", "join_burst_seg", "config3_rates_200",
                                  "partition_heal_32", "mp_joins_via_seed"])
def test_threaded_oracle_reproduces_scenario_digest(name):
    sc = {s.name: s for s in scenarios.catalog()}[name]
    assert oracle_run(sc, threads=4) == DIGESTS[sc.name]


def test_origination_reasons_partition_gossips_created():
    """swim_stats.gossips_by_reason (SWIM_ORIG_*) splits gossips_created by call site, exactly."""
    for name, d in DIGESTS.items():
        st = d["stats"]
        assert sum(v for k, v in st.items() if k.startswith("orig_")) == st["gossips_created"], name
