"""Golden checkpoints of the CPU oracle for BASELINE configs 3 and 5 at the largest sizes whose whole
runs it finishes, written to tests/golden/config_digests.json.

* config5_partition_heal_1024: N = 1,024, seeds {0, N/2}, a 2-way partition [0, N/2) | [N/2, N) from
  period 2, held past the suspicion timeout (each side REMOVEs the other), healed at period 82, run to
  period 122 (the seeds' SYNCs re-join the halves; every view all-ALIVE again); a checkpoint every 10
  periods: the digest of EVERY member's full state (view row, scalars, ping and remote lists in order,
  live gossips), the digest of that stretch's events, every counter.
  (MembershipProtocolTest.java:1035-1109 testNetworkPartitionDueNoOutboundThenRemoved /
  MembershipProtocolImpl.java:339-357,461-472: partition, removal, re-join by SYNC.)
* config5_partition_heal_4096: the same schedule at N = 4,096 (healed at period 92, run to 152), the
  checkpoints over every 64th member and the 8-shard boundaries.
* config3_churn_4096: bench.py's config-3 schedule (5 % uniform loss, 1 % kills + 1 % fresh joins through
  seed 0 per period) at N = 4,096 for 8 periods; a checkpoint every period: the digest of sampled
  members' full state including their SequenceIdCollectors, the period's events, every counter.

The oracle is multi-threaded (identical results for every thread count, tests/test_golden.py).  The
GPU tests (tests/test_gpu_configs.py) run the same schedules unsharded and over 8 in-process shards
and must reproduce every checkpoint.

    python tests/golden/make_config_digests.py [config5|config5b|config3] [THREADS]
"""
import json
import os
import resource
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, REPO)
import conftest  # noqa: F401,E402  (sys.path for swimgpu / oracle)
import bench  # noqa: E402
import oracle  # noqa: E402
import parity  # noqa: E402
from make_scenario_digests import digest, event_digest  # noqa: E402
from swimgpu import abi  # noqa: E402

C5_N, C5_PARTITION, C5_HEAL, C5_END, C5_EVERY = 1024, 2, 82, 122, 10
# config 5 at N = 4,096: held past the suspicion timeout (5 x 12 periods + 30), healed at period 92;
# after the heal the first SYNC across the cut takes ~15-35 periods, so the run goes
# to period 152; a checkpoint every 10 periods over sampled members (every 64th, the 8-shard
# boundaries) — a full readback of 4,096 members' gossips is gigabytes per checkpoint
C5B = {"n": 4096, "heal": 92, "end": 152}
C3_N, C3_PERIODS = 4096, 8


def c5_config(lib, n=C5_N):
    return abi.default_config(lib, 0, sync_stagger=1, record_fd_events=0, gossip_capacity=1 << 19,
                              message_capacity=1 << 28, event_capacity=1 << 26, timer_capacity=max(64 * n, n * n // 2),
                              timer_pool_capacity=n * n // 2 + 64 * n, collector_capacity=1 << (2 * n - 1).bit_length())


def c5_engine(lib, n=C5_N, **cfg_extra):
    cfg = c5_config(lib, n)
    for k, v in cfg_extra.items():
        setattr(cfg, k, v)
    e = abi.Engine(lib, cfg, n, n, 5)
    e.set_seeds([0, n // 2])
    return e


def c5_members(n):
    """the members whose full state a checkpoint digests: all at N = 1,024, else every 64th and the
    8-shard boundaries"""
    if n == C5_N:
        return None
    sz = n // 8
    return sorted(set(list(range(0, n, 64)) + [k * sz + d for k in range(1, 8) for d in (-1, 0)] + [1, n - 1]))


def c5_run(e, on_checkpoint, n=C5_N, heal=C5_HEAL, end=C5_END):
    """the config-5 schedule; on_checkpoint(period, events since the last one) every C5_EVERY periods"""
    side = (np.arange(n) >= n // 2).astype(np.uint16)
    evs = []
    for p in range(end):
        if p == C5_PARTITION:
            e.set_partition(side)
        if p == heal:
            e.set_partition(None)
        e.step(1)
        evs.append(e.drain_events(1 << 26 if n <= C5_N else 1 << 27))
        if (p + 1) % C5_EVERY == 0 or p + 1 == end:
            on_checkpoint(p + 1, np.concatenate(evs))
            evs = []


def c3_members(sch_ops0):
    killed = [m for op, m in sch_ops0 if op == "kill"][:6]
    joined = [m for op, m in sch_ops0 if op == "join"][:6]
    return sorted(set([0, 1, 2, 1000, 2048, C3_N - 1] + killed + joined + [C3_N + 3, C3_N + 41]))


def c3_engine(lib, **cfg_extra):
    sch = bench.Schedule("churn", C3_N, C3_PERIODS)
    members = c3_members(bench.Schedule("churn", C3_N, C3_PERIODS).ops(0))
    cfg = bench.churn_capacities(bench.make_config(lib), sch.capacity)
    for k, v in cfg_extra.items():
        setattr(cfg, k, v)
    e = abi.Engine(lib, cfg, sch.capacity, C3_N, 1)
    sch.setup(e)
    return e, sch, members


def checkpoint(e, events, members, collectors):
    st = e.stats()
    return {"state_sha256": digest(e, members, collectors), "events_sha256": event_digest(events),
            "events": int(len(events)), "stats": {k: int(st[k]) for k in parity.STAT_FIELDS}}


def make_c5(threads):
    e = c5_engine(oracle.lib())
    oracle.set_threads(e, threads)
    out = {}
    t0 = time.time()

    def on(p, ev):
        out[str(p)] = checkpoint(e, ev, None, False)
        print(f"config5 period {p}: {len(ev)} events, {time.time() - t0:.0f} s, "
              f"maxrss {resource.getrusage(resource.RUSAGE_SELF).ru_maxrss >> 20} GB", flush=True)
    c5_run(e, on)
    return {"n": C5_N, "partition_period": C5_PARTITION, "heal_period": C5_HEAL, "periods": C5_END,
            "members": "all", "collectors": False, "checkpoints": out}


def make_c5b(threads):
    n = C5B["n"]
    e = c5_engine(oracle.lib(), n)
    oracle.set_threads(e, threads)
    members = c5_members(n)
    out = {}
    t0 = time.time()

    def on(p, ev):
        out[str(p)] = checkpoint(e, ev, members, False)
        print(f"config5 N={n} period {p}: {len(ev)} events, {time.time() - t0:.0f} s, "
              f"maxrss {resource.getrusage(resource.RUSAGE_SELF).ru_maxrss >> 20} GB", flush=True)
    c5_run(e, on, n, C5B["heal"], C5B["end"])
    return {"n": n, "partition_period": C5_PARTITION, "heal_period": C5B["heal"], "periods": C5B["end"],
            "members": members, "collectors": False, "checkpoints": out}


def make_c3(threads):
    e, sch, members = c3_engine(oracle.lib())
    oracle.set_threads(e, threads)
    out = {}
    t0 = time.time()
    for p in range(C3_PERIODS):
        sch.run(e, p, p + 1)
        ev = e.drain_events(1 << 27)
        out[str(p + 1)] = checkpoint(e, ev, members, True)
        print(f"config3 period {p + 1}: {len(ev)} events, {time.time() - t0:.0f} s, "
              f"maxrss {resource.getrusage(resource.RUSAGE_SELF).ru_maxrss >> 20} GB", flush=True)
        json.dump({"partial": out}, open(os.path.join(HERE, ".config3_partial.json"), "w"))
    return {"n": C3_N, "periods": C3_PERIODS, "members": members, "collectors": True, "checkpoints": out}


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "all"
    threads = int(sys.argv[2]) if len(sys.argv) > 2 else (os.cpu_count() or 1)
    path = os.path.join(HERE, "config_digests.json")
    doc = json.load(open(path)) if os.path.exists(path) else {
        "source": "tests/golden/make_config_digests.py (CPU oracle)", "runs": {}}
    if which in ("all", "config5"):
        doc["runs"]["config5_partition_heal_1024"] = make_c5(threads)
        json.dump(doc, open(path, "w"), indent=1, sort_keys=True)
    if which in ("all", "config5b"):
        doc["runs"]["config5_partition_heal_4096"] = make_c5b(threads)
        json.dump(doc, open(path, "w"), indent=1, sort_keys=True)
    if which in ("all", "config3"):
        doc["runs"]["config3_churn_4096"] = make_c3(threads)
        json.dump(doc, open(path, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
