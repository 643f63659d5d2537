"""Volume probe for BASELINE configs 3 and 5 at a given N (run on the GPU box).

    python tools/config_probe.py partition --members 4096 [--hold P] [--after P]
    python tools/config_probe.py churn --members 16384 --periods 6

partition (config 5): seeds {0, N/2}; 2-way partition [0, N/2) | [N/2, N) from period 2, held past the
suspicion timeout (5 x ceil_log2(N) periods + 5), then healed; runs `--after` periods more.  churn
(config 3): bench.py's churn schedule.  One line per period: gossips created, GOSSIP_REQs sent, SYNCs,
events, the largest live-gossip count of a sampled member, wall time.  At the end of a partition run:
how many sampled members see every member ALIVE again.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "scalecube-cluster_amd"))
sys.path.insert(0, REPO)


def converged(e, sample):
    ok = 0
    for m in sample:
        row = e.read_view(m)
        ok += int((((row >> 34) & 1) == 1).all() and (((row >> 32) & 3) == 0).all())
    return ok


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("workload", choices=("partition", "churn"))
    ap.add_argument("--members", type=int, default=4096)
    ap.add_argument("--periods", type=int, default=6)
    ap.add_argument("--hold", type=int, default=None)
    ap.add_argument("--after", type=int, default=40)
    ap.add_argument("--stop-converged", action="store_true", help="partition: stop once the sample has converged")
    ap.add_argument("--gossip-capacity", type=int, default=1 << 17)
    ap.add_argument("--sample", type=int, default=16)
    ap.add_argument("--interval-capacity", type=int, default=1024)
    ap.add_argument("--collectors", action="store_true",
                    help="per period: collector sizes at member sample[1] (gossipers of its live gossips)")
    ap.add_argument("--message-capacity", type=int, default=1 << 28)
    ap.add_argument("--deliver", action="store_true",
                    help="per period: sampled k_gossip_deliver profile (ms / launch, messages, not flagged, accepted)")
    args = ap.parse_args()
    import swimgpu
    from swimgpu import abi
    import bench
    lib = swimgpu.load_library()
    n = args.members
    cfg = abi.default_config(lib, 0, sync_stagger=1, record_fd_events=0)
    cfg.gossip_capacity = args.gossip_capacity
    cfg.event_capacity = 1 << 26
    cfg.message_capacity = args.message_capacity
    cfg.collector_capacity = 1 << (2 * n - 1).bit_length()
    cfg.interval_capacity = args.interval_capacity
    # a partition puts a suspicion timer for every member of the other side at every viewer, falling
    # due within the few ticks the SUSPECT gossip took to spread
    cfg.timer_capacity = max(64 * n, n * n // 2)
    cfg.timer_pool_capacity = n * n // 2 + 64 * n  # N/2 pending timers at every viewer
    sample = [int(x) for x in np.linspace(0, n - 1, args.sample)]
    if args.workload == "churn":
        sch = bench.Schedule("churn", n, args.periods)
        cfg.collector_capacity = 1 << (2 * sch.capacity - 1).bit_length()
        cfg.timer_capacity = 64 * sch.capacity
        cfg.timer_pool_capacity = 1 << 28 if sch.capacity > 12288 else 1 << 27
        e = abi.Engine(lib, cfg, sch.capacity, n, 1)
        sch.setup(e)
        plan = [(p, sch.ops(p)) for p in range(args.periods)]
    else:
        e = abi.Engine(lib, cfg, n, n, 1)
        e.set_seeds([0, n // 2])
        hold = args.hold if args.hold is not None else 5 * n.bit_length() + 5
        groups = np.zeros(n, dtype=np.uint16)
        groups[n // 2:] = 1
        heal = 2 + hold
        plan = []
        for p in range(heal + args.after):
            ops = []
            if p == 2:
                ops.append(("partition", groups))
            if p == heal:
                ops.append(("partition", None))
            plan.append((p, ops))
    if args.deliver:
        e.profile_enable(True)
    t0 = time.time()
    prev = e.stats()
    ev_total = 0
    for p, ops in plan:
        for op, arg in ops:
            if op == "partition":
                e.set_partition(arg)
            else:
                getattr(e, op)(arg)
        t1 = time.time()
        try:
            e.step(1)
        except abi.SwimError as ex:
            print(json.dumps({"period": p + 1, "error": str(ex)}), flush=True)
            return 1
        ev = e.drain_events()
        ev_total += len(ev)
        st = e.stats()
        glen = max(e.read_member(m)["gossip_len"] for m in sample)
        print(json.dumps({"period": p + 1, "s": round(time.time() - t1, 3),
                          "gossips": st["gossips_created"] - prev["gossips_created"],
                          "by_reason": {r: st[f"orig_{r}"] - prev[f"orig_{r}"] for r in abi.ORIG_REASONS
                                        if st[f"orig_{r}"] != prev[f"orig_{r}"]},
                          "msgs": st["gossip_messages"] - prev["gossip_messages"],
                          "syncs": st["syncs"] - prev["syncs"], "events": len(ev),
                          "removed": int((ev["type"] == abi.EV_REMOVED).sum()) if len(ev) else 0,
                          "max_live_gossips": glen}), flush=True)
        prev = st
        if args.deliver:
            d = e.profile_deliver()
            n_l = max(1, d["launches"])
            print(json.dumps({"deliver_ms_per_launch": round(d["total_ms"] / n_l, 3), "launches": d["launches"],
                              "msgs": d["messages"], "fresh": d["alg_bytes"] // 24 - d["messages"],
                              "accepted": d["records"]}), flush=True)
            e.profile_enable(False)
            e.profile_enable(True)
        if args.collectors:
            m = sample[1]
            gs = e.read_gossips(m)
            ids, cnt = np.unique(gs["gossiper"], return_counts=True) if len(gs) else ([], [])
            sizes = sorted(((len(e.read_collector(m, int(g))), int(g), int(c)) for g, c in zip(ids, cnt)),
                           reverse=True)[:5]
            print(json.dumps({"member": m, "gossipers": len(ids), "top_collectors(intervals,gossiper,live)": sizes}),
                  flush=True)
        if args.workload == "partition" and args.stop_converged and p + 1 > heal and converged(e, sample) == len(sample):
            print(json.dumps({"converged_at_period": p + 1}), flush=True)
            break
    if args.workload == "partition":
        ok = 0
        for m in sample:
            row = e.read_view(m)
            st = (row >> 32) & 3
            intab = (row >> 34) & 1
            ok += int(intab.all() and (st == 0).all())
        st = e.stats()
        print(json.dumps({"converged_sampled": ok, "sampled": len(sample), "wall_s": round(time.time() - t0, 1),
                          "events_total": ev_total, "capacity_errors": st["capacity_errors"],
                          "gossips_by_reason": {r: st[f"orig_{r}"] for r in abi.ORIG_REASONS}}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
