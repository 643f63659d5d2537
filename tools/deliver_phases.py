"""Phase times of k_gossip_deliver over the failures window (bench.py's fanout side run: periods
30..36 after the second kill), from the profiling build (tools/phase_prof.sh):

    SWIMGPU_LIB=tools/libswimgpu_prof.so python tools/deliver_phases.py [--workload failures]

g_dbg slots: 0 big-inbox ranking, 1 big-inbox onGossipReq chains, 2 big-inbox tail (page reset,
pingMembers inserts, SYNC collection), 3 small inboxes + their collection (every wave), 4 batches,
5 big inboxes, 6/7 whole-wave serial / accepted lanes, 8-9 onGossipReq sections (slab, updateMembership), 13-15 whole-wave chunk parts.  Times are per-wave sums (100 MHz ticks); divided by the waves of a launch they give
each part's share of a launch."""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "scalecube-cluster_amd"))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="failures")
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--members", type=int, default=65536)
    args = ap.parse_args()
    import torch
    import swimgpu
    from swimgpu import abi
    import bench
    lib = swimgpu.load_library()
    sch = bench.Schedule(args.workload, args.members, args.warmup + args.steps)
    cfg = bench.make_config(lib)
    if args.workload == "churn":
        bench.churn_capacities(cfg, sch.capacity)
    e = abi.Engine(lib, cfg, sch.capacity, args.members, 1)
    sch.setup(e)
    sch.run(e, 0, args.warmup)
    torch.cuda.synchronize()
    abi.debug_counters(lib, reset=True)
    e.profile_enable(True)
    t0 = time.perf_counter()
    sch.run(e, args.warmup, args.warmup + args.steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    d = abi.debug_counters(lib, 64)
    dp = e.profile_deliver()
    launches = args.steps * 5  # gossip rounds in the window
    waves = 512 * 4  # DLV_GRID x DLV_WAVES
    per = lambda x: x / 100.0 / waves / launches  # us of an average wave per launch
    print(json.dumps({"workload": args.workload, "window_s": dt, "deliver_ms_per_launch": dp["total_ms"] / max(1, dp["launches"]),
                      "big_rank_us": per(d[0]), "big_chain_us": per(d[1]), "big_tail_us": per(d[2]),
                      "small_and_collect_us": per(d[3]), "batches": d[4], "big_inboxes": d[5],
                      # onGossipReq sections (every path; wave time, first active lane): collector
                      # ensure + add, receipt mark, slab put + index, updateMembership
                      "coop_serial_lanes": d[6], "coop_accepted": d[7], "ogr_slab_us": per(d[8]),
                      "ogr_update_us": per(d[9]),
                      # whole-wave delivery (deliver_coop) per chunk: (a) loads + collectors,
                      # (b) receipts + no-op test, (c) the serial steps and state writes
                      "coop_a_us": per(d[13]),
                      # (a)'s parts: message loads wait, gossiper grouping, coll_ensure_wave,
                      # ensure + coll_add loop; leaders (distinct gossipers) per launch
                      "coop_a_msgwait_us": per(d[29]), "coop_a_group_us": per(d[26]),
                      "coop_a_ensure_us": per(d[27]), "coop_a_ensure_add_us": per(d[28]),
                      "coop_leaders": d[30] / launches, "coop_probe_rounds": d[31] / launches,
                      # the staged collector pass: stage-in, the leader's adds, the copy back; staged
                      # collectors, their intervals and the intervals the adds shifted, per launch
                      "stage_in_us": per(d[32]), "stage_adds_us": per(d[33]), "stage_out_us": per(d[34]),
                      "staged": d[35] / launches, "staged_intervals": d[36] / launches,
                      "staged_shifted": d[37] / launches,
                      # small collectors (<= 64 intervals) in registers: time, count
                      "reg_pass_us": per(d[38]), "reg_staged": d[39] / launches, "coop_b_us": per(d[14]), "coop_c_us": per(d[15]),
                      # (c)'s lanes that take the chain's onGossipReq; slab-index rebuilds by a whole wave
                      "coop_full_lanes": d[47] / launches, "gix_wave_rebuilds": d[53] / launches,
                      "gix_rebuild_us": per(d[54]),
                      # (c)'s parts: no-op blocks (and their index notes), serial steps of the chain's
                      # onGossipReq lanes and of the others
                      "c_noop_us": per(d[49]), "c_noop_gix_notes": d[48] / launches, "c_full_us": per(d[50]),
                      "c_serial_us": per(d[51]),
                      # the big-inbox tail: pingMembers inserts applied (per launch), receivers with
                      # inserts, their lists' mean length, the largest batch, insert and collection times
                      "tail_inserts": d[41] / launches, "tail_ins_receivers": d[43] / launches,
                      "tail_ins_mean_list": d[44] / max(1, d[43]), "tail_ins_max": d[42],
                      "tail_ins_us": per(d[45]), "tail_collect_us": per(d[46]),
                      "longest_chain_msgs": d[10], "chain_msgs_per_launch": d[11] / launches,
                      "sum_of_wave_longest_chains": d[12] / launches,
                      "messages_per_launch": dp["messages"] / max(1, dp["launches"])}))


if __name__ == "__main__":
    main()
