"""Phase times of k_gossip_emit over the failures window (bench.py's fanout side run: periods 30..36
after the second kill), from the profiling build (tools/phase_prof.sh):

    SWIMGPU_LIB=tools/libswimgpu_prof.so python tools/emit_phases.py [--workload failures]

g_dbg slots 16-23: 16 target selection and per-target setup, 17 the slab passes, 18 their in-window
checks (receipt slot and words, collector probes, loss / delay draws), 19 their materialisation
(inbox reservations and message writes); counts: 20 passes, 21 passes with an in-window state, 22
passes that materialise, 23 senders; setup parts 24 target selection, 25 per-target words.  Times are per-wave sums (100 MHz ticks) divided by the grid's
waves and the launches: each part's share of an average wave's launch."""
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
    e = abi.Engine(lib, cfg, sch.capacity, args.members, 1)
    sch.setup(e)
    sch.run(e, 0, args.warmup)
    torch.cuda.synchronize()
    abi.debug_counters(lib, 32, reset=True)
    e.profile_enable(True)
    sch.run(e, args.warmup, args.warmup + args.steps)
    torch.cuda.synchronize()
    d = abi.debug_counters(lib, 32)
    fp = e.profile_fanout()
    launches = args.steps * 5
    waves = 1024 * 4  # EMIT_GRID x EMIT_WAVES
    per = lambda x: x / 100.0 / waves / launches
    print(json.dumps({"workload": args.workload, "emit_ms_per_launch": fp["total_ms"] / max(1, fp["launches"]),
                      "setup_us": per(d[16]), "passes_us": per(d[17]), "window_check_us": per(d[18]),
                      "materialise_us": per(d[19]), "select_us": per(d[24]), "target_words_us": per(d[25]),
                      "passes": d[20] / launches, "window_passes": d[21] / launches,
                      "mat_passes": d[22] / launches, "senders": d[23] / launches}))


if __name__ == "__main__":
    main()
