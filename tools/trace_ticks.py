"""Dev tool: per-kernel duration and the gap before it, averaged over the last launches of a
rocprofv3 kernel trace (tools/profile.sh output), plus the per-tick total.

    python tools/trace_ticks.py gpurun_out/prof/<tag>_stats [n_last_launches]
"""
import collections
import sqlite3
import sys

con = sqlite3.connect(f"{sys.argv[1]}/run_results.db")
rows = list(con.execute("select name, start, end from kernels order by start"))
rows = rows[-int(sys.argv[2] if len(sys.argv) > 2 else 600):]
gaps, durs = collections.defaultdict(list), collections.defaultdict(list)
for (_, _, e0), (n1, s1, e1) in zip(rows, rows[1:]):
    gaps[n1].append(s1 - e0)
    durs[n1].append(e1 - s1)
ticks = max(1, len(durs.get("k_end_tick", [])))
span = (rows[-1][2] - rows[0][1]) / 1e3
print(f"span {span:.1f} us over {ticks} ticks: {span / ticks:.1f} us/tick")
for k, d in sorted(durs.items(), key=lambda kv: -sum(kv[1])):
    print(f"{k[:28]:28s} n={len(d):4d} avg {sum(d) / len(d) / 1e3:7.2f} us  gap {sum(gaps[k]) / len(d) / 1e3:6.2f} us"
          f"  per tick {sum(d) / ticks / 1e3:7.2f} us")

# per tick (split at k_end_tick): the kernels of each of the last 20 ticks with their durations
if len(sys.argv) > 3:
    tick, out = [], []
    for n, s, e in rows:
        tick.append((n, s, e))
        if n == "k_end_tick":
            out.append(tick)
            tick = []
    for t in out[-int(sys.argv[3]):]:
        span = (t[-1][2] - t[0][1]) / 1e3
        print(f"{span:7.1f} us: " + " ".join(f"{n.replace('k_', '')[:12]}={(e - s) / 1e3:.1f}" for n, s, e in t))
