"""Summarise tools/profile.sh output (rocprofv3 SQLite databases) into committed profile files.

    python tools/prof_summary.py gpurun_out/prof/<tag> profiles/<round>_<tag> [STEPS WARMUP]

writes <out>_kernel_stats.csv (per-kernel calls / total / average / share, from the kernel-trace
pass) and <out>_pmc.json (per-kernel, per-launch HBM bytes from the separate FETCH_SIZE and
WRITE_SIZE passes; per kernel also the bytes of each launch and of its last, and the profiled bench command's
--steps / --warmup, so that bench.py attaches traffic only to the window of the same length).  Corrections follow /opt/skills/guides/MI355X_MICROARCH.md §HBM: FETCH_SIZE is
in KiB and on gfx950 reports exactly half the bytes of a wide (16 B / lane) coalesced streaming
read, so it is doubled; WRITE_SIZE (KiB) is exact for 16-B-per-lane streaming stores.
"""
import csv
import json
import sqlite3
import sys


def _db(path):
    return sqlite3.connect(f"{path}/run_results.db")


def kernel_stats(prefix):
    con = _db(f"{prefix}_stats")
    rows = list(con.execute("select name, total_calls, total_duration, average, percentage from top_kernels"))
    return [{"name": r[0], "calls": int(r[1]), "total_us": float(r[2]), "avg_us": float(r[3]), "pct": float(r[4])}
            for r in rows]


def pmc(prefix, which):
    con = _db(f"{prefix}_{which}")
    q = ("select kernel_name, counter_name, count(*), avg(value) from counters_collection "
         "group by kernel_name, counter_name")
    return {(r[0], r[1]): (int(r[2]), float(r[3])) for r in con.execute(q)}


def pmc_last(prefix, which):
    """per kernel, the counter value of its LAST dispatch (the bench's timed window is the last one)"""
    con = _db(f"{prefix}_{which}")
    q = "select kernel_name, value from counters_collection order by dispatch_id"
    last = {}
    for name, v in con.execute(q):
        last[name] = float(v)
    return last


def pmc_all(prefix, which):
    """per kernel, the counter value of each dispatch in dispatch order"""
    con = _db(f"{prefix}_{which}")
    out = {}
    for name, v in con.execute("select kernel_name, value from counters_collection order by dispatch_id"):
        out.setdefault(name, []).append(float(v))
    return out


def main(src, out):
    ks = kernel_stats(src)
    with open(f"{out}_kernel_stats.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "calls", "total_us", "avg_us", "pct"])
        for k in ks:
            w.writerow([k["name"], k["calls"], f"{k['total_us']:.3f}", f"{k['avg_us']:.3f}", f"{k['pct']:.3f}"])
    fetch, write = pmc(src, "fetch"), pmc(src, "write")
    per = {}
    for (name, ctr), (n, avg) in fetch.items():
        per.setdefault(name, {})["fetch_bytes_per_launch"] = 2.0 * avg * 1024.0
        per[name]["launches_fetch_pass"] = n
    for (name, ctr), (n, avg) in write.items():
        per.setdefault(name, {})["write_bytes_per_launch"] = avg * 1024.0
    for v in per.values():
        v["hbm_bytes_per_launch"] = v.get("fetch_bytes_per_launch", 0.0) + v.get("write_bytes_per_launch", 0.0)
    lf, lw = pmc_last(src, "fetch"), pmc_last(src, "write")
    for name, v in per.items():
        if name in lf and name in lw:
            v["last_launch_hbm_bytes"] = 2.0 * lf[name] * 1024.0 + lw[name] * 1024.0
    # every launch in dispatch order (bench.py picks the timed window's by its index: the launches
    # before it are the warm-up's, the ones after it the window-model side run's)
    af, aw = pmc_all(src, "fetch"), pmc_all(src, "write")
    for name, v in per.items():
        if name in af and name in aw and len(af[name]) == len(aw[name]):
            v["launch_hbm_bytes"] = [2.0 * f * 1024.0 + w * 1024.0 for f, w in zip(af[name], aw[name])]
    doc = {"source": src, "correction": "FETCH_SIZE KiB x 1024 x 2 (gfx950 half-count of 16-B/lane streaming "
                                        "reads, MI355X_MICROARCH.md HBM); WRITE_SIZE KiB x 1024",
           "kernels": per}
    if len(sys.argv) > 4:  # the profiled bench command's window: --steps, --warmup
        doc["bench_args"] = {"steps": int(sys.argv[3]), "warmup": int(sys.argv[4])}
    with open(f"{out}_pmc.json", "w") as f:
        json.dump(doc, f, indent=1, sort_keys=True)
    for k in ks[:12]:
        extra = per.get(k["name"], {})
        print(f"{k['name']:>24} calls {k['calls']:5d} avg {k['avg_us']:9.2f} us  "
              f"hbm/launch {extra.get('hbm_bytes_per_launch', 0) / 1e6:9.2f} MB")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
