"""Per-launch time and HBM bytes of one kernel over the LAST `k` launches of a tools/window_prof.sh
run (the bench's timed window), from the kernel-trace pass and the separate FETCH_SIZE / WRITE_SIZE
passes (corrections of /opt/skills/guides/MI355X_MICROARCH.md §HBM: FETCH_SIZE KiB x 2 on gfx950
for 16-B/lane streaming reads, WRITE_SIZE KiB exact).

    python tools/window_summary.py gpurun_out/prof/<tag> k_gossip_emit 30 > profiles/<out>.json
"""
import json
import sqlite3
import sys


def last_dispatches(db, kernel, k, table, cols):
    con = sqlite3.connect(f"{db}/run_results.db")
    q = f"select {cols} from {table} where {'name' if table == 'kernels' else 'kernel_name'} like ? order by dispatch_id"
    rows = list(con.execute(q, (kernel + "%",)))
    return rows[-k:]


def main():
    # kernel: one name, or several joined by '+' (one launch of each per round, e.g. the delivery pair
    # k_deliver_coop+k_gossip_deliver): times and bytes are summed per round
    prefix, kernel, k = sys.argv[1], sys.argv[2], int(sys.argv[3])
    names = kernel.split("+")
    ts = [last_dispatches(f"{prefix}_stats", kn, k, "kernels", "dispatch_id, duration") for kn in names]
    out = {"kernel": kernel, "launches": min(len(t) for t in ts), "window": f"last {k} launches of the run",
           "avg_us": sum(sum(r[1] for r in t) / max(1, len(t)) for t in ts) / 1e3}
    con_f = sqlite3.connect(f"{prefix}_fetch/run_results.db")
    con_w = sqlite3.connect(f"{prefix}_write/run_results.db")

    def per_launch(con, counter):
        tot, n = 0.0, None
        for kn in names:
            rows = list(con.execute("select dispatch_id, sum(value) from counters_collection where kernel_name like ? "
                                    "and counter_name = ? group by dispatch_id order by dispatch_id", (kn + "%", counter)))
            rows = rows[-k:]
            tot += sum(r[1] for r in rows) / max(1, len(rows))
            n = len(rows) if n is None else min(n, len(rows))
        return tot, n

    fetch_kib, nf = per_launch(con_f, "FETCH_SIZE")
    write_kib, nw = per_launch(con_w, "WRITE_SIZE")
    out.update({"fetch_bytes_per_launch": fetch_kib * 1024 * 2, "write_bytes_per_launch": write_kib * 1024,
                "hbm_bytes_per_launch": fetch_kib * 1024 * 2 + write_kib * 1024, "pmc_launches": [nf, nw],
                "correction": "FETCH_SIZE KiB x 1024 x 2 (gfx950 half count of 16-B/lane streaming reads), "
                              "WRITE_SIZE KiB x 1024"})
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
