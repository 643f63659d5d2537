"""Summarise tools/prof_driver.sh output (rocprofv3 SQLite databases of ONE bench command) into the
committed profile files bench.py attaches to its line.

    python tools/prof_summary.py gpurun_out/prof/<tag> profiles/<round>_<name>

writes
* <out>_kernel_stats.csv: per kernel calls / total / average / share (the kernel-trace pass);
* <out>_pmc.json: HBM bytes per launch from the memory-side request counters, for every launch of
  the kernels bench.py reports, per ENGINE of the command (an engine starts at a k_init_members
  dispatch: the headline's engine is #0, then the side runs in bench.py's order), with the
  kernel-trace duration of each launch; plus the profiled command's `bench_key` and build (the
  source hash of lib/libswimgpu.so), both from its own JSON line.  bench.py uses a profile only for a
  run with the same key and build.

Bytes.  The passes collect the raw memory-side (TCC -> fabric) request counters by size instead of
the derived FETCH_SIZE / WRITE_SIZE: read bytes = 32 x TCC_EA0_RDREQ_32B + 64 x TCC_EA0_RDREQ_64B +
128 x TCC_EA0_RDREQ_128B, write bytes = 64 x TCC_EA0_WRREQ_64B + 32 x (TCC_EA0_WRREQ - TCC_EA0_WRREQ_64B).
tools/gatherbench.hip + tools/calibrate_pmc.sh (profiles/r06_pmc_calibration.json) checked these
against known line counts: a coalesced 16 B / lane stream and a random 4-, 8- or 16-B gather each
issue 128-B read requests (FETCH_SIZE tallies every read request at 64 B, so its gfx950 x2
correction is right for both); a random 4-B store, 4-B atomic or 32-B store is one 32-B write request
(WRITE_SIZE exact).
"""
import csv
import json
import sqlite3
import sys
import time

TRACKED = ("k_quiet_apply", "k_quiet_scan", "k_gossip_emit", "k_deliver_coop", "k_gossip_deliver", "k_sync_apply",
           "k_ack_apply", "k_fd", "k_end_tick", "k_sync_classify")
READ_SIZES = {"TCC_EA0_RDREQ_32B": 32.0, "TCC_EA0_RDREQ_64B": 64.0, "TCC_EA0_RDREQ_128B": 128.0}


def _db(path):
    return sqlite3.connect(f"{path}/run_results.db")


def short(name):
    return name.split("(")[0].strip()


def kernel_stats(prefix):
    con = _db(f"{prefix}_stats")
    rows = list(con.execute("select name, total_calls, total_duration, average, percentage from top_kernels"))
    return [{"name": short(r[0]), "calls": int(r[1]), "total_us": float(r[2]), "avg_us": float(r[3]),
             "pct": float(r[4])} for r in rows]


def segments(names):
    """engine index of each dispatch: a new engine starts at a k_init_members dispatch that follows
    some non-init kernel (the shards of one engine initialise back to back)"""
    eng, seen_work, out = -1, True, []
    for nm in names:
        if nm == "k_init_members":
            if seen_work:
                eng += 1
            seen_work = False
        elif not nm.startswith("k_init"):
            seen_work = True
        out.append(max(0, eng))
    return out


def trace_launches(prefix):
    con = _db(f"{prefix}_stats")
    rows = list(con.execute("select name, dispatch_id, duration from kernels order by dispatch_id"))
    names = [short(r[0]) for r in rows]
    per = {}
    for (nm, eng), (_, _, dur) in zip(zip(names, segments(names)), rows):
        if nm in TRACKED:
            per.setdefault(eng, {}).setdefault(nm, []).append(float(dur) / 1e3)
    return per


def pmc_launches(prefix, which):
    """per engine, per tracked kernel: the bytes of each dispatch in order"""
    con = _db(f"{prefix}_{which}")
    rows = list(con.execute("select dispatch_id, kernel_name, counter_name, sum(value) from counters_collection "
                            "group by dispatch_id, counter_name order by dispatch_id"))
    disp = {}
    order = []
    for did, kn, ctr, v in rows:
        if did not in disp:
            disp[did] = (short(kn), {})
            order.append(did)
        disp[did][1][ctr.replace("_sum", "")] = float(v)
    names = [disp[d][0] for d in order]
    per = {}
    for did, eng in zip(order, segments(names)):
        nm, c = disp[did]
        if nm not in TRACKED:
            continue
        if which == "rd":
            b = sum(READ_SIZES[k] * c.get(k, 0.0) for k in READ_SIZES)
        else:
            n64 = c.get("TCC_EA0_WRREQ_64B", 0.0)
            b = 64.0 * n64 + 32.0 * (c.get("TCC_EA0_WRREQ", 0.0) - n64)
        per.setdefault(eng, {}).setdefault(nm, []).append(b)
    return per


def bench_line(prefix):
    try:
        for line in open(f"{prefix}_stats.log"):
            if line.startswith("{"):
                return json.loads(line)
    except OSError:
        pass
    return None


def main(src, out):
    ks = kernel_stats(src)
    with open(f"{out}_kernel_stats.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "calls", "total_us", "avg_us", "pct"])
        for k in ks:
            w.writerow([k["name"], k["calls"], f"{k['total_us']:.3f}", f"{k['avg_us']:.3f}", f"{k['pct']:.3f}"])
    tr, rd, wr = trace_launches(src), pmc_launches(src, "rd"), pmc_launches(src, "wr")
    engines = []
    for eng in range(max([*tr, *rd, *wr, -1]) + 1):
        kk = {}
        for nm in TRACKED:
            r, w_ = rd.get(eng, {}).get(nm), wr.get(eng, {}).get(nm)
            if not r or not w_:
                continue
            m = min(len(r), len(w_))  # (a time-budgeted tail may differ between passes; never the timed launches)
            kk[nm] = {"fetch_bytes": r[:m], "write_bytes": w_[:m], "hbm_bytes": [a + b for a, b in zip(r[:m], w_[:m])],
                      "us": tr.get(eng, {}).get(nm, []), "launches_per_pass": [len(r), len(w_)]}
        engines.append(kk)
    line = bench_line(src)
    build = line.get("build") if line else None  # the build the profiled command ran (bench.py build_hash)
    doc = {"source": src, "created": time.strftime("%Y-%m-%dT%H:%M:%S"), "build": build,
           "bench_key": line.get("bench_key") if line else None,
           "bench_value": line.get("value") if line else None,
           "bytes": "read = 32 x RDREQ_32B + 64 x RDREQ_64B + 128 x RDREQ_128B; write = 64 x WRREQ_64B + 32 x the "
                    "other WRREQ (TCC_EA0 memory-side requests; calibration: profiles/r06_pmc_calibration.json)",
           "engines": engines}
    with open(f"{out}_pmc.json", "w") as f:
        json.dump(doc, f, indent=0, sort_keys=True)
    for k in ks[:14]:
        print(f"{k['name']:>24} calls {k['calls']:6d} avg {k['avg_us']:10.2f} us")
    for i, e in enumerate(engines):
        print(f"engine {i}: " + ", ".join(f"{k} x{len(v['hbm_bytes'])} {sum(v['hbm_bytes']) / len(v['hbm_bytes']) / 1e6:.2f} MB"
                                        for k, v in e.items()))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
