"""tools/calibrate_pmc.sh output (rocprofv3 databases of tools/gatherbench) -> the counters' tally per
access of each known access shape, as committed in profiles/<round>_pmc_calibration.json.

    python tools/gatherbench_summary.py gpurun_out/cal profiles/r06_pmc_calibration.json
"""
import glob
import json
import os
import re
import sqlite3
import sys

# accesses per launch of each calibration kernel (tools/gatherbench.hip)
ACCESSES = {"k_cal_stream16": 1 << 30, "k_cal_gather4": 1 << 24, "k_cal_gather8": 1 << 24, "k_cal_gather16": 1 << 24,
            "k_cal_wave256": (1 << 24) // 64, "k_cal_atomic4": 1 << 24, "k_cal_store4": 1 << 24,
            "k_cal_store32": 1 << 24}
UNIT = {"k_cal_stream16": "byte", "k_cal_wave256": "wave (256 contiguous bytes)"}


def per_launch(db):
    con = sqlite3.connect(db)
    rows = con.execute("select kernel_name, counter_name, dispatch_id, sum(value) from counters_collection "
                       "group by dispatch_id, counter_name order by dispatch_id")
    out = {}
    for k, c, _, v in rows:
        out.setdefault((k.split("(")[0].strip(), c.replace("_sum", "")), []).append(float(v))
    return out


def main(src, dst):
    res = {}
    for db in sorted(glob.glob(os.path.join(src, "*", "run_results.db"))):
        for (k, c), vs in per_launch(db).items():
            if k not in ACCESSES:
                continue
            med = sorted(vs)[len(vs) // 2]
            unit = 1024.0 if c in ("FETCH_SIZE", "WRITE_SIZE") else 1.0  # (KiB)
            res.setdefault(k, {"accesses_per_launch": ACCESSES[k], "access": UNIT.get(k, "access")})
            res[k][c + ("_bytes_per_access" if unit > 1 else "_per_access")] = med * unit / ACCESSES[k]
    rates = {}
    plain = os.path.join(src, "plain.log")
    if os.path.exists(plain):
        for line in open(plain):
            m = re.match(r"(\S+) accesses=(\S+) us=(\S+) accesses_per_s=(\S+)", line)
            if m:
                rates[m.group(1)] = {"us": float(m.group(3)), "accesses_per_s": float(m.group(4))}
    for k, v in rates.items():
        if k in res:
            res[k].update(v)
    doc = {"tool": "tools/gatherbench.hip via tools/calibrate_pmc.sh (rocprofv3 --pmc, one counter set per pass)",
           "kernels": res,
           "reading": "FETCH_SIZE tallies 64 B per memory-side read request (TCC_EA0_RDREQ); the requests of a "
                      "coalesced 16-B/lane stream AND of random 4-, 8- or 16-B gathers are 128 B each, so FETCH_SIZE "
                      "x 2 is the read traffic of both shapes; every random 4-B store, 4-B atomic and 32-B store is "
                      "one 32-B write request (TCC_EA0_WRREQ, none 64-B), which WRITE_SIZE counts exactly"}
    with open(dst, "w") as f:
        json.dump(doc, f, indent=1, sort_keys=True)
    for k, v in res.items():
        print(k, {a: (round(b, 2) if isinstance(b, float) else b) for a, b in v.items()})


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
