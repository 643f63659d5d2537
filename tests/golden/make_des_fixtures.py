"""Generate tests/golden/des_n{N}.json: per-seed detection / convergence samples of the
reference-timing DES (oracle/des.py) for the KS tests (tests/test_ks_des.py).

The DES is deterministic per seed (Python's `random.Random`), so the fixture is a cache: the CPU
suite re-runs a few seeds live and checks they reproduce it exactly.  N=64 and N=1024 (BASELINE.json
config 2: 1,024 members, 0 % loss, single failure) with 200 seeds each (>= 200 seeds
for KS at N <= 1,024).

    python tests/golden/make_des_fixtures.py [N ...]
"""
import json
import multiprocessing as mp
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "oracle"))

import des  # noqa: E402

SEEDS = range(1, 201)
HORIZON_MS = {64: 50000.0, 1024: 70000.0}


def _one(args):
    n, seed = args
    return des.des_sample(n, seed, HORIZON_MS[n])


def main():
    ns = [int(x) for x in sys.argv[1:]] or [64, 1024]
    for n in ns:
        with mp.Pool(min(8, os.cpu_count() or 1)) as pool:
            rows = pool.map(_one, [(n, s) for s in SEEDS])
        doc = {"n": n, "seeds": list(SEEDS), "horizon_ms": HORIZON_MS[n],
               "des_config": des.Des.__init__.__defaults__ and dict(zip(
                   des.Des.__init__.__code__.co_varnames[3:3 + len(des.Des.__init__.__defaults__)],
                   des.Des.__init__.__defaults__)),
               "samples": rows}
        out = os.path.join(HERE, f"des_n{n}.json")
        with open(out, "w") as f:
            json.dump(doc, f, indent=0)
        print(f"wrote {out}: {len(rows)} runs")


if __name__ == "__main__":
    main()
