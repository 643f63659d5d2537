"""Dev tool: run one parity scenario many times on the GPU against the oracle, tick by tick, and
report the first tick whose counters or state differ (nondeterminism hunt).

    SWIMGPU_LIB=... python tools/race_hunt.py namespaces_9 40 [deliver_wave_min=1]
"""
import dataclasses
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("scalecube-cluster_amd", "oracle", "tests", os.path.join("tests", "golden")):
    sys.path.insert(0, os.path.join(REPO, p))
import oracle  # noqa: E402
import parity  # noqa: E402
import scenarios  # noqa: E402
import swimgpu  # noqa: E402

name, reps = sys.argv[1], int(sys.argv[2])
extra = dict(kv.split("=") for kv in sys.argv[3:])
sc = {s.name: s for s in scenarios.catalog()}[name]
sc = dataclasses.replace(sc, cfg={**sc.cfg, **{k: int(v) for k, v in extra.items()}})
glib, olib = swimgpu.load_library(), oracle.lib()
# the oracle's per-tick stats once
oe = scenarios.make_engine(olib, sc)
ops = sorted(sc.ops, key=lambda x: x[0])
want = []
oi = 0
for t in range(sc.ticks):
    while oi < len(ops) and ops[oi][0] <= t:
        scenarios.apply_op(oe, ops[oi][1], ops[oi][2:])
        oi += 1
    oe.step_ticks(1)
    want.append(oe.stats())
bad = 0
for r in range(reps):
    ge = scenarios.make_engine(glib, sc)
    oi = 0
    for t in range(sc.ticks):
        while oi < len(ops) and ops[oi][0] <= t:
            scenarios.apply_op(ge, ops[oi][1], ops[oi][2:])
            oi += 1
        ge.step_ticks(1)
        d = parity.diff_stats(want[t], ge.stats())
        if d:
            bad += 1
            print(f"rep {r}: tick {t + 1}: {d}", flush=True)
            break
    ge.close()
print(f"{name} {extra}: {bad} of {reps} runs diverged", flush=True)
