"""Dev tool: every catalog scenario (but the longest) through the GPU wave-delivery path and the
oracle, R rounds in one process (device memory recycled between engines, as in the test suite);
prints every run whose final counters or event stream differ."""
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

reps = int(sys.argv[1])
wave = len(sys.argv) > 2 and sys.argv[2] == "wave"
glib, olib = swimgpu.load_library(), oracle.lib()
cat = [s for s in scenarios.catalog() if s.name != "config3_rates_200"]
want = {}
for sc in cat:
    oe = scenarios.make_engine(olib, sc)
    scenarios.run(oe, sc)
    want[sc.name] = (oe.stats(), oe.drain_events())
    oe.close()
bad = 0
for r in range(reps):
    for sc in cat:
        s2 = dataclasses.replace(sc, cfg={**sc.cfg, "deliver_wave_min": 1}) if wave else sc
        ge = scenarios.make_engine(glib, s2)
        scenarios.run(ge, s2)
        d = parity.diff_stats(want[sc.name][0], ge.stats())
        ev = parity.diff_events(want[sc.name][1], ge.drain_events())
        if d or ev:
            bad += 1
            print(f"round {r} {sc.name}: {d} {'events differ' if ev else ''}", flush=True)
        ge.close()
print(f"{bad} of {reps * len(cat)} runs diverged", flush=True)
