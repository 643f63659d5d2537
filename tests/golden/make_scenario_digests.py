"""Regression pins of the CPU oracle: per-scenario digests of the final protocol state, the event
stream and the counters, written to tests/golden/scenario_digests.json.

The oracle is a restatement of the reference (the JVM reference cannot run in this image); these
digests pin ITS behaviour so that any change to the oracle (or to the shared scenarios) is a
deliberate, reviewed regeneration.  GPU runs are compared with the same digests in
test_gpu_parity.py, in addition to the live lockstep comparison with the oracle.

    python tests/golden/make_scenario_digests.py
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import conftest  # noqa: F401,E402  (sys.path for swimgpu / oracle)
import oracle  # noqa: E402
import parity  # noqa: E402
import scenarios  # noqa: E402


def digest(e, members=None, collectors=True):
    d = parity.state_digest(e, members, collectors)
    h = hashlib.sha256()
    for m in sorted(d["rows"]):
        h.update(d["rows"][m].tobytes())
        h.update(json.dumps(d["members"][m], sort_keys=True).encode())
        h.update(d["ping"][m].tobytes())
        h.update(d["remote"][m].tobytes())
        h.update(d["gossips"][m].tobytes())
        if collectors:
            h.update(json.dumps(sorted(d["coll"][m].items())).encode())
    return h.hexdigest()


def event_digest(ev):
    cols = ev[["tick", "viewer", "subject", "type", "phase", "minor"]]
    return hashlib.sha256(cols.tobytes()).hexdigest()


def run(sc, members=None, collectors=True, threads=1):
    e = scenarios.make_engine(oracle.lib(), sc)
    if threads != 1:
        oracle.set_threads(e, threads)
    scenarios.run(e, sc)
    ev = e.drain_events()
    st = e.stats()
    return {"state_sha256": digest(e, members, collectors), "events_sha256": event_digest(ev), "events": int(len(ev)),
            "stats": {k: int(st[k]) for k in parity.STAT_FIELDS}, "ticks": sc.ticks}


def main():
    # python tests/golden/make_scenario_digests.py [NAME ...]: only the named scenarios are (re)made,
    # the others' digests kept (a new scenario; the whole catalogue takes several minutes)
    only = set(sys.argv[1:])
    path = os.path.join(HERE, "scenario_digests.json")
    out = {"source": "tests/golden/make_scenario_digests.py (CPU oracle)", "scenarios": {}}
    if only:
        out["scenarios"] = json.load(open(path))["scenarios"]
    for sc in scenarios.catalog():
        if only and sc.name not in only:
            continue
        out["scenarios"][sc.name] = run(sc)
        print(sc.name, out["scenarios"][sc.name]["events"], "events")
    sc = scenarios.config2()
    if not only or sc.name in only:
        out["scenarios"][sc.name] = run(sc, members=scenarios.CONFIG2_MEMBERS, collectors=False)
    with open(path, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
