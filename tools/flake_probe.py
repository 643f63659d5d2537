"""Repeat one golden-digest scenario in one process and count digest mismatches (tools only):
    SWIMGPU_LIB=... python tools/flake_probe.py join_burst_144 4 30"""
import dataclasses
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "tests"), os.path.join(REPO, "tests", "golden"), REPO]
import conftest  # noqa: F401,E402
import scenarios  # noqa: E402
import swimgpu  # noqa: E402
from make_scenario_digests import digest, event_digest  # noqa: E402


def main():
    name, shards, reps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    lib = swimgpu.load_library()
    golden = json.load(open(os.path.join(REPO, "tests", "golden", "scenario_digests.json")))["scenarios"][name]
    sc = [s for s in scenarios.catalog() if s.name == name][0]
    sc2 = dataclasses.replace(sc, cfg={**sc.cfg, "local_shards": shards})
    bad = 0
    for r in range(reps):
        e = scenarios.make_engine(lib, sc2)
        scenarios.run(e, sc2)
        ev = e.drain_events()
        ok_ev = event_digest(ev) == golden["events_sha256"] and len(ev) == golden["events"]
        ok_st = digest(e, None, True) == golden["state_sha256"]
        if not (ok_ev and ok_st):
            bad += 1
            print(f"rep {r}: events {'ok' if ok_ev else 'DIFF'} ({len(ev)} vs {golden['events']}), state {'ok' if ok_st else 'DIFF'}",
                  flush=True)
        del e
    print(json.dumps({"lib": swimgpu.LIB_PATH, "scenario": name, "shards": shards, "reps": reps, "mismatches": bad}), flush=True)


if __name__ == "__main__":
    main()
