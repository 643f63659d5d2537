"""Dev tool (GPU box): run one scenario on the CPU oracle and on libswimgpu in lockstep, one tick at a
time from tick `start`, and report the first tick whose state, events or counters differ — with the
state diff, both engines' events of that tick and the counter diff.

    python tools/first_divergence.py <scenario> [start_tick]
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tests"))
import conftest  # noqa: E402,F401  (sys.path for swimgpu / oracle)
import numpy as np  # noqa: E402

import oracle  # noqa: E402
import parity  # noqa: E402
import scenarios  # noqa: E402
import swimgpu  # noqa: E402


def main():
    name = sys.argv[1]
    start = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    sc = next(s for s in scenarios.catalog() if s.name == name)
    oe = scenarios.make_engine(oracle.lib(), sc)
    ge = scenarios.make_engine(swimgpu.load_library(), sc)
    ops = sorted(sc.ops, key=lambda x: x[0])
    oi = 0
    for t in range(sc.ticks):
        while oi < len(ops) and ops[oi][0] <= t:
            for e in (oe, ge):
                scenarios.apply_op(e, ops[oi][1], ops[oi][2:])
            oi += 1
        oe.step_ticks(1)
        ge.step_ticks(1)
        eo, eg = oe.drain_events(), ge.drain_events()
        if t + 1 < start:
            continue
        d = parity.diff_states(parity.state_digest(oe), parity.state_digest(ge), limit=40)
        dev = parity.diff_events(eo, eg)
        dst = parity.diff_stats(oe.stats(), ge.stats())
        if d or dev or dst:
            print(f"first divergence after tick {t + 1}")
            for x in d + dev + dst:
                print("  ", x[:400])
            cols = ["tick", "viewer", "subject", "type", "phase", "minor"]
            print("oracle events:\n", np.array([[int(r[c]) for c in cols] for r in eo]))
            print("gpu events:\n", np.array([[int(r[c]) for c in cols] for r in eg]))
            return 1
    print("no divergence")
    return 0


if __name__ == "__main__":
    sys.exit(main())
