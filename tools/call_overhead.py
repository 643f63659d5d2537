"""Where the wall time of bench.py's timed quiet call goes: one e.step(K) bracketed by
torch.cuda.synchronize() as bench.py times it, repeated, with and without the counter reads and the
profiling events bench.py does around it."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "scalecube-cluster_amd"))
import torch  # noqa: E402
import bench  # noqa: E402
import swimgpu  # noqa: E402
from swimgpu import abi  # noqa: E402

N, K = 65536, int(sys.argv[1]) if len(sys.argv) > 1 else 40
lib = swimgpu.load_library()
sch = bench.Schedule("quiet", N, 10 + 12 * K)
e = abi.Engine(lib, bench.make_config(lib), sch.capacity, N, 1)
sch.setup(e)
sch.run(e, 0, 10)
p = 10


def timed(label, prof, reads):
    global p
    e.profile_enable(prof)
    if reads:
        e.drain_events()
        e.stats()
        e.quiet_stats()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e.step(K)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    p += K
    q = e.quiet_stats()
    print(f"{label}: call {1e6 * (t1 - t0):.1f} us, +sync {1e6 * (t2 - t1):.1f} us, "
          f"per period {1e6 * (t2 - t0) / K:.2f} us, windows {q['windows']} precomputed {q['precomputed']}",
          flush=True)


for r in range(3):
    timed("bench-like (profiling on, counter reads before)", True, True)
for r in range(3):
    timed("profiling on, no reads", True, False)
for r in range(3):
    timed("profiling off, no reads", False, False)
for r in range(3):
    timed("profiling off, reads", False, True)
e.close()
