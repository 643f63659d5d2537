import sys, time
sys.path[:0] = ['scalecube-cluster_amd', 'oracle', 'tests', 'tests/golden']
import ks, swimgpu
L = swimgpu.load_library()
for n in (64, 1024):
    t = time.time()
    r = ks.lockstep_sample(L, n, 1, 70000.0, timer_stagger=1, tick_ms=10)
    print(n, r, f"{time.time() - t:.2f}s", flush=True)
