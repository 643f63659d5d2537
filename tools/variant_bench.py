"""Dev tool: A/B timing of libswimgpu.so builds on the quiet bench workload (not part of the product).

    python tools/variant_bench.py LIB.so [LIB2.so ...]
    VB_STORM=1 python tools/variant_bench.py ...   # kill one member first: time its gossip storm

Loads each build explicitly, runs N = 65,536 periods and prints ms/period, the SYNC classify
kernel's and the gossip fanout kernel's event-timed averages.  Build variants with e.g.
    hipcc <HIPCC_FLAGS of __graft_entry__> -DCLS_MINWAVES=3 -o scalecube-cluster_amd/lib/variants/x.so ...
"""
import ctypes
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "scalecube-cluster_amd"))
from swimgpu import abi  # noqa: E402

N, WARM, STEPS = 65536, 8, 30
STORM = os.environ.get("VB_STORM") == "1"
for path in sys.argv[1:]:
    lib = abi.bind(ctypes.CDLL(os.path.abspath(path)))
    cfg = abi.default_config(lib, 0, sync_stagger=1)
    with abi.Engine(lib, cfg, N, N, 1) as e:
        e.step(WARM)
        if STORM:
            e.kill(17)
        e.profile_enable(True)
        t0 = time.perf_counter()
        e.step(STEPS)
        dt = time.perf_counter() - t0
        p = e.profile_merge()
        f = e.profile_fanout()
        st = e.stats()
    avg = p["total_ms"] / max(1, p["launches"])
    favg = f["total_ms"] / max(1, f["launches"])
    print(f"{os.path.basename(path):28s} {dt / STEPS * 1e3:7.3f} ms/period  classify {avg * 1e3:6.2f} us "
          f"{p['alg_bytes'] / max(1e-12, p['total_ms'] / 1e3) / 1e9:7.0f} GB/s  emit {favg * 1e3:8.1f} us  "
          f"sync_records {st['sync_records']}  accepted {st.get('gossips_accepted', '-')}", flush=True)
