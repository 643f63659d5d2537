"""Steps the failures workload period by period on G in-process shards and prints each period's
counters and error bits (diagnosis of a capacity error seen by bench.py --local-shards)."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "scalecube-cluster_amd"))
import bench  # noqa: E402
import swimgpu  # noqa: E402
from swimgpu import abi  # noqa: E402

G = int(sys.argv[1]) if len(sys.argv) > 1 else 8
P = int(sys.argv[2]) if len(sys.argv) > 2 else 36
N = 65536
lib = swimgpu.load_library()
sch = bench.Schedule("failures", N, P)
cfg = bench.make_config(lib)
cfg.local_shards = G
if len(sys.argv) > 3:
    cfg.message_capacity = int(sys.argv[3])
e = abi.Engine(lib, cfg, sch.capacity, N, 1)
sch.setup(e)
for p in range(P):
    t0 = time.time()
    try:
        sch.run(e, p, p + 1)
    except Exception as ex:  # noqa: BLE001
        print(f"period {p + 1}: {ex}", flush=True)
        print("debug", e.debug_counters(48) if hasattr(e, "debug_counters") else None, flush=True)
        break
    st = e.stats()
    print(f"period {p + 1}: {time.time() - t0:.2f}s msgs={st.get('gossip_messages')} "
          f"created={st.get('gossips_created')} err={st.get('capacity_errors')}", flush=True)
e.close()
