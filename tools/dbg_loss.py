"""Dev tool: step a lossy cluster tick by tick on the GPU and report where a capacity runs out."""
import sys
import time
sys.path[:0] = ['scalecube-cluster_amd']
import swimgpu
from swimgpu import abi

n, loss, ticks = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
gcap = int(sys.argv[4]) if len(sys.argv) > 4 else 16384
L = swimgpu.load_library()
cfg = abi.default_config(L, 0, sync_stagger=1, gossip_capacity=gcap, timer_capacity=16 * n, event_capacity=1 << 25,
                         message_capacity=min(1 << 28, 4096 * n))
e = abi.Engine(L, cfg, n, n, 1)
e.set_default_loss(loss)
t0 = time.time()
for t in range(ticks):
    try:
        e.step_ticks(1)
    except abi.SwimError as ex:
        st = e.stats()
        g = max(e.read_member(m)["gossip_len"] for m in range(0, n, max(1, n // 512)))
        print(f"tick {t + 1}: {ex} bits {st['capacity_errors']:#x} gossips_created {st['gossips_created']} "
              f"max gossip_len(sampled) {g} fd_events {st['fd_events']}", flush=True)
        break
    if (t + 1) % 50 == 0:
        st = e.stats()
        g = max(e.read_member(m)["gossip_len"] for m in range(0, n, max(1, n // 512)))
        print(f"tick {t + 1}: gossips_created {st['gossips_created']} max gossip_len {g} "
              f"msgs {st['gossip_messages']} {time.time() - t0:.1f}s", flush=True)
        e.drain_events()
