"""Multi-process host layer of the sharded engine (one process per GPU).

`ShardedEngine` is rank r's handle of ONE cluster whose member rows are sharded over the ranks of a
torch.distributed process group.  The data path (GOSSIP_REQ / SYNC / SYNC_ACK between shards) is
RCCL inside libswimgpu.so (swim_create_shard); torch.distributed only bootstraps it (rank 0's RCCL
id is broadcast) and provides the host-side collective views the reference exposes on every member:
  * `read_view(v)`      — MembershipProtocolImpl.getMembershipRecords() of any member
                          (MembershipProtocolImpl.java:903-905): the owning rank reads, then broadcasts;
  * `drain_events()`    — the merged MembershipEvent stream of the whole cluster in canonical order
                          (tick, viewer, phase, minor), gathered from every rank;
  * `stats()`           — counters summed over ranks (capacity errors OR-ed);
  * `max_time(dt)`      — the slowest rank's wall time (bench.py's timed region).
Every method is collective: all ranks call it in the same order, as with the engine itself.
"""
from __future__ import annotations

import numpy as np

from . import abi


class ShardedEngine:
    def __init__(self, lib, cfg, capacity: int, n_initial: int, seed: int, group=None, engine_factory=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.capacity = int(capacity)
        self.rows_per_shard = -(-self.capacity // self.world)
        if engine_factory is None:
            obj = [abi.comm_unique_id(lib) if self.rank == 0 else None]
            dist.broadcast_object_list(obj, src=self._global(0), group=group)
            self.engine = abi.Engine(lib, cfg, capacity, n_initial, seed, rank=self.rank, world=self.world,
                                     comm_id=obj[0])
        else:  # test hook: any engine exposing the abi.Engine interface
            self.engine = engine_factory()
        self.lo = min(self.capacity, self.rank * self.rows_per_shard)
        self.count = min(self.capacity, self.lo + self.rows_per_shard) - self.lo

    def _global(self, r: int) -> int:
        return r if self.group is None else self.dist.get_global_rank(self.group, r)

    def owner(self, v: int) -> int:
        return int(v) // self.rows_per_shard

    def owns(self, v: int) -> bool:
        return self.lo <= int(v) < self.lo + self.count

    # -- replicated control (every rank applies it; the library routes owner-only work) --------
    def __getattr__(self, name):
        if name in ("step", "step_ticks", "kill", "leave", "join", "set_seeds", "set_default_loss", "set_link_loss",
                    "set_link_inbound", "set_default_inbound", "set_partition", "profile_enable", "now"):
            return getattr(self.engine, name)
        raise AttributeError(name)

    # -- collective views -----------------------------------------------------------------------
    def read_view(self, v: int) -> np.ndarray:
        import torch
        buf = torch.zeros(self.capacity, dtype=torch.int64)
        if self.owns(v):
            buf = torch.from_numpy(self.engine.read_view(v).view(np.int64).copy())
        self.dist.broadcast(buf, src=self._global(self.owner(v)), group=self.group)
        return buf.numpy().view(np.uint64)

    def drain_events(self) -> np.ndarray:
        ev = self.engine.drain_events()
        ev = ev[(ev["viewer"] >= self.lo) & (ev["viewer"] < self.lo + self.count)]
        parts = [None] * self.world
        self.dist.all_gather_object(parts, ev.tobytes(), group=self.group)
        allev = np.concatenate([np.frombuffer(p, dtype=abi.EVENT_DTYPE) for p in parts])
        order = np.lexsort((allev["minor"], allev["phase"], allev["viewer"], allev["tick"]))
        return allev[order]

    def stats(self) -> dict:
        import torch
        st = self.engine.stats()
        keys = sorted(k for k in st if k not in ("ticks", "capacity_errors"))
        t = torch.tensor([st[k] for k in keys], dtype=torch.float64)
        self.dist.all_reduce(t, group=self.group)
        err = torch.tensor([int(st["capacity_errors"] != 0)], dtype=torch.int64)
        self.dist.all_reduce(err, op=self.dist.ReduceOp.MAX, group=self.group)
        out = {k: int(v) for k, v in zip(keys, t.tolist())}
        out["ticks"] = st["ticks"]
        out["capacity_errors"] = int(err.item())
        return out

    def max_time(self, dt: float) -> float:
        import torch
        t = torch.tensor([dt], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX, group=self.group)
        return float(t.item())

    def close(self) -> None:
        self.engine.close()
