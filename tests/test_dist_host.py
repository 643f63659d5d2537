"""The N>1 host path on CPU: world_size-2 gloo processes drive swimgpu.dist.ShardedEngine.

The device data path of a sharded run (RCCL between GPUs) cannot run here; its exchange plan is
tested bit-exactly on one GPU by the sharded parity tests (test_gpu_parity.py, cfg.local_shards).
What this covers is the multi-process HOST layer bench.py uses at N>1: rendezvous over 127.0.0.1,
rank-0 bootstrap broadcast, replicated control calls, owner-routed row reads, the merged canonical
event stream and rank-reduced counters.  Each rank's engine here is the CPU oracle running the whole
cluster; the layer exposes only the rank's own viewers, exactly as a GPU shard does, so the gathered
result must equal one unsharded run.
"""
import os
import pickle
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import oracle
import scenarios
from swimgpu import abi

SCENARIO = "churn_48"


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_path):
    import torch.distributed as dist

    from swimgpu.dist import ShardedEngine
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sc = next(s for s in scenarios.catalog() if s.name == SCENARIO)
        olib = oracle.lib()
        se = ShardedEngine(olib, None, sc.capacity, sc.n_initial, sc.seed,
                           engine_factory=lambda: scenarios.make_engine(olib, sc))
        assert se.count == (24 if rank == 0 else 24) and se.lo == 24 * rank
        scenarios.run(se, sc)
        events = se.drain_events()
        views = [se.read_view(v) for v in range(sc.capacity)]
        stats = se.stats()
        dt = se.max_time(0.5 + rank)
        if rank == 0:
            with open(out_path, "wb") as f:
                pickle.dump({"events": events.tobytes(), "views": views, "stats": stats, "dt": dt}, f)
        se.close()
    finally:
        dist.destroy_process_group()


def test_sharded_host_layer_gloo_world2(tmp_path):
    out = str(tmp_path / "r0.pkl")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    got = pickle.load(open(out, "rb"))
    sc = next(s for s in scenarios.catalog() if s.name == SCENARIO)
    ref = scenarios.make_engine(oracle.lib(), sc)
    scenarios.run(ref, sc)
    ev_ref = ref.drain_events()
    ev = np.frombuffer(got["events"], dtype=abi.EVENT_DTYPE)
    assert len(ev) == len(ev_ref) > 0
    for f in ("tick", "viewer", "subject", "type", "phase", "minor"):
        assert np.array_equal(ev[f], ev_ref[f]), f
    for v in range(sc.capacity):
        assert np.array_equal(got["views"][v], ref.read_view(v)), v
    assert got["dt"] == 1.5  # the slowest rank's time
    # each rank's oracle counts the whole cluster, so the rank-sum is exactly twice one run
    assert got["stats"]["pings"] == 2 * ref.stats()["pings"] and got["stats"]["capacity_errors"] == 0
