"""Loader for the CPU oracle (oracle/liboracle_swim.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg, never by the swimgpu package.  The oracle exports the same C ABI as libswimgpu.so
(include/swim.h), so it is driven through the same `swimgpu.abi.Engine` wrapper.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, "scalecube-cluster_amd"))

from swimgpu import abi  # noqa: E402

LIB_PATH = os.path.join(HERE, "liboracle_swim.so")
_lib = None


def build() -> str:
    """Compile the oracle with its Makefile (g++ only)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < os.path.getmtime(
                os.path.join(HERE, "swim_oracle.cpp")):
            build()
        _lib = abi.bind(ctypes.CDLL(LIB_PATH))
    return _lib


def set_threads(e: abi.Engine, threads: int) -> None:
    """Worker threads of the oracle's per-member phase loops (swim_oracle_set_threads, oracle only;
    0 = hardware concurrency).  Results are identical for every thread count."""
    fn = e.lib.swim_oracle_set_threads
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int32]
    fn.restype = ctypes.c_int32
    rc = fn(e._h, int(threads))
    if rc != 0:
        raise abi.SwimError("swim_oracle_set_threads", rc)


def engine(cfg=None, capacity=16, n_initial=None, seed=1, **overrides) -> abi.Engine:
    L = lib()
    if cfg is None:
        cfg = abi.default_config(L, 0, **overrides)
    return abi.Engine(L, cfg, capacity, capacity if n_initial is None else n_initial, seed)
