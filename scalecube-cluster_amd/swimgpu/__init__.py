"""swimgpu — MI355X-native lockstep SWIM simulation engine (drop-in for scalecube-cluster's
FailureDetector / GossipProtocol / MembershipProtocol layer).

The compute path is libswimgpu.so (hand-written HIP kernels for gfx950, C ABI in include/swim.h).
There is no CPU fallback: importing works anywhere, but creating an engine requires the built
library and an MI355X, and fails loudly otherwise.
"""
from __future__ import annotations

import ctypes
import os

from . import abi
from .abi import Engine, SwimError, default_config  # noqa: F401

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SWIMGPU_LIB", os.path.join(os.path.dirname(PKG_DIR), "lib", "libswimgpu.so"))

_lib = None


def load_library() -> ctypes.CDLL:
    """Load and bind libswimgpu.so (raises if it is missing: build it with __graft_entry__.build())."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"libswimgpu.so not found at {LIB_PATH}; build it with `python -c 'import __graft_entry__ as g; g.build()'`")
        _lib = abi.bind(ctypes.CDLL(LIB_PATH))
    return _lib


def create_engine(capacity: int, n_initial: int | None = None, seed: int = 1, preset: int = 0, cfg=None,
                  **overrides) -> Engine:
    """Create a GPU engine (swim_create) with a reference preset (0 LAN/default, 1 WAN, 2 Local)."""
    lib = load_library()
    if cfg is None:
        cfg = default_config(lib, preset, **overrides)
    return Engine(lib, cfg, capacity, capacity if n_initial is None else n_initial, seed)


from .cluster import (  # noqa: E402,F401
    ClusterConfig, ClusterMath, FailureDetectorConfig, GossipConfig, Member, MemberStatus,
    MembershipConfig, MembershipEvent, SimulatedCluster)
