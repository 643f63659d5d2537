"""The drop-in boundary: libswimgpu.so loads on a CPU-only host and exports every swim.h symbol,
and the package refuses to run without it (no CPU fallback)."""
import ctypes
import os
import re

import pytest

import swimgpu
from swimgpu import abi

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_symbols():
    src = open(os.path.join(REPO, "include", "swim.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int32_t|int64_t)\s+(swim_\w+)\s*\(", src, re.M)))


def test_header_matches_bindings():
    assert set(_header_symbols()) == set(abi.PROTOTYPES)


def test_gpu_library_exports_every_symbol():
    if not os.path.exists(swimgpu.LIB_PATH):
        pytest.skip("libswimgpu.so not built (run __graft_entry__.build())")
    lib = ctypes.CDLL(swimgpu.LIB_PATH)
    missing = [s for s in _header_symbols() if not hasattr(lib, s)]
    assert not missing, missing
    abi.bind(lib)
    # host-only entry points work without a device
    cfg = abi.default_config(lib, 0)
    assert cfg.ping_interval == 1000 and lib.swim_ceil_log2(65536) == 17


def test_oracle_exports_every_symbol():
    import oracle
    lib = oracle.lib()
    missing = [s for s in _header_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_package_fails_loudly_without_library(monkeypatch, tmp_path):
    monkeypatch.setattr(swimgpu, "LIB_PATH", str(tmp_path / "missing.so"))
    monkeypatch.setattr(swimgpu, "_lib", None)
    with pytest.raises(RuntimeError, match="libswimgpu.so not found"):
        swimgpu.load_library()


def test_create_without_device_reports_edevice():
    if not os.path.exists(swimgpu.LIB_PATH):
        pytest.skip("libswimgpu.so not built")
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    lib = swimgpu.load_library()
    with pytest.raises(abi.SwimError) as ei:
        abi.Engine(lib, abi.default_config(lib, 0), 8, 8, 1)
    assert ei.value.code == abi.SWIM_EDEVICE


def test_delay_mean_beyond_cap_is_refused():
    """delays are capped at SWIM_DELAY_TICKS_MAX ticks, so a mean the cap would truncate
    (above 64 ticks) is refused by the oracle (and, identically, by swim_delay_mean_ok in the GPU
    engine) instead of silently truncating draws."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
    import oracle
    lib = oracle.lib()
    cfg = abi.default_config(lib)  # LAN: 100 ms ticks
    e = abi.Engine(lib, cfg, 8, 8, seed=1)
    tick = cfg.tick_ms or 100  # 0: gcd of the intervals (LAN: 100 ms)
    assert tick == 100
    e.set_default_delay(64 * tick)        # at the limit: accepted
    e.set_link_delay(1, 2, 64 * tick)
    with pytest.raises(abi.SwimError) as ei:
        e.set_default_delay(64 * tick + 1)
    assert ei.value.code == abi.SWIM_EINVAL
    with pytest.raises(abi.SwimError):
        e.set_link_delay(1, 2, 64 * tick + 1)
    e.set_link_delay(1, 2, -1)            # removing an override needs no table
