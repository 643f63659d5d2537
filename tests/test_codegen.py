"""Code-generation guards on the built gfx950 library (CPU only: the device code object is unbundled
from libswimgpu.so and read with the ROCm LLVM tools).

Round 5 found the per-tick chain 1.7x slower after an unrelated change: apply_ins_batch stopped being
inlined into k_sync_apply / k_ack_apply, and the call made the kernels keep their whole Ctx in scratch
(960 B of scratch per thread, 1,200 scratch loads; 12.9 -> 22.8 us and 6.3 -> 14.6 us per launch).
These tests make such a codegen change fail loudly instead of showing up as a slower bench line.
"""
import os
import re
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "scalecube-cluster_amd", "lib", "libswimgpu.so")
LLVM = "/opt/rocm/lib/llvm/bin"

# scratch bytes per thread the hot kernels may use (the per-tick chain, the storm kernels, the
# quiet windows); measured values in round 5: 80 / 144 / 144 / 0 / 56 / 0 / 0 / 0 (k_gossip_deliver
# was 28 until onGossipReq's infected-list insert stopped indexing GossipDev.inf at run time: such an
# index puts the array in scratch; k_deliver_coop runs at its 256-VGPR cap, these are spills: 88 B
# in round 6 with the whole-wave slab-index rebuild and the cleared collectors' lookups, whose
# spills sit around those rare paths — churn's delivery went 460 -> 330 ms per launch with them)
SCRATCH_MAX = {"k_fd": 128, "k_sync_apply": 256, "k_ack_apply": 256, "k_gossip_deliver": 32,
               "k_deliver_coop": 96, "k_gossip_emit": 64, "k_quiet_scan": 0, "k_quiet_apply": 0}


@pytest.fixture(scope="module")
def device_object(tmp_path_factory):
    if not (os.path.exists(LIB) and os.path.exists(os.path.join(LLVM, "clang-offload-bundler"))):
        pytest.skip("libswimgpu.so or the ROCm LLVM tools are missing")
    d = tmp_path_factory.mktemp("codeobj")
    fat, dev = str(d / "fat.bin"), str(d / "dev.o")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", LIB, str(d / "host.so")], check=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                    f"--input={fat}", f"--output={dev}", "--unbundle"], check=True)
    return dev


def test_no_device_function_calls(device_object):
    """Every device function is inlined into its kernel: a call (s_swappc_b64) spills the caller's
    live state, the engine's Ctx included, to scratch."""
    dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", device_object], check=True, capture_output=True,
                         text=True).stdout
    assert "s_swappc_b64" not in dis


def test_hot_kernels_scratch(device_object):
    notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", device_object], check=True, capture_output=True,
                           text=True).stdout
    scratch = {}
    name = None
    for line in notes.splitlines():
        m = re.match(r"\s+\.name:\s+(\S+)", line)
        if m:
            name = m.group(1)
        m = re.match(r"\s+\.private_segment_fixed_size:\s+(\d+)", line)
        if m and name:
            scratch[name] = int(m.group(1))
    for k, lim in SCRATCH_MAX.items():
        found = [v for n, v in scratch.items() if f"swimdev{len(k)}{k}" in n or n.startswith(f"_ZN7swimdev{len(k)}{k}E")]
        assert found, f"kernel {k} not in the code object"
        assert max(found) <= lim, f"{k}: {max(found)} B of scratch per thread (limit {lim})"
