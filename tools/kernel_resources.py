"""Per-kernel resources of a built library's gfx950 code object (scratch bytes per thread, VGPRs,
LDS bytes), for comparing A/B variants:  python tools/kernel_resources.py LIB.so [kernel-substring ...]"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def resources(lib):
    with tempfile.TemporaryDirectory() as d:
        fat, dev = os.path.join(d, "fat.bin"), os.path.join(d, "dev.o")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", lib, os.path.join(d, "h.so")],
                       check=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                        f"--input={fat}", f"--output={dev}", "--unbundle"], check=True)
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", dev], check=True, capture_output=True,
                               text=True).stdout
    out, cur = {}, {}
    for line in notes.splitlines():
        m = re.match(r"\s+-?\s*\.(\w+):\s+(\S+)", line)
        if not m:
            continue
        k, v = m.groups()
        if k == "agpr_count" and cur:  # (the first field of the next kernel's record)
            if "name" in cur:
                out[cur["name"]] = cur
            cur = {}
        cur[k] = v
    if "name" in cur:
        out[cur["name"]] = cur
    return out


if __name__ == "__main__":
    res = resources(sys.argv[1])
    pats = sys.argv[2:]
    for name, r in sorted(res.items()):
        if pats and not any(p in name for p in pats):
            continue
        print(f"{name}: scratch {r.get('private_segment_fixed_size')} B, vgpr {r.get('vgpr_count')}, "
              f"lds {r.get('group_segment_fixed_size')} B")
