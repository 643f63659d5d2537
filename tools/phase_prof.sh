#!/usr/bin/env bash
# Build the phase-timing variant of the library (-DSWIM_PHASE_PROF) into tools/libswimgpu_prof.so
# (on the CPU container; the variant travels with the tree) — the product library is untouched.
set -euo pipefail
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC -Wno-unused-value -Wno-unused-result \
  -DSWIM_PHASE_PROF -o tools/libswimgpu_prof.so scalecube-cluster_amd/csrc/engine.hip -lrccl
