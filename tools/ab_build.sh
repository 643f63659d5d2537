#!/usr/bin/env bash
# A/B variants of the library for delivery experiments (tools only; the product library is untouched):
#   tools/ab_build.sh NAME "-DFLAG ..."  -> tools/libswimgpu_NAME.so
set -euo pipefail
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC -Wno-unused-value -Wno-unused-result \
  $2 -o "tools/libswimgpu_$1.so" scalecube-cluster_amd/csrc/engine.hip -lrccl
