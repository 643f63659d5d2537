#!/usr/bin/env bash
# Per-tick chain (quiet windows off) of several builds side by side: every exp/bisect/<commit>/ is a
# runnable snapshot (its swimgpu package, bench.py, built libswimgpu.so); "cur" is this tree.
set -euo pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp SWIM_QUIET=0
for d in exp/bisect/* .; do
  name=$(basename "$d"); [ "$d" = "." ] && name=cur
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/bis_${name} -o run \
    -- python3 $d/bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline > gpurun_out/bis_${name}.json 2>/dev/null
done
