#!/usr/bin/env bash
# GPU-box profiling recipe (run through gpurun from the repo root):
#   1. kernel trace + per-kernel stats of the default bench     -> gpurun_out/prof/<tag>_stats
#   2. FETCH_SIZE pass (own run, counters only)                  -> gpurun_out/prof/<tag>_fetch
#   3. WRITE_SIZE pass (own run, counters only)                  -> gpurun_out/prof/<tag>_write
# Each step is time-limited and the chain stops at the first failure.
set -euo pipefail
tag=${1:-run}
steps=${STEPS:-20}
warm=${WARMUP:-5}
wl=${WORKLOAD:-quiet}
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d gpurun_out/prof/${tag}_stats -o run \
  -- python3 bench.py --workload "$wl" --steps "$steps" --warmup "$warm" --no-cpu-baseline --no-extras > gpurun_out/prof/${tag}_stats.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T -d gpurun_out/prof/${tag}_fetch -o run \
  -- python3 bench.py --workload "$wl" --steps "${PMC_STEPS:-$steps}" --warmup "$warm" --no-cpu-baseline --no-extras > gpurun_out/prof/${tag}_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T -d gpurun_out/prof/${tag}_write -o run \
  -- python3 bench.py --workload "$wl" --steps "${PMC_STEPS:-$steps}" --warmup "$warm" --no-cpu-baseline --no-extras > gpurun_out/prof/${tag}_write.log 2>&1
