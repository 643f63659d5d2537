#!/usr/bin/env bash
# rocprofv3 passes over one bench window (run through gpurun from the repo root):
#   1. kernel trace + stats -> gpurun_out/prof/<tag>_stats
#   2. FETCH_SIZE only      -> gpurun_out/prof/<tag>_fetch
#   3. WRITE_SIZE only      -> gpurun_out/prof/<tag>_write
# the same command each time (default: the failures workload's second-kill window, the bench's
# fanout-roofline side run); tools/window_summary.py then averages the last launches of a kernel.
set -euo pipefail
tag=${1:-win}
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
ARGS=${ARGS:---workload failures --warmup 30 --steps 6 --no-cpu-baseline --no-extras}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d gpurun_out/prof/${tag}_stats -o run -- python3 bench.py $ARGS > gpurun_out/prof/${tag}_stats.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T -d gpurun_out/prof/${tag}_fetch -o run -- python3 bench.py $ARGS > gpurun_out/prof/${tag}_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T -d gpurun_out/prof/${tag}_write -o run -- python3 bench.py $ARGS > gpurun_out/prof/${tag}_write.log 2>&1
grep '^{' gpurun_out/prof/${tag}_stats.log | cut -c1-400
