#!/usr/bin/env bash
# Quiet-path checks and A/B on the GPU box: quiet-window parity tests, the headline at --steps 20 with
# and without the spinning window wait, and a kernel trace of the per-tick chain (quiet windows off).
# Each step is time-limited; the chain stops at the first failure.
set -euo pipefail
tag=${1:-r05}
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_quiet_path.py tests/test_gpu_bench_parity.py tests/test_gpu_parity.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -k "${PYTEST_K:-quiet or headline or row_cap or pull}" > gpurun_out/${tag}_quiet_tests.log 2>&1
for spin in 1 0; do
  SWIM_SPIN=$spin timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline > gpurun_out/${tag}_spin${spin}.json 2>/dev/null
done
SWIM_QUIET=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/${tag}_pertick_stats -o run \
  -- python3 bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline > gpurun_out/${tag}_pertick.json 2>/dev/null
