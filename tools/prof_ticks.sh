#!/usr/bin/env bash
# Kernel trace of a short quiet bench run, then the per-kernel / per-tick breakdown of its last
# launches (tools/trace_ticks.py) -> gpurun_out/prof/<tag>_ticks.txt
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
tag=${TAG:-ticks}
timeout -k 10 ${TLIM:-240} rocprofv3 --kernel-trace --stats -T -d gpurun_out/prof/${tag}_stats -o run \
  -- python3 bench.py --workload ${WORKLOAD:-quiet} --steps ${STEPS:-10} --warmup ${WARMUP:-5} --no-cpu-baseline --no-extras ${ARGS:-} \
  > gpurun_out/prof/${tag}_stats.log 2>&1
rc=$?
grep '^{' gpurun_out/prof/${tag}_stats.log | cut -c1-400
[ $rc -ne 0 ] && exit $rc
python3 tools/trace_ticks.py gpurun_out/prof/${tag}_stats ${LAST:-800} ${TICKS:-24} > gpurun_out/prof/${tag}_ticks.txt 2>&1
rc=$?
cat gpurun_out/prof/${tag}_ticks.txt
exit $rc
