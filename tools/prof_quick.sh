#!/usr/bin/env bash
# kernel-trace stats of one bench run -> gpurun_out/prof/<tag>_stats (the first pass of profile.sh)
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
tag=${TAG:-quick}
timeout -k 10 ${TLIM:-300} rocprofv3 --kernel-trace --stats -T -d gpurun_out/prof/${tag}_stats -o run \
  -- python3 bench.py --workload ${WORKLOAD:-quiet} --steps ${STEPS:-10} --warmup ${WARMUP:-5} --no-cpu-baseline ${ARGS:-} \
  > gpurun_out/prof/${tag}_stats.log 2>&1
rc=$?
grep '^{' gpurun_out/prof/${tag}_stats.log | cut -c1-300
exit $rc
