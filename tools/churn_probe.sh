#!/usr/bin/env bash
# config-3 churn probe on the GPU box: per-period progress + rocprofv3 kernel stats at reduced N
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
n=${N:-4096}
steps=${STEPS:-8}
gcap=${GCAP:-524288}
tag=${TAG:-r02_churn$n}
timeout -k 10 ${TLIM:-420} rocprofv3 --kernel-trace --stats -T -d gpurun_out/prof/${tag}_stats -o run \
  -- python3 -u bench.py --workload churn --members $n --steps $steps --warmup 2 --progress --no-cpu-baseline \
     --gossip-capacity $gcap > gpurun_out/${tag}.log 2>&1
rc=$?
echo "n=$n rc=$rc"; tail -3 gpurun_out/${tag}.log
exit $rc
