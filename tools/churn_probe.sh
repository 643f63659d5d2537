#!/usr/bin/env bash
mkdir -p gpurun_out
for n in 4096 16384; do
  timeout -k 10 240 python -u bench.py --workload churn --members $n --steps 6 --warmup 2 --progress --no-cpu-baseline > gpurun_out/churn_$n.log 2>&1
  rc=$?
  echo "n=$n rc=$rc"; tail -4 gpurun_out/churn_$n.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
