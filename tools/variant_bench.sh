#!/usr/bin/env bash
# A/B of compile-time variants (exp/lib_<X>.so, built beside the tree) on the quiet bench, interleaved
# twice; one JSON summary line per run -> gpurun_out/variants.log
set -uo pipefail
mkdir -p gpurun_out
for round in $(seq 1 ${ROUNDS:-2}); do
  for v in ${VARIANTS:-A B C D E}; do
    SWIMGPU_LIB=exp/lib_$v.so timeout -k 10 120 python3 bench.py --steps ${STEPS:-60} --warmup 5 --no-extras --no-cpu-baseline \
      > gpurun_out/variant_$v.log 2>&1 || { echo "variant $v failed"; tail -5 gpurun_out/variant_$v.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/variant_$v.log').read().strip().splitlines()[-1]); print('$v', round(d['ms_per_step'],4), '%.4g' % d['value'])" | tee -a gpurun_out/variants.log
  done
done
