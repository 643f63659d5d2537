#!/usr/bin/env bash
# A/B of library variants on the failures window (through gpurun, from the repo root):
#   bash tools/ab_run.sh TAG base v1 v2 ...   (base: the in-tree library; vN: tools/libswimgpu_vN.so)
# one line per run in gpurun_out/TAG_all.txt: variant, member-periods/s, emit ms, delivery ms.
set -o pipefail
tag=$1; shift
rm -f gpurun_out/${tag}_all.txt
for v in "$@"; do
  L=scalecube-cluster_amd/lib/libswimgpu.so
  [ "$v" != base ] && L=tools/libswimgpu_$v.so
  SWIMGPU_LIB=$L tools/gpu_run.sh ${tag}_$v 200 python3 -u bench.py --workload failures --warmup 30 --steps 6 \
    --no-cpu-baseline --no-extras > /dev/null || exit 1
  echo "$v $(grep -h '^{' gpurun_out/${tag}_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline_fanout"]["avg_launch_ms"], d["roofline_deliver"]["avg_launch_ms"])')" >> gpurun_out/${tag}_all.txt
done
cat gpurun_out/${tag}_all.txt
