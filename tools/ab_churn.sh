#!/usr/bin/env bash
# A/B of library variants on config 3's churn delivery at N = 4,096 (through gpurun, repo root):
#   bash tools/ab_churn.sh TAG base v1 v2 ...   (base: the in-tree library; vN: tools/libswimgpu_vN.so)
# per variant gpurun_out/TAG_vN.log: tools/config_probe.py's per-period lines with the delivery profile.
set -o pipefail
tag=$1; shift
for v in "$@"; do
  L=scalecube-cluster_amd/lib/libswimgpu.so
  [ "$v" != base ] && L=tools/libswimgpu_$v.so
  SWIMGPU_LIB=$L tools/gpu_run.sh ${tag}_$v 200 python3 -u tools/config_probe.py churn --members 4096 --periods 8 \
    --deliver > /dev/null || exit 1
done
