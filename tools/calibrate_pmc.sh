#!/usr/bin/env bash
# PMC calibration on the GPU box (tools/gatherbench.hip): one plain run, then FETCH_SIZE, WRITE_SIZE
# and the raw memory-side read-request counters, each in its own rocprofv3 pass.
set -euo pipefail
export TMPDIR=/tmp
out=gpurun_out/cal
mkdir -p $out
timeout -k 10 60 rocprofv3 --list-avail > $out/avail.txt 2>&1 || true
timeout -k 10 120 ./tools/gatherbench > $out/plain.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $out/fetch -o run -- ./tools/gatherbench > $out/fetch.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $out/write -o run -- ./tools/gatherbench > $out/write.log 2>&1
for c in ${RAW:-TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum}; do
  timeout -s KILL 90 rocprofv3 --pmc $c -d $out/raw_$c -o run -- ./tools/gatherbench > $out/raw_$c.log 2>&1 || { echo "counter $c failed: rc $?" >> $out/raw_failed.txt; break; }
done
