#!/usr/bin/env bash
# rocprofv3 passes over ONE bench command (default: the driver's `python3 bench.py --gpus 1 --steps 20
# --warmup 5`), run through gpurun from the repo root:
#   1. kernel trace + stats                                   -> gpurun_out/prof/<tag>_stats
#   2. memory-side read requests by size (counters only)      -> gpurun_out/prof/<tag>_rd
#   3. memory-side write requests, all and 64-B (counters only) -> gpurun_out/prof/<tag>_wr
# then: python tools/prof_summary.py gpurun_out/prof/<tag> profiles/<round>_<name>.
# Each pass has its own time limit; the chain stops at the first failure.  A heartbeat line every
# 50 s shows the pass is alive (the bench prints its one line only at the end).
set -uo pipefail
tag=${1:-drv}
ARGS=${ARGS:---gpus 1 --steps 20 --warmup 5}
export TMPDIR=/tmp
out=gpurun_out/prof
mkdir -p $out
pass() {
  local name=$1
  shift
  (while sleep 50; do echo "prof_driver: pass $name running $(date +%T)"; done) &
  local hb=$!
  timeout -k 10 ${PASS_TIMEOUT:-480} rocprofv3 "$@" -T -d $out/${tag}_$name -o run -- python3 bench.py $ARGS \
    > $out/${tag}_$name.log 2>&1
  local rc=$?
  kill $hb
  if [ $rc -ne 0 ]; then
    echo "prof_driver: pass $name failed rc=$rc"
    tail -5 $out/${tag}_$name.log
    exit $rc
  fi
  echo "prof_driver: pass $name ok"
}
pass stats --kernel-trace --stats
pass rd --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum
pass wr --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum
grep '^{' $out/${tag}_stats.log | cut -c1-300
