#!/usr/bin/env bash
# The GPU tests marked slow (BASELINE configs at their stated sizes), one time-limited pytest run;
# per-period logs land in gpurun_out/*.jsonl.  PYTEST_K selects a subset.
set -uo pipefail
mkdir -p gpurun_out
SWIM_GPU_SLOW=1 timeout -k 10 ${TLIM:-1000} python -u -m pytest tests -m "gpu and slow" -v --timeout ${TEST_TLIM:-900} \
  --timeout-method thread ${PYTEST_K:-} > gpurun_out/gpu_slow.log 2>&1
rc=$?
tail -15 gpurun_out/gpu_slow.log
exit $rc
