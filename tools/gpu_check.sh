#!/usr/bin/env bash
# GPU parity suite, then (optionally) the quiet bench and the config-3 churn probe; each step is
# time-limited and the chain stops at the first failure
set -uo pipefail
mkdir -p gpurun_out
if [ -z "${NOTEST:-}" ]; then
  timeout -k 10 ${TEST_TLIM:-700} python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_K:-} > gpurun_out/gputest.log 2>&1
  rc=$?
  tail -5 gpurun_out/gputest.log
  [ $rc -ne 0 ] && exit $rc
fi
if [ -n "${QUIET:-}" ]; then
  timeout -k 10 300 python -u bench.py --no-cpu-baseline ${QUIET_ARGS:-} > gpurun_out/bench_quiet.log 2>&1
  rc=$?
  tail -c 1500 gpurun_out/bench_quiet.log
  [ $rc -ne 0 ] && exit $rc
fi
if [ -n "${CHURN:-}" ]; then
  N=${CHURN} STEPS=${STEPS:-8} TLIM=${CHURN_TLIM:-300} bash tools/churn_probe.sh
fi
