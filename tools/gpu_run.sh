#!/usr/bin/env bash
# One time-limited GPU step with a heartbeat file under gpurun_out/ (long single tests print nothing
# for minutes): tools/gpu_run.sh NAME SECONDS cmd...  -> gpurun_out/NAME.log, exit status of cmd.
set -uo pipefail
name=$1; lim=$2; shift 2
mkdir -p gpurun_out
( while true; do date +%s >> gpurun_out/heartbeat.txt; sleep 20; done ) &
hb=$!
timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
rc=$?
kill $hb 2>/dev/null
tail -25 "gpurun_out/$name.log"
exit $rc
