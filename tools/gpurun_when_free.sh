#!/usr/bin/env bash
# Submit one gpurun call, re-submitting only while the pool has no free box / slot (gpurun exit 3:
# nothing ran, nothing charged), every 2 minutes, at most 15 times.  A call that ran is never repeated.
#   tools/gpurun_when_free.sh OUT TIMEOUT 'command'
out=$1; to=$2; cmd=$3
for i in $(seq 1 15); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$out" 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "status=transient" "$out"; then exit $rc; fi
  sleep 120
done
exit 3
