#!/bin/bash
# Config-5 volume sweep (run on the GPU box): partition + heal at growing N, short hold (heal while
# the other side is SUSPECT) and long hold (heal after the suspicion timeout removed it).
set -o pipefail
mkdir -p gpurun_out/heal
for n in ${SIZES:-512 1024 2048}; do
  for hold in short long; do
    h=""; [ "$hold" = short ] && h="--hold 20"
    timeout -k 10 ${T:-240} python -u tools/config_probe.py partition --members $n $h --after ${AFTER:-80} \
      --gossip-capacity ${GCAP:-524288} --stop-converged > gpurun_out/heal/n${n}_${hold}.log 2>&1
    rc=$?
    echo "n=$n hold=$hold rc=$rc $(tail -n 2 gpurun_out/heal/n${n}_${hold}.log | tr '\n' ' ')"
    [ $rc -ge 124 ] && exit $rc
  done
done
exit 0
