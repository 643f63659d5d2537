#!/usr/bin/env bash
# The cross-shard receipt filter on the one-GPU rig (tools only): the failures window (periods 30-36,
# the bench's fanout side run) unsharded, and over 8 in-process shards with the filter on and off.
set -uo pipefail
tag=${1:-rf}
mkdir -p gpurun_out
A="--workload failures --warmup 30 --steps 6 --no-extras --no-cpu-baseline"
timeout -k 10 300 python3 bench.py $A > gpurun_out/${tag}_unsharded.json 2> gpurun_out/${tag}_unsharded.err || exit 1
SWIM_RFILTER=1 timeout -k 10 400 python3 bench.py $A --local-shards 8 > gpurun_out/${tag}_ls8_on.json 2> gpurun_out/${tag}_ls8_on.err || exit 1
SWIM_RFILTER=0 timeout -k 10 400 python3 bench.py $A --local-shards 8 > gpurun_out/${tag}_ls8_off.json 2> gpurun_out/${tag}_ls8_off.err || exit 1
for f in unsharded ls8_on ls8_off; do
  python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/${tag}_'+sys.argv[1]+'.json') if l.startswith('{')][0]); print(sys.argv[1], 'ms/period', round(d['ms_per_step'],3), 'msgs', d['stats']['gossip_messages'], 'emit_ms', round(d['roofline_fanout']['avg_launch_ms'],4), 'deliver_ms', round(d['roofline_deliver']['avg_launch_ms'],4))" $f
done
