#!/usr/bin/env bash
# A/B of two library builds on the same box, interleaved (tools only): the headline command
# (--steps 20 --warmup 5, no side runs) with each of tools/libswimgpu_<A>.so and the product library,
# REPS times each; one JSON line per run -> gpurun_out/<tag>_ab.jsonl
set -uo pipefail
tag=${1:-ab}
A=${2:-base}
REPS=${REPS:-3}
ARGS=${ARGS:---steps 20 --warmup 5 --no-extras --no-cpu-baseline}
mkdir -p gpurun_out
out=gpurun_out/${tag}_ab.jsonl
: > $out
for r in $(seq 1 $REPS); do
  for lib in tools/libswimgpu_$A.so scalecube-cluster_amd/lib/libswimgpu.so; do
    SWIMGPU_LIB=$lib timeout -k 10 300 python3 bench.py $ARGS > gpurun_out/${tag}_one.json 2> gpurun_out/${tag}_one.err || { echo "ab_lib: run failed ($lib)"; tail -5 gpurun_out/${tag}_one.err; exit 1; }
    python3 - "$lib" "$r" gpurun_out/${tag}_one.json >> $out <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[3]) if l.startswith("{")][0])
r = d.get("roofline") or {}
ss = d.get("steady_state") or {}
rf = d.get("roofline_fanout") or {}
rd = d.get("roofline_deliver") or {}
print(json.dumps({"lib": sys.argv[1], "rep": int(sys.argv[2]), "value": d["value"], "ms_per_step": d["ms_per_step"],
                  "emit_ms": rf.get("avg_launch_ms"), "deliver_ms": rd.get("avg_launch_ms"),
                  "window_us": (r.get("avg_window_ms") or 0) * 1e3,
                  "steady_value": ss.get("value"), "median_call_us": ss.get("median_call_us"),
                  "per_tick_ms": (d.get("per_tick_path") or {}).get("ms_per_step"),
                  "failures_ms": (d.get("failures") or {}).get("ms_per_step")}))
PY
  done
done
cat $out
