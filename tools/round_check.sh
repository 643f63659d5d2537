#!/usr/bin/env bash
# End-of-round GPU check of the in-tree build (through gpurun, from the repo root): the full -m gpu
# suite, the default bench line, and the same-build rocprofv3 passes (quiet kernel stats + PMC,
# failures-window emit / deliver PMC).  Usage: bash tools/round_check.sh <tag>
set -o pipefail
tag=${1:-round}
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_gputest.log 2>&1 || exit 1
timeout -k 10 600 python3 bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || exit 1
bash tools/profile.sh ${tag}_quiet64k || exit 1
bash tools/window_prof.sh ${tag}_failwin || exit 1
