#!/bin/bash
# rocprofv3 kernel trace of a short bench run (the timed two-stream steps included):
# bash tools/trace_bench.sh TAG [bench args]  -> gpurun_out/trace_TAG/ ; python tools/timeline.py TAG
set -o pipefail
T=${1:?tag}; shift
O=gpurun_out/trace_$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O -o run --output-format csv -- python3 bench.py --cpu-budget 0 --soak-s 0 --steps 20 "$@" > $O/stdout.txt 2>&1
