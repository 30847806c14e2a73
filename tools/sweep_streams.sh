#!/bin/bash
# Stream / chunk / skew / profiling sweep of the default bench (config 3) on one GPU.
mkdir -p gpurun_out/sweep
set -o pipefail
for cfg in "2 1 0 1" "2 1 0 0" "1 1 0 0" "2 2 1 0" "3 1 0 0" "4 1 0 0"; do
  set -- $cfg
  timeout -k 10 120 python bench.py --streams $1 --chunks $2 --skew $3 --profile $4 --steps 30 --warmup 5 --cpu-budget 0 > gpurun_out/sweep/s$1_j$2_k$3_p$4.json 2>gpurun_out/sweep/err.log || exit 1
done
