#!/bin/bash
# c3 bench layouts (streams / batch / chunks / skew), each twice, interleaved:
# bash tools/ab_layout.sh TAG "ARGS1" "ARGS2" ...  -> gpurun_out/TAG/lay<i>_<r>.json
set -o pipefail
T=${1:?tag}; shift
mkdir -p gpurun_out/$T
for r in 1 2; do
  i=0
  for a in "$@"; do
    timeout -k 10 200 python bench.py --cpu-budget 0 --soak-s 1 --steps 30 $a > gpurun_out/$T/lay${i}_$r.json 2> gpurun_out/$T/lay${i}_$r.err || exit 1
    echo "$a" > gpurun_out/$T/lay${i}.args
    i=$((i+1))
  done
done
echo LAYOUT_DONE
