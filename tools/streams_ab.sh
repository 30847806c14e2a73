#!/bin/bash
# c3 frames/s for stream / chunk / skew layouts (two runs each)
mkdir -p gpurun_out/streams
set -o pipefail
for cfg in "1 1 0" "2 1 0" "2 2 1" "4 1 0" "2 4 1"; do
  set -- $cfg
  for r in 1 2; do
    timeout -k 10 120 python bench.py --cpu-budget 0 --steps 30 --streams $1 --chunks $2 --skew $3 > gpurun_out/streams/s$1_c$2_k$3_$r.json 2>&1 || exit 1
  done
done
echo STREAMS_DONE
