#!/bin/bash
# c3 stream phase: two sub-batch streams in lockstep (default) vs offset by half a step
# (--chunks 2 --skew 1: stream 1 waits once for stream 0's first chunk), same launch sizes
set -o pipefail
mkdir -p gpurun_out/skew
for s in "--batch 512" "--batch 1024 --chunks 2 --skew 1" "--batch 1024 --chunks 2" "--batch 1024" "--batch 512" "--batch 1024 --chunks 2 --skew 1"; do
  n=$(echo $s | tr -d ' -')
  timeout -k 10 200 python bench.py --cpu-budget 0 --soak-s 2 --steps 20 $s > gpurun_out/skew/c3_$n.json 2> gpurun_out/skew/c3_$n.err || exit 1
  mv gpurun_out/skew/c3_$n.json gpurun_out/skew/c3_${n}_$(date +%s).json
done
echo SKEW_DONE
