#!/bin/bash
# Config 4 at 32 frames per rank (the 8-GPU per-rank shape): pyramid plan and stream layouts.
# Output gpurun_out/abc/c4_<name>.json (tools/ab_cfg.sh with --per-rank 32)
set -o pipefail
export AB_ARGS="--per-rank 32"
bash tools/ab_cfg.sh c4 p32base p32small17=ORBFE_PYR_SMALL_BELOW=17 p32roll2=ORBFE_ROLL=2,ORBFE_PYR_SMALL_BELOW=17 || exit 1
for s in "--streams 1" "--streams 3" "--streams 4"; do
  n=$(echo $s | tr -d ' -')
  timeout -k 10 200 python bench.py --config c4 --per-rank 32 --cpu-budget 0 --soak-s 1 --steps 10 $s > gpurun_out/abc/c4_p32$n.json 2> gpurun_out/abc/c4_p32$n.err || exit 1
done
echo C4_32_DONE
