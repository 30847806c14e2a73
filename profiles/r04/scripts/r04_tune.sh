#!/bin/bash
# c3 batch sizes / stream layouts, c4 rolling-pyramid plans (x86 default)
set -o pipefail
mkdir -p gpurun_out/abc
for s in "--batch 512" "--batch 1024" "--streams 4 --batch 512" "--streams 1" "--streams 2 --chunks 2 --skew 1"; do
  n=$(echo $s | tr -d ' -')
  timeout -k 10 200 python bench.py --cpu-budget 0 --soak-s 1 $s > gpurun_out/abc/c3_$n.json 2> gpurun_out/abc/c3_$n.err || exit 1
done
bash tools/ab_cfg.sh c4 base roll6c32=ORBFE_ROLL=1,ORBFE_ROLL_BANDS=6,ORBFE_ROLL_CHUNK=32 roll8c34=ORBFE_ROLL=1,ORBFE_ROLL_BANDS=8,ORBFE_ROLL_CHUNK=34 roll12c34=ORBFE_ROLL=1,ORBFE_ROLL_BANDS=12,ORBFE_ROLL_CHUNK=34 || exit 1
echo TUNE_DONE
