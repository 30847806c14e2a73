#!/bin/bash
# c4 rolling-pyramid plans (x86 default) and c3 stream layouts
set -o pipefail
mkdir -p gpurun_out/abc
bash tools/ab_cfg.sh c4 base roll6c32=ORBFE_ROLL=1,ORBFE_ROLL_BANDS=6,ORBFE_ROLL_CHUNK=32 roll8c34=ORBFE_ROLL=1,ORBFE_ROLL_BANDS=8,ORBFE_ROLL_CHUNK=34 roll5c34=ORBFE_ROLL=1,ORBFE_ROLL_BANDS=5,ORBFE_ROLL_CHUNK=34 roll12c34=ORBFE_ROLL=1,ORBFE_ROLL_BANDS=12,ORBFE_ROLL_CHUNK=34 || exit 1
for s in "1" "4" "2 --chunks 2" "2 --chunks 2 --skew 1"; do
  n=$(echo $s | tr -d ' -')
  timeout -k 10 200 python bench.py --cpu-budget 0 --soak-s 1 --streams $s > gpurun_out/abc/c3_s$n.json 2> gpurun_out/abc/c3_s$n.err || exit 1
done
echo TUNE_DONE
