#!/bin/bash
# Kernel trace of the config-5 call (SearchLocalPoints, one frame per step): per-kernel
# durations and the gaps between them.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/prof_c5
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $OUT -o run --output-format csv -- python3 bench.py --config c5 --cpu-budget 0 --steps 50 > $OUT/stdout.txt 2>&1
echo C5PROF_DONE
