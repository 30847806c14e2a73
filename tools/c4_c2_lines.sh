#!/bin/bash
# Config-4 per-rank shapes (256 = 1 GPU, 32 = the 8-GPU per-rank batch) and the config-2 sweep.
set -o pipefail
R=${1:-r02}
mkdir -p gpurun_out/$R
timeout -k 10 300 python bench.py --config c4 --cpu-budget 10 > gpurun_out/$R/bench_c4.json 2> gpurun_out/$R/bench_c4.err && \
timeout -k 10 300 python bench.py --config c4 --per-rank 32 --steps 50 --cpu-budget 0 > gpurun_out/$R/bench_c4_b32.json 2> gpurun_out/$R/bench_c4_b32.err && \
timeout -k 10 300 python bench.py --config c2 --cpu-budget 10 > gpurun_out/$R/bench_c2.json 2> gpurun_out/$R/bench_c2.err && \
echo C4C2_DONE
