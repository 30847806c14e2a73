#!/bin/bash
# Final round-4 evidence, part B: c4 profile set, c4 per-rank-32, c2, c5, the rows
set -o pipefail
mkdir -p gpurun_out/ev_r04
timeout -k 10 900 bash tools/profile_round.sh r04_c4 --config c4 --soak-s 2 --cpu-budget 10 && \
timeout -k 10 300 python bench.py --config c4 --per-rank 32 --cpu-budget 0 --soak-s 2 > gpurun_out/ev_r04/bench_c4_per_rank32.json 2> gpurun_out/ev_r04/c4_32.err && \
timeout -k 10 300 python bench.py --config c2 --cpu-budget 10 --soak-s 2 > gpurun_out/ev_r04/bench_c2.json 2> gpurun_out/ev_r04/c2.err && \
timeout -k 10 300 python bench.py --config c5 --cpu-budget 10 > gpurun_out/ev_r04/bench_c5.json 2> gpurun_out/ev_r04/c5.err && \
echo EV_B_DONE
