#!/bin/bash
# Quick round-4 check in one gpurun call: the GPU suite, c3 / c4 / c4 per-rank-32 bench lines and
# the single-frame rows (Python and C++ callers).  Output: gpurun_out/chk_<tag>/
set -o pipefail
T=${1:-a}
O=gpurun_out/chk_$T
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_suite.log 2>&1 && \
timeout -k 10 300 python bench.py --cpu-budget 0 --soak-s 2 > $O/bench_c3.json 2> $O/c3.err && \
timeout -k 10 300 python bench.py --config c4 --cpu-budget 0 --soak-s 2 > $O/bench_c4.json 2> $O/c4.err && \
timeout -k 10 300 python bench.py --config c4 --per-rank 32 --cpu-budget 0 --soak-s 2 > $O/bench_c4_per_rank32.json 2> $O/c4_32.err && \
timeout -k 10 600 python tools/bench_rows.py single > $O/rows_single.jsonl 2> $O/rows.err && \
echo CHECK_DONE
