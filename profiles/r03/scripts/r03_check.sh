#!/bin/bash
# Round-3 GPU check: the whole -m gpu suite, then c3 (scalar / x86), c4 (overlapped exchange,
# 256 and 32 per rank) and c5 bench lines.  Output under gpurun_out/r03/.
set -o pipefail
O=gpurun_out/r03
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_suite.log 2>&1 && \
timeout -k 10 300 python bench.py --cpu-budget 0 > $O/c3.json 2> $O/c3.err && \
timeout -k 10 300 python bench.py --cpu-budget 0 --arith x86 > $O/c3_x86.json 2> $O/c3_x86.err && \
timeout -k 10 300 python bench.py --cpu-budget 0 --config c4 > $O/c4.json 2> $O/c4.err && \
timeout -k 10 300 python bench.py --cpu-budget 0 --config c4 --per-rank 32 > $O/c4_pr32.json 2> $O/c4_pr32.err && \
timeout -k 10 300 python bench.py --cpu-budget 0 --config c4 --per-rank 32 --streams 1 > $O/c4_pr32_s1.json 2> $O/c4_pr32_s1.err && \
timeout -k 10 300 python bench.py --cpu-budget 0 --config c5 > $O/c5.json 2> $O/c5.err && \
echo CHECK_DONE
