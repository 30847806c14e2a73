#!/bin/bash
# Final-tree check: GPU parity suite, then c3 / c4 / c4 per-rank-32 bench lines.  gpurun_out/r04f/
set -o pipefail
O=gpurun_out/r04f
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_suite.log 2>&1 && \
timeout -k 10 300 python bench.py --cpu-budget 0 > $O/c3.json 2> $O/c3.err && \
timeout -k 10 300 python bench.py --config c4 --cpu-budget 0 --soak-s 2 > $O/c4.json 2> $O/c4.err && \
timeout -k 10 300 python bench.py --config c4 --per-rank 32 --cpu-budget 0 --soak-s 2 > $O/c4_32.json 2> $O/c4_32.err && \
echo FINAL_DONE
