#!/bin/bash
# Quick bench set: c3 default line, c4 (256 and 32 per rank).  Output under gpurun_out/r04q/.
set -o pipefail
O=gpurun_out/r04q
mkdir -p $O
timeout -k 10 300 python bench.py --cpu-budget 0 > $O/c3.json 2> $O/c3.err && \
timeout -k 10 300 python bench.py --config c4 --cpu-budget 0 --soak-s 2 > $O/c4.json 2> $O/c4.err && \
timeout -k 10 300 python bench.py --config c4 --per-rank 32 --cpu-budget 0 --soak-s 2 > $O/c4_32.json 2> $O/c4_32.err && \
echo QUICK_DONE
