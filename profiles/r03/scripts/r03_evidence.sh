#!/bin/bash
# Round-3 evidence in one gpurun call: GPU suite, profile sets for c3 (scalar and x86 readings)
# and c4, the c2 sweep, the c5 line and the rows bench.  Output under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03/gpu_suite.log 2>&1 && \
bash tools/profile_round.sh r03 && \
bash tools/profile_round.sh r03_x86 --arith x86 && \
bash tools/profile_round.sh r03_c4 --config c4 && \
timeout -k 10 300 python bench.py --config c2 --cpu-budget 10 > gpurun_out/r03/bench_c2.json 2> gpurun_out/r03/bench_c2.err && \
timeout -k 10 300 python bench.py --config c5 --cpu-budget 10 > gpurun_out/r03/bench_c5.json 2> gpurun_out/r03/bench_c5.err && \
timeout -k 10 900 python tools/bench_rows.py > gpurun_out/r03/rows.jsonl 2> gpurun_out/r03/rows.err && \
echo EVIDENCE_DONE
