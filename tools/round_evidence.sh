#!/bin/bash
# Round evidence in one gpurun call: GPU suite, profile set (bench + rocprofv3 + PMC passes),
# config-5 line, rows bench.  Output under gpurun_out/.
set -o pipefail
R=${1:-r02}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_suite.log 2>&1 && \
bash tools/profile_round.sh $R && \
timeout -k 10 300 python bench.py --config c5 --cpu-budget 10 > gpurun_out/prof_$R/bench_c5.json 2> gpurun_out/prof_$R/bench_c5.err && \
timeout -k 10 900 python tools/bench_rows.py > gpurun_out/prof_$R/rows.jsonl 2> gpurun_out/prof_$R/rows.err && \
echo EVIDENCE_DONE
