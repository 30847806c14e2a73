#!/bin/bash
# Round-4 evidence in one gpurun call: GPU suite, c3 profile set (bench + rocprofv3 trace + PMC
# passes), c4 profile set, c4 per-rank-32, c2, c5 and the rows.  Output under gpurun_out/.
set -o pipefail
R=${1:-r04}
mkdir -p gpurun_out/ev_$R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ev_$R/gpu_suite.log 2>&1 && \
bash tools/profile_round.sh $R --soak-s 3 --cpu-budget 15 && \
bash tools/profile_round.sh ${R}_c4 --config c4 --soak-s 2 --cpu-budget 10 && \
timeout -k 10 300 python bench.py --config c4 --per-rank 32 --cpu-budget 0 --soak-s 2 > gpurun_out/ev_$R/bench_c4_per_rank32.json 2> gpurun_out/ev_$R/c4_32.err && \
timeout -k 10 300 python bench.py --config c2 --cpu-budget 10 --soak-s 2 > gpurun_out/ev_$R/bench_c2.json 2> gpurun_out/ev_$R/c2.err && \
timeout -k 10 300 python bench.py --config c5 --cpu-budget 10 > gpurun_out/ev_$R/bench_c5.json 2> gpurun_out/ev_$R/c5.err && \
timeout -k 10 900 python tools/bench_rows.py > gpurun_out/ev_$R/rows.jsonl 2> gpurun_out/ev_$R/rows.err && \
echo EVIDENCE_DONE
