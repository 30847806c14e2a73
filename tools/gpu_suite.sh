#!/bin/bash
# Full GPU parity suite + c3/c5 bench lines (run via gpurun from the repo root).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/gpu_suite.log 2>&1 && \
timeout -k 10 300 python bench.py --cpu-budget 0 > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err && \
timeout -k 10 300 python bench.py --config c5 --cpu-budget 0 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err && \
echo SUITE_DONE
