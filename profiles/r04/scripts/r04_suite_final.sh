#!/bin/bash
# GPU parity suite on the final tree -> gpurun_out/final_suite/
set -o pipefail
mkdir -p gpurun_out/final_suite
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final_suite/gpu_suite.log 2>&1 && \
timeout -k 10 300 python bench.py --cpu-budget 0 --soak-s 2 > gpurun_out/final_suite/c3.json 2> gpurun_out/final_suite/c3.err && \
echo SUITE_DONE
