#!/bin/bash
# Final round-4 evidence, part A: GPU suite + c3 profile set (bench, rocprofv3 trace, PMC passes)
set -o pipefail
mkdir -p gpurun_out/ev_r04
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ev_r04/gpu_suite.log 2>&1 && \
timeout -k 10 900 bash tools/profile_round.sh r04 --soak-s 3 --cpu-budget 15 && \
echo EV_A_DONE
