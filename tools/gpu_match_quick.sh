#!/bin/bash
# Matcher parity tests + config-5 bench (run via gpurun while iterating on the matchers).
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_local_points.py tests/test_gpu_match.py tests/test_sbp_keyframe.py tests/test_gpu_capacity.py tests/test_gpu_grid.py tests/test_bow.py -m gpu > gpurun_out/match_tests.log 2>&1 && \
for r in 1 2; do timeout -k 10 200 python bench.py --config c5 --cpu-budget 0 --steps 200 > gpurun_out/c5_$r.json 2>&1 || exit 1; done && echo MATCH_DONE
