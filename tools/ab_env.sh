#!/bin/bash
# A/B over environment settings: for each "NAME=VAR=VALUE" (or "base"), two c3 bench runs.
# Parity first: the extractor GPU tests under the default environment.
mkdir -p gpurun_out/ab
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_extract.py tests/test_gpu_x86_arith.py tests/test_color_mask.py -m gpu > gpurun_out/ab/tests.log 2>&1 || exit 1
for v in "$@"; do
  name=${v%%=*}
  for r in 1 2; do
    if [ "$v" = base ]; then
      timeout -k 10 120 python bench.py --cpu-budget 0 --steps 30 > gpurun_out/ab/b_${name}_$r.json 2>&1 || exit 1
    else
      timeout -k 10 120 env ${v#*=} python bench.py --cpu-budget 0 --steps 30 > gpurun_out/ab/b_${name}_$r.json 2>&1 || exit 1
    fi
  done
done
echo AB_DONE
