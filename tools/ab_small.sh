#!/bin/bash
# Small-batch latency A/B over environment settings: parity tests first, then for each
# "NAME=VAR=VALUE" (or "base") the c2 sweep (B = 1 / 64 / 256) and the single-frame rows.
mkdir -p gpurun_out/abs
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_extract.py tests/test_gpu_octree_global.py tests/test_gpu_zero_copy.py tests/test_gpu_workload.py -m gpu > gpurun_out/abs/tests.log 2>&1 || exit 1
for v in "$@"; do
  name=${v%%=*}
  if [ "$v" = base ]; then E=""; else E="${v#*=}"; fi
  timeout -k 10 200 env $E python bench.py --config c2 --cpu-budget 0 --soak-s 1 > gpurun_out/abs/c2_${name}.json 2> gpurun_out/abs/c2_${name}.err || exit 1
  timeout -k 10 200 env $E python tools/bench_rows.py single > gpurun_out/abs/rows_${name}.jsonl 2> gpurun_out/abs/rows_${name}.err || exit 1
done
echo ABS_DONE
