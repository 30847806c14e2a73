#!/bin/bash
# FAST cells per workgroup A/B (ORBFE_FAST_WAVES 1 / 2 / 4): FAST parity under 4, then c3 and c4 lines.
set -o pipefail
O=gpurun_out/fw
mkdir -p $O
ORBFE_FAST_WAVES=4 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_extract.py tests/test_gpu_fast_list.py tests/test_gpu_workload.py -m gpu > $O/tests.log 2>&1 || exit 1
for r in 1 2; do
  for v in 1 2 4; do
    timeout -k 10 200 env ORBFE_FAST_WAVES=$v python bench.py --cpu-budget 0 --soak-s 1 --steps 20 > $O/c3_w${v}_$r.json 2> $O/c3_w${v}_$r.err || exit 1
    timeout -k 10 200 env ORBFE_FAST_WAVES=$v python bench.py --config c4 --cpu-budget 0 --soak-s 1 --steps 10 > $O/c4_w${v}_$r.json 2> $O/c4_w${v}_$r.err || exit 1
  done
done
echo FW_DONE
