#!/bin/bash
# FAST ROI pitch A/B: parity of the extractor tests (default = 11-dword pitch), then c3 / c4 /
# c4 per-rank-32 lines with ORBFE_FAST_P44=0 (48-byte pitch) and default, interleaved.
set -o pipefail
O=gpurun_out/p44
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_extract.py tests/test_gpu_fast_list.py tests/test_gpu_x86_arith.py tests/test_gpu_workload.py -m gpu > $O/tests.log 2>&1 || exit 1
for r in 1 2; do
  for v in p48 p44; do
    if [ $v = p48 ]; then E="ORBFE_FAST_P44=0"; else E="ORBFE_FAST_P44=1"; fi
    timeout -k 10 200 env $E python bench.py --cpu-budget 0 --soak-s 1 --steps 20 > $O/c3_${v}_$r.json 2> $O/c3_${v}_$r.err || exit 1
    timeout -k 10 200 env $E python bench.py --config c4 --cpu-budget 0 --soak-s 1 --steps 10 > $O/c4_${v}_$r.json 2> $O/c4_${v}_$r.err || exit 1
  done
done
echo P44_DONE
