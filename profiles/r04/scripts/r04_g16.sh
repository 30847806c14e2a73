#!/bin/bash
# describe at 16 keypoints per wave (ORBFE_DESC_G16=1) A/B at c4 / c3, parity first; then the
# driver's round-end commands (smoke, default bench line, rows).
set -o pipefail
O=gpurun_out/g16
mkdir -p $O
ORBFE_DESC_G16=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_extract.py tests/test_gpu_workload.py tests/test_gpu_x86_arith.py -m gpu > $O/tests.log 2>&1 || exit 1
for r in 1 2; do
  for v in base g16; do
    if [ $v = base ]; then E="ORBFE_DESC_G16=0"; else E="ORBFE_DESC_G16=1"; fi
    timeout -k 10 200 env $E python bench.py --config c4 --cpu-budget 0 --soak-s 1 --steps 10 > $O/c4_${v}_$r.json 2> $O/c4_${v}_$r.err || exit 1
    timeout -k 10 200 env $E python bench.py --cpu-budget 0 --soak-s 1 --steps 20 > $O/c3_${v}_$r.json 2> $O/c3_${v}_$r.err || exit 1
  done
done
echo G16_DONE
bash tools/r04_driver_check.sh
