#!/bin/bash
# resizeN_kernel (3-4 pyramid levels per launch): pyramid / extractor parity, then c4 and c4
# per-rank-32 lines with ORBFE_RSN=0 (resize2 pairs) and the default, interleaved.
set -o pipefail
O=gpurun_out/rsn
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_pyramid.py tests/test_gpu_extract.py tests/test_gpu_x86_arith.py tests/test_gpu_workload.py -m gpu > $O/tests.log 2>&1 || exit 1
for r in 1 2; do
  for v in rs2 rsn; do
    if [ $v = rs2 ]; then E="ORBFE_RSN=0"; else E="ORBFE_RSN=1"; fi
    timeout -k 10 200 env $E python bench.py --config c4 --cpu-budget 0 --soak-s 1 --steps 10 > $O/c4_${v}_$r.json 2> $O/c4_${v}_$r.err || exit 1
    timeout -k 10 200 env $E python bench.py --config c4 --per-rank 32 --cpu-budget 0 --soak-s 1 --steps 20 > $O/c4_32_${v}_$r.json 2> $O/c4_32_${v}_$r.err || exit 1
  done
done
echo RSN_DONE
