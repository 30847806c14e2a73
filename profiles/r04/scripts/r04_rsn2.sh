#!/bin/bash
# resizeN chain length A/B at c4: pairs (ORBFE_RSN=0), chains of <= 3, chains of <= 4.
set -o pipefail
O=gpurun_out/rsn2
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_pyramid.py -m gpu -k "per_level_kernels_exact" > $O/tests.log 2>&1 || exit 1
for r in 1 2; do
  for v in rs2 n3 n4; do
    case $v in rs2) E="ORBFE_RSN=0";; n3) E="ORBFE_RSN_MAX=3";; n4) E="ORBFE_RSN_MAX=4";; esac
    timeout -k 10 200 env $E python bench.py --config c4 --cpu-budget 0 --soak-s 1 --steps 10 > $O/c4_${v}_$r.json 2> $O/c4_${v}_$r.err || exit 1
  done
done
echo RSN2_DONE
