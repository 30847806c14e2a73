#!/bin/bash
# Brute force with the shared reference set pre-expanded (default) vs per-workgroup expansion
# (ORBFE_BF_PRE=0): parity, then c3 lines interleaved.
set -o pipefail
O=gpurun_out/bfpre
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_match.py tests/test_gpu_workload.py tests/test_gpu_capacity.py -m gpu > $O/tests.log 2>&1 || exit 1
for r in 1 2; do
  for v in old pre; do
    if [ $v = old ]; then E="ORBFE_BF_PRE=0"; else E="ORBFE_BF_PRE=1"; fi
    timeout -k 10 200 env $E python bench.py --cpu-budget 0 --soak-s 1 --steps 20 > $O/c3_${v}_$r.json 2> $O/c3_${v}_$r.err || exit 1
  done
done
echo BFPRE_DONE
