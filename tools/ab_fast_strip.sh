#!/bin/bash
# FAST strip kernel (fast_strip_kernel, opt-in: ORBFE_FAST_STRIP=1) vs one wave per cell (the
# default, ORBFE_FAST_STRIP=0): FAST parity tests with the tree as is, then interleaved c3 / c4 lines, then the strip kernel's phase clocks
# (tools/probe/fast_timing.py, built beforehand).  Output gpurun_out/${1:-fstrip}/
set -o pipefail
O=gpurun_out/${1:-fstrip}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_extract.py tests/test_gpu_fast_list.py tests/test_gpu_workload.py tests/test_gpu_x86_arith.py -m gpu > $O/tests.log 2>&1 || { echo TESTS_FAILED; exit 1; }
for r in 1 2; do
  for v in 0 1; do
    ORBFE_FAST_STRIP=$v timeout -k 10 200 python bench.py --cpu-budget 0 --soak-s 1 --steps 20 > $O/c3_s${v}_$r.json 2> $O/c3_s${v}_$r.err || exit 1
  done
done
for v in 0 1; do
  ORBFE_FAST_STRIP=$v timeout -k 10 200 python bench.py --config c4 --cpu-budget 0 --soak-s 1 --steps 10 > $O/c4_s${v}.json 2> $O/c4_s${v}.err || exit 1
done
if [ -f tools/probe/build/liborbfe_fastt.so ]; then
  timeout -k 10 120 python tools/probe/fast_timing.py run > $O/fast_timing.json 2>&1 || exit 1
fi
echo FSTRIP_DONE
