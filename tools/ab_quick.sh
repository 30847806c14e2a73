#!/bin/bash
# Quick check of the in-tree build: the named GPU test files (default: the extraction parity
# files), then c3 lines x2 and one c4 line.  bash tools/ab_quick.sh TAG [test files...]
# Output gpurun_out/TAG/; show with python tools/ab_show_fast.py TAG
set -o pipefail
T=${1:?tag}; shift
O=gpurun_out/$T
mkdir -p $O
TESTS=${@:-tests/test_gpu_extract.py tests/test_gpu_fast_list.py tests/test_gpu_workload.py tests/test_gpu_x86_arith.py}
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread $TESTS -m gpu > $O/tests.log 2>&1 || { echo TESTS_FAILED; exit 1; }
for r in 1 2; do
  timeout -k 10 200 python bench.py --cpu-budget 0 --soak-s 1 --steps 20 > $O/c3_s_$r.json 2> $O/c3_$r.err || exit 1
done
timeout -k 10 200 python bench.py --config c4 --cpu-budget 0 --soak-s 1 --steps 10 > $O/c4_s.json 2> $O/c4.err || exit 1
echo QUICK_DONE
