#!/bin/bash
# Full GPU parity suite + c3 lines in both readings + the fetch calibration.  gpurun_out/r04s/
set -o pipefail
O=gpurun_out/r04s
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_suite.log 2>&1 && \
timeout -k 10 300 python bench.py --cpu-budget 0 > $O/bench_c3.json 2> $O/bench_c3.err && \
timeout -k 10 300 python bench.py --cpu-budget 0 --arith scalar > $O/bench_c3_scalar.json 2> $O/bench_c3_scalar.err && \
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/cal/fetch -o run --output-format csv -- ./tools/probe/fetch_cal > $O/fetch_stdout.txt 2>&1 && \
echo SUITE_DONE
