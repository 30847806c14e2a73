#!/bin/bash
# describe's band processing order (ORBFE_DESC_ORDER) A/B: extraction parity tests, then per
# config (c3, c4) and variant (band order on / off) the bench line and the describe kernel's
# FETCH_SIZE / WRITE_SIZE passes (one counter group per rocprofv3 run).
# Output: gpurun_out/order/ ; tools/summarize_order.py turns it into
# profiles/r04/experiments/describe_order.json.
set -o pipefail
O=gpurun_out/order
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_pyramid.py tests/test_gpu_x86_arith.py tests/test_gpu_zero_copy.py tests/test_shard_c4.py \
    -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 || { echo TESTS_FAILED; exit 1; }
for C in c4 c3; do
  for V in 1 0; do
    export ORBFE_DESC_ORDER=$V
    timeout -k 10 300 python bench.py --config $C --cpu-budget 0 --soak-s 1 --steps 10 > $O/${C}_order$V.json 2> $O/${C}_order$V.err || exit 1
    for P in FETCH_SIZE WRITE_SIZE; do
      timeout -k 10 300 rocprofv3 --pmc $P --kernel-trace --kernel-include-regex describe -d $O/${C}_order${V}_$P -o run \
          --output-format csv -- python3 bench.py --config $C --cpu-budget 0 --steps 3 --warmup 1 --streams 1 --soak-s 0 \
          > $O/${C}_order${V}_$P.txt 2>&1 || exit 1
    done
  done
done
unset ORBFE_DESC_ORDER
echo ORDER_DONE
