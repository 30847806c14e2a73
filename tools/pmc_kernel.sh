#!/bin/bash
# One PMC pass over a short bench run for the kernels matching $1 (regex), counters $2..:
#   bash tools/pmc_kernel.sh bf_match SQ_WAVE_CYCLES SQ_BUSY_CYCLES ...
# Output: gpurun_out/pmc_<first counter>$PMC_TAG/ (kernel-trace + the counters, no other trace domain).
set -e
RX=$1; shift
OUT=gpurun_out/pmc_$1$PMC_TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-trace --kernel-include-regex "$RX" -d $OUT -o run \
    --output-format csv -- python3 bench.py --cpu-budget 0 --steps 3 --warmup 1 --streams 1 --soak-s 0 $PMC_ARGS \
    > $OUT/stdout.txt 2>&1
