#!/bin/bash
# FETCH_SIZE calibration incl. the describe window pattern, then c4 (single stream, x86
# reading) FETCH_SIZE / WRITE_SIZE passes for the extraction kernels.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/cal
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/cal/fetch -o run --output-format csv -- ./tools/probe/fetch_cal > gpurun_out/cal/fetch_stdout.txt 2>&1 && \
PMC_ARGS="--config c4" bash tools/pmc_kernel.sh "describe|fast|resize|octree|pyramid" FETCH_SIZE && \
PMC_ARGS="--config c4" bash tools/pmc_kernel.sh "describe|fast|resize|octree|pyramid" WRITE_SIZE && echo FETCH_DONE
