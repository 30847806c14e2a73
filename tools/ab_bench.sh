#!/bin/bash
# Bench-only A/B of library build variants (attribution builds whose outputs are wrong on
# purpose, so no parity tests): bash tools/ab_bench.sh NAME... -> gpurun_out/ab/b_NAME.json
# (c3, one stream).  Extra bench arguments in $AB_ARGS.
mkdir -p gpurun_out/ab
set -o pipefail
for v in "$@"; do
  export ORBFE_LIB=$PWD/orbslam_mapsave_amd/lib/liborbfe_$v.so
  timeout -k 10 120 python bench.py --cpu-budget 0 --streams 1 --steps 30 $AB_ARGS > gpurun_out/ab/b_$v$AB_TAG.json 2> gpurun_out/ab/b_$v$AB_TAG.err || exit 1
done
