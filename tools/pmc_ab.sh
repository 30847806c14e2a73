#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes for kernels matching $1, per library variant ($2 ...)
set -e
RX=$1; shift
for v in "$@"; do
  if [ "$v" = base ]; then export ORBFE_LIB=$PWD/orbslam_mapsave_amd/lib/liborbfe.so;
  else export ORBFE_LIB=$PWD/orbslam_mapsave_amd/lib/liborbfe_$v.so; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    OUT=gpurun_out/pmcab_${v}_$c
    mkdir -p $OUT
    timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --kernel-include-regex "$RX" -d $OUT -o run --output-format csv -- python3 bench.py --cpu-budget 0 --steps 3 --warmup 1 > $OUT/stdout.txt 2>&1
  done
done
echo PMCAB_DONE
