#!/bin/bash
# bench-only A/B (variants that break parity on purpose): two c3 runs per variant
mkdir -p gpurun_out/ab
for v in "$@"; do
  if [ "$v" = base ]; then export ORBFE_LIB=$PWD/orbslam_mapsave_amd/lib/liborbfe.so;
  else export ORBFE_LIB=$PWD/orbslam_mapsave_amd/lib/liborbfe_$v.so; fi
  for r in 1 2; do
    timeout -k 10 120 python bench.py --cpu-budget 0 --steps 30 $BENCH_ARGS > gpurun_out/ab/b_${v}_$r.json 2>&1 || exit 1
  done
done
echo AB_DONE
