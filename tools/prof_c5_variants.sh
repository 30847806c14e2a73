#!/bin/bash
# rocprofv3 kernel traces of the config-5 call for library variants: gpurun_out/prof_c5_<v>/
set -e
export TMPDIR=/tmp
for v in "$@"; do
  OUT=gpurun_out/prof_c5_$v
  mkdir -p $OUT
  if [ "$v" = base ]; then export ORBFE_LIB=$PWD/orbslam_mapsave_amd/lib/liborbfe.so;
  else export ORBFE_LIB=$PWD/orbslam_mapsave_amd/lib/liborbfe_$v.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 bench.py --config c5 --cpu-budget 0 --steps 30 > $OUT/stdout.txt 2>&1
done
echo C5V_DONE
