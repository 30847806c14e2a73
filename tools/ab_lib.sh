#!/bin/bash
# A/B of two builds of the library on one box: bash tools/ab_lib.sh TAG CONFIG [CONFIG...]
# "base" = orbslam_mapsave_amd/lib/liborbfe_base.so (the tree before the change, copied there
# by hand), "new" = the in-tree liborbfe.so; each config benched base / new / base / new.
# Parity of the new build first (the pyramid and extraction tests).  Output gpurun_out/ablib_TAG/
set -o pipefail
T=$1; shift
O=gpurun_out/ablib_$T
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_pyramid.py tests/test_gpu_extract.py tests/test_gpu_x86_arith.py \
    -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 || { echo TESTS_FAILED; exit 1; }
for C in "$@"; do
  for i in 1 2; do
    for V in base new; do
      if [ $V = base ]; then export ORBFE_LIB=$PWD/orbslam_mapsave_amd/lib/liborbfe_base.so; else unset ORBFE_LIB; fi
      timeout -k 10 300 python bench.py --config $C --cpu-budget 0 --soak-s 1 --steps 10 > $O/${C}_${V}_$i.json 2> $O/${C}_${V}_$i.err || exit 1
    done
  done
done
unset ORBFE_LIB
echo ABLIB_DONE
