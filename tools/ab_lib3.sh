#!/bin/bash
# A/B of library builds on one box: bash tools/ab_lib3.sh TAG "VARIANTS" CONFIG [CONFIG...]
# VARIANTS: names of orbslam_mapsave_amd/lib/liborbfe_<name>.so ("new" = the in-tree liborbfe.so);
# parity of the in-tree build first; each config benched over the variants twice, interleaved.
# Output gpurun_out/ablib_TAG/<config>_<variant>_<i>.json (tools/ab_lib_summary.py TAG)
set -o pipefail
T=$1; V=$2; shift 2
O=gpurun_out/ablib_$T
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_pyramid.py tests/test_gpu_extract.py tests/test_gpu_x86_arith.py tests/test_gpu_zero_copy.py \
    -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 || { echo TESTS_FAILED; exit 1; }
for C in "$@"; do
  for i in 1 2; do
    for v in $V; do
      if [ $v = new ]; then unset ORBFE_LIB; else export ORBFE_LIB=$PWD/orbslam_mapsave_amd/lib/liborbfe_$v.so; fi
      timeout -k 10 300 python bench.py --config $C --cpu-budget 0 --soak-s 1 --steps 10 > $O/${C}_${v}_$i.json 2> $O/${C}_${v}_$i.err || exit 1
    done
  done
done
unset ORBFE_LIB
echo ABLIB_DONE
