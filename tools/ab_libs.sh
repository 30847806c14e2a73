#!/bin/bash
# c3 bench with alternative builds of the library (build knobs), interleaved twice:
# bash tools/ab_libs.sh TAG base name1 name2 ...  (name: orbslam_mapsave_amd/lib/liborbfe_<name>.so)
# -> gpurun_out/TAG/<name>_<r>.json ; extra bench args in $AB_ARGS
set -o pipefail
T=${1:?tag}; shift
mkdir -p gpurun_out/$T
for r in 1 2; do
  for n in "$@"; do
    if [ "$n" = base ]; then unset ORBFE_LIB; else export ORBFE_LIB=$PWD/orbslam_mapsave_amd/lib/liborbfe_$n.so; fi
    timeout -k 10 200 python bench.py --cpu-budget 0 --soak-s 1 $AB_ARGS > gpurun_out/$T/${n}_$r.json 2> gpurun_out/$T/${n}_$r.err || exit 1
  done
done
unset ORBFE_LIB
echo LIBS_DONE
