# bench.py with the in-tree library against the builds named (tools/probe/build/NAME/liborbfe.so),
# interleaved R times: bash tools/probe/bench_ab.sh TAG R NAME... ; extra bench args in $AB_ARGS
# -> gpurun_out/TAG/<name>_<r>.json
set -o pipefail
T=${1:?tag}; R=${2:?reps}; shift 2
mkdir -p gpurun_out/$T
for r in $(seq 1 $R); do
  for v in new "$@"; do
    if [ $v = new ]; then unset ORBFE_LIB; else export ORBFE_LIB=$PWD/tools/probe/build/$v/liborbfe.so; fi
    timeout -k 10 200 python bench.py --cpu-budget 0 --soak-s 1 $AB_ARGS > gpurun_out/$T/${v}_$r.json 2> gpurun_out/$T/${v}_$r.err || exit 1
  done
done
unset ORBFE_LIB
echo AB_DONE
