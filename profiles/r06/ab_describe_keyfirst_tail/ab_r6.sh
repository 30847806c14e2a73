#!/bin/bash
# round-6 A/B call: describe parity tests on the in-tree build, then interleaved c3 lines of the
# base library (tools/probe/build/base/liborbfe.so, built from HEAD's sources) and the in-tree one,
# ORBFE_TAIL=0, and the c4 / c4_32 / c5 lines.  Output gpurun_out/$1/.
set -o pipefail
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
B="python bench.py --cpu-budget 0 --soak-s 2"
timeout -k 10 600 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_workload.py tests/test_gpu_forced_paths.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit 1
for i in 1 2; do
  ORBFE_LIB=$PWD/tools/probe/build/base/liborbfe.so timeout -k 10 300 $B > $O/c3_base_$i.json 2> $O/c3_base_$i.err || exit 1
  timeout -k 10 300 $B > $O/c3_new_$i.json 2> $O/c3_new_$i.err || exit 1
  ORBFE_TAIL=0 timeout -k 10 300 $B > $O/c3_notail_$i.json 2> $O/c3_notail_$i.err || exit 1
done
timeout -k 10 300 $B --config c4 > $O/c4.json 2> $O/c4.err &&
timeout -k 10 300 $B --config c4 --per-rank 32 > $O/c4_32.json 2> $O/c4_32.err &&
timeout -k 10 300 $B --config c5 > $O/c5.json 2> $O/c5.err &&
echo AB_DONE
