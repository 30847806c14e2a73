# SearchByBoW single-call latency from C++ (tests/cpp/adapter_test's BOW_LATENCY line), the
# in-tree library against the variants named (tools/probe/build/NAME/liborbfe.so), interleaved
set -e
for i in 1 2 3; do
  for v in new "$@"; do
    if [ $v = new ]; then L=""; else L=$PWD/tools/probe/build/$v; fi
    echo -n "$v "; LD_LIBRARY_PATH=$L timeout -k 10 60 tests/cpp/build/adapter_test 2>&1 | grep BOW_LATENCY
  done
done
