# tools/probe/host_calls.py with the in-tree library and the builds named
# (tools/probe/build/NAME/liborbfe.so), interleaved
set -e
for i in 1 2 3; do
  for v in new "$@"; do
    if [ $v = new ]; then unset ORBFE_LIB; else export ORBFE_LIB=$PWD/tools/probe/build/$v/liborbfe.so; fi
    timeout -k 10 120 python tools/probe/host_calls.py
  done
done
