# bench.py --config c5 with the in-tree library and the builds named
# (tools/probe/build/NAME/liborbfe.so), interleaved; one value per line
set -e
for i in 1 2 3; do
  for v in new "$@"; do
    if [ $v = new ]; then unset ORBFE_LIB; else export ORBFE_LIB=$PWD/tools/probe/build/$v/liborbfe.so; fi
    echo -n "$v "; timeout -k 10 300 python bench.py --config c5 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print(d['value'], d['ms_per_step'], d.get('a14_alone',{}).get('ms_per_call'))"
  done
done
