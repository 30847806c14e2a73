#!/bin/bash
# Oct-tree split launch A/B: levels 0..k-1 as 512/1024-thread trees in their own launch.
set -o pipefail
O=gpurun_out/osplit
mkdir -p $O
ORBFE_OCT_SPLIT=2 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_extract.py tests/test_gpu_octree_global.py tests/test_gpu_workload.py -m gpu > $O/tests.log 2>&1 || exit 1
for r in 1 2; do
  for v in base s1b512 s1b1024 s2b512; do
    case $v in base) E="ORBFE_OCT_SPLIT=0";; s1b512) E="ORBFE_OCT_SPLIT=1 ORBFE_OCT_SPLIT_BLK=512";;
      s1b1024) E="ORBFE_OCT_SPLIT=1 ORBFE_OCT_SPLIT_BLK=1024";; s2b512) E="ORBFE_OCT_SPLIT=2 ORBFE_OCT_SPLIT_BLK=512";; esac
    timeout -k 10 200 env $E python bench.py --cpu-budget 0 --soak-s 1 --steps 20 > $O/c3_${v}_$r.json 2> $O/c3_${v}_$r.err || exit 1
    timeout -k 10 200 env $E python bench.py --config c4 --cpu-budget 0 --soak-s 1 --steps 10 > $O/c4_${v}_$r.json 2> $O/c4_${v}_$r.err || exit 1
  done
done
echo OSPLIT_DONE
