#!/bin/bash
# config 4 at 32 frames per rank: two vs three sub-batch streams, alternated three times
set -o pipefail
mkdir -p gpurun_out/p32s
timeout -k 10 300 python -u -m pytest tests/test_gpu_pyramid.py -m gpu -x -q --timeout 120 --timeout-method thread -k 'column_tiles or roll_plans' > gpurun_out/p32s/tests.txt 2>&1 || { echo TESTS_FAILED; exit 1; }
for i in 1 2 3; do
  for s in 2 3; do
    timeout -k 10 200 python bench.py --config c4 --per-rank 32 --cpu-budget 0 --soak-s 2 --steps 20 --streams $s \
        > gpurun_out/p32s/s${s}_$i.json 2> gpurun_out/p32s/s${s}_$i.err || exit 1
  done
done
echo P32S_DONE
