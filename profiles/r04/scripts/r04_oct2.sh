#!/bin/bash
# fused-sweep oct-tree: parity, phase timing, benches
set -o pipefail
O=gpurun_out/oct2
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_extract.py tests/test_gpu_octree_global.py tests/test_gpu_workload.py tests/test_gpu_capacity.py tests/test_gpu_zero_copy.py tests/test_gpu_x86_arith.py tests/test_gpu_fast_list.py -m gpu > $O/tests.log 2>&1 && \
OCT_B=1 timeout -k 10 120 python tools/probe/oct_timing.py run > $O/b1.json 2>&1 && \
OCT_B=32 OCT_W=1920 OCT_H=1080 OCT_NF=2000 timeout -k 10 120 python tools/probe/oct_timing.py run > $O/c4_32t.json 2>&1 && \
timeout -k 10 300 python bench.py --cpu-budget 0 --soak-s 2 > $O/c3.json 2> $O/c3.err && \
timeout -k 10 300 python bench.py --config c4 --per-rank 32 --cpu-budget 0 --soak-s 2 > $O/c4_32.json 2> $O/c4_32.err && \
timeout -k 10 300 python bench.py --config c2 --cpu-budget 0 --soak-s 1 > $O/c2.json 2> $O/c2.err && \
timeout -k 10 200 python tools/bench_rows.py single > $O/rows_single.jsonl 2> $O/rows_single.err && echo OCT2_DONE
