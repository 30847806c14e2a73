#!/bin/bash
# round-6 measurement call: stage-overlap probe, FAST phase clocks, c3 default vs --pipeline 1,
# then the GPU suite.  Output under gpurun_out/$1/.
set -o pipefail
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python tools/probe/stage_overlap.py > $O/overlap.json 2> $O/overlap.err &&
timeout -k 10 300 python tools/probe/fast_timing.py run > $O/fast_phases.json 2> $O/fast_phases.err &&
timeout -k 10 300 python bench.py --cpu-budget 0 --soak-s 2 > $O/bench_c3.json 2> $O/c3.err &&
timeout -k 10 300 python bench.py --cpu-budget 0 --soak-s 2 --pipeline 1 > $O/bench_c3_pipe.json 2> $O/c3p.err &&
bash tools/gpu_suite.sh $T suite
