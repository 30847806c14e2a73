#!/bin/bash
# One gpurun call's checks, chosen by name: bash tools/gpu_suite.sh TAG STEP...
#   suite      the whole -m gpu parity suite
#   smoke      __graft_entry__.smoke()
#   c2 c3 c4 c5    bench lines of that config (c3 = the default line)
#   c4_32      config 4 at 32 frames per rank (the 8-GPU per-rank shape)
#   rows       the §8(f) rows (tools/bench_rows.py)
#   prof_c3 / prof_c4   tools/profile_round.sh TAG[_c4] (bench + rocprofv3 trace + PMC passes)
# Steps run in order, each under its own time limit, and the first failure ends the call.
# Extra bench arguments in $BENCH_ARGS.  Output under gpurun_out/TAG/.
# (Replaces round 3/4's one-off r03_*.sh / r04_*.sh drivers, kept under profiles/r0N/scripts/.)
set -o pipefail
T=${1:?tag}
shift
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
B="python bench.py --cpu-budget 0 --soak-s 2 $BENCH_ARGS"
for s in "$@"; do
  case $s in
    suite) timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_suite.log 2>&1 ;;
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $O/smoke.log 2>&1 ;;
    c2) timeout -k 10 300 $B --config c2 > $O/bench_c2.json 2> $O/c2.err ;;
    c3) timeout -k 10 300 $B > $O/bench_c3.json 2> $O/c3.err ;;
    c4) timeout -k 10 300 $B --config c4 > $O/bench_c4.json 2> $O/c4.err ;;
    c4_32) timeout -k 10 300 $B --config c4 --per-rank 32 > $O/bench_c4_32.json 2> $O/c4_32.err ;;
    c5) timeout -k 10 300 $B --config c5 > $O/bench_c5.json 2> $O/c5.err ;;
    rows) timeout -k 10 600 python tools/bench_rows.py > $O/rows.jsonl 2> $O/rows.err ;;
    prof_c3) timeout -k 10 900 bash tools/profile_round.sh $T --soak-s 3 --cpu-budget 15 ;;
    prof_c4) timeout -k 10 900 bash tools/profile_round.sh ${T}_c4 --config c4 --soak-s 2 --cpu-budget 10 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac || { echo "STEP_FAILED $s"; exit 1; }
  echo "STEP_DONE $s"
done
echo SUITE_DONE
