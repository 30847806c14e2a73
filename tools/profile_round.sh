#!/bin/bash
# Collects one bench configuration's profile evidence on the GPU box (run via gpurun from the
# repo root):  tools/profile_round.sh <name> [bench.py args...]
#   1. bench.py <args> -> bench.json
#   2. rocprofv3 --kernel-trace --stats of the same command -> kernel stats
#   3. separate --pmc passes for FETCH_SIZE, WRITE_SIZE and the SQ wave counters
#      (MI355X_MICROARCH.md: one TCC counter group per pass; no trace domains mixed with --pmc)
# Output: gpurun_out/prof_<name>/ ; tools/summarize_profile.py <name> turns it into
# profiles/<name>/ and profiles/traffic_<config>.json.
set -e
R=${1:-r03}
shift || true
OUT=gpurun_out/prof_${R//\//_}
mkdir -p $OUT
export TMPDIR=/tmp
echo "$@" > $OUT/bench_args.txt
timeout -k 10 400 python3 bench.py "$@" > $OUT/bench_stdout.txt 2>&1
grep "^{" $OUT/bench_stdout.txt | tail -1 > $OUT/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py "$@" --cpu-budget 0 > $OUT/trace_stdout.txt 2>&1
grep "^{" $OUT/trace_stdout.txt > $OUT/trace_bench.json
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/pmc_fetch -o run --output-format csv -- python3 bench.py "$@" --cpu-budget 0 --steps 5 --warmup 1 --soak-s 0 > $OUT/pmc_fetch_stdout.txt 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/pmc_write -o run --output-format csv -- python3 bench.py "$@" --cpu-budget 0 --steps 5 --warmup 1 --soak-s 0 > $OUT/pmc_write_stdout.txt 2>&1
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU --kernel-trace -d $OUT/pmc_sq -o run --output-format csv -- python3 bench.py "$@" --cpu-budget 0 --steps 5 --warmup 1 --soak-s 0 > $OUT/pmc_sq_stdout.txt 2>&1
echo PROFILE_DONE
