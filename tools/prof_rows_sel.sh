#!/bin/bash
# Rows bench for the named rows (tools/bench_rows.py NAME ...) + its rocprofv3 kernel trace.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/prof_rows_sel
mkdir -p $OUT
timeout -k 10 600 python tools/bench_rows.py "$@" > $OUT/rows.jsonl 2> $OUT/rows.err
timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $OUT -o run --output-format csv -- python3 tools/bench_rows.py "$@" > $OUT/stdout.txt 2>&1
echo ROWS_DONE
