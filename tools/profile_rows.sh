set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_rows
timeout -k 10 900 python tools/bench_rows.py > gpurun_out/rows.jsonl 2> gpurun_out/rows.err
timeout -k 10 900 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/prof_rows -o run --output-format csv -- python3 tools/bench_rows.py > gpurun_out/prof_rows/stdout.txt 2>&1
echo DONE
