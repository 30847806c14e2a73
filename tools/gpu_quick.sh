# Quick GPU check used while iterating: bf_match parity, sharded path, bench (1 and 2 streams).
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 300 python -m pytest tests/test_gpu_match.py -x -q -k "bf_match or hamming" > gpurun_out/bf_test.log 2>&1 && \
timeout -k 10 300 python -m pytest tests/test_shard.py -x -q > gpurun_out/shard_test.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --streams 1 --cpu-budget 0 > gpurun_out/bench_s1.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-budget 0 > gpurun_out/bench_bf.log 2>&1
