# Full GPU check: the whole -m gpu suite, then the default bench line.
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/bench_full.log 2>&1
