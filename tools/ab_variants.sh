# A/B of library build variants: bash tools/ab_variants.sh NAME... runs the extractor parity
# tests and the c3 (1 and 2 streams) / c4 benches with ORBFE_LIB=orbslam_mapsave_amd/lib/liborbfe_NAME.so
mkdir -p gpurun_out/ab
set -o pipefail
for v in "$@"; do
  export ORBFE_LIB=$PWD/orbslam_mapsave_amd/lib/liborbfe_$v.so
  timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_extract.py -m gpu > gpurun_out/ab/t_$v.log 2>&1 || exit 1
  timeout -k 10 120 python bench.py --cpu-budget 0 --streams 1 --steps 30 > gpurun_out/ab/b_$v.json 2>&1 || exit 1
  timeout -k 10 120 python bench.py --cpu-budget 0 --streams 2 --steps 30 > gpurun_out/ab/b2_$v.json 2>&1 || exit 1
  timeout -k 10 120 python bench.py --cpu-budget 0 --config c4 > gpurun_out/ab/b4_$v.json 2>&1 || exit 1
done
