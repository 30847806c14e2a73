# Quick A/B: for each variant NAME, the extractor parity tests and two c3 bench runs with
# ORBFE_LIB=orbslam_mapsave_amd/lib/liborbfe_NAME.so ("base" = liborbfe.so).
mkdir -p gpurun_out/ab
set -o pipefail
for v in "$@"; do
  if [ "$v" = base ]; then export ORBFE_LIB=$PWD/orbslam_mapsave_amd/lib/liborbfe.so;
  else export ORBFE_LIB=$PWD/orbslam_mapsave_amd/lib/liborbfe_$v.so; fi
  timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_extract.py -m gpu > gpurun_out/ab/t_$v.log 2>&1 || exit 1
  for r in 1 2; do
    timeout -k 10 120 python bench.py --cpu-budget 0 --steps 30 > gpurun_out/ab/b_${v}_$r.json 2>&1 || exit 1
  done
done
echo AB_DONE
