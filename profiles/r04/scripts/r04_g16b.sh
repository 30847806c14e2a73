#!/bin/bash
# describe G16 as the default below 1 Mpx: GPU suite, then c3 default vs ORBFE_DESC_G16=0, c2.
set -o pipefail
O=gpurun_out/g16b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_suite.log 2>&1 || exit 1
for r in 1 2; do
  for v in g8 def; do
    if [ $v = g8 ]; then E="ORBFE_DESC_G16=0"; else E="ORBFE_DESC_G16=-1"; fi
    timeout -k 10 200 env $E python bench.py --cpu-budget 0 --soak-s 1 --steps 20 > $O/c3_${v}_$r.json 2> $O/c3_${v}_$r.err || exit 1
  done
done
timeout -k 10 300 python bench.py --config c2 --cpu-budget 0 --soak-s 2 > $O/c2.json 2> $O/c2.err && \
echo G16B_DONE
