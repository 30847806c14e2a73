#!/bin/bash
# describe_kernel attribution: the bench's probe-step stage times with builds that skip one part
# of describe each (ORBFE_DESC_SKIP: 1 blur, 2 IC moments, 4 samples, 8 window loads, 16 trig;
# outputs wrong on purpose), built by hand into orbslam_mapsave_amd/lib/liborbfe_skip<k>.so.
# Output gpurun_out/desc_attr/<k>.json
set -o pipefail
O=gpurun_out/desc_attr
mkdir -p $O
for k in 0 1 2 4 8 16; do
  if [ $k = 0 ]; then unset ORBFE_LIB; else export ORBFE_LIB=$PWD/orbslam_mapsave_amd/lib/liborbfe_skip$k.so; fi
  timeout -k 10 200 python bench.py --cpu-budget 0 --soak-s 1 --steps 10 > $O/$k.json 2> $O/$k.err || exit 1
done
unset ORBFE_LIB
echo DESC_ATTR_DONE
