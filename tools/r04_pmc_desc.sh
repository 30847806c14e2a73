#!/bin/bash
# describe_kernel FETCH_SIZE / WRITE_SIZE at c4 and c3 (single stream), strided vs grouped slots.
set -o pipefail
export TMPDIR=/tmp
for cfg in c4 c3; do
  for v in strided grouped; do
    if [ $v = grouped ]; then export ORBFE_DESC_STRIDE=0; else unset ORBFE_DESC_STRIDE; fi
    for c in FETCH_SIZE WRITE_SIZE; do
      PMC_ARGS="--config $cfg" bash tools/pmc_kernel.sh "describe" $c || exit 1
      rm -rf gpurun_out/pmcd_${cfg}_${v}_$c; mv gpurun_out/pmc_$c gpurun_out/pmcd_${cfg}_${v}_$c
    done
  done
done
echo PMCD_DONE
