#!/bin/bash
# describe / FAST / pyramid PMC detail (one rocprofv3 --pmc pass each): instruction mix, LDS
# bank conflicts and LDS activity per kernel.  Output gpurun_out/pmc_SQ_INSTS_VALU*/
set -o pipefail
export TMPDIR=/tmp
for K in describe fast_kernel pyramid_kernel; do
  OUT=gpurun_out/pmcd_$K
  mkdir -p $OUT
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU \
      --kernel-trace --kernel-include-regex $K -d $OUT -o run --output-format csv -- \
      python3 bench.py --cpu-budget 0 --steps 3 --warmup 1 --streams 1 --soak-s 0 > $OUT/stdout.txt 2>&1 || exit 1
done
echo PMCD_DONE
