#!/bin/bash
# PMC passes (two counter groups) over the c3 bench for the FAST kernel, strip form and one wave
# per cell (ORBFE_FAST_STRIP=0).  Output gpurun_out/pmc_*_{strip,cell}${TAG}/; show with
# python tools/pmc_show.py fast
set -o pipefail
for v in strip cell; do
  if [ $v = cell ]; then export ORBFE_FAST_STRIP=0; else export ORBFE_FAST_STRIP=1; fi
  PMC_TAG=_$v$TAG timeout -k 10 200 bash tools/pmc_kernel.sh "fast" SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAIT_INST_ANY || exit 1
  PMC_TAG=_$v$TAG timeout -k 10 200 bash tools/pmc_kernel.sh "fast" SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_WAVES SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE || exit 1
done
echo PMC_DONE
