set -e
bash tools/pmc_kernel.sh "blur_band" SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU
bash tools/pmc_kernel.sh "blur_band" FETCH_SIZE
bash tools/pmc_kernel.sh "blur_band" WRITE_SIZE TCC_HIT_sum TCC_MISS_sum
bash tools/pmc_kernel.sh "blur_band" SQ_BUSY_CYCLES GRBM_GUI_ACTIVE TA_BUSY_avr TA_TA_BUSY_sum
echo PMC_DONE
