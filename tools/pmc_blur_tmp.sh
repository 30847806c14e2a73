set -e
bash tools/pmc_kernel.sh "blur_kernel|describe_kernel" SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU
bash tools/pmc_kernel.sh "blur_kernel|describe_kernel" FETCH_SIZE
bash tools/pmc_kernel.sh "blur_kernel|describe_kernel" WRITE_SIZE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE
echo PMC_DONE
