#!/bin/bash
# round-4 A/B batch: VALU issue rates, the x86 resize formula (library A/B), config 4 at 32 frames
# per rank, describe attribution
set -o pipefail
timeout -k 10 120 ./tools/probe/build/valu_rate > gpurun_out/valu_rate.txt 2>&1 && \
bash tools/ab_lib.sh rs3 c3 c4 && bash tools/ab_c4_32.sh && bash tools/desc_attr.sh
