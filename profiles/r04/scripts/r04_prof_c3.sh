#!/bin/bash
# c3 profile set on the final tree -> gpurun_out/prof_r04/
set -o pipefail
timeout -k 10 900 bash tools/profile_round.sh r04 --soak-s 3 --cpu-budget 15 && echo PROF_C3_DONE
