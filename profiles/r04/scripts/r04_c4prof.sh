#!/bin/bash
# Config-4 profile set on the final tree (bench + rocprofv3 trace + PMC passes) -> gpurun_out/prof_r04_c4/
set -o pipefail
timeout -k 10 1000 bash tools/profile_round.sh r04_c4 --config c4 --soak-s 2 --cpu-budget 10 && echo C4PROF_DONE
