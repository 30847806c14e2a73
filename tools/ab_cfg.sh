#!/bin/bash
# A/B over environment settings for one bench config: bash tools/ab_cfg.sh CONFIG NAME=VARS... ;
# each variant: one bench line (single-stream per-stage table from the probe steps).
# VARS are comma-separated VAR=VALUE pairs ("base", "base2", ... = none).  Output gpurun_out/abc/CONFIG_NAME.json
mkdir -p gpurun_out/abc
set -o pipefail
C=$1; shift
for v in "$@"; do
  name=${v%%=*}
  case $v in base*) E="";; *) E=$(echo "${v#*=}" | tr ',' ' ');; esac  # base, base2, ...: no settings
  timeout -k 10 200 env $E python bench.py --config $C --cpu-budget 0 --soak-s 1 --steps 10 $AB_ARGS > gpurun_out/abc/${C}_${name}.json 2> gpurun_out/abc/${C}_${name}.err || exit 1
done
echo ABC_DONE
