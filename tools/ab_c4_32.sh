#!/bin/bash
# Config 4 at 32 frames per rank (the 8-GPU per-rank shape): pyramid plans and stream layouts.
# Output gpurun_out/abc/c4_p32<name>.json
set -o pipefail
mkdir -p gpurun_out/abc
run() {  # name, env assignments..., -- bench args...
  local n=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done
  shift
  timeout -k 10 200 env "${envs[@]}" python bench.py --config c4 --per-rank 32 --cpu-budget 0 --soak-s 1 --steps 10 "$@" \
      > gpurun_out/abc/c4_p32$n.json 2> gpurun_out/abc/c4_p32$n.err
}
run base -- && run small17 ORBFE_PYR_SMALL_BELOW=17 -- && run roll2 ORBFE_ROLL=2 ORBFE_PYR_SMALL_BELOW=17 -- && \
run s1 -- --streams 1 && run s3 -- --streams 3 && run s4 -- --streams 4 || exit 1
echo C4_32_DONE
