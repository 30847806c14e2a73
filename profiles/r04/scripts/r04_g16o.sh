#!/bin/bash
# describe wave size x slot order at c3: time (bench line) and describe traffic (FETCH / WRITE passes).
set -o pipefail
O=gpurun_out/g16o
mkdir -p $O
export TMPDIR=/tmp
for v in g8 g16 g16o2 g8o2; do
  case $v in g8) E="ORBFE_DESC_G16=0";; g16) E="ORBFE_DESC_G16=1";; g16o2) E="ORBFE_DESC_G16=1 ORBFE_DESC_ORDER=2";; g8o2) E="ORBFE_DESC_ORDER=2";; esac
  timeout -k 10 200 env $E python bench.py --cpu-budget 0 --soak-s 1 --steps 20 > $O/c3_$v.json 2> $O/c3_$v.err || exit 1
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 env $E rocprofv3 --pmc $c --kernel-trace --kernel-include-regex describe -d $O/pmc_${v}_$c -o run --output-format csv -- python3 bench.py --cpu-budget 0 --steps 5 --warmup 1 --soak-s 0 > $O/pmc_${v}_$c.txt 2>&1 || exit 1
  done
done
echo G16O_DONE
