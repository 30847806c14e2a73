#!/bin/bash
# The driver's round-end commands on the final tree: smoke(), the default bench line, then the §8(f) rows.
set -o pipefail
O=gpurun_out/drv
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $O/smoke.log 2>&1 && \
( time timeout -k 10 400 python bench.py ) > $O/bench_default.json 2> $O/bench_default.err && \
timeout -k 10 600 python tools/bench_rows.py > $O/rows.jsonl 2> $O/rows.err && \
echo DRV_DONE
