#!/usr/bin/env python3
"""Summarise gpurun_out/ablib_<tag>/ (tools/ab_lib.sh): frames/s and stage times per build."""
import glob
import json
import os
import sys

d = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out", "ablib_" + sys.argv[1])
out = {}
for f in sorted(glob.glob(os.path.join(d, "*.json"))):
    line = json.loads(open(f).read().strip().splitlines()[-1])
    out[os.path.basename(f)[:-5]] = {"frames_per_s": round(line["value"]), "ms_per_step": line["ms_per_step"],
                                     "stage_ms": line["stage_ms_per_step"]}
print(json.dumps(out, indent=1))
