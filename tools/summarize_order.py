#!/usr/bin/env python3
"""gpurun_out/order/ (tools/ab_order.sh) -> profiles/r04/experiments/describe_order.json: the
describe kernel's HBM traffic and time with the oct-tree's band processing order on / off
(ORBFE_DESC_ORDER), per config.  Traffic = 2 x FETCH_SIZE + WRITE_SIZE (the window-pattern
calibration of profiles/r04/experiments/describe_stride.json), per 256 frames, from the
bench-shape launches (the largest describe grid of each run; frames = its grid y)."""
import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "gpurun_out", sys.argv[1] if len(sys.argv) > 1 else "order")
DST = os.path.join(ROOT, "profiles", "r04", "experiments", "describe_order.json")


def counter_per_256(d, counter):
    trace = {int(r["Dispatch_Id"]): r for r in csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv")))}
    per = collections.defaultdict(float)
    grid = {}
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        if "describe" not in r["Kernel_Name"] or r["Counter_Name"] != counter:
            continue
        i = int(r["Dispatch_Id"])
        per[i] += float(r["Counter_Value"])
        grid[i] = int(r["Grid_Size"])
    big = max(grid.values())
    sel = [i for i in per if grid[i] == big]
    frames = int(trace[sel[0]]["Grid_Size_Y"]) if sel[0] in trace else None
    kb = sum(per[i] for i in sel) / len(sel)
    return kb * 1024 * 256 / frames, frames, len(sel)


out = {"what": __doc__.split("\n\n")[0].replace("\n", " "), "configs": {}}
for c in ("c3", "c4"):
    res = {}
    for v in ("1", "0"):
        f, frames, n = counter_per_256(os.path.join(SRC, f"{c}_order{v}_FETCH_SIZE"), "FETCH_SIZE")
        w, _, _ = counter_per_256(os.path.join(SRC, f"{c}_order{v}_WRITE_SIZE"), "WRITE_SIZE")
        line = json.loads(open(os.path.join(SRC, f"{c}_order{v}.json")).read().strip().splitlines()[-1])
        res["band_order" if v == "1" else "output_order"] = {
            "fetch_raw_MB": round(f / 1e6, 1), "write_MB": round(w / 1e6, 1),
            "hbm_MB_per_256_frames": round((2 * f + w) / 1e6, 1),
            "frames_per_launch": frames, "launches": n,
            "describe_ms_per_step": line["stage_ms_per_step"]["describe"],
            "frames_per_s": line["value"], "ms_per_step": line["ms_per_step"]}
    out["configs"][c] = res
json.dump(out, open(DST, "w"), indent=1)
print(json.dumps(out, indent=1))
