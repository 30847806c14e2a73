#!/usr/bin/env python3
"""Turns gpurun_out/prof_<round>/ (tools/profile_round.sh) into the committed summaries under
profiles/<round>/ and profiles/traffic_c3.json (read by bench.py for roofline.traffic).

Traffic per launch = 2 x FETCH_SIZE + WRITE_SIZE (KB -> bytes): on gfx950 FETCH_SIZE counts half
of the bytes of a coalesced streaming read (MI355X_MICROARCH.md §HBM); our kernels read dwords
per lane, a width the guide lists as uncalibrated, so the doubled figure is an estimate."""
import csv
import collections
import json
import os
import shutil
import sys

R = sys.argv[1] if len(sys.argv) > 1 else "r01"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "gpurun_out", f"prof_{R}")
DST = os.path.join(ROOT, "profiles", R)
os.makedirs(DST, exist_ok=True)

def short(name):
    return name.split("(")[0].replace("orbfe::", "").replace("void ", "")

# kernel stats (copy + a compact table)
shutil.copy(os.path.join(SRC, "trace", "run_kernel_stats.csv"), os.path.join(DST, "kernel_stats.csv"))
for f in ("bench.json", "trace_bench.json"):
    shutil.copy(os.path.join(SRC, f), os.path.join(DST, f))

# per-kernel launches of the timed bench shape (largest grid of each kernel)
def pmc(kind):
    rows = list(csv.DictReader(open(os.path.join(SRC, f"pmc_{kind}", "run_counter_collection.csv"))))
    best = {}
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in rows:
        n = short(r["Kernel_Name"])
        if not n.endswith("kernel") or "at::" in r["Kernel_Name"]:
            continue
        g = int(r["Grid_Size"])
        best[n] = max(best.get(n, 0), g)
        acc[n][g].append((r["Counter_Name"], float(r["Counter_Value"]), int(r["Dispatch_Id"])))
    out = {}
    for n, g in best.items():
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        for c, v, d in acc[n][g]:
            per[d][c] += v
        disp = list(per.values())
        out[n] = {c: sum(d[c] for d in disp) / len(disp) for c in disp[0]}
        out[n]["dispatches"] = len(disp)
        out[n]["grid"] = g
    return out

fetch, write, sq = pmc("fetch"), pmc("write"), pmc("sq")
summary, traffic = {}, {}
for n in sorted(fetch):
    f = fetch[n].get("FETCH_SIZE", 0.0) * 1024
    w = write.get(n, {}).get("WRITE_SIZE", 0.0) * 1024
    s = sq.get(n, {})
    wc = s.get("SQ_WAVE_CYCLES", 0) or 1
    waves = s.get("SQ_WAVES", 1) or 1
    summary[n] = {"grid": fetch[n]["grid"], "fetch_bytes_raw": f, "write_bytes": w,
                  "hbm_bytes_est": 2 * f + w,
                  "active_pct": round(100 * s.get("SQ_ACTIVE_INST_ANY", 0) / wc, 1),
                  "wait_pct": round(100 * s.get("SQ_WAIT_ANY", 0) / wc, 1),
                  "wait_inst_pct": round(100 * s.get("SQ_WAIT_INST_ANY", 0) / wc, 1),
                  "valu_per_wave": round(s.get("SQ_INSTS_VALU", 0) / waves, 1),
                  "lds_per_wave": round(s.get("SQ_INSTS_LDS", 0) / waves, 1)}
    stage = n.replace("_kernel", "")
    traffic[stage] = round(2 * f + w)
json.dump(summary, open(os.path.join(DST, "pmc_summary.json"), "w"), indent=1)
json.dump(traffic, open(os.path.join(ROOT, "profiles", "traffic_c3.json"), "w"), indent=1)
for n, v in summary.items():
    print(n, v)

# Average duration of the bench-shaped launches (largest grid per kernel) from the kernel trace;
# this is the figure bench.py's live roofline.avg_launch_ms must agree with.
rows = list(csv.DictReader(open(os.path.join(SRC, "trace", "run_kernel_trace.csv"))))
grid = collections.defaultdict(int)
for r in rows:
    g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
    grid[short(r["Kernel_Name"])] = max(grid[short(r["Kernel_Name"])], g)
dur = collections.defaultdict(list)
for r in rows:
    n = short(r["Kernel_Name"])
    g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
    if g == grid[n]:
        dur[n].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
launch = {n: {"launches": len(v), "grid": grid[n], "avg_ms": round(sum(v) / len(v) / 1e6, 5)}
          for n, v in dur.items() if n.endswith("kernel")}
json.dump(launch, open(os.path.join(DST, "bench_shape_launches.json"), "w"), indent=1)
for n, v in sorted(launch.items()):
    print(n, v)
