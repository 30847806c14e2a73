#!/usr/bin/env python3
"""Turns gpurun_out/prof_<name>/ (tools/profile_round.sh <name> [bench args]) into the committed
summaries under profiles/<name>/ and profiles/traffic_<config>.json (read by bench.py for
roofline.traffic; keys "<stage>" for the scalar reading, "<stage>@x86" for --arith x86).

Traffic per launch = 2 x FETCH_SIZE + WRITE_SIZE (KB -> bytes): on gfx950 FETCH_SIZE counts half
of the bytes of a coalesced streaming read (MI355X_MICROARCH.md §HBM).  The guide calibrates 16-B
reads only; tools/probe/fetch_cal.hip measures the same 0.5 for 4-B-per-lane reads and 1.0 for
WRITE_SIZE at 4 and 16 B per lane (profiles/r01/fetch_calibration.json)."""
import csv
import collections
import json
import os
import re
import shutil
import sys

R = sys.argv[1] if len(sys.argv) > 1 else "r03"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "gpurun_out", "prof_" + R.replace("/", "_"))
DST = os.path.join(ROOT, "profiles", R)
os.makedirs(DST, exist_ok=True)

def short(name):
    return re.sub(r"<.*>$", "", name.split("(")[0].replace("orbfe::", "").replace("void ", ""))

# kernel stats (copy + a compact table)
shutil.copy(os.path.join(SRC, "trace", "run_kernel_stats.csv"), os.path.join(DST, "kernel_stats.csv"))
for f in ("bench.json", "trace_bench.json", "bench_args.txt"):
    if not os.path.exists(os.path.join(SRC, f)):
        continue
    shutil.copy(os.path.join(SRC, f), os.path.join(DST, f))

# Bench-shape launches: the timed launches of bench.py process one sub-batch of FRAMES frames
# (grid y = frames for every kernel); the parity launches before timing use fewer.  The kernel
# trace has the grid per dimension; the PMC csv only the total, so the bench shapes found in the
# trace (kernel, total grid) select the PMC dispatches.  Multi-launch stages (resize: one launch
# per level) are averaged over all their bench-shape launches, as bench.py's avg_launch_ms is.
_cfg = json.loads(open(os.path.join(SRC, "bench.json")).read())["config"]
# round 4: the probe and roofline legs run the rank's whole batch in one call (the timed steps'
# sub-batch launches are not what roofline.avg_launch_ms times)
FRAMES = int(os.environ.get("BENCH_SUBBATCH", 0)) or _cfg["frames_per_rank_per_step"]
trace_rows = list(csv.DictReader(open(os.path.join(SRC, "trace", "run_kernel_trace.csv"))))
shapes = collections.defaultdict(set)


def bench_shape(r):  # frames on grid y, or on grid x (oct-tree, resize tail: a block per frame)
    return (int(r["Grid_Size_Y"]) == FRAMES or
            int(r["Grid_Size_X"]) == FRAMES * int(r["Workgroup_Size_X"]))


for r in trace_rows:
    if bench_shape(r):
        shapes[short(r["Kernel_Name"])].add(
            int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"]))

def pmc(kind):
    rows = list(csv.DictReader(open(os.path.join(SRC, f"pmc_{kind}", "run_counter_collection.csv"))))
    per = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
    for r in rows:
        n = short(r["Kernel_Name"])
        if not n.endswith("kernel") or "at::" in r["Kernel_Name"]:
            continue
        if int(r["Grid_Size"]) not in shapes.get(n, ()):
            continue
        per[n][int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    out = {}
    for n, disp in per.items():
        d = list(disp.values())
        out[n] = {c: sum(x[c] for x in d) / len(d) for c in d[0]}
        out[n]["dispatches"] = len(d)
        out[n]["grids"] = sorted(shapes[n])
    return out

fetch, write, sq = pmc("fetch"), pmc("write"), pmc("sq")
summary, traffic = {}, {}
for n in sorted(fetch):
    f = fetch[n].get("FETCH_SIZE", 0.0) * 1024
    w = write.get(n, {}).get("WRITE_SIZE", 0.0) * 1024
    s = sq.get(n, {})
    wc = s.get("SQ_WAVE_CYCLES", 0) or 1
    waves = s.get("SQ_WAVES", 1) or 1
    summary[n] = {"grids": fetch[n]["grids"], "dispatches": fetch[n]["dispatches"], "fetch_bytes_raw": f, "write_bytes": w,
                  "hbm_bytes_est": 2 * f + w,
                  "active_pct": round(100 * s.get("SQ_ACTIVE_INST_ANY", 0) / wc, 1),
                  "wait_pct": round(100 * s.get("SQ_WAIT_ANY", 0) / wc, 1),
                  "wait_inst_pct": round(100 * s.get("SQ_WAIT_INST_ANY", 0) / wc, 1),
                  "valu_per_wave": round(s.get("SQ_INSTS_VALU", 0) / waves, 1),
                  "lds_per_wave": round(s.get("SQ_INSTS_LDS", 0) / waves, 1)}
    stage = n.replace("_kernel", "")
    traffic[stage] = round(2 * f + w)
json.dump(summary, open(os.path.join(DST, "pmc_summary.json"), "w"), indent=1)
# VALU wave-instructions per bench-shape launch (SQ_INSTS_VALU is summed over the dispatch's
# waves): bench.py's roofline.valu and stage_roofline valu_frac read them
valu = {n: {"valu_per_launch": round(s_.get("SQ_INSTS_VALU", 0.0)), "waves_per_launch": round(s_.get("SQ_WAVES", 0.0)),
            "dispatches": int(s_["dispatches"])} for n, s_ in sq.items() if "SQ_INSTS_VALU" in s_}
CONF = next((c for c in ("c2", "c3", "c4") if f"--config {c}" in open(
    os.path.join(SRC, "bench_args.txt")).read()), "c3") if os.path.exists(
    os.path.join(SRC, "bench_args.txt")) else "c3"
ARITH = _cfg.get("arith", "scalar")
tpath = os.path.join(ROOT, "profiles", f"traffic_{CONF}.json")
tj = json.load(open(tpath)) if os.path.exists(tpath) else {}
if tj.get("frames_per_launch") not in (None, FRAMES):
    tj = {}
def _drop_stale(j):  # this reading's entries are replaced wholesale (a kernel no longer launched goes)
    for k in [k for k in j if isinstance(j[k], (int, float, dict)) and k != "frames_per_launch"
              and (k.endswith(f"@{ARITH}") if ARITH != "scalar" else "@" not in k)]:
        del j[k]


_drop_stale(tj)
tj.update({(k if ARITH == "scalar" else f"{k}@{ARITH}"): v for k, v in traffic.items()})
tj["frames_per_launch"] = FRAMES
tj["source"] = f"profiles/{R}: rocprofv3 --pmc, 2 x FETCH_SIZE + WRITE_SIZE per launch"
json.dump(tj, open(tpath, "w"), indent=1)
vpath = os.path.join(ROOT, "profiles", f"valu_{CONF}.json")
vj = json.load(open(vpath)) if os.path.exists(vpath) else {}
if vj.get("frames_per_launch") not in (None, FRAMES):
    vj = {}
_drop_stale(vj)
vj.update({(k if ARITH == "scalar" else f"{k}@{ARITH}"): v for k, v in valu.items()})
vj["frames_per_launch"] = FRAMES
vj["source"] = f"profiles/{R}: rocprofv3 --pmc SQ_INSTS_VALU per launch"
json.dump(vj, open(vpath, "w"), indent=1)
for n, v in summary.items():
    print(n, v)

# Average duration of the bench-shape launches from the kernel trace; the figure bench.py's
# live roofline.avg_launch_ms must agree with.
dur = collections.defaultdict(list)
for r in trace_rows:
    n = short(r["Kernel_Name"])
    if bench_shape(r) and n.endswith("kernel"):
        dur[n].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
launch = {n: {"launches": len(v), "grids": sorted(shapes[n]), "avg_ms": round(sum(v) / len(v) / 1e6, 5)}
          for n, v in dur.items()}
json.dump(launch, open(os.path.join(DST, "bench_shape_launches.json"), "w"), indent=1)
for n, v in sorted(launch.items()):
    print(n, v)

# The committed bench line was measured before this round's PMC passes: give its roofline the
# traffic just measured, and record its live launch duration beside rocprofv3's for the same
# kernel and shape.
bpath = os.path.join(DST, "bench.json")
line = json.loads(open(bpath).read().strip().splitlines()[-1])
roof = line.get("roofline") or {}
k = roof.get("kernel")
if k:
    roof["traffic"] = traffic.get(k.replace("_kernel", ""), roof.get("traffic"))
    if roof["traffic"] is not None:
        roof["traffic_source"] = f"profiles/{R}/pmc_summary.json (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this command)"
    with open(bpath, "w") as fh:
        fh.write(json.dumps(line) + "\n")
    check = {"kernel": k, "frames_per_launch": FRAMES,
             "bench_avg_launch_ms (HIP events, roofline leg)": roof.get("avg_launch_ms"),
             "rocprofv3_avg_ms (bench-shape launches)": launch.get(k, {}).get("avg_ms"),
             "traffic_bytes_per_launch (2 x FETCH_SIZE + WRITE_SIZE)": roof["traffic"],
             "algorithmic_bytes_per_launch": roof.get("bytes_per_launch")}
    json.dump(check, open(os.path.join(DST, "roofline_check.json"), "w"), indent=1)
    print(check)
