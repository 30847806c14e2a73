"""Print the FAST strip A/B lines of gpurun_out/<tag>/ (tools/ab_fast_strip.sh)."""
import glob, json, os, sys
d = os.path.join("gpurun_out", sys.argv[1] if len(sys.argv) > 1 else "fstrip")
for f in sorted(glob.glob(os.path.join(d, "c*_s*.json"))):
    j = json.load(open(f))
    s = j["stage_ms_per_step"]
    print(os.path.basename(f), round(j["value"]), j["ms_per_step"], "fast", s["fast"], "resize", s["resize"],
          "describe", s["describe"], "octree", s["octree"])
t = os.path.join(d, "fast_timing.json")
if os.path.exists(t):
    print(open(t).read())
