#!/usr/bin/env python3
"""Per-phase attribution of the default FAST kernel (fast_kernel, one wave per cell) at the
bench shapes.

Build (here, CPU):  python tools/probe/fast_timing.py build  -> tools/probe/build/liborbfe_fastt.so
Run (GPU box):      python tools/probe/fast_timing.py run    -> JSON on stdout
The variant library is liborbfe.so compiled with -DORBFE_FAST_TIMING: lane 0 of every wave of
frames < 8 records, per phase, the shader-clock cycles it spent (every mark waits for the wave's
outstanding memory operations, so a phase owns its loads' latency) and the work it did
(orbfe_extract.hip, "ORBFE_FAST_TIMING"): 0 staging, 1 pre-test sweeps, 2 list writes,
3 scoring, 4 emission, 5 overflow flushes, 6 minThFAST rerun pass, 7 total; counts 8 sweeps,
9 survivors scored, 10 corners emitted, 11 flushes, 12 rerun.  The run also times the timing
build's and the product build's fast_kernel launches (HIP events) at the same shapes, so the
clock fractions can be read against the product's time.
"""
import ctypes as C
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
OUT = os.path.join(ROOT, "tools", "probe", "build", "liborbfe_fastt.so")
PHASES = ["staging", "pretest", "list_writes", "scoring", "emission", "flushes", "rerun_pass", "total"]
COUNTS = ["sweeps", "survivors", "corners", "flushes", "rerun"]
K_FRAMES, K_CELLS = 8, 8192


def build():
    sys.path.insert(0, ROOT)
    import __graft_entry__ as g
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    subprocess.run(["/opt/rocm/bin/hipcc", *g.HIPCC_FLAGS, "-Wno-unused-value", "-DORBFE_FAST_TIMING",
                    "-o", OUT, os.path.join(g.CSRC, "orbfe_lib.hip")], check=True)


def fast_ms(lib_path, W, H, NF, B, reps=20):
    """Mean fast_kernel launch time (ms) of the given library at (W, H, NF) x B frames, and
    (for the timing build) the per-wave records of the last launch."""
    code = f"""
import json, os, sys, ctypes as C
os.environ["ORBFE_LIB"] = {lib_path!r}
sys.path.insert(0, {ROOT!r})
import numpy as np, torch
torch.zeros(1, device="cuda:0")
from orbslam_mapsave_amd import native
from orbslam_mapsave_amd.synth import synthetic_batch
W, H, NF, B = {W}, {H}, {NF}, {B}
fr = torch.from_numpy(synthetic_batch(B, W, H, first_seed=1000, distinct=min(B, 16))).cuda()
e = native.ORBextractor(NF, 1.2, 8, 20, 7, device=0, max_width=W, max_height=H, max_batch=B)
cap = e.capacity(W, H)
k = torch.empty((B, cap * 28), dtype=torch.uint8, device="cuda:0")
d = torch.empty((B, cap, 32), dtype=torch.uint8, device="cuda:0")
n = torch.empty(B, dtype=torch.int32, device="cuda:0")
def go():
    e.extract_batch_device(fr.data_ptr(), B, W, H, W, W * H, k.data_ptr(), cap, d.data_ptr(), n.data_ptr())
for _ in range(5): go()
torch.cuda.synchronize()
e.profile(True, stages=("fast",))
L = native.lib()
assert hasattr(L, "orbfe_debug_fast_timing") == {lib_path!r}.endswith("fastt.so")
if hasattr(L, "orbfe_debug_fast_timing_reset"):
    L.orbfe_debug_fast_timing_reset()
for _ in range({reps}): go()
torch.cuda.synchronize()
ms, launches = e.profile_read()["fast"]
rec = None
if hasattr(L, "orbfe_debug_fast_timing"):
    buf = (C.c_longlong * ({K_FRAMES} * {K_CELLS} * 16))()
    L.orbfe_debug_fast_timing(buf, {K_FRAMES} * {K_CELLS} * 16)
    a = np.frombuffer(buf, dtype=np.int64).reshape({K_FRAMES}, {K_CELLS}, 16)[:min(B, {K_FRAMES})]
    a = a[:, (a[..., 7] > 0).any(0)]
    rec = a.reshape(-1, 16).tolist()
print(json.dumps({{"ms": ms / max(launches, 1), "rec": rec}}))
"""
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    if r.returncode:
        raise RuntimeError(r.stderr[-3000:])
    return json.loads(r.stdout.strip().splitlines()[-1])


def summarize(rec):
    import numpy as np
    a = np.asarray(rec, dtype=np.float64)
    a = a[a[:, 7] > 0]
    tot = a[:, 7].sum()
    out = {"waves": int(len(a)),
           "cycles_per_wave": {p: round(float(a[:, i].mean()), 1) for i, p in enumerate(PHASES)},
           "share_of_total": {p: round(float(a[:, i].sum() / tot), 4) for i, p in enumerate(PHASES[:7])},
           "per_wave": {c: round(float(a[:, 8 + i].mean()), 2) for i, c in enumerate(COUNTS)}}
    return out


def run():
    sys.path.insert(0, ROOT)
    prod = os.path.join(ROOT, "orbslam_mapsave_amd", "lib", "liborbfe.so")
    res = {}
    for name, (W, H, NF, B) in {"c3": (640, 480, 1000, 512), "c4": (1920, 1080, 2000, 256)}.items():
        t = fast_ms(OUT, W, H, NF, B)
        p = fast_ms(prod, W, H, NF, B)
        res[name] = {"shape": [W, H, NF, B], "fast_ms_product": round(p["ms"], 4),
                     "fast_ms_timing_build": round(t["ms"], 4), **summarize(t["rec"])}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
