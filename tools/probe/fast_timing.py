#!/usr/bin/env python3
"""Per-phase timing of the strip FAST kernel (fast_strip_kernel) at the bench shape.

Build (here, CPU):  python tools/probe/fast_timing.py build  -> tools/probe/build/liborbfe_fastt.so
Run (GPU box):      python tools/probe/fast_timing.py run    -> mean shader cycles per phase
The variant library is liborbfe.so compiled with -DORBFE_FAST_TIMING (lane 0 of each wave records
clock64() at the phase boundaries of runs < 160 of frames < 64; orbfe_debug_fast_timing copies
them out).  Marks: 0 start, 1 ROI staged, 2 after barrier 1, 3-6 phase 1 done per wave, 7 after
barrier 2, 8-11 phase 2 done per wave, 12-15 minThFAST reruns per wave.
"""
import ctypes as C
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
OUT = os.path.join(ROOT, "tools", "probe", "build", "liborbfe_fastt.so")


def build():
    sys.path.insert(0, ROOT)
    import __graft_entry__ as g
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    subprocess.run(["/opt/rocm/bin/hipcc", *g.HIPCC_FLAGS, "-DORBFE_FAST_TIMING", "-o", OUT,
                    os.path.join(g.CSRC, "orbfe_lib.hip")], check=True)


def run():
    os.environ["ORBFE_LIB"] = OUT
    sys.path.insert(0, ROOT)
    import numpy as np
    import torch
    from orbslam_mapsave_amd import native
    from orbslam_mapsave_amd.synth import synthetic_batch
    torch.zeros(1, device="cuda:0")
    W, H, B = int(os.environ.get("FT_W", "640")), int(os.environ.get("FT_H", "480")), int(os.environ.get("FT_B", "256"))
    NF = int(os.environ.get("FT_NF", "1000"))
    frames = torch.from_numpy(synthetic_batch(B, W, H, distinct=32)).cuda()
    e = native.ORBextractor(NF, 1.2, 8, 32, 7, device=0, max_width=W, max_height=H, max_batch=B)
    cap = e.capacity(W, H)
    kps = torch.empty((B, cap * 28), dtype=torch.uint8, device="cuda")
    desc = torch.empty((B, cap, 32), dtype=torch.uint8, device="cuda")
    n = torch.empty(B, dtype=torch.int32, device="cuda")
    for _ in range(3):
        e.extract_batch_device(frames.data_ptr(), B, W, H, W, W * H, kps.data_ptr(), cap,
                               desc.data_ptr(), n.data_ptr())
    e.synchronize()
    L = native.lib()
    buf = np.zeros(64 * 160 * 16, np.int64)
    assert L.orbfe_debug_fast_timing(C.c_void_p(buf.ctypes.data), len(buf)) == 0
    t = buf.reshape(64, 160, 16)[:min(B, 64)]
    t = t[t[:, :, 0] > 0]          # runs that exist
    d = lambda a, b: float(np.mean(t[:, b] - t[:, a]))
    p1 = t[:, 3:7] - t[:, 2:3]      # per wave: phase 1
    p2 = t[:, 8:12] - t[:, 7:8]     # per wave: phase 2
    res = {"runs": int(len(t)), "stage": d(0, 1), "barrier1": d(1, 2),
           "phase1_mean_wave": float(p1.mean()), "phase1_max_wave": float(p1.max(1).mean()),
           "barrier2_after_max": float(np.mean(t[:, 7] - t[:, 3:7].max(1))),
           "phase2_mean_wave": float(p2.mean()), "phase2_max_wave": float(p2.max(1).mean()),
           "total": float(np.mean(t[:, 8:12].max(1) - t[:, 0])),
           "reruns_per_run": float(t[:, 12:16].sum(1).mean()),
           "phase2_max_wave_no_rerun": float(p2[t[:, 12:16].sum(1) == 0].max(1).mean()),
           "phase2_max_wave_rerun": float(p2[t[:, 12:16].sum(1) > 0].max(1).mean())}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
