#!/usr/bin/env python3
"""Per-phase timing of the oct-tree kernel (octree_kernel) at the bench shape.

Build (here, CPU):  python tools/probe/oct_timing.py build   -> tools/probe/build/liborbfe_octt.so
Run (GPU box):      python tools/probe/oct_timing.py run     -> per level: mean cycles per phase
The variant library is liborbfe.so compiled with -DORBFE_OCT_TIMING (thread 0 of every tree
records clock64() at the phase boundaries; orbfe_debug_oct_timing copies them out).
"""
import ctypes as C
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
OUT = os.path.join(ROOT, "tools", "probe", "build", "liborbfe_octt.so")


def build():
    sys.path.insert(0, ROOT)
    import __graft_entry__ as g
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    subprocess.run(["/opt/rocm/bin/hipcc", *g.HIPCC_FLAGS, "-DORBFE_OCT_TIMING", "-o", OUT,
                    os.path.join(g.CSRC, "orbfe_lib.hip")], check=True)


def run():
    os.environ["ORBFE_LIB"] = OUT
    sys.path.insert(0, ROOT)
    import numpy as np
    import torch
    from orbslam_mapsave_amd import native
    from orbslam_mapsave_amd.synth import synthetic_batch
    torch.zeros(1, device="cuda:0")
    W, H, B = int(os.environ.get("OCT_W", "640")), int(os.environ.get("OCT_H", "480")), int(os.environ.get("OCT_B", "256"))
    NF = int(os.environ.get("OCT_NF", "1000"))
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
    buf = np.zeros(256 * 16 * 64, np.int64)
    assert L.orbfe_debug_oct_timing(C.c_void_p(buf.ctypes.data), len(buf)) == 0
    t = buf.reshape(256, 16, 64)[:B, :8]
    start = t[:, :, 0].min()
    res = {}
    for l in range(8):
        x = t[:, l]
        meta = x[:, 30]
        npass, nround, nkeys = meta & 0xff, (meta >> 8) & 0xff, meta >> 16
        d = lambda a, b: float(np.mean(x[:, b] - x[:, a]))
        p1_end = np.array([x[i, 4 + min(npass[i], 8) - 1] if npass[i] else x[i, 3] for i in range(B)])
        res[l] = {"keys": float(nkeys.mean()), "passes": float(npass.mean()), "rounds": float(nround.mean()),
                  "count": d(0, 1), "compact": d(1, 2), "init": d(2, 3),
                  "phase1": float(np.mean(p1_end - x[:, 3])),
                  "phase2+final": float(np.mean(x[:, 31] - p1_end)),
                  "total": d(0, 31),
                  "start_offset": float(np.mean(x[:, 0] - start)), "end_max": float(x[:, 31].max() - start)}
        # fine marks (pass 1 of phase 1, round 0 of phase 2, init, final): mean step durations
        def step(a, b):
            ok = (x[:, a] > 0) & (x[:, b] > 0)
            return float(np.mean(x[ok, b] - x[ok, a])) if ok.any() else None
        res[l]["fine"] = {"init_clear": step(2, 56), "init_keys": step(56, 57), "init_scan": step(57, 58),
                          "init_node": step(58, 3),
                          "p1_clear": step(4, 32), "p1_sweep": step(32, 33), "p1_scan": step(33, 34),
                          "p1_children": step(34, 35), "p1_sweep2": step(35, 5),
                          "p2_flag": step(40, 41), "p2_sort": step(41, 43), "p2_sweep": step(43, 44),
                          "p2_cut": step(44, 45), "p2_clear": step(45, 46), "p2_proc_scan": step(46, 47),
                          "p2_kept_scan": step(47, 48), "p2_children": step(48, 49), "p2_sweep2": step(49, 12),
                          "final_best": step(52, 53), "final_out": step(53, 31)}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
