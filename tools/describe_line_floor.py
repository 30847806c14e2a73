#!/usr/bin/env python3
"""The least HBM traffic any describe implementation that reads the pyramid through 128-byte L2
lines can have, for the bench's frames: every line a keypoint's raw window touches fetched once
(perfect reuse), against the window bytes themselves (the algorithmic figure, 37 x 40 per
keypoint) and against no reuse at all (each window's lines fetched for it alone).

Keypoints come from the library (GPU), windows as describe_kernel reads them: 43 rows from
y - 21, 48 bytes from ((x - 18) & ~3) - 4 of the keypoint's level, at the slab's row pitch.
Run on the GPU box: python tools/describe_line_floor.py > profiles/r04/experiments/describe_line_floor.json
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from orbslam_mapsave_amd import native  # noqa: E402
from orbslam_mapsave_amd.synth import synthetic_frame  # noqa: E402


def floor_for(w, h, nf, frames=4):
    e = native.ORBextractor(nf, 1.2, 8, 20, 7, device=0, max_width=w, max_height=h)
    win = touched = union = 0
    try:
        for s in range(frames):
            kps, _ = e(synthetic_frame(s, w, h))
            for l in range(8):
                lw, lh = e.get_level(l).shape[1], e.get_level(l).shape[0]
                pitch = (lw + 63) // 64 * 64  # the slab's level pitch (64-byte rows)
                sel = kps[kps["octave"] == l]
                xs = np.rint(sel["x"] / 1.2 ** l).astype(np.int64)
                ys = np.rint(sel["y"] / 1.2 ** l).astype(np.int64)
                lines = set()
                for x, y in zip(xs, ys):
                    x0 = ((int(x) - 18) & ~3) - 4
                    for r in range(int(y) - 21, int(y) + 22):
                        a = r * pitch + x0
                        ls = range(a // 128, (a + 47) // 128 + 1)
                        touched += len(ls)
                        lines.update(ls)
                win += len(xs) * 37 * 40
                union += len(lines)
    finally:
        e.close()
    mb = lambda v: round(v / frames / 1e6, 3)  # noqa: E731
    return {"window_bytes_MB_per_frame": mb(win), "no_reuse_MB_per_frame": mb(128 * touched),
            "perfect_reuse_MB_per_frame": mb(128 * union),
            "floor_over_window_bytes": round(union * 128 / win, 2)}


out = {"what": __doc__.split("\n\n")[0].replace("\n", " "),
       "c3_640x480_1000": floor_for(640, 480, 1000), "c4_1920x1080_2000": floor_for(1920, 1080, 2000)}
print(json.dumps(out, indent=1))
