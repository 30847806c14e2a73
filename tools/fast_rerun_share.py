#!/usr/bin/env python3
"""CPU pricing of FAST's minThFAST rerun (ORBextractor.cc:764-831): the share of cells (and of
cell pixels) whose pass at iniThFAST finds no corner, on config 3's synthetic frames — the only
cells whose pass-1 scores a rerun could reuse.  python tools/fast_rerun_share.py"""
import math
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle
from orbslam_mapsave_amd.synth import synthetic_frame
p = oracle.params(1000, 1.2, 8, 20, 7)
tot = rerun = kp1 = kp2 = 0
px_all = px_rerun = 0
for seed in range(4):
    img = synthetic_frame(seed, 640, 480)
    levels = oracle.pyramid(p, img)
    for lev in levels:
        lev = np.asarray(lev)
        H, Wd = lev.shape
        minX, minY = 16, 16
        maxX, maxY = Wd - 16, H - 16
        width, height = maxX - minX, maxY - minY
        nCols, nRows = width // 30, height // 30
        wCell, hCell = math.ceil(width / nCols), math.ceil(height / nRows)
        for i in range(nRows):
            iniY = minY + i * hCell
            mY = iniY + hCell + 6
            if iniY >= maxY - 3: continue
            if mY > maxY: mY = maxY
            for j in range(nCols):
                iniX = minX + j * wCell
                mX = iniX + wCell + 6
                if iniX >= maxX - 6: continue
                if mX > maxX: mX = maxX
                roi = np.ascontiguousarray(lev[iniY:mY, iniX:mX])
                k = oracle.fast(roi, 20)
                tot += 1; px_all += roi.size
                if len(k) == 0:
                    rerun += 1; px_rerun += roi.size
                    kp2 += len(oracle.fast(roi, 7))
                else:
                    kp1 += len(k)
print(f"cells {tot} rerun {rerun} ({rerun/tot:.1%}) px share {px_rerun/px_all:.1%}")
