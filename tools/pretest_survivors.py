"""FAST pre-test pricing on CPU: the fraction of pyramid pixels (4 synthetic 640x480 frames,
oracle pyramid, t = 20) that pass (a) the cardinal pre-test fast_kernel uses (two consecutive of
points 0/4/8/12), (b) four consecutive of the 8 even circle points, (c) (b) and the same on the odd
points, against (d) the true 9-arc corners.  DESIGN.md §5a."""
import numpy as np, sys
sys.path.insert(0, '.')
import oracle
from orbslam_mapsave_amd.synth import synthetic_frame
p = oracle.params()
circ = [(3,0),(3,1),(2,2),(1,3),(0,3),(-1,3),(-2,2),(-3,1),(-3,0),(-3,-1),(-2,-2),(-1,-3),(0,-3),(1,-3),(2,-2),(3,-1)]  # (dy,dx)
tot = {}
for seed in range(4):
    img = synthetic_frame(seed)
    pyr = oracle.pyramid(p, img)
    for L, lev in enumerate(pyr):
        v = lev.astype(np.int32)
        H, W = v.shape
        c = v[3:H-3, 3:W-3]
        ring = np.stack([v[3+dy:H-3+dy, 3+dx:W-3+dx] for dy, dx in circ])
        t = 20
        br = ring > c + t; dk = ring < c - t
        def card(b):
            return (b[0] | b[8]) & (b[4] | b[12])
        def even4(b):
            e = b[0::2]  # 8 evens
            cc = e & np.roll(e, -1, axis=0)
            d = cc & np.roll(cc, -2, axis=0)
            return d.any(axis=0)
        def odd4(b):
            e = b[1::2]
            cc = e & np.roll(e, -1, axis=0)
            d = cc & np.roll(cc, -2, axis=0)
            return d.any(axis=0)
        def arc9(b):
            bb = np.concatenate([b, b[:8]])
            run = np.ones_like(b[0])
            res = np.zeros_like(b[0])
            for k in range(16):
                res |= np.all(bb[k:k+9], axis=0)
            return res
        n = c.size
        r = dict(card=(card(br) | card(dk)).sum(), even=(even4(br) | even4(dk)).sum(),
                 evenodd=((even4(br) & odd4(br)) | (even4(dk) & odd4(dk))).sum(),
                 corner=(arc9(br) | arc9(dk)).sum(), n=n)
        for k, x in r.items():
            tot[k] = tot.get(k, 0) + x
print({k: (v / tot['n'] if k != 'n' else v) for k, v in tot.items()})
