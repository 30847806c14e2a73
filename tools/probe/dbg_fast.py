import sys, numpy as np
sys.path.insert(0, '.')  # run from the repo root: FAST candidate lists per level vs the oracle
import oracle
from orbslam_mapsave_amd.native import ORBextractor
from orbslam_mapsave_amd.synth import synthetic_frame
for cfg in [(500, 1.5, 4, 20, 7, 1280, 720), (1000, 1.2, 8, 20, 7, 640, 480)]:
    nf, sf, nl, ini, mn, w, h = cfg
    e = ORBextractor(nf, sf, nl, ini, mn, device=0, max_width=w, max_height=h)
    p = oracle.params(nf, sf, nl, ini, mn)
    img = synthetic_frame(11, w, h)
    e(img)
    for lv, plane in enumerate(oracle.pyramid(p, img)):
        g = e.get_fast_keys(lv); o = oracle.fast_keys(p, plane)
        same = len(g) == len(o) and np.array_equal(g, o)
        print(cfg, lv, len(g), len(o), same)
        if not same:
            gs = set(map(tuple, np.asarray(g).reshape(len(g), -1).tolist())); os_ = set(map(tuple, np.asarray(o).reshape(len(o), -1).tolist()))
            print(' only gpu', sorted(gs - os_)[:10]); print(' only ora', sorted(os_ - gs)[:10])
            n = min(len(g), len(o))
            d = [i for i in range(n) if not np.array_equal(g[i], o[i])]
            print(' first order diff', d[:3], g[d[0]] if d else None, o[d[0]] if d else None)
    e.close()
