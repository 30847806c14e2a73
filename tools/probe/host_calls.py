#!/usr/bin/env python3
"""Latency of the host-form matcher calls (one call per tracked frame in the reference), for
A/B runs of two library builds: ORBFE_LIB selects the library (orbslam_mapsave_amd/native.py).

  python tools/probe/host_calls.py   (GPU box) -> one JSON line, ms per call
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def timed(fn, k, warm=5):
    for _ in range(warm):
        fn()
    t0 = time.perf_counter()
    for _ in range(k):
        fn()
    return (time.perf_counter() - t0) / k * 1e3


def vocab_arrays(k, L, seed, anchors):
    """tools/bench_rows.py's complete k-ary synthetic vocabulary (that module initialises torch,
    which this probe does not load)."""
    import numpy as np
    rng = np.random.Generator(np.random.PCG64(seed))
    parent, desc, word, weight = [np.zeros(1, np.int32)], [np.zeros((1, 32), np.uint8)], [np.zeros(1, np.uint8)], [np.zeros(1)]
    prev, prev_desc, nid = np.zeros(1, np.int64), np.zeros((1, 32), np.uint8), 1
    for level in range(1, L + 1):
        cnt = len(prev) * k
        if level == 1:
            d = anchors[np.arange(cnt) % len(anchors)]
        else:
            bits = np.unpackbits(np.repeat(prev_desc, k, axis=0), axis=1)
            bits ^= (rng.uniform(size=bits.shape) < 0.12).astype(np.uint8)
            d = np.packbits(bits, axis=1)
        leaf = level == L
        parent.append(np.repeat(prev, k).astype(np.int32))
        desc.append(d)
        word.append(np.full(cnt, int(leaf), np.uint8))
        weight.append(np.where(rng.uniform(size=cnt) < 0.03, 0.0, rng.uniform(0.5, 8.0, cnt)) if leaf else np.zeros(cnt))
        prev, prev_desc, nid = np.arange(nid, nid + cnt), d, nid + cnt
    return (np.concatenate(parent), np.concatenate(word), np.ascontiguousarray(np.concatenate(desc)),
            np.concatenate(weight))


def main():
    import scenarios as S
    from orbslam_mapsave_amd import native
    out = {"lib": os.environ.get("ORBFE_LIB", "in-tree")}
    c = S.sbp_keyframe_case(0)
    m = native.ORBmatcher(0.9, True, device=0)
    out["reloc_sbp"] = timed(lambda: m.SearchByProjectionKeyFrame(
        c["cur"], c["tcw_cur"], c["cam"], c["log_scale"], c["kf_angle"], c["kf_valid"], c["kf_bad"],
        c["found"], c["kf_xyz"], c["kf_desc"], c["kf_min"], c["kf_max"], 10, 100,
        frame_mp=c["frame_mp"], kf_ids=c["kf_ids"]), 200)
    c = S.sbp_last_case(0)
    args = (c["cur"], c["tcw_cur"], c["cam"], c["last_keys"], c["last_valid"], c["last_outlier"],
            c["last_xyz"], c["last_desc"], c["last_nobs"], c["tcw_last"])
    out["sbp_last"] = timed(lambda: m.SearchByProjectionLast(*args, 15.0, True, last_ids=c["last_ids"]), 200)
    f, mps, fmp, fobs, ids = S.sbp_local_case(0, 2000)
    out["sbp_local"] = timed(lambda: m.SearchByProjection(f, mps, 3.0, fmp, fobs, ids), 200)
    f, mps, fmp, fobs, ids = S.sbp_local_case(0, 50000)  # past the one-workgroup resolver
    out["sbp_local_50k"] = timed(lambda: m.SearchByProjection(f, mps, 3.0, fmp, fobs, ids), 50)
    f1, f2, prev = S.sfi_case(0)
    out["sfi"] = timed(lambda: m.SearchForInitialization(f1, f2, prev, 100), 100)
    m.close()
    # Frame::ComputeBoW through the host ABI: 1000 descriptors, a k = 10, L = 6 vocabulary
    import ctypes as C
    f0 = S.extract_frame(0, 1000, ini=20)
    parent, word, desc, weight = vocab_arrays(10, 6, 0, anchors=f0.desc[::97])
    L = native.lib()
    st = C.c_int(0)
    h = L.orbfe_vocabulary_create(10, 6, 0, 0, len(parent), native.ptr(parent), native.ptr(word),
                                  native.ptr(desc), native.ptr(weight), 0, C.byref(st))
    gv = native.Vocabulary.__new__(native.Vocabulary)
    gv._h = C.c_void_p(h)
    out["bow_transform"] = timed(lambda: gv.transform(f0.desc, 4), 200)
    gv.close()
    # Frame::ComputeStereoMatches through the host ABI on the pair the two extractors just made
    from orbslam_mapsave_amd.synth import synthetic_stereo_pair
    a, b = synthetic_stereo_pair(0, 640, 480)
    el = native.ORBextractor(1000, 1.2, 8, 20, 7, device=0, max_width=640, max_height=480)
    er = native.ORBextractor(1000, 1.2, 8, 20, 7, device=0, max_width=640, max_height=480)
    kl, dl = el(a)
    kr, dr = er(b)
    out["stereo"] = timed(lambda: el.ComputeStereoMatches(er, kl, dl, kr, dr, 50.0, 0.1), 200)
    el.close()
    er.close()
    print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in out.items()}), flush=True)


if __name__ == "__main__":
    main()
