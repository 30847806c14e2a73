#!/usr/bin/env python3
"""Throughput of the §8(f) rows on one MI355X next to their CPU oracle (one JSON line per row).

Each row: GPU path through the C ABI with inputs resident in HBM where the ABI has a device
form (colour extraction, stereo, BoW transform, distinctive descriptors), host forms otherwise
(relocalisation SearchByProjection, SearchByBoW: one keyframe / frame per call, as Tracking
calls them); K timed iterations after warm-up, torch.cuda.synchronize on both sides; the CPU
oracle (single thread, a port of the reference path) on the same inputs.  Algorithmic bytes per
unit are stated per row; the achieved GB/s is those bytes over the measured time.

Run on the GPU box: python tools/bench_rows.py > gpurun_out/rows.jsonl
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402

torch.cuda.init()
DEV = torch.device("cuda", 0)
torch.zeros(1, device=DEV)

import oracle  # noqa: E402  (test infrastructure: the CPU-baseline legs)
from orbslam_mapsave_amd import native  # noqa: E402
from orbslam_mapsave_amd.synth import (synthetic_color_frame, synthetic_frame,  # noqa: E402
                                       synthetic_stereo_pair, synthetic_vocabulary_text)

HBM = 8000.0


def timed(fn, k, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(k):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / k


def cpu_timed(fn, budget=4.0):
    n, t0 = 0, time.perf_counter()
    while True:
        fn()
        n += 1
        el = time.perf_counter() - t0
        if el >= budget and n >= 2:
            return el / n


def emit(row, unit, units_per_call, t_gpu, t_cpu, nbytes, note, cpu_units=None):
    """t_gpu: seconds per GPU call of units_per_call units; t_cpu: seconds per CPU call of
    cpu_units units (default: the same)."""
    cu = units_per_call if cpu_units is None else cpu_units
    line = {"row": row, "unit": unit, "value": round(units_per_call / t_gpu, 2),
            "ms_per_call": round(t_gpu * 1e3, 4), "units_per_call": units_per_call,
            "achieved_GBs": round(nbytes / t_gpu / 1e9, 2),
            "hbm_frac": round(nbytes / t_gpu / 1e9 / HBM, 5),
            "bytes_per_call": int(nbytes),
            "cpu_value": round(cu / t_cpu, 3), "cpu_cores": 1, "cpu_kind": "port",
            "gpu_over_cpu": round((units_per_call / t_gpu) / (cu / t_cpu), 1), "note": note}
    print(json.dumps(line), flush=True)


def row_color():
    B, W, H = 256, 640, 480
    cf = np.stack([synthetic_color_frame(s % 16, W, H, 3) for s in range(B)])
    d_img = torch.from_numpy(cf).to(DEV)
    ex = native.ORBextractor(1000, 1.2, 8, 32, 7, device=0, max_width=W, max_height=H, max_batch=B)
    ex.set_stream(torch.cuda.current_stream(DEV).cuda_stream)
    cap = ex.capacity(W, H)
    k = torch.empty((B, cap * 28), dtype=torch.uint8, device=DEV)
    d = torch.empty((B, cap, 32), dtype=torch.uint8, device=DEV)
    n = torch.empty(B, dtype=torch.int32, device=DEV)
    rects = torch.from_numpy(np.tile(np.array([[200, 100, 400, 300]], np.int32), (B, 1))).to(DEV)

    def go():
        ex.extract_color_batch_device(d_img.data_ptr(), native.PIX_RGB, B, W, H, 3 * W, 3 * W * H,
                                      k.data_ptr(), cap, d.data_ptr(), n.data_ptr(),
                                      d_rects=rects.data_ptr())
    t = timed(go, 10)
    p = oracle.params(1000, 1.2, 8, 32, 7)
    m = np.ones((H, W), np.uint8)
    m[100:300, 200:400] = 0
    tc = cpu_timed(lambda: oracle.extract(p, oracle.cvt_gray(cf[0], native.PIX_RGB), m))
    emit("(f)1 colour + human-mask extraction (RGB 640x480, 1000 kp)", "frames/s", B, t, tc,
         B * (3 * W * H + W * H), "device batch of 256 RGB frames, rectangle mask; bytes = the "
         "level-0 kernel's RGB read + gray write (the rest is the c3 pipeline)", cpu_units=1)
    ex.close()


def row_single():
    """Tracking's per-frame call: ORBextractor::operator() on one 640x480 frame through the host
    ABI (upload, the whole pipeline, download of keypoints and descriptors), as Frame::ExtractORB
    issues it (Frame.cc:358-364) — the latency a drop-in replacement adds per tracked frame."""
    img = synthetic_frame(3, 640, 480)
    ex = native.ORBextractor(1000, 1.2, 8, 20, 7, device=0, max_width=640, max_height=480)
    t = timed(lambda: ex(img), 200)
    p = oracle.params(1000, 1.2, 8, 20, 7)
    tc = cpu_timed(lambda: oracle.extract(p, img))
    emit("single-frame ORBextractor::operator() latency (640x480, 1000 kp, host ABI)",
         "frames/s", 1, t, tc, 640 * 480 + 1000 * 60,
         "host ABI: one frame per call, H2D upload + pipeline + D2H, synchronous", cpu_units=1)
    # the zero-copy form (orbfe_input_buffer / orbfe_extract_staged): the caller's cvtColor
    # writes the gray frame into the handle's pinned staging buffer (written here once, outside
    # the timed calls: that write is the caller's own cvtColor output, not the extractor's work),
    # the GPU reads it in place and the outputs stay in the pinned output buffers
    buf = ex.input_buffer(640, 480)
    buf[:] = img
    k0, d0 = ex(img)
    ks, ds = ex.extract_staged(640, 480, copy_out=False)
    assert ks.tobytes() == k0.tobytes() and np.array_equal(ds, d0)
    t2 = timed(lambda: ex.extract_staged(640, 480, copy_out=False), 400)
    emit("single-frame ORBextractor::operator() latency, zero-copy staging (640x480, 1000 kp)",
         "frames/s", 1, t2, tc, 640 * 480 + 1000 * 60,
         "host ABI orbfe_extract_staged: frame in the handle's pinned buffer (the caller's cvtColor "
         "target), outputs left in pinned memory (orbfe_staged_outputs), one graph launch + one "
         "synchronisation per call", cpu_units=1)
    ex.close()
    # the same calls from C++ (the adapter program, as Frame::ExtractORB would make them): no
    # Python / ctypes in the loop
    import re
    import subprocess
    exe = os.path.join(ROOT, "tests", "cpp", "build", "adapter_test")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    m = re.search(r"LATENCY host_us=([0-9.]+) staged_copy_us=([0-9.]+) staged_us=([0-9.]+)", r.stdout)
    if r.returncode == 0 and m:
        for us, what in ((float(m.group(1)), "host form (orbfe::ORBextractor::operator(), frame copied in)"),
                         (float(m.group(3)), "zero-copy staging (orbfe_extract_staged, outputs in place)")):
            emit(f"single-frame latency from C++, {what} (640x480, 1000 kp)", "frames/s", 1, us * 1e-6, tc,
                 640 * 480 + 1000 * 60, "tests/cpp/adapter_test: mean of 2,000 calls after 100 warm-up "
                 "calls, C++ caller through include/orbfe_orbslam.hpp", cpu_units=1)
    # SearchByBoW(KeyFrame*, Frame&) from C++ (Tracking.cc:1014's per-frame call), GPU against the
    # one-thread CPU port in the same program
    mb = re.search(r"BOW_LATENCY gpu_us=([0-9.]+) cpu_us=([0-9.]+) nodes=(\d+)/(\d+)", r.stdout)
    if r.returncode == 0 and mb:
        gu, cu = float(mb.group(1)), float(mb.group(2))
        emit(f"(f)4 SearchByBoW from C++ (1000 x 1000 features, {mb.group(3)}/{mb.group(4)} nodes)",
             "calls/s", 1, gu * 1e-6, cu * 1e-6, 2000 * (32 + 8),
             "tests/cpp/adapter_test: orbfe::ORBmatcher::SearchByBoW vs oracle_search_by_bow, mean of "
             "2,000 calls after 100 warm-up calls each; one kernel launch per call, the orientation "
             "filter on the host", cpu_units=1)


def row_stereo():
    B, W, H = 128, 640, 480
    pairs = [synthetic_stereo_pair(s % 16, W, H) for s in range(B)]
    L = torch.from_numpy(np.stack([a for a, _ in pairs])).to(DEV)
    R = torch.from_numpy(np.stack([b for _, b in pairs])).to(DEV)
    el = native.ORBextractor(1000, 1.2, 8, 20, 7, device=0, max_width=W, max_height=H, max_batch=B)
    er = native.ORBextractor(1000, 1.2, 8, 20, 7, device=0, max_width=W, max_height=H, max_batch=B)
    s = torch.cuda.current_stream(DEV).cuda_stream
    el.set_stream(s)
    er.set_stream(s)
    cap = el.capacity(W, H)
    bufs = {}
    for side, e, X in (("l", el, L), ("r", er, R)):
        kk = torch.empty((B, cap * 28), dtype=torch.uint8, device=DEV)
        dd = torch.empty((B, cap, 32), dtype=torch.uint8, device=DEV)
        nn = torch.empty(B, dtype=torch.int32, device=DEV)
        e.extract_batch_device(X.data_ptr(), B, W, H, W, W * H, kk.data_ptr(), cap, dd.data_ptr(),
                               nn.data_ptr())
        bufs[side] = (kk, dd, nn)
    ur = torch.empty((B, cap), dtype=torch.float32, device=DEV)
    dp = torch.empty((B, cap), dtype=torch.float32, device=DEV)
    (kl, dl, nl), (kr, dr, nr) = bufs["l"], bufs["r"]

    def go():
        el.compute_stereo_matches_device(er, B, kl.data_ptr(), dl.data_ptr(), nl.data_ptr(),
                                         kr.data_ptr(), dr.data_ptr(), nr.data_ptr(), cap, 50.0,
                                         0.1, ur.data_ptr(), dp.data_ptr())
    t = timed(go, 20)
    p = oracle.params(1000, 1.2, 8, 20, 7)
    a, b = pairs[0]
    okl, odl = oracle.extract(p, a)
    okr, odr = oracle.extract(p, b)
    tc = cpu_timed(lambda: oracle.compute_stereo_matches(p, a, b, okl, odl, okr, odr, 50.0, 0.1))
    nkp = float(nl.float().mean())
    emit("(f)2 stereo ComputeStereoMatches (640x480, 1000 kp per side)", "pairs/s", B, t, tc,
         B * nkp * (2 * 60 + 121 + 231 + 8), "device batch of 128 rectified pairs, pyramids of "
         "both extractors resident; bytes = keypoints + descriptors of both sides + the two SAD "
         "windows + outputs per left keypoint; the CPU leg (oracle) also rebuilds both pyramids "
         "per call, which the reference gets from its extractors", cpu_units=1)
    # the per-frame call (Frame.cc:82): one pair through the host ABI, on batch frame 0's pyramids
    t1 = timed(lambda: el.ComputeStereoMatches(er, okl, odl, okr, odr, 50.0, 0.1, frame=0), 100)
    emit("(f)2 stereo ComputeStereoMatches of one pair (host ABI, 640x480, 1000 kp per side)",
         "pairs/s", 1, t1, tc, nkp * (2 * 60 + 121 + 231 + 8),
         "host ABI: keypoints and descriptors of both sides in by one DMA from a pinned block, "
         "u_right | depth | status back by one; the extractors' pyramids resident", cpu_units=1)
    el.close()
    er.close()


def row_reloc():
    import scenarios as S
    c = S.sbp_keyframe_case(0)
    m = native.ORBmatcher(0.9, True, device=0)

    def go():
        m.SearchByProjectionKeyFrame(c["cur"], c["tcw_cur"], c["cam"], c["log_scale"],
                                     c["kf_angle"], c["kf_valid"], c["kf_bad"], c["found"],
                                     c["kf_xyz"], c["kf_desc"], c["kf_min"], c["kf_max"], 10, 100,
                                     frame_mp=c["frame_mp"], kf_ids=c["kf_ids"])
    t = timed(go, 50)
    tc = cpu_timed(lambda: oracle.search_by_projection_keyframe(c, 10, 100))
    n = len(c["kf_valid"])
    emit("(f)3 relocalisation SearchByProjection(Frame&, KeyFrame*) (1000-point keyframe)",
         "calls/s", 1, t, tc, n * (12 + 32 + 8 + 4 + 3) + c["cur"].n * 60,
         "host ABI (uploads included): latency-bound, 5 launches (scatter, grid, fixed-slot "
         "candidates, one-workgroup resolver, gather) and one wait on a done word")
    m.close()


def row_track():
    """The per-frame tracking-loop matchers through the host ABI (uploads included):
    TrackWithMotionModel's SearchByProjection(CurrentFrame, LastFrame, th, mono)
    (Tracking.cc:1132, ORBmatcher.cc:1331-1473) and MonocularInitialization's
    SearchForInitialization (Tracking.cc:844, ORBmatcher.cc:408-523)."""
    import scenarios as S
    c = S.sbp_last_case(0)
    args = (c["cur"], c["tcw_cur"], c["cam"], c["last_keys"], c["last_valid"], c["last_outlier"],
            c["last_xyz"], c["last_desc"], c["last_nobs"], c["tcw_last"])
    m = native.ORBmatcher(0.9, True, device=0)
    t = timed(lambda: m.SearchByProjectionLast(*args, 15.0, True, last_ids=c["last_ids"]), 50)
    tc = cpu_timed(lambda: oracle.search_by_projection_last(*args, 15.0, True, True,
                                                            last_ids=c["last_ids"]))
    n = len(c["last_valid"])
    emit("tracking SearchByProjection(CurrentFrame, LastFrame) (1000 kp each, mono th 15)",
         "calls/s", 1, t, tc, n * (12 + 32 + 28 + 8) + c["cur"].n * 60,
         "host ABI (uploads included): one call per tracked frame, latency-bound (fixed-slot "
         "candidates, one wait on a done word)")
    m.close()
    # TrackLocalMap's SearchByProjection(Frame&, vector<MapPoint*>, th) (Tracking.cc:1283,
    # ORBmatcher.cc:38-131) through the host ABI, isInFrustum's outputs given, 2000 map points
    f, mps, fmp, fobs, ids = S.sbp_local_case(0, 2000)
    m = native.ORBmatcher(0.8, True, device=0)
    t = timed(lambda: m.SearchByProjection(f, mps, 3.0, fmp, fobs, ids), 50)
    tc = cpu_timed(lambda: oracle.search_by_projection_local(f, mps, 3.0, 0.8, fmp, fobs, ids))
    emit("tracking SearchByProjection(Frame&, local map points) (2000 points, th 3)", "calls/s", 1,
         t, tc, 2000 * (32 + 24) + f.n * 60,
         "host ABI (uploads included): fixed-slot candidates, one-workgroup resolver, one wait")
    m.close()
    f1, f2, prev = S.sfi_case(0)
    m = native.ORBmatcher(0.9, True, device=0)
    t = timed(lambda: m.SearchForInitialization(f1, f2, prev, 100), 20)
    tc = cpu_timed(lambda: oracle.search_for_initialization(f1, f2, prev, 100, 0.9, True))
    emit("initialization SearchForInitialization(F1, F2, window 100) (2000 kp each)", "calls/s",
         1, t, tc, (f1.n + f2.n) * 60,
         "host ABI (uploads included): sequential greedy with steals, one wave resolves it")
    m.close()


def row_distinctive():
    from test_distinctive import make_case
    off, desc = make_case(3, n_mp=50_000, max_obs=20)
    m = native.ORBmatcher(device=0)
    d_off = torch.from_numpy(off).to(DEV)
    d_desc = torch.from_numpy(desc).to(DEV)
    best = torch.empty(len(off) - 1, dtype=torch.int32, device=DEV)
    out = torch.empty((len(off) - 1, 32), dtype=torch.uint8, device=DEV)
    m.set_stream(torch.cuda.current_stream(DEV).cuda_stream)
    import ctypes as C
    L = native.lib()

    def go():
        L.orbfe_distinctive_descriptors_device(m._h, len(off) - 1, C.c_void_p(d_off.data_ptr()),
                                               C.c_void_p(d_desc.data_ptr()),
                                               C.c_void_p(best.data_ptr()),
                                               C.c_void_p(out.data_ptr()))
    t = timed(go, 20)
    sub = 2000
    tc = cpu_timed(lambda: oracle.distinctive_descriptors(off[:sub + 1], desc[:off[sub]])) * (len(off) - 1) / sub
    emit("(f)4 ComputeDistinctiveDescriptors (50k map points, 0-20 observations)", "points/s",
         len(off) - 1, t, tc, len(desc) * 32 + (len(off) - 1) * 40,
         "device form; CPU time scaled from a 2000-point sample")
    m.close()


def vocab_arrays(k=10, L=6, seed=0, anchors=None):
    """A complete k-ary tree of depth L as node arrays (vectorised synthetic ORBvoc stand-in)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    parent, desc, word, weight = [np.zeros(1, np.int32)], [np.zeros((1, 32), np.uint8)], [np.zeros(1, np.uint8)], [np.zeros(1)]
    prev = np.zeros(1, np.int64)
    prev_desc = np.zeros((1, 32), np.uint8)
    nid = 1
    for level in range(1, L + 1):
        cnt = len(prev) * k
        par = np.repeat(prev, k)
        if level == 1:
            d = anchors[np.arange(cnt) % len(anchors)] if anchors is not None else rng.integers(0, 256, (cnt, 32), dtype=np.uint8)
        else:
            bits = np.unpackbits(np.repeat(prev_desc, k, axis=0), axis=1)
            bits ^= (rng.uniform(size=bits.shape) < 0.12).astype(np.uint8)
            d = np.packbits(bits, axis=1)
        leaf = level == L
        parent.append(par.astype(np.int32))
        desc.append(d)
        word.append(np.full(cnt, int(leaf), np.uint8))
        w = np.where(rng.uniform(size=cnt) < 0.03, 0.0, rng.uniform(0.5, 8.0, cnt)) if leaf else np.zeros(cnt)
        weight.append(w)
        prev = np.arange(nid, nid + cnt)
        prev_desc = d
        nid += cnt
    return (np.concatenate(parent), np.concatenate(word), np.ascontiguousarray(np.concatenate(desc)),
            np.concatenate(weight).astype(np.float64))


def row_bow(tmpdir):
    import ctypes as C
    import scenarios as S
    f0 = S.extract_frame(0, 1000, ini=20)
    parent, word, desc, weight = vocab_arrays(10, 6, 0, anchors=f0.desc[::97])
    L = native.lib()
    st = C.c_int(0)
    h = L.orbfe_vocabulary_create(10, 6, 0, 0, len(parent), native.ptr(parent), native.ptr(word),
                                  native.ptr(desc), native.ptr(weight), 0, C.byref(st))
    assert h, st.value
    gv = native.Vocabulary.__new__(native.Vocabulary)
    gv._h = C.c_void_p(h)
    gv.set_stream(torch.cuda.current_stream(DEV).cuda_stream)
    B, cap = 256, 1100
    fr = [S.extract_frame(s, 1000, ini=20) for s in range(8)]
    dd = np.zeros((B, cap, 32), np.uint8)
    nn = np.zeros(B, np.int32)
    for i in range(B):
        x = fr[i % 8]
        dd[i, :x.n] = x.desc
        nn[i] = x.n
    D, N = torch.from_numpy(dd).to(DEV), torch.from_numpy(nn).to(DEV)
    o = [torch.empty((B, cap), dtype=t, device=DEV) for t in (torch.int32, torch.float64, torch.int32)]
    off = torch.empty((B, cap + 1), dtype=torch.int32, device=DEV)
    feat = torch.empty((B, cap), dtype=torch.int32, device=DEV)
    cnt = [torch.empty(B, dtype=torch.int32, device=DEV) for _ in range(2)]

    def go():
        gv.transform_batch_device(B, D.data_ptr(), N.data_ptr(), cap, 4, o[0].data_ptr(),
                                  o[1].data_ptr(), cnt[0].data_ptr(), o[2].data_ptr(),
                                  off.data_ptr(), feat.data_ptr(), cnt[1].data_ptr())
    t = timed(go, 10)
    path = os.path.join(tmpdir, "voc6.txt")  # the oracle reads the text format
    with open(path, "w") as fh:
        fh.write("10 6 0 0\n")
        for i in range(1, len(parent)):
            fh.write(f"{parent[i]} {int(word[i])} " + " ".join(map(str, desc[i].tolist())) +
                     f" {float(weight[i])!r}\n")
    ov = oracle.Vocabulary(path)
    assert ov.words == int(word.sum()) and len(ov.transform(fr[0].desc, 4)[0]) > 100
    tc = cpu_timed(lambda: ov.transform(fr[0].desc, 4))
    # per descriptor: k=10 children x 6 levels x 32 B of node descriptors + its own 32 B;
    # per kept feature ~24 B of BowVector / FeatureVector output
    nb = B * 1000 * (60 * 32 + 32 + 24)
    emit("(f)4 BoW transform, ComputeBoW (k=10 L=6 1.1M-node vocabulary, 1000 desc)",
         "frames/s", B, t, tc, nb, "device batch of 256 frames; synthetic vocabulary of ORBvoc's "
         "shape (ORBvoc.txt absent)", cpu_units=1)
    # the per-keyframe call (Frame::ComputeBoW) through the host ABI
    t1 = timed(lambda: gv.transform(fr[0].desc, 4), 100)
    emit("(f)4 BoW transform, ComputeBoW of one frame (host ABI, 1000 desc, same vocabulary)",
         "frames/s", 1, t1, tc, nb // B, "host ABI: descriptors in and vectors out through one "
         "device-mapped pinned block, one synchronisation")
    kf, f = fr[0], S.extract_frame(0, 1000, shift=(2, -3), ini=20)
    kf_fv = ov.transform(kf.desc, 4)[2:]
    f_fv = ov.transform(f.desc, 4)[2:]
    ok = np.ones(kf.n, np.uint8)
    m = native.ORBmatcher(0.75, True, device=0)
    t = timed(lambda: m.SearchByBoW(kf.desc, kf.keys["angle"], ok, kf_fv, f.desc, f.keys["angle"], f_fv), 50)
    tc = cpu_timed(lambda: oracle.search_by_bow(kf.desc, kf.keys["angle"], ok, kf_fv, f.desc,
                                                f.keys["angle"], f_fv, 0.75, True))
    emit("(f)4 SearchByBoW(KeyFrame*, Frame&) (1000 x 1000 features, level-2 nodes)", "calls/s",
         1, t, tc, (kf.n + f.n) * (32 + 8), "host ABI (uploads included), latency-bound: one "
         "workgroup per common node, the host waits on the output slots")
    # Tracking::Relocalization's candidate loop (Tracking.cc:1636-1656) as one device call:
    # the current frame against P candidate keyframes, everything resident in HBM
    from test_bow import pack_slots
    P, kcap = 64, 1100
    kfr = [S.extract_frame(s, 1000, shift=(s % 5, -(s % 3)), ini=20) for s in range(8)]
    rng = np.random.Generator(np.random.PCG64(1))
    items = [(x.desc, x.keys["angle"], (rng.uniform(size=x.n) < 0.8).astype(np.uint8),
              ov.transform(x.desc, 4)[2:]) for x in kfr]
    K = [torch.from_numpy(x).to(DEV) for x in pack_slots(items, kcap)]
    F = [torch.from_numpy(x).to(DEV) for x in pack_slots([(f.desc, f.keys["angle"],
                                                           np.ones(f.n, np.uint8), f_fv)], kcap)]
    pk = torch.arange(P, dtype=torch.int32, device=DEV) % len(items)
    pf = torch.zeros(P, dtype=torch.int32, device=DEV)
    out = torch.empty((P, kcap), dtype=torch.int32, device=DEV)
    nmv = torch.empty(P, dtype=torch.int32, device=DEV)
    stv = torch.empty(1, dtype=torch.int32, device=DEV)
    m = native.ORBmatcher(0.75, True, device=0)
    m.set_stream(torch.cuda.current_stream(DEV).cuda_stream)

    def gob():
        m.search_by_bow_batch_device(P, pk.data_ptr(), pf.data_ptr(), kcap, K[0].data_ptr(),
                                     K[1].data_ptr(), K[2].data_ptr(), K[3].data_ptr(),
                                     K[4].data_ptr(), K[5].data_ptr(), K[6].data_ptr(), kcap,
                                     F[0].data_ptr(), F[1].data_ptr(), F[3].data_ptr(),
                                     F[4].data_ptr(), F[5].data_ptr(), F[6].data_ptr(),
                                     out.data_ptr(), nmv.data_ptr(), stv.data_ptr())
    t = timed(gob, 50)
    assert int(stv[0]) == 0
    x = items[1]
    tc = cpu_timed(lambda: oracle.search_by_bow(x[0], x[1], x[2], x[3], f.desc, f.keys["angle"],
                                                f_fv, 0.75, True))
    emit(f"(f)4 SearchByBoW, relocalisation candidate loop (frame vs {P} keyframes, 1000 features)",
         "pairs/s", P, t, tc, P * (kf.n + f.n) * (32 + 8),
         "device batch: one call per relocalisation attempt (Tracking.cc:1636-1656), FeatureVectors "
         "resident; 2 launches (init; search with the orientation filter in each pair's last workgroup)", cpu_units=1)
    m.close()


if __name__ == "__main__":
    import tempfile
    with tempfile.TemporaryDirectory() as td:
        rows = {"single": row_single, "color": row_color, "stereo": row_stereo, "reloc": row_reloc, "track": row_track,
                "distinctive": row_distinctive, "bow": lambda: row_bow(td)}
        for name in (sys.argv[1:] or list(rows)):
            rows[name]()
