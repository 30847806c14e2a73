"""TEST INFRASTRUCTURE ONLY — ctypes binding of the CPU parity oracle (oracle/orb_oracle.cpp).

Importable only from tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.  The
product package (orbslam_mapsave_amd) never imports this module.  PARITY UNPINNED: see
orb_oracle.h and DESIGN.md "Oracle".
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

from orbslam_mapsave_amd.abi import (KEYPOINT_DTYPE, ORBFE_OK, Camera, Frame, MapPoints,
                                     OrbfeError, Params, ptr)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "liborb_oracle.so")
_lib = None


def build(force: bool = False) -> str:
    if force or not os.path.exists(LIB_PATH):
        subprocess.run(["make", "-C", _HERE, "-s"], check=True)
    return LIB_PATH


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = C.CDLL(LIB_PATH)
    return _lib


def _check(fn: str, st: int) -> None:
    if st != ORBFE_OK:
        raise OrbfeError(fn, st)


# Build-dependent readings of the reference (orb_oracle.h, oracle/residuals.py): the default is
# the x86-64 build's (H4 FMA + H5 SSE2 + H6 SIMD), matched by the GPU's default arithmetic;
# VAR_SCALAR is OpenCV's portable reading (ORBFE_ARITH_SCALAR).
VAR_H2_ADDR, VAR_H4_COSF, VAR_H4_FMA, VAR_H5_SSE2, VAR_H6_SIMD = 1, 2, 4, 8, 16
VAR_SCALAR = 0                                    # OpenCV's portable scalar reading
VAR_X86 = VAR_H4_FMA | VAR_H5_SSE2 | VAR_H6_SIMD  # the reference's x86-64 build (the default)
DEFAULT_VARIANT = VAR_X86


def set_variant(flags: int) -> None:
    _check("oracle_set_variant", lib().oracle_set_variant(int(flags)))


class variant:
    """with oracle.variant(flags): ... — the oracle under another reading, restored on exit."""

    def __init__(self, flags: int):
        self.flags = flags

    def __enter__(self):
        self.prev = lib().oracle_get_variant()
        set_variant(self.flags)
        return self

    def __exit__(self, *exc):
        set_variant(self.prev)
        return False


def reference_constants() -> dict:
    """PATCH_SIZE, HALF_PATCH_SIZE, EDGE_THRESHOLD, TH_HIGH, TH_LOW, HISTO_LENGTH as the
    restatement uses them (oracle_reference_constants)."""
    out = (C.c_int32 * 6)()
    _check("oracle_reference_constants", lib().oracle_reference_constants(out))
    return dict(zip(CONSTANT_NAMES, list(out)))


CONSTANT_NAMES = ("PATCH_SIZE", "HALF_PATCH_SIZE", "EDGE_THRESHOLD", "TH_HIGH", "TH_LOW",
                  "HISTO_LENGTH")


def params(nfeatures=1000, scale_factor=1.2, nlevels=8, ini_th=20, min_th=7) -> Params:
    return Params(nfeatures, scale_factor, nlevels, ini_th, min_th)


def tables(p: Params):
    L = p.nlevels
    scale, inv, s2, is2 = (np.zeros(L, np.float32) for _ in range(4))
    nfeat = np.zeros(L, np.int32)
    umax = np.zeros(16, np.int32)
    _check("oracle_tables", lib().oracle_tables(C.byref(p), ptr(scale), ptr(inv), ptr(s2),
                                                ptr(is2), ptr(nfeat), ptr(umax)))
    return dict(scale=scale, inv_scale=inv, sigma2=s2, inv_sigma2=is2, nfeat=nfeat, umax=umax)


def level_sizes(p: Params, w: int, h: int):
    lw = np.zeros(p.nlevels, np.int32)
    lh = np.zeros(p.nlevels, np.int32)
    _check("oracle_level_sizes", lib().oracle_level_sizes(C.byref(p), w, h, ptr(lw), ptr(lh)))
    return lw, lh


def capacity(p: Params) -> int:
    return int(p.nfeatures) + 4 * int(p.nlevels) + 4096  # >= any oct-tree output (wide frames)


def cvt_gray(img: np.ndarray, pix: int) -> np.ndarray:
    """cvtColor(img, CV_*2GRAY) 8U (oracle_cvt_gray); pix as ORBFE_PIX_*."""
    img = np.ascontiguousarray(img, np.uint8)
    h, w, cn = img.shape
    out = np.zeros((h, w), np.uint8)
    _check("oracle_cvt_gray", lib().oracle_cvt_gray(ptr(img), pix, w, h, C.c_size_t(w * cn),
                                                    ptr(out)))
    return out


def compute_stereo_matches(p: Params, im_l: np.ndarray, im_r: np.ndarray, kl, dl, kr, dr,
                           bf: float, b: float):
    """Frame::ComputeStereoMatches (oracle_compute_stereo_matches) -> (mvuRight, mvDepth)."""
    im_l = np.ascontiguousarray(im_l, np.uint8)
    im_r = np.ascontiguousarray(im_r, np.uint8)
    h, w = im_l.shape
    kl = np.ascontiguousarray(kl, KEYPOINT_DTYPE)
    kr = np.ascontiguousarray(kr, KEYPOINT_DTYPE)
    dl = np.ascontiguousarray(dl, np.uint8)
    dr = np.ascontiguousarray(dr, np.uint8)
    ur = np.zeros(len(kl), np.float32)
    dp = np.zeros(len(kl), np.float32)
    _check("oracle_compute_stereo_matches", lib().oracle_compute_stereo_matches(
        C.byref(p), ptr(im_l), ptr(im_r), w, h, ptr(kl), ptr(dl), len(kl), ptr(kr), ptr(dr),
        len(kr), C.c_float(bf), C.c_float(b), ptr(ur), ptr(dp)))
    return ur, dp


def extract(p: Params, img: np.ndarray, mask: np.ndarray | None = None):
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    cap = capacity(p)
    kps = np.zeros(cap, KEYPOINT_DTYPE)
    desc = np.zeros((cap, 32), np.uint8)
    n = C.c_int(0)
    m = None if mask is None else np.ascontiguousarray(mask, np.uint8)
    _check("oracle_extract", lib().oracle_extract(
        C.byref(p), ptr(img), w, h, C.c_size_t(w), ptr(m), C.c_size_t(w), ptr(kps), cap,
        ptr(desc), C.byref(n)))
    return kps[:n.value].copy(), desc[:n.value].copy()


def extract_batch(p: Params, imgs: np.ndarray, nthreads: int = 1):
    imgs = np.ascontiguousarray(imgs, np.uint8)
    n, h, w = imgs.shape
    cap = capacity(p)
    kps = np.zeros((n, cap), KEYPOINT_DTYPE)
    desc = np.zeros((n, cap, 32), np.uint8)
    cnt = np.zeros(n, np.int32)
    _check("oracle_extract_batch", lib().oracle_extract_batch(
        C.byref(p), ptr(imgs), n, w, h, C.c_size_t(w * h), ptr(kps), cap, ptr(desc), ptr(cnt),
        nthreads))
    return kps, desc, cnt


def pyramid(p: Params, img: np.ndarray, mask: np.ndarray | None = None):
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    lw, lh = level_sizes(p, w, h)
    out = np.zeros(int((lw.astype(np.int64) * lh).sum()), np.uint8)
    m = None if mask is None else np.ascontiguousarray(mask, np.uint8)
    _check("oracle_pyramid", lib().oracle_pyramid(C.byref(p), ptr(img), w, h, C.c_size_t(w),
                                                  ptr(m), C.c_size_t(w), ptr(out)))
    levels, off = [], 0
    for a, b in zip(lw, lh):
        levels.append(out[off:off + a * b].reshape(b, a))
        off += a * b
    return levels


def resize_linear(src: np.ndarray, dw: int, dh: int) -> np.ndarray:
    src = np.ascontiguousarray(src, np.uint8)
    out = np.zeros((dh, dw), np.uint8)
    _check("oracle_resize_linear", lib().oracle_resize_linear(
        ptr(src), src.shape[1], src.shape[0], C.c_size_t(src.shape[1]), ptr(out), dw, dh,
        C.c_size_t(dw)))
    return out


def gaussian_blur(src: np.ndarray) -> np.ndarray:
    src = np.ascontiguousarray(src, np.uint8)
    out = np.zeros_like(src)
    _check("oracle_gaussian_blur", lib().oracle_gaussian_blur(
        ptr(src), src.shape[1], src.shape[0], C.c_size_t(src.shape[1]), ptr(out)))
    return out


def _keys_call(fn, cap, *args):
    out = np.zeros(cap, KEYPOINT_DTYPE)
    n = C.c_int(0)
    st = fn(*args, ptr(out), cap, C.byref(n))
    if st != ORBFE_OK and n.value > cap:
        return _keys_call(fn, n.value, *args)
    _check(fn.__name__, st)
    return out[:n.value].copy()


def fast(roi: np.ndarray, threshold: int):
    roi = np.ascontiguousarray(roi, np.uint8)
    return _keys_call(lib().oracle_fast, 4096, ptr(roi), roi.shape[0], roi.shape[1],
                      C.c_size_t(roi.shape[1]), threshold)


def fast_keys(p: Params, level: np.ndarray):
    level = np.ascontiguousarray(level, np.uint8)
    return _keys_call(lib().oracle_fast_keys, 65536, C.byref(p), ptr(level), level.shape[1],
                      level.shape[0], C.c_size_t(level.shape[1]))


def distribute(p: Params, level: int, lw: int, lh: int, keys: np.ndarray):
    keys = np.ascontiguousarray(keys, KEYPOINT_DTYPE)
    return _keys_call(lib().oracle_distribute, 8192, C.byref(p), level, lw, lh, ptr(keys),
                      len(keys))


def fast_atan2(y: np.ndarray, x: np.ndarray) -> np.ndarray:
    y = np.ascontiguousarray(y, np.float32)
    x = np.ascontiguousarray(x, np.float32)
    out = np.zeros_like(y)
    lib().oracle_fast_atan2(ptr(y), ptr(x), len(y), ptr(out))
    return out


def hamming(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    a = np.ascontiguousarray(a, np.uint8).reshape(-1, 32)
    b = np.ascontiguousarray(b, np.uint8).reshape(-1, 32)
    out = np.zeros(len(a), np.int32)
    _check("oracle_hamming", lib().oracle_hamming(ptr(a), ptr(b), len(a), ptr(out)))
    return out


def bf_match(q: np.ndarray, r: np.ndarray):
    q = np.ascontiguousarray(q, np.uint8).reshape(-1, 32)
    r = np.ascontiguousarray(r, np.uint8).reshape(-1, 32)
    bi, bd, sd = (np.zeros(len(q), np.int32) for _ in range(3))
    _check("oracle_bf_match", lib().oracle_bf_match(ptr(q), len(q), ptr(r), len(r), ptr(bi),
                                                    ptr(bd), ptr(sd)))
    return bi, bd, sd


def features_in_area(f: Frame, x: float, y: float, r: float, min_level=-1, max_level=-1):
    out = np.zeros(max(f.n, 1), np.int32)
    n = C.c_int(0)
    fv = f.view()
    _check("oracle_features_in_area", lib().oracle_features_in_area(
        C.byref(fv), C.c_float(x), C.c_float(y), C.c_float(r), min_level, max_level, ptr(out),
        len(out), C.byref(n)))
    return out[:n.value].copy()


def search_for_initialization(f1: Frame, f2: Frame, prev_matched: np.ndarray, window=100,
                              nnratio=0.9, check_ori=True):
    prev = np.ascontiguousarray(prev_matched, np.float32).reshape(-1, 2).copy()
    m12 = np.zeros(f1.n, np.int32)
    nm = C.c_int32(0)
    v1, v2 = f1.view(), f2.view()
    _check("oracle_search_for_initialization", lib().oracle_search_for_initialization(
        C.c_float(nnratio), int(check_ori), C.byref(v1), C.byref(v2), ptr(prev), window,
        ptr(m12), C.byref(nm)))
    return m12, nm.value, prev


def search_by_projection_local(f: Frame, mps: MapPoints, th=1.0, nnratio=0.8,
                               frame_mp=None, frame_mp_obs=None, mp_ids=None):
    fmp = (np.full(f.n, -1, np.int32) if frame_mp is None
           else np.ascontiguousarray(frame_mp, np.int32).copy())
    fobs = (np.zeros(f.n, np.int32) if frame_mp_obs is None
            else np.ascontiguousarray(frame_mp_obs, np.int32).copy())
    ids = None if mp_ids is None else np.ascontiguousarray(mp_ids, np.int32)
    nm = C.c_int32(0)
    fv, mv = f.view(), mps.view()
    _check("oracle_search_by_projection_local", lib().oracle_search_by_projection_local(
        C.c_float(nnratio), C.byref(fv), ptr(fmp), ptr(fobs), C.byref(mv), ptr(ids),
        C.c_float(th), C.byref(nm)))
    return fmp, fobs, nm.value


def search_by_projection_last(cur: Frame, tcw_cur, cam: Camera, last_keys, last_valid,
                              last_outlier, last_xyz, last_desc, last_nobs, tcw_last, th=15.0,
                              mono=True, check_ori=True, frame_mp=None, frame_mp_obs=None,
                              last_ids=None):
    fmp = (np.full(cur.n, -1, np.int32) if frame_mp is None
           else np.ascontiguousarray(frame_mp, np.int32).copy())
    fobs = (np.zeros(cur.n, np.int32) if frame_mp_obs is None
            else np.ascontiguousarray(frame_mp_obs, np.int32).copy())
    a = [np.ascontiguousarray(tcw_cur, np.float32).reshape(12),
         np.ascontiguousarray(last_keys, KEYPOINT_DTYPE),
         np.ascontiguousarray(last_valid, np.uint8), np.ascontiguousarray(last_outlier, np.uint8),
         np.ascontiguousarray(last_xyz, np.float32).reshape(-1, 3),
         np.ascontiguousarray(last_desc, np.uint8).reshape(-1, 32),
         np.ascontiguousarray(last_nobs, np.int32),
         np.ascontiguousarray(tcw_last, np.float32).reshape(12)]
    ids = None if last_ids is None else np.ascontiguousarray(last_ids, np.int32)
    nm = C.c_int32(0)
    cv = cur.view()
    _check("oracle_search_by_projection_last", lib().oracle_search_by_projection_last(
        int(check_ori), C.byref(cv), ptr(a[0]), C.byref(cam), ptr(fmp), ptr(fobs), len(a[1]),
        ptr(a[1]), ptr(a[2]), ptr(a[3]), ptr(a[4]), ptr(a[5]), ptr(a[6]), ptr(ids), ptr(a[7]),
        C.c_float(th), int(mono), C.byref(nm)))
    return fmp, fobs, nm.value


def _sbp_kf_args(c):
    return [np.ascontiguousarray(c["tcw_cur"], np.float32).reshape(12),
            np.ascontiguousarray(c["kf_angle"], np.float32),
            np.ascontiguousarray(c["kf_valid"], np.uint8),
            np.ascontiguousarray(c["kf_bad"], np.uint8),
            np.ascontiguousarray(c["found"], np.uint8),
            np.ascontiguousarray(c["kf_xyz"], np.float32).reshape(-1, 3),
            np.ascontiguousarray(c["kf_desc"], np.uint8).reshape(-1, 32),
            np.ascontiguousarray(c["kf_min"], np.float32),
            np.ascontiguousarray(c["kf_max"], np.float32),
            None if c.get("kf_ids") is None else np.ascontiguousarray(c["kf_ids"], np.int32)]


def search_by_projection_keyframe(c: dict, th=10.0, orb_dist=100, check_ori=True):
    """Relocalisation SearchByProjection(Frame&, KeyFrame*, ...) (ORBmatcher.cc:1475-1602);
    `c` holds the keys of tests/scenarios.sbp_keyframe_case.  Returns (frame_mp, nmatches)."""
    cur = c["cur"]
    fmp = np.ascontiguousarray(c["frame_mp"], np.int32).copy()
    a = _sbp_kf_args(c)
    nm = C.c_int32(0)
    cv = cur.view()
    _check("oracle_search_by_projection_keyframe", lib().oracle_search_by_projection_keyframe(
        int(check_ori), C.byref(cv), ptr(a[0]), C.byref(c["cam"]), C.c_float(c["log_scale"]),
        ptr(fmp), len(a[1]), *(ptr(x) for x in a[1:]), C.c_float(th), int(orb_dist),
        C.byref(nm)))
    return fmp, nm.value


def distinctive_descriptors(obs_off: np.ndarray, obs_desc: np.ndarray):
    """MapPoint::ComputeDistinctiveDescriptors over a CSR of observation descriptors."""
    off = np.ascontiguousarray(obs_off, np.int32)
    d = np.ascontiguousarray(obs_desc, np.uint8).reshape(-1, 32)
    n = len(off) - 1
    best = np.zeros(n, np.int32)
    out = np.zeros((n, 32), np.uint8)
    _check("oracle_distinctive_descriptors",
           lib().oracle_distinctive_descriptors(n, ptr(off), ptr(d), ptr(best), ptr(out)))
    return best, out


class Vocabulary:
    """DBoW2 text vocabulary loaded by the oracle (oracle_vocab_load_text)."""

    def __init__(self, path: str):
        L = lib()
        L.oracle_vocab_load_text.restype = C.c_void_p
        L.oracle_vocab_load_text.argtypes = [C.c_char_p, C.c_void_p]
        L.oracle_vocab_free.argtypes = [C.c_void_p]
        st = C.c_int(0)
        h = L.oracle_vocab_load_text(path.encode(), C.byref(st))
        if not h:
            raise OrbfeError("oracle_vocab_load_text", st.value)
        self._h = C.c_void_p(h)
        info = np.zeros(6, np.int32)
        _check("oracle_vocab_info", L.oracle_vocab_info(self._h, ptr(info)))
        self.k, self.L, self.scoring, self.weighting, self.nodes, self.words = map(int, info)

    def __del__(self):
        if getattr(self, "_h", None):
            lib().oracle_vocab_free(self._h)
            self._h = None

    def transform(self, desc: np.ndarray, levelsup: int = 4):
        """-> (word_ids, values, node_ids, node_off, feat): BowVector and FeatureVector."""
        d = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
        n = len(d)
        wid = np.zeros(max(n, 1), np.int32)
        val = np.zeros(max(n, 1), np.float64)
        nid = np.zeros(max(n, 1), np.int32)
        off = np.zeros(n + 2, np.int32)
        feat = np.zeros(max(n, 1), np.int32)
        nw, nn = C.c_int32(0), C.c_int32(0)
        _check("oracle_bow_transform", lib().oracle_bow_transform(
            self._h, ptr(d), n, levelsup, ptr(wid), ptr(val), C.byref(nw), ptr(nid), ptr(off),
            ptr(feat), C.byref(nn)))
        return (wid[:nw.value].copy(), val[:nw.value].copy(), nid[:nn.value].copy(),
                off[:nn.value + 1].copy(), feat[:off[nn.value]].copy())


def search_by_bow(kf_desc, kf_angle, kf_mp_ok, kf_fv, f_desc, f_angle, f_fv, nnratio=0.75,
                  check_ori=True):
    """ORBmatcher::SearchByBoW(KeyFrame*, Frame&, ...) -> (matches per frame feature, n)."""
    kd = np.ascontiguousarray(kf_desc, np.uint8).reshape(-1, 32)
    fd = np.ascontiguousarray(f_desc, np.uint8).reshape(-1, 32)
    ka = np.ascontiguousarray(kf_angle, np.float32)
    fa = np.ascontiguousarray(f_angle, np.float32)
    ok = np.ascontiguousarray(kf_mp_ok, np.uint8)
    kn, ko, kfe = (np.ascontiguousarray(x, np.int32) for x in kf_fv)
    fn, fo, ffe = (np.ascontiguousarray(x, np.int32) for x in f_fv)
    out = np.zeros(len(fd), np.int32)
    nm = C.c_int32(0)
    _check("oracle_search_by_bow", lib().oracle_search_by_bow(
        C.c_float(nnratio), int(check_ori), ptr(kd), ptr(ka), ptr(ok), ptr(kn), ptr(ko),
        ptr(kfe), len(kn), len(fd), ptr(fd), ptr(fa), ptr(fn), ptr(fo), ptr(ffe), len(fn),
        ptr(out), C.byref(nm)))
    return out, nm.value


def is_in_frustum(xyz, normal, min_dist, max_dist, tcw, cam: Camera, bounds, log_scale,
                  cos_limit=0.5):
    xyz = np.ascontiguousarray(xyz, np.float32).reshape(-1, 3)
    n = len(xyz)
    normal = np.ascontiguousarray(normal, np.float32).reshape(-1, 3)
    mn = np.ascontiguousarray(min_dist, np.float32)
    mx = np.ascontiguousarray(max_dist, np.float32)
    t = np.ascontiguousarray(tcw, np.float32).reshape(12)
    inv = np.zeros(n, np.uint8)
    px, py, pxr, vc = (np.zeros(n, np.float32) for _ in range(4))
    pl = np.zeros(n, np.int32)
    _check("oracle_is_in_frustum", lib().oracle_is_in_frustum(
        n, ptr(xyz), ptr(normal), ptr(mn), ptr(mx), ptr(t), C.byref(cam),
        *(C.c_float(b) for b in bounds), C.c_float(log_scale), C.c_float(cos_limit), ptr(inv),
        ptr(px), ptr(py), ptr(pxr), ptr(pl), ptr(vc)))
    return inv, px, py, pxr, pl, vc


__all__ = ["build", "lib", "params", "tables", "level_sizes", "extract", "extract_batch",
           "pyramid", "resize_linear", "gaussian_blur", "fast", "fast_keys", "distribute",
           "fast_atan2", "hamming", "bf_match", "features_in_area", "search_for_initialization",
           "search_by_projection_local", "search_by_projection_last", "is_in_frustum", "Frame",
           "MapPoints", "Camera"]
