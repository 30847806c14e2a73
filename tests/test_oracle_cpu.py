"""CPU tests of the parity oracle (no GPU).

The reference ships no tests or golden vectors for this path and cannot be built here, so the
oracle is pinned by (a) the known-answer constants the reference holds (bit_pattern_31_,
TH_HIGH/TH_LOW/HISTO_LENGTH, the YAML parameters and the level-size table SURVEY.md §8 derived
independently), (b) independent numpy / pure-Python restatements of every primitive written
straight from the definitions and of the oct-tree's list semantics
(ORBextractor.cc:538-762), and (c) regression fixtures in tests/golden (make_golden.py).
"""
import math
import os

import numpy as np
import pytest

import oracle
import scenarios as S
from orbslam_mapsave_amd.abi import KEYPOINT_DTYPE
from orbslam_mapsave_amd.synth import synthetic_frame, synthetic_mask

GOLD = os.path.join(os.path.dirname(__file__), "golden")
P = oracle.params(1000, 1.2, 8, 32, 7)


@pytest.fixture(autouse=True)
def _scalar_reading():
    """The restatements below follow OpenCV's portable scalar formulas, and the golden fixtures
    were made in that reading (make_golden.py): the module runs the oracle in it (its default is
    the x86 build's reading, tested against the GPU in test_gpu_x86_arith / the GPU suite)."""
    with oracle.variant(oracle.VAR_SCALAR):
        yield


# ---- (a) known answers ------------------------------------------------------------------
def test_tables_match_survey():
    t = oracle.tables(P)
    assert t["nfeat"].tolist() == [217, 181, 151, 126, 105, 87, 73, 60]
    assert t["umax"].tolist() == [15, 15, 15, 15, 14, 14, 14, 13, 13, 12, 11, 10, 9, 8, 6, 3]
    np.testing.assert_allclose(t["scale"], 1.2 ** np.arange(8), rtol=1e-6)
    t2 = oracle.tables(oracle.params(2000, 1.2, 8, 20, 7))
    assert t2["nfeat"].tolist() == [434, 362, 302, 251, 209, 175, 145, 122]


def test_level_sizes_match_survey():
    lw, lh = oracle.level_sizes(P, 640, 480)
    assert list(zip(lw, lh)) == [(640, 480), (533, 400), (444, 333), (370, 278), (309, 231),
                                 (257, 193), (214, 161), (179, 134)]
    assert int((lw.astype(int) * lh).sum()) == 950532
    lw, lh = oracle.level_sizes(P, 1920, 1080)
    assert int((lw.astype(int) * lh).sum()) == 6419321


def test_pattern_constants():
    path = os.path.join(os.path.dirname(__file__), "..", "include", "orbfe_pattern.inc")
    txt = open(path).read().split("*/", 1)[1]
    v = np.array([int(x) for x in txt.replace(",", " ").split()])
    assert len(v) == 1024 and v.sum() == -406 and np.abs(v).sum() == 6854
    assert v[:4].tolist() == [8, -3, 9, 5] and v[-4:].tolist() == [-1, -6, 0, -11]


def test_pattern_matches_reference_fixture():
    """include/orbfe_pattern.inc (compiled into the kernels and the oracle) equals the
    reference's bit_pattern_31_ (ORBextractor.cc:149-407) value for value, as read from the
    reference text by tests/golden/make_pattern_fixture.py."""
    import json
    d = os.path.dirname(__file__)
    fx = json.load(open(os.path.join(d, "golden", "pattern_fixture.json")))
    txt = open(os.path.join(d, "..", "include", "orbfe_pattern.inc")).read().split("*/", 1)[1]
    v = [int(x) for x in txt.replace(",", " ").split()]
    assert fx["count"] == 1024 and v == fx["values"]


def test_fast_atan2_known_answers():
    y = np.array([0, 1, 0, -1, 1, -1, 3, 0], np.float32)
    x = np.array([1, 0, -1, 0, 1, -1, -4, 0], np.float32)
    a = oracle.fast_atan2(y, x)
    assert a[0] == 0 and a[1] == 90 and a[2] == 180 and a[3] == 270 and a[7] == 0
    ref = np.degrees(np.arctan2(y.astype(np.float64), x)) % 360
    assert np.all(np.abs(a - ref)[:7] < 0.02)  # OpenCV: ~0.01 degree polynomial accuracy
    rng = np.random.default_rng(0)
    yy, xx = rng.integers(-200000, 200000, (2, 20000)).astype(np.float32)
    d = np.abs(oracle.fast_atan2(yy, xx) - np.degrees(np.arctan2(yy, xx)) % 360)
    assert np.minimum(d, 360 - d).max() < 0.02


def test_hamming_vs_popcount():
    rng = np.random.default_rng(1)
    a, b = rng.integers(0, 256, (2, 3000, 32), dtype=np.uint8)
    exp = np.unpackbits(a ^ b, axis=1).sum(1)
    assert np.array_equal(oracle.hamming(a, b), exp)


def test_bf_match_first_wins():
    rng = np.random.default_rng(2)
    base = rng.integers(0, 256, (3, 32), dtype=np.uint8)
    r = base[[0, 1, 1, 2, 0]]
    bi, bd, sd = oracle.bf_match(base, r)
    assert bi.tolist() == [0, 1, 3] and bd.tolist() == [0, 0, 0]  # first occurrence wins
    assert sd.tolist()[0] == 0 and sd.tolist()[1] == 0 and sd[2] > 0  # duplicates: second == best
    bi, bd, sd = oracle.bf_match(base[:1], np.zeros((0, 32), np.uint8))
    assert bi.tolist() == [-1] and bd.tolist() == [256] and sd.tolist() == [256]


# ---- (b) independent restatements -------------------------------------------------------
CIRCLE = [(0, 3), (1, 3), (2, 2), (3, 1), (3, 0), (3, -1), (2, -2), (1, -3), (0, -3), (-1, -3),
          (-2, -2), (-3, -1), (-3, 0), (-3, 1), (-2, 2), (-1, 3)]


def _corner(vals, v, t):
    dark = [x < v - t for x in vals]
    bright = [x > v + t for x in vals]
    for flags in (dark, bright):
        run = 0
        for f in flags + flags[:9]:
            run = run + 1 if f else 0
            if run >= 9:
                return True
    return False


def py_fast(roi, t):
    """cv::FAST TYPE_9_16 with nonmax from its definition: segment test, score = the largest
    threshold that keeps the pixel a corner, strict 3x3 maximum (zero outside)."""
    R, C = roi.shape
    r = roi.astype(int)
    score = np.zeros((R, C), int)
    for y in range(3, R - 3):
        for x in range(3, C - 3):
            vals = [r[y + dy, x + dx] for dx, dy in CIRCLE]
            if _corner(vals, r[y, x], t):
                s = t
                while s + 1 <= 255 and _corner(vals, r[y, x], s + 1):
                    s += 1
                score[y, x] = s
    out = []
    for y in range(3, R - 3):
        for x in range(3, C - 3):
            s = score[y, x]
            if s and all(s > score[y + dy, x + dx] for dy in (-1, 0, 1) for dx in (-1, 0, 1)
                         if dy or dx):
                out.append((x, y, s))
            elif s == 0 and _corner([r[y + dy, x + dx] for dx, dy in CIRCLE], r[y, x], t):
                pass  # a zero score never beats its neighbours
    return out


@pytest.mark.parametrize("y0,x0,t", [(200, 200, 32), (200, 200, 7), (100, 400, 20), (300, 60, 7)])
def test_fast_vs_definition(y0, x0, t):
    lev = oracle.pyramid(P, synthetic_frame(0))[0]
    roi = np.ascontiguousarray(lev[y0:y0 + 38, x0:x0 + 37])
    got = [(int(k["x"]), int(k["y"]), int(k["response"])) for k in oracle.fast(roi, t)]
    assert got == py_fast(roi, t)


def np_resize(src, dw, dh):
    """cv::resize INTER_LINEAR 8U, scalar fixed-point path."""
    sh, sw = src.shape
    sx_ = 1.0 / (dw / sw)
    sy_ = 1.0 / (dh / sh)

    def coefs(n, s, lim):
        f = ((np.arange(n) + 0.5) * s - 0.5).astype(np.float32)
        i = np.floor(f).astype(np.int64)
        f = (f - i.astype(np.float32)).astype(np.float32)
        return i, f

    xi, fx = coefs(dw, sx_, sw)
    lo = xi < 0
    fx[lo], xi[lo] = 0, 0
    hi = xi >= sw - 1
    fx[hi], xi[hi] = 0, sw - 1
    a0 = np.rint((np.float32(1) - fx) * np.float32(2048)).astype(np.int64)
    a1 = np.rint(fx * np.float32(2048)).astype(np.int64)
    yi, fy = coefs(dh, sy_, sh)
    b0 = np.rint((np.float32(1) - fy) * np.float32(2048)).astype(np.int64)
    b1 = np.rint(fy * np.float32(2048)).astype(np.int64)
    s = src.astype(np.int64)
    x1 = np.minimum(xi + 1, sw - 1)
    T = s[:, xi] * a0 + s[:, x1] * a1
    r0 = np.clip(yi, 0, sh - 1)
    r1 = np.clip(yi + 1, 0, sh - 1)
    v = (T[r0] * b0[:, None] + T[r1] * b1[:, None] + (1 << 21)) >> 22
    return np.clip(v, 0, 255).astype(np.uint8)


@pytest.mark.parametrize("shape,dst", [((480, 640), (533, 400)), ((400, 533), (444, 333)),
                                       ((37, 29), (24, 19)), ((1080, 1920), (1600, 900))])
def test_resize_vs_definition(shape, dst):
    rng = np.random.default_rng(sum(shape))
    src = rng.integers(0, 256, shape, dtype=np.uint8)
    assert np.array_equal(oracle.resize_linear(src, *dst), np_resize(src, *dst))


def np_blur(src):
    """GaussianBlur 7x7 sigma 2 REFLECT_101, 8U integer smooth path (App. A.2)."""
    g = np.exp(-((np.arange(7) - 3.0) ** 2) / 8).astype(np.float32)
    s = float(np.sum(g.astype(np.float64)))
    g = (g.astype(np.float64) * (1.0 / s)).astype(np.float32)
    k = np.rint(g * np.float32(256)).astype(np.int64)
    assert k.tolist() == [18, 34, 49, 55, 49, 34, 18]  # sums to 257, as OpenCV's 8U path does
    p = np.pad(src.astype(np.int64), 3, mode="reflect")  # numpy 'reflect' == REFLECT_101
    rows = sum(k[i] * p[:, i:i + src.shape[1]] for i in range(7))
    acc = sum(k[j] * rows[j:j + src.shape[0]] for j in range(7))
    return np.clip((acc + (1 << 15)) >> 16, 0, 255).astype(np.uint8)


@pytest.mark.parametrize("shape", [(134, 179), (480, 640), (7, 9)])
def test_blur_vs_definition(shape):
    rng = np.random.default_rng(shape[0])
    src = rng.integers(0, 256, shape, dtype=np.uint8)
    assert np.array_equal(oracle.gaussian_blur(src), np_blur(src))
    flat = np.full(shape, 255, np.uint8)  # 257/256 gain saturates white
    assert np.array_equal(oracle.gaussian_blur(flat), flat)


def py_distribute(keys, min_x, max_x, min_y, max_y, N):
    """DistributeOctTree (538-762) restated over a Python list; H2: phase-2 ties between
    equal-size nodes go to the higher creation sequence."""
    seq = [0]

    def node(ul, ur, bl, br, ks):
        seq[0] += 1
        return {"ul": ul, "ur": ur, "bl": bl, "br": br, "k": ks, "no": len(ks) == 1, "s": seq[0]}

    def divide(n):
        hx = math.ceil((n["ur"][0] - n["ul"][0]) / 2)
        hy = math.ceil((n["br"][1] - n["ul"][1]) / 2)
        ul = n["ul"]
        c1 = ((ul[0], ul[1]), (ul[0] + hx, ul[1]), (ul[0], ul[1] + hy), (ul[0] + hx, ul[1] + hy))
        c2 = (c1[1], n["ur"], c1[3], (n["ur"][0], ul[1] + hy))
        c3 = (c1[2], c1[3], n["bl"], (c1[3][0], n["bl"][1]))
        c4 = (c3[1], c2[3], c3[3], n["br"])
        parts = [[], [], [], []]
        for k in n["k"]:
            if k[0] < c1[1][0]:
                parts[0 if k[1] < c1[3][1] else 2].append(k)
            else:
                parts[1 if k[1] < c1[3][1] else 3].append(k)
        return [(c, p) for c, p in zip((c1, c2, c3, c4), parts)]

    n_ini = int(np.round(np.float32(max_x - min_x) / np.float32(max_y - min_y)))
    hX = np.float32(max_x - min_x) / np.float32(n_ini)
    L = []
    for i in range(n_ini):
        x0, x1 = int(hX * np.float32(i)), int(hX * np.float32(i + 1))
        L.append(node((x0, 0), (x1, 0), (x0, max_y - min_y), (x1, max_y - min_y), []))
        L[-1]["no"] = False
    for k in keys:
        L[min(int(np.float32(k[0]) / hX), n_ini - 1)]["k"].append(k)
    L = [n for n in L if n["k"]]
    for n in L:
        n["no"] = len(n["k"]) == 1
    while True:
        prev = len(L)
        front, keep, expand = [], [], []
        for n in L:
            if n["no"]:
                keep.append(n)
                continue
            for c, ks in divide(n):
                if ks:
                    ch = node(*c, ks)
                    front.insert(0, ch)
                    if len(ks) > 1:
                        expand.append(ch)
        L = front + keep
        if len(L) >= N or len(L) == prev:
            break
        if len(L) + 3 * len(expand) > N:
            done = False
            while not done:
                prev2 = len(L)
                order = sorted(expand, key=lambda n: (len(n["k"]), n["s"]))
                expand = []
                for n in reversed(order):
                    L.remove(n)
                    for c, ks in divide(n):
                        if ks:
                            ch = node(*c, ks)
                            L.insert(0, ch)
                            if len(ks) > 1:
                                expand.append(ch)
                    if len(L) >= N:
                        break
                if len(L) >= N or len(L) == prev2:
                    done = True
            break
    out = []
    for n in L:
        best = n["k"][0]
        for k in n["k"][1:]:
            if k[2] > best[2]:
                best = k
        out.append(best)
    return out


@pytest.mark.parametrize("level", range(8))
def test_distribute_vs_restatement(level):
    levels = oracle.pyramid(P, synthetic_frame(level))
    lev = levels[level]
    keys = oracle.fast_keys(P, lev)
    got = oracle.distribute(P, level, lev.shape[1], lev.shape[0], keys)
    kk = [(float(k["x"]), float(k["y"]), float(k["response"])) for k in keys]
    N = int(oracle.tables(P)["nfeat"][level])
    exp = py_distribute(kk, 16, lev.shape[1] - 16, 16, lev.shape[0] - 16, N)
    assert [(k["x"] - 16, k["y"] - 16, k["response"]) for k in got] == list(exp)


def test_distribute_phase2_ties():
    """Many equal-size nodes force the H2 tie rule in phase 2."""
    rng = np.random.default_rng(5)
    pts = set()
    while len(pts) < 300:
        cx, cy = rng.integers(0, 40, 2) * 15
        pts.add((int(cx + rng.integers(0, 2)), int(cy + rng.integers(0, 2))))
    keys = np.zeros(len(pts), KEYPOINT_DTYPE)
    for i, (x, y) in enumerate(sorted(pts)):
        keys[i] = (x, y, 7, -1, rng.integers(1, 4), 0, -1)
    for N in (50, 77, 130):
        p = oracle.params(N * 4, 1.2, 8, 20, 7)
        nf = int(oracle.tables(p)["nfeat"][0])
        got = oracle.distribute(p, 0, 632, 632, keys)
        kk = [(float(k["x"]), float(k["y"]), float(k["response"])) for k in keys]
        exp = py_distribute(kk, 16, 616, 16, 616, nf)
        assert [(k["x"] - 16, k["y"] - 16, k["response"]) for k in got] == list(exp)


def test_extract_edge_cases():
    kps, desc = oracle.extract(P, synthetic_frame(0, kind="constant"))
    assert len(kps) == 0 and desc.shape == (0, 32)
    kps, _ = oracle.extract(P, synthetic_frame(7, kind="low_contrast"))
    assert len(kps) > 0  # the minThFAST fallback finds corners
    img = synthetic_frame(3)
    m = np.zeros_like(img)
    kps, _ = oracle.extract(P, img, m)  # all-zero mask: black image
    assert len(kps) == 0


def test_extract_keypoint_invariants():
    kps, desc = oracle.extract(P, synthetic_frame(1))
    t = oracle.tables(P)
    assert np.all(np.diff(kps["octave"]) >= 0)  # level-major order (1079-1107)
    assert np.all(kps["class_id"] == -1)
    assert np.all(kps["size"] == np.floor(31 * t["scale"][kps["octave"]]))
    assert np.all((kps["angle"] >= 0) & (kps["angle"] < 360))
    counts = np.bincount(kps["octave"], minlength=8)
    assert np.all(counts <= t["nfeat"] + 3)


# ---- (c) golden regression pins ---------------------------------------------------------
def test_golden_extract():
    g = np.load(os.path.join(GOLD, "extract_golden.npz"))
    import hashlib
    sha = lambda a: hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()  # noqa
    for seed in range(5):
        img = synthetic_frame(seed)
        assert sha(img) == g[f"img_sha_{seed}"]
        levels = oracle.pyramid(P, img)
        assert [sha(l) for l in levels] == list(g[f"pyr_sha_{seed}"])
        kps, desc = oracle.extract(P, img)
        assert kps.tobytes() == g[f"kps_{seed}"].tobytes()
        assert np.array_equal(desc, g[f"desc_{seed}"])
        if seed == 0:
            assert np.array_equal(levels[7], g["level7_0"])
            assert np.array_equal(oracle.gaussian_blur(levels[7]), g["blur7_0"])
            assert oracle.fast_keys(P, levels[0]).tobytes() == g["fast_l0_0"].tobytes()
            assert oracle.fast_keys(P, levels[5]).tobytes() == g["fast_l5_0"].tobytes()
    kps, desc = oracle.extract(P, synthetic_frame(3), synthetic_mask(640, 480, 3))
    assert kps.tobytes() == g["kps_mask3"].tobytes()
    assert np.array_equal(desc, g["desc_mask3"])
    for name, pp in (("p1000", P), ("p2000", oracle.params(2000, 1.2, 8, 20, 7)),
                     ("rgbd", oracle.params(1000, 1.5, 4, 20, 7))):
        for k, v in oracle.tables(pp).items():
            assert np.array_equal(v, g[f"tab_{name}_{k}"])


@pytest.mark.slow
def test_golden_extract_1080():
    import hashlib
    g = np.load(os.path.join(GOLD, "extract_golden.npz"))
    kps, desc = oracle.extract(oracle.params(2000, 1.2, 8, 20, 7), synthetic_frame(0, 1920, 1080))
    assert len(kps) == int(g["n_1080"])
    assert hashlib.sha256(kps.tobytes()).hexdigest() == g["kps_1080_sha"]
    assert hashlib.sha256(desc.tobytes()).hexdigest() == g["desc_1080_sha"]


def test_golden_matchers():
    g = np.load(os.path.join(GOLD, "match_golden.npz"))
    f1, f2, prev = S.sfi_case(0)
    m12, nm, _ = oracle.search_for_initialization(f1, f2, prev, 100, 0.9, True)
    assert nm == int(g["sfi_nm"]) and np.array_equal(m12, g["sfi_m12"])
    assert nm == int((m12 >= 0).sum())
    f, mps, fmp, fobs, ids = S.sbp_local_case(0, 50000)
    r = oracle.search_by_projection_local(f, mps, 1.0, 0.8, fmp, fobs, ids)
    assert r[2] == int(g["sbpl_nm"]) and np.array_equal(r[0], g["sbpl_fmp"])
    c = S.sbp_last_case(0)
    args = (c["cur"], c["tcw_cur"], c["cam"], c["last_keys"], c["last_valid"],
            c["last_outlier"], c["last_xyz"], c["last_desc"], c["last_nobs"], c["tcw_last"])
    r = oracle.search_by_projection_last(*args, 15.0, True, True, last_ids=c["last_ids"])
    assert r[2] == int(g["sbpk_nm"]) and np.array_equal(r[0], g["sbpk_fmp"])
    fr = oracle.is_in_frustum(**S.frustum_case(0))
    assert np.array_equal(fr[0], g["fr_in"])
    assert np.array_equal(np.where(fr[0] == 1, fr[4], -99), g["fr_lvl"])


def test_fast_pretest_lerp_identity():
    """fast_kernel's byte-parallel pre-test: with v_lerp_u8 semantics per byte,
    lerp(a, b, r) = (a + b + (r & 1)) >> 1, the high bit of lerp(lerp(c, ~v, t & 1), M, 0) with
    M = 128 - ceil(t / 2) equals c > v + t, and lerp(lerp(v, ~c, t & 1), M, 0) equals c < v - t,
    for every byte c, v and threshold t."""
    c = np.arange(256)[:, None]
    v = np.arange(256)[None, :]
    for t in range(256):
        r, M = t & 1, 128 - ((t + 1) >> 1)
        bright = ((((c + (255 - v) + r) >> 1) + M) >> 1) >= 128
        dark = ((((v + (255 - c) + r) >> 1) + M) >> 1) >= 128
        assert np.array_equal(bright, c > v + t), t
        assert np.array_equal(dark, c < v - t), t


def test_fast_strip_dark_identity():
    """fast_strip_kernel's dark test without a per-byte NOT: lerp(v, ~c, r) = ~lerp(c, ~v, r ^ 1),
    so c < v - t equals NOT the high bit of lerp(lerp(c, ~v, (t & 1) ^ 1), 256 - M, 0) with
    M = 128 - ceil(t / 2), for every byte c, v and threshold t < 255 (t = 255 has no corners and
    is skipped by the kernel)."""
    c = np.arange(256)[:, None]
    v = np.arange(256)[None, :]
    for t in range(255):
        r, M = t & 1, 128 - ((t + 1) >> 1)
        y = (c + (255 - v) + (r ^ 1)) >> 1
        not_dark = ((y + (256 - M)) >> 1) >= 128
        assert np.array_equal(~not_dark, c < v - t), t
