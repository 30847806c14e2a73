"""§8(f) row 2 — stereo matching, Frame::ComputeStereoMatches (Frame.cc:584-756).

CPU: the C oracle (oracle_compute_stereo_matches) against an independent pure-Python/numpy
restatement written from the same reference lines, on seeded rectified pairs.  GPU: the HIP
kernels (stereo_rows / stereo_match / stereo_filter) through the C ABI, bit-exact
(mvuRight / mvDepth float bits) against the oracle, host and batched-device forms.
Parity of the whole row is "unpinned" in the DESIGN.md sense: the reference holds no stereo
fixtures; the oracle is pinned by the restatement here.
"""
import math

import numpy as np
import pytest

import oracle
from orbslam_mapsave_amd.synth import synthetic_stereo_pair

F32 = np.float32
BF, B = 50.0, 0.1  # mbf = fx * baseline (fx 500, 10 cm), mb = mbf / fx


def popcount_rows(a, b):
    return np.unpackbits(a ^ b, axis=-1).sum(-1)


def restated(p, im_l, im_r, kl, dl, kr, dr, bf, b):
    """Frame::ComputeStereoMatches restated line by line (float32 scalars, python ints)."""
    scale = oracle.tables(p)["scale"]
    inv = oracle.tables(p)["inv_scale"]
    pl, pr = oracle.pyramid(p, im_l), oracle.pyramid(p, im_r)
    nl, nr = len(kl), len(kr)
    ur_out = np.full(nl, -1, F32)
    dp_out = np.full(nl, -1, F32)
    rows = [[] for _ in range(im_l.shape[0])]
    for ir in range(nr):
        y = F32(kr["y"][ir])
        r = F32(2.0) * scale[kr["octave"][ir]]
        for yi in range(math.floor(y - r), math.ceil(y + r) + 1):
            rows[yi].append(ir)
    min_d = F32(-3)
    max_d = F32(bf) / F32(b)
    acc = []
    for il in range(nl):
        lvl = int(kl["octave"][il])
        vl, ul = F32(kl["y"][il]), F32(kl["x"][il])
        cand = rows[int(vl)]
        if not cand:
            continue
        min_u, max_u = ul - max_d, ul - min_d
        if max_u < 0:
            continue
        best, best_ir = 100, 0
        for ir in cand:
            if kr["octave"][ir] < lvl - 1 or kr["octave"][ir] > lvl + 1:
                continue
            u = F32(kr["x"][ir])
            if min_u <= u <= max_u:
                d = int(popcount_rows(dl[il], dr[ir]))
                if d < best:
                    best, best_ir = d, ir
        if best >= 100:
            continue
        sf = inv[lvl]
        rnd = lambda v: F32(math.floor(abs(float(v)) + 0.5) * (1 if v >= 0 else -1))  # round()
        sul, svl, sur0 = rnd(F32(kl["x"][il]) * sf), rnd(F32(kl["y"][il]) * sf), rnd(F32(kr["x"][best_ir]) * sf)
        PL, PR = pl[lvl].astype(np.int64), pr[lvl].astype(np.int64)
        r0, c0 = int(svl) - 5, int(sul) - 5
        if sur0 < 0 or sur0 + 11 >= PR.shape[1]:
            continue
        IL = PL[r0:r0 + 11, c0:c0 + 11]
        IL = IL - IL[5, 5]
        dists = []
        for inc in range(-5, 6):
            cc = int(sur0) + inc - 5
            IR = PR[r0:r0 + 11, cc:cc + 11]
            dists.append(int(np.abs(IL - (IR - IR[5, 5])).sum()))
        bi = int(np.argmin(dists)) - 5  # first minimum
        if bi in (-5, 5):
            continue
        d1, d2, d3 = (F32(dists[5 + bi + k]) for k in (-1, 0, 1))
        delta = (d1 - d3) / (F32(2.0) * (d1 + d3 - F32(2.0) * d2))
        if delta < -1 or delta > 1:
            continue
        bur = scale[lvl] * ((sur0 + F32(bi)) + delta)
        disp = ul - bur
        if disp >= 0 and disp < max_d:
            if disp <= 0:
                disp = F32(0.01)
                bur = F32(float(ul) - 0.01)
            dp_out[il] = F32(bf) / disp
            ur_out[il] = bur
            acc.append((dists[5 + bi], il))
    if acc:
        acc.sort()
        median = F32(acc[len(acc) // 2][0])
        th = (F32(1.5) * F32(1.4)) * median
        for s, il in acc:
            if not F32(s) < th:
                ur_out[il] = dp_out[il] = -1
    return ur_out, dp_out


def case(seed, w=640, h=480, nf=1000, ini=20):
    p = oracle.params(nf, 1.2, 8, ini, 7)
    L, R = synthetic_stereo_pair(seed, w, h)
    kl, dl = oracle.extract(p, L)
    kr, dr = oracle.extract(p, R)
    return p, L, R, kl, dl, kr, dr


@pytest.mark.parametrize("seed", range(3))
def test_oracle_vs_restatement(seed):
    p, L, R, kl, dl, kr, dr = case(seed)
    ur, dp = oracle.compute_stereo_matches(p, L, R, kl, dl, kr, dr, BF, B)
    rur, rdp = restated(p, L, R, kl, dl, kr, dr, BF, B)
    assert np.array_equal(ur.view(np.uint32), rur.view(np.uint32))
    assert np.array_equal(dp.view(np.uint32), rdp.view(np.uint32))
    ok = ur >= 0
    assert ok.sum() > 0.3 * len(kl)
    # geometry of the synthetic pair: disparity = ramp 4..40 px (+ <=3 px tilt)
    disp = kl["x"][ok] - ur[ok]
    assert np.median(np.abs(disp - (4 + 36 * kl["y"][ok] / 479 + 3 * kl["x"][ok] / 639))) < 1.0
    assert np.allclose(dp[ok], BF / disp, rtol=1e-6)


def test_oracle_no_right_keypoints():
    p, L, R, kl, dl, kr, dr = case(4)
    ur, dp = oracle.compute_stereo_matches(p, L, R, kl, dl, kr[:0], dr[:0], BF, B)
    assert (ur == -1).all() and (dp == -1).all()


# ---------------------------------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [(0, 640, 480, 1000, 20), (1, 640, 480, 1000, 32),
                                 (2, 752, 480, 1200, 20), (3, 1280, 720, 2000, 20)])
def test_gpu_stereo_bit_exact(cfg):
    from orbslam_mapsave_amd.native import ORBextractor
    seed, w, h, nf, ini = cfg
    p, L, R, okl, odl, okr, odr = case(seed, w, h, nf, ini)
    el = ORBextractor(nf, 1.2, 8, ini, 7, device=0, max_width=w, max_height=h)
    er = ORBextractor(nf, 1.2, 8, ini, 7, device=0, max_width=w, max_height=h)
    kl, dl = el(L)
    kr, dr = er(R)
    assert kl.tobytes() == okl.tobytes() and kr.tobytes() == okr.tobytes()
    ur, dp = el.ComputeStereoMatches(er, kl, dl, kr, dr, BF, B)
    our, odp = oracle.compute_stereo_matches(p, L, R, okl, odl, okr, odr, BF, B)
    assert (our >= 0).sum() > 0
    assert np.array_equal(ur.view(np.uint32), our.view(np.uint32)), (ur != our).sum()
    assert np.array_equal(dp.view(np.uint32), odp.view(np.uint32))
    # no right keypoints: nothing matches
    ur0, dp0 = el.ComputeStereoMatches(er, kl, dl, kr[:0], dr[:0], BF, B)
    assert (ur0 == -1).all() and (dp0 == -1).all()
    el.close()
    er.close()


@pytest.mark.gpu
def test_gpu_stereo_batch_device():
    import torch
    from orbslam_mapsave_amd.native import ORBextractor
    n, w, h = 4, 640, 480
    dev = torch.device("cuda", 0)
    pairs = [synthetic_stereo_pair(10 + f, w, h) for f in range(n)]
    Ls = torch.from_numpy(np.stack([a for a, _ in pairs])).to(dev)
    Rs = torch.from_numpy(np.stack([b for _, b in pairs])).to(dev)
    el = ORBextractor(1000, 1.2, 8, 20, 7, device=0, max_width=w, max_height=h, max_batch=n)
    er = ORBextractor(1000, 1.2, 8, 20, 7, device=0, max_width=w, max_height=h, max_batch=n)
    cap = el.capacity(w, h)
    out = {}
    for side, e, X in (("l", el, Ls), ("r", er, Rs)):
        k = torch.zeros((n, cap * 28), dtype=torch.uint8, device=dev)
        d = torch.zeros((n, cap, 32), dtype=torch.uint8, device=dev)
        c = torch.zeros(n, dtype=torch.int32, device=dev)
        e.extract_batch_device(X.data_ptr(), n, w, h, w, w * h, k.data_ptr(), cap, d.data_ptr(),
                               c.data_ptr())
        out[side] = (k, d, c)
    ur = torch.zeros((n, cap), dtype=torch.float32, device=dev)
    dp = torch.zeros((n, cap), dtype=torch.float32, device=dev)
    (kl, dl, nl), (kr, dr, nr) = out["l"], out["r"]
    el.compute_stereo_matches_device(er, n, kl.data_ptr(), dl.data_ptr(), nl.data_ptr(),
                                     kr.data_ptr(), dr.data_ptr(), nr.data_ptr(), cap, BF, B,
                                     ur.data_ptr(), dp.data_ptr())
    el.stereo_status()
    p = oracle.params(1000, 1.2, 8, 20, 7)
    nl_h = nl.cpu().numpy()
    for f in range(n):
        L, R = pairs[f]
        okl, odl = oracle.extract(p, L)
        okr, odr = oracle.extract(p, R)
        assert nl_h[f] == len(okl)
        our, odp = oracle.compute_stereo_matches(p, L, R, okl, odl, okr, odr, BF, B)
        g_ur = ur[f, :nl_h[f]].cpu().numpy()
        g_dp = dp[f, :nl_h[f]].cpu().numpy()
        assert np.array_equal(g_ur.view(np.uint32), our.view(np.uint32))
        assert np.array_equal(g_dp.view(np.uint32), odp.view(np.uint32))
    el.close()
    er.close()
