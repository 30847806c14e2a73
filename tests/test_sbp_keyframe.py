"""§8(f) row 3 — relocalisation SearchByProjection(Frame&, KeyFrame*, sAlreadyFound, th,
ORBdist) (ORBmatcher.cc:1475-1602), called by Tracking::Relocalization with (10, 100) and
(3, 64) (Tracking.cc:1723, 1737).

CPU: the C oracle against an independent pure-Python restatement (greedy in map-point order,
assigned slots block, orientation histogram with ComputeThreeMaxima).  GPU: the HIP path
(sbp_kf_cand_kernel + the greedy wave resolve) bit-exact against the oracle: frame_mp and
nmatches.
"""
import math

import numpy as np
import pytest

import oracle
import scenarios as S

F32 = np.float32


def restated(c, th, orb_dist, check_ori=True):
    cur = c["cur"]
    k = cur.keys
    fmp = c["frame_mp"].copy()
    T = c["tcw_cur"].astype(F32)
    cam = c["cam"]
    scale = cur.scale_factors
    W, H = F32(cur.max_x), F32(cur.max_y)
    ow = [F32(-(float(T[0, i]) * float(T[0, 3]) + float(T[1, i]) * float(T[1, 3]) +
                float(T[2, i]) * float(T[2, 3]))) for i in range(3)]
    gw, gh = F32(cur.grid_w_inv), F32(cur.grid_h_inv)
    hist = [[] for _ in range(30)]
    nm = 0
    for i in range(len(c["kf_valid"])):
        if not c["kf_valid"][i] or c["kf_bad"][i] or c["found"][i]:
            continue
        P = c["kf_xyz"][i]
        pc = [((T[r, 0] * P[0] + T[r, 1] * P[1]) + T[r, 2] * P[2]) + T[r, 3] for r in range(3)]
        invz = F32(1.0 / float(pc[2]))
        u = F32(cam.fx) * pc[0] * invz + F32(cam.cx)
        v = F32(cam.fy) * pc[1] * invz + F32(cam.cy)
        if u < 0 or u > W or v < 0 or v > H:
            continue
        po = [P[j] - ow[j] for j in range(3)]
        d3 = F32(math.sqrt(sum(float(x) * float(x) for x in po)))
        if d3 < F32(0.8) * c["kf_min"][i] or d3 > F32(1.2) * c["kf_max"][i]:
            continue
        ratio = c["kf_max"][i] / d3
        lvl = int(math.ceil(F32(math.log(float(ratio))) / F32(c["log_scale"])))
        assert 0 <= lvl < 8
        r = F32(th) * scale[lvl]
        # GetFeaturesInArea(u, v, r, lvl-1, lvl+1) (Frame.cc:445-498): candidates come in grid
        # order -- cell column ix, then row iy, then insertion (keypoint index) order
        gx = np.floor(((k["x"] - F32(0)) * gw).astype(np.float64) + 0.5).astype(int)  # std::round
        gy = np.floor(((k["y"] - F32(0)) * gh).astype(np.float64) + 0.5).astype(int)
        cands = []
        for i2 in range(cur.n):
            if not (0 <= gx[i2] < 64 and 0 <= gy[i2] < 48):
                continue
            if k["octave"][i2] < lvl - 1 or k["octave"][i2] > lvl + 1:
                continue
            if not (abs(k["x"][i2] - u) < r and abs(k["y"][i2] - v) < r):
                continue
            cands.append((gx[i2], gy[i2], i2))
        best, bi = 256, -1
        for _, _, i2 in sorted(cands):
            if fmp[i2] >= 0:
                continue
            d = int(np.unpackbits(c["kf_desc"][i] ^ cur.desc[i2]).sum())
            if d < best:
                best, bi = d, i2
        if best <= orb_dist:
            fmp[bi] = c["kf_ids"][i]
            nm += 1
            if check_ori:
                rot = c["kf_angle"][i] - k["angle"][bi]
                if rot < 0.0:
                    rot += F32(360.0)
                b = math.floor(float(rot * (F32(1.0) / F32(30))) + 0.5)  # std::round, rot >= 0
                hist[0 if b == 30 else b].append(bi)
    if check_ori:
        sizes = [len(h) for h in hist]
        m1 = m2 = m3 = 0
        i1 = i2_ = i3 = -1
        for i, s in enumerate(sizes):
            if s > m1:
                m3, m2, m1, i3, i2_, i1 = m2, m1, s, i2_, i1, i
            elif s > m2:
                m3, m2, i3, i2_ = m2, s, i2_, i
            elif s > m3:
                m3, i3 = s, i
        if m2 < F32(0.1) * F32(m1):
            i2_ = i3 = -1
        elif m3 < F32(0.1) * F32(m1):
            i3 = -1
        for i in range(30):
            if i not in (i1, i2_, i3):
                for bi in hist[i]:
                    fmp[bi] = -1
                    nm -= 1
    return fmp, nm


@pytest.mark.parametrize("seed,th,od", [(0, 10, 100), (1, 3, 64), (2, 10, 100)])
def test_oracle_vs_restatement(seed, th, od):
    c = S.sbp_keyframe_case(seed)
    fmp, nm = oracle.search_by_projection_keyframe(c, th, od)
    rfmp, rnm = restated(c, th, od)
    assert nm == rnm and np.array_equal(fmp, rfmp)
    assert nm > 50


@pytest.mark.gpu
@pytest.mark.parametrize("seed,th,od,ori", [(0, 10, 100, True), (1, 3, 64, True),
                                            (2, 10, 100, False), (3, 3, 64, True),
                                            (4, 40, 100, True)])
def test_gpu_sbp_keyframe(seed, th, od, ori):
    """The host form: candidates in fixed slots (16 per map point, one kernel) and, when a point
    has more (th = 40), the rerun on the CSR path from the saved slots — both bit-exact."""
    from orbslam_mapsave_amd.native import ORBmatcher
    c = S.sbp_keyframe_case(seed)
    m = ORBmatcher(0.9, ori, device=0)
    fmp, nm = m.SearchByProjectionKeyFrame(
        c["cur"], c["tcw_cur"], c["cam"], c["log_scale"], c["kf_angle"], c["kf_valid"],
        c["kf_bad"], c["found"], c["kf_xyz"], c["kf_desc"], c["kf_min"], c["kf_max"], th, od,
        frame_mp=c["frame_mp"], kf_ids=c["kf_ids"])
    ofmp, onm = oracle.search_by_projection_keyframe(c, th, od, ori)
    assert nm == onm and np.array_equal(fmp, ofmp)
    if th >= 40:
        assert m.capacity_retries() >= 1  # the fixed slots overflowed
    m.close()
