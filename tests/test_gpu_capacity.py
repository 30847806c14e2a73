"""Capacity and workspace-reuse edges of the C ABI.

* Candidate overflow: the matchers fill their candidate CSR without a host round trip, bounded
  by a grow-only device buffer (64 per query for SearchForInitialization and the last-frame /
  keyframe SearchByProjection, 16 per map point for SearchLocalPoints).  When the true total
  is larger, the lists that end past the buffer are not filled and the resolution kernels must
  read them as empty (never past the buffer); the host then sees the total and reruns the call
  with the exact size.  Each case below is sized so that the FIRST call on a fresh matcher
  overflows (asserted through orbfe_matcher_capacity_retries) and must still be bit-exact.
* The single-frame HIP graph must not replay launches that captured buffers a later call of
  another size or batch reallocated.
* Keypoint capacity: a wide frame can return more than N + 4 keypoints per level (4 nIni from
  the first oct-tree pass); orbfe_keypoint_capacity_for covers it, and the device path refuses
  a smaller kps_cap before running anything (no frame is ever truncated).
"""
import numpy as np
import pytest

import oracle
import scenarios as S
from orbslam_mapsave_amd.synth import synthetic_frame, synthetic_local_map

pytestmark = pytest.mark.gpu


def fresh_matcher(nnratio=0.9, ori=True):
    from orbslam_mapsave_amd.native import ORBmatcher
    return ORBmatcher(nnratio, ori, device=0)


def test_sfi_first_call_overflows():
    f1, f2, prev = S.sfi_case(4)
    m = fresh_matcher(0.9, True)
    g12, gn, gprev = m.SearchForInitialization(f1, f2, prev, 400)
    e12, en, eprev = oracle.search_for_initialization(f1, f2, prev, 400, 0.9, True)
    assert m.capacity_retries() >= 1
    assert gn == en and np.array_equal(g12, e12) and np.array_equal(gprev, eprev)
    m.close()


def test_sbp_last_first_call_overflows():
    c = S.sbp_last_case(5)
    args = (c["cur"], c["tcw_cur"], c["cam"], c["last_keys"], c["last_valid"], c["last_outlier"],
            c["last_xyz"], c["last_desc"], c["last_nobs"], c["tcw_last"])
    m = fresh_matcher(0.9, True)
    g = m.SearchByProjectionLast(*args, 150.0, True, last_ids=c["last_ids"])
    e = oracle.search_by_projection_last(*args, 150.0, True, True, last_ids=c["last_ids"])
    assert m.capacity_retries() >= 1
    assert g[2] == e[2] and np.array_equal(g[0], e[0]) and np.array_equal(g[1], e[1])
    m.close()


def test_sbp_keyframe_first_call_overflows():
    c = S.sbp_keyframe_case(6)
    m = fresh_matcher(0.9, True)
    fmp, nm = m.SearchByProjectionKeyFrame(
        c["cur"], c["tcw_cur"], c["cam"], c["log_scale"], c["kf_angle"], c["kf_valid"],
        c["kf_bad"], c["found"], c["kf_xyz"], c["kf_desc"], c["kf_min"], c["kf_max"], 120, 100,
        frame_mp=c["frame_mp"], kf_ids=c["kf_ids"])
    ofmp, onm = oracle.search_by_projection_keyframe(c, 120, 100, True)
    assert m.capacity_retries() >= 1
    assert nm == onm and np.array_equal(fmp, ofmp)
    m.close()


def test_local_points_first_call_overflows():
    import torch
    from test_local_points import LOG_SCALE, oracle_search_local_points
    f = S.extract_frame(7, 1000)
    M, th = 3000, 30.0
    lm = synthetic_local_map(f.keys, f.desc, M, seed=7)
    cam = S.camera()
    inv, fmp, fobs, nm, nto = oracle_search_local_points(f, lm, cam, th)
    dev = torch.device("cuda", 0)
    T = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in lm.items()}
    d_keys = torch.from_numpy(f.keys.view(np.uint8).copy()).to(dev)
    d_desc = torch.from_numpy(f.desc).to(dev)
    d_inv = torch.zeros(M, dtype=torch.uint8, device=dev)
    m = fresh_matcher(0.8, False)
    torch.cuda.synchronize()
    gnm, gnto = m.search_local_points_device(
        f.n, d_keys.data_ptr(), d_desc.data_ptr(), None, S.W, S.H, f.scale_factors, lm["tcw"],
        cam, LOG_SCALE, 0.5, M, T["xyz"].data_ptr(), T["normal"].data_ptr(),
        T["min_dist"].data_ptr(), T["max_dist"].data_ptr(), T["desc"].data_ptr(),
        T["nobs"].data_ptr(), T["bad"].data_ptr(), T["skip"].data_ptr(), T["ids"].data_ptr(),
        0.8, th, T["frame_mp"].data_ptr(), T["frame_mp_obs"].data_ptr(), d_inv.data_ptr())
    assert m.capacity_retries() >= 1
    assert (gnm, gnto) == (nm, nto)
    assert np.array_equal(d_inv.cpu().numpy(), inv)
    assert np.array_equal(T["frame_mp"].cpu().numpy(), fmp)
    assert np.array_equal(T["frame_mp_obs"].cpu().numpy(), fobs)
    m.close()


def _check_single(ex, img, p):
    kps, desc = ex(img)
    okps, odesc = oracle.extract(p, img)
    assert kps.tobytes() == okps.tobytes()
    assert np.array_equal(desc, odesc)


def test_single_frame_graph_survives_reallocation():
    """single 640 (graph captured) -> masked 1280 batch (new plan, bigger workspaces) ->
    single 640 again: the replayed graph must not use freed or re-planned buffers."""
    from orbslam_mapsave_amd.native import ORBextractor
    p = oracle.params(1000, 1.2, 8, 32, 7)
    ex = ORBextractor(1000, 1.2, 8, 32, 7, device=0, max_width=640, max_height=480)
    a, b = synthetic_frame(11, 640, 480), synthetic_frame(12, 640, 480)
    _check_single(ex, a, p)
    _check_single(ex, b, p)  # graph replay
    big = np.stack([synthetic_frame(20 + i, 1280, 720) for i in range(3)])
    masks = np.ones_like(big)
    masks[:, 100:300, 200:500] = 0
    kps, desc, cnt = ex.extract_batch(big, masks)
    for i in range(3):
        okps, odesc = oracle.extract(p, big[i], masks[i])
        assert cnt[i] == len(okps)
        assert kps[i, :cnt[i]].tobytes() == okps.tobytes()
        assert np.array_equal(desc[i, :cnt[i]], odesc)
    _check_single(ex, a, p)  # re-captured against the current buffers
    _check_single(ex, b, p)
    ex.close()


def test_wide_frame_capacity():
    """3000 x 300 at 300 features: nIni = round(2968 / 268) = 11 at level 0, so the first
    oct-tree pass can leave up to 44 nodes on a level whose budget is far lower."""
    from orbslam_mapsave_amd.native import ORBextractor
    nf = 300
    p = oracle.params(nf, 1.2, 8, 20, 7)
    ex = ORBextractor(nf, 1.2, 8, 20, 7, device=0, max_width=3000, max_height=300)
    img = synthetic_frame(3, 3000, 300)
    cap = ex.capacity(3000, 300)
    assert cap <= ex.capacity()
    kps, desc = ex(img)
    okps, odesc = oracle.extract(p, img)
    assert len(kps) == len(okps) > nf + 4
    assert kps.tobytes() == okps.tobytes() and np.array_equal(desc, odesc)
    ex.close()


def test_device_path_refuses_short_capacity():
    """kps_cap below orbfe_keypoint_capacity_for: ORBFE_ERR_CAPACITY before any device work
    (a frame is never truncated); at exactly that capacity the outputs are bit-exact."""
    import torch
    from orbslam_mapsave_amd.abi import KEYPOINT_DTYPE, OrbfeError
    from orbslam_mapsave_amd.native import ORBextractor
    p = oracle.params(1000, 1.2, 8, 32, 7)
    W, H, n = 640, 480, 2
    imgs = np.stack([synthetic_frame(30 + i, W, H) for i in range(n)])
    dev = torch.device("cuda", 0)
    d_img = torch.from_numpy(imgs).to(dev)
    ex = ORBextractor(1000, 1.2, 8, 32, 7, device=0, max_width=W, max_height=H, max_batch=n)
    cap = ex.capacity(W, H)
    d_kps = torch.zeros((n, cap * 28), dtype=torch.uint8, device=dev)
    d_desc = torch.zeros((n, cap, 32), dtype=torch.uint8, device=dev)
    d_n = torch.full((n,), -5, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    with pytest.raises(OrbfeError) as e:
        ex.extract_batch_device(d_img.data_ptr(), n, W, H, W, W * H, d_kps.data_ptr(), cap - 1,
                                d_desc.data_ptr(), d_n.data_ptr())
    assert e.value.status == -2
    ex.synchronize()
    assert (d_n.cpu().numpy() == -5).all()  # nothing ran
    ex.extract_batch_device(d_img.data_ptr(), n, W, H, W, W * H, d_kps.data_ptr(), cap,
                            d_desc.data_ptr(), d_n.data_ptr())
    ex.synchronize()
    for i in range(n):
        okps, odesc = oracle.extract(p, imgs[i])
        c = int(d_n[i])
        assert c == len(okps)
        got = d_kps[i].cpu().numpy().view(KEYPOINT_DTYPE)[:c]
        assert got.tobytes() == okps.tobytes()
        assert np.array_equal(d_desc[i, :c].cpu().numpy(), odesc)
    ex.close()


def _chain_case(L, seed=3):
    """A contended local map whose greedy resolution needs L + 1 Jacobi rounds: L map points
    at the same projection all rank the same L keypoints in the same order (distances 2, 8, 14,
    ... from one descriptor; octaves alternate 1 / 2, so best and second never share a level and
    the ratio test never rejects), and each blocks what it takes (Observations() = 1), so point
    j ends on keypoint j only after round j.  Added to a real frame + a 300-point map."""
    from orbslam_mapsave_amd.abi import KEYPOINT_DTYPE, Frame
    f = S.extract_frame(seed, 1000)
    far = (np.abs(f.keys["x"] - 320) > 12) | (np.abs(f.keys["y"] - 240) > 12)
    rng = np.random.default_rng(seed)
    D = rng.integers(0, 256, 32, dtype=np.uint8)
    ck = np.zeros(L, KEYPOINT_DTYPE)
    ck["x"] = 320 + 0.05 * np.arange(L)
    ck["y"] = 240
    ck["size"] = 31
    ck["octave"] = 1 + np.arange(L) % 2
    ck["class_id"] = -1
    cd = np.unpackbits(np.tile(D, (L, 1)), axis=1)
    for j in range(L):
        cd[j, :2 + 6 * j] ^= 1
    keys = np.concatenate([f.keys[far], ck])
    desc = np.concatenate([f.desc[far], np.packbits(cd, axis=1)])
    fr = Frame(keys, desc, S.W, S.H, f.scale_factors)
    lm = synthetic_local_map(f.keys[far], f.desc[far], 300, seed=seed)  # none near the chain
    lm["frame_mp"] = np.concatenate([lm["frame_mp"], np.full(L, -1, np.int32)])
    lm["frame_mp_obs"] = np.concatenate([lm["frame_mp_obs"], np.zeros(L, np.int32)])
    z, s = 4.0, np.float64(np.float32(1.2))
    maxd = z * s ** 1.5  # PredictScale -> level 2
    add = dict(xyz=np.tile([0.0, 0.0, z], (L, 1)), normal=np.tile([0.0, 0.0, 1.0], (L, 1)),
               min_dist=np.full(L, maxd / s ** 7), max_dist=np.full(L, maxd),
               desc=np.tile(D, (L, 1)), nobs=np.ones(L), bad=np.zeros(L), skip=np.zeros(L),
               ids=np.arange(L) + 900_000)
    for k, v in add.items():
        lm[k] = np.concatenate([lm[k], v.astype(lm[k].dtype)])
    return fr, lm


@pytest.mark.parametrize("L", [4, 5, 6, 12])
def test_local_points_round_limit(L):
    """The fused SearchLocalPoints path runs 6 blind greedy rounds, the last merged into the
    accept kernel (round index 5).  A chain converging by round 5 (L <= 5; L = 5 is decided in
    the merged round itself) is returned from the fused path; a longer one (L >= 6: the map
    still changes in round 5) restores the slots and reruns on the CSR path — both bit-exact
    against the in-order oracle, and the fallback counted by orbfe_matcher_capacity_retries."""
    import torch
    from test_local_points import LOG_SCALE, oracle_search_local_points
    fr, lm = _chain_case(L)
    cam = S.camera()
    inv, fmp, fobs, nm, nto = oracle_search_local_points(fr, lm, cam, 1.0)
    M = len(lm["xyz"])
    # the chain resolved in order: chain point j holds chain keypoint j
    assert np.array_equal(fmp[-L:], lm["ids"][-L:])
    dev = torch.device("cuda", 0)
    T = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in lm.items()}
    d_keys = torch.from_numpy(fr.keys.view(np.uint8).copy()).to(dev)
    d_desc = torch.from_numpy(fr.desc).to(dev)
    d_inv = torch.zeros(M, dtype=torch.uint8, device=dev)
    m = fresh_matcher(0.8, False)
    torch.cuda.synchronize()
    gnm, gnto = m.search_local_points_device(
        fr.n, d_keys.data_ptr(), d_desc.data_ptr(), None, S.W, S.H, fr.scale_factors,
        lm["tcw"], cam, LOG_SCALE, 0.5, M, T["xyz"].data_ptr(), T["normal"].data_ptr(),
        T["min_dist"].data_ptr(), T["max_dist"].data_ptr(), T["desc"].data_ptr(),
        T["nobs"].data_ptr(), T["bad"].data_ptr(), T["skip"].data_ptr(), T["ids"].data_ptr(),
        0.8, 1.0, T["frame_mp"].data_ptr(), T["frame_mp_obs"].data_ptr(), d_inv.data_ptr())
    assert (gnm, gnto) == (nm, nto)
    assert np.array_equal(d_inv.cpu().numpy(), inv)
    assert np.array_equal(T["frame_mp"].cpu().numpy(), fmp)
    assert np.array_equal(T["frame_mp_obs"].cpu().numpy(), fobs)
    assert m.capacity_retries() == (1 if L >= 6 else 0)
    if L >= 6:
        assert m.last_rounds() >= L + 1
    m.close()
