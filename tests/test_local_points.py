"""Tracking::SearchLocalPoints on device-resident data (BASELINE config 5): isInFrustum over a
50k-point local map + SearchByProjection(F, vpLocalMapPoints, th), through
orbfe_search_local_points_device, bit-exact against the oracle's isInFrustum and
SearchByProjection composed the way Tracking.cc:1403-1455 composes them.
"""
import numpy as np
import pytest

import oracle
import scenarios as S
from orbslam_mapsave_amd.abi import MapPoints
from orbslam_mapsave_amd.synth import synthetic_local_map

LOG_SCALE = float(np.log(np.float32(1.2)).astype(np.float32))


def oracle_search_local_points(frame, lm, cam, th=1.0, nnratio=0.8):
    inv, px, py, pxr, pl, vc = oracle.is_in_frustum(
        lm["xyz"], lm["normal"], lm["min_dist"], lm["max_dist"], lm["tcw"], cam,
        (0.0, float(S.W), 0.0, float(S.H)), LOG_SCALE, 0.5)
    inv[(lm["skip"] > 0) | (lm["bad"] > 0)] = 0  # skipped points: mbTrackInView = false (1419)
    mps = MapPoints(px, py, pl, vc, lm["desc"], lm["nobs"], track_in_view=inv,
                    is_bad=lm["bad"], proj_xr=pxr)
    fmp, fobs, nm = oracle.search_by_projection_local(frame, mps, th, nnratio, lm["frame_mp"],
                                                      lm["frame_mp_obs"], lm["ids"])
    return inv, fmp, fobs, nm, int(inv.sum())


def test_local_map_generator_predicts_levels():
    f = S.extract_frame(0, 1000)
    lm = synthetic_local_map(f.keys, f.desc, 20000, seed=0)
    inv, px, py, pxr, pl, vc = oracle.is_in_frustum(
        lm["xyz"], lm["normal"], lm["min_dist"], lm["max_dist"], lm["tcw"], S.camera(),
        (0.0, float(S.W), 0.0, float(S.H)), LOG_SCALE, 0.5)
    assert 0.85 < inv.mean() < 0.97
    assert pl[inv > 0].min() >= 0 and pl[inv > 0].max() <= 7
    inv2, fmp, fobs, nm, nto = oracle_search_local_points(f, lm, S.camera())
    assert nm > 300


def _slp_device(mt, f, lm, m, th, calls=1):
    """orbfe_search_local_points_device on device copies of (f, lm), `calls` times on one
    matcher (the frame's slots reset before each call); returns the last call's outputs."""
    import torch
    dev = torch.device("cuda", 0)
    T = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in lm.items()}
    d_keys = torch.from_numpy(f.keys.view(np.uint8).copy()).to(dev)
    d_desc = torch.from_numpy(f.desc).to(dev)
    d_ur = torch.from_numpy(f.u_right).to(dev) if f.u_right is not None else None
    d_inv = torch.zeros(m, dtype=torch.uint8, device=dev)
    fmp0, fobs0 = T["frame_mp"].clone(), T["frame_mp_obs"].clone()
    for _ in range(calls):
        T["frame_mp"].copy_(fmp0)
        T["frame_mp_obs"].copy_(fobs0)
        torch.cuda.synchronize()  # the inputs (and d_inv's fill) on torch's stream are complete
        r = mt.search_local_points_device(
            f.n, d_keys.data_ptr(), d_desc.data_ptr(), d_ur.data_ptr() if d_ur is not None else None,
            S.W, S.H, f.scale_factors, lm["tcw"], S.camera(), LOG_SCALE, 0.5, m,
            T["xyz"].data_ptr(), T["normal"].data_ptr(), T["min_dist"].data_ptr(),
            T["max_dist"].data_ptr(), T["desc"].data_ptr(), T["nobs"].data_ptr(),
            T["bad"].data_ptr(), T["skip"].data_ptr(), T["ids"].data_ptr(), 0.8, th,
            T["frame_mp"].data_ptr(), T["frame_mp_obs"].data_ptr(), d_inv.data_ptr())
    return r, d_inv.cpu().numpy(), T["frame_mp"].cpu().numpy(), T["frame_mp_obs"].cpu().numpy()


@pytest.mark.gpu
@pytest.mark.parametrize("seed,m,th,stereo", [(0, 50000, 1.0, False), (1, 50000, 3.0, False),
                                              (2, 20000, 1.0, True), (3, 1000, 5.0, False)])
@pytest.mark.parametrize("zc", ["1", "0"])
def test_gpu_search_local_points(seed, m, th, stereo, zc, monkeypatch):
    """...with the tallies written by the last workgroup into device-mapped pinned memory
    (ORBFE_ZERO_COPY=1) and through a D2H copy (0), three calls on one matcher (the done
    counter and tally buffers reused)."""
    monkeypatch.setenv("ORBFE_ZERO_COPY", zc)
    from orbslam_mapsave_amd.native import ORBmatcher
    f = S.extract_frame(seed, 1000, u_right=stereo)
    lm = synthetic_local_map(f.keys, f.desc, m, seed=seed)
    inv, fmp, fobs, nm, nto = oracle_search_local_points(f, lm, S.camera(), th)
    mt = ORBmatcher(0.8, False, device=0)
    (gnm, gnto), ginv, gfmp, gfobs = _slp_device(mt, f, lm, m, th, calls=3)
    assert (gnm, gnto) == (nm, nto)
    assert np.array_equal(ginv, inv)
    assert np.array_equal(gfmp, fmp)
    assert np.array_equal(gfobs, fobs)
    print(f"rounds={mt.last_rounds()} nmatches={nm} nToMatch={nto}")
    mt.close()


@pytest.mark.gpu
def test_gpu_local_points_problem_sequence():
    """One matcher through a sequence of different problems (new buffers, map sizes, keypoint
    counts and thresholds): every call bit-exact against the oracle."""
    from orbslam_mapsave_amd.native import ORBmatcher
    mt = ORBmatcher(0.8, False, device=0)
    probs = [(0, 50000, 1.0, 1000), (3, 1000, 5.0, 600), (1, 20000, 3.0, 1000), (0, 50000, 1.0, 1000)]
    for seed, m, th, nf in probs:
        f = S.extract_frame(seed, nf)
        lm = synthetic_local_map(f.keys, f.desc, m, seed=seed)
        inv, fmp, fobs, nm, nto = oracle_search_local_points(f, lm, S.camera(), th)
        (gnm, gnto), ginv, gfmp, gfobs = _slp_device(mt, f, lm, m, th, calls=2)
        assert (gnm, gnto) == (nm, nto), (seed, m)
        assert np.array_equal(ginv, inv) and np.array_equal(gfmp, fmp)
        assert np.array_equal(gfobs, fobs)
    mt.close()


def dense_frame(seed: int = 5, nfeatures: int = 2000):
    """A frame of ~2000 keypoints for the fused kernel's in-LDS grid (its second keypoint per
    thread, k >= 1024): 300 of them moved into three 64x48-grid cells (~100 per cell, the
    per-cell insertion sort at its longest), 40 moved off the image (no grid cell)."""
    from orbslam_mapsave_amd.abi import Frame
    f0 = S.extract_frame(seed, nfeatures)
    keys = f0.keys.copy()
    rng = np.random.default_rng(seed)
    idx = rng.choice(len(keys), 340, replace=False)
    cl, off = idx[:300], idx[300:]
    cx = np.array([101.0, 320.5, 600.0])[np.arange(300) % 3]
    cy = np.array([101.0, 240.5, 400.0])[np.arange(300) % 3]
    keys["x"][cl] = (cx + rng.uniform(0, 9.5, 300)).astype(np.float32)  # cells of 10 x 10 px
    keys["y"][cl] = (cy + rng.uniform(0, 9.5, 300)).astype(np.float32)
    keys["x"][off] = np.where(np.arange(40) % 2, -3.0 - np.arange(40), S.W + 2.0 + np.arange(40))
    return Frame(keys, f0.desc, S.W, S.H, f0.scale_factors)


@pytest.mark.gpu
@pytest.mark.parametrize("m,th", [(50000, 1.0), (20000, 3.0)])
def test_gpu_fused_grid_dense_frame(m, th):
    """The fused kernel's frame grid built in LDS (both forms: isInFrustum evaluated in the
    kernel, and read from resident outputs) on a dense, clustered frame with off-image
    keypoints, bit-exact against the oracle."""
    import torch
    from orbslam_mapsave_amd.native import ORBmatcher
    f = dense_frame()
    assert 1024 < f.n <= 2048
    lm = synthetic_local_map(f.keys, f.desc, m, seed=7)
    inv, fmp, fobs, nm, nto = oracle_search_local_points(f, lm, S.camera(), th)
    mt = ORBmatcher(0.8, False, device=0)
    (gnm, gnto), ginv, gfmp, gfobs = _slp_device(mt, f, lm, m, th, calls=2)
    assert (gnm, gnto) == (nm, nto)
    assert np.array_equal(ginv, inv) and np.array_equal(gfmp, fmp) and np.array_equal(gfobs, fobs)
    # kPre = true: the resident isInFrustum outputs
    _, px, py, pxr, pl, vc = oracle.is_in_frustum(
        lm["xyz"], lm["normal"], lm["min_dist"], lm["max_dist"], lm["tcw"], S.camera(),
        (0.0, float(S.W), 0.0, float(S.H)), LOG_SCALE, 0.5)
    dev = torch.device("cuda", 0)
    up = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    D = {k: up(v) for k, v in dict(inv=inv, bad=lm["bad"], px=px, py=py, pxr=pxr, pl=pl, vc=vc,
                                   desc=lm["desc"], nobs=lm["nobs"], ids=lm["ids"],
                                   fmp=lm["frame_mp"], fobs=lm["frame_mp_obs"]).items()}
    d_keys, d_desc = up(f.keys.view(np.uint8)), up(f.desc)
    torch.cuda.synchronize()
    gnm2 = mt.search_by_projection_local_device(
        f.n, d_keys.data_ptr(), d_desc.data_ptr(), None, S.W, S.H, f.scale_factors, m,
        D["inv"].data_ptr(), D["bad"].data_ptr(), D["px"].data_ptr(), D["py"].data_ptr(),
        D["pxr"].data_ptr(), D["pl"].data_ptr(), D["vc"].data_ptr(), D["desc"].data_ptr(),
        D["nobs"].data_ptr(), D["ids"].data_ptr(), 0.8, th, D["fmp"].data_ptr(),
        D["fobs"].data_ptr())
    assert gnm2 == nm
    assert np.array_equal(D["fmp"].cpu().numpy(), fmp)
    assert np.array_equal(D["fobs"].cpu().numpy(), fobs)
    mt.close()


@pytest.mark.gpu
@pytest.mark.parametrize("seed,m,th,stereo", [(0, 50000, 1.0, False), (2, 20000, 1.0, True),
                                              (3, 1000, 5.0, False), (3, 1000, 12.0, False)])
@pytest.mark.parametrize("path", ["fused", "csr"])
def test_gpu_search_by_projection_local_device(seed, m, th, stereo, path, monkeypatch):
    """A14 alone on device-resident isInFrustum outputs (orbfe_search_by_projection_local_device,
    config 5's "A14 alone" leg): slots, Observations and nmatches exact vs the oracle, on the
    fused fixed-slot path (th = 12: points past its 16 candidates, so the CSR fallback) and with
    the CSR path forced (ORBFE_SBP_DEVICE_CSR)."""
    import torch
    if path == "csr":
        monkeypatch.setenv("ORBFE_SBP_DEVICE_CSR", "1")
    else:
        monkeypatch.delenv("ORBFE_SBP_DEVICE_CSR", raising=False)
    from orbslam_mapsave_amd.native import ORBmatcher
    f = S.extract_frame(seed, 1000, u_right=stereo)
    lm = synthetic_local_map(f.keys, f.desc, m, seed=seed)
    cam = S.camera()
    inv, px, py, pxr, pl, vc = oracle.is_in_frustum(
        lm["xyz"], lm["normal"], lm["min_dist"], lm["max_dist"], lm["tcw"], cam,
        (0.0, float(S.W), 0.0, float(S.H)), LOG_SCALE, 0.5)
    inv[(lm["skip"] > 0) | (lm["bad"] > 0)] = 0
    mps = MapPoints(px, py, pl, vc, lm["desc"], lm["nobs"], track_in_view=inv,
                    is_bad=lm["bad"], proj_xr=pxr)
    fmp, fobs, nm = oracle.search_by_projection_local(f, mps, th, 0.8, lm["frame_mp"],
                                                      lm["frame_mp_obs"], lm["ids"])
    dev = torch.device("cuda", 0)
    up = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    D = {k: up(v) for k, v in dict(inv=inv, bad=lm["bad"], px=px, py=py, pxr=pxr, pl=pl, vc=vc,
                                   desc=lm["desc"], nobs=lm["nobs"], ids=lm["ids"],
                                   fmp=lm["frame_mp"], fobs=lm["frame_mp_obs"]).items()}
    d_keys = up(f.keys.view(np.uint8))
    d_desc = up(f.desc)
    d_ur = up(f.u_right) if f.u_right is not None else None
    mt = ORBmatcher(0.8, False, device=0)
    torch.cuda.synchronize()
    gnm = mt.search_by_projection_local_device(
        f.n, d_keys.data_ptr(), d_desc.data_ptr(), d_ur.data_ptr() if d_ur is not None else None,
        S.W, S.H, f.scale_factors, m, D["inv"].data_ptr(), D["bad"].data_ptr(),
        D["px"].data_ptr(), D["py"].data_ptr(), D["pxr"].data_ptr(), D["pl"].data_ptr(),
        D["vc"].data_ptr(), D["desc"].data_ptr(), D["nobs"].data_ptr(), D["ids"].data_ptr(), 0.8,
        th, D["fmp"].data_ptr(), D["fobs"].data_ptr())
    assert gnm == nm
    assert np.array_equal(D["fmp"].cpu().numpy(), fmp)
    assert np.array_equal(D["fobs"].cpu().numpy(), fobs)
    if path == "fused" and th == 12.0:
        assert mt.capacity_retries() >= 1
    mt.close()
