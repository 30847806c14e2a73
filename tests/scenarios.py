"""Seeded matcher scenarios shared by the CPU (oracle/golden) and GPU (parity) tests.

Frames come from the oracle extractor on synthetic images, so no GPU is needed to build them.
"""
from __future__ import annotations

import numpy as np

import oracle
from orbslam_mapsave_amd.abi import KEYPOINT_DTYPE, Camera, Frame, MapPoints
from orbslam_mapsave_amd.synth import synthetic_frame

W, H = 640, 480
FX = FY = 500.0
CX, CY = 320.0, 240.0


def extract_frame(seed: int, nfeatures=1000, shift=(0, 0), w=W, h=H, ini=32, u_right=False):
    img = synthetic_frame(seed, w, h)
    if shift != (0, 0):
        img = np.roll(img, shift, axis=(0, 1))
    p = oracle.params(nfeatures, 1.2, 8, ini, 7)
    kps, desc = oracle.extract(p, img)
    scale = oracle.tables(p)["scale"]
    ur = None
    if u_right:
        rng = np.random.Generator(np.random.PCG64(seed + 77))
        ur = np.where(rng.uniform(size=len(kps)) < 0.5, kps["x"] - rng.uniform(2, 40, len(kps)),
                      -1).astype(np.float32)
    return Frame(kps, desc, w, h, scale, ur)


def sfi_case(seed: int = 0):
    """Monocular initialization: F1 with the 2x-feature init extractor (Tracking.cc:215),
    F2 = the image shifted by a few pixels."""
    f1 = extract_frame(seed, 2000)
    f2 = extract_frame(seed, 2000, shift=(3, -4))
    prev = np.stack([f1.keys["x"], f1.keys["y"]], 1).astype(np.float32)
    return f1, f2, prev


def flip_bits(desc: np.ndarray, rng, p: float) -> np.ndarray:
    bits = np.unpackbits(desc, axis=-1)
    flip = (rng.uniform(size=bits.shape) < p).astype(np.uint8)
    return np.packbits(bits ^ flip, axis=-1)


def sbp_local_case(seed: int = 0, m: int = 50000, frame: Frame | None = None, stereo=False,
                   prior=False):
    """Config 5: M map points, 60% within 2 px of a real keypoint with its
    descriptor ~8% bit-flipped, level = keypoint octave +{0,1} clipped to the pyramid,
    viewCos ~ U[0.5, 1]; the rest uniform with random descriptors."""
    rng = np.random.Generator(np.random.PCG64(seed + 5))
    f = frame if frame is not None else extract_frame(seed, 1000, u_right=stereo)
    n = f.n
    true = rng.uniform(size=m) < 0.6
    src = rng.integers(0, n, m)
    px = np.where(true, f.keys["x"][src] + rng.uniform(-2, 2, m), rng.uniform(0, W, m))
    py = np.where(true, f.keys["y"][src] + rng.uniform(-2, 2, m), rng.uniform(0, H, m))
    lvl = np.where(true, f.keys["octave"][src] + rng.integers(0, 2, m), rng.integers(0, 8, m))
    lvl = np.clip(lvl, 0, 7)
    desc = np.where(true[:, None], flip_bits(f.desc[src], rng, 0.08),
                    rng.integers(0, 256, (m, 32), dtype=np.uint8)).astype(np.uint8)
    vcos = rng.uniform(0.5, 1.0, m)
    vcos[rng.uniform(size=m) < 0.1] = 0.999  # the 2.5-radius branch
    nobs = rng.integers(1, 6, m)
    nobs[rng.uniform(size=m) < 0.05] = 0     # observation-less points do not block
    pxr = px - rng.uniform(2, 40, m) if stereo else np.full(m, -1.0)
    mps = MapPoints(px, py, lvl, vcos, desc, nobs,
                    track_in_view=(rng.uniform(size=m) < 0.95).astype(np.uint8),
                    is_bad=(rng.uniform(size=m) < 0.02).astype(np.uint8), proj_xr=pxr)
    fmp = fobs = None
    if prior:
        fmp = np.where(rng.uniform(size=n) < 0.2, rng.integers(0, 1000, n), -1).astype(np.int32)
        fobs = np.where(fmp >= 0, rng.integers(0, 3, n), 0).astype(np.int32)
    ids = (np.arange(m) + 100000).astype(np.int32)
    return f, mps, fmp, fobs, ids


def pose(rng, angle=0.02, trans=0.05) -> np.ndarray:
    ax = rng.normal(size=3)
    ax /= np.linalg.norm(ax)
    k = np.array([[0, -ax[2], ax[1]], [ax[2], 0, -ax[0]], [-ax[1], ax[0], 0]])
    R = np.eye(3) + np.sin(angle) * k + (1 - np.cos(angle)) * k @ k
    t = rng.normal(size=3) * trans
    return np.hstack([R, t[:, None]]).astype(np.float32)


def camera(bf=40.0) -> Camera:
    return Camera(FX, FY, CX, CY, bf, bf / FX)


def sbp_last_case(seed: int = 0, stereo=False, motion=(0.02, 0.05)):
    """Tracking with the motion model: the last frame's keypoints hold map points placed at
    random depth along their rays (last pose = identity); the current frame is the same scene
    seen after a small motion (image shifted to roughly follow it)."""
    rng = np.random.Generator(np.random.PCG64(seed + 9))
    last = extract_frame(seed, 1000)
    cur = extract_frame(seed, 1000, shift=(2, 3), u_right=stereo)
    n = last.n
    z = rng.uniform(2.0, 8.0, n)
    xyz = np.stack([(last.keys["x"] - CX) / FX * z, (last.keys["y"] - CY) / FY * z, z], 1)
    valid = (rng.uniform(size=n) < 0.85).astype(np.uint8)
    outlier = (rng.uniform(size=n) < 0.05).astype(np.uint8)
    desc = flip_bits(last.desc, rng, 0.05)
    nobs = rng.integers(1, 5, n)
    nobs[rng.uniform(size=n) < 0.1] = 0
    tcw_last = np.hstack([np.eye(3), np.zeros((3, 1))]).astype(np.float32)
    tcw_cur = pose(rng, *motion)
    return dict(cur=cur, tcw_cur=tcw_cur, cam=camera(), last_keys=last.keys, last_valid=valid,
                last_outlier=outlier, last_xyz=xyz.astype(np.float32), last_desc=desc,
                last_nobs=nobs.astype(np.int32), tcw_last=tcw_last,
                last_ids=(np.arange(n) + 500).astype(np.int32))


def frustum_case(seed: int = 0, m: int = 20000):
    rng = np.random.Generator(np.random.PCG64(seed + 13))
    xyz = np.stack([rng.uniform(-6, 6, m), rng.uniform(-5, 5, m), rng.uniform(-2, 12, m)], 1)
    normal = rng.normal(size=(m, 3))
    normal /= np.linalg.norm(normal, axis=1, keepdims=True)
    normal[:, 2] = np.abs(normal[:, 2])
    maxd = rng.uniform(2, 15, m)
    scale7 = np.float32(1.2) ** 7
    mind = maxd / scale7
    tcw = pose(rng, 0.05, 0.2)
    return dict(xyz=xyz.astype(np.float32), normal=normal.astype(np.float32),
                min_dist=mind.astype(np.float32), max_dist=maxd.astype(np.float32), tcw=tcw,
                cam=camera(), bounds=(0.0, float(W), 0.0, float(H)),
                log_scale=float(np.log(np.float32(1.2)).astype(np.float32)), cos_limit=0.5)


def random_desc(rng, n) -> np.ndarray:
    return rng.integers(0, 256, (n, 32), dtype=np.uint8)


def sbp_keyframe_case(seed: int = 0, motion=(0.01, 0.03)):
    """Relocalisation (Tracking.cc:1723/1737): a candidate keyframe whose keypoints hold map
    points along their rays (keyframe pose = identity); the current frame sees the scene after
    a small motion and already holds some map points (from SearchByBoW + PnP).  mfMaxDistance
    = 0.97 * dist * scale[octave] keeps the predicted level inside the pyramid."""
    rng = np.random.Generator(np.random.PCG64(seed + 21))
    kf = extract_frame(seed, 1000)
    cur = extract_frame(seed, 1000, shift=(1, 2))
    n = kf.n
    z = rng.uniform(2.0, 8.0, n)
    xyz = np.stack([(kf.keys["x"] - CX) / FX * z, (kf.keys["y"] - CY) / FY * z, z], 1)
    dist = np.linalg.norm(xyz, axis=1)
    scale = np.float32(1.2) ** np.arange(8, dtype=np.float32)
    maxd = (0.97 * dist * scale[kf.keys["octave"]]).astype(np.float32)
    mind = (maxd / scale[7]).astype(np.float32)
    valid = (rng.uniform(size=n) < 0.9).astype(np.uint8)
    bad = (rng.uniform(size=n) < 0.03).astype(np.uint8)
    found = (rng.uniform(size=n) < 0.2).astype(np.uint8)
    desc = flip_bits(kf.desc, rng, 0.06)
    frame_mp = np.where(rng.uniform(size=cur.n) < 0.15, rng.integers(0, 10_000, cur.n), -1)
    return dict(cur=cur, tcw_cur=pose(rng, *motion), cam=camera(),
                log_scale=float(np.log(np.float32(1.2)).astype(np.float32)),
                frame_mp=frame_mp.astype(np.int32), kf_angle=kf.keys["angle"].astype(np.float32),
                kf_valid=valid, kf_bad=bad, found=found, kf_xyz=xyz.astype(np.float32),
                kf_desc=desc, kf_min=mind, kf_max=maxd,
                kf_ids=(np.arange(n) + 20_000).astype(np.int32))
