"""Seeded synthetic frames for parity tests and the bench (SURVEY.md §8d "Synthetic images").

Textured, not white noise (noise would saturate every FAST cell): multi-octave value noise
smoothed with a sigma=1.5 Gaussian, 200 filled rectangles/ellipses of random gray and 50
anti-aliased lines, clipped to u8.  Variants exercise the reference's edge paths:
``low_contrast`` (x0.15 around mid-gray: the minThFAST fallback, ORBextractor.cc:811-815),
``constant`` (no corners: the zero-keypoint path, ORBextractor.cc:1067-1068) and a mask with a
zero rectangle (Mat::copyTo(dst, mask), ORBextractor.cc:1053).

Pure numpy (PCG64), identical here and on the GPU box.
"""
from __future__ import annotations

import numpy as np


def _gauss1d(sigma: float) -> np.ndarray:
    r = int(np.ceil(3 * sigma))
    x = np.arange(-r, r + 1, dtype=np.float64)
    k = np.exp(-0.5 * (x / sigma) ** 2)
    return (k / k.sum()).astype(np.float32)


def _smooth(img: np.ndarray, sigma: float) -> np.ndarray:
    k = _gauss1d(sigma)
    r = len(k) // 2
    p = np.pad(img, ((0, 0), (r, r)), mode="reflect")
    out = sum(k[i] * p[:, i:i + img.shape[1]] for i in range(len(k)))
    p = np.pad(out, ((r, r), (0, 0)), mode="reflect")
    return sum(k[i] * p[i:i + img.shape[0], :] for i in range(len(k)))


def _value_noise(rng: np.random.Generator, h: int, w: int) -> np.ndarray:
    img = np.zeros((h, w), np.float32)
    for cell, amp in ((96, 55.0), (24, 35.0), (6, 22.0)):
        gh, gw = h // cell + 2, w // cell + 2
        g = rng.uniform(-1.0, 1.0, (gh, gw)).astype(np.float32)
        ys = np.arange(h, dtype=np.float32) / cell
        xs = np.arange(w, dtype=np.float32) / cell
        y0 = ys.astype(np.int64)
        x0 = xs.astype(np.int64)
        fy = (ys - y0)[:, None]
        fx = (xs - x0)[None, :]
        v = (g[y0][:, x0] * (1 - fy) * (1 - fx) + g[y0 + 1][:, x0] * fy * (1 - fx)
             + g[y0][:, x0 + 1] * (1 - fy) * fx + g[y0 + 1][:, x0 + 1] * fy * fx)
        img += amp * v
    return img + 128.0


def synthetic_frame(seed: int, w: int = 640, h: int = 480, kind: str = "textured") -> np.ndarray:
    """Return an (h, w) uint8 frame for `seed`; kind in textured|low_contrast|constant."""
    if kind == "constant":
        return np.full((h, w), 97, np.uint8)
    rng = np.random.Generator(np.random.PCG64(seed))
    img = _smooth(_value_noise(rng, h, w), 1.5)
    scale = max(w, h) / 640.0
    for _ in range(200):  # filled rectangles / ellipses
        cx, cy = rng.uniform(0, w), rng.uniform(0, h)
        rx, ry = rng.uniform(4, 40) * scale, rng.uniform(4, 40) * scale
        gray = rng.uniform(0, 255)
        x0, x1 = int(max(cx - rx, 0)), int(min(cx + rx + 1, w))
        y0, y1 = int(max(cy - ry, 0)), int(min(cy + ry + 1, h))
        if x1 <= x0 or y1 <= y0:
            continue
        if rng.uniform() < 0.5:
            img[y0:y1, x0:x1] = gray
        else:
            yy, xx = np.mgrid[y0:y1, x0:x1]
            inside = ((xx - cx) / rx) ** 2 + ((yy - cy) / ry) ** 2 <= 1.0
            img[y0:y1, x0:x1][inside] = gray
    for _ in range(50):  # anti-aliased lines: coverage from distance to the segment
        ax, ay, bx, by = rng.uniform(0, w), rng.uniform(0, h), rng.uniform(0, w), rng.uniform(0, h)
        width = rng.uniform(0.8, 3.0) * scale
        gray = rng.uniform(0, 255)
        x0, x1 = int(max(min(ax, bx) - width - 1, 0)), int(min(max(ax, bx) + width + 2, w))
        y0, y1 = int(max(min(ay, by) - width - 1, 0)), int(min(max(ay, by) + width + 2, h))
        if x1 <= x0 or y1 <= y0:
            continue
        yy, xx = np.mgrid[y0:y1, x0:x1].astype(np.float32)
        dx, dy = bx - ax, by - ay
        t = np.clip(((xx - ax) * dx + (yy - ay) * dy) / max(dx * dx + dy * dy, 1e-6), 0, 1)
        dist = np.hypot(xx - (ax + t * dx), yy - (ay + t * dy))
        cov = np.clip(width / 2 + 0.5 - dist, 0, 1)
        sub = img[y0:y1, x0:x1]
        img[y0:y1, x0:x1] = sub * (1 - cov) + gray * cov
    if kind == "low_contrast":
        img = 128.0 + (img - 128.0) * 0.15
    elif kind != "textured":
        raise ValueError(f"unknown kind {kind!r}")
    return np.clip(np.rint(img), 0, 255).astype(np.uint8)


def synthetic_mask(w: int = 640, h: int = 480, seed: int = 0) -> np.ndarray:
    """A human-mask-like u8 mask: ones with one zero rectangle (DetectHumanPose.cpp:453-489)."""
    rng = np.random.Generator(np.random.PCG64(seed + 1000))
    m = np.ones((h, w), np.uint8)
    x0, y0 = int(rng.uniform(0.2, 0.5) * w), int(rng.uniform(0.1, 0.4) * h)
    m[y0:y0 + h // 3, x0:x0 + w // 4] = 0
    return m


def synthetic_batch(n: int, w: int = 640, h: int = 480, first_seed: int = 0,
                    distinct: int | None = None) -> np.ndarray:
    """(n, h, w) uint8 frames; with `distinct` set, that many seeds are generated and cycled."""
    d = n if distinct is None else max(1, min(distinct, n))
    frames = [synthetic_frame(first_seed + i, w, h) for i in range(d)]
    return np.stack([frames[i % d] for i in range(n)])


def synthetic_color_frame(seed: int, w: int = 640, h: int = 480, channels: int = 3) -> np.ndarray:
    """(h, w, channels) uint8 colour frame: three correlated textured planes (the gray texture
    plus a per-channel tint and a second texture), alpha random for 4 channels."""
    base = synthetic_frame(seed, w, h).astype(np.float32)
    other = synthetic_frame(seed + 50_000, w, h).astype(np.float32)
    rng = np.random.Generator(np.random.PCG64(seed + 7))
    planes = []
    for c in range(3):
        a, b, t = rng.uniform(0.5, 1.0), rng.uniform(0.0, 0.4), rng.uniform(-30, 30)
        planes.append(np.clip(np.rint(a * base + b * other + t), 0, 255).astype(np.uint8))
    if channels == 4:
        planes.append(rng.integers(0, 256, (h, w), dtype=np.uint8))
    return np.ascontiguousarray(np.stack(planes, -1))


def synthetic_stereo_pair(seed: int, w: int = 640, h: int = 480, d0: float = 4.0,
                          d1: float = 40.0) -> tuple[np.ndarray, np.ndarray]:
    """A rectified pair: the right image samples the left one at x + d(x, y) with a disparity
    ramp d from d0 (top) to d1 (bottom) plus a gentle x tilt (a slanted plane), bilinear, so
    matches are sub-pixel and the ORB keypoints of both images correspond."""
    left = synthetic_frame(seed, w, h + 0).astype(np.float32)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
    d = d0 + (d1 - d0) * yy / max(h - 1, 1) + 3.0 * xx / max(w - 1, 1)
    sx = np.clip(xx + d, 0, w - 1)
    x0 = np.floor(sx).astype(np.int64)
    x1 = np.minimum(x0 + 1, w - 1)
    t = sx - x0
    rows = np.arange(h)[:, None]
    right = left[rows, x0] * (1 - t) + left[rows, x1] * t
    return left.astype(np.uint8), np.clip(np.rint(right), 0, 255).astype(np.uint8)


def synthetic_local_map(keys: np.ndarray, desc: np.ndarray, m: int = 50_000, seed: int = 0,
                        w: int = 640, h: int = 480, fx: float = 500.0, fy: float = 500.0,
                        cx: float = 320.0, cy: float = 240.0, nlevels: int = 8,
                        scale: float = 1.2) -> dict:
    """BASELINE config 5 as world-space map points seen by a camera at the
    identity pose: 60% project within 2 px of a real keypoint with its descriptor ~8% bit-flipped
    and a predicted level of the keypoint's octave + {0, 1}; the rest project uniformly with
    random descriptors and levels.  mfMaxDistance = dist * scale^(level - 1/2) makes
    MapPoint::PredictScale return that level; mfMinDistance = mfMaxDistance / scale^(nlevels-1).
    Normals make viewing cosines ~U[0.5, 1] (10% above 0.998); a few points lie behind the
    camera or outside the image; Observations() in 1..5 (5% zero), 2% bad, 3% already matched
    (skip)."""
    rng = np.random.Generator(np.random.PCG64(seed + 5))
    n = len(keys)
    true = rng.uniform(size=m) < 0.6
    src = rng.integers(0, max(n, 1), m)
    kx = keys["x"][src] if n else np.zeros(m)
    ky = keys["y"][src] if n else np.zeros(m)
    ko = keys["octave"][src] if n else np.zeros(m, np.int32)
    u = np.where(true, kx + rng.uniform(-2, 2, m), rng.uniform(0, w, m))
    v = np.where(true, ky + rng.uniform(-2, 2, m), rng.uniform(0, h, m))
    lvl = np.clip(np.where(true, ko + rng.integers(0, 2, m), rng.integers(0, nlevels, m)), 0,
                  nlevels - 1)
    z = rng.uniform(2.0, 8.0, m)
    off = rng.uniform(size=m)
    u = np.where(off < 0.03, u + 2 * w, u)                       # outside the image
    z = np.where((off >= 0.03) & (off < 0.05), -z, z)            # behind the camera
    xyz = np.stack([(u - cx) / fx * np.abs(z), (v - cy) / fy * np.abs(z), z], 1)
    dist = np.linalg.norm(xyz, axis=1)
    s = np.float64(np.float32(scale))
    maxd = dist * s ** (lvl - 0.5)
    mind = maxd / s ** (nlevels - 1)
    d = xyz / dist[:, None]
    cosv = np.where(rng.uniform(size=m) < 0.1, rng.uniform(0.9985, 1.0, m), rng.uniform(0.5, 1, m))
    perp = np.cross(d, rng.normal(size=(m, 3)))
    perp /= np.linalg.norm(perp, axis=1, keepdims=True)
    normal = d * cosv[:, None] + perp * np.sqrt(1 - cosv ** 2)[:, None]
    bits = np.unpackbits(desc[src] if n else np.zeros((m, 32), np.uint8), axis=1)
    flipped = np.packbits(bits ^ (rng.uniform(size=bits.shape) < 0.08).astype(np.uint8), axis=1)
    mdesc = np.where(true[:, None], flipped, rng.integers(0, 256, (m, 32), dtype=np.uint8))
    nobs = rng.integers(1, 6, m)
    nobs[rng.uniform(size=m) < 0.05] = 0
    fmp = np.where(rng.uniform(size=n) < 0.1, rng.integers(0, 1000, n), -1)
    return dict(xyz=xyz.astype(np.float32), normal=normal.astype(np.float32),
                min_dist=mind.astype(np.float32), max_dist=maxd.astype(np.float32),
                desc=np.ascontiguousarray(mdesc, np.uint8), nobs=nobs.astype(np.int32),
                bad=(rng.uniform(size=m) < 0.02).astype(np.uint8),
                skip=(rng.uniform(size=m) < 0.03).astype(np.uint8),
                ids=(np.arange(m) + 100_000).astype(np.int32),
                frame_mp=fmp.astype(np.int32),
                frame_mp_obs=np.where(fmp >= 0, rng.integers(0, 3, n), 0).astype(np.int32),
                tcw=np.hstack([np.eye(3), np.zeros((3, 1))]).astype(np.float32))


def synthetic_vocabulary_text(path: str, k: int = 10, L: int = 4, seed: int = 0,
                              scoring: int = 0, weighting: int = 0,
                              anchors: np.ndarray | None = None) -> None:
    """Writes a DBoW2 TemplatedVocabulary<FORB> text file (the ORBvoc.txt format,
    TemplatedVocabulary.h:1351-1436 / saveToTextFile): header "k L scoring weighting", then one
    line per node in id order "parent isLeaf d0 .. d31 weight" with weights printed like
    iostream's default (6 significant digits).  A complete k-ary tree of depth L: level-1
    centroids are `anchors` rows (e.g. real ORB descriptors) or random bytes, every child is its
    parent with ~12% of the bits flipped; leaf weights are idf-like, 3% stopped (0).  The file
    ends with a newline, as saveToTextFile writes it."""
    rng = np.random.Generator(np.random.PCG64(seed))
    lines = [f"{k} {L}  {scoring} {weighting}"]
    parents = [0]           # node ids of the previous level
    descs = {0: None}
    nid = 1
    for level in range(1, L + 1):
        nxt = []
        leaf = level == L
        for p in parents:
            for c in range(k):
                if level == 1:
                    d = (anchors[c % len(anchors)] if anchors is not None
                         else rng.integers(0, 256, 32, dtype=np.uint8))
                else:
                    bits = np.unpackbits(descs[p])
                    bits ^= (rng.uniform(size=256) < 0.12).astype(np.uint8)
                    d = np.packbits(bits)
                descs[nid] = d
                w = 0.0 if (leaf and rng.uniform() < 0.03) else (rng.uniform(0.5, 8.0) if leaf else 0.0)
                lines.append(f"{p} {int(leaf)} " + " ".join(str(int(x)) for x in d) + f" {w:.6g}")
                nxt.append(nid)
                nid += 1
        parents = nxt
    with open(path, "w") as fh:
        fh.write("\n".join(lines) + "\n")
