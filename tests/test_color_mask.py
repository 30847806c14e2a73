"""§8(f) row 1 — colour conversion + human mask in front of the extractor.

Reference: Tracking::GrabImage{Stereo,RGBD,Monocular} convert with cvtColor(CV_*2GRAY)
(Tracking.cc:286-310, 350-363, 409-422) and pass OpDetector's square mask
(DetectHumanPose.cpp:453-489) to Frame::ExtractORBMask -> operator()(gray, mask)
(Frame.cc:366-371, ORBextractor.cc:1053).  The GPU fuses both into one level-0 kernel
(level0_kernel); parity is bit-exact against oracle_cvt_gray + oracle_extract.

The oracle's cvtColor is OpenCV's RGB2Gray<uchar> table path; it is pinned here
against an independent restatement of the published integer formula.  OpDetector's rectangle is
restated in Python and compared with the C helper orbfe_human_mask_rect (host-only code).
"""
import math

import numpy as np
import pytest

import oracle
from orbslam_mapsave_amd import native
from orbslam_mapsave_amd.synth import synthetic_color_frame, synthetic_mask

R2Y, G2Y, B2Y = 4899, 9617, 1868
PIX = {"RGB": (native.PIX_RGB, 3), "BGR": (native.PIX_BGR, 3), "RGBA": (native.PIX_RGBA, 4),
       "BGRA": (native.PIX_BGRA, 4)}


def gray_formula(img: np.ndarray, name: str) -> np.ndarray:
    """Y = (R*4899 + G*9617 + B*1868 + 2^13) >> 14 (OpenCV yuv_shift = 14 fixed point)."""
    x = img.astype(np.int64)
    r, g, b = (x[..., 0], x[..., 1], x[..., 2]) if name.startswith("RGB") else (x[..., 2], x[..., 1], x[..., 0])
    return ((r * R2Y + g * G2Y + b * B2Y + (1 << 13)) >> 14).astype(np.uint8)


@pytest.mark.parametrize("name", sorted(PIX))
def test_oracle_cvt_gray_formula(name):
    pix, cn = PIX[name]
    rng = np.random.Generator(np.random.PCG64(3))
    img = rng.integers(0, 256, (300, 257, cn), dtype=np.uint8)
    img[0, :8, :3] = [[0, 0, 0], [255, 255, 255], [255, 0, 0], [0, 255, 0], [0, 0, 255],
                      [255, 255, 0], [1, 2, 3], [128, 128, 128]]
    assert np.array_equal(oracle.cvt_gray(img, pix), gray_formula(img, name))


def test_oracle_cvt_gray_exhaustive_rgb():
    v = np.arange(256, dtype=np.uint8)
    r, g, b = np.meshgrid(v, v, v, indexing="ij")
    img = np.stack([r.ravel(), g.ravel(), b.ravel()], -1).reshape(4096, 4096, 3)
    assert np.array_equal(oracle.cvt_gray(img, native.PIX_RGB), gray_formula(img, "RGB"))


def rect_restated(joints: np.ndarray, w: int, h: int):
    """DetectHumanPose.cpp:453-489 restated: float ternary then static_cast<int> (truncation)."""
    xmin, ymin, xmax, ymax = w - 1, h - 1, 0, 0
    for x, y, _ in np.asarray(joints, np.float32).tolist():  # exact float32 values as Python floats
        xmin = math.trunc(x if x < xmin else float(xmin))
        xmax = math.trunc(x if x > xmax else float(xmax))
        ymin = math.trunc(y if y < ymin else float(ymin))
        ymax = math.trunc(y if y > ymax else float(ymax))
    xmin, xmax, ymin, ymax = xmin - 30, xmax + 30, ymin - 30, ymax + 30
    return (max(xmin, 0) if xmin > 0 else 0, max(ymin, 0) if ymin > 0 else 0,
            w - 1 if xmax >= w - 1 else xmax, h - 1 if ymax >= h - 1 else ymax)


@pytest.mark.parametrize("seed", range(6))
def test_human_mask_rect(seed):
    rng = np.random.Generator(np.random.PCG64(seed))
    cx, cy = rng.uniform(0, 640), rng.uniform(0, 480)
    j = np.stack([cx + rng.normal(0, 60, 25), cy + rng.normal(0, 90, 25), rng.uniform(0, 1, 25)], 1)
    if seed == 0:
        j[:] = 0  # no detection: all-zero joints
    assert native.human_mask_rect(j, 640, 480) == rect_restated(j, 640, 480)


def rect_mask(rect, w, h):
    m = np.ones((h, w), np.uint8)
    x0, y0, x1, y1 = rect
    m[y0:y1, x0:x1] = 0
    return m


# ---------------------------------------------------------------------------------------------
# GPU parity
CFG = (1000, 1.2, 8, 32, 7)


@pytest.fixture(scope="module")
def ex():
    e = native.ORBextractor(*CFG, device=0, max_width=640, max_height=480)
    yield e
    e.close()


def _same(k, d, ok, od):
    assert len(k) == len(ok), (len(k), len(ok))
    assert k.tobytes() == ok.tobytes()
    assert np.array_equal(d, od)


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(PIX))
def test_extract_color_bit_exact(ex, name):
    pix, cn = PIX[name]
    img = synthetic_color_frame(21, 640, 480, cn)
    kps, desc = ex.extract_color(img, pix)
    gray = oracle.cvt_gray(img, pix)
    assert np.array_equal(ex.get_level(0), gray)
    okps, odesc = oracle.extract(oracle.params(*CFG), gray)
    _same(kps, desc, okps, odesc)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["plane", "rect", "both"])
def test_extract_color_masks(ex, mode):
    img = synthetic_color_frame(22, 640, 480, 3)
    plane = synthetic_mask(640, 480, 5)
    rng = np.random.Generator(np.random.PCG64(9))
    j = np.stack([300 + rng.normal(0, 40, 25), 200 + rng.normal(0, 60, 25), np.ones(25)], 1)
    rect = native.human_mask_rect(j, 640, 480)
    m = {"plane": plane, "rect": rect_mask(rect, 640, 480),
         "both": plane & rect_mask(rect, 640, 480)}[mode]
    kps, desc = ex.extract_color(img, native.PIX_BGR, mask=plane if mode != "rect" else None,
                                 rect=rect if mode != "plane" else None)
    gray = oracle.cvt_gray(img, native.PIX_BGR)
    okps, odesc = oracle.extract(oracle.params(*CFG), gray, m)
    _same(kps, desc, okps, odesc)
    assert np.array_equal(ex.get_level(0), np.where(m > 0, gray, 0))


@pytest.mark.gpu
def test_extract_gray_rect_only(ex):
    from orbslam_mapsave_amd.synth import synthetic_frame
    img = synthetic_frame(23, 640, 480)
    rect = (100, 50, 400, 300)
    kps, desc = ex.extract_color(img, native.PIX_GRAY, rect=rect)
    okps, odesc = oracle.extract(oracle.params(*CFG), img, rect_mask(rect, 640, 480))
    _same(kps, desc, okps, odesc)


@pytest.mark.gpu
def test_color_batch_device_unaligned():
    """Device colour batch with an odd row stride (byte-load path), masks and rectangles."""
    import torch
    n, w, h = 3, 641, 479
    e = native.ORBextractor(*CFG, device=0, max_width=w, max_height=h, max_batch=n)
    imgs = np.stack([synthetic_color_frame(30 + f, w, h, 3) for f in range(n)])
    stride = w * 3 + 1
    buf = np.zeros((n, h, stride), np.uint8)
    buf[:, :, :w * 3] = imgs.reshape(n, h, w * 3)
    masks = np.stack([synthetic_mask(w, h, f) for f in range(n)])
    rects = np.array([[10, 20, 300, 200], [0, 0, 0, 0], [500, 400, 640, 478]], np.int32)
    dev = torch.device("cuda", 0)
    d_img = torch.from_numpy(buf).to(dev)
    d_m = torch.from_numpy(masks).to(dev)
    d_r = torch.from_numpy(rects).to(dev)
    cap = e.capacity(w, h)
    d_k = torch.zeros((n, cap * 28), dtype=torch.uint8, device=dev)
    d_d = torch.zeros((n, cap, 32), dtype=torch.uint8, device=dev)
    d_n = torch.zeros(n, dtype=torch.int32, device=dev)
    e.extract_color_batch_device(d_img.data_ptr(), native.PIX_RGB, n, w, h, stride, h * stride,
                                 d_k.data_ptr(), cap, d_d.data_ptr(), d_n.data_ptr(),
                                 d_masks=d_m.data_ptr(), mask_stride=w, mask_frame_pitch=w * h,
                                 d_rects=d_r.data_ptr())
    e.synchronize()
    cnt = d_n.cpu().numpy()
    kb = d_k.cpu().numpy()
    db = d_d.cpu().numpy()
    p = oracle.params(*CFG)
    for f in range(n):
        gray = oracle.cvt_gray(imgs[f], native.PIX_RGB)
        m = masks[f] & rect_mask(rects[f], w, h)
        okps, odesc = oracle.extract(p, gray, m)
        assert cnt[f] == len(okps)
        assert kb[f, :cnt[f] * 28].tobytes() == okps.tobytes()
        assert np.array_equal(db[f, :cnt[f]], odesc)
    e.close()


@pytest.mark.gpu
def test_unsupported_rect(ex):
    img = synthetic_color_frame(24, 640, 480, 3)
    with pytest.raises(native.OrbfeError):
        ex.extract_color(img, native.PIX_RGB, rect=(300, 10, 200, 50))
