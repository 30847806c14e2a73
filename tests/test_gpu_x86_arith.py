"""ORBFE_ARITH_X86_SIMD: the extractor reproducing an x86-64 build of the reference's OpenCV
3.3 primitives (include/orbfe.h orbfe_set_arithmetic) bit-exactly against the
oracle switched to the same reading (oracle.variant(VAR_H4_FMA | VAR_H5_SSE2 | VAR_H6_SIMD)):

* pyramid levels: VResizeLinearVec_32s8u's SSE2 body (H5) on [0, sse2_body_resize(w)), the
  scalar FixedPtCast tail after it;
* blurred levels: SymmColumnVec_32s8u's float body, ties to even (H6);
* descriptors: the rotation FMA-contracted as GCC -O3 -march=<FMA host> builds it (H4).

The residual study (tests/golden/residuals.json) shows why the mode exists: ~18 % of the pixels
of levels 1-7 and about half of the descriptors differ between the two readings.
"""
import numpy as np
import pytest

import oracle
from orbslam_mapsave_amd.synth import synthetic_frame, synthetic_mask

pytestmark = pytest.mark.gpu

X86 = oracle.VAR_H4_FMA | oracle.VAR_H5_SSE2 | oracle.VAR_H6_SIMD


@pytest.fixture(scope="module")
def ex():
    from orbslam_mapsave_amd.native import ORBextractor
    e = ORBextractor(1000, 1.2, 8, 32, 7, device=0, max_width=640, max_height=480)
    e.set_arithmetic(e.ARITH_X86_SIMD)
    yield e
    e.close()


@pytest.fixture(scope="module")
def p():
    return oracle.params(1000, 1.2, 8, 32, 7)


def same(kps, desc, okps, odesc):
    assert len(kps) == len(okps)
    assert kps.tobytes() == okps.tobytes()
    assert np.array_equal(desc, odesc)


@pytest.mark.parametrize("seed", range(4))
def test_x86_stages_and_extract(ex, p, seed):
    img = synthetic_frame(seed, 640, 480)
    kps, desc = ex(img)
    with oracle.variant(oracle.VAR_H5_SSE2):
        levels = oracle.pyramid(p, img)
    with oracle.variant(oracle.VAR_SCALAR):
        scalar = oracle.pyramid(p, img)
    assert sum(int((a != b).sum()) for a, b in zip(levels, scalar)) > 0  # the modes differ
    for l, lev in enumerate(levels):
        assert np.array_equal(ex.get_level(l), lev), f"level {l}"
        with oracle.variant(oracle.VAR_H6_SIMD):
            ob = oracle.gaussian_blur(lev)
        assert np.array_equal(ex.get_blurred_level(l), ob), f"blur {l}"
    with oracle.variant(X86):
        okps, odesc = oracle.extract(p, img)
    same(kps, desc, okps, odesc)


def test_x86_masked_and_1080(p):
    from orbslam_mapsave_amd.native import ORBextractor
    e = ORBextractor(2000, 1.2, 8, 32, 7, device=0, max_width=1920, max_height=1080)
    e.set_arithmetic(e.ARITH_X86_SIMD)
    p2 = oracle.params(2000, 1.2, 8, 32, 7)
    img = synthetic_frame(0, 1920, 1080)
    kps, desc = e(img)
    with oracle.variant(X86):
        okps, odesc = oracle.extract(p2, img)
    same(kps, desc, okps, odesc)
    img = synthetic_frame(3, 1280, 720)
    m = synthetic_mask(1280, 720, 3)
    kps, desc = e(img, m)
    with oracle.variant(X86):
        okps, odesc = oracle.extract(p2, img, m)
    same(kps, desc, okps, odesc)
    e.close()


def test_x86_device_batch(p):
    """The throughput path (resize_tail_kernel for the top levels, the 8-keypoint describe
    waves) in x86 mode."""
    import torch
    from orbslam_mapsave_amd.abi import KEYPOINT_DTYPE
    from orbslam_mapsave_amd.native import ORBextractor
    W, H, n = 640, 480, 16
    imgs = np.stack([synthetic_frame(40 + i, W, H) for i in range(n)])
    e = ORBextractor(1000, 1.2, 8, 32, 7, device=0, max_width=W, max_height=H, max_batch=n)
    e.set_arithmetic(e.ARITH_X86_SIMD)
    cap = e.capacity(W, H)
    dev = torch.device("cuda", 0)
    d_img = torch.from_numpy(imgs).to(dev)
    d_kps = torch.zeros((n, cap * 28), dtype=torch.uint8, device=dev)
    d_desc = torch.zeros((n, cap, 32), dtype=torch.uint8, device=dev)
    d_n = torch.zeros(n, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    e.extract_batch_device(d_img.data_ptr(), n, W, H, W, W * H, d_kps.data_ptr(), cap,
                           d_desc.data_ptr(), d_n.data_ptr())
    e.synchronize()
    for i in range(n):
        with oracle.variant(X86):
            okps, odesc = oracle.extract(p, imgs[i])
        c = int(d_n[i])
        same(d_kps[i].cpu().numpy().view(KEYPOINT_DTYPE)[:c], d_desc[i, :c].cpu().numpy(),
             okps, odesc)
    e.close()


def test_mode_switch_keeps_single_frame_graph_honest(p):
    """scalar -> x86 -> scalar on one handle (the single-frame graph is re-captured)."""
    from orbslam_mapsave_amd.native import ORBextractor
    e = ORBextractor(1000, 1.2, 8, 32, 7, device=0, max_width=640, max_height=480)
    img = synthetic_frame(9, 640, 480)
    for mode, var in ((0, 0), (1, X86), (0, 0), (1, X86)):
        e.set_arithmetic(mode)
        for _ in range(2):  # capture, then replay
            kps, desc = e(img)
            with oracle.variant(var):
                okps, odesc = oracle.extract(p, img)
            same(kps, desc, okps, odesc)
    e.close()


def test_x86_preblur_path(p, monkeypatch):
    """ORBFE_PREBLUR=1 in x86 mode: blur_mfma_kernel<true> (half-to-even column rounding on the
    SIMD body) feeding the pre-blurred describe, batch and single frame, against the oracle's
    x86 reading."""
    from orbslam_mapsave_amd.native import ORBextractor
    monkeypatch.setenv("ORBFE_PREBLUR", "1")
    e = ORBextractor(1000, 1.2, 8, 32, 7, device=0, max_width=643, max_height=481)
    e.set_arithmetic(e.ARITH_X86_SIMD)
    try:
        imgs = np.stack([synthetic_frame(40 + s, 643, 481) for s in range(2)])
        kps, desc, cnt = e.extract_batch(imgs)
        for f in range(2):
            with oracle.variant(X86):
                okps, odesc = oracle.extract(p, imgs[f])
            same(kps[f, :cnt[f]], desc[f, :cnt[f]], okps, odesc)
        k1, d1 = e(imgs[1])
        with oracle.variant(X86):
            okps, odesc = oracle.extract(p, imgs[1])
        same(k1, d1, okps, odesc)
    finally:
        e.close()
