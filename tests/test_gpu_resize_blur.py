"""resize_blur_kernel (orbfe_extract.hip, K1 + K4 fused; ORBFE_RESIZE_BLUR=1, off by default:
measured slower overall): every level made by a per-level resize launch is also blurred in the same launch (GaussianBlur 7x7 sigma 2 REFLECT_101,
ORBextractor.cc:1088-1089), and describe reads those levels' blurred windows.  The blurred
slab is read back exactly as the extraction left it (ORBFE_PROBE_AS_EXTRACTED=1: no K4 pass
on demand) and compared with the oracle's blur of the oracle's level, every pixel, including
the reflected borders of tiles narrower than 4 px; keypoints and descriptors stay bit-exact.
Single frames take per-level resize launches for levels 1-7; batches of 8+ frames for the
levels below the one-workgroup tail (levels 1-4 at 640x480)."""
import numpy as np
import pytest

import oracle
from orbslam_mapsave_amd.synth import synthetic_frame

pytestmark = pytest.mark.gpu

X86 = oracle.VAR_H4_FMA | oracle.VAR_H5_SSE2 | oracle.VAR_H6_SIMD


def _check(e, p, img, arith_var, levels_made, frame=0):
    with oracle.variant(arith_var & oracle.VAR_H5_SSE2):
        levels = oracle.pyramid(p, img)
    for l in levels_made:
        with oracle.variant(arith_var & oracle.VAR_H6_SIMD):
            ob = oracle.gaussian_blur(levels[l])
        gb = e.get_blurred_level(l, frame)
        assert gb.shape == ob.shape
        bad = np.argwhere(gb != ob)
        assert bad.size == 0, f"level {l} {ob.shape}: {len(bad)} px differ, first {bad[:4].tolist()}"


# (769, 97): level 1 is 641 px wide, its last 128-px tile one column wide
@pytest.mark.parametrize("size", [(640, 480), (769, 97), (643, 481), (1920, 1080), (333, 257), (130, 66)])
@pytest.mark.parametrize("arith", ["scalar", "x86"])
def test_single_frame_levels(size, arith, monkeypatch):
    from orbslam_mapsave_amd.native import ORBextractor
    monkeypatch.setenv("ORBFE_PROBE_AS_EXTRACTED", "1")
    monkeypatch.setenv("ORBFE_RESIZE_BLUR", "1")
    w, h = size
    nf = 2000 if w > 1000 else 1000
    p = oracle.params(nf, 1.2, 8, 20, 7)
    e = ORBextractor(nf, 1.2, 8, 20, 7, device=0, max_width=w, max_height=h)
    var = X86 if arith == "x86" else 0
    e.set_arithmetic(e.ARITH_X86_SIMD if arith == "x86" else e.ARITH_SCALAR)
    try:
        img = synthetic_frame(w + h, w, h)
        kps, desc = e(img)
        _check(e, p, img, var, range(1, 8))
        with oracle.variant(var):
            okps, odesc = oracle.extract(p, img)
        assert kps.tobytes() == okps.tobytes()
        assert np.array_equal(desc, odesc)
    finally:
        e.close()


@pytest.mark.parametrize("arith", ["scalar", "x86"])
def test_batch_levels(arith, monkeypatch):
    from orbslam_mapsave_amd.native import ORBextractor
    monkeypatch.setenv("ORBFE_PROBE_AS_EXTRACTED", "1")
    monkeypatch.setenv("ORBFE_RESIZE_BLUR", "1")
    p = oracle.params(1000, 1.2, 8, 20, 7)
    e = ORBextractor(1000, 1.2, 8, 20, 7, device=0, max_width=640, max_height=480)
    var = X86 if arith == "x86" else 0
    e.set_arithmetic(e.ARITH_X86_SIMD if arith == "x86" else e.ARITH_SCALAR)
    try:
        imgs = np.stack([synthetic_frame(40 + s, 640, 480) for s in range(9)])
        kps, desc, cnt = e.extract_batch(imgs)
        for f in (0, 4, 8):
            _check(e, p, imgs[f], var, range(1, 5), frame=f)
            with oracle.variant(var):
                okps, odesc = oracle.extract(p, imgs[f])
            assert kps[f, :cnt[f]].tobytes() == okps.tobytes()
            assert np.array_equal(desc[f, :cnt[f]], odesc)
    finally:
        e.close()


def test_resize_blur_off_is_identical(monkeypatch):
    """ORBFE_RESIZE_BLUR=1 and 0 (every window blurred inside describe) give the same outputs."""
    from orbslam_mapsave_amd.native import ORBextractor
    imgs = np.stack([synthetic_frame(70 + s, 640, 480) for s in range(8)])
    outs = []
    for flag in ("1", "0"):
        monkeypatch.setenv("ORBFE_RESIZE_BLUR", flag)
        e = ORBextractor(1000, 1.2, 8, 20, 7, device=0, max_width=640, max_height=480)
        try:
            kps, desc, cnt = e.extract_batch(imgs)
            outs.append((kps.copy(), desc.copy(), cnt.copy()))
        finally:
            e.close()
    assert np.array_equal(outs[0][2], outs[1][2])
    for f in range(len(imgs)):
        n = outs[0][2][f]
        assert outs[0][0][f, :n].tobytes() == outs[1][0][f, :n].tobytes()
        assert np.array_equal(outs[0][1][f, :n], outs[1][1][f, :n])
