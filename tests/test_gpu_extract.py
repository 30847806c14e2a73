"""GPU parity of the extractor (liborbfe.so through the C ABI) against the CPU oracle.

Bar (DESIGN.md "Parity"): every stage is integer/byte/index work or float work evaluated in
the reference's exact operation order, so every comparison here is bit-exact: pyramid levels,
per-level FAST candidates (vToDistributeKeys), blurred levels, final keypoints (all 28 bytes
including the float angle) and 32-byte descriptors.
"""
import numpy as np
import pytest

import oracle
from orbslam_mapsave_amd.synth import synthetic_frame, synthetic_mask

pytestmark = pytest.mark.gpu

CFG = dict(nfeatures=1000, scale_factor=1.2, nlevels=8, ini_th=32, min_th=7)


@pytest.fixture(scope="module")
def ex():
    from orbslam_mapsave_amd.native import ORBextractor
    e = ORBextractor(1000, 1.2, 8, 32, 7, device=0, max_width=640, max_height=480)
    yield e
    e.close()


@pytest.fixture(scope="module")
def p():
    return oracle.params(**CFG)


def _assert_same_keys(k, ok):
    assert len(k) == len(ok), (len(k), len(ok))
    if len(k):
        bad = np.nonzero(k.view(np.uint8).reshape(len(k), 28) != ok.view(np.uint8).reshape(len(ok), 28))[0]
        assert bad.size == 0, f"{np.unique(bad).size} keypoints differ, first {k[bad[0]]} vs {ok[bad[0]]}"


@pytest.mark.parametrize("seed", range(5))
def test_pyramid_fast_blur_stages(ex, p, seed):
    img = synthetic_frame(seed, 640, 480)
    ex(img)
    levels = oracle.pyramid(p, img)
    for l, lev in enumerate(levels):
        g = ex.get_level(l)
        assert g.shape == lev.shape
        assert np.array_equal(g, lev), f"level {l}: {(g != lev).sum()} pixels differ"
        assert np.array_equal(ex.get_blurred_level(l), oracle.gaussian_blur(lev)), f"blur {l}"
        fk = ex.get_fast_keys(l)
        ofk = oracle.fast_keys(p, lev)
        _assert_same_keys(fk, ofk)


@pytest.mark.parametrize("seed", range(5))
def test_extract_bit_exact(ex, p, seed):
    img = synthetic_frame(seed, 640, 480)
    kps, desc = ex(img)
    okps, odesc = oracle.extract(p, img)
    _assert_same_keys(kps, okps)
    assert np.array_equal(desc, odesc)


@pytest.mark.parametrize("kind", ["low_contrast", "constant"])
def test_edge_images(ex, p, kind):
    img = synthetic_frame(7, 640, 480, kind=kind)
    kps, desc = ex(img)
    okps, odesc = oracle.extract(p, img)
    _assert_same_keys(kps, okps)
    assert np.array_equal(desc, odesc)
    if kind == "constant":
        assert len(kps) == 0


def test_masked(ex, p):
    img = synthetic_frame(3, 640, 480)
    m = synthetic_mask(640, 480, 3)
    kps, desc = ex(img, m)
    okps, odesc = oracle.extract(p, img, m)
    _assert_same_keys(kps, okps)
    assert np.array_equal(desc, odesc)


def test_batch_matches_single(ex, p):
    imgs = np.stack([synthetic_frame(s, 640, 480) for s in range(4)])
    kps, desc, cnt = ex.extract_batch(imgs)
    for f in range(4):
        okps, odesc = oracle.extract(p, imgs[f])
        _assert_same_keys(kps[f, :cnt[f]], okps)
        assert np.array_equal(desc[f, :cnt[f]], odesc)


@pytest.mark.parametrize("order,stride,g16", [("0", "1", "0"), ("1", "1", "0"), ("2", "1", "0"), ("2", "0", "0"),
                                            ("1", "1", "1"), ("2", "1", "1")])
def test_describe_slot_orders(p, order, stride, g16, monkeypatch):
    """describe's wave-to-keypoint assignment in batches (>= 8 frames): strided slots in the
    oct-tree's output order (ORBFE_DESC_ORDER=0), in its 32-row band order (2: at every size;
    1, the default: frames of >= 1 Mpx only) or grouped slots (ORBFE_DESC_STRIDE=0, the band
    order then unused), 8 or 16 (ORBFE_DESC_G16=1) keypoints per wave — the processing order
    never changes the outputs or their order."""
    from orbslam_mapsave_amd.native import ORBextractor
    monkeypatch.setenv("ORBFE_DESC_ORDER", order)
    monkeypatch.setenv("ORBFE_DESC_STRIDE", stride)
    monkeypatch.setenv("ORBFE_DESC_G16", g16)
    e = ORBextractor(1000, 1.2, 8, 32, 7, device=0, max_width=640, max_height=480)
    try:
        imgs = np.stack([synthetic_frame(40 + s, 640, 480) for s in range(9)])
        kps, desc, cnt = e.extract_batch(imgs)
        for f in (0, 4, 8):
            okps, odesc = oracle.extract(p, imgs[f])
            _assert_same_keys(kps[f, :cnt[f]], okps)
            assert np.array_equal(desc[f, :cnt[f]], odesc)
    finally:
        e.close()


def test_describe_band_order_1080p():
    """The default at >= 1 Mpx: describe's strided waves take the oct-tree's 32-row band order
    (batches of >= 8 frames) — keypoints and descriptors of a 1920 x 1080 batch identical to the
    oracle's, in the output order."""
    from orbslam_mapsave_amd.native import ORBextractor
    p2 = oracle.params(2000, 1.2, 8, 20, 7)
    e = ORBextractor(2000, 1.2, 8, 20, 7, device=0, max_width=1920, max_height=1080)
    try:
        imgs = np.stack([synthetic_frame(60 + s, 1920, 1080) for s in range(8)])
        kps, desc, cnt = e.extract_batch(imgs)
        for f in (0, 7):
            okps, odesc = oracle.extract(p2, imgs[f])
            _assert_same_keys(kps[f, :cnt[f]], okps)
            assert np.array_equal(desc[f, :cnt[f]], odesc)
    finally:
        e.close()


def test_profile_stage_mask(ex, p):
    """orbfe_profile: events on every launch, or on the masked stages' launches only (bench.py's
    timed steps); results stay bit-exact either way."""
    imgs = np.stack([synthetic_frame(s, 640, 480) for s in range(2)])
    okps, odesc = oracle.extract(p, imgs[1])
    ex.profile(True)
    ex.profile_read()
    kps, desc, cnt = ex.extract_batch(imgs)
    every = ex.profile_read()
    ex.profile(True, stages=("fast", "describe"))
    kps2, desc2, cnt2 = ex.extract_batch(imgs)
    masked = ex.profile_read()
    ex.profile(False)
    for st in ("resize", "fast", "octree", "describe"):
        assert every[st][1] >= 1 and every[st][0] > 0, (st, every)
    assert masked["fast"][1] == every["fast"][1] and masked["describe"][1] == every["describe"][1]
    assert all(masked[st][1] == 0 for st in ("mask", "resize", "octree", "blur")), masked
    _assert_same_keys(kps[1, :cnt[1]], okps)
    _assert_same_keys(kps2[1, :cnt2[1]], okps)
    assert np.array_equal(desc[1, :cnt[1]], odesc) and np.array_equal(desc2[1, :cnt2[1]], odesc)


@pytest.mark.parametrize("cfg", [(2000, 1.2, 8, 32, 7, 640, 480), (2000, 1.2, 8, 20, 7, 1920, 1080),
                                 (500, 1.5, 4, 20, 7, 1280, 720), (1000, 1.2, 8, 32, 7, 752, 480)])
def test_other_configs(cfg):
    from orbslam_mapsave_amd.native import ORBextractor
    nf, sf, nl, ini, mn, w, h = cfg
    e = ORBextractor(nf, sf, nl, ini, mn, device=0, max_width=w, max_height=h)
    pp = oracle.params(nf, sf, nl, ini, mn)
    img = synthetic_frame(11, w, h)
    kps, desc = e(img)
    okps, odesc = oracle.extract(pp, img)
    _assert_same_keys(kps, okps)
    assert np.array_equal(desc, odesc)
    e.close()


@pytest.mark.parametrize("w,h", [(641, 479), (333, 257), (200, 170), (1024, 1024), (1600, 480),
                                 (2048, 512), (3000, 300)])
def test_odd_sizes(w, h):
    """Ragged sizes (odd widths / heights, levels whose rows are not multiples of 4, square and
    wide frames: nIni = round(w / h) from 1 to 20, ORBextractor.cc:542), against the oracle."""
    from orbslam_mapsave_amd.native import ORBextractor
    e = ORBextractor(1000, 1.2, 8, 20, 7, device=0, max_width=w, max_height=h)
    pp = oracle.params(1000, 1.2, 8, 20, 7)
    img = synthetic_frame(w + h, w, h)
    kps, desc = e(img)
    okps, odesc = oracle.extract(pp, img)
    _assert_same_keys(kps, okps)
    assert np.array_equal(desc, odesc)
    e.close()


def test_strided_roi(ex, p):
    """A cv::Mat ROI (row step > cols) is read in place through the stride argument."""
    big = synthetic_frame(21, 700, 520)
    view = big[17:497, 31:671]
    assert view.strides[0] == 700
    kps, desc = ex(view)
    okps, odesc = oracle.extract(p, np.ascontiguousarray(view))
    _assert_same_keys(kps, okps)
    assert np.array_equal(desc, odesc)


def test_unsupported_inputs_are_refused():
    """Frames above 4096 px (the workspace plan) fail loudly with
    ORBFE_ERR_UNSUPPORTED, never silently."""
    from orbslam_mapsave_amd.abi import ORBFE_ERR_UNSUPPORTED, OrbfeError
    from orbslam_mapsave_amd.native import ORBextractor
    e = ORBextractor(1000, 1.2, 8, 20, 7, device=0)
    for shape in ((200, 4100), (4100, 300)):
        with pytest.raises(OrbfeError) as ei:
            e(np.zeros(shape, np.uint8))
        assert ei.value.status == ORBFE_ERR_UNSUPPORTED
    e.close()


@pytest.mark.parametrize("size", [(643, 481), (1281, 722), (331, 247), (97, 73), (61, 44), (40, 30)])
def test_blur_levels_odd_sizes(size):
    """K4 (blur_row_kernel) on level widths of every residue mod 4 / mod 8 / mod 16, including
    levels narrower than 16 px or lower than 8 rows (the per-pixel "tiny" slots), against the
    oracle's GaussianBlur 7x7 REFLECT_101 (ORBextractor.cc:1088-1089)."""
    from orbslam_mapsave_amd.native import ORBextractor
    w, h = size
    p = oracle.params(**CFG)
    e = ORBextractor(1000, 1.2, 8, 32, 7, device=0, max_width=w, max_height=h)
    try:
        img = synthetic_frame(11, w, h)
        e(img)
        for l, lev in enumerate(oracle.pyramid(p, img)):
            gb, ob = e.get_blurred_level(l), oracle.gaussian_blur(lev)
            assert gb.shape == ob.shape
            assert np.array_equal(gb, ob), f"{size} level {l} {lev.shape}: {(gb != ob).sum()} px differ"
    finally:
        e.close()


@pytest.mark.parametrize("size", [(640, 480), (643, 481), (1920, 1080), (331, 247)])
def test_preblur_path(size, monkeypatch):
    """ORBFE_PREBLUR=1: K4 over every level (blur_row_kernel), describe reading the blurred
    levels; keypoints and descriptors stay bit-exact against the oracle, batch and single."""
    from orbslam_mapsave_amd.native import ORBextractor
    w, h = size
    monkeypatch.setenv("ORBFE_PREBLUR", "1")
    nf = 2000 if w > 1000 else 1000
    e = ORBextractor(nf, 1.2, 8, 20, 7, device=0, max_width=w, max_height=h)
    pp = oracle.params(nf, 1.2, 8, 20, 7)
    try:
        imgs = np.stack([synthetic_frame(s + w, w, h) for s in range(3)])
        kps, desc, cnt = e.extract_batch(imgs)
        for f in range(3):
            okps, odesc = oracle.extract(pp, imgs[f])
            _assert_same_keys(kps[f, :cnt[f]], okps)
            assert np.array_equal(desc[f, :cnt[f]], odesc)
        k1, d1 = e(imgs[0])
        okps, odesc = oracle.extract(pp, imgs[0])
        _assert_same_keys(k1, okps)
        assert np.array_equal(d1, odesc)
    finally:
        e.close()
