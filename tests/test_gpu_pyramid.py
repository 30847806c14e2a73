"""pyramid_kernel (orbfe_extract.hip): the whole cascaded pyramid (ORBextractor.cc:1110-1135,
cv::resize INTER_LINEAR) in one launch, a horizontal band of every frame per workgroup, each
level made from the previous one in LDS.  Every level of every frame must be byte-exact against
the oracle — band seams (rows recomputed by two bands), thin bands of the top levels, odd
widths, single frames (the small-batch band plan) and batches, both arithmetic readings —
and identical to the per-level kernels (ORBFE_PYR=0).  ORBFE_PYR=2 forces the band kernel
where the default plan would pick the per-level kernels (thin bands at 1080p).  Scale factors whose source columns do
not fit the kernel's 8-byte window fall back to the per-level kernels."""
import numpy as np
import pytest

import oracle
from orbslam_mapsave_amd.synth import synthetic_frame

pytestmark = pytest.mark.gpu


def _levels_exact(e, p, imgs, var):
    for f, img in enumerate(imgs):
        with oracle.variant(var):
            levels = oracle.pyramid(p, img)
        for l, lev in enumerate(levels):
            g = e.get_level(l, f)
            assert g.shape == lev.shape
            bad = np.argwhere(g != lev)
            assert bad.size == 0, f"frame {f} level {l} {lev.shape}: {len(bad)} px differ, first {bad[:4].tolist()}"


@pytest.mark.parametrize("size", [(640, 480), (643, 481), (1920, 1080), (331, 247), (97, 73), (1281, 722)])
@pytest.mark.parametrize("batch", [1, 9])
@pytest.mark.parametrize("arith", ["scalar", "x86"])
def test_levels_bit_exact(size, batch, arith, monkeypatch):
    from orbslam_mapsave_amd.native import ORBextractor
    monkeypatch.setenv("ORBFE_PYR", "2")  # the band kernel at every size (thin bands included)
    w, h = size
    nf = 2000 if w > 1000 else 1000
    p = oracle.params(nf, 1.2, 8, 20, 7)
    e = ORBextractor(nf, 1.2, 8, 20, 7, device=0, max_width=w, max_height=h)
    var = oracle.VAR_H5_SSE2 if arith == "x86" else 0
    e.set_arithmetic(e.ARITH_X86_SIMD if arith == "x86" else e.ARITH_SCALAR)
    try:
        imgs = np.stack([synthetic_frame(3 * w + s, w, h) for s in range(batch)])
        if batch == 1:
            e(imgs[0])
        else:
            e.extract_batch(imgs)
        assert e.pyramid_path(batch) == "bands"
        _levels_exact(e, p, imgs, var)
    finally:
        e.close()


@pytest.mark.parametrize("lds_kb", ["30", "40", "150"])
def test_band_plans(lds_kb, monkeypatch):
    """Other LDS caps -> other band counts (more seams, or one band per frame half)."""
    from orbslam_mapsave_amd.native import ORBextractor
    monkeypatch.setenv("ORBFE_PYR_LDS_KB", lds_kb)
    monkeypatch.setenv("ORBFE_PYR", "2")
    p = oracle.params(1000, 1.2, 8, 20, 7)
    e = ORBextractor(1000, 1.2, 8, 20, 7, device=0, max_width=640, max_height=480)
    try:
        imgs = np.stack([synthetic_frame(90 + s, 640, 480) for s in range(8)])
        kps, desc, cnt = e.extract_batch(imgs)
        assert e.pyramid_path(len(imgs)) == "bands"
        _levels_exact(e, p, imgs, oracle.DEFAULT_VARIANT)
        okps, odesc = oracle.extract(p, imgs[3])
        assert kps[3, :cnt[3]].tobytes() == okps.tobytes()
        assert np.array_equal(desc[3, :cnt[3]], odesc)
    finally:
        e.close()


@pytest.mark.parametrize("size", [(50, 40), (41, 33)])
@pytest.mark.parametrize("arith", ["scalar", "x86"])
def test_narrow_levels_exact(size, arith, monkeypatch):
    """Frames whose top levels are narrower than 16 bytes (50 px: level 7 is 14 px wide): the
    per-level staging (stage_rows16) then rebuilds every chunk from bytes instead of its
    unconditional 16-byte load; levels byte-exact in both readings, batch and single frame."""
    from orbslam_mapsave_amd.native import ORBextractor
    monkeypatch.setenv("ORBFE_PYR", "0")
    w, h = size
    p = oracle.params(200, 1.2, 8, 20, 7)
    e = ORBextractor(200, 1.2, 8, 20, 7, device=0, max_width=w, max_height=h)
    var = oracle.VAR_H5_SSE2 if arith == "x86" else 0
    e.set_arithmetic(e.ARITH_X86_SIMD if arith == "x86" else e.ARITH_SCALAR)
    try:
        imgs = np.stack([synthetic_frame(11 * w + s, w, h) for s in range(9)])
        e.extract_batch(imgs)
        _levels_exact(e, p, imgs[:3], var)
        e(imgs[4])
        _levels_exact(e, p, imgs[4:5], var)
    finally:
        e.close()


@pytest.mark.parametrize("sf,nl", [(1.5, 5), (2.0, 4), (1.1, 10)])
def test_other_scale_factors(sf, nl, monkeypatch):
    """Fallback (or band kernel, where the window fits) for other scale factors."""
    from orbslam_mapsave_amd.native import ORBextractor
    monkeypatch.setenv("ORBFE_PYR", "2")
    p = oracle.params(1000, sf, nl, 20, 7)
    e = ORBextractor(1000, sf, nl, 20, 7, device=0, max_width=640, max_height=480)
    try:
        imgs = np.stack([synthetic_frame(120 + s, 640, 480) for s in range(8)])
        e.extract_batch(imgs)
        _levels_exact(e, p, imgs[:2], oracle.DEFAULT_VARIANT)
    finally:
        e.close()


@pytest.mark.parametrize("size,batch,path,env", [((640, 480), 1, "bands", None), ((640, 480), 9, "per_level", None),
                                                 ((640, 480), 9, "bands", "band"),
                                                 ((1920, 1080), 1, "bands", None), ((1920, 1080), 9, "per_level", None)])
def test_default_paths(size, batch, path, env, monkeypatch):
    """The pyramid path each shape takes by default (the measured choices of DESIGN.md §5e, §5g:
    batches take the per-level kernels, ORBFE_PYR_BATCH=band the band kernel where it plans)."""
    from orbslam_mapsave_amd.native import ORBextractor
    for v in ("ORBFE_PYR", "ORBFE_PYR_BATCH"):
        monkeypatch.delenv(v, raising=False)
    if env:
        monkeypatch.setenv("ORBFE_PYR_BATCH", env)
    w, h = size
    nf = 2000 if w > 1000 else 1000
    e = ORBextractor(nf, 1.2, 8, 20, 7, device=0, max_width=w, max_height=h)
    try:
        imgs = np.stack([synthetic_frame(11 * w + s, w, h) for s in range(batch)])
        e(imgs[0]) if batch == 1 else e.extract_batch(imgs)
        assert e.pyramid_path(batch) == path
    finally:
        e.close()


def test_per_level_path_identical(monkeypatch):
    from orbslam_mapsave_amd.native import ORBextractor
    imgs = np.stack([synthetic_frame(150 + s, 640, 480) for s in range(8)])
    outs = []
    for flag in ("2", "0"):
        monkeypatch.setenv("ORBFE_PYR", flag)
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


@pytest.mark.parametrize("size", [(640, 480), (1920, 1080), (643, 481), (97, 73)])
@pytest.mark.parametrize("arith", ["scalar", "x86"])
@pytest.mark.parametrize("table,rs2", [("1", "1"), ("1", "0"), ("0", "1")])
def test_per_level_kernels_exact(size, arith, table, rs2, monkeypatch):
    """The per-level path (ORBFE_PYR=0; the default for batches): level pairs per launch
    (resize2_kernel, default) or one level per launch (resize_kernel, ORBFE_RS2=0), on the
    column-group tables or with resize_kernel's horizontal pass by byte gathers
    (ORBFE_RESIZE_TABLE=0); the one-workgroup tail for batches; every level byte-exact in both
    readings."""
    from orbslam_mapsave_amd.native import ORBextractor
    monkeypatch.setenv("ORBFE_PYR", "0")
    monkeypatch.setenv("ORBFE_RESIZE_TABLE", table)
    monkeypatch.setenv("ORBFE_RS2", rs2)
    w, h = size
    nf = 2000 if w > 1000 else 1000
    p = oracle.params(nf, 1.2, 8, 20, 7)
    e = ORBextractor(nf, 1.2, 8, 20, 7, device=0, max_width=w, max_height=h)
    var = oracle.VAR_H5_SSE2 if arith == "x86" else 0
    e.set_arithmetic(e.ARITH_X86_SIMD if arith == "x86" else e.ARITH_SCALAR)
    try:
        imgs = np.stack([synthetic_frame(7 * w + s, w, h) for s in range(9)])
        e.extract_batch(imgs)
        assert e.pyramid_path(len(imgs)) == "per_level"
        _levels_exact(e, p, imgs[:3], var)
        e(imgs[4])
        _levels_exact(e, p, imgs[4:5], var)
    finally:
        e.close()
