"""Every surviving path switch of the extractor, forced, against the oracle.

The library reads a few environment switches at handle creation.  Each selects
another kernel or launch shape for the same stage of ORBextractor::operator()
(ORBextractor.cc:1042-1108); none may change a byte of the output.  For every switch this runs
the extraction parity set:
  * 640x480 @1000, scale 1.2, 8 levels (the bench frames): a 9-frame batch and single frames;
  * 1280x720 @1000, scale 1.5, 4 levels: other cell and level geometry (where a removed FAST
    kernel once failed, gpurun_out/fs2 of round 5);
  * 1920x1080 @2000, scale 1.2, 8 levels: >= 1 Mpx (describe's band order, the per-level pyramid);
and compares all 28 bytes of every keypoint and every descriptor with the oracle's.
"""
import numpy as np
import pytest

import oracle
from orbslam_mapsave_amd.synth import synthetic_frame

pytestmark = pytest.mark.gpu

# (name, {env}) — every switch that selects another extraction path
SWITCHES = [
    ("default", {}),
    ("pyr_per_level", {"ORBFE_PYR": "0"}),
    ("pyr_bands_forced", {"ORBFE_PYR": "2"}),
    ("pyr_batch_band", {"ORBFE_PYR_BATCH": "band"}),
    ("pyr_lds_40kb", {"ORBFE_PYR": "2", "ORBFE_PYR_LDS_KB": "40"}),
    ("pyr_small_below_2", {"ORBFE_PYR_SMALL_BELOW": "2"}),
    ("resize_one_level", {"ORBFE_PYR": "0", "ORBFE_RS2": "0"}),
    ("resize_byte_gather", {"ORBFE_PYR": "0", "ORBFE_RESIZE_TABLE": "0"}),
    ("desc_valu_blur", {"ORBFE_DESC_MFMA": "0"}),
    ("desc_grouped", {"ORBFE_DESC_STRIDE": "0"}),
    ("desc_order_output", {"ORBFE_DESC_ORDER": "0"}),
    ("desc_order_bands", {"ORBFE_DESC_ORDER": "2"}),
    ("desc_g16", {"ORBFE_DESC_G16": "1"}),
    ("oct_256", {"ORBFE_OCT_SMALL": "0"}),
    ("preblur", {"ORBFE_PREBLUR": "1"}),
    ("preblur_mask", {"ORBFE_PREBLUR": "1", "ORBFE_PRE_MASK": "fe"}),
    ("no_graph", {"ORBFE_NO_GRAPH": "1"}),
    ("dma_staging", {"ORBFE_ZERO_COPY": "0"}),
]
ALL_ENV = sorted({k for _, env in SWITCHES for k in env} | {"ORBFE_PROBE_AS_EXTRACTED"})

# (name, w, h, nfeatures, scale, levels, iniTh, minTh, batch frames checked against the oracle)
CONFIGS = [
    ("640x480_s1.2_l8", 640, 480, 1000, 1.2, 8, 20, 7, (0, 4, 8)),
    ("1280x720_s1.5_l4", 1280, 720, 1000, 1.5, 4, 20, 7, (0, 8)),
    ("1920x1080_s1.2_l8", 1920, 1080, 2000, 1.2, 8, 20, 7, (0, 7)),
]
_ORACLE = {}


def _frames(cfg):
    name, w, h = cfg[:3]
    n = 9 if w < 1000 or h < 1000 else 8
    return np.stack([synthetic_frame(1000 + 17 * s + w, w, h) for s in range(n)])


def _oracle(cfg, f):
    key = (cfg[0], f)
    if key not in _ORACLE:
        _, w, h, nf, sf, nl, ini, mn, _ = cfg
        _ORACLE[key] = oracle.extract(oracle.params(nf, sf, nl, ini, mn), _frames(cfg)[f])
    return _ORACLE[key]


def _same(kps, desc, okps, odesc, what):
    assert len(kps) == len(okps), (what, len(kps), len(okps))
    k8 = kps.view(np.uint8).reshape(len(kps), 28)
    o8 = okps.view(np.uint8).reshape(len(okps), 28)
    bad = np.nonzero((k8 != o8).any(axis=1))[0]
    assert bad.size == 0, f"{what}: {bad.size} keypoints differ, first {kps[bad[0]]} vs {okps[bad[0]]}"
    assert np.array_equal(desc, odesc), f"{what}: {(desc != odesc).any(axis=1).sum()} descriptors differ"


@pytest.mark.parametrize("cfg", CONFIGS, ids=[c[0] for c in CONFIGS])
@pytest.mark.parametrize("name,env", SWITCHES, ids=[s[0] for s in SWITCHES])
def test_forced_path_extraction(name, env, cfg, monkeypatch):
    from orbslam_mapsave_amd.native import ORBextractor
    for k in ALL_ENV:
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    _, w, h, nf, sf, nl, ini, mn, check = cfg
    imgs = _frames(cfg)
    e = ORBextractor(nf, sf, nl, ini, mn, device=0, max_width=w, max_height=h)
    try:
        kps, desc, cnt = e.extract_batch(imgs)
        for f in check:
            okps, odesc = _oracle(cfg, f)
            _same(kps[f, :cnt[f]], desc[f, :cnt[f]], okps, odesc, f"{name} batch frame {f}")
        # the single-frame host call (Frame::ExtractORB's form: graph / zero-copy staging), twice
        for f in check[:2]:
            k1, d1 = e(imgs[f])
            okps, odesc = _oracle(cfg, f)
            _same(k1, d1, okps, odesc, f"{name} single frame {f}")
    finally:
        e.close()


@pytest.mark.parametrize("arith", ["scalar", "x86"])
def test_preblur_probe_as_extracted(arith, monkeypatch):
    """ORBFE_PREBLUR=1 with ORBFE_PROBE_AS_EXTRACTED=1: the blurred slab the extraction itself
    wrote (not a K4 pass on demand) equals the oracle's GaussianBlur of every level
    (ORBextractor.cc:1088-1089), batch and single frame, in both arithmetic readings."""
    from orbslam_mapsave_amd.native import ORBextractor
    for k in ALL_ENV:
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("ORBFE_PREBLUR", "1")
    monkeypatch.setenv("ORBFE_PROBE_AS_EXTRACTED", "1")
    x86 = oracle.VAR_H4_FMA | oracle.VAR_H5_SSE2 | oracle.VAR_H6_SIMD
    var = x86 if arith == "x86" else 0
    p = oracle.params(1000, 1.2, 8, 20, 7)
    e = ORBextractor(1000, 1.2, 8, 20, 7, device=0, max_width=643, max_height=481)
    e.set_arithmetic(e.ARITH_X86_SIMD if arith == "x86" else e.ARITH_SCALAR)
    try:
        imgs = np.stack([synthetic_frame(60 + s, 643, 481) for s in range(9)])
        for batch in (True, False):
            if batch:
                e.extract_batch(imgs)
            else:
                e(imgs[4])
            for f in ((0, 8) if batch else (0,)):
                img = imgs[f] if batch else imgs[4]
                with oracle.variant(var & oracle.VAR_H5_SSE2):
                    levels = oracle.pyramid(p, img)
                for l, lev in enumerate(levels):
                    with oracle.variant(var & oracle.VAR_H6_SIMD):
                        ob = oracle.gaussian_blur(lev)
                    gb = e.get_blurred_level(l, f)
                    assert np.array_equal(gb, ob), f"batch={batch} frame {f} level {l}: {(gb != ob).sum()} px"
    finally:
        e.close()


def test_stage_mask_split_and_replay(monkeypatch):
    """orbfe_set_stage_mask: a batch extracted in two calls on one handle (pyramid + FAST +
    oct-tree, then describe — bench.py --pipeline's split) equals one full call and the oracle;
    orbfe_debug_replay of single stages (FAST alone, the oct-tree alone, describe alone) leaves
    the handle's state intact, so the next full extraction is still bit-exact."""
    import torch
    from orbslam_mapsave_amd.native import ORBextractor
    for k in ALL_ENV:
        monkeypatch.delenv(k, raising=False)
    cfg = CONFIGS[0]
    _, w, h, nf, sf, nl, ini, mn, check = cfg
    imgs = _frames(cfg)
    B = len(imgs)
    dev = torch.device("cuda", 0)
    e = ORBextractor(nf, sf, nl, ini, mn, device=0, max_width=w, max_height=h, max_batch=B)
    try:
        cap = e.capacity(w, h)
        fr = torch.from_numpy(imgs).to(dev)
        k = torch.zeros((B, cap * 28), dtype=torch.uint8, device=dev)
        d = torch.zeros((B, cap, 32), dtype=torch.uint8, device=dev)
        n = torch.zeros(B, dtype=torch.int32, device=dev)
        e.set_stream(0)

        def extract():
            e.extract_batch_device(fr.data_ptr(), B, w, h, w, w * h, k.data_ptr(), cap, d.data_ptr(),
                                   n.data_ptr())

        def check_all(what):
            torch.cuda.synchronize()
            kk = k.cpu().numpy().view(np.uint8).reshape(B, cap, 28)
            dd, nn = d.cpu().numpy(), n.cpu().numpy()
            from orbslam_mapsave_amd.abi import KEYPOINT_DTYPE
            for f in check:
                okps, odesc = _oracle(cfg, f)
                _same(kk[f, :nn[f]].copy().view(KEYPOINT_DTYPE).reshape(-1), dd[f, :nn[f]], okps, odesc,
                      f"{what} frame {f}")

        e.set_stages(("resize", "fast", "octree"))
        extract()
        e.set_stages(("describe",))
        extract()
        e.set_stages(None)
        check_all("two-call split")
        for st in (("fast",), ("octree",), ("describe",), ("resize",)):
            e.replay(st, 3)
        d.zero_()
        extract()
        check_all("full call after stage replays")
    finally:
        e.close()
