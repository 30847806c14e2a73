"""The C-ABI library loads and exports every symbol include/orbfe.h declares; the ctypes mirrors
match the C layout; without a usable gfx950 device the product fails loudly (no CPU
fallback).  No compute calls: this runs in the CPU container."""
import ctypes as C
import os
import re

import pytest

from orbslam_mapsave_amd import abi, native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    txt = open(os.path.join(ROOT, "include", "orbfe.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(orbfe_[a-z_0-9]+)\s*\(", txt)))


def test_header_matches_binding_list():
    assert header_functions() == sorted(native.EXPORTED)


def test_library_exports_every_symbol():
    lib = native.lib()
    missing = [f for f in header_functions() if not hasattr(lib, f)]
    assert not missing, missing


def test_oracle_exports_mirror():
    import oracle
    L = oracle.lib()
    for f in ("extract", "extract_batch", "hamming", "bf_match", "search_for_initialization",
              "search_by_projection_local", "search_by_projection_last", "is_in_frustum"):
        assert hasattr(L, "oracle_" + f)


def test_struct_layouts():
    assert C.sizeof(abi.Keypoint) == 28  # cv::KeyPoint
    assert C.sizeof(abi.Params) == 20
    assert C.sizeof(abi.Camera) == 24
    assert abi.FrameView.scale_factors.offset == 56 and C.sizeof(abi.FrameView) == 72
    assert C.sizeof(abi.MapPointView) == 80


def _has_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.mark.skipif(_has_gpu(), reason="checks the no-GPU failure path")
def test_no_gpu_fails_loudly():
    with pytest.raises(abi.OrbfeError) as e:
        native.ORBextractor(1000, 1.2, 8, 32, 7)
    assert e.value.status == abi.ORBFE_ERR_HIP
    with pytest.raises(abi.OrbfeError):
        native.ORBmatcher(0.9, True)


def test_null_and_bad_arguments_do_not_crash():
    lib = native.lib()
    assert lib.orbfe_get_levels(None) == abi.ORBFE_ERR_ARG
    assert lib.orbfe_extract(None, None, 0, 0, C.c_size_t(0), None, C.c_size_t(0), None, 0,
                             None, None) == abi.ORBFE_ERR_ARG
    st = C.c_int(0)
    p = abi.Params(1000, 1.0, 8, 20, 7)  # scaleFactor must exceed 1
    assert not lib.orbfe_create(C.byref(p), 0, 0, 0, 0, C.byref(st))
    assert st.value in (abi.ORBFE_ERR_ARG, abi.ORBFE_ERR_HIP)
    assert lib.orbfe_hamming(None, None, None, -1, None) == abi.ORBFE_ERR_ARG


@pytest.mark.parametrize("nf,sf,nl,w,h", [(2000, 1.2, 8, 1920, 1080), (1000, 1.2, 8, 640, 480),
                                          (1000, 1.5, 4, 1280, 720), (500, 1.2, 8, 3000, 300)])
def test_keypoint_capacity_params_host_only(nf, sf, nl, w, h):
    """orbfe_keypoint_capacity_params needs no device (host arithmetic only): the sum over levels
    of the oct-tree output bound max(N_l + 4, 4 nIni_l, 20) (ORBextractor.cc:538-762), restated
    here from the oracle's level sizes and feature budgets (ORBextractor.cc:434-445, 772-775, 542)."""
    import numpy as np
    import oracle
    p = oracle.params(nf, sf, nl, 20, 7)
    lw, lh = oracle.level_sizes(p, w, h)
    nfeat = oracle.tables(p)["nfeat"] if "nfeat" in oracle.tables(p) else None
    if nfeat is None:  # ORBextractor.cc:434-445 in float, as the ctor computes it
        f = np.float32(1.0) / np.float32(sf)
        desired = np.float32(nf) * (np.float32(1) - f) / (np.float32(1) - np.float32(f ** nl))
        nfeat, tot = [], 0
        for _ in range(nl - 1):
            n = int(np.rint(desired))
            nfeat.append(n)
            tot += n
            desired = np.float32(desired * f)
        nfeat.append(max(nf - tot, 0))
    cap = 0
    for l in range(nl):
        bw, bh = int(lw[l]) - 32, int(lh[l]) - 32  # maxBorder - minBorder = size - 16 - 16
        nini = int(round(bw / bh)) if bw >= 30 and bh >= 30 else 0
        cap += max(int(nfeat[l]) + 4, 4 * nini, 20)
    assert native.keypoint_capacity(nf, sf, nl, 20, 7, w, h) == cap
