"""Zero-copy host paths (ORBFE_ZERO_COPY, default on): the single-frame host call
(ORBextractor::operator(), ORBextractor.cc:1042) reads its frame from the pinned staging buffer
inside the pyramid kernel and has describe write keypoints / descriptors / count straight into
the pinned outputs; the host-form matchers scatter their uploads from, and gather their results
into, the device-mapped staging buffer.  Outputs must be identical to the DMA path
(ORBFE_ZERO_COPY=0) and to the oracle, call after call (the staging buffers are reused)."""
import numpy as np
import pytest

import oracle
from orbslam_mapsave_amd.synth import synthetic_frame

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("size", [(640, 480), (1920, 1080), (331, 247)])
def test_single_frame_zero_copy(size, monkeypatch):
    from orbslam_mapsave_amd.native import ORBextractor
    w, h = size
    nf = 2000 if w > 1000 else 1000
    p = oracle.params(nf, 1.2, 8, 20, 7)
    imgs = [synthetic_frame(500 + s, w, h) for s in range(3)]
    res = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("ORBFE_ZERO_COPY", flag)
        e = ORBextractor(nf, 1.2, 8, 20, 7, device=0, max_width=w, max_height=h)
        try:
            res[flag] = [tuple(x.copy() for x in e(img)) for img in imgs + imgs[:1]]
            assert np.array_equal(e.get_level(0), imgs[0])  # level 0 reached the slab
        finally:
            e.close()
    for (k1, d1), (k0, d0) in zip(res["1"], res["0"]):
        assert k1.tobytes() == k0.tobytes()
        assert np.array_equal(d1, d0)
    for img, (k, d) in zip(imgs, res["1"]):
        ok, od = oracle.extract(p, img)
        assert k.tobytes() == ok.tobytes()
        assert np.array_equal(d, od)


def test_matcher_zero_copy(monkeypatch):
    import scenarios as S
    from orbslam_mapsave_amd.native import ORBmatcher
    c = S.sbp_keyframe_case(0)
    outs = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("ORBFE_ZERO_COPY", flag)
        m = ORBmatcher(0.9, True, device=0)
        try:
            outs[flag] = [m.SearchByProjectionKeyFrame(c["cur"], c["tcw_cur"], c["cam"], c["log_scale"],
                                                       c["kf_angle"], c["kf_valid"], c["kf_bad"], c["found"],
                                                       c["kf_xyz"], c["kf_desc"], c["kf_min"], c["kf_max"], 10, 100,
                                                       frame_mp=c["frame_mp"].copy(), kf_ids=c["kf_ids"])
                          for _ in range(3)]
        finally:
            m.close()
    rfmp, rnm = oracle.search_by_projection_keyframe(c, 10, 100)
    for (f1, n1), (f0, n0) in zip(outs["1"], outs["0"]):
        assert n1 == n0 and np.array_equal(f1, f0)
    assert outs["1"][0][1] == rnm and np.array_equal(outs["1"][0][0], rfmp)


@pytest.mark.parametrize("size", [(640, 480), (1920, 1080), (331, 247)])
def test_staged_input_buffer(size):
    """orbfe_input_buffer / orbfe_extract_staged / orbfe_staged_outputs (the zero-copy form of
    Frame::ExtractORB, Frame.cc:358-364): the caller writes each frame into the handle's pinned
    staging buffer (as GrabImageMonocular's cvtColor would, Tracking.cc:409-422); results are
    identical to orbfe_extract and to the oracle, call after call, copied out or left in the
    handle's pinned outputs."""
    from orbslam_mapsave_amd.native import ORBextractor
    w, h = size
    nf = 2000 if w > 1000 else 1000
    p = oracle.params(nf, 1.2, 8, 20, 7)
    imgs = [synthetic_frame(700 + s, w, h) for s in range(3)]
    e = ORBextractor(nf, 1.2, 8, 20, 7, device=0, max_width=w, max_height=h)
    try:
        for i, img in enumerate(imgs + imgs[:1]):
            buf = e.input_buffer(w, h)
            assert buf.shape == (h, w) and buf.flags["WRITEABLE"]
            buf[:] = img
            ok, od = oracle.extract(p, img)
            if i % 2 == 0:
                k, d = e.extract_staged(w, h)
            else:  # outputs left in the pinned buffers
                kv, dv = e.extract_staged(w, h, copy_out=False)
                k, d = kv.copy(), dv.copy()
            assert k.tobytes() == ok.tobytes()
            assert np.array_equal(d, od)
            k2, d2 = e(img)  # the copying form agrees
            assert k2.tobytes() == k.tobytes() and np.array_equal(d2, d)
            ks, ds = e.staged_outputs()  # the last single-frame call's outputs
            assert ks.tobytes() == k.tobytes() and np.array_equal(ds, d)
    finally:
        e.close()


def test_staged_requires_buffer():
    from orbslam_mapsave_amd.abi import OrbfeError
    from orbslam_mapsave_amd.native import ORBextractor
    e = ORBextractor(1000, 1.2, 8, 20, 7, device=0)
    try:
        with pytest.raises(OrbfeError):
            e.extract_staged(640, 480)  # no staging buffer handed out yet
        e.input_buffer(320, 240)
        with pytest.raises(OrbfeError):
            e.extract_staged(640, 480)  # the buffer handed out is smaller than the frame
    finally:
        e.close()


def test_staged_buffer_survives_copying_calls():
    """The handed-out buffer is not the copy staging: orbfe_extract calls of the same and of a
    larger size between orbfe_input_buffer and orbfe_extract_staged neither move it nor
    overwrite the frame staged in it."""
    from orbslam_mapsave_amd.native import ORBextractor
    p = oracle.params(1000, 1.2, 8, 20, 7)
    small, big = synthetic_frame(811, 640, 480), synthetic_frame(812, 960, 720)
    other = synthetic_frame(813, 640, 480)
    e = ORBextractor(1000, 1.2, 8, 20, 7, device=0, max_width=960, max_height=720)
    try:
        buf = e.input_buffer(640, 480)
        addr = buf.ctypes.data
        buf[:] = small
        e(other)   # same size, copying form
        e(big)     # larger frame, copying form
        buf2 = e.input_buffer(640, 480)
        assert buf2.ctypes.data == addr and np.array_equal(buf2, small)
        k, d = e.extract_staged(640, 480)
        ok, od = oracle.extract(p, small)
        assert k.tobytes() == ok.tobytes() and np.array_equal(d, od)
    finally:
        e.close()


def test_staged_after_copying_call_requires_buffer():
    """A copying orbfe_extract does not count as a handed-out buffer."""
    from orbslam_mapsave_amd.abi import OrbfeError
    from orbslam_mapsave_amd.native import ORBextractor
    e = ORBextractor(1000, 1.2, 8, 20, 7, device=0)
    try:
        e(synthetic_frame(814, 640, 480))
        with pytest.raises(OrbfeError):
            e.extract_staged(640, 480)
    finally:
        e.close()
