"""§8(f) row 4 (data format) — the map-archive records of the extractor outputs: keypoints as
serialize(Archive&, cv::KeyPoint&) writes them (MapPoint.h:196-209) and descriptors as cv::Mat
save / load records (MapPoint.h:215-247), produced from and read back into HBM by
orbfe_archive_*_device.

CPU: the numpy restatement (oracle/archive.py) against hand-built known answers (struct).
GPU: a batch of frames extracted on the device is archived on the device; the bytes equal the
restatement's, and reading them back restores the keypoints (size 0, as the reference's load
leaves it) and descriptors; map-point descriptors (1 x 32 records); corrupt headers are
rejected.  Parity is against the cited source lines: the reference holds no archive file.
"""
import struct

import numpy as np
import pytest

import scenarios as S
from oracle import archive as A
from orbslam_mapsave_amd import native
from orbslam_mapsave_amd.abi import KEYPOINT_DTYPE


def test_keypoint_record_known_answer():
    k = np.zeros(2, KEYPOINT_DTYPE)
    k[0] = (10.5, 20.25, 31.0, 123.5, 0.75, 3, -1)
    k[1] = (1.0, 2.0, 37.2, -1.0, 17.0, 0, 5)
    want = (struct.pack("<fiiffff", 123.5, -1, 3, 0.75, 0.75, 10.5, 20.25) +
            struct.pack("<fiiffff", -1.0, 5, 0, 17.0, 17.0, 1.0, 2.0))
    got = A.keypoints_bytes(k)
    assert got == want and len(got) == 56
    back = A.keypoints_from_bytes(got, 2)
    assert back["size"].tolist() == [0.0, 0.0]
    for f in ("x", "y", "angle", "response", "octave", "class_id"):
        assert np.array_equal(back[f], k[f])


def test_mat_record_known_answer():
    d = np.arange(3 * 32, dtype=np.uint8).reshape(3, 32)
    b = A.mat_bytes(d)
    assert b[:24] == struct.pack("<iiQQ", 32, 3, 1, 0) and b[24:] == d.tobytes()
    assert A.mat_from_bytes(b) == (3, 32, 1, 0, d.tobytes())
    assert native.archive_mat_bytes(3, 32, 1) == len(b) == 24 + 96
    assert native.archive_mat_bytes(0, 32, 1) == 24
    assert native.archive_mat_bytes(-1, 32, 1) == -1


@pytest.mark.gpu
def test_gpu_archive_extracted_frames():
    import torch
    from orbslam_mapsave_amd.native import ORBextractor
    from orbslam_mapsave_amd.synth import synthetic_frame
    dev = torch.device("cuda", 0)
    W, H, B = S.W, S.H, 3
    ex = ORBextractor(1000, 1.2, 8, 20, 7, device=0)
    cap = ex.capacity(W, H)
    imgs = np.stack([synthetic_frame(s, W, H) for s in range(B)])
    D = torch.from_numpy(imgs).to(dev)
    kps = torch.zeros((B, cap * 28), dtype=torch.uint8, device=dev)
    desc = torch.zeros((B, cap, 32), dtype=torch.uint8, device=dev)
    n = torch.zeros(B, dtype=torch.int32, device=dev)
    ex.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    ex.extract_batch_device(D.data_ptr(), B, W, H, W, W * H, kps.data_ptr(), cap, desc.data_ptr(),
                            n.data_ptr())
    ex.synchronize()  # the extractor runs on its own stream (torch's default stream is NULL)
    s = torch.cuda.current_stream(dev).cuda_stream
    kp_pitch = cap * 28
    mat_pitch = (native.archive_mat_bytes(cap) + 7) // 8 * 8
    ko = torch.full((B, kp_pitch), 0xAB, dtype=torch.uint8, device=dev)
    mo = torch.full((B, mat_pitch), 0xAB, dtype=torch.uint8, device=dev)
    ln = torch.zeros(B, dtype=torch.int64, device=dev)
    native.archive_write_keypoints_device(B, kps.data_ptr(), cap, n.data_ptr(), cap, ko.data_ptr(),
                                          kp_pitch, s)
    native.archive_write_descriptors_device(B, desc.data_ptr(), cap * 32, n.data_ptr(), 0, cap,
                                            mo.data_ptr(), mat_pitch, ln.data_ptr(), s)
    # read back into fresh buffers
    k2 = torch.zeros_like(kps)
    d2 = torch.zeros_like(desc)
    rows = torch.zeros(B, dtype=torch.int32, device=dev)
    st = torch.full((1,), 9, dtype=torch.int32, device=dev)
    native.archive_read_keypoints_device(B, ko.data_ptr(), kp_pitch, n.data_ptr(), cap,
                                         k2.data_ptr(), cap, s)
    native.archive_read_descriptors_device(B, mo.data_ptr(), mat_pitch, cap, d2.data_ptr(),
                                           cap * 32, rows.data_ptr(), st.data_ptr(), s)
    torch.cuda.synchronize()
    nh = n.cpu().numpy()
    assert int(st[0]) == 0 and rows.cpu().numpy().tolist() == nh.tolist()
    K = kps.cpu().numpy()
    for f in range(B):
        nf = int(nh[f])
        assert nf > 500
        keys = K[f, :nf * 28].view(KEYPOINT_DTYPE)
        dsc = desc[f, :nf].cpu().numpy()
        assert ko[f, :nf * 28].cpu().numpy().tobytes() == A.keypoints_bytes(keys)
        want = A.mat_bytes(dsc)
        assert int(ln[f]) == len(want)
        assert mo[f, :len(want)].cpu().numpy().tobytes() == want
        back = k2[f, :nf * 28].cpu().numpy().view(KEYPOINT_DTYPE)
        ref = A.keypoints_from_bytes(A.keypoints_bytes(keys), nf)
        assert back.tobytes() == ref.tobytes()
        assert np.array_equal(d2[f, :nf].cpu().numpy(), dsc)
    ex.close()


@pytest.mark.gpu
def test_gpu_archive_mappoint_descriptors_and_bad_headers():
    """MapPoint::mDescriptor: one 1 x 32 record per map point (MapPoint.cc:121); a record whose
    header is not a CV_8UC1 32-column Mat within capacity is refused."""
    import torch
    dev = torch.device("cuda", 0)
    rng = np.random.Generator(np.random.PCG64(3))
    M = 5000
    dsc = rng.integers(0, 256, (M, 32), dtype=np.uint8)
    D = torch.from_numpy(dsc).to(dev)
    rec = native.archive_mat_bytes(1)
    pitch = (rec + 7) // 8 * 8  # 56
    out = torch.zeros((M, pitch), dtype=torch.uint8, device=dev)
    native.archive_write_descriptors_device(M, D.data_ptr(), 32, None, 1, 1, out.data_ptr(), pitch)
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    for i in (0, 1, 77, M - 1):
        assert o[i, :rec].tobytes() == A.mat_bytes(dsc[i:i + 1])
    bad = o.copy()
    bad[3, 0] = 31                               # cols 31
    bad[4, 8] = 4                                # elemSize 4
    bad[5, 16] = 5                               # type CV_32F
    bad[6, 4:8] = np.frombuffer(struct.pack("<i", 2), np.uint8)  # rows 2 > cap 1
    B_ = torch.from_numpy(bad).to(dev)
    back = torch.zeros((M, 32), dtype=torch.uint8, device=dev)
    rows = torch.zeros(M, dtype=torch.int32, device=dev)
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    native.archive_read_descriptors_device(M, B_.data_ptr(), pitch, 1, back.data_ptr(), 32,
                                           rows.data_ptr(), st.data_ptr())
    torch.cuda.synchronize()
    r = rows.cpu().numpy()
    assert int(st[0]) == -1
    assert r[3:7].tolist() == [-1] * 4 and (np.delete(r, [3, 4, 5, 6]) == 1).all()
    b = back.cpu().numpy()
    keep = np.ones(M, bool)
    keep[3:7] = False
    assert np.array_equal(b[keep], dsc[keep]) and not b[3:7].any()
