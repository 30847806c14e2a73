"""Parity at the benchmark's full size (BASELINE configs[2], bench.py's default workload): 640x480
frames extracted on the device and every frame brute-force matched against the 2000-keypoint
reference frame, in the launch patterns bench.py runs — 512 frames as two 256-frame sub-batches
on two HIP streams (the timed steps; handle 0 planned for 512 frames, as in bench.py), one
512-frame call on that handle (the probe and roofline legs), and 256 as 2 x 128 — and every frame
compared with the CPU oracle: keypoints (28-byte records), descriptors, and the (best index,
best, second) triple of every query.  64 distinct seeds, each used 4-8 times, so the oracle side
runs in about a second and repeated frames in different sub-batches / streams must also agree
with each other."""
import numpy as np
import pytest

import oracle
from orbslam_mapsave_amd.abi import KEYPOINT_DTYPE

pytestmark = pytest.mark.gpu

S, W, H, NF, NREF, DISTINCT = 2, 640, 480, 1000, 2000, 64

# (frames, sub-batch streams, max_batch of handle 0): 256 as 2 x 128; the bench's timed steps,
# 512 as 2 x 256 on a handle 0 planned for 512 (bench.py run_extract); its probe / roofline legs,
# one 512-frame call on that handle (step_single)
LAYOUTS = {"256_as_2x128": (256, 2, 128), "512_as_2x256": (512, 2, 512), "512_single": (512, 1, 512)}
_EXPECT = {}


def _expected(frames_np, ref_img, ref_desc_np):
    if not _EXPECT:
        _, oref = oracle.extract(oracle.params(NREF, 1.2, 8, 32, 7), ref_img)
        _EXPECT["ref"] = oref
        p = oracle.params(NF, 1.2, 8, 32, 7)
        for s in range(DISTINCT):
            okps, odesc = oracle.extract(p, frames_np[s])
            _EXPECT[s] = (okps, odesc, oracle.bf_match(odesc, oref))
    return _EXPECT


@pytest.mark.parametrize("layout", list(LAYOUTS))
def test_bench_workload_parity(layout):
    import torch
    from orbslam_mapsave_amd.native import ORBextractor, ORBmatcher
    from orbslam_mapsave_amd.synth import synthetic_batch, synthetic_frame
    B, NS, maxb0 = LAYOUTS[layout]
    dev = torch.device("cuda", 0)
    frames_np = synthetic_batch(B, W, H, first_seed=0, distinct=DISTINCT)
    frames = torch.from_numpy(frames_np).to(dev)
    C = B // NS
    streams = [torch.cuda.Stream(dev) for _ in range(NS)]
    exs = []
    for k in range(NS):
        e = ORBextractor(NF, 1.2, 8, 32, 7, device=0, max_width=W, max_height=H,
                         max_batch=maxb0 if k == 0 else C)
        e.set_stream(streams[k].cuda_stream)
        exs.append(e)
    cap = exs[0].capacity(W, H)
    d_kps = torch.zeros((B, cap * 28), dtype=torch.uint8, device=dev)
    d_desc = torch.zeros((B, cap, 32), dtype=torch.uint8, device=dev)
    d_n = torch.zeros(B, dtype=torch.int32, device=dev)
    d_out = torch.full((B, cap, 3), -7, dtype=torch.int32, device=dev)
    ref_img = synthetic_frame(999_999, W, H)
    ex_ref = ORBextractor(NREF, 1.2, 8, 32, 7, device=0, max_width=W, max_height=H)
    _, ref_desc_np = ex_ref(ref_img)
    ex_ref.close()
    ref_desc = torch.from_numpy(np.ascontiguousarray(ref_desc_np)).to(dev)
    d_nr = torch.full((B,), len(ref_desc_np), dtype=torch.int32, device=dev)
    mt = ORBmatcher(0.9, True, device=0)
    torch.cuda.synchronize()
    for k in range(NS):
        f0 = k * C
        exs[k].extract_batch_device(frames[f0].data_ptr(), C, W, H, W, W * H, d_kps[f0].data_ptr(),
                                    cap, d_desc[f0].data_ptr(), d_n[f0:].data_ptr())
        mt.set_stream(streams[k].cuda_stream)
        mt.bf_match_batch_device(d_desc[f0].data_ptr(), cap * 32, d_n[f0:].data_ptr(), cap,
                                 ref_desc.data_ptr(), 0, d_nr[f0:].data_ptr(), C,
                                 d_out[f0].data_ptr())
    torch.cuda.synchronize()
    kps, desc, n, out = d_kps.cpu().numpy(), d_desc.cpu().numpy(), d_n.cpu().numpy(), d_out.cpu().numpy()
    expect = _expected(frames_np, ref_img, ref_desc_np)
    # the reference frame itself: GPU 2x-feature extraction == oracle
    assert np.array_equal(ref_desc_np, expect["ref"])
    for f in range(B):
        okps, odesc, (bi, bd, sd) = expect[f % DISTINCT]
        nf = int(n[f])
        assert nf == len(okps), (f, nf, len(okps))
        assert kps[f, :nf * 28].tobytes() == okps.view(np.uint8).tobytes(), f
        assert np.array_equal(desc[f, :nf], odesc), f
        got = out[f, :nf]
        assert np.array_equal(got[:, 0], bi) and np.array_equal(got[:, 1], bd), f
        assert np.array_equal(got[:, 2], sd), f
    assert KEYPOINT_DTYPE.itemsize == 28
    for e in exs:
        e.close()
    mt.close()


def test_config4_workload_parity():
    """BASELINE configs[3] at full frame size: 1920x1080 @2000 keypoints (ORBextractor(2000,
    1.2, 8, 32, 7), as bench.py --config c4), 64 frames in two sub-batches on two streams, each frame matched against its
    predecessor (bench.py --config c4's frame f vs f-1 step, here within one rank), compared with
    the oracle frame by frame (16 distinct seeds)."""
    import torch
    from orbslam_mapsave_amd.native import ORBextractor, ORBmatcher
    from orbslam_mapsave_amd.synth import synthetic_batch
    W4, H4, NF4, B4, D4 = 1920, 1080, 2000, 64, 16
    dev = torch.device("cuda", 0)
    frames_np = synthetic_batch(B4, W4, H4, first_seed=500, distinct=D4)
    frames = torch.from_numpy(frames_np).to(dev)
    C = B4 // S
    streams = [torch.cuda.Stream(dev) for _ in range(S)]
    exs = []
    for k in range(S):
        e = ORBextractor(NF4, 1.2, 8, 32, 7, device=0, max_width=W4, max_height=H4, max_batch=C)
        e.set_stream(streams[k].cuda_stream)
        exs.append(e)
    cap = exs[0].capacity(W4, H4)
    d_kps = torch.zeros((B4, cap * 28), dtype=torch.uint8, device=dev)
    d_desc = torch.zeros((B4, cap, 32), dtype=torch.uint8, device=dev)
    d_n = torch.zeros(B4, dtype=torch.int32, device=dev)
    for k in range(S):
        f0 = k * C
        exs[k].extract_batch_device(frames[f0].data_ptr(), C, W4, H4, W4, W4 * H4,
                                    d_kps[f0].data_ptr(), cap, d_desc[f0].data_ptr(),
                                    d_n[f0:].data_ptr())
    torch.cuda.synchronize()
    prev = torch.roll(d_desc, 1, 0).contiguous()  # frame f - 1 (frame 0 against the last)
    prev_n = torch.roll(d_n, 1, 0).contiguous()
    out = torch.full((B4, cap, 3), -7, dtype=torch.int32, device=dev)
    mt = ORBmatcher(0.9, True, device=0)
    mt.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    mt.bf_match_batch_device(d_desc.data_ptr(), cap * 32, d_n.data_ptr(), cap, prev.data_ptr(),
                             cap * 32, prev_n.data_ptr(), B4, out.data_ptr())
    torch.cuda.synchronize()
    kps, desc, n, o = d_kps.cpu().numpy(), d_desc.cpu().numpy(), d_n.cpu().numpy(), out.cpu().numpy()
    p = oracle.params(NF4, 1.2, 8, 32, 7)
    expect = [oracle.extract(p, frames_np[s]) for s in range(D4)]
    for f in range(B4):
        okps, odesc = expect[f % D4]
        nf = int(n[f])
        assert nf == len(okps), (f, nf, len(okps))
        assert kps[f, :nf * 28].tobytes() == okps.view(np.uint8).tobytes(), f
        assert np.array_equal(desc[f, :nf], odesc), f
    for f in range(0, B4, 7):  # the matches, on a sample of frames (the oracle BF is O(n^2))
        bi, bd, sd = oracle.bf_match(expect[f % D4][1], expect[(f - 1) % D4][1])
        nf = int(n[f])
        assert np.array_equal(o[f, :nf, 0], bi) and np.array_equal(o[f, :nf, 1], bd), f
        assert np.array_equal(o[f, :nf, 2], sd), f
    for e in exs:
        e.close()
    mt.close()
