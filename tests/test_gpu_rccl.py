"""Config 4's exchange step (orbslam_mapsave_amd.shard.PredecessorMatch) through RCCL on the
MI355X: a one-rank "nccl" process group on cuda:0 with the collective forced at world 1, so the
slabs go through dist.all_gather_into_tensor with async handles queued behind the producing
streams exactly as bench.py --config c4 issues them, and the GPU brute-force matcher runs on the
gathered predecessors.  The result must equal the copy path's (no collective) and the oracle's
f vs f - 1 match.  The multi-rank exchange itself is covered over gloo (tests/test_shard*.py);
one GPU cannot host two RCCL ranks."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu

B, CAP = 4, 512


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.fixture(scope="module")
def rccl_group():
    dev = torch.device("cuda", 0)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0,
                            world_size=1, device_id=dev)
    assert dist.get_backend() == "nccl"
    yield dev
    dist.destroy_process_group()


@pytest.mark.parametrize("parts", [1, 2])
def test_rccl_exchange_and_match(rccl_group, parts):
    import oracle
    from orbslam_mapsave_amd.native import ORBmatcher
    from orbslam_mapsave_amd.shard import PredecessorMatch
    dev = rccl_group
    rng = np.random.default_rng(7 + parts)
    n = rng.integers(CAP // 2, CAP + 1, size=B).astype(np.int32)
    desc = np.zeros((B, CAP, 32), np.uint8)
    for f in range(B):
        desc[f, :n[f]] = rng.integers(0, 256, size=(n[f], 32), dtype=np.uint8)
    d_desc = torch.from_numpy(desc).to(dev)
    d_n = torch.from_numpy(n).to(dev)
    mt = ORBmatcher(0.8, False, device=0)
    streams = [torch.cuda.Stream(dev) for _ in range(parts)]
    try:
        def bf(q, qn, r, rn, out):
            mt.set_stream(torch.cuda.current_stream(dev).cuda_stream)
            mt.bf_match_batch_device(q.data_ptr(), CAP * 32, qn.data_ptr(), CAP, r.data_ptr(),
                                     CAP * 32, rn.data_ptr(), q.shape[0], out.data_ptr())

        outs = {}
        for collective in (True, False):
            pm = PredecessorMatch(0, 1, B, CAP, dev, bf, parts=parts, collective=collective)
            out = torch.full((B, CAP, 3), -7, dtype=torch.int32, device=dev)
            torch.cuda.synchronize(dev)
            per = B // parts
            for p, s in enumerate(streams):  # each part's gather queued behind its own stream
                with torch.cuda.stream(s):
                    # the part's "extraction": its slabs rewritten on this stream first
                    part = d_desc[p * per:(p + 1) * per]
                    part.copy_(part.clone())
                    pm.gather_part(p, d_desc, d_n)
            main = torch.cuda.current_stream(dev)
            for s in streams:
                main.wait_stream(s)
            pm.finish(d_desc, d_n, out)
            torch.cuda.synchronize(dev)
            outs[collective] = out.cpu().numpy()
        assert np.array_equal(outs[True], outs[False])
        for f in range(B):
            prv = (f - 1) % B
            bi, bd, sd = oracle.bf_match(desc[f, :n[f]], desc[prv, :n[prv]])
            assert np.array_equal(outs[True][f, :n[f]], np.stack([bi, bd, sd], 1)), f"frame {f}"
    finally:
        mt.close()


@pytest.mark.parametrize("parts", [1, 2])
def test_rccl_config4_rank_shape(rccl_group, parts):
    """BASELINE configs[3] at its 8-GPU per-rank shape, through RCCL: 32 frames of 1920 x 1080
    extracted on the GPU at 2000 keypoints (x86 reading) in `parts` sub-batches on their own
    streams, each part's all-gather of its capacity(1920, 1080)-row slabs queued behind its
    extraction (the order bench.py --config c4 issues), the predecessors selected from the
    gathered array and brute-force matched on the GPU.  Must equal the copy path and the oracle's
    frame f vs f - 1 match (ORBmatcher.cc:1331-1473's pairing) on the same descriptors; two
    frames' extraction is checked against the oracle too."""
    import oracle
    from orbslam_mapsave_amd.native import ORBextractor, ORBmatcher
    from orbslam_mapsave_amd.shard import PredecessorMatch
    from orbslam_mapsave_amd.synth import synthetic_frame
    dev = rccl_group
    W, H, NF, B = 1920, 1080, 2000, 32
    base = [synthetic_frame(4000 + i, W, H) for i in range(8)]
    # 32 distinct frames: each base frame shifted by a different number of columns
    frames_np = np.stack([np.roll(base[i % 8], 7 * (i // 8), axis=1) for i in range(B)])
    frames = torch.from_numpy(frames_np).to(dev)
    C = B // parts
    streams = [torch.cuda.Stream(dev) for _ in range(parts)]
    exs = []
    for k in range(parts):
        e = ORBextractor(NF, 1.2, 8, 20, 7, device=0, max_width=W, max_height=H, max_batch=C)
        e.set_stream(streams[k].cuda_stream)
        exs.append(e)
    cap = exs[0].capacity(W, H)
    mt = ORBmatcher(0.9, True, device=0)
    main = torch.cuda.current_stream(dev)
    try:
        def bf(q, qn, r, rn, out):
            mt.set_stream(main.cuda_stream)
            mt.bf_match_batch_device(q.data_ptr(), cap * 32, qn.data_ptr(), cap, r.data_ptr(),
                                     cap * 32, rn.data_ptr(), q.shape[0], out.data_ptr())

        outs = {}
        for collective in (True, False):
            d_kps = torch.empty((B, cap * 28), dtype=torch.uint8, device=dev)
            d_desc = torch.zeros((B, cap, 32), dtype=torch.uint8, device=dev)
            d_n = torch.zeros(B, dtype=torch.int32, device=dev)
            out = torch.full((B, cap, 3), -7, dtype=torch.int32, device=dev)
            pm = PredecessorMatch(0, 1, B, cap, dev, bf, parts=parts, collective=collective)
            torch.cuda.synchronize(dev)
            for k in range(parts):
                f0 = k * C
                exs[k].extract_batch_device(frames[f0].data_ptr(), C, W, H, W, W * H,
                                            d_kps[f0].data_ptr(), cap, d_desc[f0].data_ptr(),
                                            d_n[f0:].data_ptr())
                with torch.cuda.stream(streams[k]):
                    pm.gather_part(k, d_desc, d_n)
            for s in streams:
                main.wait_stream(s)
            pm.finish(d_desc, d_n, out)
            torch.cuda.synchronize(dev)
            outs[collective] = (out.cpu().numpy(), d_desc.cpu().numpy(), d_n.cpu().numpy())
        o, desc, n = outs[True]
        assert np.array_equal(o, outs[False][0])
        assert np.array_equal(n, outs[False][2]) and np.array_equal(desc, outs[False][1])
        assert n.min() > 1500 and n.max() <= cap
        for f in range(B):
            prv = (f - 1) % B
            bi, bd, sd = oracle.bf_match(desc[f, :n[f]], desc[prv, :n[prv]])
            assert np.array_equal(o[f, :n[f]], np.stack([bi, bd, sd], 1)), f"frame {f}"
        p = oracle.params(NF, 1.2, 8, 20, 7)
        for f in (0, B - 1):
            _, od = oracle.extract(p, frames_np[f])
            assert np.array_equal(desc[f, :n[f]], od), f"frame {f} descriptors"
    finally:
        mt.close()
        for e in exs:
            e.close()
