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
