"""Multi-rank path on CPU: frame sharding + the descriptor all-gather of config 4, world size 2
over gloo (the GPU run uses the same functions over RCCL).  The exchanged slabs are checked to
deliver, for every local frame, exactly its global predecessor's descriptors, and the
f vs f-1 matches computed from them equal a single-process computation (oracle brute force)."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from orbslam_mapsave_amd.shard import (gather_slabs, global_frame, gathered_row,
                                       predecessor_index)


def test_predecessor_mapping():
    for world in (1, 2, 4, 8):
        per = 6
        total = world * per
        for parts in (1, 2, 3):
            pp = per // parts
            seen, rows_all = set(), set()
            for r in range(world):
                rows = predecessor_index(r, world, per, parts)
                for j, row in enumerate(rows):
                    f = global_frame(r, world, j)
                    seen.add(f)
                    p = (f - 1) % total
                    assert row == gathered_row(p, world, per, parts)
                    # part-major, then rank-major: the row is where part (p // world) // pp of
                    # rank p % world lands
                    part, jj = divmod(p // world, pp)
                    assert row == part * world * pp + (p % world) * pp + jj
                    rows_all.add(row)
            assert seen == set(range(total))
            assert rows_all == set(range(total))  # a permutation of the gathered rows


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _slab(f, cap=24):
    rng = np.random.default_rng(f)
    return rng.integers(0, 256, (cap, 32), dtype=np.uint8), int(rng.integers(5, cap))


def _worker(rank, world, port, per, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import oracle
    cap = 24
    desc = torch.zeros((per, cap, 32), dtype=torch.uint8)
    cnt = torch.zeros(per, dtype=torch.int32)
    for j in range(per):
        d, n = _slab(global_frame(rank, world, j))
        desc[j] = torch.from_numpy(d)
        cnt[j] = n
    g_desc = torch.zeros((world * per, cap, 32), dtype=torch.uint8)
    g_cnt = torch.zeros(world * per, dtype=torch.int32)
    gather_slabs(desc, cnt, g_desc, g_cnt, world)
    pred = torch.tensor(predecessor_index(rank, world, per))
    prev, prev_n = g_desc[pred], g_cnt[pred]
    res = {}
    for j in range(per):
        f = global_frame(rank, world, j)
        bi, bd, sd = oracle.bf_match(desc[j, :cnt[j]].numpy(), prev[j, :prev_n[j]].numpy())
        res[f] = (bi.tolist(), bd.tolist(), sd.tolist())
    out[rank] = res
    dist.destroy_process_group()


def test_gloo_world2_exchange_and_match():
    world, per = 2, 3
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), per, out), nprocs=world, join=True)
    import oracle
    merged = {}
    for r in range(world):
        merged.update(out[r])
    total = world * per
    assert sorted(merged) == list(range(total))
    for f in range(total):
        d, n = _slab(f)
        pd, pn = _slab((f - 1) % total)
        bi, bd, sd = oracle.bf_match(d[:n], pd[:pn])
        assert merged[f] == (bi.tolist(), bd.tolist(), sd.tolist())


def test_collective_forced_at_world1():
    """gather_slabs / PredecessorMatch with the collective forced at world 1 (the path
    tests/test_gpu_rccl.py drives through RCCL on one GPU): over a one-rank gloo group the
    gathered slabs and the predecessor selection equal the copy path's."""
    from orbslam_mapsave_amd.shard import PredecessorMatch
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        per, cap = 4, 16
        g = torch.Generator().manual_seed(3)
        desc = torch.randint(0, 256, (per, cap, 32), dtype=torch.uint8, generator=g)
        cnt = torch.randint(1, cap + 1, (per,), dtype=torch.int32, generator=g)
        seen = {}
        for collective in (True, False):
            got = []

            def match(d, n, prev, prev_n, out, got=got):
                got.append((prev.clone(), prev_n.clone()))

            pm = PredecessorMatch(0, 1, per, cap, "cpu", match, parts=2, collective=collective)
            pm.step(desc, cnt, None)
            seen[collective] = got[0]
        assert torch.equal(seen[True][0], seen[False][0]) and torch.equal(seen[True][1], seen[False][1])
        # frame f's predecessor is f - 1 (frame 0's the last)
        assert torch.equal(seen[True][0], desc[[per - 1, 0, 1, 2]])
    finally:
        dist.destroy_process_group()
