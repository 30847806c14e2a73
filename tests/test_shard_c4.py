"""Config 4's real step function (orbslam_mapsave_amd.shard.PredecessorMatch: all-gather of the
descriptor slabs, predecessor selection, frame f vs f - 1 match) — the one bench.py --config c4
runs over RCCL — executed over gloo at world sizes 1, 2, 4 and 8 at configs[3]'s shape: a global
batch of 256 frames (32 per rank at world 8), slabs of capacity(1920, 1080) rows of descriptors
of oracle-extracted 1920x1080 @2000-keypoint frames.  SURVEY §4: the rank-sharded results must be
byte-identical to the single-process run, for every global frame.

Eight frames are extracted by the oracle; the other 248 slabs are those eight with each frame's
descriptors XOR-ed with a per-frame 32-byte mask and its count trimmed by f % 13, so every global
frame's slab is distinct (a wrong predecessor row cannot match by accident)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from orbslam_mapsave_amd.native import keypoint_capacity
from orbslam_mapsave_amd.shard import PredecessorMatch, global_frame

GLOBAL = 256   # global batch (BASELINE configs[3])
BASE = 8       # oracle-extracted frames the slabs derive from
# slab rows: the keypoint capacity of a 1920 x 1080 frame at 2000 keypoints, as the library
# plans it (orbfe_keypoint_capacity_params: host arithmetic, no device) — the rows bench.py
# --config c4 all-gathers per frame
CAP = keypoint_capacity(2000, 1.2, 8, 32, 7, 1920, 1080)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _extract(f):
    import oracle
    from orbslam_mapsave_amd.synth import synthetic_frame
    return oracle.extract(oracle.params(2000, 1.2, 8, 32, 7), synthetic_frame(500 + f, 1920, 1080))[1]


@pytest.fixture(scope="module")
def slabs():
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(4) as ex:
        base = list(ex.map(_extract, range(BASE)))
    desc = np.zeros((GLOBAL, CAP, 32), np.uint8)
    cnt = np.zeros(GLOBAL, np.int32)
    rng = np.random.default_rng(2024)
    for f in range(GLOBAL):
        d = base[f % BASE]
        assert len(d) <= CAP
        n = len(d) - f % 13
        mask = rng.integers(0, 256, 32, dtype=np.uint8) if f >= BASE else np.zeros(32, np.uint8)
        desc[f, :n] = d[:n] ^ mask
        cnt[f] = n
    return desc, cnt


def oracle_match(desc, counts, prev, prev_n, out):
    import oracle
    out.fill_(-7)
    for j in range(desc.shape[0]):
        q = desc[j, :int(counts[j])].numpy()
        r = prev[j, :int(prev_n[j])].numpy()
        bi, bd, sd = oracle.bf_match(q, r)
        out[j, :len(q)] = torch.from_numpy(np.stack([bi, bd, sd], 1).astype(np.int32))


def _worker(rank, world, port, desc, cnt, res, parts=1):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    per = GLOBAL // world
    mine = [global_frame(rank, world, j) for j in range(per)]
    d = torch.from_numpy(desc[mine].copy())
    n = torch.from_numpy(cnt[mine].copy())
    out = torch.zeros((per, CAP, 3), dtype=torch.int32)
    pm = PredecessorMatch(rank, world, per, CAP, "cpu", oracle_match, parts=parts)
    for p in range(parts):  # the overlapped order bench.py --config c4 issues
        pm.gather_part(p, d, n)
    pm.finish(d, n, out)
    res[rank] = {f: out[j].numpy().tobytes() for j, f in enumerate(mine)}
    if world > 1:
        dist.destroy_process_group()


def run_world(world, desc, cnt, parts=1):
    if world == 1:
        res = {}
        _worker(0, 1, 0, desc, cnt, res, parts)
        return res[0]
    out = mp.Manager().dict()
    mp.spawn(_worker, args=(world, _free_port(), desc, cnt, out, parts), nprocs=world, join=True)
    merged = {}
    for r in range(world):
        merged.update(out[r])
    return merged


def test_c4_step_identical_across_world_sizes(slabs):
    desc, cnt = slabs
    base = run_world(1, desc, cnt)
    assert sorted(base) == list(range(GLOBAL))
    # world 1 itself is the plain f vs f - 1 match (frame 0 against the last frame)
    import oracle
    for f in (0, 5):
        p = (f - 1) % GLOBAL
        bi, bd, sd = oracle.bf_match(desc[f, :cnt[f]], desc[p, :cnt[p]])
        got = np.frombuffer(base[f], np.int32).reshape(CAP, 3)[:cnt[f]]
        assert np.array_equal(got, np.stack([bi, bd, sd], 1))
    for world in (2, 4, 8):
        assert run_world(world, desc, cnt) == base, f"world {world} differs from world 1"
    # the overlapped exchange: sub-batches per rank gathered separately (bench.py --config c4
    # runs two, one per extraction stream; world 8 is the 8-GPU node's 32 frames per rank)
    for world, parts in ((8, 2), (4, 2), (2, 2), (1, 4)):
        assert run_world(world, desc, cnt, parts) == base, f"world {world} parts {parts}"
