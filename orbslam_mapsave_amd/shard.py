"""Frame sharding across ranks (one process per GPU) and the descriptor exchange of config 4.

Frames of a global batch are dealt round-robin: global frame f lives on rank f % world as local
frame f // world.  Cross-frame matching (frame f vs frame f-1, the tracking pattern of
SearchByProjection on the last frame) needs the predecessor's descriptor slab, which for
world > 1 lives on another GPU: an all-gather of the fixed-capacity slabs (RCCL over xGMI with
the "nccl" backend) gives every rank every frame.  This is the only collective in the package.

The per-rank batch may be exchanged in `parts` sub-batches (local frames [p·B/parts,
(p+1)·B/parts) form part p), so that part p's all-gather runs on the communication stream while
part p+1 is still being extracted.  The gathered array is part-major: part p of every rank, rank
by rank, then part p+1.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def global_frame(rank: int, world: int, local: int) -> int:
    return local * world + rank


def gathered_row(f: int, world: int, per_rank: int, parts: int = 1) -> int:
    """Row of global frame f in the part-major, rank-major all-gather output."""
    per_part = per_rank // parts
    part, j = divmod(f // world, per_part)
    return part * world * per_part + (f % world) * per_part + j


def predecessor_index(rank: int, world: int, per_rank: int, parts: int = 1) -> list[int]:
    """For each local frame, the gathered row of its predecessor (frame 0 wraps to the last)."""
    total = world * per_rank
    rows = []
    for j in range(per_rank):
        f = global_frame(rank, world, j)
        p = f - 1 if f > 0 else total - 1
        rows.append(gathered_row(p, world, per_rank, parts))
    return rows


def gather_slabs(desc: torch.Tensor, counts: torch.Tensor, g_desc: torch.Tensor,
                 g_counts: torch.Tensor, world: int, async_op: bool = False,
                 collective: bool | None = None) -> list:
    """All-gather the per-rank descriptor slabs (B x cap x 32 u8) and keypoint counts into the
    rank-major g_desc / g_counts.  With async_op (RCCL) the collectives are queued behind the
    current stream's work and the returned handles are waited on later; gloo (the CPU tests) and
    world 1 complete before returning.  collective (default: world > 1) = False copies instead of
    calling the collective; True calls it at world 1 too (tests/test_gpu_rccl.py runs the RCCL
    path on one GPU that way)."""
    if collective is None:
        collective = world > 1
    if not collective:
        g_desc.copy_(desc)
        g_counts.copy_(counts)
        return []
    if dist.get_backend() == "gloo":  # CPU test path: list form
        parts = [torch.empty_like(desc) for _ in range(world)]
        dist.all_gather(parts, desc)
        g_desc.copy_(torch.cat(parts))
        cparts = [torch.empty_like(counts) for _ in range(world)]
        dist.all_gather(cparts, counts)
        g_counts.copy_(torch.cat(cparts))
        return []
    works = [dist.all_gather_into_tensor(g_desc, desc, async_op=async_op),
             dist.all_gather_into_tensor(g_counts, counts, async_op=async_op)]
    return [w for w in works if w is not None] if async_op else []


class PredecessorMatch:
    """Config 4's exchange + match step (BASELINE configs[3]), one instance per rank: every
    rank holds B = per_rank frames' descriptor slabs (B x cap x 32 u8) and keypoint counts,
    all-gathers them (gather_slabs: RCCL over xGMI on the GPU, gloo in the CPU tests) in `parts`
    sub-batches, picks each local frame's global predecessor (predecessor_index) and calls
    match(desc, counts, prev_desc, prev_counts, out) — frame f's queries against frame f - 1,
    the tracking pattern of SearchByProjection(CurrentFrame, LastFrame) (ORBmatcher.cc:1331).
    The buffers live on `device`; bench.py passes the GPU brute-force matcher as `match`.

    Overlapped use (bench.py --config c4): after part p's extraction is queued on stream s_p,
    call gather_part(p, ...) with s_p current; once every part is queued, finish(...) on the
    stream that runs the match.  step() does both in sequence."""

    def __init__(self, rank: int, world: int, per_rank: int, cap: int, device, match,
                 parts: int = 1, collective: bool | None = None):
        if parts < 1 or per_rank % parts:
            raise ValueError(f"per_rank {per_rank} is not a multiple of parts {parts}")
        self.world = world
        self.collective = collective
        self.parts = parts
        self.per_part = per_rank // parts
        self.match = match
        self.g_desc = torch.zeros((world * per_rank, cap, 32), dtype=torch.uint8, device=device)
        self.g_n = torch.zeros(world * per_rank, dtype=torch.int32, device=device)
        self.prev = torch.zeros((per_rank, cap, 32), dtype=torch.uint8, device=device)
        self.prev_n = torch.zeros(per_rank, dtype=torch.int32, device=device)
        self.pred = torch.as_tensor(predecessor_index(rank, world, per_rank, parts),
                                    device=device)
        self._works: list = []

    def gather_part(self, p: int, desc: torch.Tensor, counts: torch.Tensor) -> None:
        """Queue part p's all-gather behind the current stream (which must be the one that
        produced part p's slabs)."""
        a, b = p * self.per_part, (p + 1) * self.per_part
        ga, gb = p * self.world * self.per_part, (p + 1) * self.world * self.per_part
        self._works += gather_slabs(desc[a:b], counts[a:b], self.g_desc[ga:gb],
                                    self.g_n[ga:gb], self.world, async_op=True,
                                    collective=self.collective)

    def finish(self, desc: torch.Tensor, counts: torch.Tensor, out) -> None:
        """Make the current stream wait for every queued gather, select the predecessors and
        match."""
        for w in self._works:
            w.wait()
        self._works = []
        torch.index_select(self.g_desc, 0, self.pred, out=self.prev)
        torch.index_select(self.g_n, 0, self.pred, out=self.prev_n)
        self.match(desc, counts, self.prev, self.prev_n, out)

    def step(self, desc: torch.Tensor, counts: torch.Tensor, out) -> None:
        for p in range(self.parts):
            self.gather_part(p, desc, counts)
        self.finish(desc, counts, out)
