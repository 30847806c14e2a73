"""Frame sharding across ranks (one process per GPU) and the descriptor exchange of config 4.

Frames of a global batch are dealt round-robin: global frame f lives on rank f % world as local
frame f // world.  Cross-frame matching (frame f vs frame f-1, the tracking pattern of
SearchByProjection on the last frame) needs the predecessor's descriptor slab, which for
world > 1 lives on another GPU: one all-gather of the fixed-capacity slabs (RCCL over xGMI with
the "nccl" backend) gives every rank every frame.  This is the only collective in the package.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def global_frame(rank: int, world: int, local: int) -> int:
    return local * world + rank


def gathered_row(f: int, world: int, per_rank: int) -> int:
    """Row of global frame f in the rank-major all-gather output."""
    return (f % world) * per_rank + f // world


def predecessor_index(rank: int, world: int, per_rank: int) -> list[int]:
    """For each local frame, the gathered row of its predecessor (frame 0 wraps to the last)."""
    total = world * per_rank
    rows = []
    for j in range(per_rank):
        f = global_frame(rank, world, j)
        p = f - 1 if f > 0 else total - 1
        rows.append(gathered_row(p, world, per_rank))
    return rows


def gather_slabs(desc: torch.Tensor, counts: torch.Tensor, g_desc: torch.Tensor,
                 g_counts: torch.Tensor, world: int) -> None:
    """All-gather the per-rank descriptor slabs (B x cap x 32 u8) and keypoint counts."""
    if world == 1:
        g_desc.copy_(desc)
        g_counts.copy_(counts)
        return
    if dist.get_backend() == "gloo":  # CPU test path: list form
        parts = [torch.empty_like(desc) for _ in range(world)]
        dist.all_gather(parts, desc)
        g_desc.copy_(torch.cat(parts))
        cparts = [torch.empty_like(counts) for _ in range(world)]
        dist.all_gather(cparts, counts)
        g_counts.copy_(torch.cat(cparts))
        return
    dist.all_gather_into_tensor(g_desc, desc)
    dist.all_gather_into_tensor(g_counts, counts)


class PredecessorMatch:
    """Config 4's exchange + match step (BASELINE configs[3]), one instance per rank: every
    rank holds B = per_rank frames' descriptor slabs (B x cap x 32 u8) and keypoint counts,
    all-gathers them (gather_slabs: RCCL over xGMI on the GPU, gloo in the CPU tests), picks
    each local frame's global predecessor (predecessor_index) and calls
    match(desc, counts, prev_desc, prev_counts, out) — frame f's queries against frame f - 1,
    the tracking pattern of SearchByProjection(CurrentFrame, LastFrame) (ORBmatcher.cc:1331).
    The buffers live on `device`; bench.py passes the GPU brute-force matcher as `match`."""

    def __init__(self, rank: int, world: int, per_rank: int, cap: int, device, match):
        self.world = world
        self.match = match
        self.g_desc = torch.zeros((world * per_rank, cap, 32), dtype=torch.uint8, device=device)
        self.g_n = torch.zeros(world * per_rank, dtype=torch.int32, device=device)
        self.prev = torch.zeros((per_rank, cap, 32), dtype=torch.uint8, device=device)
        self.prev_n = torch.zeros(per_rank, dtype=torch.int32, device=device)
        self.pred = torch.as_tensor(predecessor_index(rank, world, per_rank), device=device)

    def step(self, desc: torch.Tensor, counts: torch.Tensor, out) -> None:
        gather_slabs(desc, counts, self.g_desc, self.g_n, self.world)
        torch.index_select(self.g_desc, 0, self.pred, out=self.prev)
        torch.index_select(self.g_n, 0, self.pred, out=self.prev_n)
        self.match(desc, counts, self.prev, self.prev_n, out)

