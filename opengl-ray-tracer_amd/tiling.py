"""tiling.py — image sharding across GPUs (one process per GPU).

Pixels are independent (gpu_shader.comp:434-623 reads no other pixel), so a
frame shards by rows. Rank r of P renders the interleaved stripe set
{ rows y : (y // stripe) % P == r } — every P-th band of `stripe` rows — which
balances the uneven per-row cost (sky rows are cheap, rows through the car's
giant BVH leaves are not) without any per-frame re-planning. Each rank writes
its rows compacted into a [rows_max, W, 4] buffer (rt_dispatch_rows with
y0 = r*stripe, step = P); one fan-in gather brings the P buffers to rank 0,
which scatters the stripes back into image order.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass(frozen=True)
class StripePlan:
    height: int
    world: int
    stripe: int

    def rows(self, rank: int) -> int:
        """Image rows owned by `rank`."""
        full, rem = divmod(self.height, self.stripe * self.world)
        n = full * self.stripe
        extra = rem - rank * self.stripe
        return n + max(0, min(self.stripe, extra))

    @property
    def rows_max(self) -> int:
        return max(self.rows(r) for r in range(self.world))

    def y0(self, rank: int) -> int:
        return rank * self.stripe

    def image_rows(self, rank: int) -> torch.Tensor:
        """Image row of each compacted output row of `rank` (the rt_dispatch_rows mapping)."""
        r = torch.arange(self.rows(rank))
        return self.y0(rank) + (r // self.stripe) * self.stripe * self.world + (r % self.stripe)


@dataclass(frozen=True)
class SharePlan:
    """The rows of rt_group with a root share (csrc/rt_group.hip rank_rows,
    include/rt_group.h rt_group_set_root_share): periods of (share + P - 1)
    stripes, rank 0 the first `share` of each, rank r >= 1 the stripe
    share - 1 + r. share = 1 is StripePlan's interleave."""
    height: int
    world: int
    stripe: int
    share: int = 1

    def mapping(self, rank: int):
        """(y0, stripe, period, rows) of `rank` (the rt_dispatch_rows_ex arguments)."""
        period = (self.share + self.world - 1) * self.stripe
        y0 = 0 if rank == 0 else (self.share - 1 + rank) * self.stripe
        st = self.share * self.stripe if rank == 0 else self.stripe
        full, rem = divmod(self.height, period)
        return y0, st, period, full * st + max(0, min(st, rem - y0))

    def image_rows(self, rank: int) -> torch.Tensor:
        y0, st, period, n = self.mapping(rank)
        r = torch.arange(n)
        return y0 + (r // st) * period + (r % st)


def unpermute(gathered: torch.Tensor, plan: StripePlan) -> torch.Tensor:
    """[world, rows_max, W, 4] compacted stripes -> [H, W, 4] image (on gathered's device)."""
    W = gathered.shape[2]
    out = torch.empty((plan.height, W, gathered.shape[3]), dtype=gathered.dtype, device=gathered.device)
    for r in range(plan.world):
        n = plan.rows(r)
        if n:
            out.index_copy_(0, plan.image_rows(r).to(gathered.device), gathered[r, :n])
    return out


def gather_to_root(local: torch.Tensor, plan: StripePlan, group=None) -> torch.Tensor | None:
    """Fan-in of every rank's [rows_max, W, 4] buffer to rank 0 (RCCL over xGMI on
    GPUs, gloo on CPU). Returns the assembled image on rank 0, None elsewhere."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if world == 1:
        return unpermute(local.unsqueeze(0), plan)
    if local.is_cuda and dist.get_backend(group) == "gloo":
        # rehearsal path (several ranks sharing one GPU): gloo gathers host tensors
        out = gather_to_root(local.cpu(), plan, group)
        return None if out is None else out.to(local.device)
    if rank == 0:
        bufs = torch.empty((world, *local.shape), dtype=local.dtype, device=local.device)
        dist.gather(local, gather_list=list(bufs.unbind(0)), dst=0, group=group)
        return unpermute(bufs, plan)
    dist.gather(local, gather_list=None, dst=0, group=group)
    return None
