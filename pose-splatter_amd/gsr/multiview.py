"""Multi-view / multi-GPU data parallelism for the render path.

One process per GPU.  Views (cameras) of one Gaussian set are independent renders; the only
exchange is the sum of the per-rank parameter gradients (``all_reduce(SUM)``, RCCL over
xGMI on MI355X — torch.distributed's "nccl" backend).  The reference has no distributed
code at all; this is the MI355X design, not a translation.

* ``view_shard`` — contiguous, balanced split of C views over ``world`` ranks.
* ``sharded_backward`` — render this rank's views, backprop the caller's cotangents, and
  all-reduce the parameter gradient so every rank ends with the full multi-view gradient.
"""
from __future__ import annotations

from typing import Callable

import torch
import torch.distributed as dist

__all__ = ["view_shard", "sharded_backward"]


def view_shard(C: int, world: int, rank: int) -> slice:
    """Views [start, stop) of rank ``rank``: sizes differ by at most one, earlier ranks larger."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of world {world}")
    base, extra = divmod(C, world)
    start = rank * base + min(rank, extra)
    return slice(start, start + base + (1 if rank < extra else 0))


def sharded_backward(render: Callable, params: torch.Tensor, viewmats: torch.Tensor, Ks: torch.Tensor,
                     v_rgb: torch.Tensor, v_alpha: torch.Tensor, group=None) -> torch.Tensor:
    """Gradient of sum(rgb*v_rgb + alpha*v_alpha) over ALL views, computed view-sharded.

    ``render(params, viewmats, Ks) -> (rgb [c,H,W,3], alpha [c,H,W])`` renders a subset of
    views; v_rgb/v_alpha hold the cotangents of all C views.  Returns the summed gradient
    (identical on every rank).
    """
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    sl = view_shard(viewmats.shape[0], world, rank)
    p = params.detach().requires_grad_(True)
    if sl.stop > sl.start:
        rgb, alpha = render(p, viewmats[sl], Ks[sl])
        torch.autograd.backward([rgb, alpha], [v_rgb[sl], v_alpha[sl]])
        grad = p.grad
    else:
        grad = torch.zeros_like(p)
    if world > 1:
        dist.all_reduce(grad, op=dist.ReduceOp.SUM, group=group)
    return grad
