"""Multi-view / multi-GPU data parallelism for the render path.

One process per GPU.  Views (cameras) of one Gaussian set are independent renders; the only
exchange is the sum of the per-rank parameter gradients (``all_reduce(SUM)``, RCCL over
xGMI on MI355X — torch.distributed's "nccl" backend).  The reference has no distributed
code at all; this is the MI355X design, not a translation.

* ``view_shard`` — contiguous, balanced split of C views over ``world`` ranks.
* ``sharded_backward`` — render this rank's views, backprop the caller's cotangents, and
  all-reduce the parameter gradient so every rank ends with the full multi-view gradient.
* ``band_shard`` / ``sharded_backward_bands`` — when there are fewer views than GPUs (config
  3/5: 6 views on 8 GPUs), every rank renders ALL views but bins only its
  band of tile rows (``RenderOptions3D.band``); bands are balanced by per-row work (e.g. the
  previous step's per-row list lengths).  Projection is repeated on every rank (O(N) work);
  the raster work splits.  The same single all-reduce sums the gradients.
"""
from __future__ import annotations

from typing import Callable

import torch
import torch.distributed as dist

__all__ = ["view_shard", "sharded_backward", "band_shard", "sharded_backward_bands", "row_work"]


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


def band_shard(rows: int, world: int, rank: int, weights=None) -> tuple:
    """Tile rows [y0, y1) of rank ``rank``: contiguous bands with balanced total weight
    (``weights[r]`` = work of tile row r summed over views; uniform if None).  Every row goes
    to exactly one rank; a rank may get an empty band when rows < world."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of world {world}")
    if weights is None:
        base, extra = divmod(rows, world)
        y0 = rank * base + min(rank, extra)
        return y0, y0 + base + (1 if rank < extra else 0)
    w = [max(float(x), 0.0) for x in weights]
    if len(w) != rows:
        raise ValueError(f"weights must have {rows} entries")
    total = sum(w) or 1.0
    # boundary k sits where the running sum first reaches k/world of the total
    bounds = [0]
    acc, k = 0.0, 1
    for r, x in enumerate(w):
        acc += x
        while k < world and acc >= total * k / world - 1e-12:
            bounds.append(r + 1)
            k += 1
    while len(bounds) < world:
        bounds.append(rows)
    bounds.append(rows)
    return bounds[rank], bounds[rank + 1]


def row_work(stats_tile_len, C: int, th: int, tw: int):
    """Per-tile-row work (list entries summed over views and columns) from a [C*th*tw]
    tensor of per-tile list lengths — the weights for ``band_shard``."""
    t = stats_tile_len.reshape(C, th, tw).sum(dim=(0, 2))
    return [float(x) for x in t.cpu()]


def sharded_backward_bands(render_band: Callable, params: torch.Tensor, viewmats: torch.Tensor, Ks: torch.Tensor,
                           v_rgb: torch.Tensor, v_alpha: torch.Tensor, rows: int, weights=None,
                           group=None) -> torch.Tensor:
    """Gradient of sum(rgb*v_rgb + alpha*v_alpha) over all views, band-sharded: this rank
    renders every view but only its tile rows (``render_band(params, viewmats, Ks, band)``),
    backprops, and all-reduces.  Returns the summed gradient (identical on every rank)."""
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    band = band_shard(rows, world, rank, weights)
    p = params.detach().requires_grad_(True)
    if band[1] > band[0]:
        rgb, alpha = render_band(p, viewmats, Ks, band)
        torch.autograd.backward([rgb, alpha], [v_rgb, v_alpha])
        grad = p.grad
    else:
        grad = torch.zeros_like(p)
    if world > 1:
        dist.all_reduce(grad, op=dist.ReduceOp.SUM, group=group)
    return grad
