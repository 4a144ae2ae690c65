"""Multi-view / multi-GPU data parallelism for the render path.

One process per GPU.  Views (cameras) of one Gaussian set are independent renders; the only
exchange is the sum of the per-rank parameter gradients (``all_reduce(SUM)``, RCCL over
xGMI on MI355X — torch.distributed's "nccl" backend).  The reference has no distributed
code at all; this is the MI355X design, not a translation.

* ``view_shard`` — contiguous, balanced split of C views over ``world`` ranks.
* ``sharded_backward`` — render this rank's views, backprop the caller's cotangents, and
  all-reduce the parameter gradient so every rank ends with the full multi-view gradient.
* ``unit_shard`` / ``sharded_backward_units`` — STRONG scaling of one multi-view job (config
  3/5: 6 views on 8 GPUs).  The work units are (view, tile row); laid out
  view-major they form C*th "global rows", which are cut into ``world`` contiguous ranges of
  balanced work (per-row list lengths of a previous render).  A rank therefore touches one
  or two views (plus whole views in between when C > world) and projects ONLY those, binning
  only its rows (``RenderOptions3D.band`` in global rows).  Its partial v_params is
  all-reduced in Gaussian-range buckets, each launched as soon as the projection backward
  has enqueued its rows, so the collective overlaps the remaining backward.
* ``frame_view_units`` / ``sharded_backward_frames`` — config 4 (2D, 8 frames x 6 views = 48
  units): unit u = f*V + v goes to rank u % world, so every frame's views span ranks; each
  rank renders all its units in ONE batched launch sequence per frame bucket
  (``gsr.render.render2d_units``) and the [F,N,9] gradient is all-reduced per frame bucket
  (async, overlapping the next bucket's render).
* ``GradRows`` / ``rows_backward_units`` — the strong layout's SPARSE exchange on the device:
  the share's backward writes only the gradient rows of the Gaussians it touched into a
  fixed-capacity row block (no dense [N,14] write), the blocks are all-gathered (one
  equal-size collective, no host read of counts) and ``gsr_rows_scatter_add`` sums them into
  the dense gradient in rank order -- the same bits on every rank.  Capacity overflow is
  caught on the device (NaN gradient + GSR_OVF_EXCHANGE in the sticky status).  Nothing in
  the step waits on the host, so it can be captured in a HIP graph with RCCL.
* ``frame_owner_units`` / ``owned_backward_frames`` — config 4 in the frame-owner layout: frame
  f with all its views goes to rank f % world.  Frames have disjoint Gaussian sets, so every
  frame's gradient is complete on its owner: no Gaussian-gradient exchange at all (optionally an
  all-gather of the frames, for callers that want the whole [F,N,9] on every rank).
"""
from __future__ import annotations

from typing import Callable

import torch
import torch.distributed as dist

__all__ = ["view_shard", "sharded_backward", "band_shard", "row_work", "unit_bounds", "unit_shard",
           "sharded_backward_units", "GradRows", "rows_backward_units", "rows_capacity",
           "frame_view_units", "frame_buckets", "sharded_backward_frames", "bucket_bounds",
           "frame_owner_units", "owned_backward_frames", "sparse_sum"]


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


def unit_bounds(C: int, rows: int, world: int, weights=None, view_cost: float = 0.0) -> list:
    """Boundaries g_0 = 0 <= g_1 <= ... <= g_world = C*rows of a contiguous partition of the
    view-major (view, tile row) units that minimises the largest rank cost
        cost(range) = sum of its unit weights + view_cost * (number of views it touches)
    -- every touched view costs a rank a projection forward and backward of all N Gaussians,
    whatever share of its rows the rank renders.  view_cost 0: plain weight balancing
    (``band_shard``).  Bisection on the bottleneck with a greedy fill (optimal for contiguous
    ranges, since a range's cost only grows when it is extended)."""
    U = C * rows
    if world < 1:
        raise ValueError(f"bad world {world}")
    w = [1.0] * U if weights is None else [max(float(x), 0.0) for x in weights]
    if len(w) != U:
        raise ValueError(f"weights must have {U} entries")
    if view_cost <= 0.0:
        return [band_shard(U, world, r, w)[0] for r in range(world)] + [U]

    def fill(B):
        """Greedy ranges under bottleneck B: their starts (None if more than world needed)."""
        starts, cost, view = [0], 0.0, -1
        for u in range(U):
            v = u // rows
            add = w[u] + (view_cost if v != view else 0.0)
            if cost > 0.0 and cost + add > B:
                starts.append(u)
                if len(starts) > world:
                    return None
                cost, view = w[u] + view_cost, v
            else:
                cost += add
                view = v
        return starts

    lo = max(max(w) + view_cost, (sum(w) + C * view_cost) / world)
    hi = sum(w) + C * view_cost
    for _ in range(60):
        mid = 0.5 * (lo + hi)
        if fill(mid) is None:
            lo = mid
        else:
            hi = mid
    starts = fill(hi)
    # fewer ranges than ranks: the last ones stay empty (the bottleneck is already optimal)
    return starts + [U] * (world + 1 - len(starts))


def unit_shard(C: int, rows: int, world: int, rank: int, weights=None, view_cost: float = 0.0) -> tuple:
    """This rank's contiguous share of the C*rows (view, tile row) units, view-major, balanced by
    ``weights`` (C*rows per-unit work; uniform if None) plus ``view_cost`` per touched view
    (``unit_bounds``).  Returns (v0, v1, band): the views [v0, v1) the rank touches and its
    rows as a band of global rows relative to view v0 (the ``RenderOptions3D.band`` of a
    render of views v0..v1-1).  An empty share gives v0 == v1."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of world {world}")
    b = unit_bounds(C, rows, world, weights, view_cost)
    g0, g1 = b[rank], b[rank + 1]
    if g1 <= g0:
        return 0, 0, (0, 0)
    v0, v1 = g0 // rows, (g1 - 1) // rows + 1
    return v0, v1, (g0 - v0 * rows, g1 - v0 * rows)


def bucket_bounds(n: int, buckets: int) -> list:
    """Gaussian-range bucket boundaries used by gsr.render's bucketed projection backward."""
    nb = max(1, min(int(buckets), n)) if n > 0 else 1
    return [n * k // nb for k in range(nb + 1)]


def sparse_sum(grad: torch.Tensor, group=None) -> torch.Tensor:
    """The sum over ranks of a partial gradient of which each rank holds only the rows it touched
    (a (view, tile-row) share: config 5 at 8 ranks touches 2-12 % of the Gaussians per rank,
    tools/touched.py), exchanging only those rows instead of all-reducing the dense [N, D]:
    every rank lists its nonzero rows (index + values), the lists are all-gathered (padded to the
    longest: index 0 with a zero row, which adds nothing) and every rank adds them into a dense
    result in rank order -- the same sum, bitwise, on every rank (a list holds an index once, so
    each add is one value per row).  One small all-gather of the counts precedes it (a host
    read: the padded size)."""
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    if world == 1:
        return grad
    flat = grad.reshape(grad.shape[0], -1)
    idx = torch.nonzero(flat.ne(0).any(1)).flatten()
    k = torch.tensor([idx.numel()], device=grad.device, dtype=torch.int64)
    ks = [torch.zeros_like(k) for _ in range(world)]
    dist.all_gather(ks, k, group=group)
    kmax = max(int(x) for x in ks)
    if kmax == 0:
        return torch.zeros_like(grad)
    idx_pad = torch.zeros(kmax, device=grad.device, dtype=torch.int64)
    val_pad = torch.zeros(kmax, flat.shape[1], device=grad.device, dtype=grad.dtype)
    idx_pad[:idx.numel()] = idx
    val_pad[:idx.numel()] = flat[idx]
    idxs = [torch.empty_like(idx_pad) for _ in range(world)]
    vals = [torch.empty_like(val_pad) for _ in range(world)]
    dist.all_gather(idxs, idx_pad, group=group)
    dist.all_gather(vals, val_pad, group=group)
    out = torch.zeros_like(flat)
    for i, v in zip(idxs, vals):
        out.index_add_(0, i, v)
    return out.view_as(grad)


def sharded_backward_units(render_band: Callable, params: torch.Tensor, viewmats: torch.Tensor, Ks: torch.Tensor,
                           v_rgb: torch.Tensor, v_alpha: torch.Tensor, rows: int, weights=None, buckets: int = 0,
                           group=None, view_cost: float = 0.0, exchange: str = "dense") -> torch.Tensor:
    """Gradient of sum(rgb*v_rgb + alpha*v_alpha) over all C views, (view, row)-unit sharded.

    ``render_band(p, viewmats_sub, Ks_sub, band, hook)`` renders views v0..v1-1 binned to
    ``band``.  With ``buckets`` > 0 it must produce the gradient in ``bucket_bounds(N,
    buckets)`` Gaussian ranges and call ``hook(rows)`` with each range as soon as it is
    enqueued (gsr.render: ``RenderOptions3D(grad_buckets=buckets, grad_hook=hook)``); each
    range is all-reduced asynchronously at once, overlapping the remaining backward.  With
    ``buckets`` == 0 one all-reduce follows the backward.  ``exchange="sparse"``: the rows a
    rank touched are exchanged instead (``sparse_sum``, after the backward; buckets ignored).
    Returns the summed gradient (identical on every rank)."""
    if exchange not in ("dense", "sparse"):
        raise ValueError(f"exchange must be 'dense' or 'sparse', got {exchange!r}")
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    v0, v1, band = unit_shard(viewmats.shape[0], rows, world, rank, weights, view_cost)
    p = params.detach().requires_grad_(True)
    if exchange == "sparse":
        if v1 > v0:
            rgb, alpha = render_band(p, viewmats[v0:v1], Ks[v0:v1], band, None)
            torch.autograd.backward([rgb, alpha], [v_rgb[v0:v1], v_alpha[v0:v1]])
            grad = p.grad
        else:
            grad = torch.zeros_like(p)
        return sparse_sum(grad, group)
    pieces, works = [], []

    def hook(t):
        pieces.append(t)
        if world > 1:
            works.append(dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group, async_op=True))

    use_hook = buckets > 0
    if v1 > v0:
        rgb, alpha = render_band(p, viewmats[v0:v1], Ks[v0:v1], band, hook if use_hook else None)
        torch.autograd.backward([rgb, alpha], [v_rgb[v0:v1], v_alpha[v0:v1]])
        grad = p.grad
    else:
        grad = torch.zeros_like(p)
        if use_hook:   # same collectives, same sizes, on every rank
            b = bucket_bounds(p.shape[0], buckets)
            for n0, n1 in zip(b[:-1], b[1:]):
                hook(grad[n0:n1])
    if use_hook:
        for w in works:
            w.wait()
        return pieces[0] if len(pieces) == 1 and pieces[0].shape == p.shape else torch.cat(pieces)
    if world > 1:
        dist.all_reduce(grad, op=dist.ReduceOp.SUM, group=group)
    return grad


class GradRows:
    """A device row block of ``cap`` sparse gradient rows (include/gsr.h GSR_ROW_FLOATS layout:
    row 0 = header {count, cap}, row 1 + i = {n, 0, v_params[n][0..13]}), written by a band
    render's backward when passed as ``RenderOptions3D(grad_rows=...)``."""

    def __init__(self, cap: int, device):
        from . import _lib
        self.cap = int(cap)
        self.block = torch.zeros(self.cap + 1, _lib.ROW_FLOATS, device=device, dtype=torch.float32)
        # the exchange's buffers, kept across steps (stable addresses for a captured step, and no
        # per-step allocation of world blocks + a dense [N,14]): see buffers()
        self._gathered = None
        self._out = None

    def buffers(self, world: int, N: int):
        """(gathered [world, cap+1, ROW_FLOATS], out [N, 14]) owned by this block, allocated on
        first use and whenever world or N change; `out` is zeroed here on every call."""
        dev = self.block.device
        if self._gathered is None or self._gathered.shape[0] != world:
            self._gathered = torch.empty((world,) + tuple(self.block.shape), device=dev, dtype=self.block.dtype)
        if self._out is None or self._out.shape[0] != N:
            self._out = torch.empty(N, 14, device=dev, dtype=torch.float32)
        self._out.zero_()
        return self._gathered, self._out

    def count(self) -> int:
        """Rows the last backward listed (a host read: diagnostics and capacity sizing only)."""
        return int(self.block[0].view(torch.int32)[0])


def rows_capacity(touched: int, group=None, margin: float = 1.25, slack: int = 1024) -> int:
    """One capacity for every rank's row block (the all-gather needs equal sizes): the largest
    touched-row count over the ranks (one host read, at setup) plus a margin."""
    t = torch.tensor([int(touched)], dtype=torch.int64)
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        if dist.get_backend(group) == "nccl":
            t = t.cuda()
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return int(int(t) * margin) + slack


def rows_backward_units(render_band_rows: Callable, params: torch.Tensor, viewmats: torch.Tensor,
                        Ks: torch.Tensor, v_rgb: torch.Tensor, v_alpha: torch.Tensor, rows: int,
                        grad_rows: GradRows, weights=None, group=None, view_cost: float = 0.0,
                        status: torch.Tensor | None = None, reuse_output: bool = False) -> torch.Tensor:
    """Gradient of sum(rgb*v_rgb + alpha*v_alpha) over all C views, (view, row)-unit sharded,
    with the device sparse exchange.  ``render_band_rows(p, viewmats_sub, Ks_sub, band, grad_rows)``
    renders views v0..v1-1 binned to ``band`` with ``RenderOptions3D(grad_rows=grad_rows)``;
    its backward leaves the touched rows in ``grad_rows.block``.  The blocks of all ranks are
    all-gathered and summed in rank order (``gsr_rows_scatter_add``): identical bits on every
    rank, no host synchronisation (a rank with more touched rows than the capacity makes the
    result NaN and sets GSR_OVF_EXCHANGE in ``status``).  The dense result is built in a buffer
    of ``grad_rows`` that the next call overwrites: a copy is returned unless ``reuse_output``
    (a caller that consumes the gradient before its next call, e.g. bench.py)."""
    from . import _lib
    L = _lib.lib()
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    v0, v1, band = unit_shard(viewmats.shape[0], rows, world, rank, weights, view_cost)
    dev = params.device
    stream = torch.cuda.current_stream(dev).cuda_stream
    p = params.detach().requires_grad_(True)
    if v1 > v0:
        rgb, alpha = render_band_rows(p, viewmats[v0:v1], Ks[v0:v1], band, grad_rows)
        torch.autograd.backward([rgb, alpha], [v_rgb[v0:v1], v_alpha[v0:v1]])
    else:   # an empty share: a header with no rows
        _lib.check(L.gsr3d_touched_rows(None, None, None, None, None, 0, 0, grad_rows.cap, None,
                                        grad_rows.block.data_ptr(), stream), "gsr3d_touched_rows")
    blk = grad_rows.block
    # the gathered blocks and the dense result live in grad_rows (reused every step)
    gathered, out = grad_rows.buffers(world, params.shape[0])
    if world > 1:
        if dist.get_backend(group) == "nccl":
            dist.all_gather_into_tensor(gathered, blk, group=group)
        else:
            dist.all_gather(list(gathered.unbind(0)), blk, group=group)
    else:
        gathered = blk[None]
    _lib.check(L.gsr_rows_scatter_add(gathered.data_ptr(), world, grad_rows.cap, out.data_ptr(), params.shape[0],
                                      None if status is None else status.data_ptr(), stream), "gsr_rows_scatter_add")
    return out if reuse_output else out.clone()


def frame_view_units(F: int, V: int, world: int, rank: int) -> list:
    """(frame, view) units of ``rank``: unit u = f*V + v goes to rank u % world (round robin), so
    each frame's views span ranks.  Grouped by frame."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of world {world}")
    return [(u // V, u % V) for u in range(F * V) if u % world == rank]


def frame_owner_units(F: int, V: int, world: int, rank: int) -> list:
    """(frame, view) units of ``rank`` in the frame-owner layout: frame f and ALL its views go
    to rank f % world (config 4 at 8 ranks: one frame, 6 units per rank).  The frames' Gaussian
    sets are disjoint, so each frame's gradient is complete on its owner and no Gaussian-gradient
    exchange is needed (data-parallel training over frames: the owner back-propagates its
    frames into the network, whose weight gradients DP all-reduces anyway).  Grouped by frame."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of world {world}")
    return [(f, v) for f in range(F) if f % world == rank for v in range(V)]


def owned_backward_frames(render_units: Callable, params: torch.Tensor, units: list, v_rgb: torch.Tensor,
                          v_alpha: torch.Tensor, gather: bool = False, group=None) -> torch.Tensor:
    """Multi-frame 2D step in the frame-owner layout (``frame_owner_units``).  params [F,N,9];
    this rank renders all its units in ONE batched launch sequence and backprops them.  Returns
    the [F,N,9] gradient with this rank's frames filled (other frames zero) -- complete for every
    owned frame, with no collective.  ``gather=True`` also all-gathers every frame's gradient
    from its owner (an all-gather, half an all-reduce's traffic), so every rank ends with the
    full [F,N,9] gradient, identical to the single-process one."""
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    F = params.shape[0]
    grad = torch.zeros_like(params)
    owned = sorted({f for f, _ in units})
    if units:
        f0, f1 = owned[0], owned[-1] + 1
        p = params[f0:f1].detach().requires_grad_(True)
        rgb, alpha = render_units(p, [f - f0 for f, _ in units])
        torch.autograd.backward([rgb, alpha], [v_rgb, v_alpha])
        for f in owned:   # frames between owned ones (world 1 excepted) are not this rank's
            grad[f].copy_(p.grad[f - f0])
    if gather and world > 1:
        # frames f, f + world, ... belong to rank f % world: gather one frame slot per round
        for f0 in range(0, F, world):
            n = min(world, F - f0)
            mine = grad[f0 + rank] if rank < n else torch.zeros_like(grad[0])
            slots = [torch.empty_like(grad[0]) for _ in range(world)]
            dist.all_gather(slots, mine.contiguous(), group=group)
            for r in range(n):
                grad[f0 + r].copy_(slots[r])
    return grad


def frame_buckets(F: int, buckets: int) -> list:
    """Frame ranges [f0, f1) of the all-reduce buckets (identical on every rank)."""
    nb = max(1, min(int(buckets), F))
    return [(F * k // nb, F * (k + 1) // nb) for k in range(nb)]


def sharded_backward_frames(render_units: Callable, params: torch.Tensor, units: list, v_rgb: torch.Tensor,
                            v_alpha: torch.Tensor, buckets: int = 2, group=None) -> torch.Tensor:
    """Multi-frame 2D step (config 4).  params [F,N,9]: every rank holds all F frames' sets;
    ``units``: this rank's (frame, view) units, grouped by frame (``frame_view_units``);
    v_rgb [len(units),H,W,3] / v_alpha [len(units),H,W]: their cotangents.  The frames are cut
    into ``buckets`` ranges; per range the rank renders its units in one batched sequence
    (``render_units(params_range [Fr,N,9], unit_sets) -> (rgb [u,H,W,3], alpha [u,H,W])``),
    backprops, and launches an async all-reduce of the range's [Fr,N,9] gradient, which runs
    while the next range renders.  Returns the summed gradient [F,N,9] (identical on every rank)."""
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    F = params.shape[0]
    grad = torch.zeros_like(params)
    works = []
    for f0, f1 in frame_buckets(F, buckets):
        idx = [i for i, (f, _) in enumerate(units) if f0 <= f < f1]
        if idx:
            p = params[f0:f1].detach().requires_grad_(True)
            sets = [units[i][0] - f0 for i in idx]
            rgb, alpha = render_units(p, sets)
            a, b = idx[0], idx[-1] + 1   # units are grouped by frame: a contiguous range
            torch.autograd.backward([rgb, alpha], [v_rgb[a:b], v_alpha[a:b]])
            grad[f0:f1].copy_(p.grad)
        if world > 1:
            works.append(dist.all_reduce(grad[f0:f1], op=dist.ReduceOp.SUM, group=group, async_op=True))
    for w in works:
        w.wait()
    return grad
