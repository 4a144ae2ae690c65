"""CPU, world_size 2 (gloo): view-sharded rendering + all-reduce of the parameter gradient
equals the single-process multi-view gradient (the multi-GPU path of bench.py / §8(e)).

The renderer inside the ranks is the CPU oracle (test infrastructure); on the GPU box the
same gsr.multiview code runs with libgsr and backend "nccl" (RCCL).
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _scene():
    from gsr.scenes import gaussians3d, ring_cameras
    p = gaussians3d(300, 5, extent=0.05)
    p[:, 3:6] += 1.0
    V, K = ring_cameras(5, 40, 32)
    g = torch.Generator().manual_seed(9)
    vr = torch.randn(5, 32, 40, 3, generator=g)
    va = torch.randn(5, 32, 40, generator=g)
    return p, V, K, vr, va


def _render(p, V, K):
    from oracle.oracle3d import render3d
    return render3d(p, V, K, 40, 32, torch.ones(3))


def _render_band(p, V, K, band):
    from oracle.oracle3d import render3d
    return render3d(p, V, K, 40, 32, torch.ones(3), band=band)


class _HookRender(torch.autograd.Function):
    """The oracle band render, with the GPU path's bucketed-gradient contract: the backward
    hands each Gaussian-range bucket of the gradient to ``hook`` (gsr.render's grad_hook)."""

    @staticmethod
    def forward(ctx, p, V, K, band, hook, buckets):
        with torch.enable_grad():
            pp = p.detach().requires_grad_(True)
            rgb, a = _render_band(pp, V, K, band)
        ctx.saved = (pp, rgb, a, hook, buckets)
        return rgb.detach(), a.detach()

    @staticmethod
    def backward(ctx, gr, ga):
        from gsr.multiview import bucket_bounds
        pp, rgb, a, hook, buckets = ctx.saved
        (g,) = torch.autograd.grad([rgb, a], [pp], [gr, ga])
        if hook is not None:
            b = bucket_bounds(g.shape[0], buckets)
            for n0, n1 in zip(b[:-1], b[1:]):
                hook(g[n0:n1])
        return g, None, None, None, None, None


def _frames2d():
    g = torch.Generator().manual_seed(13)
    P = torch.randn(4, 60, 9, generator=g)
    P[..., 0] = torch.rand(4, 60, generator=g) * 24
    P[..., 1] = torch.rand(4, 60, generator=g) * 20
    vr = torch.randn(4 * 3, 20, 24, 3, generator=g)
    va = torch.randn(4 * 3, 20, 24, generator=g)
    return P, vr, va


def _render_units2d(p, sets):
    from oracle.oracle2d import render2d_dense
    outs = [render2d_dense(p[f], 24, 20, torch.ones(3)) for f in sets]
    return torch.stack([o[0] for o in outs]), torch.stack([o[1] for o in outs])


def _frames_single():
    """Single-process gradient of the 4-frame x 3-view 2D job: every unit rendered locally."""
    from gsr.multiview import frame_view_units, sharded_backward_frames
    P, vr, va = _frames2d()
    units = frame_view_units(4, 3, 1, 0)
    return sharded_backward_frames(_render_units2d, P, units, vr, va, buckets=1)


def _worker(rank, world, port, out, mode="views"):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "pose-splatter_amd")]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from gsr.multiview import (frame_view_units, sharded_backward, sharded_backward_frames,
                               sharded_backward_units)
    p, V, K, vr, va = _scene()
    if mode == "views":
        grad = sharded_backward(_render, p, V, K, vr, va)
    elif mode == "units":
        grad = sharded_backward_units(lambda q, v, k, band, hook: _render_band(q, v, k, band), p, V, K, vr, va,
                                      rows=2, weights=[3.0, 1.0, 2.0, 2.0, 1.0, 1.0, 0.5, 4.0, 1.0, 1.0])
    elif mode == "units_sparse":
        grad = sharded_backward_units(lambda q, v, k, band, hook: _render_band(q, v, k, band), p, V, K, vr, va,
                                      rows=2, weights=[3.0, 1.0, 2.0, 2.0, 1.0, 1.0, 0.5, 4.0, 1.0, 1.0],
                                      exchange="sparse")
    elif mode == "units_buckets":
        grad = sharded_backward_units(lambda q, v, k, band, hook: _HookRender.apply(q, v, k, band, hook, 3),
                                      p, V, K, vr, va, rows=2, buckets=3)
    elif mode in ("owned", "owned_gather"):
        from gsr.multiview import frame_owner_units, owned_backward_frames
        P, vr2, va2 = _frames2d()
        units = frame_owner_units(4, 3, world, rank)
        idx = [f * 3 + v for f, v in units]
        grad = owned_backward_frames(_render_units2d, P, units, vr2[idx], va2[idx], gather=mode == "owned_gather")
        out[rank] = (grad, sorted({f for f, _ in units}))
        dist.destroy_process_group()
        return
    else:
        P, vr2, va2 = _frames2d()
        units = frame_view_units(4, 3, world, rank)
        idx = [f * 3 + v for f, v in units]
        grad = sharded_backward_frames(_render_units2d, P, units, vr2[idx], va2[idx], buckets=2)
    out[rank] = grad
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_view_sharded_allreduce_matches_single_process(world):
    from gsr.multiview import sharded_backward
    p, V, K, vr, va = _scene()
    ref = sharded_backward(_render, p, V, K, vr, va)     # world 1: all views locally
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    for r in range(world):
        assert torch.allclose(out[r], ref, rtol=1e-5, atol=1e-6 * float(ref.abs().max())), r
    assert torch.equal(out[0], out[1])


def test_band_shard_partition():
    from gsr.multiview import band_shard
    for rows, world in [(32, 8), (5, 8), (36, 3), (1, 2)]:
        bands = [band_shard(rows, world, r) for r in range(world)]
        assert bands[0][0] == 0 and bands[-1][1] == rows
        assert all(bands[i][1] == bands[i + 1][0] for i in range(world - 1))
    w = [1.0] * 10 + [9.0] * 2 + [1.0] * 20          # one heavy pair of rows
    bands = [band_shard(32, 4, r, w) for r in range(4)]
    assert bands[0][0] == 0 and bands[-1][1] == 32
    assert all(bands[i][1] == bands[i + 1][0] for i in range(3))
    loads = [sum(w[a:b]) for a, b in bands]
    assert max(loads) <= sum(w) / 4 + max(w)


def test_band_render_equals_full_render_in_band():
    """Oracle: binning only a range of (view, tile row) units -- global rows, view-major --
    leaves those rows' pixels unchanged, and the ranges' gradients sum to the full gradient."""
    from gsr.multiview import unit_shard
    from oracle.oracle3d import render3d
    p, V, K, vr, va = _scene()
    C, th = V.shape[0], 2
    full_rgb, full_a = render3d(p, V, K, 40, 32, torch.ones(3))
    total = torch.zeros_like(p)
    for r in range(3):
        v0, v1, band = unit_shard(C, th, 3, r)
        pc = p.clone().requires_grad_(True)
        rgb, a = render3d(pc, V[v0:v1], K[v0:v1], 40, 32, torch.ones(3), band=band)
        for c in range(v0, v1):
            y0 = min(max(band[0] - (c - v0) * th, 0), th)
            y1 = min(max(band[1] - (c - v0) * th, 0), th)
            rows = slice(16 * y0, min(32, 16 * y1))
            assert torch.equal(rgb[c - v0, rows], full_rgb[c, rows]) and torch.equal(a[c - v0, rows], full_a[c, rows])
        # cotangents outside the band meet no Gaussians there
        torch.autograd.backward([rgb, a], [vr[v0:v1], va[v0:v1]])
        total += pc.grad
    pf = p.clone().requires_grad_(True)
    torch.autograd.backward(list(render3d(pf, V, K, 40, 32, torch.ones(3))), [vr, va])
    assert torch.allclose(total, pf.grad, rtol=1e-5, atol=1e-6 * float(pf.grad.abs().max()))


@pytest.mark.parametrize("world,mode", [(2, "units"), (3, "units"), (2, "units_buckets"), (3, "units_buckets"),
                                        (2, "units_sparse"), (4, "units_sparse")])
def test_unit_sharded_allreduce_matches_single_process(world, mode):
    """(view, row)-unit sharding (strong scaling of one multi-view job): ranks render disjoint
    view/row ranges; the (bucketed, async) all-reduce of their gradients -- or the exchange of
    only the rows each rank touched (units_sparse) -- is the full gradient."""
    from gsr.multiview import sharded_backward
    p, V, K, vr, va = _scene()
    ref = sharded_backward(_render, p, V, K, vr, va)
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out, mode), nprocs=world, join=True)
    for r in range(world):
        assert torch.allclose(out[r], ref, rtol=1e-5, atol=1e-6 * float(ref.abs().max())), r
    if mode == "units_sparse":   # the same sum, in the same order, on every rank
        assert all(torch.equal(out[0], out[r]) for r in range(world))


def _sparse_worker(rank, world, port, out):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "pose-splatter_amd")]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from gsr.multiview import sparse_sum
    g = torch.Generator().manual_seed(100 + rank)
    part = torch.zeros(50, 14)
    rows = torch.randperm(50, generator=g)[: 5 + 7 * rank]   # ragged, overlapping, rank 0 small
    part[rows] = torch.randn(len(rows), 14, generator=g)
    if rank == world - 1:
        part.zero_()          # a rank that touched nothing
    out[rank] = (part, sparse_sum(part))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_sparse_sum_equals_dense_sum(world):
    """sparse_sum: ragged and overlapping touched-row sets, a rank with none -- the dense sum."""
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_sparse_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    dense = sum(out[r][0] for r in range(world))
    for r in range(world):
        assert torch.allclose(out[r][1], dense, rtol=1e-6, atol=1e-6)
        assert torch.equal(out[r][1], out[0][1])


@pytest.mark.parametrize("world", [2, 4])
def test_frame_sharded_allreduce_matches_single_process(world):
    """Config 4's layout: (frame, view) units round-robin over ranks, batched per frame bucket,
    async per-bucket all-reduce of the [F,N,9] gradient == the single-process gradient."""
    ref = _frames_single()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out, "frames"), nprocs=world, join=True)
    for r in range(world):
        assert torch.allclose(out[r], ref, rtol=1e-5, atol=1e-6 * float(ref.abs().max())), r
    assert torch.equal(out[0], out[1])


@pytest.mark.parametrize("world,mode", [(2, "owned"), (3, "owned"), (2, "owned_gather"), (3, "owned_gather")])
def test_frame_owner_layout_matches_single_process(world, mode):
    """Config 4's frame-owner layout: each rank renders all views of its frames (f % world) and
    holds those frames' complete gradient with no collective; with gather=True every rank ends
    with the full [F,N,9] gradient (an all-gather of the owners' frames)."""
    ref = _frames_single()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out, mode), nprocs=world, join=True)
    owners = {}
    for r in range(world):
        grad, frames = out[r]
        assert frames == [f for f in range(4) if f % world == r]
        for f in range(4):
            if f in frames or mode == "owned_gather":
                assert torch.allclose(grad[f], ref[f], rtol=1e-5, atol=1e-6 * float(ref.abs().max())), (r, f)
            else:
                assert float(grad[f].abs().max()) == 0.0
        for f in frames:
            owners[f] = r
    assert sorted(owners) == [0, 1, 2, 3]
    if mode == "owned_gather":
        assert all(torch.equal(out[0][0], out[r][0]) for r in range(world))


def test_unit_and_frame_partitions():
    from gsr.multiview import frame_buckets, frame_view_units, unit_shard
    for C, rows, world in [(6, 32, 8), (6, 64, 8), (1, 5, 8), (3, 2, 2), (6, 32, 1)]:
        seen = []
        for r in range(world):
            v0, v1, (b0, b1) = unit_shard(C, rows, world, r)
            seen += list(range(v0 * rows + b0, v0 * rows + b1))
            if v1 > v0:   # the band starts in view v0 and ends in view v1 - 1
                assert 0 <= b0 < rows and (v1 - 1 - v0) * rows < b1 <= (v1 - v0) * rows
        assert seen == list(range(C * rows))
    for F, V, world in [(8, 6, 8), (8, 6, 4), (8, 6, 3), (8, 6, 1)]:
        units = [u for r in range(world) for u in frame_view_units(F, V, world, r)]
        assert sorted(units) == [(f, v) for f in range(F) for v in range(V)]
        for r in range(world):
            fs = [f for f, _ in frame_view_units(F, V, world, r)]
            assert fs == sorted(fs)
    assert frame_buckets(8, 2) == [(0, 4), (4, 8)] and frame_buckets(3, 8) == [(0, 1), (1, 2), (2, 3)]
    from gsr.multiview import frame_owner_units
    for F, V, world in [(8, 6, 8), (8, 6, 4), (8, 6, 3), (8, 6, 1), (3, 6, 8)]:
        units = [u for r in range(world) for u in frame_owner_units(F, V, world, r)]
        assert sorted(units) == [(f, v) for f in range(F) for v in range(V)]
        for r in range(world):
            own = frame_owner_units(F, V, world, r)
            assert own == sorted(own) and all(f % world == r for f, _ in own)


def test_unit_bounds_charge_touched_views():
    """With a per-view cost the partition keeps ranks on few views: the bottleneck (max over
    ranks of weights + view_cost x views touched) is never worse than plain weight balancing's
    and is optimal against brute force on small cases."""
    import itertools
    from gsr.multiview import unit_bounds, unit_shard

    def cost(b, w, rows, vc):
        out = []
        for g0, g1 in zip(b[:-1], b[1:]):
            views = len({u // rows for u in range(g0, g1)})
            out.append(sum(w[g0:g1]) + vc * views)
        return max(out)

    g = torch.Generator().manual_seed(3)
    for C, rows, world, vc in [(6, 8, 8, 5.0), (6, 8, 4, 20.0), (3, 4, 2, 3.0), (2, 5, 3, 0.5), (6, 32, 8, 40.0)]:
        w = [float(x) for x in torch.rand(C * rows, generator=g) * 10]
        b = unit_bounds(C, rows, world, w, vc)
        assert b[0] == 0 and b[-1] == C * rows and all(x <= y for x, y in zip(b, b[1:])) and len(b) == world + 1
        plain = unit_bounds(C, rows, world, w, 0.0)
        assert cost(b, w, rows, vc) <= cost(plain, w, rows, vc) + 1e-9
        if C * rows <= 12:   # brute force over all contiguous partitions
            U = C * rows
            best = min(cost([0, *cuts, U], w, rows, vc)
                       for cuts in itertools.combinations_with_replacement(range(U + 1), world - 1))
            assert cost(b, w, rows, vc) <= best + 1e-6
        seen = []
        for r in range(world):
            v0, v1, (b0, b1) = unit_shard(C, rows, world, r, w, vc)
            seen += list(range(v0 * rows + b0, v0 * rows + b1))
        assert seen == list(range(C * rows))
