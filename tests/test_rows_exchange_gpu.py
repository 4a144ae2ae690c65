"""The strong layout's device sparse exchange (gsr3d_touched_rows, gsr3d_project_bwd_rows,
gsr_rows_scatter_add; gsr.multiview.rows_backward_units), on one GPU.

The ranks of a (view, tile-row) unit partition are played one after the other in this
process (the collective is then the stacking of their blocks; the gloo / RCCL all-gather
itself is exercised by tools/gpu_dist.sh and the driver's multi-GPU runs):
* each share's row block lists exactly the Gaussians owning a list entry before their tile's cut
  (the partial rows the raster backward writes), and each listed row is bitwise the dense
  backward's row of the same share (unlisted rows are zero there);
* the rank-ordered scatter-add of the blocks equals ((0 + g_0) + g_1) + ... of the dense
  partial gradients, bitwise -- the sum a rank-ordered dense reduction gives, on every rank;
* with one share covering everything, rows_backward_units equals the dense gradient bitwise;
* a block too small for its share: NaN gradient and GSR_OVF_EXCHANGE in the sticky status;
* a share whose bounded forward overflowed poisons the exchange the same way (its header is
  set past the cap), so a captured step cannot sum a share that silently lacks its rows.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _scene(dev):
    from gsr.scenes import gaussians3d, ring_cameras
    W, H, C = 192, 170, 3
    p = gaussians3d(20000, 17).to(dev)
    V, K = ring_cameras(C, W, H)
    g = torch.Generator().manual_seed(18)
    vr = torch.randn(C, H, W, 3, generator=g).to(dev)
    va = torch.randn(C, H, W, generator=g).to(dev)
    return p, V.to(dev), K.to(dev), W, H, vr, va


def _share(p, V, K, W, H, vr, va, v0, v1, band, grad_rows=None):
    from gsr import render as R
    pg = p.detach().clone().requires_grad_(True)
    opts = R.RenderOptions3D(band=band, grad_rows=grad_rows, capacity="exact")
    rgb, alpha = R.render3d(pg, V[v0:v1], K[v0:v1], W, H, torch.ones(3, device=p.device), opts)
    torch.autograd.backward([rgb, alpha], [vr[v0:v1], va[v0:v1]])
    torch.cuda.synchronize()
    return pg.grad, R.last_stats()["_bins"]


def _scatter(blocks, cap, N, status=None):
    from gsr import _lib
    out = torch.zeros(N, 14, device=blocks.device)
    _lib.check(_lib.lib().gsr_rows_scatter_add(blocks.data_ptr(), blocks.shape[0], cap, out.data_ptr(), N,
                                               None if status is None else status.data_ptr(),
                                               torch.cuda.current_stream().cuda_stream), "gsr_rows_scatter_add")
    torch.cuda.synchronize()
    return out


def test_rows_equal_dense_partials_and_rank_ordered_sum(cuda):
    from gsr.multiview import GradRows, unit_shard
    p, V, K, W, H, vr, va = _scene(cuda)
    N, C, th = p.shape[0], V.shape[0], (H + 15) // 16
    world = 4
    blocks, dense = [], []
    for r in range(world):
        v0, v1, band = unit_shard(C, th, world, r)
        g_dense, b = _share(p, V, K, W, H, vr, va, v0, v1, band)
        gr = GradRows(N, cuda)
        g_none, b2 = _share(p, V, K, W, H, vr, va, v0, v1, band, gr)
        assert g_none is None                       # no dense gradient in rows mode
        cnt = gr.count()
        # the Gaussians owning an entry before their tile's cut (tile_end): exactly the partial
        # rows the raster backward wrote
        off, te = b2.tile_off.long(), b2.tile_end.long()
        CT = off.numel() - 1
        I = int(off[-1])
        tile_of = torch.repeat_interleave(torch.arange(CT, device=cuda), off[1:] - off[:-1])
        used = torch.arange(I, device=cuda) < te[tile_of]
        touched = torch.zeros(N, dtype=torch.bool, device=cuda)
        touched[b2.sorted_ids[:I].long()[used] % N] = True
        assert cnt == int(touched.sum()) and cnt > 0, (cnt, int(touched.sum()))
        rows = gr.block[1:1 + cnt]
        n = rows[:, 0].contiguous().view(torch.int32).long()
        assert torch.equal(torch.sort(n).values, torch.nonzero(touched).flatten())
        assert torch.equal(rows[:, 2:], g_dense[n])                  # bitwise the dense rows
        mask = torch.ones(N, dtype=torch.bool, device=cuda)
        mask[n] = False
        assert float(g_dense[mask].abs().max()) == 0.0               # nothing outside the list
        blocks.append(gr.block.clone())
        dense.append(g_dense)
        print(f"[rows] share {r}: views {v0}-{v1 - 1} band {band}: {cnt} of {N} Gaussians touched")
    out = _scatter(torch.stack(blocks), N, N)
    ref = torch.zeros(N, 14, device=cuda)
    for g in dense:
        ref = ref + g
    assert torch.equal(out, ref)


def test_rows_backward_units_single_share_equals_dense(cuda):
    from gsr import render as R
    from gsr.multiview import GradRows, rows_backward_units
    p, V, K, W, H, vr, va = _scene(cuda)
    N, th = p.shape[0], (H + 15) // 16
    bg = torch.ones(3, device=cuda)

    def render_band_rows(q, Vs, Ks, band, gr):
        return R.render3d(q, Vs, Ks, W, H, bg, R.RenderOptions3D(band=band, grad_rows=gr))

    pg = p.clone().requires_grad_(True)
    rgb, alpha = R.render3d(pg, V, K, W, H, bg)
    torch.autograd.backward([rgb, alpha], [vr, va])
    got = rows_backward_units(render_band_rows, p, V, K, vr, va, th, GradRows(N, cuda))
    torch.cuda.synchronize()
    assert torch.equal(got, pg.grad)


def test_rows_capacity_overflow_is_nan(cuda):
    from gsr import _lib, render as R
    from gsr.multiview import GradRows, unit_shard
    p, V, K, W, H, vr, va = _scene(cuda)
    N, C, th = p.shape[0], V.shape[0], (H + 15) // 16
    v0, v1, band = unit_shard(C, th, 2, 0)
    probe = GradRows(N, cuda)
    _share(p, V, K, W, H, vr, va, v0, v1, band, probe)
    cnt = probe.count()
    small = GradRows(cnt // 2, cuda)
    _share(p, V, K, W, H, vr, va, v0, v1, band, small)
    assert small.count() == cnt                  # the header counts every touched Gaussian
    status = torch.zeros(1, dtype=torch.int32, device=cuda)
    out = _scatter(torch.stack([probe.block[:small.cap + 1], small.block]), small.cap, N, status)
    assert torch.isnan(out).all()
    assert int(status.item()) & 64, _lib.describe_overflow(int(status.item()))
    R.overflow_status(cuda, reset=True)


def test_rows_forward_overflow_poisons_exchange(cuda):
    """A bounded band share whose forward overflowed: the raster backward skips its
    rows, so gsr3d_touched_rows sets the block's header past the cap; the exchange then
    NaN-fills and reports GSR_OVF_EXCHANGE -- the only signal a captured step has, where no
    host check runs -- instead of a finite gradient without this rank's share."""
    from gsr import _lib, render as R
    from gsr.multiview import GradRows, unit_shard
    p, V, K, W, H, vr, va = _scene(cuda)
    N, C, th = p.shape[0], V.shape[0], (H + 15) // 16
    v0, v1, band = unit_shard(C, th, 2, 1)
    gr = GradRows(N, cuda)
    bg = torch.ones(3, device=cuda)

    def share(capacity):
        pg = p.detach().clone().requires_grad_(True)
        opts = R.RenderOptions3D(band=band, grad_rows=gr, capacity=capacity)
        rgb, alpha = R.render3d(pg, V[v0:v1], K[v0:v1], W, H, bg, opts)
        torch.autograd.backward([rgb, alpha], [vr[v0:v1], va[v0:v1]])
        torch.cuda.synchronize()

    share("exact")
    good = gr.count()
    assert 0 < good <= gr.cap
    key = R.last_stats()["_bins"].key
    h = dict(R._size_hint[key])
    R._size_hint[key] = dict(h, I=h["I"] // 4)
    try:
        with pytest.raises(R.CapacityOverflowError):
            share("bounded")   # eager: the backward's host check raises after enqueueing
    finally:
        R._size_hint[key] = h
    assert gr.count() > gr.cap, (gr.count(), gr.cap)
    status = torch.zeros(1, dtype=torch.int32, device=cuda)
    out = _scatter(torch.stack([gr.block]), gr.cap, N, status)
    assert torch.isnan(out).all()
    assert int(status.item()) & 64, _lib.describe_overflow(int(status.item()))
    R.overflow_status(cuda, reset=True)
    share("exact")   # the next call is sized exactly and lists the rows again
    assert gr.count() == good
