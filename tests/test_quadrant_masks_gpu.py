"""3D quadrant masks (include/gsr.h gsr_bin_emit `rec`, gsr3d_raster_fwd `k_of_s`).

The emission stores, for every (Gaussian, tile) list entry, which 8x8 quadrants of the tile
the entry can reach (the raster's exact cull, csrc/gsr_common.h cull_keep, evaluated by the
emission on the same record and the same box bounds) in bits 28..31 of its emission index;
the raster forward's quadrant workgroups then gather only the entries of their quadrant.  An
entry whose bit is clear has alpha < 1/255 at every pixel of that quadrant, so the compositor
would have skipped it anyway: rgb, alpha and the gradients must be the SAME BITS with the masks
on and off, for every forward layout, with the lazy depth order, in bounded mode and at
config 3's full size.  The masks also have to agree with the cull they replace: a set bit for
every quadrant a CPU restatement of the test keeps by a clear margin.
"""
import pytest
import torch

from _util import forced_fwd_lanes

pytestmark = pytest.mark.gpu


class _masks:
    def __init__(self, on):
        self.on = on

    def __enter__(self):
        from gsr import render as R
        self.old = R._quadrant_masks
        R.set_quadrant_masks(self.on)

    def __exit__(self, *exc):
        from gsr import render as R
        R.set_quadrant_masks(self.old)


def _scene(dev, N=20000, C=2, W=192, H=170, seed=13):
    from gsr.scenes import gaussians3d, ring_cameras
    p = gaussians3d(N, seed)
    V, K = ring_cameras(C, W, H)
    g = torch.Generator().manual_seed(seed + 1)
    return (p.to(dev), V.to(dev), K.to(dev), W, H, torch.randn(C, H, W, 3, generator=g).to(dev),
            torch.randn(C, H, W, generator=g).to(dev))


def _step(p, V, K, W, H, vr, va, capacity="exact"):
    from gsr import render as R
    pg = p.clone().requires_grad_(True)
    rgb, alpha = R.render3d(pg, V, K, W, H, torch.ones(3, device=p.device), R.RenderOptions3D(capacity=capacity))
    torch.autograd.backward([rgb, alpha], [vr, va])
    torch.cuda.synchronize()
    return rgb.detach(), alpha.detach(), pg.grad, R.last_stats()["_bins"]


def _same(a, b):
    return all(torch.equal(x, y) for x, y in zip(a[:3], b[:3]))


@pytest.mark.parametrize("lanes", [0, 4, 16])
def test_masks_do_not_change_a_bit(cuda, lanes):
    sc = _scene(cuda)
    with forced_fwd_lanes(lanes):
        with _masks(False):
            off = _step(*sc)
            assert not off[3].masks
        with _masks(True):
            on = _step(*sc)
            assert on[3].masks
            assert _same(off, on)
            on2 = _step(*sc, capacity="bounded")   # bounds from the call before
            assert on2[3].bounded and on2[3].masks
            assert _same(off, on2)


def test_masks_with_lazy_order(cuda):
    from gsr import _lib
    L = _lib.lib()
    sc = _scene(cuda)
    _lib.check(L.gsr_set_lazy_sort(512, 256), "gsr_set_lazy_sort")
    try:
        with _masks(False):
            off = _step(*sc)
        with _masks(True):
            on = _step(*sc)
        assert on[3].n_lazy > 0 and on[3].masks
        assert _same(off, on)
    finally:
        _lib.check(L.gsr_set_lazy_sort(16384, 4096), "gsr_set_lazy_sort")


def test_masks_match_the_cull(cuda):
    """Every list entry's mask vs a CPU restatement of cull_keep on its quadrants: a quadrant the
    restatement keeps with a margin must have its bit set, one it culls with a margin must not
    (decisions within 1e-4 of the threshold may differ by fp32 contraction)."""
    p, V, K, W, H, vr, va = _scene(cuda)
    with _masks(True):   # (off by default since round 4)
        _, _, _, b = _step(p, V, K, W, H, vr, va)
    assert b.masks
    I = b.n_isect
    off = b.tile_off.long()
    CT = off.numel() - 1
    tile = torch.repeat_interleave(torch.arange(CT, device=cuda), off[1:] - off[:-1])
    ids = b.sorted_ids[:I].long()
    mask = (b.k_of_s[:I].long() >> 28) & 0xF
    rec = b.rec.view(-1, 12)[ids].double()
    T = b.tw * b.th
    t = tile % T
    tx, ty = (t % b.tw).double(), (t // b.tw).double()
    x, y, Lc = rec[:, 0], rec[:, 1], rec[:, 3]
    a, bb, c, s1, s2 = rec[:, 4], rec[:, 5], rec[:, 6], rec[:, 7], rec[:, 11]
    pd = (a > 0) & (c > 0) & (4 * a * c > bb * bb)
    n_checked = 0
    for q in range(4):
        bx0 = 16 * tx + 8 * (q & 1) + 0.5
        by0 = 16 * ty + 8 * (q >> 1) + 0.5
        bx1, by1 = bx0 + 7, by0 + 7
        dxe = x - torch.minimum(torch.maximum(x, bx0), bx1)
        dye = y - torch.minimum(torch.maximum(y, by0), by1)
        dy1 = torch.minimum(torch.maximum(s1 * dxe, y - by1), y - by0)
        dx2 = torch.minimum(torch.maximum(s2 * dye, x - bx1), x - bx0)
        v = torch.minimum(a * dxe * dxe + bb * dxe * dy1 + c * dy1 * dy1, a * dx2 * dx2 + bb * dx2 * dye + c * dye * dye)
        thr = Lc * 1.001 + 1e-3
        keep_sure = (Lc >= 0) & (~pd | (v < thr - 1e-4 * (1 + thr.abs())))
        cull_sure = (Lc < 0) | (pd & (v > thr + 1e-4 * (1 + thr.abs())))
        bit = ((mask >> q) & 1).bool()
        assert bool(bit[keep_sure].all()), q
        assert not bool(bit[cull_sure].any()), q
        n_checked += int(keep_sure.sum() + cull_sure.sum())
    assert n_checked > 3.9 * I
    pop = sum(((mask >> q) & 1) for q in range(4)).double().mean()
    print(f"[masks] {I} entries, mean quadrants per entry {float(pop):.2f}")
    assert 0.5 < float(pop) < 4.0


def test_masks_fullsize_cfg3(cuda):
    """Config 3's whole 6-view step: the masked forward equals the unmasked one bitwise."""
    from gsr.scenes import CONFIGS, gaussians3d, ring_cameras
    c = CONFIGS[3]
    p = gaussians3d(c.N, c.seed).to(cuda)
    V, K = ring_cameras(c.views, c.width, c.height)
    g = torch.Generator().manual_seed(5)
    vr = torch.randn(c.views, c.height, c.width, 3, generator=g).to(cuda)
    va = torch.randn(c.views, c.height, c.width, generator=g).to(cuda)
    sc = (p, V.to(cuda), K.to(cuda), c.width, c.height, vr, va)
    with _masks(False):
        off = _step(*sc)
    with _masks(True):
        on = _step(*sc)
    assert on[3].masks and _same(off, on)
