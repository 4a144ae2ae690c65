"""Lazy depth order (gsr_bin_sort_lazy + gsr3d_raster_fwd_lazy, include/gsr.h).

Long tile lists are sorted only up to a depth prefix; a tile whose forward reaches the end of
its prefix is sorted whole and rendered again.  The outputs must equal those of the full sort
bit for bit (same entries, same order, same arithmetic), for every forward layout, with the
prefix so short that most tiles take the re-render path, with a prefix that some tiles
outrun, and with a prefix longer than every list.  The consumed part of every list (up to
tile_end) must be the exact stable depth order.
"""
import pytest
import torch

from _util import forced_fwd_lanes

pytestmark = pytest.mark.gpu


class lazy_sort:
    def __init__(self, min_len, prefix):
        self.args = (min_len, prefix)

    def __enter__(self):
        from gsr import _lib
        L = _lib.lib()
        self.prev = L.gsr_lazy_min_len()
        _lib.check(L.gsr_set_lazy_sort(*self.args), "gsr_set_lazy_sort")

    def __exit__(self, *exc):
        from gsr import _lib
        _lib.check(_lib.lib().gsr_set_lazy_sort(16384, 4096), "gsr_set_lazy_sort")


def _scene(dev):
    from gsr.scenes import gaussians3d, ring_cameras
    W, H, C = 192, 170, 2
    p = gaussians3d(20000, 11)
    V, K = ring_cameras(C, W, H)
    g = torch.Generator().manual_seed(5)
    vr = torch.randn(C, H, W, 3, generator=g).to(dev)
    va = torch.randn(C, H, W, generator=g).to(dev)
    return p.to(dev), V.to(dev), K.to(dev), W, H, vr, va


def _run(p, V, K, W, H, vr, va):
    from gsr import render as R
    dev = p.device
    bg = torch.ones(3, device=dev)
    pg = p.clone().requires_grad_(True)
    rgb, alpha = R.render3d(pg, V, K, W, H, bg)
    torch.autograd.backward([rgb, alpha], [vr, va])
    _, _, b, _ = R.debug_forward3d(p, V, K, bg, W, H)
    CT = b.CT
    start = b.tile_off[:-1].to(torch.int64)
    te = b.tile_end.to(torch.int64)
    n = int(b.n_isect)
    pos = torch.arange(n, device=dev)
    tile_of = torch.repeat_interleave(torch.arange(CT, device=dev), (b.tile_off[1:] - b.tile_off[:-1]).long())
    consumed = pos < te[tile_of]
    ids = torch.where(consumed, b.sorted_ids[:n].long(), -1)
    # k_of_s of a consumed entry = its emission index: the Gaussian's claimed offset (arrival
    # order of the projection's workgroups, so it differs between calls) + the tile's
    # row-major index in the Gaussian's rect
    N = p.shape[0]
    T = b.tw * b.th
    cn = ids[consumed]
    t = tile_of[consumed] % T
    assert bool((tile_of[consumed] // T == cn // N).all())
    r = b.rect.view(-1, 2).to(torch.int64)[cn] & 0xFFFFFFFF
    x0, x1, y0 = r[:, 0] & 0xFFFF, r[:, 0] >> 16, r[:, 1] & 0xFFFF
    kexp = b.isect_off.to(torch.int64)[cn] + (t // b.tw - y0) * (x1 - x0) + (t % b.tw - x0)
    assert torch.equal(b.k_of_s[:n].long()[consumed] & 0x0FFFFFFF, kexp), "k_of_s is not the emission index"
    flagged = int(b.lazy[3 * CT]) if getattr(b, "n_lazy", 0) else 0
    return (rgb.detach(), alpha.detach(), pg.grad.detach(), te.clone(), ids, b.tile_cut.clone()), flagged, b


@pytest.mark.parametrize("lanes", [4, 16, 1])
def test_lazy_equals_full_sort(cuda, lanes):
    p, V, K, W, H, vr, va = _scene(cuda)
    with forced_fwd_lanes(lanes):
        with lazy_sort(0, 1):
            ref, _, b0 = _run(p, V, K, W, H, vr, va)
        assert int(b0.max_seg) > 256, "the scene needs long lists"
        seen = {}
        for min_len, prefix in [(64, 8), (256, 200), (64, 100000)]:
            with lazy_sort(min_len, prefix):
                got, flagged, b = _run(p, V, K, W, H, vr, va)
            assert getattr(b, "n_lazy", 0) > 0, "lazy path not taken"
            seen[(min_len, prefix)] = flagged
            for name, x, y in zip(("rgb", "alpha", "v_params", "tile_end", "ids", "tile_cut"), ref, got):
                assert torch.equal(x, y), f"{name} differs (lanes {lanes}, min_len {min_len}, prefix {prefix})"
        print(f"[lazy] lanes {lanes}: tiles re-rendered per setting {seen}")
        assert seen[(64, 8)] > 0, "the 8-entry prefix must send tiles through the re-render"
        assert seen[(64, 100000)] == 0


def test_lazy_prefix_is_exact_order(cuda):
    """The sorted prefix of every lazily sorted list is the exact stable depth order of the
    tile's whole list (not just of the prefix's own entries)."""
    from gsr import render as R
    p, V, K, W, H, _, _ = _scene(cuda)
    bg = torch.ones(3, device=cuda)
    with lazy_sort(0, 1):
        _, _, b0, _ = R.debug_forward3d(p, V, K, bg, W, H)
        full = b0.sorted_ids[:b0.n_isect].clone()
    kept = 0
    for prefix in (200, 1000, 3000):
        with lazy_sort(64, prefix):
            _, _, b, _ = R.debug_forward3d(p, V, K, bg, W, H)
        CT = b.CT
        ts = b.lazy[:CT].to(torch.int64)
        off = b.tile_off.to(torch.int64)
        n = int(b.n_isect)
        pos = torch.arange(n, device=cuda)
        tile_of = torch.repeat_interleave(torch.arange(CT, device=cuda), (off[1:] - off[:-1]))
        busy = off[1:] > off[:-1]
        # the lists that stayed lazy keep a proper prefix; every consumed entry is inside it
        lazy_tiles = busy & (ts < off[1:])
        kept += int(lazy_tiles.sum())
        assert bool((b.tile_end.to(torch.int64)[lazy_tiles] < ts[lazy_tiles]).all())
        in_prefix = pos < ts[tile_of]
        assert torch.equal(b.sorted_ids[:n][in_prefix], full[in_prefix])
        print(f"[lazy] prefix {prefix}: {int(lazy_tiles.sum())} lists kept a partial sort, "
              f"{int(in_prefix.sum())} of {n} entries sorted")
    assert kept > 0


class emit_staged:
    def __init__(self, on):
        self.on = on

    def __enter__(self):
        from gsr import _lib
        _lib.check(_lib.lib().gsr_set_emit_staged(self.on), "gsr_set_emit_staged")

    def __exit__(self, *exc):
        from gsr import _lib
        _lib.check(_lib.lib().gsr_set_emit_staged(1), "gsr_set_emit_staged")


@pytest.mark.parametrize("kind", ["3d", "2d"])
def test_staged_emit_equals_scatter(cuda, kind):
    """LDS-staged emission (runs per tile) and the direct scatter claim the same slots up to
    the order inside a tile's bucket, which the per-tile sort removes: sorted lists, renders
    and gradients are bit-identical."""
    from gsr import render as R
    from gsr.scenes import gaussians2d
    outs = []
    for on in (0, 1):
        with emit_staged(on):
            if kind == "3d":
                p, V, K, W, H, vr, va = _scene(cuda)
                res, _, b = _run(p, V, K, W, H, vr, va)
                outs.append(res + (b.sorted_ids[:b.n_isect].clone(),))
            else:
                W, H = 96, 80
                q = gaussians2d(3000, W, H, 9).to(cuda).requires_grad_(True)
                bg = torch.zeros(3, device=cuda)
                rgb, alpha = R.render2d(q, W, H, bg)
                g = torch.Generator().manual_seed(2)
                torch.autograd.backward([rgb, alpha], [torch.randn(rgb.shape, generator=g).to(cuda),
                                                       torch.randn(alpha.shape, generator=g).to(cuda)])
                _, _, b, _ = R.debug_forward2d(q.detach(), bg, W, H)
                outs.append((rgb.detach(), alpha.detach(), q.grad.detach(), b.sorted_ids[:b.n_isect].clone()))
    for x, y in zip(*outs):
        assert torch.equal(x, y)


class split_sort:
    def __init__(self, on):
        self.on = on

    def __enter__(self):
        from gsr import _lib
        _lib.check(_lib.lib().gsr_set_split_sort(self.on), "gsr_set_split_sort")

    def __exit__(self, *exc):
        from gsr import _lib
        _lib.check(_lib.lib().gsr_set_split_sort(1), "gsr_set_split_sort")


def test_split_sort_equals_one_workgroup_sort(cuda):
    """Few busy tiles with long lists (BASELINE config 2's scene: 36 busy tiles, lists up to
    8 649): the block sorts + rank merge give exactly the one-workgroup-per-list order, and
    the same renders and gradients."""
    from gsr import render as R
    from gsr.scenes import CONFIGS, gaussians3d, ring_cameras
    c = CONFIGS[2]
    p = gaussians3d(c.N, c.seed).to(cuda)
    V, K = ring_cameras(c.views, c.width, c.height)
    V, K = V.to(cuda), K.to(cuda)
    g = torch.Generator().manual_seed(8)
    vr = torch.randn(c.views, c.height, c.width, 3, generator=g).to(cuda)
    va = torch.randn(c.views, c.height, c.width, generator=g).to(cuda)
    outs = []
    for on in (0, 1):
        with split_sort(on):
            res, _, b = _run(p, V, K, c.width, c.height, vr, va)
            assert b.n_busy <= 128 and b.max_seg > 1024, (b.n_busy, b.max_seg)
            outs.append(res + (b.sorted_ids[:b.n_isect].clone(),))
    for x, y in zip(*outs):
        assert torch.equal(x, y)
