"""HIP path (libgsr.so through the C ABI) vs the CPU oracle and the reference fixtures.

Tolerances (BASELINE.json north_star: 1e-4 relative fp32):
  * forward rgb/alpha: |a-e| <= 1e-4*|e| + 1e-6 (abs floor for near-zero background pixels)
  * gradients: |a-e| <= 1e-4*|e| + 1e-5*max|e| (abs floor scaled to the tensor: per-pixel
    sums are accumulated in a different order on the GPU)
  * integer work (tile lists, offsets, intersection counts): bit-exact.
3D discrete decisions (alpha >= 1/255 skip, T <= 1e-4 stop) can flip on fp32 ties between
two correct implementations; the large-scene tests allow a tiny fraction of flipped pixels
(bounded by one Gaussian's contribution) and report it.
"""
import math

import numpy as np
import pytest
import torch

from _util import assert_close, close_at_ties, grad_close, untie_cotangent

pytestmark = pytest.mark.gpu


def test_selftest_reduce64(cuda):
    """The transposed permlane/DPP butterfly reduction gives lane l the sum of value l."""
    from gsr import _lib
    out = torch.empty(64, device=cuda)
    _lib.check(_lib.lib().gsr_selftest_reduce64(out.data_ptr(), torch.cuda.current_stream().cuda_stream), "selftest")
    lanes = torch.arange(64, dtype=torch.float64)[:, None]
    i = torch.arange(64, dtype=torch.float64)[None, :]
    v = ((lanes * 7 + i * 13) % 97) + 0.25 * i
    assert torch.allclose(out.cpu().double(), v.sum(0), rtol=0, atol=1e-3), out


def test_selftest_reduce_box16(cuda):
    """The raster backward's per-box butterfly: lane l ends with the sums, over the 16 lanes
    of its box (equal lane bits 0-1), of values 4*(l>>2) .. 4*(l>>2)+3."""
    from gsr import _lib
    out = torch.empty(256, device=cuda)
    _lib.check(_lib.lib().gsr_selftest_reduce_box16(out.data_ptr(), torch.cuda.current_stream().cuda_stream),
               "selftest")
    lanes = torch.arange(64, dtype=torch.float64)[:, None]
    i = torch.arange(64, dtype=torch.float64)[None, :]
    v = ((lanes * 7 + i * 13) % 97) + 0.25 * i          # v[lane, value]
    exp = torch.empty(64, 4, dtype=torch.float64)
    for l in range(64):
        same_box = [m for m in range(64) if m % 4 == l % 4]
        for k in range(4):
            exp[l, k] = v[same_box, 4 * (l // 4) + k].sum()
    assert torch.allclose(out.cpu().double().view(64, 4), exp, rtol=0, atol=1e-3), out.view(64, 4)


def _b128_group(l):
    """ds_read_b128 lane group of lane l (MI355X_MICROARCH.md §LDS: {0-3,12-15,20-27}, ...)."""
    groups = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
              list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
    groups += [[x + 32 for x in g] for g in groups]
    return next(i for i, g in enumerate(groups) if l in g)


@pytest.mark.parametrize("box_lanes", [16, 8])
def test_selftest_reduce_grp(cuda, box_lanes):
    """The b128-group-aligned box reductions of the raster backward: every walk box lies inside
    one ds_read_b128 lane group; each box's positions and each output box's slots are a
    permutation; lane l's sums are the sums over the lanes of its output box."""
    from gsr import _lib
    G = 4 if box_lanes == 16 else 8
    out = torch.empty(64 * (G + 4), device=cuda)
    _lib.check(_lib.lib().gsr_selftest_reduce_grp(out.data_ptr(), box_lanes,
                                                  torch.cuda.current_stream().cuda_stream), "selftest")
    out = out.cpu().double()
    sums = out[:64 * G].view(64, G)
    meta = out[64 * G:].view(64, 4).long()
    walk, pos, obox, slot = (meta[:, k].tolist() for k in range(4))
    nbox = 64 // box_lanes
    for b in range(nbox):
        lanes = [l for l in range(64) if walk[l] == b]
        assert len(lanes) == box_lanes
        assert len({_b128_group(l) for l in lanes}) == 1, (b, lanes)
        assert sorted(pos[l] for l in lanes) == list(range(box_lanes))
        holders = [l for l in range(64) if obox[l] == b]
        assert sorted(slot[l] for l in holders) == list(range(64 // G))
    lanes_t = torch.arange(64, dtype=torch.float64)[:, None]
    i = torch.arange(64, dtype=torch.float64)[None, :]
    v = ((lanes_t * 7 + i * 13) % 97) + 0.25 * i
    exp = torch.empty(64, G, dtype=torch.float64)
    for l in range(64):
        members = [m for m in range(64) if walk[m] == obox[l]]
        for k in range(G):
            exp[l, k] = v[members, G * slot[l] + k].sum()
    assert torch.allclose(sums, exp, rtol=0, atol=1e-3), (sums - exp).abs().max()


def test_selftest_lds_order(cuda):
    """The tile sort ranks keys with returning LDS atomics, relying on same-address atomics of
    one wave instruction being applied in lane order."""
    from gsr import _lib
    out = torch.full((1,), -1, device=cuda, dtype=torch.int32)
    _lib.check(_lib.lib().gsr_selftest_lds_order(out.data_ptr(), torch.cuda.current_stream().cuda_stream),
               "selftest")
    assert int(out.item()) == 0


@pytest.fixture(params=[1, 4, 16, 0], ids=["box", "lanes4", "lanes16", "auto"])
def fwd_lanes(request, cuda):
    """Run a test under each forward layout (1 lane per pixel / one workgroup per tile, 4 / 4,
    16 / 16 -- 3D only; 2D runs the box layout for 16), forced through gsr_set_fwd_lanes, and the
    automatic choice (0: the only one that splits off heavy tiles, gsr_set_fwd_heavy);
    automatic selection afterwards."""
    from gsr import _lib
    _lib.check(_lib.lib().gsr_set_fwd_lanes(request.param), "gsr_set_fwd_lanes")
    yield request.param
    _lib.check(_lib.lib().gsr_set_fwd_lanes(0), "gsr_set_fwd_lanes")


@pytest.fixture(params=[1, 2], ids=["bwd1", "bwd2"])
def bwd_layout(request, cuda):
    """Run a 3D test under each raster-backward layout (1: one pixel per lane, 4-wave chunk
    workgroups; 2: two pixels per lane, 2-wave workgroups), forced through gsr_set_bwd_layout
    (the automatic choice takes 2 only for calls with >= 64 tiles per CU); automatic afterwards."""
    from gsr import _lib
    _lib.check(_lib.lib().gsr_set_bwd_layout(request.param), "gsr_set_bwd_layout")
    yield request.param
    _lib.check(_lib.lib().gsr_set_bwd_layout(0), "gsr_set_bwd_layout")


@pytest.fixture(params=[0, 6], ids=["heavy0", "heavy6"])
def fwd_heavy(request, cuda):
    """Run a 3D test without the forward's heavy-tile split (the default) and with it at 64
    entries (most busy tiles of a small scene take the 8-wave layout on the side stream, with
    the automatic layout), through gsr_set_fwd_heavy; off afterwards."""
    from gsr import _lib
    _lib.check(_lib.lib().gsr_set_fwd_heavy(request.param), "gsr_set_fwd_heavy")
    yield request.param
    _lib.check(_lib.lib().gsr_set_fwd_heavy(0), "gsr_set_fwd_heavy")


def _oracle3d():
    from oracle import oracle3d
    return oracle3d


def _scene3d(N, W, H, C, seed, extent=0.11, scale_shift=0.0):
    from gsr.scenes import gaussians3d, ring_cameras
    p = gaussians3d(N, seed, extent=extent)
    p[:, 3:6] += scale_shift
    V, K = ring_cameras(C, W, H)
    return p, V, K


def _run_gpu3d(p, V, K, W, H, bg, cuda, v_rgb=None, v_alpha=None, radius_mode="opacity_aabb"):
    from src.gaussian_renderer import GaussianRenderer3D
    # exact capacity: these tests change scenes within one shape (the drop-in's "auto" default
    # would size a later call from an earlier, smaller one and raise; tests/test_headline_mode_gpu.py)
    r = GaussianRenderer3D(W, H, device="cuda", radius_mode=radius_mode, capacity="exact")
    r.set_background_color(bg.to(cuda))
    pg = p.to(cuda).requires_grad_(True)
    rgb, alpha = r.render(pg, V.to(cuda), K.to(cuda))
    grad = None
    if v_rgb is not None:
        ((rgb * v_rgb.to(cuda)).sum() + (alpha * v_alpha.to(cuda)).sum()).backward()
        grad = pg.grad.detach().cpu()
    return rgb.detach().cpu(), alpha.detach().cpu(), grad


def _run_oracle3d(p, V, K, W, H, bg, v_rgb=None, v_alpha=None, radius_mode=0):
    o = _oracle3d()
    pc = p.clone().requires_grad_(True)
    rgb, alpha = o.render3d(pc, V, K, W, H, bg, radius_mode=radius_mode)
    grad = None
    if v_rgb is not None:
        ((rgb * v_rgb).sum() + (alpha * v_alpha).sum()).backward()
        grad = pc.grad.detach()
    return rgb.detach(), alpha.detach(), grad


def _cot(C, H, W, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(C, H, W, 3, generator=g), torch.randn(C, H, W, generator=g)


@pytest.mark.parametrize("N,W,H,C,seed,shift", [
    (1, 32, 24, 1, 1, 2.0),
    (12, 40, 32, 1, 2, 2.5),
    (200, 48, 40, 2, 3, 1.0),
    (2000, 96, 80, 3, 4, 0.0),
])
def test_3d_small_vs_oracle(cuda, fwd_lanes, bwd_layout, fwd_heavy, N, W, H, C, seed, shift):
    p, V, K = _scene3d(N, W, H, C, seed, extent=0.05, scale_shift=shift)
    bg = torch.tensor([0.1, 0.5, 0.9])
    vr, va = _cot(C, H, W, seed + 100)
    rgb_g, a_g, g_g = _run_gpu3d(p, V, K, W, H, bg, cuda, vr, va)
    rgb_o, a_o, g_o = _run_oracle3d(p, V, K, W, H, bg, vr, va)
    assert_close(rgb_g, rgb_o, what="rgb")
    assert_close(a_g, a_o, what="alpha")
    grad_close(g_g, g_o, what="grad")


def test_3d_multiview_equals_single_views(cuda):
    W, H, C = 64, 48, 4
    p, V, K = _scene3d(3000, W, H, C, 7)
    bg = torch.ones(3)
    rgb_b, a_b, _ = _run_gpu3d(p, V, K, W, H, bg, cuda)
    for c in range(C):
        rgb_c, a_c, _ = _run_gpu3d(p, V[c:c + 1], K[c:c + 1], W, H, bg, cuda)
        assert torch.equal(rgb_b[c], rgb_c[0]) and torch.equal(a_b[c], a_c[0])


def test_3d_deterministic(cuda, fwd_lanes, bwd_layout, fwd_heavy):
    W, H, C = 96, 80, 2
    p, V, K = _scene3d(20000, W, H, C, 8)
    bg = torch.ones(3)
    vr, va = _cot(C, H, W, 9)
    r1 = _run_gpu3d(p, V, K, W, H, bg, cuda, vr, va)
    r2 = _run_gpu3d(p, V, K, W, H, bg, cuda, vr, va)
    for a, b in zip(r1, r2):
        assert torch.equal(a, b)


@pytest.mark.parametrize("heavy", [0, 6, 10, 12])
def test_3d_heavy_tiles_vs_oracle(cuda, heavy):
    """Long lists whose pixels never saturate (low opacity, a dense cluster: the walks that set
    the quad forward's span).  With the heavy-tile split on (lists >= 2^heavy entries, up to 64
    tiles in the 8-wave layout on the side stream) the render and gradient match the oracle, and
    the split's tile count is the device's (gsr_bin_stats.n_heavy)."""
    from gsr import _lib, render as R
    _lib.check(_lib.lib().gsr_set_fwd_heavy(heavy), "gsr_set_fwd_heavy")
    try:
        W, H, C = 64, 48, 1
        p, V, K = _scene3d(12000, W, H, C, 31, extent=0.02)
        p[:, 13] = -3.5   # opacity ~0.03: the pixels stay live through lists of thousands of entries
        bg = torch.tensor([0.2, 0.4, 0.6])
        vr, va = _cot(C, H, W, 32)
        rgb_g, a_g, g_g = _run_gpu3d(p, V, K, W, H, bg, cuda, vr, va)
        b = R.last_stats()["_bins"]
        st = b.pre.view("stats_dev", torch.int32)[:20].cpu()
        n_heavy, max_seg = int(st[18]), int(st[2])
        assert max_seg > 2048, max_seg
        if heavy:
            # lists >= 2^b for the smallest b >= heavy leaving at most 64 tiles (a set fixed by the
            # list lengths: the cap never depends on the busy order's arrival order)
            lens = (b.tile_off[1:] - b.tile_off[:-1]).cpu()
            exp = next(int((lens >= 2 ** k).sum()) for k in range(heavy, 33) if int((lens >= 2 ** k).sum()) <= 64)
            assert n_heavy == exp and n_heavy <= 64, (n_heavy, exp, heavy)
            assert n_heavy > 0 or heavy > 11, (n_heavy, heavy)   # (lists here reach > 2048)
        else:
            assert n_heavy == 0
        rgb_o, a_o, g_o = _run_oracle3d(p, V, K, W, H, bg, vr, va)
        assert_close(rgb_g, rgb_o, what="rgb")
        assert_close(a_g, a_o, what="alpha")
        grad_close(g_g, g_o, what="grad")
        print(f"[heavy {heavy}] max list {max_seg}, {n_heavy} heavy tiles")
    finally:
        _lib.check(_lib.lib().gsr_set_fwd_heavy(0), "gsr_set_fwd_heavy")


def test_3d_binning_exact(cuda):
    """Tile lists are integer work: compare bit-exactly with a CPU re-sort of the GPU's own
    projection output (rect + depth bits), and the rects with the oracle's projection."""
    W, H, C = 192, 170, 2
    p, V, K = _scene3d(10000, W, H, C, 11)
    b = _check_binning_exact(p, V, K, W, H, C, cuda)
    N = p.shape[0]
    cnt = b.cnt.cpu().to(torch.int64)
    I = b.n_isect
    # projection rects vs the oracle's (float decisions: near-total agreement)
    o = _oracle3d()
    m, q, s, col, op = o.activations3d(p)
    pr = o.project3d(m, q, s, op, V, K, W, H)
    _, oids = o.isect_tiles(pr.means2d, pr.radii, pr.depths, W, H)
    agree = float((cnt.view(C, N) == 0).eq(~pr.valid).double().mean())
    assert agree > 0.999, agree
    assert abs(len(oids) - I) <= max(5, I // 2000)


@pytest.mark.parametrize("N,W,H,extent,dup", [(12000, 48, 40, 0.02, 1), (12000, 48, 40, 0.02, 2),
                                             (24000, 32, 32, 0.004, 2), (24000, 32, 32, 0.004, 3000)])
def test_3d_binning_exact_long_lists(cuda, N, W, H, extent, dup):
    """Lists of thousands of entries (the sample-partitioned group sort) and runs of `dup`
    Gaussians sharing one mean (equal depths: ties in c*N+n order, across group borders)."""
    p, V, K = _scene3d(N, W, H, 1, 23, extent=extent)
    src = (torch.arange(N) // dup) * dup
    p[:, 0:3] = p[src, 0:3]
    b = _check_binning_exact(p, V, K, W, H, 1, cuda)
    assert b.max_seg > 2048, b.max_seg


def _check_binning_exact(p, V, K, W, H, C, cuda):
    from gsr import render as R
    rgb, alpha, b, _ = R.debug_forward3d(p.to(cuda), V.to(cuda), K.to(cuda), torch.ones(3, device=cuda), W, H)
    N = p.shape[0]
    rect = b.rect.cpu().view(C * N, 2).to(torch.int64) & 0xFFFFFFFF
    x0, x1 = rect[:, 0] & 0xFFFF, rect[:, 0] >> 16
    y0, y1 = rect[:, 1] & 0xFFFF, rect[:, 1] >> 16
    cnt = b.cnt.cpu().to(torch.int64)
    assert torch.equal(cnt, (x1 - x0) * (y1 - y0))
    depth = b.depth.cpu()[:C * N].contiguous()
    tw, th = (W + 15) // 16, (H + 15) // 16
    T = tw * th
    # expected lists: (camera, tile) then (depth bits, c*N+n)
    keys = []
    for cn in torch.nonzero(cnt > 0).flatten().tolist():
        c = cn // N
        dbits = int(np.float32(depth[cn].item()).view(np.uint32))
        for ty in range(int(y0[cn]), int(y1[cn])):
            for tx in range(int(x0[cn]), int(x1[cn])):
                keys.append((c * T + ty * tw + tx, dbits, cn))
    keys.sort()
    exp_ids = torch.tensor([k[2] for k in keys], dtype=torch.int64)
    exp_tiles = torch.tensor([k[0] for k in keys], dtype=torch.int64)
    I = b.n_isect
    assert I == len(keys)
    assert torch.equal(b.sorted_ids.cpu()[:I].to(torch.int64), exp_ids)
    exp_off = torch.zeros(C * T + 1, dtype=torch.int64)
    exp_off[1:] = torch.cumsum(torch.bincount(exp_tiles, minlength=C * T), 0)
    assert torch.equal(b.tile_off.cpu().to(torch.int64), exp_off)
    # k_of_s: the emission entry of each sorted entry (a permutation).  The (c,n) ranges
    # [isect_offset, +count) tile [0, I) (workgroup arrival order), and emission entry
    # k = isect_offset[cn] + j belongs to Gaussian cn and to tile j (row-major) of its rect
    ks = b.k_of_s.cpu()[:I].to(torch.int64) & 0x0FFFFFFF   # bits 28..31: quadrant masks
    assert torch.equal(torch.sort(ks).values, torch.arange(I))
    off = b.isect_off.cpu()[:C * N].to(torch.int64)
    nz = cnt > 0
    o_s, perm = torch.sort(off[nz])
    c_s = cnt[nz][perm]
    assert int(o_s[0]) == 0 and torch.equal(o_s[1:], torch.cumsum(c_s, 0)[:-1]) and int(c_s.sum()) == I
    ids = b.sorted_ids.cpu()[:I].to(torch.int64)
    j = ks - off[ids]
    assert bool(((j >= 0) & (j < cnt[ids])).all())
    w = (x1 - x0)[ids]
    tile_of_j = (ids // N) * T + (y0[ids] + j // w) * tw + (x0[ids] + j % w)
    tiles_of_s = torch.searchsorted(exp_off, torch.arange(I), right=True) - 1
    assert torch.equal(tile_of_j, tiles_of_s)
    return b


def test_3d_cfg1_vs_oracle(cuda, fwd_lanes):
    """BASELINE config 1 scene (10k Gaussians, 192x170, 1 view) fwd+bwd vs the oracle."""
    from gsr.scenes import CONFIGS, gaussians3d, ring_cameras
    c = CONFIGS[1]
    p = gaussians3d(c.N, c.seed)
    V, K = ring_cameras(c.views, c.width, c.height)
    bg = torch.ones(3)
    vr, va = _cot(1, c.height, c.width, 5)
    # no outlier fraction: the forward may differ only at the oracle's discrete-
    # decision ties, which carry no cotangent, so the gradient compares with no exemption
    tie_pix, vr, va = untie_cotangent(p, V, K, c.width, c.height, vr, va)
    rgb_g, a_g, g_g = _run_gpu3d(p, V, K, c.width, c.height, bg, cuda, vr, va)
    rgb_o, a_o, g_o = _run_oracle3d(p, V, K, c.width, c.height, bg, vr, va)
    close_at_ties(rgb_g, rgb_o, tie_pix, what="rgb")
    close_at_ties(a_g, a_o, tie_pix, what="alpha")
    grad_close(g_g, g_o, what="grad")
    # PSNR of the rendering against the oracle render must agree to 0.05 dB vs any target
    tgt = (rgb_o + 0.05 * torch.randn(rgb_o.shape, generator=torch.Generator().manual_seed(1))).clamp(0, 1)
    psnr = lambda x: float(10 * torch.log10(1.0 / ((x - tgt) ** 2).mean()))
    assert abs(psnr(rgb_g) - psnr(rgb_o)) < 0.05


def test_3d_isotropic_radius_mode(cuda):
    W, H = 64, 48
    p, V, K = _scene3d(500, W, H, 1, 21, extent=0.05, scale_shift=1.0)
    p[0:6, 13] = -200.0        # sigmoid underflows to exactly 0: no 0/0 in dL/dopacity
    p[6:12, 13] = -7.0         # opacity < 1/255: never composited
    bg = torch.zeros(3)
    vr, va = _cot(1, H, W, 22)
    rgb_g, a_g, g_g = _run_gpu3d(p, V, K, W, H, bg, cuda, vr, va, radius_mode="isotropic_3sigma")
    rgb_o, a_o, g_o = _run_oracle3d(p, V, K, W, H, bg, vr, va, radius_mode=1)
    assert bool(torch.isfinite(g_g).all())
    assert float(g_g[0:12].abs().max()) == 0.0
    assert_close(rgb_g, rgb_o, what="rgb")
    grad_close(g_g, g_o, what="grad")


def test_3d_edge_cases(cuda, fwd_lanes, bwd_layout):
    W, H = 48, 40
    p, V, K = _scene3d(64, W, H, 1, 31, extent=0.05, scale_shift=1.5)
    bg = torch.tensor([0.2, 0.3, 0.4])
    # push some behind the camera, some far off-screen, some huge, one zero-opacity-ish
    cam_pos = -V[0, :3, :3].T @ V[0, :3, 3]
    p[0:8, 0:3] = cam_pos * 2.0           # behind the camera
    p[8:16, 0:3] = torch.tensor([5.0, 5.0, 5.0])
    p[16:20, 3:6] = -1.0                  # huge (covers the image)
    p[20:24, 13] = -8.0                   # opacity < 1/255: culled by the opacity-aware rule
    vr, va = _cot(1, H, W, 32)
    rgb_g, a_g, g_g = _run_gpu3d(p, V, K, W, H, bg, cuda, vr, va)
    rgb_o, a_o, g_o = _run_oracle3d(p, V, K, W, H, bg, vr, va)
    assert_close(rgb_g, rgb_o, what="rgb")
    grad_close(g_g, g_o, what="grad")
    # nothing visible at all → background, zero grads
    q = p.clone()
    q[:, 0:3] = cam_pos * 2.0
    rgb_g, a_g, g_g = _run_gpu3d(q, V, K, W, H, bg, cuda, vr, va)
    assert torch.allclose(rgb_g, bg.view(1, 1, 3).expand_as(rgb_g))
    assert float(a_g.abs().max()) == 0.0 and float(g_g.abs().max()) == 0.0


def test_3d_speculative_arena_regrow(cuda):
    """The emit is enqueued before the stats readback into an arena sized from the previous
    call of the same shapes; when this call's I does not fit, that emit must do nothing and
    the sort emits again: results equal a render with no size hint at all."""
    from gsr import render as R
    W, H, C = 96, 80, 2
    small, V, K = _scene3d(3000, W, H, C, 61, scale_shift=-2.0)
    big, _, _ = _scene3d(3000, W, H, C, 61, scale_shift=1.0)
    bg = torch.ones(3)
    vr, va = _cot(C, H, W, 62)
    R._size_hint.clear()
    _run_gpu3d(small, V, K, W, H, bg, cuda, vr, va)
    i_small = R.last_stats()["n_isect"]
    rgb1, a1, g1 = _run_gpu3d(big, V, K, W, H, bg, cuda, vr, va)
    assert R.last_stats()["n_isect"] > 1.25 * i_small + 1024   # beyond the speculative arena
    R._size_hint.clear()
    rgb2, a2, g2 = _run_gpu3d(big, V, K, W, H, bg, cuda, vr, va)
    assert torch.equal(rgb1, rgb2) and torch.equal(a1, a2) and torch.equal(g1, g2)
    rgb3, a3, g3 = _run_gpu3d(big, V, K, W, H, bg, cuda, vr, va)   # hint now fits: early emit
    assert torch.equal(rgb1, rgb3) and torch.equal(a1, a3) and torch.equal(g1, g3)


def test_3d_long_tile_lists(cuda, fwd_lanes, bwd_layout):
    """> 16384 entries in one tile list: exercises the run-sort + global merge path."""
    W, H = 32, 32
    N = 40000
    p, V, K = _scene3d(N, W, H, 1, 41, extent=0.004)
    p[:, 13] = -3.5                       # faint, so pixels terminate late
    bg = torch.zeros(3)
    vr, va = _cot(1, H, W, 42)
    tie_pix, vr, va = untie_cotangent(p, V, K, W, H, vr, va)
    from gsr import render as R
    rgb_g, a_g, g_g = _run_gpu3d(p, V, K, W, H, bg, cuda, vr, va)
    st = R.last_stats()
    assert st["max_seg"] > 16384, st
    rgb_o, a_o, g_o = _run_oracle3d(p, V, K, W, H, bg, vr, va)
    close_at_ties(rgb_g, rgb_o, tie_pix, what="rgb")
    grad_close(g_g, g_o, what="grad")


# ------------------------------------------------------------------------------------ 2D

def _golden(name):
    import os
    d = os.path.join(os.path.dirname(__file__), "golden")
    return np.load(os.path.join(d, f"ref2d_{name}.npz"))


GOLDEN_2D = ["n1_64x48_black", "n2_64x48_white", "n40_64x48_white", "n40_96x80_grey",
             "n256_96x80_white", "n256_96x80_dense", "n64_offscreen_64x48",
             "n2500_128x96_cfg4", "n5200_64x48_cfg4density"]


def _run_gpu2d(p, W, H, bg, cuda, v_rgb=None, v_alpha=None):
    from src.gaussian_renderer import GaussianRenderer2D
    r = GaussianRenderer2D(W, H, device="cuda", capacity="exact")
    r.set_background_color(bg.to(cuda))
    pg = p.to(cuda).requires_grad_(True)
    rgb, alpha = r.render(pg, None, None)
    grad = None
    if v_rgb is not None:
        ((rgb * v_rgb.to(cuda)).sum() + (alpha * v_alpha.to(cuda)).sum()).backward()
        grad = pg.grad.detach().cpu()
    return rgb.detach().cpu(), alpha.detach().cpu(), grad


@pytest.mark.parametrize("name", GOLDEN_2D)
def test_2d_vs_reference_golden(cuda, name):
    z = _golden(name)
    W, H = int(z["width"]), int(z["height"])
    p = torch.from_numpy(z["params"])
    bg = torch.from_numpy(z["background"])
    rgb, alpha, grad = _run_gpu2d(p, W, H, bg, cuda, torch.from_numpy(z["v_rgb"]), torch.from_numpy(z["v_alpha"]))
    assert_close(rgb, torch.from_numpy(z["rgb"]), what="rgb")
    assert_close(alpha, torch.from_numpy(z["alpha"]), what="alpha")
    grad_close(grad, torch.from_numpy(z["grad"]), what="grad")


def test_2d_kat_centre(cuda):
    z = np.load(__import__("os").path.join(__import__("os").path.dirname(__file__), "golden", "ref2d_kat_centre.npz"))
    rgb, alpha, _ = _run_gpu2d(torch.from_numpy(z["params"]), 256, 256, torch.zeros(3), cuda)
    assert abs(float(rgb[128, 128, 0]) - 0.8807970285415649) < 1e-6
    assert float(rgb[128, 128, 1]) == 0.0 and float(rgb[128, 128, 2]) == 0.0
    assert abs(float(alpha[0, 0]) - float(z["alpha_corner"])) < 1e-6


def _oracle2d(p, W, H, bg, vr, va):
    from oracle.oracle2d import render2d_dense
    pc = p.clone().requires_grad_(True)
    rgb, alpha = render2d_dense(pc, W, H, bg)
    ((rgb * vr).sum() + (alpha * va).sum()).backward()
    return rgb.detach(), alpha.detach(), pc.grad.detach()


# (70 x 45: ragged edge tiles -- the pair kernels' per-pixel image masks, rows r and r + 2)
@pytest.mark.parametrize("N,W,H,seed,mu", [(3000, 128, 96, 51, 0.4), (1500, 64, 64, 52, 1.8), (1200, 70, 45, 53, 0.8)])
def test_2d_vs_oracle_dense(cuda, fwd_lanes, N, W, H, seed, mu):
    from gsr.scenes import gaussians2d
    p = gaussians2d(N, W, H, seed)
    p[:, 2:4] += mu - 0.4
    bg = torch.ones(3)
    g = torch.Generator().manual_seed(seed)
    vr, va = torch.randn(H, W, 3, generator=g), torch.randn(H, W, generator=g)
    rgb, alpha, grad = _run_gpu2d(p, W, H, bg, cuda, vr, va)
    rgb_o, a_o, g_o = _oracle2d(p, W, H, bg, vr, va)
    assert_close(rgb, rgb_o, what="rgb")
    assert_close(alpha, a_o, what="alpha")
    grad_close(grad, g_o, what="grad")


def test_2d_saturation_and_long_lists(cuda, fwd_lanes):
    """Opaque stacks drive A to exactly 1.0f (exact early stop + division-free backward);
    > 2048-entry lists exercise several checkpoint chunks, > 16384 the merge sort."""
    W, H = 32, 32
    N = 20000
    g = torch.Generator().manual_seed(61)
    p = torch.empty(N, 9)
    p[:, 0:2] = 8.0 + torch.rand(N, 2, generator=g) * 16.0
    p[:, 2:4] = 1.0 + 0.3 * torch.randn(N, 2, generator=g)
    p[:, 4] = torch.rand(N, generator=g) * 6.28
    p[:, 5:8] = torch.rand(N, 3, generator=g)
    p[:, 8] = torch.randn(N, generator=g) * 3.0
    p[:50, 8] = 20.0                       # sigmoid == 1.0f exactly
    bg = torch.tensor([0.0, 1.0, 0.0])
    vr, va = torch.randn(H, W, 3, generator=g), torch.randn(H, W, generator=g)
    rgb, alpha, grad = _run_gpu2d(p, W, H, bg, cuda, vr, va)
    from gsr import render as R
    assert R.last_stats()["max_seg"] > 16384
    rgb_o, a_o, g_o = _oracle2d(p, W, H, bg, vr, va)
    assert_close(rgb, rgb_o, what="rgb")
    assert_close(alpha, a_o, what="alpha")
    grad_close(grad, g_o, what="grad")


def test_2d_deterministic(cuda):
    from gsr.scenes import gaussians2d
    W, H = 192, 160
    p = gaussians2d(30000, W, H, 71)
    g = torch.Generator().manual_seed(72)
    vr, va = torch.randn(H, W, 3, generator=g), torch.randn(H, W, generator=g)
    a = _run_gpu2d(p, W, H, torch.ones(3), cuda, vr, va)
    b = _run_gpu2d(p, W, H, torch.ones(3), cuda, vr, va)
    for x, y in zip(a, b):
        assert torch.equal(x, y)


@pytest.mark.gpu
def test_3d_band_sharding(cuda):
    """Multi-GPU (view, row)-unit sharding on one device: each rank's share
    renders only the views it touches, binned to its global rows; those rows are bitwise the
    full render's rows, and the shares' gradients (bucketed projection backward with a
    gradient hook, as the all-reduce path uses it) sum to the full gradient."""
    from gsr.render import RenderOptions3D, render3d
    from gsr.multiview import unit_shard
    W, H, C = 96, 80, 3
    p, V, K = _scene3d(20000, W, H, C, 21)
    bg = torch.ones(3, device=cuda)
    vr, va = _cot(C, H, W, 22)
    vr, va = vr.to(cuda), va.to(cuda)
    pf = p.to(cuda).requires_grad_(True)
    rgb_f, a_f = render3d(pf, V.to(cuda), K.to(cuda), W, H, bg)
    torch.autograd.backward([rgb_f, a_f], [vr, va])
    th = (H + 15) // 16
    total = torch.zeros_like(pf)
    for world in (4, 7):
        total.zero_()
        for r in range(world):
            v0, v1, band = unit_shard(C, th, world, r)
            if v1 == v0:
                continue
            pieces = []
            pb = p.to(cuda).requires_grad_(True)
            opts = RenderOptions3D(band=band, grad_buckets=3, grad_hook=pieces.append)
            rgb, a = render3d(pb, V[v0:v1].to(cuda), K[v0:v1].to(cuda), W, H, bg, opts)
            for c in range(v0, v1):
                y0 = min(max(band[0] - (c - v0) * th, 0), th)
                y1 = min(max(band[1] - (c - v0) * th, 0), th)
                rows = slice(16 * y0, min(H, 16 * y1))
                assert torch.equal(rgb[c - v0, rows], rgb_f[c, rows]) and torch.equal(a[c - v0, rows], a_f[c, rows])
            torch.autograd.backward([rgb, a], [vr[v0:v1], va[v0:v1]])
            assert len(pieces) == 3 and torch.equal(torch.cat(pieces), pb.grad)
            total += pb.grad
        grad_close(total.cpu(), pf.grad.cpu(), what=f"unit-summed grad, world {world}")


def test_3d_two_streams(cuda):
    """Renders of the same shapes on two streams do not share the projection's tile-count
    buffer: interleaved fwd+bwd on streams A and B equal the single-stream results."""
    from gsr import render as R
    W, H, C = 96, 80, 2
    pa, V, K = _scene3d(3000, W, H, C, 71, extent=0.05)
    pb, _, _ = _scene3d(3000, W, H, C, 72, extent=0.05)
    bg = torch.ones(3, device=cuda)
    vr, va = _cot(C, H, W, 73)
    vr, va, Vd, Kd = vr.to(cuda), va.to(cuda), V.to(cuda), K.to(cuda)

    def run(p):
        pg = p.to(cuda).requires_grad_(True)
        rgb, alpha = R.render3d(pg, Vd, Kd, W, H, bg)
        torch.autograd.backward([rgb, alpha], [vr, va])
        return rgb.detach().clone(), pg.grad.detach().clone()

    ref_a, ref_b = run(pa), run(pb)
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    outs = []
    for _ in range(3):
        with torch.cuda.stream(sa):
            oa = run(pa)
        with torch.cuda.stream(sb):
            ob = run(pb)
        outs.append((oa, ob))
    torch.cuda.synchronize()
    for oa, ob in outs:
        assert torch.equal(oa[0], ref_a[0]) and torch.equal(oa[1], ref_a[1])
        assert torch.equal(ob[0], ref_b[0]) and torch.equal(ob[1], ref_b[1])
