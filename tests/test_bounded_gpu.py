"""Capacity-bounded (sync-free) renders: gsr_bin_caps / stats->overflow (include/gsr.h).

A bounded call sizes every buffer and grid from the previous call of the same shape and never
reads the stats back, so a step can be captured in a HIP graph.  Contract checked here:
* bounded == exact, bit for bit (3D all layouts incl. the split sort and the lazy depth order;
  2D multi-unit), forward and gradients;
* a bound that fails is caught on the device for each kind of bound (intersections, chunks,
  busy tiles, split-sort list length, lazily sorted tiles): rgb / alpha / v_params are NaN,
  the sticky status names the bound, check_overflow() raises, the next bounded call of the
  shape raises, and the next exact call renders correctly (the emission counters were left
  zero);
* a whole fwd+bwd step captured in a CUDA(HIP) graph replays to the eager result, also after
  the parameters change in place.
"""
import math

import pytest
import torch

from _util import forced_bwd_layout, forced_fwd_lanes

pytestmark = pytest.mark.gpu


def _scene3d(dev, N=20000, C=2, W=192, H=170, seed=11):
    from gsr.scenes import gaussians3d, ring_cameras
    p = gaussians3d(N, seed)
    V, K = ring_cameras(C, W, H)
    g = torch.Generator().manual_seed(seed + 1)
    vr = torch.randn(C, H, W, 3, generator=g).to(dev)
    va = torch.randn(C, H, W, generator=g).to(dev)
    return p.to(dev), V.to(dev), K.to(dev), W, H, vr, va


def _step3d(p, V, K, W, H, vr, va, capacity):
    from gsr import render as R
    bg = torch.ones(3, device=p.device)
    pg = p.detach().clone().requires_grad_(True)
    rgb, alpha = R.render3d(pg, V, K, W, H, bg, R.RenderOptions3D(capacity=capacity))
    torch.autograd.backward([rgb, alpha], [vr, va])
    return rgb.detach(), alpha.detach(), pg.grad


def _poison(dev, byte=0xFF):
    """Hand 0xFF-filled blocks (-1 words, NaN floats) to the caching allocator: the next
    arenas reuse them, so a kernel reading a slot no kernel of this call wrote shows up."""
    ts = [torch.full((1 << k,), byte, dtype=torch.uint8, device=dev) for k in range(10, 27) for _ in range(3)]
    del ts


def _same(a, b):
    return all(torch.equal(x, y) for x, y in zip(a, b))


@pytest.fixture(autouse=True)
def _clean_status(cuda):
    from gsr import render as R
    R.overflow_status(cuda, reset=True)
    yield
    R.overflow_status(cuda, reset=True)
    R._size_hint.clear()
    R._monitors.clear()


@pytest.mark.parametrize("lanes", [0, 1, 4, 16])
def test_bounded_equals_exact_3d(cuda, lanes):
    from gsr import render as R
    sc = _scene3d(cuda)
    with forced_fwd_lanes(lanes):
        ex = _step3d(*sc, capacity="exact")
        for _ in range(2):   # the first bounded call uses the exact call's bounds, the second its own
            _poison(cuda)
            bd = _step3d(*sc, capacity="bounded")
            torch.cuda.synchronize()
            assert _same(ex, bd)
    R.check_overflow(cuda)


def test_bounded_equals_exact_3d_pair_backward(cuda):
    """The two-pixels-per-lane backward (k_raster_bwd_pair3d) over a bounded grid: workgroups
    past the device's active-chunk count leave before reading anything (poisoned arenas)."""
    from gsr import render as R
    sc = _scene3d(cuda)
    with forced_bwd_layout(2):
        ex = _step3d(*sc, capacity="exact")
        for _ in range(2):
            _poison(cuda)
            bd = _step3d(*sc, capacity="bounded")
            torch.cuda.synchronize()
            assert _same(ex, bd)
    R.check_overflow(cuda)


def test_bounded_forward_only(cuda):
    """A bounded render with no gradient (no chunk records, so no chunk bound) equals the exact
    one, also when its bounds come from a training step of the same shape."""
    from gsr import render as R
    p, V, K, W, H, vr, va = _scene3d(cuda)
    bg = torch.ones(3, device=cuda)
    with torch.no_grad():
        ex = R.render3d(p, V, K, W, H, bg, R.RenderOptions3D(capacity="exact"))
        for _ in range(3):
            _poison(cuda)
            assert _same(ex, R.render3d(p, V, K, W, H, bg, R.RenderOptions3D(capacity="bounded")))
    _step3d(p, V, K, W, H, vr, va, "bounded")
    with torch.no_grad():
        assert _same(ex, R.render3d(p, V, K, W, H, bg, R.RenderOptions3D(capacity="bounded")))
    torch.cuda.synchronize()
    R.check_overflow(cuda)


def test_bounded_split_sort_and_lazy(cuda):
    """Few busy tiles (split sort) and long lists (lazy depth order) under bounds."""
    from gsr import _lib, render as R
    L = _lib.lib()
    # one view of a dense, close scene: few busy tiles with lists > 1024 (split sort)
    sc = _scene3d(cuda, N=30000, C=1, W=96, H=80, seed=3)
    ex = _step3d(*sc, capacity="exact")
    b = R.last_stats()["_bins"]
    assert b.n_busy <= 128 and b.max_seg > 1024, (b.n_busy, b.max_seg)
    _poison(cuda)   # the lazy re-render's list past its device count is stale (was: NaN tiles)
    assert _same(ex, _step3d(*sc, capacity="bounded"))
    # lazy: lists longer than 512 sorted to a 256-entry prefix, most tiles re-rendered
    _lib.check(L.gsr_set_lazy_sort(512, 256), "gsr_set_lazy_sort")
    try:
        sc = _scene3d(cuda, N=20000, C=2)
        R._size_hint.clear()
        ex = _step3d(*sc, capacity="exact")
        assert R.last_stats()["_bins"].n_lazy > 0
        _poison(cuda)
        assert _same(ex, _step3d(*sc, capacity="bounded"))
    finally:
        _lib.check(L.gsr_set_lazy_sort(16384, 4096), "gsr_set_lazy_sort")
    R.check_overflow(cuda)


def test_bounded_2d_units(cuda):
    from gsr import render as R
    from gsr.scenes import gaussians2d
    W, H = 96, 80
    p = torch.stack([gaussians2d(3000, W, H, 40 + f) for f in range(3)]).to(cuda)
    sets = (0, 0, 1, 2, 2)
    g = torch.Generator().manual_seed(9)
    vr = torch.randn(len(sets), H, W, 3, generator=g).to(cuda)
    va = torch.randn(len(sets), H, W, generator=g).to(cuda)
    bg = torch.ones(3, device=cuda)
    out = []
    for cap in ("exact", "bounded", "bounded"):
        pg = p.clone().requires_grad_(True)
        rgb, alpha = R.render2d_units(pg, sets, W, H, bg, capacity=cap)
        torch.autograd.backward([rgb, alpha], [vr, va])
        out.append((rgb.detach(), alpha.detach(), pg.grad))
    torch.cuda.synchronize()
    assert _same(out[0], out[1]) and _same(out[0], out[2])
    R.check_overflow(cuda)


def _shrunk(key_fn, **scale):
    from gsr import render as R
    (key,) = [k for k in R._size_hint if key_fn(k)]
    h = dict(R._size_hint[key])
    for k, f in scale.items():
        h[k] = int(h[k] * f)
    R._size_hint[key] = h
    return key


def _overflowing_step3d(p, V, K, W, H, vr, va):
    """A bounded training step whose forward overflows: NaN rgb / alpha, and the backward
    raises CapacityOverflowError before any gradient reaches .grad (ADVICE r3 / VERDICT r3)."""
    from gsr import render as R
    pg = p.detach().clone().requires_grad_(True)
    rgb, alpha = R.render3d(pg, V, K, W, H, torch.ones(3, device=p.device), R.RenderOptions3D(capacity="bounded"))
    torch.cuda.synchronize()
    assert torch.isnan(rgb).all() and torch.isnan(alpha).all()
    with pytest.raises(R.CapacityOverflowError):
        torch.autograd.backward([rgb, alpha], [vr, va])
    assert pg.grad is None
    return rgb


@pytest.mark.parametrize("bound,bit", [("I", 1), ("chunks", 2), ("busy", 4)])
def test_forced_overflow_3d(cuda, bound, bit):
    from gsr import _lib, render as R
    sc = _scene3d(cuda)
    ex = _step3d(*sc, capacity="exact")
    _shrunk(lambda k: True, **{bound: 0.25})
    _overflowing_step3d(*sc)
    bits = R.overflow_status(cuda)
    assert bits & bit, _lib.describe_overflow(bits)
    with pytest.raises(R.CapacityOverflowError):
        R.check_overflow(cuda)
    # the backward dropped the shape's bounds: the next call sizes exactly, and it is correct
    # (the emission counters were left zero); the one after is bounded again
    assert _same(ex, _step3d(*sc, capacity="bounded"))
    assert not R.last_stats()["_bins"].bounded
    assert _same(ex, _step3d(*sc, capacity="bounded"))
    assert R.last_stats()["_bins"].bounded
    R.check_overflow(cuda)


def test_forced_overflow_forward_only_next_call_raises(cuda):
    """No backward to check it: a forward-only bounded call that overflowed is reported by the
    next call of the shape, also when several calls were queued behind it unchecked (the
    monitors are a FIFO per shape)."""
    from gsr import render as R
    p, V, K, W, H, vr, va = _scene3d(cuda)
    bg = torch.ones(3, device=cuda)
    opts = R.RenderOptions3D(capacity="bounded")
    with torch.no_grad():
        ex = R.render3d(p, V, K, W, H, bg, R.RenderOptions3D(capacity="exact"))
        key = _shrunk(lambda k: True)
        good = dict(R._size_hint[key])
        R._size_hint[key] = dict(good, I=good["I"] // 8)
        torch.cuda.synchronize()
        torch.cuda._sleep(400_000_000)   # keep the GPU busy while the host queues the calls
        bad = R.render3d(p, V, K, W, H, bg, opts)   # overflows; nothing waits for it
        R._size_hint[key] = good
        later = [R.render3d(p, V, K, W, H, bg, opts) for _ in range(3)]   # queued behind it
        with pytest.raises(R.CapacityOverflowError):
            torch.cuda.synchronize()
            R.render3d(p, V, K, W, H, bg, opts)
    assert torch.isnan(bad[0]).all()
    assert all(_same(ex, o) for o in later)
    R.overflow_status(cuda, reset=True)


def test_forced_overflow_split_sort_segment(cuda):
    from gsr import render as R
    sc = _scene3d(cuda, N=30000, C=1, W=96, H=80, seed=3)
    _step3d(*sc, capacity="exact")
    b = R.last_stats()["_bins"]
    assert b.n_busy <= 128 and b.max_seg > 2200, (b.n_busy, b.max_seg)
    _shrunk(lambda k: True, max_seg=0.3)
    _overflowing_step3d(*sc)
    assert R.overflow_status(cuda, reset=True) & 8


def test_forced_overflow_lazy(cuda):
    """More lazily sorted tiles flagged by the forward than the re-render's grid covers.  The
    grid is the bound on lists of >= 8192 entries when min_len >= 8191 (else every busy tile),
    so this needs config 3's scene (lists up to ~12k entries) with min_len 8192."""
    from gsr import _lib, render as R
    L = _lib.lib()
    _lib.check(L.gsr_set_lazy_sort(8192, 256), "gsr_set_lazy_sort")
    try:
        sc = _scene3d(cuda, N=200000, C=6, W=576, H=512, seed=1003)
        _step3d(*sc, capacity="exact")
        b = R.last_stats()["_bins"]
        assert b.n_lazy > 0 and b.n_sort_big > 4, (b.n_lazy, b.n_sort_big)
        key = _shrunk(lambda k: True)
        R._size_hint[key]["big"] = 0   # the re-render covers 4 tiles (the margin)
        _overflowing_step3d(*sc)
        bits = R.overflow_status(cuda, reset=True)
        assert bits & 16, _lib.describe_overflow(bits)
    finally:
        _lib.check(L.gsr_set_lazy_sort(16384, 4096), "gsr_set_lazy_sort")


def test_forced_overflow_2d(cuda):
    from gsr import render as R
    from gsr.scenes import gaussians2d
    W, H = 96, 80
    p = gaussians2d(3000, W, H, 7).to(cuda)
    bg = torch.ones(3, device=cuda)
    pg = p.clone().requires_grad_(True)
    R.render2d(pg, W, H, bg, capacity="exact")   # (a training call: the bounds of the key)
    _shrunk(lambda k: True, I=0.2)
    pg = p.clone().requires_grad_(True)
    rgb, alpha = R.render2d(pg, W, H, bg, capacity="bounded")
    torch.cuda.synchronize()
    assert torch.isnan(rgb).all()
    with pytest.raises(R.CapacityOverflowError):
        (rgb.sum() + alpha.sum()).backward()
    assert pg.grad is None
    assert R.overflow_status(cuda, reset=True) & 1


def test_graph_capture_3d_step(cuda):
    """A bounded fwd+bwd step captured once and replayed: equal to the eager step, also after
    the parameters are updated in place (the graph reads them at replay)."""
    from gsr import render as R
    p0, V, K, W, H, vr, va = _scene3d(cuda, N=20000, C=3)
    bg = torch.ones(3, device=cuda)
    params = p0.clone().requires_grad_(True)
    opts = R.RenderOptions3D(capacity="bounded")

    def step():
        params.grad = None
        rgb, alpha = R.render3d(params, V, K, W, H, bg, opts)
        torch.autograd.backward([rgb, alpha], [vr, va])
        return rgb, alpha

    _step3d(p0, V, K, W, H, vr, va, "exact")   # bounds for the shape
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            step()
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        g_rgb, g_alpha = step()
    g_grad = params.grad
    for k in range(3):
        with torch.no_grad():
            params.copy_(p0)
            params[:, 0:3] += 0.001 * k
        graph.replay()
        torch.cuda.synchronize()
        ref = _step3d(params.detach(), V, K, W, H, vr, va, "exact")
        assert _same(ref, (g_rgb, g_alpha, g_grad)), k
    R.check_overflow(cuda)
