"""Multi-frame 2D batches: F frames' parameter sets rendered as
C (frame, view) units in ONE projection -> binning -> raster sequence (gsr.render.render2d_units).

Checks, on the GPU through the C ABI:
  * every unit's image is bitwise the single-frame render of its frame (the raster of a
    tile does not depend on the other units in the batch);
  * each frame's gradient equals the sum over its units of single-unit gradients (to fp32
    reordering), and is exactly zero for a frame with no unit;
  * one unit of the batch against the CPU oracle (oracle/oracle2d.py, pinned to the
    reference fixtures) at the reference tolerance.
"""
import pytest
import torch

from _util import assert_close, grad_close

pytestmark = pytest.mark.gpu


def _frames(F, N, W, H, seed):
    from gsr.scenes import gaussians2d
    return torch.stack([gaussians2d(N, W, H, seed + f) for f in range(F)])


# (0, 0, 1, 2, 2, 2): 6 cameras over 3 sets -> the per-set backward (k_raster2d_bwd_frame, two
# cameras per pass: set 2 takes a second pass, set 1 a padded one); (0, 0, 2, 2, 2): the same
# with a set no camera renders; (0, 2, 2) and (1,): one camera per set on average -> the
# per-camera backward (k_raster2d_bwd_pair); (1, 1, 1) and (1, 1, 2, 2): the launch sees only the
# rendered range of sets (one frame of three views: a frame owner's share), so the per-set path
# applies and the sets outside the range get zero gradients through autograd's slice
@pytest.mark.parametrize("sets", [(0, 0, 1, 2, 2, 2), (0, 0, 2, 2, 2), (0, 2, 2), (1,), (1, 1, 1), (1, 1, 2, 2)])
def test_units_match_single_renders(cuda, sets):
    from gsr import render as R
    F, N, W, H = 3, 1200, 96, 80
    P = _frames(F, N, W, H, 71)
    bg = torch.tensor([1.0, 0.5, 0.0])
    C = len(sets)
    g = torch.Generator().manual_seed(72)
    vr, va = torch.randn(C, H, W, 3, generator=g), torch.randn(C, H, W, generator=g)
    pb = P.to(cuda).requires_grad_(True)
    rgb, alpha = R.render2d_units(pb, sets, W, H, bg.to(cuda))
    assert rgb.shape == (C, H, W, 3) and alpha.shape == (C, H, W)
    torch.autograd.backward([rgb, alpha], [vr.to(cuda), va.to(cuda)])
    ref_grad = torch.zeros(F, N, 9, dtype=torch.float64)
    for c, f in enumerate(sets):
        ps = P[f].to(cuda).requires_grad_(True)
        r1, a1 = R.render2d(ps, W, H, bg.to(cuda))
        assert torch.equal(r1, rgb[c].detach()), f"unit {c} rgb differs from its single render"
        assert torch.equal(a1, alpha[c].detach()), f"unit {c} alpha differs from its single render"
        torch.autograd.backward([r1, a1], [vr[c].to(cuda), va[c].to(cuda)])
        ref_grad[f] += ps.grad.double().cpu()
    for f in range(F):
        if f not in sets:
            assert torch.count_nonzero(pb.grad[f]) == 0
        else:
            grad_close(pb.grad[f], ref_grad[f], rtol=1e-5, rel_floor=1e-6, what=f"frame {f} grad")


def test_unit_vs_oracle(cuda):
    from gsr import render as R
    from oracle.oracle2d import render2d_dense
    F, N, W, H = 2, 800, 64, 48
    P = _frames(F, N, W, H, 81)
    bg = torch.ones(3)
    sets = (0, 1, 1)
    g = torch.Generator().manual_seed(82)
    vr, va = torch.randn(3, H, W, 3, generator=g), torch.randn(3, H, W, generator=g)
    vr[1:2].zero_(), va[1:2].zero_()   # frame 1's gradient comes from unit 2 only
    vr[0].zero_(), va[0].zero_()       # frame 0 gets no cotangent
    pb = P.to(cuda).requires_grad_(True)
    rgb, alpha = R.render2d_units(pb, sets, W, H, bg.to(cuda))
    torch.autograd.backward([rgb, alpha], [vr.to(cuda), va.to(cuda)])
    po = P[1].clone().requires_grad_(True)
    rgb_o, a_o = render2d_dense(po, W, H, bg)
    ((rgb_o * vr[2]).sum() + (a_o * va[2]).sum()).backward()
    assert_close(rgb[2].detach(), rgb_o.detach(), what="unit 2 rgb")
    assert_close(alpha[1].detach(), a_o.detach(), what="unit 1 alpha")
    grad_close(pb.grad[1], po.grad, what="frame 1 grad")
    assert torch.count_nonzero(pb.grad[0]) == 0


@pytest.mark.parametrize("target", [160, 4608])
def test_split_set_backward_matches_whole_walks(cuda, target):
    """The split per-set backward (gsr_set_bwd2d_parts: each tile's list in unit-aligned parts,
    every part starting from the forward's suffix state at its end -- T anchor and colour planes)
    against the same call with whole-list walks (target 0), and both against the sum of the
    views' single-camera backward passes.  One frame of four views at 160x128 (80 tiles: 2 parts
    per tile at target 160, the cap of 16 at 4 608) over lists of ~10 128-entry units."""
    from gsr import render as R
    from gsr import _lib
    F, N, W, H = 2, 20000, 160, 128
    P = _frames(F, N, W, H, 91)
    bg = torch.tensor([0.2, 0.4, 0.9])
    sets = (1, 1, 1, 1)
    g = torch.Generator().manual_seed(92)
    vr, va = torch.randn(4, H, W, 3, generator=g), torch.randn(4, H, W, generator=g)
    L = _lib.lib()
    grads, imgs = [], []
    try:
        for t in (target, 0):
            assert L.gsr_set_bwd2d_parts(t) == 0
            pb = P.to(cuda).requires_grad_(True)
            rgb, alpha = R.render2d_units(pb, sets, W, H, bg.to(cuda))
            torch.autograd.backward([rgb, alpha], [vr.to(cuda), va.to(cuda)])
            grads.append(pb.grad.detach().cpu())
            imgs.append((rgb.detach().cpu(), alpha.detach().cpu()))
    finally:
        L.gsr_set_bwd2d_parts(_lib.BWD2D_PART_WORKGROUPS)
    assert R.last_stats().get("n_isect", 0) > 80 * 128 * 4, "lists too short to split"
    assert torch.equal(imgs[0][0], imgs[1][0]) and torch.equal(imgs[0][1], imgs[1][1])   # forward unchanged
    assert torch.count_nonzero(grads[0][0]) == 0
    grad_close(grads[0][1], grads[1][1].double(), rtol=1e-5, rel_floor=1e-6, what="split vs whole walks")
    ref = torch.zeros(N, 9, dtype=torch.float64)
    for c in range(4):
        ps = P[1].to(cuda).requires_grad_(True)
        r1, a1 = R.render2d(ps, W, H, bg.to(cuda))
        torch.autograd.backward([r1, a1], [vr[c].to(cuda), va[c].to(cuda)])
        ref += ps.grad.double().cpu()
    grad_close(grads[0][1], ref, rtol=1e-5, rel_floor=1e-6, what="split vs single-camera passes")


def test_layout_change_between_forward_and_backward_fails_loudly(cuda):
    """the split per-set backward (gsr_set_bwd2d_parts) starts its parts from colour
    planes the FORWARD writes only if it split too.  A setting changed between the two calls must
    not give silently wrong gradients: the forward records the planes in gsr_bin_stats.masks, and
    a backward that would read unwritten planes refuses -- NaN gradients, GSR_OVF_LAYOUT in the
    sticky status."""
    from gsr import _lib, render as R
    F, N, W, H = 1, 400, 64, 48
    P = _frames(F, N, W, H, 91)
    sets = (0, 0, 0)
    bg = torch.ones(3)
    g = torch.Generator().manual_seed(92)
    vr, va = torch.randn(3, H, W, 3, generator=g), torch.randn(3, H, W, generator=g)
    L = _lib.lib()
    R.overflow_status(cuda, reset=True)
    try:
        _lib.check(L.gsr_set_bwd2d_parts(0), "gsr_set_bwd2d_parts")        # forward: whole walks, no planes
        pb = P.to(cuda).requires_grad_(True)
        rgb, alpha = R.render2d_units(pb, sets, W, H, bg.to(cuda), capacity="exact")
        assert torch.isfinite(rgb).all()
        _lib.check(L.gsr_set_bwd2d_parts(_lib.BWD2D_PART_WORKGROUPS), "gsr_set_bwd2d_parts")   # backward: split
        torch.autograd.backward([rgb, alpha], [vr.to(cuda), va.to(cuda)])
        assert not bool(torch.isfinite(pb.grad).any()), "a split backward over unwritten planes must not compute"
        bits = R.overflow_status(cuda, reset=True)
        assert bits & 128, bits
        # the consistent calls (both split) are fine
        pb2 = P.to(cuda).requires_grad_(True)
        rgb2, alpha2 = R.render2d_units(pb2, sets, W, H, bg.to(cuda), capacity="exact")
        torch.autograd.backward([rgb2, alpha2], [vr.to(cuda), va.to(cuda)])
        assert torch.isfinite(pb2.grad).all() and R.overflow_status(cuda, reset=True) == 0
    finally:
        _lib.check(L.gsr_set_bwd2d_parts(_lib.BWD2D_PART_WORKGROUPS), "gsr_set_bwd2d_parts")


def test_lists_layout_change_between_projection_and_forward_fails_loudly(cuda, monkeypatch):
    """gsr2d_project_fwd bins only each set's first camera when the forward will share
    its lists (automatic layout).  A forward forced to another layout after that projection
    (gsr_set_fwd_lanes changed between the two calls) would render the other cameras from their
    own, empty, lists as background; it writes NaN there instead and flags GSR_OVF_LAYOUT."""
    from gsr import _lib, render as R
    F, N, W, H = 1, 400, 64, 48
    P = _frames(F, N, W, H, 93)
    real = _lib.lib()

    class Proxy:   # flips the forward layout between the projection and the raster forward
        def __getattr__(self, name):
            fn = getattr(real, name)
            if name != "gsr2d_raster_fwd":
                return fn

            def wrapped(*a):
                _lib.check(real.gsr_set_fwd_lanes(1), "gsr_set_fwd_lanes")
                return fn(*a)
            return wrapped

    monkeypatch.setattr(R, "lib", lambda: Proxy())
    R.overflow_status(cuda, reset=True)
    try:
        with torch.no_grad():
            rgb, alpha = R.render2d_units(P.to(cuda), (0, 0, 0), W, H, torch.ones(3, device=cuda), capacity="exact")
    finally:
        _lib.check(real.gsr_set_fwd_lanes(0), "gsr_set_fwd_lanes")
    assert torch.isfinite(rgb[0]).all()                         # the set's first camera renders its list
    bad = ~torch.isfinite(rgb[1:])
    assert bool(bad.any())                                      # the others: NaN where it has entries,
    assert bool((rgb[1:][~bad] == 1.0).all())                   # background only where it has none
    assert R.overflow_status(cuda, reset=True) & 128
