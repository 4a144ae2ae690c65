"""Backward work units of several sub-chunks (gsr_bin_caps.chunk_entries, include/gsr.h).

A unit of U list entries gets one chunk record per pixel in the forward and one workgroup in
the backward, which walks it back to front in 128-entry sub-chunks carrying each pixel's
transmittance and suffix term.  The forward's alpha does not depend on U (bitwise); its rgb
sums the entries' colours per chunk, so it is regrouped (fp32 rounding, 1e-6); the gradients
differ only by the fp32 rounding of T recovered through more divisions in a row (<= 2 ulps
per entry, checked at 1e-4 relative plus an absolute floor).  A backward called
with another U than the forward used is flagged (GSR_OVF_UNIT) and returns NaN gradients.
"""
import pytest
import torch

from _util import assert_close, grad_close

pytestmark = pytest.mark.gpu


class chunk_entries:
    def __init__(self, mode, n):
        self.mode, self.n = mode, n

    def __enter__(self):
        from gsr import render as R
        self.old = R._chunk_entries[self.mode]
        R.set_chunk_entries(self.mode, self.n)

    def __exit__(self, *exc):
        from gsr import render as R
        R.set_chunk_entries(self.mode, self.old)


def _scene3d(dev):
    from gsr.scenes import gaussians3d, ring_cameras
    W, H, C = 192, 170, 2
    p = gaussians3d(30000, 21)
    V, K = ring_cameras(C, W, H)
    g = torch.Generator().manual_seed(22)
    return (p.to(dev), V.to(dev), K.to(dev), W, H, torch.randn(C, H, W, 3, generator=g).to(dev),
            torch.randn(C, H, W, generator=g).to(dev))


def _run3d(p, V, K, W, H, vr, va):
    from gsr import render as R
    pg = p.clone().requires_grad_(True)
    rgb, alpha = R.render3d(pg, V, K, W, H, torch.ones(3, device=p.device))
    torch.autograd.backward([rgb, alpha], [vr, va])
    return rgb.detach().cpu(), alpha.detach().cpu(), pg.grad.cpu()


@pytest.mark.parametrize("units", [256, 512, 1024])
def test_3d_units_match_single_chunks(cuda, units):
    sc = _scene3d(cuda)
    with chunk_entries("3d", 128):
        ref = _run3d(*sc)
    with chunk_entries("3d", units):
        got = _run3d(*sc)
    assert torch.equal(ref[1], got[1])
    assert_close(got[0], ref[0], rtol=1e-6, atol=1e-6, what="rgb")
    grad_close(got[2], ref[2], what=f"3d grad, {units}-entry units")


@pytest.mark.parametrize("units", [256, 512, 1024, 4096])
def test_2d_units_match_default(cuda, units):
    from gsr import render as R
    from gsr.scenes import gaussians2d
    W, H = 160, 128
    p = torch.stack([gaussians2d(20000, W, H, 60 + f) for f in range(2)]).to(cuda)
    sets = (0, 0, 1)
    g = torch.Generator().manual_seed(61)
    vr = torch.randn(3, H, W, 3, generator=g).to(cuda)
    va = torch.randn(3, H, W, generator=g).to(cuda)
    bg = torch.ones(3, device=cuda)

    def run():
        pg = p.clone().requires_grad_(True)
        rgb, alpha = R.render2d_units(pg, sets, W, H, bg)
        torch.autograd.backward([rgb, alpha], [vr, va])
        return rgb.detach().cpu(), alpha.detach().cpu(), pg.grad.cpu()

    ref = run()   # default: 128-entry units (no sub-chunk loop)
    assert R.last_stats()["_bins"].chunk_entries == 128
    with chunk_entries("2d", units):
        got = run()
    assert torch.equal(ref[1], got[1])
    assert_close(got[0], ref[0], rtol=1e-6, atol=1e-6, what="rgb")
    grad_close(got[2], ref[2], what=f"2d grad, {units}-entry units")


def test_unit_mismatch_is_flagged(cuda):
    """A backward told 128-entry units after a 512-entry forward: NaN gradients + GSR_OVF_UNIT."""
    from gsr import _lib, render as R
    p, V, K, W, H, vr, va = _scene3d(cuda)
    R.overflow_status(cuda, reset=True)
    with chunk_entries("3d", 512):
        rgb, alpha, b, meta = R.debug_forward3d(p, V, K, torch.ones(3, device=cuda), W, H)
    assert b.chunk_entries == 512
    L = _lib.lib()
    q = b.p
    bgc = meta[4]

    def raster(L, q, partial, stream):
        _lib.check(L.gsr3d_raster_bwd(q["rec"], q["sorted_ids"], q["tile_off"], q["tile_end"], q["chunk_base"],
                                      q["chunk_state"], q["chunk_list"], q["stats_dev"], b.n_chunks, 128, b.C, W, H,
                                      bgc.data_ptr(), q["final_T"], q["last"], vr.data_ptr(), va.data_ptr(),
                                      q["k_of_s"], partial.data_ptr(), None, stream), "gsr3d_raster_bwd")
    v = R.backward3d(b, meta, raster)
    torch.cuda.synchronize()
    assert torch.isnan(v).all()
    st = b.pre.view("stats_dev", torch.int32).tolist()
    assert st[12] & 32, st
    # ... and reported to the sticky status word: check_overflow() raises
    with pytest.raises(R.CapacityOverflowError, match="chunk_entries differs"):
        R.check_overflow(cuda)


@pytest.mark.parametrize("lanes", [0, 1, 4, 16])
def test_forward_only_matches(cuda, lanes):
    """A render with no gradient needed writes no chunk records and skips the finalize; its
    rgb / alpha equal the training forward's bitwise, and the tile work (list entries read,
    the multi-GPU balancing weights) is the same."""
    from gsr import render as R
    from _util import forced_fwd_lanes
    p, V, K, W, H, vr, va = _scene3d(cuda)
    bg = torch.ones(3, device=cuda)
    with forced_fwd_lanes(lanes):
        pg = p.clone().requires_grad_(True)
        rgb, alpha = R.render3d(pg, V, K, W, H, bg)
        work = R.tile_work().clone()
        with torch.no_grad():
            rgb2, alpha2 = R.render3d(p, V, K, W, H, bg)
        assert not R.last_stats()["_bins"].need_bwd
        work2 = R.tile_work()
    assert torch.equal(rgb.detach(), rgb2) and torch.equal(alpha.detach(), alpha2)
    assert torch.equal(work, work2)


def test_forward_only_2d(cuda):
    from gsr import render as R
    from gsr.scenes import gaussians2d
    W, H = 96, 80
    p = gaussians2d(3000, W, H, 71).to(cuda)
    bg = torch.ones(3, device=cuda)
    pg = p.clone().requires_grad_(True)
    rgb, alpha = R.render2d(pg, W, H, bg)
    with torch.no_grad():
        rgb2, alpha2 = R.render2d(p, W, H, bg)
    assert torch.equal(rgb.detach(), rgb2) and torch.equal(alpha.detach(), alpha2)
