"""Box survivor masks (include/gsr.h ABI 14, `box_masks`).

The 3D quad forward stores, per 128-entry chunk and 4x4 pixel box, the mask of the chunk's
entries that survive its two culls (8x8 quadrant, then 4x4 box); the chunk backward lists each
box's entries from those masks, cut at the box's last composited entry, instead of culling the
chunk again.  The lists are the culls' lists without entries past every pixel of the box (whose
contributions are exact zeros), so the gradients equal the culling backward's up to the
association of a box's lane reduction (an entry can sit at another slot of its group of 7).
Scenes: the units test's 30k-Gaussian view pair and the race fixture's dense overlapping
clusters (entries shared by boxes at different list positions).
"""
import pytest
import torch

from _util import assert_close, forced_bwd_layout, forced_fwd_lanes

pytestmark = pytest.mark.gpu


def _masks_word():
    from gsr import _lib
    return _lib.BinStats.masks.offset // 4


def _scene_units(dev):
    from gsr.scenes import gaussians3d, ring_cameras
    W, H, C = 192, 170, 2
    p = gaussians3d(30000, 21)
    V, K = ring_cameras(C, W, H)
    return p.to(dev), V.to(dev), K.to(dev), W, H


def _scene_clusters(dev):
    from test_race_gpu import _cluster_scene3d
    W, H = 64, 64
    p, V, K = _cluster_scene3d(1500, W, H, 2, 2606)
    return p.to(dev), V.to(dev), K.to(dev), W, H


def _bwd(b, meta, vr, va, W, H, masks):
    from gsr import _lib, render as R
    bgc = meta[4]

    def raster(L, q, partial, stream):
        _lib.check(L.gsr3d_raster_bwd(q["rec"], q["sorted_ids"], q["tile_off"], q["tile_end"], q["chunk_base"],
                                      q["chunk_state"], q["chunk_list"], q["stats_dev"], b.n_chunks,
                                      b.chunk_entries, b.C, W, H, bgc.data_ptr(), q["final_T"], q["last"],
                                      vr.data_ptr(), va.data_ptr(), q["k_of_s"], partial.data_ptr(),
                                      q["box_masks"] if masks else None, stream), "gsr3d_raster_bwd")
    v = R.backward3d(b, meta, raster)
    torch.cuda.synchronize()
    return v.cpu()


@pytest.mark.parametrize("layout", [1, 2], ids=["k_raster_bwd", "k_raster_bwd_pair3d"])
@pytest.mark.parametrize("scene", ["units", "clusters"])
def test_box_masks_match_culls(cuda, scene, layout):
    from gsr import render as R
    p, V, K, W, H = _scene_units(cuda) if scene == "units" else _scene_clusters(cuda)
    # the quad forward (the masks' writer) and a chunk backward (their reader) at any shape
    with forced_bwd_layout(layout), forced_fwd_lanes(4):
        rgb, alpha, b, meta = R.debug_forward3d(p, V, K, torch.ones(3, device=cuda), W, H)
        st = b.pre.view("stats_dev", torch.int32).tolist()
        assert st[_masks_word()] & 4, "the forward wrote no box masks"
        g = torch.Generator().manual_seed(5)
        C = V.shape[0]
        vr = torch.randn(C, H, W, 3, generator=g).to(cuda)
        va = torch.randn(C, H, W, generator=g).to(cuda)
        culled = _bwd(b, meta, vr, va, W, H, masks=False)
        listed = _bwd(b, meta, vr, va, W, H, masks=True)
    assert torch.isfinite(listed).all()
    # the lists differ only by entries past every pixel of a box (exact zeros): the same sums,
    # up to the association of a box's lane reduction when its list starts earlier (an entry's
    # slot in its group of 7)
    ndiff = int((listed != culled).sum())
    print(f"[box masks, {scene}, layout {layout}] {ndiff} of {listed.numel()} gradient values differ from the culling backward")
    assert_close(listed, culled, rtol=1e-5, atol=1e-8 * float(culled.abs().max()), what="box-mask grads")


def test_masks_need_quad_forward(cuda):
    """The 16-lane forward (small calls) writes no masks: the stats bit stays clear, and the
    backward culls; rgb / alpha of the quad forward do not depend on whether it writes them."""
    from gsr import render as R
    p, V, K, W, H = _scene_units(cuda)
    with forced_fwd_lanes(16):
        _, _, b, _ = R.debug_forward3d(p, V, K, torch.ones(3, device=cuda), W, H)
        assert not b.pre.view("stats_dev", torch.int32).tolist()[_masks_word()] & 4
    with forced_fwd_lanes(4):
        rgb1, alpha1, b, _ = R.debug_forward3d(p, V, K, torch.ones(3, device=cuda), W, H)
        assert b.pre.view("stats_dev", torch.int32).tolist()[_masks_word()] & 4
        opts = R.RenderOptions3D()
        rgb2, alpha2, b2, _ = R._forward3d(p, V, K, torch.ones(3, device=cuda), W, H, opts, need_bwd=False)
        assert not b2.pre.view("stats_dev", torch.int32).tolist()[_masks_word()] & 4
    assert torch.equal(alpha1.cpu(), alpha2.cpu())
    assert_close(rgb1.cpu(), rgb2.cpu(), rtol=0, atol=0, what="rgb")


@pytest.mark.parametrize("layout", [1, 2], ids=["k_raster_bwd", "k_raster_bwd_pair3d"])
def test_box_masks_with_lazy_rerun(cuda, layout):
    """A lazily sorted list whose walk reaches the end of its sorted prefix is re-sorted whole and
    its tile rendered again (gsr3d_raster_fwd_lazy): the second walk must rewrite that tile's box
    masks for the final order.  The sort-class scene (lists of 1 023 to 8 192 entries) with lazy
    prefixes of 256 entries re-renders tiles; its gradients must equal the whole sort's bit for
    bit in both chunk layouts (the lists, and so the masks, are the same)."""
    from gsr import render as R
    from test_sort_classes_gpu import W as SW, H as SH, _lazy, _scene, _step
    p, V, K = (x.to(cuda) for x in _scene())
    with forced_bwd_layout(layout), forced_fwd_lanes(4):
        with _lazy(0, 4096):   # every list sorted whole
            ref = _step(p, V, K)
        with _lazy(1023, 256):
            _, _, b, _ = R.debug_forward3d(p, V, K, torch.ones(3, device=cuda), SW, SH)
            st = b.pre.view("stats_dev", torch.int32).tolist()
            assert st[_masks_word()] & 4, "the forward wrote no box masks"
            reran = int(b.pre.view("lazy", torch.int32)[3 * b.CT].item())
            print(f"[box masks, lazy, layout {layout}] {reran} tile(s) re-rendered after a whole re-sort")
            assert reran > 0, "no tile reached the end of its sorted prefix"
            lz = _step(p, V, K)
    for x, y, what in zip(ref, lz, ("rgb", "alpha", "grad")):
        assert torch.equal(x, y), what
    R.check_overflow(cuda)
