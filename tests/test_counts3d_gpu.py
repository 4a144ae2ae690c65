"""The 3D projection's isect_count is an optional output (include/gsr.h revision 14): with a
buffer it holds each (camera, Gaussian)'s entry count, the rect's area, which is what the
product path (NULL) derives on the host; and the rest of the call is the same either way."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_counts_written_match_rect_area(cuda):
    from gsr import render as R
    from gsr.scenes import gaussians3d, ring_cameras
    W, H = 192, 170
    p = gaussians3d(20000, 7).to(cuda)
    V, K = ring_cameras(3, W, H)
    V, K = V.to(cuda), K.to(cuda)
    bg = torch.ones(3, device=cuda)
    rgb0, alpha0, b0, _ = R.debug_forward3d(p, V, K, bg, W, H)
    derived = b0.cnt.cpu()
    try:
        R._counts3d = True
        rgb1, alpha1, b1, _ = R.debug_forward3d(p, V, K, bg, W, H)
        written = b1.pre.view("cnt", torch.int32).cpu()[:derived.numel()]
    finally:
        R._counts3d = False
    assert int((derived > 0).sum()) > 0
    assert torch.equal(written, derived)
    from gsr import _lib
    n_isect = b1.pre.view("stats_dev", torch.int64).tolist()[_lib.BinStats.n_isect.offset // 8]
    assert int(derived.to(torch.int64).sum()) == n_isect
    assert torch.equal(rgb0.cpu(), rgb1.cpu()) and torch.equal(alpha0.cpu(), alpha1.cpu())
