"""Shape carving: gsr.carve against the oracle restatement of
src/shape_carver.py (oracle/carve.py), including its scatter-min visibility.

Occupancy and visibility are integer decisions taken after float projections (rounded to
the nearest pixel): a voxel whose projection lands within rounding of a pixel boundary may
go either way between two fp32 implementations, so up to 1e-3 of the voxels may differ;
everything else matches to 1e-5."""
import math

import pytest
import torch

from _util import assert_close


def _scene(C=6, H=96, W=128, n=32, seed=0, flips=0.002):
    from gsr.scenes import ring_cameras
    from oracle.carve import project_points_torch
    V, K = ring_cameras(C, W, H)
    g = torch.Generator().manual_seed(seed)
    # silhouettes of an ellipsoid blob, plus a few flipped pixels for partial votes
    pts = torch.randn(20000, 3, generator=g) * torch.tensor([0.03, 0.02, 0.025])
    uv = project_points_torch(pts, K, V).round().long()
    mask = torch.zeros(C, 1, H, W)
    for c in range(C):
        x, y = uv[c, :, 0].clamp(0, W - 1), uv[c, :, 1].clamp(0, H - 1)
        mask[c, 0, y, x] = 1.0
    flip = torch.rand(C, 1, H, W, generator=g) < flips
    mask = torch.where(flip, 1.0 - mask, mask)
    rgb = torch.rand(C, 3, H, W, generator=g)
    from gsr.carve import create_3d_grid
    grid = torch.tensor(create_3d_grid(0.18, n)).float()
    return grid, K, V, mask, rgb


def test_carver_api_cpu():
    from gsr.carve import ShapeCarver
    grid, K, V, mask, rgb = _scene(C=3, n=8)
    sc = ShapeCarver(0.18, 8, K.numpy(), V.numpy(), device="cpu")
    assert sc.grid.shape == (8, 8, 8, 3) and sc.C == 3
    with pytest.raises(NotImplementedError):
        sc(mask, rgb, torch.zeros(3), 0.0, adaptive=True)
    with pytest.raises(RuntimeError):
        sc(mask, rgb, torch.zeros(3), 0.0)       # no CPU compute path


def test_oracle_scatter_min_ties_to_lowest_index():
    from oracle.carve import scatter_min
    src = torch.tensor([3.0, 1.0, 1.0, 2.0, 5.0])
    idx = torch.tensor([0, 0, 0, 1, 1])
    out, arg = scatter_min(src, idx, torch.full((3,), float("inf")))
    assert out.tolist()[:2] == [1.0, 2.0] and math.isinf(out[2])
    assert arg.tolist() == [1, 3, 5]


@pytest.mark.gpu
@pytest.mark.parametrize("C,n,angle,seed", [(6, 32, 0.0, 1), (6, 40, 0.9, 2), (4, 24, -2.2, 3)])
def test_carve_vs_oracle(cuda, C, n, angle, seed):
    from gsr.carve import carve_volume
    from oracle.carve import shape_carver_forward
    grid, K, V, mask, rgb = _scene(C=C, n=n, seed=seed)
    center = torch.tensor([0.004, -0.003, 0.002])
    out = carve_volume(grid.to(cuda), center.to(cuda), angle, K, V, mask.to(cuda), rgb.to(cuda)).cpu()
    ref = shape_carver_forward(grid, K, V, mask, rgb, center, angle)
    assert out.shape == ref.shape == (4, n, n, n)
    occ_diff = (out[0] != ref[0])
    assert float(occ_diff.float().mean()) <= 1e-3, int(occ_diff.sum())
    assert float(ref[0].gt(0).float().mean()) > 0.001          # the scene carves something
    same = ~occ_diff
    assert_close(out[1:][:, same], ref[1:][:, same], rtol=1e-5, atol=1e-6, max_frac=1e-3, max_outlier=1.0, what="colours")


@pytest.mark.gpu
def test_carve_deterministic(cuda):
    from gsr.carve import carve_volume
    grid, K, V, mask, rgb = _scene(C=6, n=48, seed=4)
    a = carve_volume(grid.to(cuda), torch.zeros(3, device=cuda), 0.3, K, V, mask.to(cuda), rgb.to(cuda))
    b = carve_volume(grid.to(cuda), torch.zeros(3, device=cuda), 0.3, K, V, mask.to(cuda), rgb.to(cuda))
    assert torch.equal(a, b)
