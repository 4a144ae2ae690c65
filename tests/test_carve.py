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
    with pytest.raises(RuntimeError):
        sc(mask, rgb, torch.zeros(3), 0.0, adaptive=True)   # no CPU compute path (medoids on the device)
    with pytest.raises(RuntimeError):
        sc(mask, rgb, torch.zeros(3), 0.0)       # no CPU compute path


def test_oracle_adjust_principal_points_known_answer():
    """A seed at a known point, masks whose medoids are its exact projections: the DLT recovers
    the point and the principal points do not move."""
    import numpy as np
    from gsr.scenes import ring_cameras
    from oracle.carve import adjust_principal_points_to_seed
    C, H, W = 4, 60, 80
    V, K = ring_cameras(C, W, H)
    X = np.array([0.01, -0.02, 0.015])
    Kn, Vn = K.numpy().astype(np.float64), V.numpy().astype(np.float64)
    masks = np.zeros((C, H, W), dtype=np.float32)
    for c in range(C):
        Xc = Vn[c, :3, :3] @ X + Vn[c, :3, 3]
        u = Kn[c, 0, 0] * Xc[0] / Xc[2] + Kn[c, 0, 2]
        v = Kn[c, 1, 1] * Xc[1] / Xc[2] + Kn[c, 1, 2]
        Kn[c, 0, 2] += round(u) - u      # make the projection land on a pixel centre exactly
        Kn[c, 1, 2] += round(v) - v
        masks[c, int(round(v)) - 2:int(round(v)) + 3, int(round(u)) - 2:int(round(u)) + 3] = 1.0
    new, Xr, med = adjust_principal_points_to_seed(masks, Kn, Vn)
    assert np.allclose(Xr, X, atol=1e-9)
    assert np.allclose(new, Kn, atol=1e-6)


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


def _blob_masks(C, H, W, seed):
    """Silhouettes of an off-centre ellipsoid blob (the medoid differs from the image centre)."""
    from gsr.scenes import ring_cameras
    from oracle.carve import project_points_torch
    V, K = ring_cameras(C, W, H)
    g = torch.Generator().manual_seed(seed)
    pts = torch.randn(20000, 3, generator=g) * torch.tensor([0.03, 0.02, 0.025]) + torch.tensor([0.02, -0.01, 0.01])
    uv = project_points_torch(pts, K, V).round().long()
    mask = torch.zeros(C, 1, H, W)
    for c in range(C):
        mask[c, 0, uv[c, :, 1].clamp(0, H - 1), uv[c, :, 0].clamp(0, W - 1)] = 1.0
    return V, K, mask


@pytest.mark.gpu
@pytest.mark.parametrize("C,H,W,seed", [(6, 96, 128, 11), (4, 64, 64, 12), (3, 300, 411, 13)])
def test_medoids_and_adapted_cameras_vs_oracle(cuda, C, H, W, seed):
    """Device medoids == numpy's nonzero/mean/argmin; the adapted K and seed equal the reference
    routine's bit for bit (same float32 / float64 arithmetic on the host)."""
    import numpy as np
    from gsr.carve import adjust_principal_points_to_seed, mask_medoids
    from oracle.carve import adjust_principal_points_to_seed as ref_adjust
    V, K, mask = _blob_masks(C, H, W, seed)
    new_r, X_r, med_r = ref_adjust(mask[:, 0].numpy(), K.numpy(), V.numpy())
    med = mask_medoids(mask.to(cuda))
    assert np.array_equal(med, med_r), (med, med_r)
    new, X = adjust_principal_points_to_seed(mask.to(cuda), K.numpy(), V.numpy())
    assert new.dtype == np.float32 and np.array_equal(new, new_r)
    assert np.array_equal(X, X_r)
    # ties: a symmetric mask whose centroid is equidistant from several pixels -> lowest index
    sym = torch.zeros(1, 1, 8, 8)
    sym[0, 0, 2:4, 2:4] = 1.0
    assert np.array_equal(mask_medoids(sym.to(cuda)), np.array([[2.0, 2.0]]))
    with pytest.raises(ValueError, match="empty"):
        mask_medoids(torch.zeros(2, 1, 8, 8, device=cuda))


@pytest.mark.gpu
def test_carve_adaptive_vs_oracle(cuda):
    """ShapeCarver.forward(adaptive=True) == the reference branch restated: masks projected with
    the adapted intrinsics around the triangulated seed, colours with the carver's K."""
    import numpy as np
    from gsr.carve import ShapeCarver
    from oracle.carve import adjust_principal_points_to_seed as ref_adjust, shape_carver_forward
    C, H, W, n = 6, 96, 128, 32
    V, K, mask = _blob_masks(C, H, W, 14)
    rgb = torch.rand(C, 3, H, W, generator=torch.Generator().manual_seed(15))
    sc = ShapeCarver(0.18, n, K.numpy(), V.numpy(), device="cuda")
    out, temp_K = sc(mask.to(cuda), rgb.to(cuda), torch.zeros(3, device=cuda), 0.4, adaptive=True)
    new_r, X_r, _ = ref_adjust(mask[:, 0].numpy(), K.numpy(), V.numpy())
    assert torch.equal(temp_K.cpu(), torch.tensor(new_r).float())
    ref = shape_carver_forward(sc.grid.cpu(), K, V, mask, rgb, torch.tensor(X_r).float(), 0.4,
                               K_mask=torch.tensor(new_r).float())
    occ_diff = out[0].cpu() != ref[0]
    assert float(occ_diff.float().mean()) <= 1e-3, int(occ_diff.sum())
    assert float(ref[0].gt(0).float().mean()) > 0.001
    same = ~occ_diff
    assert_close(out.cpu()[1:][:, same], ref[1:][:, same], rtol=1e-5, atol=1e-6, max_frac=1e-3, max_outlier=1.0,
                 what="adaptive colours")
