"""Shape carving on the MI355X: a drop-in for pose-splatter's
ShapeCarver (src/shape_carver.py:304-374) without torch_scatter.

`ShapeCarver(ell, grid_size, K, E, volume_idx, device, volume_fill_color)(mask, rgb, center,
angle)` returns the same [4, n1, n2, n3] volume as the reference (mask occupancy averaged
over the two thresholds, then colour), computed by three libgsr kernels with no host
synchronisation (gsr_carve_volume).  With adaptive=True (src/shape_carver.py:328-335) the
principal points are moved so that the seed triangulated from the mask medoids projects
through each medoid (adjust_principal_points_to_seed, src/shape_carving.py:173-245): the
medoids come from libgsr (gsr_carve_medoids), the 2C x 4 DLT and its SVD stay on the host in
float64 as in the reference (one 4-byte-per-view read-back, where the reference copies the
masks to the host); it returns (volume, K_adapted) like the reference.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn

from ._lib import check, lib
from .render import _ptr, _require_device, _stream

__all__ = ["carve_volume", "create_3d_grid", "ShapeCarver", "mask_medoids", "adjust_principal_points_to_seed"]


def create_3d_grid(length, n, volume_idx=None):
    """src/shape_carving.py:10-18: n^3 points on [-length/2, length/2]^3 ('ij' order), cropped."""
    offset = np.linspace(-length / 2, length / 2, n)
    gx, gy, gz = np.meshgrid(offset, offset, offset, indexing="ij")
    pts = np.stack([gx, gy, gz], axis=-1)
    if volume_idx is not None:
        (i1, i2), (i3, i4), (i5, i6) = volume_idx
        pts = pts[i1:i2, i3:i4, i5:i6]
    return pts


def carve_volume(grid: torch.Tensor, center: torch.Tensor, angle: float, K, E, mask: torch.Tensor,
                 rgb: torch.Tensor, volume_fill_color: float = 0.45, nonvisible_weight: float = 0.25,
                 K_mask=None) -> torch.Tensor:
    """grid [n1,n2,n3,3] (un-posed), center [3], K [C,3,3], E [C,4,4] (any device; read on
    the host), mask [C,1,H,W], rgb [C,3,H,W] -> volume [4,n1,n2,n3] float32.  K_mask: the
    mask volume's intrinsics when they differ from K (the adaptive path); default K."""
    _require_device(rgb, "ShapeCarver")
    if grid.dim() != 4 or grid.shape[-1] != 3:
        raise ValueError(f"grid must be [n1,n2,n3,3], got {tuple(grid.shape)}")
    C, _, H, W = rgb.shape
    if rgb.shape[1] != 3 or mask.shape != (C, 1, H, W):
        raise ValueError(f"mask must be [C,1,H,W] and rgb [C,3,H,W]; got {tuple(mask.shape)}, {tuple(rgb.shape)}")
    Kh = torch.as_tensor(K, dtype=torch.float32).detach().cpu().contiguous()
    Eh = torch.as_tensor(E, dtype=torch.float32).detach().cpu().contiguous()
    if Kh.shape != (C, 3, 3) or Eh.shape != (C, 4, 4):
        raise ValueError(f"K must be [C,3,3] and E [C,4,4] with C={C}")
    Kmh = None
    if K_mask is not None:
        Kmh = torch.as_tensor(K_mask, dtype=torch.float32).detach().cpu().contiguous()
        if Kmh.shape != (C, 3, 3):
            raise ValueError(f"K_mask must be [C,3,3] with C={C}")
    L = lib()
    dev = rgb.device
    n1, n2, n3 = grid.shape[:3]
    nv = n1 * n2 * n3
    g = grid.detach().to(device=dev, dtype=torch.float32).reshape(-1, 3).contiguous()
    ctr = torch.as_tensor(center).detach().to(device=dev, dtype=torch.float32).reshape(3).contiguous()
    m = mask.detach().to(device=dev, dtype=torch.float32).contiguous()
    im = rgb.detach().to(dtype=torch.float32).contiguous()
    ws = torch.empty(int(L.gsr_carve_workspace(nv, C, H)) + 8, device=dev, dtype=torch.uint8)
    out = torch.empty(4, n1, n2, n3, device=dev, dtype=torch.float32)
    check(L.gsr_carve_volume(_ptr(g), nv, _ptr(ctr), float(angle), Kh.data_ptr(),
                             Kmh.data_ptr() if Kmh is not None else None, Eh.data_ptr(), C, _ptr(m),
                             _ptr(im), H, W, float(volume_fill_color), float(nonvisible_weight), _ptr(ws),
                             ws.numel(), _ptr(out), _stream(dev)), "gsr_carve_volume")
    return out


def mask_medoids(mask: torch.Tensor) -> np.ndarray:
    """[C,1,H,W] or [C,H,W] device masks -> float64 [C,2] (u*, v*) = (x, y) of each mask's medoid
    (the mask pixel nearest its centroid, first in row-major order on ties), computed by
    gsr_carve_medoids; one read-back of C int32.  An empty mask raises ValueError, as in the
    reference (src/shape_carving.py:203-206)."""
    _require_device(mask, "ShapeCarver")
    m = mask.detach()
    if m.dim() == 4:
        m = m[:, 0]
    if m.dim() != 3:
        raise ValueError(f"masks must be [C,1,H,W] or [C,H,W], got {tuple(mask.shape)}")
    m = m.to(torch.float32).contiguous()
    C, H, W = m.shape
    L = lib()
    dev = m.device
    ws = torch.empty(int(L.gsr_carve_medoids_workspace(C)) + 8, device=dev, dtype=torch.uint8)
    idx = torch.empty(C, device=dev, dtype=torch.int32)
    check(L.gsr_carve_medoids(_ptr(m), C, H, W, _ptr(ws), ws.numel(), _ptr(idx), _stream(dev)), "gsr_carve_medoids")
    flat = idx.cpu().numpy().astype(np.int64)
    for i in range(C):
        if flat[i] >= H * W:
            raise ValueError(f"Mask {i} is empty")
    return np.stack([flat % W, flat // W], axis=1).astype(np.float64)


def adjust_principal_points_to_seed(masks: torch.Tensor, Ks: np.ndarray, extrinsics: np.ndarray):
    """src/shape_carving.py:173-245 with the medoids from the device: the seed X is the DLT
    triangulation of the medoids (float64 SVD on the host, the 2C x 4 system of the reference),
    and each view's principal point moves so that X projects through its medoid.  Ks / extrinsics
    keep the caller's dtypes (float32 model cameras), so every product rounds as the reference's
    does.  Returns (new_Ks [C,3,3] in Ks' dtype, X [3] float64)."""
    C = len(Ks)
    assert Ks.shape == (C, 3, 3) and extrinsics.shape == (C, 4, 4)
    uv = mask_medoids(masks)
    rows = []
    for i in range(C):
        P = Ks[i] @ np.concatenate([extrinsics[i][:3, :3], extrinsics[i][:3, 3:]], axis=1)   # [3,4]
        rows.append(uv[i, 0] * P[2] - P[0])
        rows.append(uv[i, 1] * P[2] - P[1])
    _, _, vt = np.linalg.svd(np.vstack(rows))
    Xh = vt[-1]
    Xh /= Xh[3]
    X = Xh[:3]
    new_Ks = Ks.copy()
    for i in range(C):
        Xc = extrinsics[i][:3, :3] @ X + extrinsics[i][:3, 3]
        new_Ks[i, 0, 2] = uv[i, 0] - Ks[i, 0, 0] * (Xc[0] / Xc[2])
        new_Ks[i, 1, 2] = uv[i, 1] - Ks[i, 1, 1] * (Xc[1] / Xc[2])
    return new_Ks, X


class ShapeCarver(nn.Module):
    """Same constructor and forward as src/shape_carver.py:304-366."""

    def __init__(self, ell, grid_size, K, E, volume_idx=None, device="cuda", volume_fill_color=0.45):
        super().__init__()
        self.device = device
        self.volume_fill_color = volume_fill_color
        self.grid = torch.tensor(create_3d_grid(ell, grid_size, volume_idx=volume_idx)).to(device, torch.float32)
        self.K = torch.tensor(np.asarray(K)).to(device, torch.float32)
        self.E = torch.tensor(np.asarray(E)).to(device, torch.float32)
        self._K_host = self.K.cpu()
        self._E_host = self.E.cpu()
        self.C = len(K)

    def forward(self, mask, rgb, center, angle, adaptive=False):
        assert mask.ndim == 4   # [C,1,H,W]
        assert rgb.ndim == 4    # [C,3,H,W]
        assert len(mask) == self.C, f"{mask.shape}, {self.C}"
        assert len(rgb) == self.C, f"{rgb.shape}, {self.C}"
        if adaptive:
            # src/shape_carver.py:328-335, 370-371: masks projected with the adapted intrinsics,
            # colours sampled with the carver's own K; returns (volume, adapted K on the device)
            new_K, X = adjust_principal_points_to_seed(mask, self._K_host.numpy(), self._E_host.numpy())
            temp_K = torch.tensor(new_K).to(rgb.device, torch.float32)
            seed = torch.tensor(X).to(rgb.device, torch.float32)
            out = carve_volume(self.grid, seed, angle, self._K_host, self._E_host, mask, rgb, self.volume_fill_color,
                               K_mask=temp_K.cpu())
            return out, temp_K
        return carve_volume(self.grid, center, angle, self._K_host, self._E_host, mask, rgb, self.volume_fill_color)
