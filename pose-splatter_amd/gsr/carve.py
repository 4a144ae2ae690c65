"""Shape carving on the MI355X: a drop-in for pose-splatter's
ShapeCarver (src/shape_carver.py:304-374) without torch_scatter.

`ShapeCarver(ell, grid_size, K, E, volume_idx, device, volume_fill_color)(mask, rgb, center,
angle)` returns the same [4, n1, n2, n3] volume as the reference (mask occupancy averaged
over the two thresholds, then colour), computed by three libgsr kernels with no host
synchronisation (gsr_carve_volume).  The adaptive-camera path (adjust_principal_points_to_seed,
a host numpy routine) is not provided: adaptive=True raises NotImplementedError.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn

from ._lib import check, lib
from .render import _ptr, _require_device, _stream

__all__ = ["carve_volume", "create_3d_grid", "ShapeCarver"]


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
                 rgb: torch.Tensor, volume_fill_color: float = 0.45, nonvisible_weight: float = 0.25) -> torch.Tensor:
    """grid [n1,n2,n3,3] (un-posed), center [3], K [C,3,3], E [C,4,4] (any device; read on
    the host), mask [C,1,H,W], rgb [C,3,H,W] -> volume [4,n1,n2,n3] float32."""
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
    check(L.gsr_carve_volume(_ptr(g), nv, _ptr(ctr), float(angle), Kh.data_ptr(), Eh.data_ptr(), C, _ptr(m),
                             _ptr(im), H, W, float(volume_fill_color), float(nonvisible_weight), _ptr(ws),
                             ws.numel(), _ptr(out), _stream(dev)), "gsr_carve_volume")
    return out


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
            raise NotImplementedError("adaptive cameras (adjust_principal_points_to_seed) run on the host in the "
                                      "reference; not provided by the MI355X carver")
        return carve_volume(self.grid, center, angle, self._K_host, self._E_host, mask, rgb, self.volume_fill_color)
