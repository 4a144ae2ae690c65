"""Deterministic synthetic scenes for the benchmark configs.

Host-side helpers only (CPU tensors); callers move them to the device.  Seeds follow the
survey: ``1000 + config#``.

* cameras: C views on a ring of radius 1.0 around the origin (the reference normalises its
  cameras to max distance 1, src/utils.py:99-100), elevation 30°, azimuth 2πc/C, OpenCV
  convention (x right, y down, z forward), world→camera ``viewmat`` [4,4];
  fx = fy = 0.9·W, cx = W/2, cy = H/2.
* 3D Gaussians, distribution A (model-like): means ~ U([−0.11,0.11]³) (half of ell=0.22),
  log_scales = −5.5 − ln(N/16000)/3 + N(0,0.3) (src/model.py:86,219 offset; max_n=16000),
  quats ~ N(0,1)⁴ raw, colors ~ U(0,1), logit_op ~ N(0,2); packed [N,14] in the
  src/gaussian_renderer.py:183-187 layout.
* 2D Gaussians (config 4): means ~ U([0,W)×[0,H)), log_s ~ N(0.4,0.3), rot ~ U(−π,π),
  colors ~ U(0,1), logit_op ~ N(0,2); packed [N,9] (src/gaussian_renderer.py:314-318).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch

__all__ = ["ring_cameras", "gaussians3d", "gaussians2d", "CONFIGS", "BenchConfig"]


def ring_cameras(C: int, width: int, height: int, radius: float = 1.0,
                 elevation_deg: float = 30.0, azimuth0: float = 0.0):
    """Return (viewmats [C,4,4], Ks [C,3,3]) float32."""
    el = math.radians(elevation_deg)
    views, Ks = [], []
    up = torch.tensor([0.0, 0.0, 1.0], dtype=torch.float64)
    for c in range(C):
        az = azimuth0 + 2.0 * math.pi * c / C
        p = radius * torch.tensor([math.cos(el) * math.cos(az), math.cos(el) * math.sin(az),
                                   math.sin(el)], dtype=torch.float64)
        f = -p / p.norm()
        x = torch.linalg.cross(f, up)
        x = x / x.norm()
        y = torch.linalg.cross(f, x)
        R = torch.stack([x, y, f], 0)
        V = torch.eye(4, dtype=torch.float64)
        V[:3, :3] = R
        V[:3, 3] = -R @ p
        views.append(V)
        K = torch.tensor([[0.9 * width, 0.0, width / 2.0],
                          [0.0, 0.9 * width, height / 2.0],
                          [0.0, 0.0, 1.0]], dtype=torch.float64)
        Ks.append(K)
    return torch.stack(views).float(), torch.stack(Ks).float()


def gaussians3d(N: int, seed: int, extent: float = 0.11) -> torch.Tensor:
    g = torch.Generator().manual_seed(seed)
    p = torch.empty(N, 14)
    p[:, 0:3] = (torch.rand(N, 3, generator=g) * 2.0 - 1.0) * extent
    p[:, 3:6] = -5.5 - math.log(max(N, 1) / 16000.0) / 3.0 + 0.3 * torch.randn(N, 3, generator=g)
    p[:, 6:10] = torch.randn(N, 4, generator=g)
    p[:, 10:13] = torch.rand(N, 3, generator=g)
    p[:, 13] = 2.0 * torch.randn(N, generator=g)
    return p


def gaussians2d(N: int, width: int, height: int, seed: int) -> torch.Tensor:
    g = torch.Generator().manual_seed(seed)
    p = torch.empty(N, 9)
    p[:, 0] = torch.rand(N, generator=g) * width
    p[:, 1] = torch.rand(N, generator=g) * height
    p[:, 2:4] = 0.4 + 0.3 * torch.randn(N, 2, generator=g)
    p[:, 4] = (torch.rand(N, generator=g) * 2.0 - 1.0) * math.pi
    p[:, 5:8] = torch.rand(N, 3, generator=g)
    p[:, 8] = 2.0 * torch.randn(N, generator=g)
    return p


@dataclass(frozen=True)
class BenchConfig:
    index: int
    mode: str          # "3d" | "2d"
    N: int
    width: int
    height: int
    views: int
    frames: int
    backward: bool

    @property
    def seed(self) -> int:
        return 1000 + self.index

    @property
    def name(self) -> str:
        return (f"cfg{self.index}:{self.mode}:N={self.N}:{self.width}x{self.height}:"
                f"views={self.views}" + (f"x{self.frames}frames" if self.frames > 1 else "") +
                (":fwd+bwd" if self.backward else ":fwd"))


# BASELINE.json "configs" (restated in SURVEY.md §0 / §8(d)); H = 1024 // downsample.
CONFIGS = {
    1: BenchConfig(1, "3d", 10_000, 192, 170, 1, 1, True),
    2: BenchConfig(2, "3d", 50_000, 288, 256, 1, 1, False),
    3: BenchConfig(3, "3d", 200_000, 576, 512, 6, 1, True),
    4: BenchConfig(4, "2d", 500_000, 576, 512, 6, 8, True),
    5: BenchConfig(5, "3d", 2_000_000, 1152, 1024, 6, 1, True),
}
