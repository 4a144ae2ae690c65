"""
Gaussian Renderer Module — MI355X drop-in for pose-splatter's ``src/gaussian_renderer.py``.

Same public surface as the reference (src/gaussian_renderer.py:23-616): the abstract
``GaussianRenderer`` (nn.Module + ABC, ``background_color`` buffer, ``set_background_color``),
``GaussianRenderer3D`` (P=14), ``GaussianRenderer2D`` (P=9, ``kernel_size`` /
``sigma_cutoff`` / ``batch_size`` attributes), ``create_renderer`` and the two
``NotImplementedError`` converters — with the same argument meanings, output shapes and
error messages.  The arithmetic runs in libgsr.so (hand-written gfx950 kernels, C ABI in
include/gsr.h) instead of gsplat (3D) or the dense PyTorch compositor (2D).

Differences a caller can observe:
  * no gsplat dependency, so ``GaussianRenderer3D.__init__`` never raises ImportError;
  * rendering needs a CUDA (ROCm/HIP) device; on a CPU tensor ``render`` raises a
    RuntimeError whose message contains "CUDA" (the reference's own tests accept that for
    3D, tests/test_gaussian_renderer.py:325-332).  The N == 0 case returns the background
    on any device, as in the reference (:299-311).
  * 2D compositing is tiled: contributions with opacity*exp(-q) < eps_cut (default 1e-8)
    outside a Gaussian's tile rect are dropped (the reference evaluates every pixel).
"""
__date__ = "November 2025"

from abc import ABC, abstractmethod
from typing import Tuple

import torch
import torch.nn as nn

try:  # package-relative when installed next to gsr/, absolute when used as a drop-in file
    from gsr import render as _gsr_render
except ImportError:  # pragma: no cover
    import importlib
    _gsr_render = importlib.import_module("gsr.render")


def _check_capacity(capacity: str) -> None:
    if capacity not in _gsr_render._MODES:
        raise ValueError(f"Unknown capacity '{capacity}'. Expected one of {list(_gsr_render._MODES)}.")


class GaussianRenderer(ABC, nn.Module):
    """Abstract base class for Gaussian renderers (src/gaussian_renderer.py:23-107)."""

    def __init__(self, width: int, height: int, device: str = "cuda"):
        super().__init__()
        self.width = width
        self.height = height
        self.device = device
        # Default black background; the model overwrites it with white (src/model.py:68,79)
        self.register_buffer('background_color', torch.zeros(3, device=device))

    @abstractmethod
    def get_num_params(self) -> int:
        """Return number of parameters per Gaussian."""

    @abstractmethod
    def render(
        self,
        gaussian_params: torch.Tensor,
        viewmat: torch.Tensor,
        K: torch.Tensor,
    ) -> Tuple[torch.Tensor, torch.Tensor]:
        """Render Gaussians: returns rgb [H, W, 3] and alpha [H, W]."""

    def set_background_color(self, color: torch.Tensor):
        """Set background color (RGB [3], values in [0, 1])."""
        if color.shape != (3,):
            raise ValueError(f"Expected color shape (3,), got {color.shape}")
        self.background_color.copy_(color.to(self.background_color.device))


class GaussianRenderer3D(GaussianRenderer):
    """3D Gaussian splatting on MI355X (replaces gsplat, src/gaussian_renderer.py:110-211).

    Parameters per Gaussian: 14 — means [0:3], log_scales [3:6], quats [6:10] (w,x,y,z),
    colors [10:13], logit opacity [13].  Activations exp / q/(|q|+1e-8) / clamp(0,1) /
    sigmoid are fused into the projection kernel, and so is their backward.

    ``radius_mode`` selects gsplat's per-Gaussian extent rule: ``"opacity_aabb"`` (gsplat
    >= 1.5, default) or ``"isotropic_3sigma"`` (gsplat <= 1.4).

    ``capacity`` (gsr.render): ``"auto"`` (default) sizes a training call's intersection
    buffers from the previous call of the same shape with no host wait and checks them in
    the backward (which raises ``CapacityOverflowError`` before any NaN gradient is
    returned); ``"exact"`` reads the intersection count back every forward, as gsplat does.
    """

    def __init__(self, width: int, height: int, device: str = "cuda", radius_mode: str = "opacity_aabb",
                 capacity: str = "auto"):
        super().__init__(width, height, device)
        modes = {"opacity_aabb": 0, "isotropic_3sigma": 1}
        if radius_mode not in modes:
            raise ValueError(f"Unknown radius_mode '{radius_mode}'. Expected one of {sorted(modes)}.")
        self.radius_mode = radius_mode
        _check_capacity(capacity)
        self.capacity = capacity
        self._opts = _gsr_render.RenderOptions3D(radius_mode=modes[radius_mode], capacity=capacity)

    def get_num_params(self) -> int:
        return 14

    def render(
        self,
        gaussian_params: torch.Tensor,
        viewmat: torch.Tensor,
        K: torch.Tensor,
    ) -> Tuple[torch.Tensor, torch.Tensor]:
        """gaussian_params [N,14], viewmat [4,4] or [C,4,4], K [3,3] or [C,3,3] →
        rgb [H,W,3] / [C,H,W,3], alpha [H,W] / [C,H,W] (not clamped, like the reference)."""
        if gaussian_params.shape[1] != 14:
            raise ValueError(
                f"Expected 14 parameters per Gaussian, got {gaussian_params.shape[1]}"
            )
        single = viewmat.dim() == 2
        viewmats = viewmat[None] if single else viewmat
        Ks = K[None] if K.dim() == 2 else K
        if Ks.shape[0] != viewmats.shape[0]:
            Ks = Ks.expand(viewmats.shape[0], 3, 3)
        C = viewmats.shape[0]
        if gaussian_params.shape[0] == 0:
            dev = gaussian_params.device
            rgb = torch.zeros(C, self.height, self.width, 3, device=dev) + \
                self.background_color.to(dev).view(1, 1, 1, 3)
            alpha = torch.zeros(C, self.height, self.width, device=dev)
            rgb = rgb + 0.0 * gaussian_params.sum()   # keep the autograd edge
        else:
            rgb, alpha = _gsr_render.render3d(gaussian_params, viewmats, Ks, self.width, self.height,
                                              self.background_color, self._opts)
        if single:
            return rgb[0], alpha[0]
        return rgb, alpha


class GaussianRenderer2D(GaussianRenderer):
    """2D Gaussian splatting on MI355X (replaces src/gaussian_renderer.py:214-427).

    Parameters per Gaussian: 9 — means_2d [0:2] (pixels, x=column, y=row), log_scales_2d
    [2:4], rotation [4] (radians), colors [5:8], logit opacity [8].  Compositing follows
    parameter index order with integer pixel centres, exactly like the reference.
    ``viewmat`` and ``K`` are ignored.  ``kernel_size``, ``sigma_cutoff`` and ``batch_size``
    are accepted and stored but, as in the reference's live path, unused.  ``capacity``: as
    for GaussianRenderer3D.
    """

    def __init__(
        self,
        width: int,
        height: int,
        device: str = "cuda",
        kernel_size: int = 5,
        sigma_cutoff: float = 3.0,
        batch_size: int = 1,
        eps_cut: float = 1e-8,
        capacity: str = "auto",
    ):
        super().__init__(width, height, device)
        self.kernel_size = kernel_size
        self.sigma_cutoff = sigma_cutoff
        self.batch_size = batch_size
        self.eps_cut = eps_cut
        _check_capacity(capacity)
        self.capacity = capacity

    def get_num_params(self) -> int:
        return 9

    def render(
        self,
        gaussian_params: torch.Tensor,
        viewmat: torch.Tensor,
        K: torch.Tensor,
    ) -> Tuple[torch.Tensor, torch.Tensor]:
        """gaussian_params [N,9] → rgb [H,W,3], alpha [H,W]."""
        if gaussian_params.shape[1] != 9:
            raise ValueError(
                f"Expected 9 parameters per Gaussian, got {gaussian_params.shape[1]}"
            )
        N = gaussian_params.shape[0]
        if N == 0:
            dev = gaussian_params.device
            canvas = torch.zeros((self.height, self.width, 3), device=dev, dtype=torch.float32)
            alpha_canvas = torch.zeros((self.height, self.width), device=dev, dtype=torch.float32)
            final_rgb = canvas + self.background_color.to(dev).view(1, 1, 3)
            return final_rgb, alpha_canvas
        return _gsr_render.render2d(gaussian_params, self.width, self.height, self.background_color,
                                    self.eps_cut, capacity=self.capacity)


def create_renderer(
    mode: str,
    width: int,
    height: int,
    device: str = "cuda",
    **kwargs
) -> GaussianRenderer:
    """Factory (src/gaussian_renderer.py:522-563): "2d" or "3d", case-insensitive.

    2D forwards ``**kwargs`` (kernel_size, sigma_cutoff, batch_size, eps_cut, capacity); 3D
    drops them like the reference, except ``radius_mode`` and ``capacity``, which only this
    implementation knows.
    """
    mode = mode.lower()

    if mode == "2d":
        return GaussianRenderer2D(width, height, device, **kwargs)
    elif mode == "3d":
        extra = {k: kwargs[k] for k in ("radius_mode", "capacity") if k in kwargs}
        return GaussianRenderer3D(width, height, device, **extra)
    else:
        raise ValueError(
            f"Unknown renderer mode: '{mode}'. Expected '2d' or '3d'."
        )


def convert_3d_to_2d_params(
    params_3d: torch.Tensor,
    viewmat: torch.Tensor,
    K: torch.Tensor,
) -> torch.Tensor:
    """Placeholder kept for API parity (src/gaussian_renderer.py:567-590)."""
    raise NotImplementedError("3D to 2D parameter conversion not yet implemented")


def convert_2d_to_3d_params(
    params_2d: torch.Tensor,
    depth: torch.Tensor,
    viewmat: torch.Tensor,
    K: torch.Tensor,
) -> torch.Tensor:
    """Placeholder kept for API parity (src/gaussian_renderer.py:593-616)."""
    raise NotImplementedError("2D to 3D parameter conversion not yet implemented")
