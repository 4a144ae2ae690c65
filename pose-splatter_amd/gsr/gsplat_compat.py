"""`gsplat.rendering.rasterization`-compatible entry point over libgsr.

pose-splatter calls gsplat directly in two places besides the renderer adapter:
`PoseSplatter.splat` (src/model.py:339-365) and the plotting helpers (src/plots.py:41-60,
93-112, 168-187).  They pass ACTIVATED inputs (scales = exp(.), opacities = sigmoid(.)),
`packed=False`, `render_mode="RGB"`, `rasterize_mode="classic"`, `sh_degree=None`,
`absgrad=True` (the meta dict is discarded by every caller), no `backgrounds` (the callers
add `(1-alpha)*bg` themselves) and `radius_clip` 2.0 (model) or the default 0.

This module takes that call unchanged and runs it on the MI355X kernels with
`input_mode=GSPLAT` (no exp / sigmoid / clamp; the quaternion is only renormalised, as
gsplat does).  To serve the unmodified callers, alias it before importing them:

    import sys, gsr.gsplat_compat as gc
    sys.modules.setdefault("gsplat", gc.gsplat_module())
    sys.modules.setdefault("gsplat.rendering", gc)

Supported: colors [N,3] (RGB), pinhole cameras, tile_size 16, classic mode, packed True or
False (same result), radius_clip, eps2d, near/far planes, optional backgrounds [C,3].
Anything else raises NotImplementedError instead of silently rendering something different.
"""
from __future__ import annotations

import types

import torch

from . import _lib
from .render import RenderOptions3D, _Render3D, _require_device

__all__ = ["rasterization", "gsplat_module"]


def rasterization(means, quats, scales, opacities, colors, viewmats, Ks, width, height,
                  near_plane=0.01, far_plane=1e10, radius_clip=0.0, eps2d=0.3, sh_degree=None,
                  packed=True, tile_size=16, backgrounds=None, render_mode="RGB", sparse_grad=False,
                  absgrad=False, rasterize_mode="classic", channel_chunk=32, distributed=False,
                  camera_model="pinhole", **kwargs):
    """Returns (render_colors [C,H,W,3], render_alphas [C,H,W,1], meta)."""
    unsupported = []
    if sh_degree is not None:
        unsupported.append("sh_degree (spherical harmonics colours)")
    if render_mode != "RGB":
        unsupported.append(f"render_mode={render_mode!r}")
    if rasterize_mode != "classic":
        unsupported.append(f"rasterize_mode={rasterize_mode!r}")
    if tile_size != 16:
        unsupported.append(f"tile_size={tile_size}")
    if camera_model != "pinhole":
        unsupported.append(f"camera_model={camera_model!r}")
    if distributed:
        unsupported.append("distributed=True (use gsr.multiview for view sharding)")
    if sparse_grad:
        unsupported.append("sparse_grad=True")
    for k, v in kwargs.items():
        if v is not None and v is not False:
            unsupported.append(f"{k}={v!r}")
    if colors.dim() != 2 or colors.shape[-1] != 3:
        unsupported.append(f"colors of shape {tuple(colors.shape)} (only [N,3] RGB)")
    if unsupported:
        raise NotImplementedError("gsr rasterization: unsupported " + ", ".join(unsupported))
    _require_device(means, "rasterization")
    N = means.shape[0]
    if not (quats.shape == (N, 4) and scales.shape == (N, 3) and opacities.shape == (N,)):
        raise ValueError(f"rasterization: expected means [N,3], quats [N,4], scales [N,3], opacities [N]; "
                         f"got {tuple(means.shape)}, {tuple(quats.shape)}, {tuple(scales.shape)}, "
                         f"{tuple(opacities.shape)}")
    C = viewmats.shape[0]
    # rows in the renderer's layout (mean, scale, quat, colour, opacity), activated values
    rows = torch.cat([means, scales, quats, colors, opacities[:, None]], dim=1).float()
    bg = torch.zeros(C, 3, device=means.device) if backgrounds is None else backgrounds.reshape(C, 3)
    opts = RenderOptions3D(near_plane=float(near_plane), far_plane=float(far_plane),
                           radius_clip=float(radius_clip), eps2d=float(eps2d),
                           input_mode=_lib.INPUT_GSPLAT)
    rgb, alpha = _Render3D.apply(rows, viewmats, Ks, bg, int(width), int(height), opts)
    meta = {"width": int(width), "height": int(height), "tile_size": 16, "n_cameras": C,
            "note": "gsr: per-Gaussian intermediates (radii, means2d, absgrad) are not exported"}
    return rgb, alpha[..., None], meta


def gsplat_module() -> types.ModuleType:
    """A `gsplat` package object whose `rendering` attribute is this module (for aliasing)."""
    import sys
    m = types.ModuleType("gsplat")
    m.rendering = sys.modules[__name__]
    m.rasterization = rasterization
    return m
