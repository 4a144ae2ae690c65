"""Loss-fused render: the reference training step's IoU + L1 image loss
(scripts/training/train_script.py:30-36 `get_iou_loss`, :128-130 `img_loss`) evaluated and
differentiated on the MI355X without materialising any cotangent image, and its SSIM term
(:129, torchmetrics SSIM, data_range 1.0) as two libgsr kernels (`ssim`).

    iou_loss, img_loss, rgb, alpha = render3d_iou_l1(params, viewmats, Ks, W, H, bg,
                                                     target_img, target_mask, img_lambda)
    total = iou_loss + img_loss + ssim_lambda * (1 - gsr.loss.ssim(target_img, rgb))
    total.backward()

Forward: render (gsr3d_*), then one streaming pass (gsr_loss_iou_l1_fwd) reduces
{sum a m, sum a + m - a m, sum m, sum |t - rgb|} per view in a fixed order and forms the two
losses on the device (no host sync).  Backward: the raster backward generates every pixel's
cotangent from those sums and the incoming loss gradients (gsr3d_raster_bwd_loss); gradients
that reach `rgb` / `alpha` through other terms (the SSIM term's rgb gradient, written by
gsr_ssim_bwd) are added in the same kernel.

Shapes follow the reference's per-view tensors stacked over C views: target_img [C,3,H,W]
(planar, the loader's layout; [3,H,W] accepted for C=1), target_mask [C,H,W] ([H,W] for C=1).
With C > 1 the IoU term is the mean over views of the per-view IoU and the image term sums
over all views, i.e. exactly the reference functions applied to the stacked tensors.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from ._lib import check, lib
from .render import (RenderOptions3D, _forward3d, _ptr, _require_device, _stream, _timed, backward3d)

__all__ = ["render3d_iou_l1", "ssim"]


def _taps11() -> torch.Tensor:
    """torchmetrics' 1-D Gaussian for sigma 1.5 (11 taps), computed with the same float32 ops
    (host tensor: libgsr copies the taps into the kernel arguments)."""
    dist = torch.arange(-5.0, 6.0, 1.0, dtype=torch.float32)
    g = torch.exp(-torch.pow(dist / 1.5, 2) / 2)
    return (g / g.sum()).contiguous()


_TAPS = None


def _strides4(t: torch.Tensor, channels_last: bool):
    """(view, channel, row, column) element strides of a [C,3,H,W] or [C,H,W,3] image."""
    s = t.stride()
    return (s[0], s[3], s[1], s[2]) if channels_last else (s[0], s[1], s[2], s[3])


class _Ssim(torch.autograd.Function):
    @staticmethod
    def forward(ctx, target_img, rgb):
        global _TAPS
        if _TAPS is None:
            _TAPS = _taps11()
        L = lib()
        dev = rgb.device
        C, H, W = rgb.shape[0], rgb.shape[1], rgb.shape[2]
        x = target_img.detach().to(device=dev, dtype=torch.float32)
        y = rgb.detach().float()
        xs = torch.tensor(_strides4(x, False), dtype=torch.int64)
        ys = torch.tensor(_strides4(y, True), dtype=torch.int64)
        ws = torch.empty(int(L.gsr_ssim_workspace(C, W, H)), device=dev, dtype=torch.uint8)
        out = torch.empty((), device=dev, dtype=torch.float32)
        # the backward's per-window factors, stored by the forward only when a backward can follow
        need = bool(ctx.needs_input_grad[1])
        fac = torch.empty(int(L.gsr_ssim_factors_size(C, W, H)) if need else 0, device=dev, dtype=torch.float32)
        with _timed("ssim_fwd"):
            check(L.gsr_ssim_fwd(_ptr(x), xs.data_ptr(), _ptr(y), ys.data_ptr(), C, W, H, _TAPS.data_ptr(), _ptr(ws),
                                 ws.numel(), _ptr(out), _ptr(fac) if need else None, _stream(dev)), "gsr_ssim_fwd")
        ctx.save_for_backward(x, y, fac)
        ctx.strides = (xs, ys)
        return out

    @staticmethod
    def backward(ctx, g):
        x, y, fac = ctx.saved_tensors
        xs, ys = ctx.strides
        L = lib()
        dev = y.device
        C, H, W = y.shape[0], y.shape[1], y.shape[2]
        gy = torch.empty_strided(y.shape, y.stride(), device=dev, dtype=torch.float32)
        g = g.detach().float().reshape(()).contiguous()
        with _timed("ssim_bwd"):
            check(L.gsr_ssim_bwd(_ptr(x), xs.data_ptr(), _ptr(y), ys.data_ptr(), C, W, H, _TAPS.data_ptr(), _ptr(fac),
                                 _ptr(g), _ptr(gy), _stream(dev)), "gsr_ssim_bwd")
        return None, gy


def ssim(target_img: torch.Tensor, rgb: torch.Tensor) -> torch.Tensor:
    """The reference's SSIM term on the device: torchmetrics
    StructuralSimilarityIndexMeasure(data_range=1.0)(target_img, rgb) for C views at once (the
    batch mean, scripts/training/train_script.py:129), differentiable w.r.t. ``rgb``.
    target_img [C,3,H,W] (planar, the loader's layout; [3,H,W] for C=1), rgb [C,H,W,3] (the
    renderer's layout; [H,W,3] for C=1), read in place; H, W > 10."""
    if rgb.dim() == 3:
        rgb = rgb[None]
    if target_img.dim() == 3:
        target_img = target_img[None]
    if rgb.dim() != 4 or rgb.shape[-1] != 3:
        raise ValueError(f"rgb must be [C,H,W,3], got {tuple(rgb.shape)}")
    C, H, W, _ = rgb.shape
    if target_img.shape != (C, 3, H, W):
        raise ValueError(f"target_img must be [C,3,H,W] = {(C, 3, H, W)}, got {tuple(target_img.shape)}")
    if H <= 10 or W <= 10:
        raise ValueError(f"SSIM needs images larger than 10x10 (11x11 Gaussian window), got {H}x{W}")
    _require_device(rgb, "ssim")
    return _Ssim.apply(target_img, rgb)


class _RenderIouL1(torch.autograd.Function):
    @staticmethod
    def forward(ctx, params, viewmats, Ks, bg, width, height, opts, target_img, target_mask, img_lambda):
        rgb, alpha, b, meta = _forward3d(params, viewmats, Ks, bg, width, height, opts)
        L = lib()
        dev = params.device
        C = b.C
        t = target_img.detach().to(device=dev, dtype=torch.float32).contiguous()
        m = target_mask.detach().to(device=dev, dtype=torch.float32).contiguous()
        ws = torch.empty(int(L.gsr_loss_workspace(C, width, height)), device=dev, dtype=torch.uint8)
        sums = torch.empty((C + 1) * 4, device=dev, dtype=torch.float32)
        iou = torch.empty((), device=dev, dtype=torch.float32)
        img = torch.empty((), device=dev, dtype=torch.float32)
        with _timed("loss_fwd"):
            check(L.gsr_loss_iou_l1_fwd(_ptr(rgb), _ptr(alpha), _ptr(t), _ptr(m), C, width, height,
                                        float(img_lambda), _ptr(ws), ws.numel(), _ptr(sums), _ptr(iou),
                                        _ptr(img), _stream(dev)), "gsr_loss_iou_l1_fwd")
        ctx.b, ctx.meta, ctx.params_shape = b, meta, params.shape
        ctx.img_lambda = float(img_lambda)
        ctx.save_for_backward(rgb, t, m, sums)
        return iou, img, rgb, alpha

    @staticmethod
    def backward(ctx, g_iou, g_img, v_rgb, v_alpha):
        rgb, t, m, sums = ctx.saved_tensors
        b = ctx.b
        _, _, _, _, bgc, width, height, _ = ctx.meta
        dev = rgb.device
        zero = torch.zeros((), device=dev)
        grad_out = torch.stack([zero if g_iou is None else g_iou.float().reshape(()),
                                zero if g_img is None else g_img.float().reshape(())])
        v_rgb = None if v_rgb is None else v_rgb.float().contiguous()
        v_alpha = None if v_alpha is None else v_alpha.float().contiguous()
        terms = _lib.LossTerms(_ptr(rgb), _ptr(t), _ptr(m), _ptr(sums), _ptr(grad_out), _ptr(v_rgb),
                               _ptr(v_alpha), ctx.img_lambda, 0)

        def raster(L, q, partial, stream):
            check(L.gsr3d_raster_bwd_loss(q["rec"], q["sorted_ids"], q["tile_off"], q["tile_end"],
                                          q["chunk_base"], q["chunk_state"], q["chunk_list"],
                                          q["stats_dev"], b.n_chunks, b.chunk_entries, b.C, width, height, _ptr(bgc),
                                          q["final_T"], q["last"], ctypes.byref(terms), q["k_of_s"],
                                          _ptr(partial), q.get("box_masks"), stream), "gsr3d_raster_bwd_loss")
        v_params = backward3d(b, ctx.meta, raster)
        return (v_params.view(ctx.params_shape),) + (None,) * 9


def render3d_iou_l1(params: torch.Tensor, viewmats: torch.Tensor, Ks: torch.Tensor, width: int, height: int,
                    background: torch.Tensor, target_img: torch.Tensor, target_mask: torch.Tensor,
                    img_lambda: float = 1.0, opts: RenderOptions3D = RenderOptions3D()):
    """Render C views and evaluate the reference IoU + L1 losses against the targets.

    Returns (iou_loss, img_loss, rgb [C,H,W,3], alpha [C,H,W]); all four are differentiable
    w.r.t. ``params`` ([N,14] raw adapter rows, or activated rows with
    ``opts.input_mode = INPUT_GSPLAT``)."""
    C = viewmats.shape[0]
    if viewmats.dim() != 3 or viewmats.shape[1:] != (4, 4) or Ks.shape != (C, 3, 3):
        raise ValueError(f"viewmats must be [C,4,4] and Ks [C,3,3], got {tuple(viewmats.shape)}, {tuple(Ks.shape)}")
    if C == 1 and target_img.dim() == 3:
        target_img = target_img[None]
    if C == 1 and target_mask.dim() == 2:
        target_mask = target_mask[None]
    if target_img.shape != (C, 3, height, width):
        raise ValueError(f"target_img must be [C,3,H,W] = {(C, 3, height, width)}, got {tuple(target_img.shape)}")
    if target_mask.shape != (C, height, width):
        raise ValueError(f"target_mask must be [C,H,W] = {(C, height, width)}, got {tuple(target_mask.shape)}")
    _require_device(params, "render3d_iou_l1")
    return _RenderIouL1.apply(params, viewmats, Ks, background, int(width), int(height), opts, target_img,
                              target_mask, float(img_lambda))
