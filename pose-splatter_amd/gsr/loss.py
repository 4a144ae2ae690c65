"""Loss-fused render: the reference training step's IoU + L1 image loss
(scripts/training/train_script.py:30-36 `get_iou_loss`, :128-130 `img_loss`) evaluated and
differentiated on the MI355X without materialising any cotangent image.

    iou_loss, img_loss, rgb, alpha = render3d_iou_l1(params, viewmats, Ks, W, H, bg,
                                                     target_img, target_mask, img_lambda)
    total = iou_loss + img_loss + ssim_lambda * (1 - ssim(target_img, rgb))   # optional SSIM
    total.backward()

Forward: render (gsr3d_*), then one streaming pass (gsr_loss_iou_l1_fwd) reduces
{sum a m, sum a + m - a m, sum m, sum |t - rgb|} per view in a fixed order and forms the two
losses on the device (no host sync).  Backward: the raster backward generates every pixel's
cotangent from those sums and the incoming loss gradients (gsr3d_raster_bwd_loss); gradients
that reach `rgb` / `alpha` through other terms (SSIM) are added in the same kernel.

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

__all__ = ["render3d_iou_l1"]


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
                                          q["stats_dev"], b.n_chunks, b.C, width, height, _ptr(bgc),
                                          q["final_T"], q["last"], ctypes.byref(terms), q["k_of_s"],
                                          _ptr(partial), stream), "gsr3d_raster_bwd_loss")
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
