"""Gaussian parameter head + pose transform on the MI355X.

Replaces, in PoseSplatter.forward (src/model.py:134-160):

* the mask-threshold loops of get_gaussian_params_from_volume_unified (src/model.py:185-205),
  which synchronise the host once per step of the search, by one device search plus an
  ordered compaction (`select_gaussians`: one 16-byte read-back for N);
* the post-MLP activations (src/model.py:209-234) and apply_pose_transform_3d
  (src/model.py:258-298, with its per-Gaussian float64 torch.linalg.eigh) by one fused
  per-Gaussian kernel, forward and backward (`gaussian_params_3d`, `pose_transform_3d`).

The MLP itself stays a torch nn.Sequential (two small GEMMs on hipBLASLt).  No CPU path:
the functions raise on CPU tensors.
"""
from __future__ import annotations

import ctypes

import torch

from ._lib import check, lib
from .render import _ptr, _require_device, _stream

__all__ = ["select_gaussians", "gaussian_params_3d", "pose_transform_3d", "params_from_volume_3d"]

_info_host = {}


def select_gaussians(volume0: torch.Tensor, mask_threshold: float = 0.25, prob_threshold: float = 0.25,
                     delta: float = 0.05, min_n: int = 1024, max_n: int = 16000, max_iter: int = 100000):
    """Voxels passing sigmoid(volume0 - mt) > prob_threshold after the reference's threshold
    search (src/model.py:185-205).  Returns (idx [N] int64 increasing, mt float).  When the
    search ends above max_n the reference's random subsample (CPU torch.randperm) is applied."""
    _require_device(volume0, "select_gaussians")
    L = lib()
    dev = volume0.device
    v0 = volume0.detach().reshape(-1).float().contiguous()
    M = v0.numel()
    ws = torch.empty(int(L.gsr_head_select_workspace(M)), device=dev, dtype=torch.uint8)
    out = torch.empty(4, device=dev, dtype=torch.float64)         # [0] mt, [1:] int32 info
    idx = torch.empty(max(M, 1), device=dev, dtype=torch.int64)
    info = out[1:].view(torch.int32)
    check(L.gsr_head_select(_ptr(v0), M, float(mask_threshold), float(prob_threshold), float(delta), int(min_n),
                            int(max_n), int(max_iter), _ptr(ws), ws.numel(), _ptr(info), _ptr(out), _ptr(idx),
                            _stream(dev)), "gsr_head_select")
    host = _info_host.get(dev)
    if host is None:
        host = _info_host[dev] = torch.empty(4, dtype=torch.float64, pin_memory=True)
    host.copy_(out)        # the one host read: N sizes every later tensor
    mt = float(host[0])
    cnt, _, hit = (int(x) for x in host[1:].view(torch.int32)[:3])
    if hit:
        raise RuntimeError(f"select_gaussians: threshold search did not settle within {max_iter} steps "
                           f"(min_n={min_n}, max_n={max_n}, {M} voxels)")
    idx = idx[:cnt]
    if cnt > max_n:
        rand_idx = torch.randperm(cnt)[:max_n].to(dev)
        idx = torch.sort(idx[rand_idx]).values
    return idx, mt


class _Head3D(torch.autograd.Function):
    @staticmethod
    def forward(ctx, net, v0_sel, scale, grid_sel, mt, pt, clip, voxel_size, angle, p3d):
        L = lib()
        dev = net.device
        N = net.shape[0]
        net_c = net.detach().float().contiguous()
        v0 = v0_sel.detach().float().contiguous()
        grid = grid_sel.detach().float().contiguous()
        sc = scale.detach().float().reshape(-1).contiguous()
        pose = angle is not None
        p3 = p3d.detach().to(device=dev, dtype=torch.float32).reshape(3).contiguous() if pose else None
        out = torch.empty(N, 14, device=dev, dtype=torch.float32)
        check(L.gsr_head3d_fwd(_ptr(net_c), N, 14, _ptr(v0), _ptr(grid), _ptr(sc), float(mt), float(pt),
                               float(clip[0]), float(clip[1]), float(voxel_size), int(pose),
                               float(angle) if pose else 0.0, _ptr(p3), _ptr(out), _stream(dev)),
              "gsr_head3d_fwd")
        ctx.save_for_backward(net_c, v0, grid)
        ctx.cfg = (float(mt), float(pt), float(clip[0]), float(clip[1]), float(voxel_size), int(pose),
                   float(angle) if pose else 0.0)
        return out

    @staticmethod
    def backward(ctx, g_out):
        L = lib()
        net_c, v0, grid = ctx.saved_tensors
        mt, pt, lo, hi, vs, pose, angle = ctx.cfg
        dev = net_c.device
        N = net_c.shape[0]
        g = g_out.float().contiguous()
        g_net = torch.empty(N, 14, device=dev, dtype=torch.float32)
        g_v0 = torch.empty(N, device=dev, dtype=torch.float32)
        check(L.gsr_head3d_bwd(_ptr(net_c), N, 14, _ptr(v0), _ptr(grid), mt, pt, lo, hi, vs, pose, angle,
                               _ptr(g), _ptr(g_net), _ptr(g_v0), _stream(dev)), "gsr_head3d_bwd")
        g_scale = g[:, 3:6].sum().reshape(1)
        return g_net, g_v0, g_scale, None, None, None, None, None, None, None


class _Pose3D(torch.autograd.Function):
    @staticmethod
    def forward(ctx, params, angle, p3d):
        L = lib()
        dev = params.device
        p = params.detach().float()
        if p.stride(1) != 1:
            p = p.contiguous()
        p3 = p3d.detach().to(device=dev, dtype=torch.float32).reshape(3).contiguous()
        out = torch.empty(p.shape[0], 14, device=dev, dtype=torch.float32)
        check(L.gsr_pose3d_fwd(_ptr(p), p.shape[0], p.stride(0) if p.shape[0] else 14, float(angle), _ptr(p3),
                               _ptr(out), _stream(dev)), "gsr_pose3d_fwd")
        ctx.save_for_backward(p)
        ctx.angle = float(angle)
        return out

    @staticmethod
    def backward(ctx, g_out):
        L = lib()
        (p,) = ctx.saved_tensors
        g = g_out.float().contiguous()
        g_p = torch.empty(p.shape[0], 14, device=p.device, dtype=torch.float32)
        check(L.gsr_pose3d_bwd(_ptr(p), p.shape[0], p.stride(0) if p.shape[0] else 14, ctx.angle, _ptr(g),
                               _ptr(g_p), _stream(p.device)), "gsr_pose3d_bwd")
        return g_p, None, None


def gaussian_params_3d(net_out: torch.Tensor, v0_sel: torch.Tensor, scale: torch.Tensor, grid_sel: torch.Tensor,
                       mt: float, prob_threshold: float = 0.25, color_clip=(0.0, 0.99), voxel_size: float = 0.18 / 64,
                       angle=None, p_3d=None) -> torch.Tensor:
    """Renderer rows [N,14] from the MLP output net_out [N,14], the selected volume[0]
    logits v0_sel [N] (probs = sigmoid(v0_sel - mt)), the scale offset [1] and the selected
    grid points [N,3]; with angle/p_3d the pose transform is fused in.  Differentiable
    w.r.t. net_out, v0_sel and scale."""
    _require_device(net_out, "gaussian_params_3d")
    if net_out.dim() != 2 or net_out.shape[1] != 14:
        raise ValueError(f"net_out must be [N,14], got {tuple(net_out.shape)}")
    N = net_out.shape[0]
    if v0_sel.shape != (N,) or grid_sel.shape != (N, 3):
        raise ValueError(f"v0_sel must be [N], grid_sel [N,3]; got {tuple(v0_sel.shape)}, {tuple(grid_sel.shape)}")
    if (angle is None) != (p_3d is None):
        raise ValueError("angle and p_3d go together")
    if p_3d is not None and not isinstance(p_3d, torch.Tensor):
        p_3d = torch.tensor(p_3d, dtype=torch.float32)
    return _Head3D.apply(net_out, v0_sel, scale, grid_sel, mt, prob_threshold, tuple(color_clip), voxel_size,
                         angle, p_3d)


def pose_transform_3d(params: torch.Tensor, angle: float, p_3d) -> torch.Tensor:
    """apply_pose_transform_3d (src/model.py:258-298) on renderer rows [N,14]."""
    _require_device(params, "pose_transform_3d")
    if params.dim() != 2 or params.shape[1] != 14:
        raise ValueError(f"params must be [N,14], got {tuple(params.shape)}")
    if not isinstance(p_3d, torch.Tensor):
        p_3d = torch.tensor(p_3d, dtype=torch.float32)
    return _Pose3D.apply(params, float(angle), p_3d)


def params_from_volume_3d(volume: torch.Tensor, mlp, grid: torch.Tensor, scale: torch.Tensor, *,
                          mask_threshold=0.25, prob_threshold=0.25, mask_threshold_delta=0.05, min_n=1024,
                          max_n=16000, color_clip=(0.0, 0.99), voxel_size=0.18 / 64, angle=None, p_3d=None):
    """get_gaussian_params_from_volume_unified (3D) followed, when angle/p_3d are given, by
    apply_pose_transform_3d — the model's sequence (src/model.py:151-156) on libgsr.
    volume [c, M] (U-Net output), grid [M,3] (model.grid.view(-1,3)), scale [1]."""
    idx, mt = select_gaussians(volume[0], mask_threshold, prob_threshold, mask_threshold_delta, min_n, max_n)
    net_out = mlp(volume.index_select(1, idx).T)
    v0_sel = volume[0].index_select(0, idx)
    grid_sel = grid.reshape(-1, 3).index_select(0, idx)
    return gaussian_params_3d(net_out, v0_sel, scale, grid_sel, mt, prob_threshold, color_clip, voxel_size,
                              angle, p_3d)
