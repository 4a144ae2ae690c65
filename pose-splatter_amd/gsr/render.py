"""Host orchestration of libgsr: projection → binning → rasterisation, fwd and bwd.

``render3d`` / ``render2d`` are differentiable w.r.t. the raw ``[N,14]`` / ``[N,9]``
parameters (the same tensor ``GaussianRenderer.render`` receives,
src/gaussian_renderer.py:157-211 and :269-334).  All device memory comes from PyTorch's
caching allocator; every libgsr call is enqueued on ``torch.cuda.current_stream()``.
The one host synchronisation per forward is the 16-byte ``gsr_bin_stats`` read that
sizes the intersection buffers (gsplat reads its intersection count the same way).
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from . import _lib
from ._lib import check, lib

__all__ = ["render3d", "render2d", "RenderOptions3D", "last_stats"]

_TILE = _lib.TILE


def _ptr(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()


def _stream(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def _require_device(t: torch.Tensor, who: str) -> None:
    if t.device.type != "cuda":
        raise RuntimeError(
            f"{who}: the MI355X rasterizer runs on a CUDA (ROCm/HIP) device; got a tensor on "
            f"'{t.device}'. Move the renderer and its inputs to 'cuda' (there is no CPU path).")


def _rows(params: torch.Tensor, width: int) -> tuple[torch.Tensor, int]:
    p = params.detach()
    if p.dtype != torch.float32:
        p = p.float()
    if p.stride(1) != 1 or p.stride(0) < width:
        p = p.contiguous()
    return p, int(p.stride(0)) if p.shape[0] > 0 else width


@dataclass(frozen=True)
class RenderOptions3D:
    """gsplat ``rasterization`` defaults used by the reference adapter (packed=False)."""
    near_plane: float = 0.01
    far_plane: float = 1e10
    radius_clip: float = 0.0
    eps2d: float = 0.3
    radius_mode: int = _lib.RADIUS_OPACITY_AABB


_last_stats = {}
_timers = None   # name -> [(start_event, end_event)] while kernel timing is enabled


def enable_kernel_timing(enabled: bool = True) -> None:
    """Bracket each libgsr launch with CUDA(HIP) events on the current stream (bench.py)."""
    global _timers
    _timers = {} if enabled else None


def kernel_times_ms() -> dict:
    """Average duration (ms) and launch count per bracketed libgsr call (synchronises)."""
    if not _timers:
        return {}
    torch.cuda.synchronize()
    return {k: (sum(s.elapsed_time(e) for s, e in v) / len(v), len(v)) for k, v in _timers.items()}


class _timed:
    __slots__ = ("name", "s")

    def __init__(self, name):
        self.name = name

    def __enter__(self):
        if _timers is not None:
            self.s = torch.cuda.Event(enable_timing=True)
            self.s.record()
        return self

    def __exit__(self, *exc):
        if _timers is not None:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            _timers.setdefault(self.name, []).append((self.s, e))
        return False


def last_stats() -> dict:
    """Binning statistics of the most recent forward (I, I_eff, max list, busy tiles)."""
    return dict(_last_stats)


class _Bins:
    """Per-call intermediates shared by forward and backward (all device tensors)."""

    def __init__(self, device, C, N, width, height):
        self.C, self.N, self.W, self.H = C, N, width, height
        self.tw = (width + _TILE - 1) // _TILE
        self.th = (height + _TILE - 1) // _TILE
        self.CT = C * self.tw * self.th
        CN = C * N
        i32 = dict(device=device, dtype=torch.int32)
        self.rec = torch.empty(max(CN, 1) * 12, device=device, dtype=torch.float32)
        self.rect = torch.empty(max(CN, 1) * 2, **i32)
        self.cnt = torch.empty(max(CN, 1), **i32)
        self.tile_cnt = torch.zeros(self.CT, **i32)
        self.isect_off = torch.empty(max(CN, 1), **i32)
        self.tile_off = torch.empty(self.CT + 1, **i32)
        self.busy = torch.empty(self.CT, **i32)
        self.chunk_base = torch.empty(self.CT + 1, **i32)
        self.stats_dev = torch.zeros(8, **i32)   # gsr_bin_stats (32 B)
        self.n_chunks = 0
        self.n_isect = 0
        self.max_seg = 0
        self.n_busy = 0

    def offsets(self, stream):
        L = lib()
        CN = self.C * self.N
        ws = torch.empty(int(L.gsr_bin_offsets_workspace(CN, self.CT)), device=self.rec.device,
                         dtype=torch.uint8)
        with _timed("bin_offsets"):
          check(L.gsr_bin_offsets(_ptr(self.cnt), CN, _ptr(self.tile_cnt), self.CT, _ptr(ws), ws.numel(),
                                _ptr(self.isect_off), _ptr(self.tile_off), _ptr(self.chunk_base),
                                _ptr(self.busy), _ptr(self.stats_dev), stream), "gsr_bin_offsets")
        st = self.stats_dev.cpu()   # the one D2H sync of the forward
        self.n_isect = (int(st[0]) & 0xFFFFFFFF) | (int(st[1]) << 32)
        self.max_seg = int(st[2])
        self.n_busy = int(st[3])
        self.n_chunks = int(st[4])
        if self.n_isect >= 2 ** 31:
            raise RuntimeError(f"gsr: {self.n_isect} intersections exceed the 32-bit index range")

    def sort(self, order, stream):
        L = lib()
        dev = self.rec.device
        I = self.n_isect
        self.sorted_ids = torch.empty(max(I, 1), device=dev, dtype=torch.int32)
        self.k_of_s = torch.empty(max(I, 1), device=dev, dtype=torch.int32)
        ws = torch.empty(int(L.gsr_bin_sort_workspace(I, self.CT)), device=dev, dtype=torch.uint8)
        with _timed("bin_sort"):
          check(L.gsr_bin_sort(_ptr(self.rec), _ptr(self.rect), _ptr(self.isect_off), _ptr(self.tile_off),
                             _ptr(self.busy), self.C, self.N, self.W, self.H, order, I, self.max_seg,
                             self.n_busy, _ptr(ws), ws.numel(), _ptr(self.sorted_ids), _ptr(self.k_of_s),
                             stream), "gsr_bin_sort")


def _record_stats(b: _Bins):
    _last_stats.clear()
    _last_stats.update(n_isect=b.n_isect, max_seg=b.max_seg, n_busy=b.n_busy, tiles=b.CT)
    _last_stats["_tile_end"] = b.tile_end
    _last_stats["_tile_off"] = b.tile_off


def effective_isect(stats: dict | None = None) -> int:
    """I_eff = sum over tiles of (tile_end - start): list entries the raster actually read."""
    s = _last_stats if stats is None else stats
    if "_tile_end" not in s:
        return 0
    te = s["_tile_end"].to(torch.int64)
    st = s["_tile_off"][:-1].to(torch.int64)
    return int((te - st).clamp(min=0).sum())


def _forward3d(params, viewmats, Ks, bg, width, height, opts):
    """Projection → binning → raster fwd.  Returns (rgb, alpha, bins, meta)."""
    L = lib()
    dev = params.device
    stream = _stream(dev)
    C = viewmats.shape[0]
    N = params.shape[0]
    p, stride = _rows(params, 14)
    V = viewmats.detach().to(device=dev, dtype=torch.float32).contiguous()
    Kc = Ks.detach().to(device=dev, dtype=torch.float32).contiguous()
    bgc = bg.detach().to(device=dev, dtype=torch.float32).reshape(-1, 3).expand(C, 3).contiguous()
    b = _Bins(dev, C, N, width, height)
    if N > 0:
        with _timed("project3d_fwd"):
          check(L.gsr3d_project_fwd(_ptr(p), N, stride, _ptr(V), _ptr(Kc), C, width, height,
                                  opts.near_plane, opts.far_plane, opts.radius_clip, opts.eps2d,
                                  opts.radius_mode, _ptr(b.rec), _ptr(b.rect), _ptr(b.cnt),
                                  _ptr(b.tile_cnt), stream), "gsr3d_project_fwd")
    b.offsets(stream)
    b.sort(_lib.ORDER_DEPTH, stream)
    rgb = torch.empty(C, height, width, 3, device=dev, dtype=torch.float32)
    alpha = torch.empty(C, height, width, device=dev, dtype=torch.float32)
    b.final_T = torch.empty(C, height, width, device=dev, dtype=torch.float32)
    b.last = torch.empty(C, height, width, device=dev, dtype=torch.int32)
    b.tile_end = torch.empty(b.CT, device=dev, dtype=torch.int32)
    b.tile_cut = torch.empty(b.CT, device=dev, dtype=torch.int64)
    b.chunk_state = torch.empty(max(b.n_chunks, 1) * 256 * 4, device=dev, dtype=torch.float32)
    b.chunk_tile = torch.empty(max(b.n_chunks, 1), device=dev, dtype=torch.int32)
    b.chunk_list = torch.empty(max(b.n_chunks, 1), device=dev, dtype=torch.int32)
    with _timed("raster3d_fwd"):
      check(L.gsr3d_raster_fwd(_ptr(b.rec), _ptr(b.sorted_ids), _ptr(b.tile_off), _ptr(b.busy), _ptr(b.chunk_base),
                             C, width, height, _ptr(bgc), b.n_busy, _ptr(b.stats_dev), _ptr(rgb), _ptr(alpha),
                             _ptr(b.final_T), _ptr(b.last), _ptr(b.tile_end), _ptr(b.tile_cut), _ptr(b.chunk_state),
                             _ptr(b.chunk_tile), _ptr(b.chunk_list), stream), "gsr3d_raster_fwd")
    _record_stats(b)
    return rgb, alpha, b, (p, stride, V, Kc, bgc, width, height, opts)


def _forward2d(params, bg, width, height, eps_cut):
    L = lib()
    dev = params.device
    stream = _stream(dev)
    N = params.shape[0]
    p, stride = _rows(params, 9)
    bgc = bg.detach().to(device=dev, dtype=torch.float32).reshape(1, 3).contiguous()
    b = _Bins(dev, 1, N, width, height)
    with _timed("project2d_fwd"):
      check(L.gsr2d_project_fwd(_ptr(p), N, stride, width, height, eps_cut, _ptr(b.rec), _ptr(b.rect),
                              _ptr(b.cnt), _ptr(b.tile_cnt), stream), "gsr2d_project_fwd")
    b.offsets(stream)
    b.sort(_lib.ORDER_INDEX, stream)
    rgb = torch.empty(height, width, 3, device=dev, dtype=torch.float32)
    alpha = torch.empty(height, width, device=dev, dtype=torch.float32)
    b.last = torch.empty(height, width, device=dev, dtype=torch.int32)
    b.tile_end = torch.empty(b.CT, device=dev, dtype=torch.int32)
    b.tile_cut = torch.empty(b.CT, device=dev, dtype=torch.int64)
    with _timed("raster2d_fwd"):
      check(L.gsr2d_raster_fwd(_ptr(b.rec), _ptr(b.sorted_ids), _ptr(b.tile_off), width, height, _ptr(bgc),
                             _ptr(rgb), _ptr(alpha), _ptr(b.last), _ptr(b.tile_end), _ptr(b.tile_cut), stream),
          "gsr2d_raster_fwd")
    _record_stats(b)
    return rgb, alpha, b, (p, stride, bgc, width, height)


def debug_forward3d(params, viewmats, Ks, bg, width, height, opts=None):
    """Test hook: the forward plus all binning intermediates (no autograd)."""
    return _forward3d(params, viewmats, Ks, bg, width, height, opts or RenderOptions3D())


def debug_forward2d(params, bg, width, height, eps_cut=1e-8):
    return _forward2d(params, bg, width, height, eps_cut)


class _Render3D(torch.autograd.Function):
    @staticmethod
    def forward(ctx, params, viewmats, Ks, bg, width, height, opts: RenderOptions3D):
        rgb, alpha, b, meta = _forward3d(params, viewmats, Ks, bg, width, height, opts)
        ctx.b = b
        ctx.meta = meta
        ctx.params_shape = params.shape
        return rgb, alpha

    @staticmethod
    def backward(ctx, v_rgb, v_alpha):
        L = lib()
        b = ctx.b
        p, stride, V, Kc, bgc, width, height, opts = ctx.meta
        dev = p.device
        stream = _stream(dev)
        C, N = b.C, b.N
        if v_rgb is None:
            v_rgb = torch.zeros(C, height, width, 3, device=dev)
        if v_alpha is None:
            v_alpha = torch.zeros(C, height, width, device=dev)
        v_rgb = v_rgb.float().contiguous()
        v_alpha = v_alpha.float().contiguous()
        v_params = torch.empty(N, 14, device=dev, dtype=torch.float32)
        if N > 0:
            partial = torch.empty(max(b.n_isect, 1) * _lib.PARTIAL_STRIDE, device=dev, dtype=torch.float32)
            with _timed("raster3d_bwd"):
              check(L.gsr3d_raster_bwd(_ptr(b.rec), _ptr(b.sorted_ids), _ptr(b.tile_off), _ptr(b.tile_end),
                                     _ptr(b.chunk_base), _ptr(b.chunk_tile), _ptr(b.chunk_state),
                                     _ptr(b.chunk_list), _ptr(b.stats_dev), b.n_chunks,
                                     C, width, height, _ptr(bgc), _ptr(b.final_T), _ptr(b.last), _ptr(v_rgb),
                                     _ptr(v_alpha), _ptr(b.k_of_s), _ptr(partial), stream),
                  "gsr3d_raster_bwd")
            with _timed("project3d_bwd"):
              check(L.gsr3d_project_bwd(_ptr(p), N, stride, _ptr(V), _ptr(Kc), C, width, height, opts.eps2d,
                                      _ptr(b.rec), _ptr(b.rect), _ptr(b.isect_off), _ptr(b.cnt), _ptr(b.tile_cut),
                                      _ptr(partial), _ptr(v_params), stream),
                  "gsr3d_project_bwd")
        return v_params.view(ctx.params_shape), None, None, None, None, None, None


class _Render2D(torch.autograd.Function):
    @staticmethod
    def forward(ctx, params, bg, width, height, eps_cut):
        rgb, alpha, b, meta = _forward2d(params, bg, width, height, eps_cut)
        ctx.b = b
        ctx.meta = meta
        ctx.params_shape = params.shape
        return rgb, alpha

    @staticmethod
    def backward(ctx, v_rgb, v_alpha):
        L = lib()
        b = ctx.b
        p, stride, bgc, width, height = ctx.meta
        dev = p.device
        stream = _stream(dev)
        N = b.N
        if v_rgb is None:
            v_rgb = torch.zeros(height, width, 3, device=dev)
        if v_alpha is None:
            v_alpha = torch.zeros(height, width, device=dev)
        v_rgb = v_rgb.float().contiguous()
        v_alpha = v_alpha.float().contiguous()
        v_params = torch.empty(N, 9, device=dev, dtype=torch.float32)
        if N > 0:
            partial = torch.empty(max(b.n_isect, 1) * _lib.PARTIAL_STRIDE, device=dev, dtype=torch.float32)
            ws = torch.empty(int(L.gsr2d_raster_bwd_workspace(b.n_isect, b.CT)), device=dev, dtype=torch.uint8)
            with _timed("raster2d_bwd"):
              check(L.gsr2d_raster_bwd(_ptr(b.rec), _ptr(b.sorted_ids), _ptr(b.tile_off), _ptr(b.tile_end),
                                     _ptr(b.busy), b.n_busy, width, height, _ptr(bgc), _ptr(b.last),
                                     _ptr(v_rgb), _ptr(v_alpha), _ptr(ws), ws.numel(), _ptr(b.k_of_s), _ptr(partial),
                                     stream),
                  "gsr2d_raster_bwd")
            with _timed("project2d_bwd"):
              check(L.gsr2d_project_bwd(_ptr(p), N, stride, width, height, _ptr(b.rect), _ptr(b.isect_off),
                                      _ptr(b.cnt), _ptr(b.tile_cut), _ptr(partial),
                                      _ptr(v_params), stream), "gsr2d_project_bwd")
        return v_params.view(ctx.params_shape), None, None, None, None


def render3d(params: torch.Tensor, viewmats: torch.Tensor, Ks: torch.Tensor, width: int, height: int,
             background: torch.Tensor, opts: RenderOptions3D = RenderOptions3D()):
    """[N,14] raw params, viewmats [C,4,4], Ks [C,3,3], background [3] or [C,3] →
    rgb [C,H,W,3], alpha [C,H,W] (differentiable w.r.t. params)."""
    _require_device(params, "GaussianRenderer3D")
    if viewmats.dim() != 3 or viewmats.shape[1:] != (4, 4):
        raise ValueError(f"viewmats must be [C,4,4], got {tuple(viewmats.shape)}")
    if Ks.dim() != 3 or Ks.shape[1:] != (3, 3) or Ks.shape[0] != viewmats.shape[0]:
        raise ValueError(f"Ks must be [C,3,3] matching viewmats, got {tuple(Ks.shape)}")
    return _Render3D.apply(params, viewmats, Ks, background, int(width), int(height), opts)


def render2d(params: torch.Tensor, width: int, height: int, background: torch.Tensor,
             eps_cut: float = 1e-8):
    """[N,9] raw params → rgb [H,W,3], alpha [H,W] (index-order compositing)."""
    _require_device(params, "GaussianRenderer2D")
    return _Render2D.apply(params, background, int(width), int(height), float(eps_cut))
