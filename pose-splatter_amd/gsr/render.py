"""Host orchestration of libgsr: projection → binning → rasterisation, fwd and bwd.

``render3d`` / ``render2d`` are differentiable w.r.t. the raw ``[N,14]`` / ``[N,9]``
parameters (the same tensor ``GaussianRenderer.render`` receives,
src/gaussian_renderer.py:157-211 and :269-334).  All device memory comes from PyTorch's
caching allocator; every libgsr call is enqueued on ``torch.cuda.current_stream()``.

Two capacity modes ("Threading / streams"):

* ``"exact"`` (default): one host synchronisation per forward, the ``gsr_bin_stats`` read
  (into pinned host memory) that sizes the intersection buffers exactly (gsplat reads its
  intersection count the same way, src/gaussian_renderer.py:196-208).
* ``"bounded"``: NO host synchronisation.  Buffers and grids are sized from upper bounds
  derived from an earlier call of the same shape (+25 % intersections / chunks, +12.5 %
  busy tiles); the device checks every bound and, if one fails, the call writes NaN to
  rgb / alpha / v_params and ORs ``GSR_OVF_*`` bits into a sticky per-device status word.
  Every bounded eager call's stats are copied to pinned memory behind its kernels and queued
  (per shape, oldest first); completed copies are checked at the next call of the shape
  (raising ``CapacityOverflowError`` for the first one that overflowed, refreshing the
  shape's bounds from the others), and the autograd backward of a bounded call waits for its
  own forward's copy -- after enqueuing its kernels -- and raises before returning, so a NaN
  gradient never reaches ``.grad`` / the optimizer.  ``check_overflow()`` checks the sticky
  word explicitly (e.g. after a captured HIP graph replays).  A bounded step has no host
  wait, so it can be captured in a HIP graph (``torch.cuda.CUDAGraph``).
* ``"auto"`` (the drop-in renderers' default, src/gaussian_renderer.py): bounded when a
  backward will follow (it checks the forward as above) and an earlier call of the shape
  left bounds; exact otherwise (the first call of a shape, forward-only calls).  An eager
  ``model``-style training step then has no mid-forward host wait; the backward's check
  waits only for a forward that finished long before (the loss kernels run meanwhile).
  The shape key of this mode leaves the Gaussian count out: pose-splatter's N changes on
  almost every step (src/model.py:190-204), so the bounds come from the shape's previous
  call at whatever N, its per-Gaussian counts scaled by N / N_prev (``_rescaled``).

Intermediates live in two arenas per forward (see ``_Arena``).
"""
from __future__ import annotations

import collections
import math
import contextlib
from dataclasses import dataclass, field

import torch

import ctypes

from . import _lib
from ._lib import check, lib

__all__ = ["render3d", "render2d", "render2d_units", "RenderOptions3D", "last_stats", "set_capacity_mode",
           "capacity_mode", "check_overflow", "overflow_status", "CapacityOverflowError", "set_chunk_entries",
           "set_quadrant_masks"]

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
    input_mode: int = _lib.INPUT_ADAPTER   # INPUT_GSPLAT: rows hold activated gsplat inputs
    # tile rows [y0, y1) binned, counted over the C views' rows end to end (row r of view c is
    # c*ceil(H/16) + r): a rank's contiguous share of (view, row) units (multi-GPU sharding)
    band: tuple = (0, -1)
    # backward: v_params is produced in `grad_buckets` contiguous Gaussian ranges, and
    # grad_hook(rows) is called with each range's rows as soon as its kernels are enqueued
    # (multi-GPU: an async all-reduce of finished rows overlaps the later ranges)
    grad_buckets: int = 1
    grad_hook: object = field(default=None, compare=False)
    # "exact" | "bounded" | "auto" | None (the module default, set_capacity_mode)
    capacity: str | None = None
    # sparse gradient rows (gsr.multiview.GradRows): the backward writes only the rows of the
    # Gaussians this (band) render touched into grad_rows.block (gsr3d_touched_rows +
    # gsr3d_project_bwd_rows) and returns no dense gradient (params.grad stays None)
    grad_rows: object = field(default=None, compare=False)
    # distinguishes calls of one shape whose lists differ (e.g. different view groups rendered
    # concurrently): a bounded call takes its bounds from the previous call with the same tag
    tag: int = 0


class CapacityOverflowError(RuntimeError):
    """A capacity-bounded render exceeded its bounds: its outputs were written as NaN."""


_capacity_default = "exact"
# 3D quadrant masks (include/gsr.h gsr_bin_emit `rec`): the emission stores which 8x8 quadrants
# of its tile each list entry can reach, and the raster forward gathers an entry only for
# those quadrants.  Same outputs bit for bit.  OFF by default: measured on MI355X (round 4,
# profiles/r04_masks_ab.txt) the emission's four quadrant tests cost more than the gathers they
# save -- config 3 emit 29 -> 45 us for raster fwd 106 -> 105 us (step 0.395 -> 0.403 ms),
# config 5 emit 236 -> 366 us (2.25 -> 2.35 ms); the forward's span is its heavy tiles' serial
# walks, not its gather traffic.
_quadrant_masks = False
_MASK_MAX_ENTRIES = 1 << 28   # the masks live in bits 28..31 of the emission index


def set_quadrant_masks(on: bool) -> None:
    """Enable or disable (default) the 3D quadrant masks (outputs are identical either way)."""
    global _quadrant_masks
    _quadrant_masks = bool(on)
# list entries per backward work unit (gsr_bin_caps.chunk_entries).  Units of several 128-entry
# sub-chunks re-read the pixel state and write chunk records less often, but the sub-chunk
# loop's back-edge costs the backward a wave per SIMD (127 VGPRs, 84 without the loop), which
# the saved traffic does not repay: config 4 raster bwd 19.0 ms at 128 against 20.1 / 20.2 ms
# at 256 / 512 (21.5-22.8 ms when forced to 5 waves, with spills); config 3 148 vs 167 us at
# 256 (tools/gpu_units.sh, profiles/r03_units_*.json).  128 for both.
_chunk_entries = {"3d": 128, "2d": 128}


def set_chunk_entries(mode: str, entries: int) -> None:
    """Backward work-unit length for "3d" or "2d" renders (a power of two >= 128)."""
    if mode not in _chunk_entries or entries < 128 or entries & (entries - 1):
        raise ValueError(f"chunk entries for {mode!r} must be a power of two >= 128, got {entries}")
    _chunk_entries[mode] = int(entries)


_MODES = ("exact", "bounded", "auto")


def set_capacity_mode(mode: str) -> None:
    """Module default for calls that do not choose: "exact" (one stats read-back per forward),
    "bounded" (no host synchronisation; bounds from the previous call of the same shape) or
    "auto" (bounded when a backward will follow and bounds exist, else exact)."""
    global _capacity_default
    if mode not in _MODES:
        raise ValueError(f"capacity mode must be one of {_MODES}, got {mode!r}")
    _capacity_default = mode


@contextlib.contextmanager
def capacity_mode(mode: str):
    """``with capacity_mode("bounded"): ...`` -- the module default inside the block."""
    old = _capacity_default
    set_capacity_mode(mode)
    try:
        yield
    finally:
        set_capacity_mode(old)


_status = {}   # device -> int32 [1] sticky overflow bits (device memory, OR-ed by the kernels)


def _status_buf(device) -> torch.Tensor:
    key = str(device)
    t = _status.get(key)
    if t is None:
        t = _status[key] = torch.zeros(1, device=device, dtype=torch.int32)
    return t


_scratch = {}   # device -> int32 [1]: the status word of auto-mode calls that verify themselves


def _scratch_status(device) -> torch.Tensor:
    key = str(device)
    t = _scratch.get(key)
    if t is None:
        t = _scratch[key] = torch.zeros(1, device=device, dtype=torch.int32)
    return t


def overflow_status(device=None, reset: bool = False) -> int:
    """The sticky GSR_OVF_* bits of every call on ``device`` since the last reset (synchronises)."""
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    t = _status_buf(dev)
    bits = int(t.item())
    if reset:
        t.zero_()
    return bits


def check_overflow(device=None) -> None:
    """Raise CapacityOverflowError if any call on ``device`` overflowed its bounds since the
    last check (synchronises; resets the status)."""
    bits = overflow_status(device, reset=True)
    if bits:
        _size_hint.clear()
        raise CapacityOverflowError(f"gsr: a capacity-bounded render exceeded its bounds ({_lib.describe_overflow(bits)}); "
                                    "its outputs were NaN -- the bounds are reset, re-run the step")


_last_stats = {}
_timers = None   # name -> [(start_event, end_event)] while kernel timing is enabled
_timed_only = None


def enable_kernel_timing(enabled: bool = True, only=None) -> None:
    """Bracket libgsr launches with CUDA(HIP) events on the current stream (bench.py).
    ``only``: a set of call names to time (default: all).  Every event record is a packet
    on the stream, so time only what is needed inside a measured region."""
    global _timers, _timed_only
    _timers = {} if enabled else None
    _timed_only = set(only) if only else None


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
        self.s = None

    def __enter__(self):
        # (nothing while a HIP graph is being captured: ROCm rejects timing events inside a
        # captured graph, "External events are disallowed in rocm" -- ADVICE r3)
        if (_timers is not None and (_timed_only is None or self.name in _timed_only)
                and not _capturing()):
            self.s = torch.cuda.Event(enable_timing=True)
            self.s.record()
        return self

    def __exit__(self, *exc):
        if self.s is not None:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            _timers.setdefault(self.name, []).append((self.s, e))
        return False


class _Arena:
    """One device allocation carved into 256-byte-aligned sub-buffers.

    The hot path only needs raw pointers (``ptr``), so a forward costs one caching-allocator
    call per arena instead of one per buffer; typed tensor views are built on demand."""

    def __init__(self, device, spec: dict):
        self.off = {}
        total = 0
        for name, nbytes in spec.items():
            self.off[name] = (total, int(nbytes))
            total += (int(nbytes) + 255) // 256 * 256
        self.buf = torch.empty(max(total, 256), device=device, dtype=torch.uint8)
        base = self.buf.data_ptr()
        self.ptr = {name: base + o for name, (o, _) in self.off.items()}

    def view(self, name, dtype, count=None):
        o, n = self.off[name]
        t = self.buf[o:o + n].view(dtype)
        return t if count is None else t[:count]


_I32, _I64, _F32 = torch.int32, torch.int64, torch.float32
# tensor views exposed for tests / debugging: name -> (arena attribute, dtype)
_VIEWS = {"rec": ("pre", _F32), "depth": ("pre", _F32), "rect": ("pre", _I32), "cnt": ("pre", _I32),
          "isect_off": ("pre", _I32), "tile_off": ("pre", _I32), "busy": ("pre", _I32),
          "chunk_base": ("pre", _I32), "stats_dev": ("pre", _I32),
          "sorted_ids": ("post", _I32), "k_of_s": ("post", _I32), "final_T": ("pre", _F32),
          "last": ("pre", _I32), "tile_end": ("pre", _I32), "tile_cut": ("pre", _I64),
          "chunk_state": ("chunks", _F32), "chunk_list": ("chunks", _I32), "lazy": ("pre", _I32)}

_pinned = {}
# (device, C, N, W, H) -> stats of the last exactly sized (or observed bounded) forward of that
# shape: I, chunks, max_seg, busy, big, mid -- the bounds of bounded calls and the speculative
# arena sizes of exact ones
_size_hint = {}
_monitors = {}    # shape key -> deque of _Monitor: bounded eager forwards, oldest first
_monitor_pool = []   # free pinned stats buffers
_MAX_PENDING = 16    # per shape: past this many unchecked forwards the oldest is waited for
_bg_cache = {}
_STATS_BYTES = 128   # >= sizeof(gsr_bin_stats) (80)
_STATS_I32 = _STATS_BYTES // 4


def _pinned_stats(device) -> torch.Tensor:
    t = _pinned.get(device)
    if t is None:
        t = _pinned[device] = torch.empty(8, dtype=torch.int32, pin_memory=True)
    return t


def _hint_from(st, N: int) -> dict:
    """Hint dict from the int32 words of a gsr_bin_stats (first 8 words), observed at N Gaussians."""
    return {"I": (st[0] & 0xFFFFFFFF) | (st[1] << 32), "max_seg": st[2], "busy": st[3], "chunks": st[4],
            "big": st[6], "mid": st[7], "N": int(N)}


# the hint quantities that grow with the Gaussian count (busy tiles and the sort-class counts are
# capped by the call's tile count where they are used)
_PER_N = ("I", "chunks", "max_seg", "busy", "big", "mid")


def _rescaled(h: dict, N: int) -> dict:
    """A hint observed at h["N"] Gaussians, restated for N (the "auto" mode's shape key leaves N
    out: pose-splatter's Gaussian count changes on almost every step, src/model.py:190-204).
    The per-Gaussian quantities scale by N / h["N"]; the device still checks every bound."""
    n0 = int(h.get("N") or 0)
    if n0 <= 0 or n0 == N:
        return h
    r = N / n0
    out = {k: (int(math.ceil(v * r)) if k in _PER_N else v) for k, v in h.items()}
    out["N"] = int(N)
    return out


def _capturing() -> bool:
    return torch.cuda.is_current_stream_capturing()


class _Monitor:
    """One bounded eager forward's stats, copied to pinned memory behind its kernels."""
    __slots__ = ("key", "host", "event", "done", "N")

    def __init__(self, key, host, event, N=0):
        self.key, self.host, self.event, self.done, self.N = key, host, event, False, int(N)


def _monitor_process(m: _Monitor) -> None:
    """A monitor whose copy has arrived: raise if its forward overflowed, else refresh the
    shape's bounds from what it observed.  Runs once per monitor."""
    if m.done:
        return
    m.done = True
    st = m.host.tolist()
    _monitor_pool.append(m.host)
    ovf = st[12]   # gsr_bin_stats.overflow (byte 48)
    if ovf:
        _size_hint.pop(m.key, None)
        raise CapacityOverflowError(f"gsr: a capacity-bounded render of this shape exceeded its bounds "
                                    f"({_lib.describe_overflow(ovf)}); its outputs and gradients were NaN -- the "
                                    "bounds are reset (the next call sizes exactly), re-run the step")
    h = _hint_from(st, m.N)
    old = _size_hint.get(m.key)
    if old is not None:   # keep bounds monotone over a window: shrink slowly, grow at once
        old = _rescaled(old, m.N)   # (auto mode: the shape's previous observation at another N)
        h = {k: (max(v, int(0.9 * old[k])) if k in _PER_N else v) for k, v in h.items()}
    _size_hint[m.key] = h


def _monitor_check(key) -> None:
    """Every bounded forward of this shape whose stats have arrived, oldest first (no wait):
    raise on the first overflow, refresh the bounds from the others (one slot
    per shape dropped the earlier calls of a host running several steps ahead)."""
    dq = _monitors.get(key)
    while dq:
        m = dq[0]
        if not m.done and not m.event.query():
            return
        dq.popleft()
        _monitor_process(m)


def _monitor_enqueue(b) -> None:
    """Copy this bounded forward's stats to pinned memory behind its kernels (no wait) and
    queue them for the checks (b.monitor: the backward's own check)."""
    b.monitor = None
    if _capturing():
        return
    dq = _monitors.setdefault(b.key, collections.deque())
    if len(dq) >= _MAX_PENDING:   # a host far ahead of the GPU: wait for the oldest
        m = dq.popleft()
        m.event.synchronize()
        _monitor_process(m)
    host = _monitor_pool.pop() if _monitor_pool else torch.empty(_STATS_I32, dtype=torch.int32, pin_memory=True)
    host.copy_(b.pre.view("stats_dev", _I32), non_blocking=True)
    ev = torch.cuda.Event()
    ev.record()
    b.monitor = _Monitor(b.key, host, ev, b.N)
    dq.append(b.monitor)


def _backward_check(b) -> None:
    """After a bounded call's backward kernels are enqueued: wait for ITS forward's stats copy
    (finished long before, in a training step) and raise if the forward overflowed -- the
    NaN v_params is never returned to autograd.  (The backward's own GSR_OVF_UNIT goes to the
    sticky word, check_overflow.)"""
    m = getattr(b, "monitor", None)
    if m is None or m.done:
        return
    m.event.synchronize()
    _monitor_process(m)


# Per (device, tile count, stream): the projection's tile histogram + emission counter, shared
# by successive calls ON ONE STREAM.  project -> offsets -> sort leaves it all zero (the emit
# counts each tile down, the offsets kernel resets the counter), so the next projection skips
# its memset; a call that stops in between leaves the flag False and the next one clears it.
# Keying by stream keeps renders on different streams (or threads) from sharing a buffer:
# calls on one stream are ordered, so no two pipelines overlap on the same counts.
_tc_cache = {}


def _tile_counts(device, CT: int, stream: int) -> list:
    key = (str(device), CT, stream)
    e = _tc_cache.get(key)
    if e is None:
        e = _tc_cache[key] = [torch.empty(CT + 1, device=device, dtype=torch.int32), False]
    return e


class _Bins:
    """Per-call intermediates shared by forward and backward: two arenas, one sized before
    the stats readback (per-Gaussian and per-tile buffers) and one after it (per-intersection
    buffers).  A bounded call sizes both before any kernel runs and never reads back."""

    def __init__(self, device, C, N, width, height, capacity=None, key_extra=None, chunk_entries=128,
                 need_bwd=True, retry=False):
        self.device = device
        self.C, self.N, self.W, self.H = C, N, width, height
        self.tw = (width + _TILE - 1) // _TILE
        self.th = (height + _TILE - 1) // _TILE
        self.CT = C * self.tw * self.th
        CN = max(C * N, 1)
        self.pre = _Arena(device, {
            "rec": CN * 48, "depth": CN * 4, "rect": CN * 8, "cnt": CN * 4,
            "isect_off": CN * 4, "tile_off": (self.CT + 1) * 4, "busy": self.CT * 4,
            "chunk_base": (self.CT + 1) * 4, "tile_end": self.CT * 4, "tile_cut": self.CT * 8,
            "stats_dev": _STATS_BYTES, "final_T": C * width * height * 8, "last": C * width * height * 4,
            "lazy": (3 * self.CT + 4) * 4})
        self.p = dict(self.pre.ptr)
        self.tc = _tile_counts(device, self.CT, _stream(device))
        self.p["tile_cnt"] = self.tc[0].data_ptr()
        self.post = self.chunks = None
        self.post_cap = self.chunk_cap = 0
        self.emitted = False
        self.masks = False   # this call's emission carries quadrant masks (mask_rec)
        self.n_chunks = self.n_isect = self.max_seg = self.n_busy = self.n_lazy = 0
        self.n_sort_big = self.n_sort_mid = self.n_lazy_max = 0
        # the shape whose previous call bounds this one (band / unit grouping included: they
        # change the lists as much as the shape does)
        self.key = (str(device), C, N, width, height, key_extra)
        mode = capacity or _capacity_default
        if mode == "auto":
            # the drop-in's mode: bounds from the previous call of the shape WHATEVER its N,
            # rescaled to this N (_rescaled) -- the real caller's N changes on
            # almost every step (src/model.py:190-204)
            self.key = (str(device), C, "N*", width, height, key_extra)
        # 2D: the chunk list holds one backward unit per slot of the tile sweep (include/gsr.h ABI 7)
        self.min_units = self.CT + 8 if key_extra and key_extra[0] == "2d" else 0
        # 3D: the forward's box survivor masks for the backward (include/gsr.h ABI 14), 256 B per chunk
        self.box_masks = bool(key_extra and key_extra[0] == "3d")
        self.need_bwd = need_bwd   # False: no chunk records, no finalize (tile_end left raw)
        if mode not in _MODES:
            raise ValueError(f"capacity mode must be one of {_MODES}, got {mode!r}")
        self.bounded = False
        self.monitor = None
        # auto mode, eager: the forward checks its own bounds (verify_launch / verify_overflow) and
        # renders again, sized exactly, if they failed -- the caller never sees an overflow
        self.verify = False
        status = _status_buf(device)
        if mode == "auto":
            # bounded only where a backward follows, and where bounds exist; `retry`: the exact
            # re-render of a call whose bounds failed (same key, so it re-seeds the bounds)
            if need_bwd and not _capturing():
                _monitor_check(self.key)
            mode = "bounded" if need_bwd and not retry and (self.key in _size_hint or _capturing()) else "exact"
            if mode == "bounded" and not _capturing():
                self.verify = True
                # the failed call's kernels report to a word nobody reads: the re-render replaces
                # it, so the sticky status (check_overflow) must not see its bits
                status = _scratch_status(device)
        if mode == "bounded":
            if not _capturing():
                _monitor_check(self.key)
            hint = _size_hint.get(self.key)
            if hint is not None:
                self._set_bounds(_rescaled(hint, N) if N > int(hint.get("N") or 0) else hint)
            elif _capturing():
                raise RuntimeError("gsr: a bounded render captured in a graph needs bounds from an earlier call "
                                   "of the same shape (run one step before capturing)")
        self.chunk_entries = int(chunk_entries)
        # (a forward with no backward writes no chunk records: no chunk bound to check)
        self.caps = _lib.BinCaps(self.post_cap if self.bounded else 0,
                                 self.chunk_cap if self.bounded and need_bwd else 0,
                                 status.data_ptr(), self.chunk_entries, 0)

    def _set_bounds(self, h: dict) -> None:
        """Bounded call: every buffer and grid from the shape's hint plus margins (the device
        checks each bound; gsr_bin_stats.overflow)."""
        self.bounded = True
        self.alloc_post(int(h["I"] * 1.25) + 4096)
        self.alloc_chunks(int(h["chunks"] * 1.25) + 64 if self.need_bwd else 1)
        self.n_isect = self.post_cap
        self.n_chunks = self.chunk_cap
        self.n_busy = min(self.CT, int(h["busy"] * 1.125) + 8)
        self.max_seg = int(h["max_seg"] * 1.25) + 64
        self.n_sort_big = min(h["big"], self.n_busy)
        self.n_sort_mid = min(h["mid"], self.n_busy - self.n_sort_big)
        if self.max_seg >= 4096 and self.n_sort_big + self.n_sort_mid == 0:
            self.n_sort_mid = 1   # the 1024-thread sort shape (any shape sorts every list correctly)
        self.n_lazy_max = min(self.n_busy, int(h["big"] * 1.25) + 4)

    def mask_rec(self, order):
        """The records to pass to the emission for quadrant masks (3D depth order, masks on, an
        emission workspace of at most 2^28 entries), else None; records the decision."""
        use = (_quadrant_masks and order == _lib.ORDER_DEPTH and self.post is not None
               and self.post_cap <= _MASK_MAX_ENTRIES)
        self.masks = bool(use)
        return self.p["rec"] if use else None

    def verify_launch(self) -> None:
        """Auto mode, eager: copy the stats to pinned memory behind the last kernel of the forward
        that can set an overflow bit (the sort; the lazy forward's own re-sort), no wait."""
        if not self.verify:
            return
        self._vhost = _monitor_pool.pop() if _monitor_pool else torch.empty(_STATS_I32, dtype=torch.int32,
                                                                            pin_memory=True)
        self._vhost.copy_(self.pre.view("stats_dev", _I32), non_blocking=True)
        self._vev = torch.cuda.Event()
        self._vev.record()

    def verify_overflow(self) -> int:
        """The GSR_OVF_* bits of this call's forward (waits for verify_launch's copy, which the
        GPU reaches while the raster forward enqueued behind it still has to run); 0 unless
        verifying.  (the drop-in's default mode must not raise on a caller whose
        footprints grow past the previous step's bounds.)"""
        if not self.verify:
            return 0
        self._vev.synchronize()
        st = self._vhost.tolist()
        _monitor_pool.append(self._vhost)
        return int(st[12])

    def take_tile_counts(self) -> int:
        """For the projection call: 1 if the shared tile_count buffer is known to be zero."""
        z, self.tc[1] = self.tc[1], False
        return int(z)

    def guess_post(self, with_chunks: bool):
        """Before the stats readback: size the per-intersection and per-chunk arenas from the
        last call with the same shapes (plus 25 %), so their allocation overlaps the GPU's
        projection/scan and the emit can be enqueued before the readback (emit_early)."""
        if self.bounded:
            return
        hint = _size_hint.get(self.key)
        if hint is not None:
            hint = _rescaled(hint, self.N)
            self.alloc_post(int(hint["I"] * 1.25) + 1024)
            if with_chunks:
                self.alloc_chunks(int(hint["chunks"] * 1.25) + 16)

    def __getattr__(self, name):
        # typed views of arena buffers (not used on the hot path)
        if name == "cnt" and self.__dict__.get("box_masks"):
            # 3D: the projection does not write the counts (include/gsr.h: optional); each
            # (camera, Gaussian)'s entry count is its tile rect's area
            r = self.pre.view("rect", torch.int32).view(-1, 2).to(torch.int64) & 0xFFFFFFFF
            w = (r[:, 0] >> 16) - (r[:, 0] & 0xFFFF)
            h = (r[:, 1] >> 16) - (r[:, 1] & 0xFFFF)
            return (w * h).to(torch.int32)
        if name in _VIEWS:
            where, dt = _VIEWS[name]
            arena = self.__dict__.get(where)
            if arena is not None:
                return arena.view(name, dt)
        raise AttributeError(name)

    def offsets(self, stream):
        """Tile scan, then the one host sync of the forward: the 32-byte stats readback."""
        self.offsets_launch(stream)
        self.offsets_wait()

    def offsets_launch(self, stream):
        L = lib()
        p = self.p
        with _timed("bin_offsets"):
          check(L.gsr_bin_offsets(p["tile_cnt"], self.CT, p["tile_off"], p["chunk_base"], p["busy"], p["tile_end"],
                                p["tile_cut"], ctypes.byref(self.caps), p["stats_dev"], stream), "gsr_bin_offsets")
        if self.bounded:
            return
        self._host = _pinned_stats(self.device)
        self._host.copy_(self.pre.view("stats_dev", _I32)[:8], non_blocking=True)
        self._ev = torch.cuda.Event()
        self._ev.record()

    def emit_early(self, order, stream):
        """Enqueue the emit into the speculative arena before the readback: the GPU runs it
        while the host waits; if this call's I does not fit, the kernel does nothing and
        sort() emits again into an arena sized from the readback."""
        if self.post is None:
            return
        L = lib()
        p = self.p
        with _timed("bin_emit"):
          check(L.gsr_bin_emit(p["depth"] if order == _lib.ORDER_DEPTH else None, self.mask_rec(order), p["rect"],
                               p["isect_off"],
                               p["tile_off"], p["tile_cnt"], self.C, self.N, self.W, self.H, order, p["stats_dev"],
                               p["sort_ws"], self.post.off["sort_ws"][1], stream), "gsr_bin_emit")
        self.emitted = True

    def offsets_wait(self):
        if self.bounded:   # nothing to wait for: the bounds are set
            return
        ev = self._ev
        while not ev.query():   # the one host sync of the forward (spin: lowest wake-up latency)
            pass
        st = self._host.tolist()
        self.n_isect = (st[0] & 0xFFFFFFFF) | (st[1] << 32)
        self.max_seg, self.n_busy, self.n_chunks = st[2], st[3], st[4]
        self.n_sort_big, self.n_sort_mid = st[6], st[7]
        if self.n_isect >= 2 ** 31:
            raise RuntimeError(f"gsr: {self.n_isect} intersections exceed the 32-bit index range")

    def alloc_post(self, n_isect: int):
        L = lib()
        I = max(n_isect, 1)
        self.post = _Arena(self.device, {
            "sorted_ids": I * 4, "k_of_s": I * 4, "sort_ws": int(L.gsr_bin_sort_workspace(I, self.CT))})
        self.post_cap = I
        self.p.update(self.post.ptr)

    def alloc_chunks(self, n_chunks: int):
        K = max(n_chunks, 1)
        spec = {"chunk_state": K * 256 * 16, "chunk_list": max(K, self.min_units) * 16}
        if self.box_masks:
            spec["box_masks"] = K * 256
        self.chunks = _Arena(self.device, spec)
        self.chunk_cap = K
        self.p.update(self.chunks.ptr)

    def ensure_post(self, with_chunks: bool):
        """After the stats readback: keep the speculatively sized arenas if they are big enough
        (an emit_early into a too-small arena did nothing; sort() then emits)."""
        if self.bounded:
            return
        if self.post is None or self.n_isect > self.post_cap:
            self.alloc_post(int(self.n_isect * 1.25))
            self.emitted = False
        if with_chunks and (self.chunks is None or self.n_chunks > self.chunk_cap):
            self.alloc_chunks(int(self.n_chunks * 1.25))
        elif self.chunks is None:
            self.alloc_chunks(1)
        _size_hint[self.key] = {"I": self.n_isect, "chunks": self.n_chunks, "max_seg": self.max_seg,
                                "busy": self.n_busy, "big": self.n_sort_big, "mid": self.n_sort_mid, "N": self.N}

    def sort(self, order, stream):
        L = lib()
        p = self.p
        with _timed("bin_sort"):
          rec = self.mask_rec(order) if not self.emitted else (p["rec"] if self.masks else None)
          check(L.gsr_bin_sort(p["depth"] if order == _lib.ORDER_DEPTH else None, rec, p["rect"], p["isect_off"],
                               p["tile_off"], p["tile_cnt"], p["busy"],
                             self.C, self.N,
                             self.W, self.H, order, self.n_isect, self.max_seg, self.n_busy, self.n_sort_big,
                             self.n_sort_mid, int(self.emitted), p["stats_dev"], p["sort_ws"],
                             self.post.off["sort_ws"][1], p["sorted_ids"], p["k_of_s"], stream), "gsr_bin_sort")
        self.tc[1] = True   # offsets reset the counter, the emit counted every tile back to 0

    def lazy_bound(self) -> int:
        """0 when every list is sorted whole; else the grid of the lazy re-sort / re-render
        (gsr_bin_sort_lazy: lists longer than gsr_lazy_min_len): the lists of >= 8192 entries
        when min_len >= 8191 (the device flags GSR_OVF_LAZY if more tiles need it)."""
        m = lib().gsr_lazy_min_len()
        if m <= 0 or self.max_seg <= m:
            return 0
        if self.bounded:
            return max(1, self.n_lazy_max if m >= 8191 else self.n_busy)
        return self.n_sort_big if m >= 8191 else self.n_busy

    def sort_lazy(self, stream):
        L = lib()
        p = self.p
        with _timed("bin_sort"):
          rec = self.mask_rec(_lib.ORDER_DEPTH) if not self.emitted else (p["rec"] if self.masks else None)
          check(L.gsr_bin_sort_lazy(p["depth"], rec, p["rect"], p["isect_off"], p["tile_off"], p["tile_cnt"], p["busy"],
                                  self.C, self.N, self.W, self.H, self.n_isect, self.max_seg, self.n_busy,
                                  self.n_sort_big, self.n_sort_mid, int(self.emitted), p["stats_dev"], p["sort_ws"],
                                  self.post.off["sort_ws"][1], p["sorted_ids"], p["k_of_s"], p["lazy"], stream),
                "gsr_bin_sort_lazy")
        self.tc[1] = True


def _record_stats(b: _Bins):
    _last_stats.clear()
    _last_stats["tiles"] = b.CT
    _last_stats["_bins"] = b
    if b.bounded:   # read lazily (last_stats synchronises) -- the forward itself never waits
        _last_stats["_lazy"] = True
        _monitor_enqueue(b)
    else:
        _last_stats.update(n_isect=b.n_isect, max_seg=b.max_seg, n_busy=b.n_busy)


def last_stats() -> dict:
    """Binning statistics of the most recent forward (I, max list, busy tiles; a bounded
    call's are read from the device here, which synchronises)."""
    if _last_stats.pop("_lazy", False):
        b = _last_stats["_bins"]
        h = _hint_from(b.pre.view("stats_dev", _I32)[:8].tolist(), b.N)
        _last_stats.update(n_isect=h["I"], max_seg=h["max_seg"], n_busy=h["busy"])
    return dict(_last_stats)


def effective_isect(stats: dict | None = None) -> int:
    """I_eff = sum over tiles of (tile_end - start): list entries the raster actually read."""
    s = _last_stats if stats is None else stats
    if "_bins" not in s:
        return 0
    return int(_tile_entries(s["_bins"]).sum())


def _tile_entries(b) -> torch.Tensor:
    """Per-tile list entries the raster read, [C*T] int64 (tile_end - start; a forward with
    no backward leaves tile_end raw: the maximum last, -1 for none, the start for empty tiles)."""
    te = b.tile_end.to(torch.int64)
    st = b.tile_off[:-1].to(torch.int64)
    if not b.need_bwd:
        ln = b.tile_off[1:].to(torch.int64) - st
        te = torch.where((ln > 0) & (te >= st), te + 1, st)
    return (te - st).clamp(min=0)


def tile_work(stats: dict | None = None) -> torch.Tensor:
    """Per-tile list entries the last forward's raster read (tile_end - start), [C*T] int64 —
    the work weights for multi-GPU band balancing (gsr.multiview.band_shard)."""
    s = _last_stats if stats is None else stats
    if "_bins" not in s:
        raise RuntimeError("tile_work: no forward has run")
    return _tile_entries(s["_bins"])


def _background(bg: torch.Tensor, C: int, dev) -> torch.Tensor:
    """bg [3] or [C,3] -> contiguous float32 [C,3] on dev (expanded copies are cached per
    source tensor version, so a fixed background costs no kernel per call).  The cache entry
    holds the source tensor, so its address cannot be recycled by a different background
    while the entry is alive."""
    b = bg.detach()
    if b.device == dev and b.dtype == torch.float32 and b.is_contiguous() and b.numel() == 3 * C:
        return b.reshape(C, 3)
    key = (b.data_ptr(), b._version, tuple(b.shape), C, str(dev))
    hit = _bg_cache.get(key)
    if hit is None:
        if len(_bg_cache) > 64:
            _bg_cache.clear()
        hit = _bg_cache[key] = (b, b.to(device=dev, dtype=torch.float32).reshape(-1, 3).expand(C, 3).contiguous())
    return hit[1]


def _forward3d(params, viewmats, Ks, bg, width, height, opts, need_bwd=True, retry=False):
    """Projection → binning → raster fwd.  Returns (rgb, alpha, bins, meta).  need_bwd False: no
    backward will follow (no grad needed), so no chunk records and no finalize.  An auto-mode
    call whose bounds fail renders again, sized exactly (retry)."""
    L = lib()
    dev = params.device
    stream = _stream(dev)
    C = viewmats.shape[0]
    N = params.shape[0]
    p, stride = _rows(params, 14)
    V = viewmats.detach().to(device=dev, dtype=torch.float32).contiguous()
    Kc = Ks.detach().to(device=dev, dtype=torch.float32).contiguous()
    bgc = _background(bg, C, dev)
    b = _Bins(dev, C, N, width, height, opts.capacity, ("3d", opts.band, opts.input_mode, opts.radius_mode, opts.tag),
              _chunk_entries["3d"], need_bwd, retry)
    q = b.p
    with _timed("project3d_fwd"):
      check(L.gsr3d_project_fwd(_ptr(p), N, stride, _ptr(V), _ptr(Kc), C, width, height,
                              opts.near_plane, opts.far_plane, opts.radius_clip, opts.eps2d,
                              opts.radius_mode, opts.input_mode, opts.band[0], opts.band[1], q["rec"], q["depth"],
                              q["rect"], q["cnt"] if _counts3d else None, q["isect_off"], q["tile_cnt"],
                              b.take_tile_counts(), stream),
          "gsr3d_project_fwd")
    b.guess_post(with_chunks=need_bwd)
    b.offsets_launch(stream)
    b.emit_early(_lib.ORDER_DEPTH, stream)
    b.offsets_wait()
    b.ensure_post(with_chunks=need_bwd)
    cs, cl = (q["chunk_state"], q["chunk_list"]) if need_bwd else (None, None)
    bm = q.get("box_masks") if need_bwd else None
    n_lazy = b.n_lazy = b.lazy_bound()
    if n_lazy:
        b.sort_lazy(stream)
    else:
        b.sort(_lib.ORDER_DEPTH, stream)
        b.verify_launch()
    rgb = torch.empty(C, height, width, 3, device=dev, dtype=torch.float32)
    alpha = torch.empty(C, height, width, device=dev, dtype=torch.float32)
    with _timed("raster3d_fwd"):
      if n_lazy:
        check(L.gsr3d_raster_fwd_lazy(q["rec"], q["depth"], q["sorted_ids"], q["tile_off"], q["busy"],
                                      q["chunk_base"], C, width, height, _ptr(bgc), b.n_busy, q["stats_dev"],
                                      _ptr(rgb), _ptr(alpha), q["final_T"], q["last"], q["tile_end"], q["tile_cut"],
                                      cs, cl, q["lazy"], n_lazy, b.max_seg,
                                      q["sort_ws"], b.post.off["sort_ws"][1], q["k_of_s"], bm, stream),
              "gsr3d_raster_fwd_lazy")
      else:
        check(L.gsr3d_raster_fwd(q["rec"], q["depth"], q["sorted_ids"], q["k_of_s"], q["tile_off"],
                                 q["busy"], q["chunk_base"],
                                 C, width, height, _ptr(bgc), b.n_busy, q["stats_dev"], _ptr(rgb), _ptr(alpha),
                                 q["final_T"], q["last"], q["tile_end"], q["tile_cut"], cs, cl, bm, stream),
              "gsr3d_raster_fwd")
    if n_lazy:
        b.verify_launch()   # (the lazy forward's re-sort can still flag GSR_OVF_LAZY)
    if b.verify_overflow():
        return _forward3d(params, viewmats, Ks, bg, width, height, opts, need_bwd, retry=True)
    _record_stats(b)
    return rgb, alpha, b, (p, stride, V, Kc, bgc, width, height, opts)


_set_cache = {}


def _set_begin(unit_sets: tuple, F: int, dev):
    """Device int32 [F+1] CSR of the cameras of each parameter set (cameras grouped by set),
    cached per (sets, device); None for the single-set, single-camera case."""
    if F == 1 and len(unit_sets) == 1:
        return None
    key = (unit_sets, F, str(dev))
    t = _set_cache.get(key)
    if t is None:
        if any(b < a for a, b in zip(unit_sets, unit_sets[1:])) or not all(0 <= f < F for f in unit_sets):
            raise ValueError(f"unit sets must be non-decreasing in [0, {F}), got {unit_sets}")
        begin = [0] * (F + 1)
        for f in unit_sets:
            begin[f + 1] += 1
        for f in range(F):
            begin[f + 1] += begin[f]
        if len(_set_cache) > 64:
            _set_cache.clear()
        t = _set_cache[key] = torch.tensor(begin, dtype=torch.int32).to(dev)
    return t


def _sets2d(params: torch.Tensor):
    """[N,9] or [F,N,9] -> (rows, F, N, row stride, set stride) with unit row-element stride."""
    p = params.detach()
    if p.dtype != torch.float32:
        p = p.float()
    if p.dim() == 2:
        p, stride = _rows(p, 9)
        return p, 1, p.shape[0], stride, 0
    F, N = p.shape[0], p.shape[1]
    if p.stride(2) != 1 or p.stride(1) < 9 or (N > 0 and p.stride(0) < N * p.stride(1)):
        p = p.contiguous()
    return p, F, N, int(p.stride(1)) if N > 0 else 9, int(p.stride(0))


def _forward2d(params, bg, width, height, eps_cut, unit_sets=(0,), capacity=None, need_bwd=True, retry=False):
    """unit_sets[c] = parameter set rendered by camera (unit) c (non-decreasing)."""
    L = lib()
    dev = params.device
    stream = _stream(dev)
    p, F, N, stride, set_stride = _sets2d(params)
    C = len(unit_sets)
    sb = _set_begin(tuple(unit_sets), F, dev)
    bgc = _background(bg, C, dev)
    b = _Bins(dev, C, N, width, height, capacity, ("2d", tuple(unit_sets), F), _chunk_entries["2d"], need_bwd,
              retry)
    q = b.p
    with _timed("project2d_fwd"):
      check(L.gsr2d_project_fwd(_ptr(p), N, stride, set_stride, _ptr(sb), F, C, width, height, eps_cut, q["rec"],
                              q["rect"], q["cnt"], q["isect_off"], q["tile_cnt"], b.take_tile_counts(), stream),
          "gsr2d_project_fwd")
    b.guess_post(with_chunks=need_bwd)
    b.offsets_launch(stream)
    b.emit_early(_lib.ORDER_INDEX, stream)
    b.offsets_wait()
    b.ensure_post(with_chunks=need_bwd)
    b.sort(_lib.ORDER_INDEX, stream)
    b.verify_launch()
    cs, cl = (q["chunk_state"], q["chunk_list"]) if need_bwd else (None, None)
    rgb = torch.empty(C, height, width, 3, device=dev, dtype=torch.float32)
    alpha = torch.empty(C, height, width, device=dev, dtype=torch.float32)
    with _timed("raster2d_fwd"):
      check(L.gsr2d_raster_fwd(q["rec"], q["sorted_ids"], q["tile_off"], q["busy"], q["chunk_base"], C, width, height,
                             eps_cut, _ptr(bgc), b.n_busy, q["stats_dev"], _ptr(rgb), _ptr(alpha), q["final_T"],
                             q["last"], q["tile_end"], q["tile_cut"], cs, cl, N, _ptr(sb), F, stream),
          "gsr2d_raster_fwd")
    if b.verify_overflow():
        return _forward2d(params, bg, width, height, eps_cut, unit_sets, capacity, need_bwd, retry=True)
    _record_stats(b)
    return rgb, alpha, b, (p, F, stride, set_stride, sb, bgc, width, height, eps_cut)


# measurement hook: the 3D projection also writes isect_count (a (camera, Gaussian)'s entry count
# is its rect's area; no 3D kernel reads the counts, so the product path passes NULL)
_counts3d = False


def debug_forward3d(params, viewmats, Ks, bg, width, height, opts=None):
    """Test hook: the forward plus all binning intermediates (no autograd)."""
    return _forward3d(params, viewmats, Ks, bg, width, height, opts or RenderOptions3D())


def debug_forward2d(params, bg, width, height, eps_cut=1e-8):
    rgb, alpha, b, meta = _forward2d(params, bg, width, height, eps_cut)
    return rgb[0], alpha[0], b, meta


class _Render3D(torch.autograd.Function):
    @staticmethod
    def forward(ctx, params, viewmats, Ks, bg, width, height, opts: RenderOptions3D, need_bwd=True):
        rgb, alpha, b, meta = _forward3d(params, viewmats, Ks, bg, width, height, opts, need_bwd)
        ctx.b = b
        ctx.meta = meta
        ctx.params_shape = params.shape
        return rgb, alpha

    @staticmethod
    def backward(ctx, v_rgb, v_alpha):
        b = ctx.b
        _, _, _, _, bgc, width, height, _ = ctx.meta
        C, dev = b.C, b.device
        if v_rgb is None:
            v_rgb = torch.zeros(C, height, width, 3, device=dev)
        if v_alpha is None:
            v_alpha = torch.zeros(C, height, width, device=dev)
        v_rgb = v_rgb.float().contiguous()
        v_alpha = v_alpha.float().contiguous()

        def raster(L, q, partial, stream):
            check(L.gsr3d_raster_bwd(q["rec"], q["sorted_ids"], q["tile_off"], q["tile_end"], q["chunk_base"],
                                     q["chunk_state"], q["chunk_list"], q["stats_dev"],
                                     b.n_chunks, b.chunk_entries, C, width, height, _ptr(bgc), q["final_T"], q["last"],
                                     _ptr(v_rgb), _ptr(v_alpha), q["k_of_s"], _ptr(partial), q.get("box_masks"),
                                     stream),
                  "gsr3d_raster_bwd")
        v_params = backward3d(b, ctx.meta, raster)
        _backward_check(b)   # a bounded forward that overflowed raises here, before .grad
        if v_params is None:   # sparse gradient rows (opts.grad_rows): no dense gradient
            return None, None, None, None, None, None, None, None
        return v_params.view(ctx.params_shape), None, None, None, None, None, None, None


def backward3d(b, meta, raster) -> torch.Tensor:
    """Raster backward (``raster(L, q, partial, stream)`` issues the raster call that writes
    the partial rows) followed by the projection backward: v_params [N,14]."""
    L = lib()
    p, stride, V, Kc, bgc, width, height, opts = meta
    stream = _stream(p.device)
    C, N = b.C, b.N
    if opts.grad_rows is not None:
        return _backward3d_rows(L, b, meta, raster, stream)
    v_params = torch.empty(N, 14, device=p.device, dtype=torch.float32)
    if N > 0:
        partial = torch.empty(max(b.n_isect, 1) * _lib.PARTIAL_STRIDE, device=p.device, dtype=torch.float32)
        q = b.p
        with _timed("raster3d_bwd"):
            raster(L, q, partial, stream)
        nb = max(1, min(int(opts.grad_buckets), N))
        bounds = [N * k // nb for k in range(nb + 1)]
        for n0, n1 in zip(bounds[:-1], bounds[1:]):
            with _timed("project3d_bwd"):
              check(L.gsr3d_project_bwd(_ptr(p), N, stride, _ptr(V), _ptr(Kc), C, width, height, opts.eps2d,
                                        opts.input_mode,
                                        q["depth"], q["rect"], q["isect_off"], None, q["tile_cut"],
                                        _ptr(partial), n0, n1, q["stats_dev"], _ptr(v_params), stream),
                    "gsr3d_project_bwd")
            if opts.grad_hook is not None:
                opts.grad_hook(v_params[n0:n1])
    elif opts.grad_hook is not None:
        opts.grad_hook(v_params)
    return v_params


def _backward3d_rows(L, b, meta, raster, stream) -> None:
    """The backward of a band share whose gradient leaves as sparse rows (opts.grad_rows, a
    gsr.multiview.GradRows): list the Gaussians the share touched, run the raster backward, and
    chain only their partial rows into the row block -- no dense [N,14] write."""
    p, stride, V, Kc, bgc, width, height, opts = meta
    rows = opts.grad_rows
    C, N = b.C, b.N
    q = b.p
    flags = torch.empty((N + 3) // 4 * 4, device=p.device, dtype=torch.uint8)
    check(L.gsr3d_touched_rows(q["sorted_ids"], q["tile_off"], q["tile_end"], q["busy"], q["stats_dev"], b.n_busy, N,
                               rows.cap, flags.data_ptr(), rows.block.data_ptr(), stream), "gsr3d_touched_rows")
    if N == 0:
        return None
    partial = torch.empty(max(b.n_isect, 1) * _lib.PARTIAL_STRIDE, device=p.device, dtype=torch.float32)
    with _timed("raster3d_bwd"):
        raster(L, q, partial, stream)
    with _timed("project3d_bwd"):
        check(L.gsr3d_project_bwd_rows(_ptr(p), N, stride, _ptr(V), _ptr(Kc), C, width, height, opts.eps2d,
                                       opts.input_mode, q["depth"], q["rect"], q["isect_off"], None,
                                       q["tile_cut"], _ptr(partial), q["stats_dev"], rows.cap,
                                       rows.block.data_ptr(), stream), "gsr3d_project_bwd_rows")
    return None


class _Render2D(torch.autograd.Function):
    @staticmethod
    def forward(ctx, params, bg, width, height, eps_cut, unit_sets, capacity=None, need_bwd=True):
        rgb, alpha, b, meta = _forward2d(params, bg, width, height, eps_cut, unit_sets, capacity, need_bwd)
        ctx.b = b
        ctx.meta = meta
        ctx.params_shape = params.shape
        return rgb, alpha

    @staticmethod
    def backward(ctx, v_rgb, v_alpha):
        L = lib()
        b = ctx.b
        p, F, stride, set_stride, sb, bgc, width, height, eps_cut = ctx.meta
        dev = p.device
        stream = _stream(dev)
        N, C = b.N, b.C
        if v_rgb is None:
            v_rgb = torch.zeros(C, height, width, 3, device=dev)
        if v_alpha is None:
            v_alpha = torch.zeros(C, height, width, device=dev)
        v_rgb = v_rgb.float().contiguous()
        v_alpha = v_alpha.float().contiguous()
        v_params = torch.empty(F, N, 9, device=dev, dtype=torch.float32)
        if N > 0:
            partial = torch.empty(max(b.n_isect, 1) * _lib.PARTIAL_STRIDE, device=dev, dtype=torch.float32)
            q = b.p
            with _timed("raster2d_bwd"):
              check(L.gsr2d_raster_bwd(q["rec"], q["sorted_ids"], q["tile_off"], q["tile_end"], q["chunk_base"],
                                     q["chunk_state"], q["chunk_list"], q["stats_dev"],
                                     # (2D backward units: one per slot of the tile sweep; n_chunks unused)
                                     b.n_busy, b.chunk_entries, C, width, height, eps_cut, _ptr(bgc), q["final_T"],
                                     q["last"],
                                     _ptr(v_rgb), _ptr(v_alpha), q["k_of_s"], _ptr(partial), N, _ptr(sb), F,
                                     stream),
                  "gsr2d_raster_bwd")
            with _timed("project2d_bwd"):
              check(L.gsr2d_project_bwd(_ptr(p), N, stride, set_stride, _ptr(sb), F, C, width, height, q["rect"],
                                      q["isect_off"], q["cnt"], q["tile_cut"], _ptr(partial), q["stats_dev"],
                                      _ptr(v_params), stream),
                  "gsr2d_project_bwd")
        _backward_check(b)   # a bounded forward that overflowed raises here, before .grad
        return v_params.view(ctx.params_shape), None, None, None, None, None, None, None


def _needs_grad(params: torch.Tensor) -> bool:
    """Whether a backward can follow this render (else no chunk records / finalize)."""
    return torch.is_grad_enabled() and params.requires_grad


def render3d(params: torch.Tensor, viewmats: torch.Tensor, Ks: torch.Tensor, width: int, height: int,
             background: torch.Tensor, opts: RenderOptions3D = RenderOptions3D()):
    """[N,14] raw params, viewmats [C,4,4], Ks [C,3,3], background [3] or [C,3] →
    rgb [C,H,W,3], alpha [C,H,W] (differentiable w.r.t. params)."""
    _require_device(params, "GaussianRenderer3D")
    if viewmats.dim() != 3 or viewmats.shape[1:] != (4, 4):
        raise ValueError(f"viewmats must be [C,4,4], got {tuple(viewmats.shape)}")
    if Ks.dim() != 3 or Ks.shape[1:] != (3, 3) or Ks.shape[0] != viewmats.shape[0]:
        raise ValueError(f"Ks must be [C,3,3] matching viewmats, got {tuple(Ks.shape)}")
    return _Render3D.apply(params, viewmats, Ks, background, int(width), int(height), opts, _needs_grad(params))


def render2d(params: torch.Tensor, width: int, height: int, background: torch.Tensor,
             eps_cut: float = 1e-8, capacity: str | None = None):
    """[N,9] raw params → rgb [H,W,3], alpha [H,W] (index-order compositing)."""
    _require_device(params, "GaussianRenderer2D")
    if params.dim() != 2:
        raise ValueError(f"render2d: params must be [N,9], got {tuple(params.shape)}")
    rgb, alpha = _Render2D.apply(params, background, int(width), int(height), float(eps_cut), (0,), capacity,
                                 _needs_grad(params))
    return rgb[0], alpha[0]


def render2d_units(params: torch.Tensor, unit_sets, width: int, height: int, background: torch.Tensor,
                   eps_cut: float = 1e-8, capacity: str | None = None):
    """Multi-frame 2D batch in ONE launch sequence: params [F,N,9] (F frames' raw parameter
    sets), unit_sets[c] = the frame rendered by unit (camera) c, non-decreasing (units grouped
    by frame; a frame may have any number of units, including none).  Returns rgb [C,H,W,3],
    alpha [C,H,W]; the gradient w.r.t. params [F,N,9] sums each frame's units.  The reference
    ignores the camera in 2D (src/gaussian_renderer.py:280-281), so the units of a frame are
    identical renders -- each is still rendered (units = frame x view)."""
    _require_device(params, "GaussianRenderer2D")
    if params.dim() != 3 or params.shape[-1] != 9:
        raise ValueError(f"render2d_units: params must be [F,N,9], got {tuple(params.shape)}")
    sets = tuple(int(f) for f in unit_sets)
    if not sets:
        raise ValueError("render2d_units: no units")
    _set_begin(sets, params.shape[0], params.device)   # validates the grouping
    # Only the sets [sets[0], sets[-1]] are rendered: the launch sees that range (a view, no copy;
    # autograd's slice backward gives the other sets a zero gradient).  The per-set backward and the
    # shared lists key on C > F, so a frame owner's one frame of six views (params [8,N,9], sets
    # (f,)*6) takes them as the full batch does (profiles/r05_rankshare_cfg4.json).
    f0, f1 = sets[0], sets[-1] + 1
    if (f0, f1) != (0, params.shape[0]):
        params = params[f0:f1]
        sets = tuple(f - f0 for f in sets)
    return _Render2D.apply(params, background, int(width), int(height), float(eps_cut), sets, capacity,
                           _needs_grad(params))
