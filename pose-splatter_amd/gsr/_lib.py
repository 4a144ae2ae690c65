"""ctypes binding of libgsr.so (the C ABI declared in include/gsr.h).

The library is loaded lazily on first use.  There is no fallback: if libgsr.so is
missing (not built) or cannot be loaded, every render on a device raises
``GsrLibraryError`` — the product never computes on a silent CPU/PyTorch path.
"""
from __future__ import annotations

import ctypes
import os
import threading

__all__ = ["LIB_PATH", "GsrLibraryError", "lib", "check", "BinStats", "BinCaps", "LossTerms", "EXPORTS", "ABI_VERSION",
           "RADIUS_OPACITY_AABB", "RADIUS_ISOTROPIC_3SIGMA", "ORDER_DEPTH", "ORDER_INDEX", "TILE"]

LIB_PATH = os.environ.get(
    "GSR_LIBRARY", os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "libgsr.so"))

TILE = 16
PARTIAL_STRIDE = 9
CHUNK = 128
RADIUS_OPACITY_AABB = 0
RADIUS_ISOTROPIC_3SIGMA = 1
ORDER_DEPTH = 0
ORDER_INDEX = 1
INPUT_ADAPTER = 0
INPUT_GSPLAT = 1

ABI_VERSION = 14   # include/gsr.h GSR_ABI_VERSION this binding is written for
# gsr_set_bwd2d_parts at load (profiles/r05_ab5_bwd2d_parts_sweep.txt; GSR_BWD2D_PART_WGS overrides it
# for measurements, tools/parts_sweep.sh)
BWD2D_PART_WORKGROUPS = int(os.environ.get("GSR_BWD2D_PART_WGS", "4608"))

# stats->overflow bits of a capacity-bounded call (include/gsr.h GSR_OVF_*)
OVF_BITS = {1: "intersections > isect cap", 2: "chunks > chunk cap", 4: "busy tiles > n_busy bound",
            8: "list longer than the split sort's max_seg", 16: "lazily sorted tiles > n_lazy_max bound",
            32: "raster backward chunk_entries differs from the forward's",
            64: "a rank touched more Gaussians than its gradient row block holds",
            128: "a 2D call's layout decisions changed between its calls (gsr_set_* settings)"}
ROW_FLOATS = 16   # GSR_ROW_FLOATS: floats per row of a sparse gradient row block

GSR_EINVAL = -1
GSR_ELAUNCH = -2
GSR_ECAPACITY = -3


class GsrLibraryError(RuntimeError):
    """libgsr.so is unavailable (CUDA/HIP device path cannot run)."""


class BinStats(ctypes.Structure):
    _fields_ = [("n_isect", ctypes.c_int64), ("max_seg", ctypes.c_int32), ("n_busy", ctypes.c_int32),
                ("n_chunks", ctypes.c_int32), ("n_active", ctypes.c_int32),
                ("n_sort_big", ctypes.c_int32), ("n_sort_mid", ctypes.c_int32),
                ("isect_cap", ctypes.c_int64), ("chunk_cap", ctypes.c_int64), ("overflow", ctypes.c_int32),
                ("chunk_entries", ctypes.c_int32), ("status", ctypes.c_void_p), ("n_sort_long", ctypes.c_int32),
                ("masks", ctypes.c_int32), ("n_heavy", ctypes.c_int32),
                ("heavy_min_len", ctypes.c_int32)]


class BinCaps(ctypes.Structure):
    """gsr_bin_caps: bounds of a call that does not read the stats back (0 = unbounded)."""
    _fields_ = [("isect", ctypes.c_int64), ("chunks", ctypes.c_int64), ("status", ctypes.c_void_p),
                ("chunk_entries", ctypes.c_int32), ("reserved", ctypes.c_int32)]


def describe_overflow(bits: int) -> str:
    return ", ".join(v for k, v in OVF_BITS.items() if bits & k) or "none"


class LossTerms(ctypes.Structure):
    """gsr_loss_terms (include/gsr.h): device pointers + img_lambda for gsr3d_raster_bwd_loss."""
    _fields_ = [("rgb", ctypes.c_void_p), ("target_img", ctypes.c_void_p), ("target_mask", ctypes.c_void_p),
                ("sums", ctypes.c_void_p), ("grad_out", ctypes.c_void_p), ("v_rgb_extra", ctypes.c_void_p),
                ("v_alpha_extra", ctypes.c_void_p), ("img_lambda", ctypes.c_float), ("reserved", ctypes.c_int32)]


_P = ctypes.c_void_p
_I32 = ctypes.c_int32
_I64 = ctypes.c_int64
_F = ctypes.c_float
_D = ctypes.c_double
_SZ = ctypes.c_size_t

# name -> (restype, argtypes); must list every function declared in include/gsr.h
EXPORTS = {
    "gsr_version": (ctypes.c_int, []),
    "gsr_abi_version": (ctypes.c_int, []),
    "gsr_last_error": (ctypes.c_char_p, []),
    "gsr_selftest_reduce64": (ctypes.c_int, [_P, _P]),
    "gsr_selftest_reduce_box16": (ctypes.c_int, [_P, _P]),
    "gsr_selftest_reduce_grp": (ctypes.c_int, [_P, ctypes.c_int, _P]),
    "gsr_set_fwd_heavy": (ctypes.c_int, [ctypes.c_int]),
    "gsr_set_bwd2d_parts": (ctypes.c_int, [ctypes.c_int]),
    "gsr_set_fwd_lanes": (ctypes.c_int, [_I32]),
    "gsr_set_bwd_layout": (ctypes.c_int, [_I32]),
    "gsr_selftest_lds_order": (ctypes.c_int, [_P, _P]),
    "gsr3d_project_fwd": (ctypes.c_int, [_P, _I64, _I64, _P, _P, _I32, _I32, _I32, _F, _F, _F, _F,
                                         _I32, _I32, _I32, _I32, _P, _P, _P, _P, _P, _P, _I32, _P]),
    "gsr2d_project_fwd": (ctypes.c_int, [_P, _I64, _I64, _I64, _P, _I32, _I32, _I32, _I32, _F, _P, _P, _P,
                                         _P, _P, _I32, _P]),
    "gsr_bin_offsets": (ctypes.c_int, [_P, _I64, _P, _P, _P, _P, _P, ctypes.POINTER(BinCaps), _P, _P]),
    "gsr_bin_sort_workspace": (_SZ, [_I64, _I64]),
    "gsr_bin_emit": (ctypes.c_int, [_P, _P, _P, _P, _P, _P, _I32, _I64, _I32, _I32, _I32, _P, _P, _SZ, _P]),
    "gsr_bin_sort": (ctypes.c_int, [_P, _P, _P, _P, _P, _P, _P, _I32, _I64, _I32, _I32, _I32, _I64, _I32,
                                    _I32, _I32, _I32, _I32, _P, _P, _SZ, _P, _P, _P]),
    "gsr3d_raster_fwd": (ctypes.c_int, [_P, _P, _P, _P, _P, _P, _P, _I32, _I32, _I32, _P, _I32, _P, _P, _P,
                                        _P, _P, _P, _P, _P, _P, _P, _P]),
    "gsr_set_emit_staged": (ctypes.c_int, [_I32]),
    "gsr_set_split_sort": (ctypes.c_int, [_I32]),
    "gsr_lazy_workspace": (_SZ, [_I64]),
    "gsr_set_lazy_sort": (ctypes.c_int, [_I32, _I32]),
    "gsr_lazy_min_len": (ctypes.c_int, []),
    "gsr_bin_sort_lazy": (ctypes.c_int, [_P, _P, _P, _P, _P, _P, _P, _I32, _I64, _I32, _I32, _I64, _I32, _I32,
                                         _I32, _I32, _I32, _P, _P, _SZ, _P, _P, _P, _P]),
    "gsr3d_raster_fwd_lazy": (ctypes.c_int, [_P, _P, _P, _P, _P, _P, _I32, _I32, _I32, _P, _I32, _P, _P, _P,
                                             _P, _P, _P, _P, _P, _P, _P, _I32, _I32, _P, _SZ, _P, _P, _P]),
    "gsr3d_raster_bwd": (ctypes.c_int, [_P, _P, _P, _P, _P, _P, _P, _P, _I32, _I32, _I32, _I32, _I32, _P,
                                        _P, _P, _P, _P, _P, _P, _P, _P]),
    "gsr2d_raster_fwd": (ctypes.c_int, [_P, _P, _P, _P, _P, _I32, _I32, _I32, _F, _P, _I32, _P, _P, _P, _P, _P,
                                        _P, _P, _P, _P, _I64, _P, _I32, _P]),
    "gsr2d_raster_bwd": (ctypes.c_int, [_P, _P, _P, _P, _P, _P, _P, _P, _I32, _I32, _I32, _I32, _I32, _F, _P, _P,
                                        _P, _P, _P, _P, _P, _I64, _P, _I32, _P]),
    "gsr3d_project_bwd": (ctypes.c_int, [_P, _I64, _I64, _P, _P, _I32, _I32, _I32, _F, _I32, _P, _P,
                                         _P, _P, _P, _P, _I64, _I64, _P, _P, _P]),
    "gsr3d_touched_rows": (ctypes.c_int, [_P, _P, _P, _P, _P, _I32, _I64, _I64, _P, _P, _P]),
    "gsr3d_project_bwd_rows": (ctypes.c_int, [_P, _I64, _I64, _P, _P, _I32, _I32, _I32, _F, _I32, _P, _P,
                                              _P, _P, _P, _P, _P, _I64, _P, _P]),
    "gsr_rows_scatter_add": (ctypes.c_int, [_P, _I32, _I64, _P, _I64, _P, _P]),
    "gsr2d_project_bwd": (ctypes.c_int, [_P, _I64, _I64, _I64, _P, _I32, _I32, _I32, _I32, _P, _P, _P, _P, _P,
                                         _P, _P, _P]),
    "gsr_loss_workspace": (_SZ, [_I32, _I32, _I32]),
    "gsr_loss_iou_l1_fwd": (ctypes.c_int, [_P, _P, _P, _P, _I32, _I32, _I32, _F, _P, _SZ, _P, _P, _P, _P]),
    "gsr3d_raster_bwd_loss": (ctypes.c_int, [_P, _P, _P, _P, _P, _P, _P, _P, _I32, _I32, _I32, _I32, _I32, _P,
                                             _P, _P, ctypes.POINTER(LossTerms), _P, _P, _P, _P]),
    "gsr_head_select_workspace": (_SZ, [_I64]),
    "gsr_head_select": (ctypes.c_int, [_P, _I64, _D, _F, _D, _I32, _I32, _I32, _P, _SZ, _P, _P, _P, _P]),
    "gsr_head3d_fwd": (ctypes.c_int, [_P, _I64, _I64, _P, _P, _P, _F, _F, _F, _F, _F, _I32, _D, _P, _P, _P]),
    "gsr_head3d_bwd": (ctypes.c_int, [_P, _I64, _I64, _P, _P, _F, _F, _F, _F, _F, _I32, _D, _P, _P, _P, _P]),
    "gsr_pose3d_fwd": (ctypes.c_int, [_P, _I64, _I64, _D, _P, _P, _P]),
    "gsr_pose3d_bwd": (ctypes.c_int, [_P, _I64, _I64, _D, _P, _P, _P]),
    "gsr_ssim_workspace": (_SZ, [_I32, _I32, _I32]),
    "gsr_ssim_factors_size": (_SZ, [_I32, _I32, _I32]),
    "gsr_ssim_fwd": (ctypes.c_int, [_P, _P, _P, _P, _I32, _I32, _I32, _P, _P, _SZ, _P, _P, _P]),
    "gsr_ssim_bwd": (ctypes.c_int, [_P, _P, _P, _P, _I32, _I32, _I32, _P, _P, _P, _P, _P]),
    "gsr_carve_workspace": (_SZ, [_I64, _I32, _I32]),
    "gsr_carve_volume": (ctypes.c_int, [_P, _I64, _P, _D, _P, _P, _P, _I32, _P, _P, _I32, _I32, _F, _F, _P, _SZ,
                                        _P, _P]),
    "gsr_carve_medoids_workspace": (_SZ, [_I32]),
    "gsr_carve_medoids": (ctypes.c_int, [_P, _I32, _I32, _I32, _P, _SZ, _P, _P]),
}

_lock = threading.Lock()
_lib = None


def lib():
    """Load (once) and return the ctypes handle; raises GsrLibraryError if unavailable."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise GsrLibraryError(
                f"libgsr.so not found at {LIB_PATH}: the CUDA (ROCm/HIP) renderer needs the native "
                "library — build it with `make -C pose-splatter_amd/csrc` (or __graft_entry__.build()).")
        try:
            handle = ctypes.CDLL(LIB_PATH)
        except OSError as e:
            raise GsrLibraryError(f"cannot load {LIB_PATH}: {e}") from e
        try:
            abi = handle.gsr_abi_version
        except AttributeError:
            raise GsrLibraryError(f"{LIB_PATH} predates gsr_abi_version (ABI < 3): rebuild it "
                                  "(`make -C pose-splatter_amd/csrc`)") from None
        abi.restype = ctypes.c_int
        if abi() != ABI_VERSION:
            raise GsrLibraryError(f"{LIB_PATH} has ABI revision {abi()}, this binding expects {ABI_VERSION}: "
                                  "rebuild the library or update gsr/_lib.py")
        for name, (res, args) in EXPORTS.items():
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        # the split 2D per-set backward for few (set, tile) pairs: render.py allocates chunk_state
        # with 4 floats per slot, which its colour planes need (include/gsr.h).  A process-wide
        # library setting: another C-ABI caller in this process that sizes chunk_state by the
        # one-float contract must turn it off (gsr_set_bwd2d_parts(0)); the backward refuses to
        # split a walk whose forward wrote no colour planes (GSR_OVF_LAYOUT)
        rc = handle.gsr_set_bwd2d_parts(BWD2D_PART_WORKGROUPS)
        if rc != 0:
            raise GsrLibraryError(f"gsr_set_bwd2d_parts({BWD2D_PART_WORKGROUPS}) failed (code {rc}): "
                                  f"{handle.gsr_last_error().decode(errors='replace')}")
        _lib = handle
        return _lib


def check(rc: int, name: str) -> None:
    if rc == 0:
        return
    msg = lib().gsr_last_error().decode(errors="replace")
    if rc == GSR_EINVAL:
        raise ValueError(f"{name}: {msg}")
    raise RuntimeError(f"{name} failed (code {rc}): {msg}")
