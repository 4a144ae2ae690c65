"""gsr — MI355X-native Gaussian-splatting rasterizer (host side of libgsr.so).

Package layout:
  _lib.py    ctypes binding of the C ABI (include/gsr.h); fails loudly if missing
  render.py  projection → binning → rasterisation orchestration + autograd
  scenes.py  deterministic synthetic scenes for the benchmark configs
"""
from ._lib import GsrLibraryError, LIB_PATH
from .render import RenderOptions3D, last_stats, render2d, render3d

__all__ = ["render3d", "render2d", "RenderOptions3D", "last_stats", "GsrLibraryError", "LIB_PATH"]
__version__ = "0.1.0"
