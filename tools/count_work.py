"""Work counters of the raster kernels (needs a -DGSR_EXP_COUNT build via GSR_LIBRARY).

Prints, for one fwd+bwd of a bench config: forward batches traversed per wave (sum, max),
forward survivors, backward survivors / 7-groups / max per wave / active chunk blocks.
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pose-splatter_amd"))
import torch  # noqa: E402
from gsr import render as R  # noqa: E402
from gsr._lib import lib  # noqa: E402
from gsr.scenes import CONFIGS, gaussians3d, ring_cameras  # noqa: E402

cfg = CONFIGS[int(sys.argv[1]) if len(sys.argv) > 1 else 3]
dev = torch.device("cuda:0")
p = gaussians3d(cfg.N, cfg.seed).to(dev).requires_grad_(True)
V, K = ring_cameras(cfg.views, cfg.width, cfg.height)
V, K = V.to(dev), K.to(dev)
bg = torch.ones(3, device=dev)
L = lib()
f = L.gsr_debug_counters
f.argtypes = [ctypes.c_void_p, ctypes.c_int]
out = (ctypes.c_ulonglong * 16)()
fb = L.gsr_debug_counters_bin
fb.argtypes = [ctypes.c_void_p, ctypes.c_int]
outb = (ctypes.c_ulonglong * 16)()
rgb, alpha = R.render3d(p, V, K, cfg.width, cfg.height, bg)
(rgb.sum() + alpha.sum()).backward()
f(out, 1)
fb(outb, 1)
R.enable_kernel_timing(True)
rgb, alpha = R.render3d(p, V, K, cfg.width, cfg.height, bg)
(rgb.sum() + alpha.sum()).backward()
f(out, 1)
fb(outb, 1)
print({k: round(v[0], 4) for k, v in R.kernel_times_ms().items()})
names = ["fwd_batches", "fwd_max_batches_per_wave", "fwd_survivors", "fwd_cycles_cull+issue",
         "fwd_cycles_composite", "fwd_cycles_wave_total", "fwd_cycles_wave_max", "-",
         "bwd_survivors", "bwd_groups", "bwd_cycles_prologue", "bwd_cycles_groups", "bwd_cycles_epilogue",
         "bwd_active_blocks", "bwd_cycles_wave_max", "-"]
for n, v in zip(names, out):
    print(f"{n:28s} {v}")
for n, v in zip(["sort_cycles_load", "sort_cycles_radix", "sort_cycles_out", "sort_cycles_block_max",
                 "sort_blocks_lds", "sort_cycles_fixup", "sort_fix_iters", "sort_fix_iters_max"], outb):
    print(f"{n:28s} {v}")
st = R.last_stats()
print({k: v for k, v in st.items() if not k.startswith("_")})

# per-workgroup timeline of the last forward (s_memrealtime ticks, 100 MHz)
fbk = L.gsr_debug_blocks
fbk.argtypes = [ctypes.c_void_p]
import numpy as np
blk = np.zeros((32768, 3), dtype=np.uint64)
fbk(blk.ctypes.data)
nb = 32 * ((st["n_busy"] + 7) // 8)
b = blk[:nb].astype(np.int64)
b = b[b[:, 1] > 0]
t0 = b[:, 0].min()
s, e, ln = (b[:, 0] - t0) / 100.0, (b[:, 1] - t0) / 100.0, b[:, 2]   # microseconds
print("busy blocks", len(b), "span (first start .. last end) us", round(e.max() - s.min(), 1))
for k in np.argsort(-e)[:8]:
    print(f"  len {ln[k]:6d} start {s[k]:7.1f} end {e[k]:7.1f} dur {e[k]-s[k]:7.1f}")
for lo, hi in [(0, 512), (512, 2048), (2048, 4096), (4096, 8192), (8192, 1 << 30)]:
    m = (ln >= lo) & (ln < hi)
    if m.any():
        print(f"  len [{lo},{hi}): n={m.sum():4d} mean dur {np.mean(e[m]-s[m]):7.1f} max dur {np.max(e[m]-s[m]):7.1f} "
              f"mean start {np.mean(s[m]):6.1f} max end {np.max(e[m]):6.1f}")
