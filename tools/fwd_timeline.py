"""Per-workgroup timeline of the 3D raster forward (needs a -DGSR_EXP_TIMELINE build via
GSR_LIBRARY; s_memrealtime stamps, 100 MHz).  Prints the busy span, the last-finishing
workgroups and duration statistics by list length."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pose-splatter_amd"))
import torch  # noqa: E402
from gsr import render as R  # noqa: E402
from gsr._lib import lib  # noqa: E402
from gsr.scenes import CONFIGS, gaussians3d, ring_cameras  # noqa: E402

cfg = CONFIGS[int(sys.argv[1]) if len(sys.argv) > 1 else 3]
dev = torch.device("cuda:0")
p = gaussians3d(cfg.N, cfg.seed).to(dev)
V, K = ring_cameras(cfg.views, cfg.width, cfg.height)
V, K = V.to(dev), K.to(dev)
bg = torch.ones(3, device=dev)
L = lib()
fbk = L.gsr_debug_blocks
fbk.argtypes = [ctypes.c_void_p]
with torch.no_grad():
    for _ in range(3):
        R.render3d(p, V, K, cfg.width, cfg.height, bg)
torch.cuda.synchronize()
R.enable_kernel_timing(True)
with torch.no_grad():
    R.render3d(p, V, K, cfg.width, cfg.height, bg)
print({k: round(v[0], 4) for k, v in R.kernel_times_ms().items()})
st = R.last_stats()
blk = np.zeros((32768, 3), dtype=np.uint64)
fbk(blk.ctypes.data)
nb = 32 * ((st["n_busy"] + 7) // 8)
b = blk[:nb].astype(np.int64)
b = b[b[:, 1] > 0]
t0 = b[:, 0].min()
s, e, ln = (b[:, 0] - t0) / 100.0, (b[:, 1] - t0) / 100.0, b[:, 2]
print("busy blocks", len(b), "span us", round(e.max() - s.min(), 1))
for k in np.argsort(-e)[:6]:
    print(f"  len {ln[k]:6d} start {s[k]:7.1f} end {e[k]:7.1f} dur {e[k]-s[k]:7.1f}")
for lo, hi in [(0, 512), (512, 2048), (2048, 4096), (4096, 8192), (8192, 1 << 30)]:
    m = (ln >= lo) & (ln < hi)
    if m.any():
        print(f"  len [{lo},{hi}): n={m.sum():4d} mean dur {np.mean(e[m]-s[m]):7.1f} max dur {np.max(e[m]-s[m]):7.1f} "
              f"mean start {np.mean(s[m]):6.1f} max end {np.max(e[m]):6.1f}")
# occupancy profile: workgroups in flight over time
ts = np.linspace(0, e.max(), 12)
print("in flight:", [int(((s <= t) & (e > t)).sum()) for t in ts])
