"""Per-workgroup phase timing of the per-tile 2D raster backward (k_raster2d_bwd_tile; timing
build: -DGSR_BWD_TRACE, build_var/libgsr_trace.so).  Usage: python tools/bwd2d_trace.py [config]
(default 4).  Per workgroup (one tile): start, end, sub-chunks, and wave 0's time summed over
its sub-chunks in: top barrier + record staging, culls, group walk, pre-rows barrier, rows."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("GSR_LIBRARY", os.path.join(ROOT, "build_var", "libgsr_trace.so"))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pose-splatter_amd")]
import ctypes
import torch
import bench
from gsr import _lib, render as R
from gsr.scenes import CONFIGS

cfg = CONFIGS[int(sys.argv[1]) if len(sys.argv) > 1 else 4]
dev = torch.device("cuda:0")
R.set_capacity_mode("bounded")
w = bench.Workload(cfg, dev, 1, 0, "units" if cfg.index == 4 else "views", 0, "none", comm=False)
for _ in range(3):
    w.step()
torch.cuda.synchronize()
L = _lib.lib()
buf = torch.zeros(1 << 22, dtype=torch.int64, device=dev)
L.gsr_debug_bwd_trace.argtypes = [ctypes.c_void_p]
assert L.gsr_debug_bwd_trace(buf.data_ptr()) == 0
for rep in range(2):
    buf.zero_()
    w.step()
    torch.cuda.synchronize()
    t16 = buf.view(-1, 16).cpu()
    t = t16[t16[:, 0] != 0].double()
    n = t.shape[0]
    t0 = t[:, 0].min()
    span = float(t[:, 1].max() - t0) * 0.01   # us (100 MHz wall clock)
    life = (t[:, 1] - t[:, 0]) * 0.01
    nsub = (t[:, 2].long() & 0xFFFFFFFF).double()
    cu = t[:, 2].long() >> 32
    n_cu = len(torch.unique(cu))
    print(f"rep {rep}: {n} tile WGs on {n_cu} CUs, span {span:.0f} us, mean WG {float(life.mean()):.1f} us "
          f"({float(nsub.mean()):.1f} sub-chunks, {float((life / nsub).mean()):.2f} us each), "
          f"avg WGs resident per CU {float(life.sum()) / span / n_cu:.2f}")
    names = ["top+staging", "culls", "groups", "rows barrier", "rows"]
    for i, nm in enumerate(names):
        x = t[:, 3 + i] * 0.01 / nsub
        print(f"   {nm:13s} per sub-chunk mean {float(x.mean()):6.2f} us  p90 {float(torch.quantile(x, 0.9)):6.2f}")
    end = (t[:, 1] - t0) * 0.01
    q = torch.quantile(end, torch.tensor([0.5, 0.9, 0.99, 1.0], dtype=torch.float64))
    print("   WG end time p50/p90/p99/max (us):", [round(float(v), 0) for v in q])
