"""Per-workgroup timing of the per-tile sort (timing build: -DGSR_SORT_TRACE,
build_var/libgsr_strace.so).  Usage: python tools/sort_trace.py [config] [variant]."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
var = sys.argv[2] if len(sys.argv) > 2 else "strace"
os.environ.setdefault("GSR_LIBRARY", os.path.join(ROOT, "build_var", f"libgsr_{var}.so"))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pose-splatter_amd")]
import ctypes
import torch
import bench
from gsr import _lib, render as R
from gsr.scenes import CONFIGS

cfg = CONFIGS[int(sys.argv[1]) if len(sys.argv) > 1 else 3]
dev = torch.device("cuda:0")
R.set_capacity_mode("bounded")
w = bench.Workload(cfg, dev, 1, 0, "views", 0, "none", comm=False)
for _ in range(4):
    w.step()
torch.cuda.synchronize()
L = _lib.lib()
buf = torch.zeros(12 << 16, dtype=torch.int64, device=dev)
L.gsr_debug_sort_trace.argtypes = [ctypes.c_void_p]
assert L.gsr_debug_sort_trace(buf.data_ptr()) == 0
for rep in range(2):
    buf.zero_()
    w.step()
    torch.cuda.synchronize()
    t12 = buf.view(-1, 12).cpu()
    t12 = t12[t12[:, 0] != 0].double()
    t = t12[:, :4]
    ph = t12[:, 4:]   # s_sort_ts: [1] varying done, [2..5] after LSD pass of digit 0..3, [6] passes done, [7] fix-up done
    a = (t[:, 0] - t[:, 0].min()) * 0.01
    e = (t[:, 1] - t[:, 0].min()) * 0.01
    ln = t[:, 2]
    d = e - a
    span = float(e.max())
    print(f"rep {rep}: {t.shape[0]} WGs, span {span:.1f} us, mean WG {float(d.mean()):.2f} us, "
          f"WG-us/CU {float(d.sum()) / 256:.1f}")
    order = torch.argsort(ln, descending=True)
    for i in order[:8].tolist():
        p = ph[i]
        rel = lambda k: (float(p[k] - t[i, 0]) * 0.01) if p[k] > 0 else -1.0
        print(f"   len {int(ln[i]):6d} start {float(a[i]):6.1f} end {float(e[i]):6.1f} dur {float(d[i]):6.1f}  "
              f"stage+or {rel(1):.1f} passes " + " ".join(f"{rel(k):.1f}" for k in range(2, 6)) +
              f" | radix done {rel(6):.1f} fixup done {rel(7):.1f}")
    for lo, hi in ((0, 1024), (1024, 2048), (2048, 4096), (4096, 8192), (8192, 16384), (16384, 1 << 30)):
        m = (ln >= lo) & (ln < hi)
        if m.any():
            print(f"   len [{lo},{hi}): {int(m.sum())} WGs, mean {float(d[m].mean()):.1f} us, "
                  f"us per 1k keys {float((d[m] / ln[m] * 1000).mean()):.2f}, total {float(d[m].sum()) / 256:.1f} us/CU")
    st = a.sort().values
    print("   start of the 50/90/99/100% WG:", [round(float(st[int(len(st) * f) - 1]), 1) for f in (0.5, 0.9, 0.99, 1.0)])
