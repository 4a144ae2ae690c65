"""Per-workgroup phase timing of the 3D raster forward (timing build: -DGSR_FWD_TRACE,
build_var/libgsr_ftrace.so).  Usage: python tools/fwd_trace.py [config]."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("GSR_LIBRARY", os.path.join(ROOT, "build_var", "libgsr_ftrace.so"))
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
buf = torch.zeros(16 << 17, dtype=torch.int64, device=dev)
L.gsr_debug_fwd_trace.argtypes = [ctypes.c_void_p]
assert L.gsr_debug_fwd_trace(buf.data_ptr()) == 0
for rep in range(2):
    buf.zero_()
    w.step()
    torch.cuda.synchronize()
    t = buf.view(-1, 16).cpu()
    t = t[t[:, 0] != 0].double()
    t0 = t[:, 0].min()
    a, f, wd, e = [(t[:, k] - t0) * 0.01 for k in range(4)]
    rounds, ln = t[:, 4], t[:, 5]
    smid = t[:, 6].long()
    d = e - a
    span = float(e.max())
    n_cu = len(torch.unique(smid))
    print(f"rep {rep}: {t.shape[0]} WGs on {n_cu} CUs, span {span:.1f} us, mean WG {float(d.mean()):.2f} us, "
          f"avg WGs resident per CU {float(d.sum()) / span / n_cu:.2f}")
    first = f - a
    walk = wd - f
    epi = e - wd
    print(f"   to first round {float(first.mean()):.2f} (p90 {float(torch.quantile(first, 0.9)):.2f})  "
          f"walk {float(walk.mean()):.2f} (p90 {float(torch.quantile(walk, 0.9)):.2f})  "
          f"epilogue {float(epi.mean()):.2f} (p90 {float(torch.quantile(epi, 0.9)):.2f}) us")
    print(f"   rounds mean {float(rounds.mean()):.1f} max {int(rounds.max())}; us per round {float((walk / rounds.clamp(min=1)).mean()):.2f}")
    order = torch.argsort(d, descending=True)
    ph = t[:, 8:12] * 0.01   # wave 0's per-phase totals (us): gather+cull, barrier, box culls, composites
    groups, surv = t[:, 12], t[:, 13]
    for i in order[:12].tolist():
        r = max(int(rounds[i]), 1)
        print(f"   WG len {int(ln[i])} rounds {int(rounds[i])} start {float(a[i]):.1f} first {float(first[i]):.1f} "
              f"walk {float(walk[i]):.1f} epi {float(epi[i]):.1f} end {float(e[i]):.1f} | per round (us): "
              f"gather+cull {float(ph[i, 0]) / r:.2f} barrier {float(ph[i, 1]) / r:.2f} "
              f"boxcull {float(ph[i, 2]) / r:.2f} composite {float(ph[i, 3]) / r:.2f} | wave0 groups/round "
              f"{float(groups[i]) / r:.1f} survivors/round {float(surv[i]) / r:.1f} "
              f"ns/group {1000.0 * float(ph[i, 3]) / max(float(groups[i]), 1.0):.0f}")
    tot = ph.sum(0)
    print(f"   all WGs, wave 0 phase totals (us): gather+cull {float(tot[0]):.0f} barrier {float(tot[1]):.0f} "
          f"boxcull {float(tot[2]):.0f} composite {float(tot[3]):.0f}; ns per composite group "
          f"{1000.0 * float(tot[3]) / max(float(groups.sum()), 1.0):.0f}")
    hist = torch.bincount(rounds.long())
    print("   WGs by rounds:", {i: int(c) for i, c in enumerate(hist.tolist()) if c})
    for thr in (8, 10, 12, 16):
        m = rounds >= thr
        print(f"   rounds >= {thr}: {int(m.sum())} WGs ({int(m.sum()) // 4} tiles), their WG-us {float(d[m].sum()):.0f} "
              f"of {float(d.sum()):.0f}")
    st = a.sort().values
    print("   start of the 50/90/99/100% WG:", [round(float(st[int(len(st) * q) - 1]), 1) for q in (0.5, 0.9, 0.99, 1.0)])
    bins = []
    for t_ in range(0, int(span) + 10, 10):
        bins.append(round(float(((a <= t_ + 5) & (e >= t_ + 5)).sum()) / n_cu, 2))
    print("   WGs alive per CU at 5,15,25.. us:", bins)
