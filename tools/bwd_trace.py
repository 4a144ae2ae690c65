"""Per-workgroup phase timing of the 3D raster backward (timing build: -DGSR_BWD_TRACE,
build_var/libgsr_trace.so).  Usage: python tools/bwd_trace.py [config]  (default 3)."""
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

cfg = CONFIGS[int(sys.argv[1]) if len(sys.argv) > 1 else 3]
dev = torch.device("cuda:0")
R.set_capacity_mode("bounded")
w = bench.Workload(cfg, dev, 1, 0, "views", 0, "none", comm=False)
for _ in range(4):
    w.step()
torch.cuda.synchronize()
L = _lib.lib()
buf = torch.zeros(1 << 22, dtype=torch.int64, device=dev)
L.gsr_debug_bwd_trace.argtypes = [ctypes.c_void_p]
assert L.gsr_debug_bwd_trace(buf.data_ptr()) == 0
for rep in range(3):
    buf.zero_()
    w.step()
    torch.cuda.synchronize()
    t16 = buf.view(-1, 16).cpu()
    keep = t16[:, 0] != 0
    nbox = t16[keep][:, 8:].contiguous().view(torch.int32).double()   # [wg, 16] survivors per 4x4 box
    t = t16[keep][:, :8].double()
    t0 = t[:, 0].min()
    ph = t[:, :7] - t0
    span = float(ph[:, 6].max() - ph[:, 0].min()) * 0.01
    d = (t[:, 1:7] - t[:, 0:6]) * 0.01   # us (100 MHz wall clock)
    smid = (t[:, 7].long() >> 32)
    ngrp = (t[:, 7].long() & 0xFFFFFFFF).double()
    n_cu = len(torch.unique(smid))
    busy = float((t[:, 6] - t[:, 0]).sum()) * 0.01
    print(f"rep {rep}: {t.shape[0]} WGs on {n_cu} CUs, span {span:.1f} us, mean WG {busy / t.shape[0]:.2f} us, "
          f"avg WGs resident per CU {busy / span / n_cu:.2f}")
    names = ["desc+stats", "loads->LDS", "culls", "groups", "barrier", "rows"]
    for i, nm in enumerate(names):
        x = d[:, i]
        q = torch.quantile(x, torch.tensor([0.1, 0.5, 0.9], dtype=torch.float64))
        print(f"   {nm:11s} mean {float(x.mean()):6.2f}  p10 {float(q[0]):6.2f}  p50 {float(q[1]):6.2f}  p90 {float(q[2]):6.2f} us"
              f"   sum/span/CUs {float(x.sum()) / span / n_cu:.2f}")
    print(f"   groups/wave0 mean {float(ngrp.mean()):.1f}, us per group {float((d[:, 3] / ngrp.clamp(min=1)).mean()):.3f}")
    # start-time histogram: how fast WGs get dispatched
    st = (ph[:, 0] * 0.01).sort().values
    k = [int(len(st) * f) for f in (0.1, 0.25, 0.5, 0.75, 0.9)]
    print("   dispatch time of the 10/25/50/75/90% WG:", [round(float(st[i]), 1) for i in k])
    # the group walk's cost model: now max over each wave's 4 boxes of ceil(n/7) (the slowest wave
    # sets the workgroup); entry-split alternative: a wave walks one box at a time, 4 lanes per
    # pixel (28 entries per group), boxes dealt to the waves -> max over waves of sum ceil(n/28)
    if rep == 0:
        os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
        torch.save({"nbox": nbox, "t": t}, os.path.join(ROOT, "gpurun_out", f"bwd_trace_cfg{cfg.index}.pt"))
    g7 = torch.ceil(nbox / 7)
    now = g7.view(-1, 4, 4).max(2).values.max(1).values
    g28 = torch.ceil(nbox / 28)
    srt = g28.sort(1, descending=True).values
    waves = torch.zeros(srt.shape[0], 4, dtype=torch.float64)
    for j in range(16):   # greedy: largest box to the least loaded wave
        i = waves.argmin(1)
        waves[torch.arange(srt.shape[0]), i] += srt[:, j]
    split = waves.max(1).values
    print(f"   groups per WG (critical wave): now {float(now.mean()):.1f}, entry-split {float(split.mean()):.1f}; "
          f"box survivors mean {float(nbox.mean()):.1f} max/box {float(nbox.max(1).values.mean()):.1f}")
    # residency: WGs alive per CU (max over the run), and all CUs' WGs alive per 10 us bin
    a, e = ph[:, 0] * 0.01, ph[:, 6] * 0.01
    mx = []
    for cu in torch.unique(smid).tolist():
        m = smid == cu
        ev = sorted([(float(x), 1) for x in a[m]] + [(float(x), -1) for x in e[m]], key=lambda z: (z[0], z[1]))
        cur = best = 0
        for _, dlt in ev:
            cur += dlt
            best = max(best, cur)
        mx.append(best)
    mx = torch.tensor(mx)
    print(f"   max WGs alive on one CU: min {int(mx.min())} median {int(mx.median())} max {int(mx.max())}")
    bins = []
    for t_ in range(0, int(span) + 10, 10):
        alive = ((a <= t_ + 5) & (e >= t_ + 5)).sum()
        bins.append(round(float(alive) / n_cu, 2))
    print("   WGs alive per CU at 5,15,25.. us:", bins)
