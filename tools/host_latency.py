"""Host-side timeline of one fwd+bwd step (GPU box): host time (us) of each library call
relative to the end of the forward's stats readback, medians over steps.  If the host
reaches a launch later than the GPU finishes the previous kernel, the GPU idles."""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "pose-splatter_amd"))
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
marks = []
L = lib()
for name in ["gsr3d_project_fwd", "gsr_bin_offsets", "gsr_bin_emit", "gsr_bin_sort", "gsr3d_raster_fwd",
             "gsr3d_raster_bwd", "gsr3d_project_bwd"]:
    f = getattr(L, name)

    def wrap(*a, _f=f, _n=name):
        marks.append((_n, time.perf_counter_ns()))
        return _f(*a)
    setattr(L, name, wrap)
orig_wait = R._Bins.offsets_wait


def wait(self):
    marks.append(("wait_begin", time.perf_counter_ns()))
    orig_wait(self)
    marks.append(("wait_end", time.perf_counter_ns()))


R._Bins.offsets_wait = wait
vr = torch.randn(cfg.views, cfg.height, cfg.width, 3, device=dev)
va = torch.randn(cfg.views, cfg.height, cfg.width, device=dev)
steps = []
for i in range(40):
    marks.clear()
    params_grad = None
    p.grad = None
    rgb, alpha = R.render3d(p, V, K, cfg.width, cfg.height, bg)
    torch.autograd.backward([rgb, alpha], [vr, va])
    marks.append(("step_end", time.perf_counter_ns()))
    steps.append(list(marks))
torch.cuda.synchronize()
ref = "wait_end"
names = [n for n, _ in steps[-1]]
for n in names:
    vals = []
    for s in steps[10:]:
        d = dict(s)
        vals.append((d[n] - d[ref]) / 1e3)
    print(f"{n:22s} {statistics.median(vals):9.1f} us")
