"""Host-side latency of the forward's readback path (GPU box): the wait for the stats,
the host time from the wait to the sort call, and the sort call itself."""
import os, sys, time
sys.path.insert(0, "pose-splatter_amd")
import torch
from gsr import render as R
from gsr.scenes import CONFIGS, gaussians3d, ring_cameras
cfg = CONFIGS[3]
dev = torch.device("cuda:0")
p = gaussians3d(cfg.N, cfg.seed).to(dev).requires_grad_(True)
V, K = ring_cameras(cfg.views, cfg.width, cfg.height)
V, K = V.to(dev), K.to(dev)
bg = torch.ones(3, device=dev)
T = {}
orig_off, orig_sort = R._Bins.offsets_wait, R._Bins.sort
def off(self):
    T.setdefault("off_enter", []).append(time.perf_counter_ns())
    orig_off(self)
    T.setdefault("off_exit", []).append(time.perf_counter_ns())
def sort(self, o, s):
    T.setdefault("sort_enter", []).append(time.perf_counter_ns())
    orig_sort(self, o, s)
    T.setdefault("sort_exit", []).append(time.perf_counter_ns())
R._Bins.offsets_wait, R._Bins.sort = off, sort
vr = torch.randn(cfg.views, cfg.height, cfg.width, 3, device=dev)
va = torch.randn(cfg.views, cfg.height, cfg.width, device=dev)
for i in range(30):
    rgb, alpha = R.render3d(p, V, K, cfg.width, cfg.height, bg)
    torch.autograd.backward([rgb, alpha], [vr, va])
torch.cuda.synchronize()
import statistics
n = len(T["off_exit"])
d1 = [(T["sort_enter"][i] - T["off_exit"][i]) / 1e3 for i in range(10, n)]
d2 = [(T["sort_exit"][i] - T["sort_enter"][i]) / 1e3 for i in range(10, n)]
d3 = [(T["off_exit"][i] - T["off_enter"][i]) / 1e3 for i in range(10, n)]
print("readback wait us", statistics.median(d3), "off_exit->sort_enter us", statistics.median(d1), "sort call us", statistics.median(d2))
