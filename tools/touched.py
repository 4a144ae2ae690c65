"""Share of the Gaussians each rank of the (view, tile-row) strong layout touches (nonzero
gradient rows): what a sparse gradient exchange could save over the dense all-reduce.
Usage: python tools/touched.py [config] [N]"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pose-splatter_amd")]
import json
import torch
import bench
from gsr import render as R
from gsr.multiview import unit_shard
from gsr.scenes import CONFIGS
cfg = CONFIGS[int(sys.argv[1]) if len(sys.argv) > 1 else 5]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 8
dev = torch.device("cuda:0")
w = bench.Workload(cfg, dev, 1, 0, "views", 0, "none", comm=False)
with torch.no_grad():
    R.render3d(w.params, w.Vd, w.Kd, cfg.width, cfg.height, w.bg)
th = (cfg.height + 15) // 16
tw = (cfg.width + 15) // 16
weights = [float(x) for x in R.tile_work().reshape(cfg.views * th, tw).sum(1).cpu()]
N = cfg.N
frac = []
union = torch.zeros(N, dtype=torch.bool, device=dev)
for r in range(n):
    v0, v1, band = unit_shard(cfg.views, th, n, r, weights, 0.3 * N)
    if v1 <= v0:
        frac.append(0.0)
        continue
    p = w.params.detach().clone().requires_grad_(True)
    rgb, alpha = R.render3d(p, w.Vd[v0:v1], w.Kd[v0:v1], cfg.width, cfg.height, w.bg, R.RenderOptions3D(band=band))
    torch.autograd.backward([rgb, alpha], [w.v_rgb_all[v0:v1], w.v_alpha_all[v0:v1]])
    nz = (p.grad != 0).any(1)
    frac.append(float(nz.float().mean()))
    print(f"rank {r}: views {v0}-{v1 - 1} band {band}: {float(nz.float().mean()) * 100:.1f}% of Gaussians touched", flush=True)
dense = N * 14 * 4
print(json.dumps({"config": cfg.name, "n": n, "touched_frac": frac, "max_touched_frac": max(frac),
                  "dense_bytes": dense,
                  "sparse_bytes_per_rank_max": max(frac) * N * (14 * 4 + 4)}))
