"""Where does a bounded step (fwd+bwd) of the split-sort scene first differ from the exact one?"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pose-splatter_amd")]
import torch
from gsr import render as R
from gsr.scenes import gaussians3d, ring_cameras
dev = torch.device("cuda:0")
W, H, C, N = 96, 80, 1, 30000
p = gaussians3d(N, 3).to(dev)
V, K = [t.to(dev) for t in ring_cameras(C, W, H)]
g = torch.Generator().manual_seed(4)
vr = torch.randn(C, H, W, 3, generator=g).to(dev)
va = torch.randn(C, H, W, generator=g).to(dev)
bg = torch.ones(3, device=dev)
outs = []
def poison(byte):
    # hand garbage to the caching allocator: later torch.empty calls reuse these blocks
    ts = [torch.full((n,), byte, dtype=torch.uint8, device=dev) for n in
          [1 << k for k in range(10, 27)] * 3]
    del ts
for i, cap in enumerate(("exact", "bounded", "exact", "bounded")):
    poison(0xFF if i % 2 else 0x7F)
    pg = p.clone().requires_grad_(True)
    rgb, alpha = R.render3d(pg, V, K, W, H, bg, R.RenderOptions3D(capacity=cap))
    b = R.last_stats()["_bins"]
    torch.autograd.backward([rgb, alpha], [vr, va])
    torch.cuda.synchronize()
    outs.append(dict(rgb=rgb.detach().clone(), grad=pg.grad.clone(), te=b.tile_end.clone(), cut=b.tile_cut.clone(),
                     stats=b.pre.view("stats_dev", torch.int32)[:16].tolist(), n_chunks=b.n_chunks,
                     ce=b.chunk_entries, lazy=b.n_lazy))
print("status", R.overflow_status(dev))
for i in range(1, 4):
    a, o = outs[0], outs[i]
    print(i, "stats", o["stats"][:8], "ovf", o["stats"][12], "ce", o["stats"][13], "n_chunks", o["n_chunks"], "lazy", o["lazy"])
    for k in ("rgb", "grad", "te", "cut"):
        if not torch.equal(a[k], o[k]):
            d = (a[k] != o[k]).nonzero()
            print("   ", k, "DIFF at", d[:5].tolist(), "count", int(d.shape[0]),
                  "max abs", float((a[k].double() - o[k].double()).abs().max()))
print("exact", outs[0]["stats"][:8], outs[0]["n_chunks"], outs[0]["lazy"])
