"""Tile list-length distribution of a bench config (which sort class / path each tile takes)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pose-splatter_amd"))
import torch  # noqa: E402
from gsr import render as R  # noqa: E402
from gsr.scenes import CONFIGS, gaussians3d, ring_cameras  # noqa: E402

cfg = CONFIGS[int(sys.argv[1]) if len(sys.argv) > 1 else 5]
dev = torch.device("cuda:0")
p = gaussians3d(cfg.N, cfg.seed).to(dev)
V, K = ring_cameras(cfg.views, cfg.width, cfg.height)
with torch.no_grad():
    _, _, b, _ = R.debug_forward3d(p, V.to(dev), K.to(dev), torch.ones(3, device=dev), cfg.width, cfg.height)
off = b.tile_off.cpu().to(torch.int64)
ln = off[1:] - off[:-1]
te = (b.tile_end.cpu().to(torch.int64) - off[:-1]).clamp(min=0)
print(cfg.name, "I", int(ln.sum()), "I_eff", int(te.sum()), "busy", int((ln > 0).sum()))
for lo, hi in [(1, 1024), (1024, 4096), (4096, 8192), (8192, 16385), (16385, 1 << 30)]:
    m = (ln >= lo) & (ln < hi)
    print(f"  len [{lo},{hi}): tiles {int(m.sum()):6d} entries {int(ln[m].sum()):10d} read {int(te[m].sum()):10d}")
busy = ln > 0
r = te[busy].double() / ln[busy].double()
print("  walk/len quantiles (tiles):", [round(float(torch.quantile(r, q)), 3) for q in (0.5, 0.9, 0.99, 1.0)])
for f in (0.25, 0.5, 0.75):
    over = busy & (te.double() > f * ln.double())
    print(f"  prefix {f:.2f} of each list: tiles that read past it {int(over.sum())}, their entries {int(ln[over].sum())}")
for lo in (8192, 16385):
    m = ln >= lo
    if int(m.sum()) == 0:
        continue
    w = te[m].double()
    print(f"  lists >= {lo}: walk quantiles", [int(torch.quantile(w, q)) for q in (0.5, 0.9, 0.95, 0.99, 1.0)])
    for P in (2048, 4096, 8192):
        print(f"    fixed prefix {P}: tiles reading past it {int((te[m] >= P).sum())}")
