"""Eager model-style training step through the drop-in renderer (src/gaussian_renderer.py) at
BASELINE config 3: create_renderer("3d", 576, 512) with a white background, params [N,14]
requiring grad, all 6 views in one render call (model.py's multi-view path), a scalar loss and
loss.backward() -- no HIP graph, no capacity flags beyond the renderer's own.  Times
capacity="auto" (the drop-in default) against capacity="exact" (gsplat-style read-back every
forward).  Usage: python tools/dropin_timing.py [steps] > profiles/r04_dropin_cfg3.json
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pose-splatter_amd")]

import torch  # noqa: E402

from gsr import render as R  # noqa: E402
from gsr.scenes import CONFIGS, gaussians3d, ring_cameras  # noqa: E402
from src.gaussian_renderer import create_renderer  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    cfg = CONFIGS[3]
    dev = torch.device("cuda:0")
    p0 = gaussians3d(cfg.N, cfg.seed).to(dev)
    V, K = ring_cameras(cfg.views, cfg.width, cfg.height)
    V, K = V.to(dev), K.to(dev)
    g = torch.Generator().manual_seed(cfg.seed + 1)
    vr = torch.randn(cfg.views, cfg.height, cfg.width, 3, generator=g).to(dev)
    va = torch.randn(cfg.views, cfg.height, cfg.width, generator=g).to(dev)
    out = {"workload": cfg.name, "step": "eager: render 6 views + scalar loss + loss.backward()", "steps": steps}
    for cap in ("exact", "auto", "exact", "auto"):
        r = create_renderer("3d", cfg.width, cfg.height, device="cuda", capacity=cap)
        r.set_background_color(torch.ones(3, device=dev))
        params = p0.clone().requires_grad_(True)

        def step():
            params.grad = None
            rgb, alpha = r.render(params, V, K)
            loss = (rgb * vr).sum() + (alpha * va).sum()
            loss.backward()

        for _ in range(5):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        ms = 1000.0 * (time.perf_counter() - t0) / steps
        out.setdefault(cap, []).append(round(ms, 4))
        out.setdefault("bounded_" + cap, R.last_stats()["_bins"].bounded)
        R.check_overflow(dev)
        print(f"{cap}: {ms:.4f} ms/step", file=sys.stderr)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
