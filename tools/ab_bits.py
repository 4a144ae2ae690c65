"""Bitwise A/B of two libgsr builds on fixed scenes (timing changes must not move a bit).

Usage (on the GPU box):  python tools/ab_bits.py OUT.npz [SCENE ...]   -- GSR_LIBRARY selects the build
                          python tools/ab_bits.py --cmp A.npz B.npz
Scenes: the fit test's start scene (300 Gaussians, 48x40, one view), config 3 (200k, 576x512, six
views) and a config-5-sized band, each forward + backward with a fixed random cotangent.
"""
import sys

import numpy as np
import torch

sys.path.insert(0, "pose-splatter_amd")


def scenes():
    from gsr.scenes import gaussians3d, ring_cameras
    V, K = ring_cameras(1, 48, 40, radius=0.3)
    yield "fit", gaussians3d(300, 1001), V, K, 48, 40
    V, K = ring_cameras(6, 576, 512)
    yield "cfg3", gaussians3d(200000, 1003), V, K, 576, 512
    V, K = ring_cameras(2, 1152, 1024)
    yield "big", gaussians3d(2000000, 1005), V, K, 1152, 1024


def run(out, only=None):
    from gsr import render as R
    dev = torch.device("cuda:0")
    res = {}
    for name, p, V, K, W, H in scenes():
        if only and name not in only:
            continue
        p = p.to(dev).requires_grad_(True)
        bg = torch.ones(3, device=dev)
        rgb, a = R.render3d(p, V.to(dev), K.to(dev), W, H, bg)
        g = torch.Generator(device="cpu").manual_seed(7)
        vr = torch.randn(rgb.shape, generator=g).to(dev)
        va = torch.randn(a.shape, generator=g).to(dev)
        (rgb * vr).sum().add_((a * va).sum()).backward()
        res[name + "_rgb"] = rgb.detach().cpu().numpy()
        res[name + "_alpha"] = a.detach().cpu().numpy()
        res[name + "_grad"] = p.grad.detach().cpu().numpy()
        print(name, "done", flush=True)
    np.savez(out, **res)


def cmp(a, b):
    A, B = np.load(a), np.load(b)
    bad = 0
    for k in A.files:
        x, y = A[k], B[k]
        same = np.array_equal(x.view(np.uint32), y.view(np.uint32))
        d = float(np.nanmax(np.abs(x - y))) if not same else 0.0
        n = int((x.view(np.uint32) != y.view(np.uint32)).sum())
        print(f"{k:12s} {'identical' if same else 'DIFFERS'}  elements differing {n}  max |diff| {d:.3e}")
        bad += not same
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    if sys.argv[1] == "--cmp":
        cmp(sys.argv[2], sys.argv[3])
    else:
        run(sys.argv[1], sys.argv[2:])
