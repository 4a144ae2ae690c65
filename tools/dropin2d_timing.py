"""Single-camera 2D render (the drop-in GaussianRenderer2D.render call: one image per call) at
config 4's scene (500k Gaussians, 576x512): fwd+bwd per call, eager, HIP-event timed."""
import sys

import torch

sys.path.insert(0, "pose-splatter_amd")


def main():
    from gsr import render as R
    from gsr.scenes import gaussians2d
    dev = torch.device("cuda:0")
    W, H = 576, 512
    p = gaussians2d(500000, W, H, 1004).to(dev)
    bg = torch.ones(3, device=dev)
    g = torch.Generator(device="cpu").manual_seed(5)
    vr, va = torch.randn(H, W, 3, generator=g).to(dev), torch.randn(H, W, generator=g).to(dev)

    def step():
        pg = p.detach().requires_grad_(True)
        rgb, a = R.render2d(pg, W, H, bg)
        torch.autograd.backward([rgb, a], [vr, va])
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 10
    e0.record()
    for _ in range(n):
        step()
    e1.record()
    torch.cuda.synchronize()
    print(f"single-camera render2d fwd+bwd: {e0.elapsed_time(e1) / n:.3f} ms per call")


if __name__ == "__main__":
    main()
