"""Bitwise comparison of two builds of libgsr.so on the 2D path (forward images, T and last
records, and the parameter gradient of a multi-frame batch), e.g. the packed-FP32 pair forward
against its scalar build:  python3 tools/cmp_libs2d.py build_var/libgsr_pk0.so pose-splatter_amd/gsr/lib/libgsr.so
Each build runs in its own process (the library is chosen at import by GSR_LIBRARY)."""
import os
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")


def child(tag: str):
    sys.path.insert(0, os.path.join(ROOT, "pose-splatter_amd"))
    from gsr import render as R
    from gsr.scenes import gaussians2d
    dev = torch.device("cuda:0")
    W, H, F, views = 576, 512, 2, 3
    res = {}
    for N in (20000, 120000):
        p = torch.stack([gaussians2d(N, W, H, 11 + f) for f in range(F)]).to(dev).requires_grad_(True)
        sets = [f for f in range(F) for _ in range(views)]
        bg = torch.ones(3, device=dev)
        rgb, alpha = R.render2d_units(p, sets, W, H, bg)
        g = torch.Generator().manual_seed(4)
        vr = torch.randn(rgb.shape, generator=g).to(dev)
        va = torch.randn(alpha.shape, generator=g).to(dev)
        torch.autograd.backward([rgb, alpha], [vr, va])
        torch.cuda.synchronize()
        res[f"rgb{N}"], res[f"alpha{N}"], res[f"grad{N}"] = rgb.detach().cpu(), alpha.detach().cpu(), p.grad.cpu()
    torch.save(res, os.path.join(OUT, f"cmp2d_{tag}.pt"))
    print("child", tag, "done", flush=True)


def main():
    if sys.argv[1] == "--child":
        child(sys.argv[2])
        return
    os.makedirs(OUT, exist_ok=True)
    for tag, lib in (("a", sys.argv[1]), ("b", sys.argv[2])):
        env = dict(os.environ, GSR_LIBRARY=os.path.abspath(lib))
        subprocess.run([sys.executable, "-u", os.path.abspath(__file__), "--child", tag], env=env, check=True,
                       timeout=300)
    a = torch.load(os.path.join(OUT, "cmp2d_a.pt"), weights_only=True)
    b = torch.load(os.path.join(OUT, "cmp2d_b.pt"), weights_only=True)
    ok = True
    for k in a:
        same = torch.equal(a[k], b[k])
        ok &= same
        print(k, "bitwise equal" if same else f"DIFFER: {int((a[k] != b[k]).sum())} of {a[k].numel()}, "
              f"max |d| {float((a[k] - b[k]).abs().max()):.3e}")
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
