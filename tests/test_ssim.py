"""SSIM term of the reference training loss (scripts/training/train_script.py:129):
gsr.loss.ssim (gsr_ssim_fwd / gsr_ssim_bwd) against oracle/ssim.py, a restatement of torchmetrics'
StructuralSimilarityIndexMeasure (torchmetrics is not installed: parity unpinned beyond that
restatement and the closed-form cases below)."""
import pytest
import torch

from _util import assert_close, grad_close


def test_oracle_identity_and_constant_images():
    from oracle.ssim import gaussian_taps, ssim
    g = torch.Generator().manual_seed(0)
    x = torch.rand(2, 3, 24, 30, generator=g)
    assert abs(float(ssim(x, x)) - 1.0) < 1e-6
    a, b = 0.3, 0.7
    # float64: in fp32 the variances E[x^2] - mx^2 of a constant image round to ~1e-7, which is
    # 1e-4 of C2
    xa, yb = torch.full((1, 3, 20, 20), a, dtype=torch.float64), torch.full((1, 3, 20, 20), b, dtype=torch.float64)
    c1, c2 = 0.01 ** 2, 0.03 ** 2
    exp = (2 * a * b + c1) / (a * a + b * b + c1)      # zero variances: the contrast term is c2 / c2
    assert abs(float(ssim(xa, yb)) - exp) < 1e-9
    t = gaussian_taps()
    assert t.numel() == 11 and abs(float(t.sum()) - 1.0) < 1e-6 and torch.equal(t, t.flip(0))


def test_ssim_api_cpu():
    from gsr.loss import ssim
    with pytest.raises(RuntimeError, match="CUDA|HIP|device"):
        ssim(torch.rand(3, 16, 16), torch.rand(16, 16, 3))
    with pytest.raises(ValueError):
        ssim(torch.rand(3, 8, 8), torch.rand(8, 8, 3))          # smaller than the 11x11 window
    with pytest.raises(ValueError):
        ssim(torch.rand(2, 3, 16, 16), torch.rand(1, 16, 16, 3))


@pytest.mark.gpu
@pytest.mark.parametrize("C,H,W,seed", [(1, 24, 30, 1), (2, 40, 56, 2), (6, 96, 128, 3), (1, 512, 576, 4)])
def test_ssim_vs_oracle(cuda, C, H, W, seed):
    from gsr.loss import ssim
    from oracle.ssim import ssim as ref
    g = torch.Generator().manual_seed(seed)
    x = torch.rand(C, 3, H, W, generator=g)
    y = (x.permute(0, 2, 3, 1) + 0.2 * torch.randn(C, H, W, 3, generator=g)).clamp(0, 1)   # correlated
    yd = y.to(cuda).requires_grad_(True)
    s = ssim(x.to(cuda), yd)
    s.backward(torch.tensor(0.7, device=cuda))
    yo = y.clone().requires_grad_(True)
    so = ref(x, yo.permute(0, 3, 1, 2))      # ssim(target_img, rgb) argument order as the reference
    (0.7 * so).backward()
    assert_close(s.detach().cpu()[None], so.detach()[None], rtol=1e-5, atol=1e-6, what="ssim")
    grad_close(yd.grad.cpu(), yo.grad, what="d ssim / d rgb")
    s2 = ssim(x.to(cuda), yd.detach())
    assert torch.equal(s.detach(), s2)       # fixed-order reduction


@pytest.mark.gpu
def test_ssim_in_fused_training_loss(cuda):
    """The full reference loss (IoU + L1 fused in the raster backward, plus ssim_lambda * (1 - SSIM)
    from gsr_ssim_*) gives the gradient of the same loss built from torch ops and the oracle SSIM."""
    from gsr.loss import render3d_iou_l1, ssim
    from gsr.render import render3d
    from gsr.scenes import gaussians3d, ring_cameras
    from oracle.ssim import ssim as ref_ssim
    W, H, C = 96, 80, 2
    p = gaussians3d(3000, 31, extent=0.05)
    V, K = ring_cameras(C, W, H)
    g = torch.Generator().manual_seed(32)
    timg = torch.rand(C, 3, H, W, generator=g).to(cuda)
    tmask = (torch.rand(C, H, W, generator=g) < 0.3).float().to(cuda)
    bg = torch.ones(3, device=cuda)
    lam = 0.8
    p1 = p.to(cuda).requires_grad_(True)
    li, lm, rgb, _ = render3d_iou_l1(p1, V.to(cuda), K.to(cuda), W, H, bg, timg, tmask, 1.0)
    (li + lm + lam * (1 - ssim(timg, rgb))).backward()
    p2 = p.to(cuda).requires_grad_(True)
    rgb2, a2 = render3d(p2, V.to(cuda), K.to(cuda), W, H, bg)
    inter = (a2 * tmask).sum(dim=(-2, -1))
    union = (a2 + tmask - a2 * tmask).sum(dim=(-2, -1))
    li2 = 1 - ((inter + 1e-6) / (union + 1e-6)).mean()
    lm2 = torch.abs(timg - rgb2.permute(0, 3, 1, 2)).sum() / tmask.sum()
    (li2 + lm2 + lam * (1 - ref_ssim(timg, rgb2.permute(0, 3, 1, 2)))).backward()
    grad_close(p1.grad.cpu(), p2.grad.cpu(), what="v_params with SSIM")
