"""Loss-fused render: gsr.loss.render3d_iou_l1 against the unfused
reference loss (oracle/loss.py restating scripts/training/train_script.py:30-36,128-130)
applied (a) to the same GPU render through ordinary autograd and (b) to the CPU oracle
render.  Tolerances: loss values 1e-5 relative (fp32 reductions in a different order),
gradients 1e-4 relative (north_star)."""
import pytest
import torch

from _util import assert_close, grad_close


def _case(N, W, H, C, seed, mask_frac=0.4):
    from gsr.scenes import gaussians3d, ring_cameras
    p = gaussians3d(N, seed, extent=0.05)
    p[:, 3:6] += 1.0
    V, K = ring_cameras(C, W, H)
    g = torch.Generator().manual_seed(seed + 5)
    timg = torch.rand(C, 3, H, W, generator=g)
    tmask = (torch.rand(C, H, W, generator=g) < mask_frac).float()
    return p, V, K, timg, tmask


def test_shape_validation_cpu():
    from gsr.loss import render3d_iou_l1
    p, V, K, timg, tmask = _case(10, 32, 24, 2, 1)
    with pytest.raises(ValueError, match="target_img"):
        render3d_iou_l1(p, V, K, 32, 24, torch.ones(3), timg[:, :, :, :16], tmask)
    with pytest.raises(ValueError, match="target_mask"):
        render3d_iou_l1(p, V, K, 32, 24, torch.ones(3), timg, tmask[:1])
    with pytest.raises(RuntimeError):
        render3d_iou_l1(p, V, K, 32, 24, torch.ones(3), timg, tmask)   # no CPU compute path


def test_oracle_loss_matches_reference_formula_by_hand():
    """The restatement on a 2x2 example worked by hand."""
    from oracle.loss import get_iou_loss, img_loss
    a = torch.tensor([[[0.5, 1.0], [0.0, 0.25]]])
    m = torch.tensor([[[1.0, 1.0], [0.0, 0.0]]])
    inter = 0.5 + 1.0
    union = (0.5 + 1 - 0.5) + (1 + 1 - 1) + 0 + 0.25
    assert abs(float(get_iou_loss(a, m)) - (1 - (inter + 1e-6) / (union + 1e-6))) < 1e-7
    rgb = torch.zeros(1, 2, 2, 3)
    t = torch.ones(1, 3, 2, 2)
    assert abs(float(img_loss(rgb, t, m, 2.0)) - 2.0 * 12 / 2) < 1e-6


def _unfused_gpu(p, V, K, W, H, bg, timg, tmask, lam, cuda, extra):
    from gsr.render import render3d
    from oracle.loss import get_iou_loss, img_loss
    pg = p.to(cuda).requires_grad_(True)
    rgb, alpha = render3d(pg, V.to(cuda), K.to(cuda), W, H, bg.to(cuda))
    li = get_iou_loss(alpha, tmask.to(cuda))
    lm = img_loss(rgb, timg.to(cuda), tmask.to(cuda), lam)
    tot = li + lm + (extra(rgb, alpha) if extra else 0)
    tot.backward()
    return li.detach().cpu(), lm.detach().cpu(), pg.grad.cpu()


def _fused_gpu(p, V, K, W, H, bg, timg, tmask, lam, cuda, extra):
    from gsr.loss import render3d_iou_l1
    pg = p.to(cuda).requires_grad_(True)
    li, lm, rgb, alpha = render3d_iou_l1(pg, V.to(cuda), K.to(cuda), W, H, bg.to(cuda), timg.to(cuda),
                                         tmask.to(cuda), lam)
    tot = li + lm + (extra(rgb, alpha) if extra else 0)
    tot.backward()
    return li.detach().cpu(), lm.detach().cpu(), pg.grad.cpu()


def _ssim_like(rgb, alpha):
    # a smooth extra term on rgb and alpha (stands in for SSIM): exercises the extra cotangents
    return 0.3 * (rgb * rgb).mean() + 0.1 * (alpha * alpha).mean()


@pytest.mark.gpu
@pytest.mark.parametrize("N,W,H,C,seed,lam,extra", [
    (500, 64, 48, 1, 11, 1.0, False),
    (4000, 96, 80, 3, 12, 0.5, True),
])
def test_fused_equals_unfused(cuda, N, W, H, C, seed, lam, extra):
    p, V, K, timg, tmask = _case(N, W, H, C, seed)
    bg = torch.ones(3)
    ex = _ssim_like if extra else None
    li_u, lm_u, g_u = _unfused_gpu(p, V, K, W, H, bg, timg, tmask, lam, cuda, ex)
    li_f, lm_f, g_f = _fused_gpu(p, V, K, W, H, bg, timg, tmask, lam, cuda, ex)
    assert_close(li_f, li_u, rtol=1e-5, what="iou_loss")
    assert_close(lm_f, lm_u, rtol=1e-5, what="img_loss")
    grad_close(g_f, g_u, what="v_params")


@pytest.mark.gpu
def test_fused_vs_cpu_oracle(cuda):
    from oracle import oracle3d
    from oracle.loss import get_iou_loss, img_loss
    W, H, C = 48, 40, 2
    p, V, K, timg, tmask = _case(300, W, H, C, 13)
    bg = torch.ones(3)
    li_f, lm_f, g_f = _fused_gpu(p, V, K, W, H, bg, timg, tmask, 1.0, cuda, None)
    pc = p.clone().requires_grad_(True)
    rgb, alpha = oracle3d.render3d(pc, V, K, W, H, bg)
    li, lm = get_iou_loss(alpha, tmask), img_loss(rgb, timg, tmask, 1.0)
    (li + lm).backward()
    assert_close(li_f, li.detach(), rtol=1e-5, what="iou_loss")
    assert_close(lm_f, lm.detach(), rtol=1e-5, what="img_loss")
    # sign(rgb - t) flips where the two renders straddle the target (|rgb - t| ~ 1e-7): rare
    grad_close(g_f, pc.grad, what="v_params", max_frac=2e-3, outlier_rel=2e-3)


@pytest.mark.gpu
def test_fused_deterministic(cuda):
    p, V, K, timg, tmask = _case(3000, 80, 64, 2, 14)
    r1 = _fused_gpu(p, V, K, 80, 64, torch.ones(3), timg, tmask, 1.0, cuda, None)
    r2 = _fused_gpu(p, V, K, 80, 64, torch.ones(3), timg, tmask, 1.0, cuda, None)
    assert all(torch.equal(a, b) for a, b in zip(r1, r2))
