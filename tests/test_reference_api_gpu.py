"""GPU: the reference's renderer tests (tests/test_gaussian_renderer.py) run against the
drop-in on a HIP device — same inputs, same assertions, plus numeric checks against the
reference fixtures where the reference test is only qualitative."""
import math

import pytest
import torch

from src.gaussian_renderer import GaussianRenderer2D, GaussianRenderer3D, create_renderer

pytestmark = pytest.mark.gpu


def test_single_gaussian_render(cuda):
    r = GaussianRenderer2D(256, 256, device="cuda")
    params = torch.tensor([[128.0, 128.0, 1.0, 1.0, 0.0, 1.0, 0.0, 0.0, 2.0]], device=cuda)
    rgb, alpha = r.render(params, None, None)
    assert rgb.shape == (256, 256, 3) and alpha.shape == (256, 256)
    assert rgb[128, 128, 0] > 0.5 and rgb[128, 128, 1] < 0.1 and rgb[128, 128, 2] < 0.1
    assert alpha[128, 128] > 0.5 and alpha[0, 0] < 0.1
    assert abs(float(rgb[128, 128, 0]) - 0.8807970285415649) < 1e-6


def test_out_of_bounds_gaussian(cuda):
    r = GaussianRenderer2D(256, 256, device="cuda")
    rgb, alpha = r.render(torch.tensor([[-100.0, -100.0, 1.0, 1.0, 0.0, 1.0, 0.0, 0.0, 2.0]], device=cuda), None, None)
    assert alpha.max() < 0.01


def test_multiple_gaussians(cuda):
    r = GaussianRenderer2D(256, 256, device="cuda")
    params = torch.tensor([[64.0, 128.0, 1.0, 1.0, 0.0, 1.0, 0.0, 0.0, 2.0],
                           [192.0, 128.0, 1.0, 1.0, 0.0, 0.0, 0.0, 1.0, 2.0]], device=cuda)
    rgb, _ = r.render(params, None, None)
    assert rgb[128, 64, 0] > 0.5 and rgb[128, 64, 2] < 0.1
    assert rgb[128, 192, 2] > 0.5 and rgb[128, 192, 0] < 0.1


def test_rotation(cuda):
    r = GaussianRenderer2D(256, 256, device="cuda")
    ph = torch.tensor([[128.0, 128.0, math.log(5.0), math.log(2.0), 0.0, 1.0, 0.0, 0.0, 2.0]], device=cuda)
    pv = torch.tensor([[128.0, 128.0, math.log(5.0), math.log(2.0), math.pi / 2, 1.0, 0.0, 0.0, 2.0]], device=cuda)
    _, ah = r.render(ph, None, None)
    _, av = r.render(pv, None, None)
    assert ah[128, 120] > ah[120, 128]
    assert av[120, 128] > av[128, 120]


def test_background_color_empty(cuda):
    r = GaussianRenderer2D(256, 256, device="cuda")
    r.set_background_color(torch.tensor([0.0, 0.0, 1.0]))
    rgb, _ = r.render(torch.zeros((0, 9), device=cuda), None, None)
    assert torch.allclose(rgb[0, 0].cpu(), torch.tensor([0.0, 0.0, 1.0]), atol=1e-5)


def test_3d_render_basic(cuda):
    r = GaussianRenderer3D(256, 256, device="cuda")
    params = torch.randn(100, 14, generator=torch.Generator().manual_seed(0)).to(cuda)
    viewmat = torch.eye(4, device=cuda)
    K = torch.tensor([[256, 0, 128], [0, 256, 128], [0, 0, 1]], dtype=torch.float32, device=cuda)
    rgb, alpha = r.render(params, viewmat, K)
    assert rgb.shape == (256, 256, 3) and alpha.shape == (256, 256)
    assert torch.isfinite(rgb).all() and torch.isfinite(alpha).all()
    assert float(alpha.min()) >= 0.0 and float(alpha.max()) <= 1.0


def test_output_consistency(cuda):
    width, height = 128, 96
    rgb2, a2 = create_renderer("2d", width, height, device="cuda").render(torch.randn(10, 9, device=cuda), None, None)
    assert rgb2.shape == (height, width, 3) and a2.shape == (height, width)
    rgb3, a3 = create_renderer("3d", width, height, device="cuda").render(
        torch.randn(10, 14, device=cuda), torch.eye(4, device=cuda), torch.eye(3, device=cuda))
    assert rgb3.shape == (height, width, 3) and a3.shape == (height, width)


def test_model_caller_contract(cuda):
    """src/model.py:164-172: rgb[None] [1,H,W,3], alpha[None,...,None] [1,H,W,1], white bg,
    and multi-view eval (viewmat [C,4,4], K [C,3,3]) → [C,H,W,3] / [C,H,W]."""
    from gsr.scenes import gaussians3d, ring_cameras
    W, H = 96, 80
    r = create_renderer("3d", W, H, device="cuda")
    r.set_background_color(torch.ones(3, device=cuda))
    p = gaussians3d(2000, 3).to(cuda).requires_grad_(True)
    V, K = ring_cameras(3, W, H)
    rgb, alpha = r.render(p, V[1].to(cuda), K[1].to(cuda))
    assert rgb[None].shape == (1, H, W, 3) and alpha[None, ..., None].shape == (1, H, W, 1)
    assert float(rgb[0, 0].min()) == 1.0            # empty corner shows the white background
    (rgb.mean() + alpha.mean()).backward()
    assert p.grad.shape == p.shape and torch.isfinite(p.grad).all() and float(p.grad.abs().max()) > 0
    rgbC, alphaC = r.render(p.detach(), V.to(cuda), K.to(cuda))
    assert rgbC.shape == (3, H, W, 3) and alphaC.shape == (3, H, W)
    assert torch.equal(rgbC[1], rgb.detach())
