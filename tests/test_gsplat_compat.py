"""The gsplat `rasterization(**kw)` entry point: the direct gsplat calls
in src/model.py:339-365 and src/plots.py:41-60 served by libgsr with activated inputs.

CPU: argument validation (unsupported modes raise, no CPU compute path).
GPU: forward and gradients w.r.t. every input against the oracle restatement
(oracle3d.render3d(activated=True)), tolerance 1e-4 relative (north_star)."""
import pytest
import torch

from _util import assert_close, grad_close


def _inputs(N, C, W, H, seed, device="cpu"):
    from gsr.scenes import gaussians3d, ring_cameras
    p = gaussians3d(N, seed, extent=0.06)
    g = torch.Generator().manual_seed(seed + 1)
    means = p[:, 0:3].clone()
    scales = torch.exp(p[:, 3:6] + 1.0)
    quats = p[:, 6:10] * 3.0                     # un-normalised: gsplat renormalises
    colors = torch.rand(N, 3, generator=g) * 1.2 - 0.1   # not clamped by gsplat
    opac = torch.sigmoid(p[:, 13])
    V, K = ring_cameras(C, W, H)
    return [t.to(device) for t in (means, quats, scales, opac, colors)], V.to(device), K.to(device)


def test_rejects_unsupported_modes():
    from gsr.gsplat_compat import rasterization
    (m, q, s, o, c), V, K = _inputs(4, 1, 32, 32, 1)
    bad = [dict(sh_degree=3), dict(render_mode="RGB+D"), dict(rasterize_mode="antialiased"),
           dict(tile_size=8), dict(camera_model="fisheye"), dict(distributed=True)]
    for kw in bad:
        with pytest.raises(NotImplementedError):
            rasterization(m, q, s, o, c, V, K, 32, 32, **kw)


def test_no_cpu_path():
    from gsr.gsplat_compat import rasterization
    (m, q, s, o, c), V, K = _inputs(4, 1, 32, 32, 1)
    with pytest.raises(RuntimeError, match="CUDA|HIP|device"):
        rasterization(m, q, s, o, c, V, K, 32, 32)


def test_module_alias():
    import gsr.gsplat_compat as gc
    mod = gc.gsplat_module()
    assert mod.rendering is gc and mod.rasterization is gc.rasterization


def _oracle(m, q, s, o, c, V, K, W, H, bg, radius_clip, vr, va):
    from oracle import oracle3d
    leaves = [t.detach().clone().double().requires_grad_(True) for t in (m, q, s, o, c)]
    rows = torch.cat([leaves[0], leaves[2], leaves[1], leaves[4], leaves[3][:, None]], 1)
    rgb, alpha = oracle3d.render3d(rows, V.double(), K.double(), W, H, bg.double(),
                                   radius_clip=radius_clip, activated=True)
    ((rgb * vr.double()).sum() + (alpha * va.double()).sum()).backward()
    return rgb.detach(), alpha.detach(), [t.grad for t in leaves]


@pytest.mark.gpu
@pytest.mark.parametrize("N,C,W,H,seed,radius_clip,with_bg", [
    (300, 2, 64, 48, 3, 0.0, False),
    (3000, 3, 96, 80, 4, 2.0, True),
])
def test_vs_oracle(cuda, N, C, W, H, seed, radius_clip, with_bg):
    from gsr.gsplat_compat import rasterization
    (m, q, s, o, c), V, K = _inputs(N, C, W, H, seed)
    bg = torch.rand(C, 3, generator=torch.Generator().manual_seed(seed)) if with_bg else torch.zeros(C, 3)
    g = torch.Generator().manual_seed(seed + 7)
    vr, va = torch.randn(C, H, W, 3, generator=g), torch.randn(C, H, W, 1, generator=g)
    leaves = [t.to(cuda).requires_grad_(True) for t in (m, q, s, o, c)]
    rgb, alpha, meta = rasterization(*leaves, V.to(cuda), K.to(cuda), W, H, radius_clip=radius_clip,
                                     packed=False, absgrad=True, sh_degree=None,
                                     backgrounds=bg.to(cuda) if with_bg else None)
    assert rgb.shape == (C, H, W, 3) and alpha.shape == (C, H, W, 1)
    ((rgb * vr.to(cuda)).sum() + (alpha * va.to(cuda)).sum()).backward()
    rgb_o, a_o, g_o = _oracle(m, q, s, o, c, V, K, W, H, bg, radius_clip, vr, va[..., 0])
    assert_close(rgb.detach().cpu(), rgb_o, what="rgb")
    assert_close(alpha.detach().cpu()[..., 0], a_o, what="alpha")
    for name, t, e in zip(("means", "quats", "scales", "opacities", "colors"), leaves, g_o):
        grad_close(t.grad.cpu(), e, what=f"v_{name}", max_frac=1e-3, outlier_rel=2e-3)


@pytest.mark.gpu
def test_matches_adapter_path(cuda):
    """rasterization(activated) == GaussianRenderer3D.render(raw) on the same scene."""
    from gsr.gsplat_compat import rasterization
    from gsr.scenes import gaussians3d, ring_cameras
    from src.gaussian_renderer import GaussianRenderer3D
    W, H, C = 80, 64, 2
    p = gaussians3d(2000, 11, extent=0.06)
    V, K = ring_cameras(C, W, H)
    r = GaussianRenderer3D(W, H, device="cuda")
    r.set_background_color(torch.zeros(3, device=cuda))
    rgb_a, a_a = r.render(p.to(cuda), V.to(cuda), K.to(cuda))
    q = p[:, 6:10] / (p[:, 6:10].norm(dim=-1, keepdim=True) + 1e-8)
    rgb_s, a_s, _ = rasterization(p[:, 0:3].to(cuda), q.to(cuda), torch.exp(p[:, 3:6]).to(cuda),
                                  torch.sigmoid(p[:, 13]).to(cuda), p[:, 10:13].clamp(0, 1).to(cuda),
                                  V.to(cuda), K.to(cuda), W, H)
    assert_close(rgb_s, rgb_a, what="rgb")
    assert_close(a_s[..., 0], a_a, what="alpha")


def _sphere_cameras(W, H, n_theta=4, n_phi=8, radius=1.0, fov_deg=7.5):
    """The visual-feature renderer's cameras (scripts/preprocessing/calculate_visual_features.py
    :164-189): Gauss-Legendre polar angles x azimuths on a sphere, looking at the origin with
    +Z up, f = W / (2 tan(fov/2))."""
    import math
    import numpy as np
    x, _ = np.polynomial.legendre.leggauss(n_theta)
    f = 0.5 * W / math.tan(math.radians(fov_deg) / 2)
    K = torch.tensor([[f, 0.0, W / 2], [0.0, f, H / 2], [0.0, 0.0, 1.0]], dtype=torch.float64)
    views = []
    for th in np.arccos(x):
        for ph in np.linspace(0, 2 * np.pi, n_phi, endpoint=False):
            c = radius * torch.tensor([math.sin(th) * math.cos(ph), math.sin(th) * math.sin(ph), math.cos(th)],
                                      dtype=torch.float64)
            z = -c / c.norm()
            xa = torch.linalg.cross(z, torch.tensor([0.0, 0.0, 1.0], dtype=torch.float64))
            xa = xa / xa.norm()
            ya = torch.linalg.cross(z, xa)
            R = torch.stack([xa, ya, z])
            V = torch.eye(4, dtype=torch.float64)
            V[:3, :3] = R
            V[:3, 3] = -R @ c
            views.append(V)
    C = len(views)
    return torch.stack(views).float(), K[None].expand(C, 3, 3).float().contiguous()


def _model_splat_inputs(N, seed):
    """Activated inputs as src/model.py's Gaussian head hands them to splat (:339-365)."""
    from gsr.scenes import gaussians3d
    p = gaussians3d(N, seed)
    q = p[:, 6:10] / p[:, 6:10].norm(dim=-1, keepdim=True)
    return [p[:, 0:3].clone(), q, torch.exp(p[:, 3:6]), torch.sigmoid(p[:, 13]), p[:, 10:13].clamp(0, 1)]


def _oracle_f32(leaves, V, K, W, H, band, vr, va):
    from oracle import oracle3d
    lv = [t.detach().clone().requires_grad_(True) for t in leaves]
    rows = torch.cat([lv[0], lv[2], lv[1], lv[4], lv[3][:, None]], 1)
    rgb, alpha = oracle3d.render3d(rows, V, K, W, H, torch.zeros(3), radius_clip=2.0, activated=True, band=band)
    torch.autograd.backward([rgb, alpha], [vr, va])
    return rgb.detach(), alpha.detach(), [t.grad for t in lv]


@pytest.mark.gpu
def test_render_image_shape_1152x1024(cuda):
    """scripts/visualization/render_image.py:158-168: one 1152x1024 view of a model-sized scene
    (16k Gaussians) through model.splat's call (radius_clip 2.0, packed False, absgrad).  The
    oracle is restricted to three central tile rows; the cotangent is supported on them."""
    from gsr.gsplat_compat import rasterization
    from gsr.scenes import ring_cameras
    W, H = 1152, 1024
    leaves = _model_splat_inputs(16000, 21)
    V, K = ring_cameras(1, W, H)
    row = (H // 16) // 2 - 1
    y0, y1 = 16 * row, 16 * row + 48
    g = torch.Generator().manual_seed(22)
    vr, va = torch.randn(1, H, W, 3, generator=g), torch.randn(1, H, W, generator=g)
    vr[:, :y0] = 0
    vr[:, y1:] = 0
    va[:, :y0] = 0
    va[:, y1:] = 0
    lg = [t.to(cuda).requires_grad_(True) for t in leaves]
    rgb, alpha, _ = rasterization(*lg, V.to(cuda), K.to(cuda), W, H, near_plane=0.01, far_plane=1e10,
                                  packed=False, absgrad=True, sh_degree=None, radius_clip=2.0)
    torch.autograd.backward([rgb, alpha[..., 0]], [vr.to(cuda), va.to(cuda)])
    rgb_o, a_o, g_o = _oracle_f32(leaves, V, K, W, H, (row, row + 3), vr, va)
    assert float(a_o[:, y0:y1].max()) > 0.5
    assert_close(rgb.detach().cpu()[:, y0:y1], rgb_o[:, y0:y1], max_frac=2e-4, max_outlier=0.02, what="rgb band")
    assert_close(alpha.detach().cpu()[:, y0:y1, :, 0], a_o[:, y0:y1], max_frac=2e-4, max_outlier=0.02,
                 what="alpha band")
    for name, t, e in zip(("means", "quats", "scales", "opacities", "colors"), lg, g_o):
        grad_close(t.grad.cpu(), e, what=f"v_{name}", max_frac=2e-3, outlier_rel=2e-3)


@pytest.mark.gpu
def test_visual_features_shape_32x224(cuda):
    """scripts/preprocessing/calculate_visual_features.py:164-189,268-278: C = N_THETA * N_PHI = 32
    cameras at 224x224 (fov 7.5 deg) in ONE call.  Three of the 32 views (first, middle,
    last) are checked against the oracle, with the cotangent supported on those views, so the
    gradient also checks that the other 29 views contribute nothing they should not."""
    from gsr.gsplat_compat import rasterization
    W = H = 224
    V, K = _sphere_cameras(W, H)
    C = V.shape[0]
    assert C == 32
    leaves = _model_splat_inputs(8000, 23)
    sel = [0, 13, 31]
    g = torch.Generator().manual_seed(24)
    vr, va = torch.zeros(C, H, W, 3), torch.zeros(C, H, W)
    vr[sel] = torch.randn(len(sel), H, W, 3, generator=g)
    va[sel] = torch.randn(len(sel), H, W, generator=g)
    lg = [t.to(cuda).requires_grad_(True) for t in leaves]
    rgb, alpha, _ = rasterization(*lg, V.to(cuda), K.to(cuda), W, H, packed=False, absgrad=True,
                                  sh_degree=None, radius_clip=2.0)
    assert rgb.shape == (C, H, W, 3)
    torch.autograd.backward([rgb, alpha[..., 0]], [vr.to(cuda), va.to(cuda)])
    rgb_o, a_o, g_o = _oracle_f32(leaves, V[sel], K[sel], W, H, None, vr[sel], va[sel])
    assert float(a_o.max()) > 0.5
    assert_close(rgb.detach().cpu()[sel], rgb_o, max_frac=2e-4, max_outlier=0.02, what="rgb 3 of 32 views")
    assert_close(alpha.detach().cpu()[sel][..., 0], a_o, max_frac=2e-4, max_outlier=0.02, what="alpha")
    for name, t, e in zip(("means", "quats", "scales", "opacities", "colors"), lg, g_o):
        grad_close(t.grad.cpu(), e, what=f"v_{name}", max_frac=2e-3, outlier_rel=2e-3)
