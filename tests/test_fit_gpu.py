"""BASELINE.json's third metric term, dPSNR vs the reference, as a TRAINING outcome (SURVEY.md
§8(d)): the same scene is fitted for 200 Adam steps once through the HIP path and once through
the oracle (the CPU restatement of the reference semantics), from the same start toward the
same target image, and the final PSNRs (get_psnr, scripts/utils/evaluate_model.py:240-243)
must agree within 0.03 dB (the north star's bar is 0.05 dB; VERDICT r5 asked for 0.03).

The oracle costs ~0.3 s per fwd+bwd even on a small image (it walks every tile list position
by position), so the fitted scene is a small one: 300 Gaussians of the config-1 distribution
seen from 0.3 away on a 48x40 view (the object fills the frame).  The loss is a squared error
on the image and on alpha; Adam with the learning rate decayed linearly to 0.  (Round 5 used the
reference's L1 image term, scripts/training/train_script.py:128-130.  Its gradient is sign(rgb -
target): at converged pixels roundoff decides the sign, Adam normalises that noise to full-size
steps, and two correct renderers' fits random-walk apart -- a third start showed 1.4 dB between
the HIP and oracle fits with nothing wrong in either, profiles/r06_fit_contract.txt.  A smooth
loss makes the test measure the renderer, not the chaos.)
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

STEPS = 200


def _psnr(pred, gt):
    mse = ((pred.double() - gt.double()) ** 2).mean()
    return float(10 * torch.log10(1.0 / mse))


def _fit(render, p0, target_rgb, target_a, lr, steps, record):
    p = p0.clone().requires_grad_(True)
    opt = torch.optim.Adam([p], lr=lr)
    # linear decay to 0: the last steps settle instead of oscillating, so the final PSNR is a
    # property of the converged fit rather than of the phase of an Adam oscillation
    sched = torch.optim.lr_scheduler.LambdaLR(opt, lambda s: 1.0 - s / steps)
    for s in range(steps + 1):
        rgb, alpha = render(p)
        if s in record:
            record[s] = _psnr(rgb.detach().cpu(), target_rgb)
        if s == steps:
            break
        loss = ((rgb - target_rgb.to(rgb.device)) ** 2).mean() + ((alpha - target_a.to(alpha.device)) ** 2).mean()
        opt.zero_grad()
        loss.backward()
        opt.step()
        sched.step()
    return p.detach().cpu()


SEEDS = (5, 6, 7)


@pytest.mark.timeout(1200)
def test_adam_fit_200_steps_dpsnr(cuda):
    """Three starts (perturbation seeds) of the same fit (one seed's dPSNR was decided
    by how the compiler fused one rounding): each final PSNR within 0.03 dB of the oracle's (the
    north-star bar is 0.05), the largest printed -- 0.022 dB on the round-6 tree, 0.029 dB with the
    projection backward built without fp contraction (GSR_PBWD_CONTRACT=0), so contraction is not
    what decides it (profiles/r06_fit_contract.txt)."""
    from gsr import render as R
    from gsr.scenes import gaussians3d, ring_cameras
    from oracle.oracle3d import render3d as oracle3d
    N, W, H = 300, 48, 40
    V, K = ring_cameras(1, W, H, radius=0.3)
    truth = gaussians3d(N, 1001)
    bg = torch.ones(3)
    with torch.no_grad():
        t_rgb, t_a = oracle3d(truth, V, K, W, H, bg)
    Vd, Kd, bgd = V.to(cuda), K.to(cuda), bg.to(cuda)
    worst = 0.0
    for seed in SEEDS:
        g = torch.Generator().manual_seed(seed)
        start = truth.clone()
        start[:, 0:3] += 0.004 * torch.randn(N, 3, generator=g)
        start[:, 10:13] = (start[:, 10:13] + 0.15 * torch.randn(N, 3, generator=g)).clamp(0, 1)
        start[:, 13] += 0.5 * torch.randn(N, generator=g)
        rec_g = {0: None, 50: None, 100: None, 150: None, STEPS: None}
        rec_o = dict(rec_g)
        p_g = _fit(lambda p: R.render3d(p, Vd, Kd, W, H, bgd), start.to(cuda), t_rgb, t_a, 2e-3, STEPS, rec_g)
        p_o = _fit(lambda p: oracle3d(p, V, K, W, H, bg), start, t_rgb, t_a, 2e-3, STEPS, rec_o)
        d = abs(rec_g[STEPS] - rec_o[STEPS])
        worst = max(worst, d)
        print(f"[fit] seed {seed}: PSNR (dB) by step, HIP {rec_g}, oracle {rec_o}; dPSNR {d:.4f} dB; "
              f"max |param difference| {float((p_g - p_o).abs().max()):.3e}", flush=True)
        assert rec_g[0] == pytest.approx(rec_o[0], abs=1e-3)
        assert rec_g[STEPS] > rec_g[0] + 3.0, "the fit did not converge"   # a real optimisation, not a no-op
        assert d <= 0.03, (seed, rec_g, rec_o)
    print(f"[fit] max dPSNR over seeds {SEEDS}: {worst:.4f} dB (bar 0.03)")
