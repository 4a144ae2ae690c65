"""CPU restatement of the reference's SSIM loss term -- TEST INFRASTRUCTURE ONLY (the checker
for gsr.loss.ssim; never imported by the product path).

scripts/training/train_script.py:129 calls torchmetrics' StructuralSimilarityIndexMeasure
(data_range=1.0; train_script.py:270) as ssim(target_img[None], rgb[None]).  torchmetrics is not
installed here (no network), so this restates its published algorithm (torchmetrics
functional `_ssim_update` / `_ssim_compute`, gaussian kernel): taps from
int(3.5 sigma + 0.5) * 2 + 1 = 11, the normalised 1-D Gaussian (dist = -5..5, exp(-(d/s)^2/2))
and its outer product as an 11x11 depthwise conv2d kernel; reflection padding by 5; the
five maps x, y, x^2, y^2, xy convolved; S = (2 mx my + C1)(2 sxy + C2) / ((mx^2 + my^2 + C1)
(sx + sy + C2)) with C1 = (0.01 data_range)^2, C2 = (0.03 data_range)^2; the 5-pixel border
cropped; mean per image, then over the batch ('elementwise_mean').  Parity unpinned (no
torchmetrics fixtures in the reference).
"""
import torch
import torch.nn.functional as F


def gaussian_taps(sigma: float = 1.5, dtype=torch.float32) -> torch.Tensor:
    k = int(3.5 * sigma + 0.5) * 2 + 1
    dist = torch.arange((1 - k) / 2, (1 + k) / 2, 1, dtype=dtype)
    g = torch.exp(-torch.pow(dist / sigma, 2) / 2)
    return g / g.sum()


def ssim(preds: torch.Tensor, target: torch.Tensor, data_range: float = 1.0, sigma: float = 1.5,
         k1: float = 0.01, k2: float = 0.03) -> torch.Tensor:
    """[B,C,H,W] x2 -> scalar (batch mean), differentiable."""
    C = preds.shape[1]
    g = gaussian_taps(sigma, preds.dtype).to(preds.device)
    k = g.numel()
    pad = (k - 1) // 2
    kern = torch.matmul(g[:, None], g[None, :]).expand(C, 1, k, k)
    p = F.pad(preds, (pad, pad, pad, pad), mode="reflect")
    t = F.pad(target, (pad, pad, pad, pad), mode="reflect")
    out = F.conv2d(torch.cat((p, t, p * p, t * t, p * t)), kern, groups=C)
    mp, mt, pp, tt, pt = out.split(preds.shape[0])
    mp2, mt2, mpt = mp.pow(2), mt.pow(2), mp * mt
    sp, st, spt = pp - mp2, tt - mt2, pt - mpt
    c1, c2 = (k1 * data_range) ** 2, (k2 * data_range) ** 2
    full = ((2 * mpt + c1) * (2 * spt + c2)) / ((mp2 + mt2 + c1) * (sp + st + c2))
    crop = full[..., pad:-pad, pad:-pad]
    return crop.reshape(crop.shape[0], -1).mean(-1).mean()
