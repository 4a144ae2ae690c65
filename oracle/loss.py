"""CPU/torch restatement of the reference training losses — TEST INFRASTRUCTURE ONLY (the
checker for gsr.loss; never imported by the product path).

* get_iou_loss — scripts/training/train_script.py:30-36 (per-view IoU over the last two dims,
  1 - mean over the leading dims, eps 1e-6).
* img_loss — scripts/training/train_script.py:128-130: img_lambda * sum|target - rgb| / sum mask,
  with rgb permuted to [3,H,W] as at :121-122 (stacked: [C,3,H,W]).

Works on any device: the tests apply it to the GPU render (unfused autograd) and to the
oracle render on the CPU.
"""
import torch


def get_iou_loss(predicted_mask: torch.Tensor, target_mask: torch.Tensor, eps: float = 1e-6) -> torch.Tensor:
    if predicted_mask.shape != target_mask.shape:
        raise ValueError("Predicted and target masks must have the same shape.")
    inter = (predicted_mask * target_mask).sum(dim=(-2, -1))
    union = (predicted_mask + target_mask - predicted_mask * target_mask).sum(dim=(-2, -1))
    return 1 - ((inter + eps) / (union + eps)).mean()


def img_loss(rgb_hwc: torch.Tensor, target_img: torch.Tensor, target_mask: torch.Tensor,
             img_lambda: float) -> torch.Tensor:
    """rgb_hwc [C,H,W,3] (renderer layout), target_img [C,3,H,W], target_mask [C,H,W]."""
    rgb = rgb_hwc.permute(0, 3, 1, 2)
    return img_lambda * torch.abs(target_img - rgb).sum() / target_mask.sum()
