"""CPU/torch restatement of the reference parameter head and pose transform — TEST
INFRASTRUCTURE ONLY (the checker for gsr.head; never imported by the product path).

Restates, operation by operation and dtype by dtype (parity pinned by source reading: the
reference's src/model.py is not importable here because gsplat and torch_scatter are absent,
SURVEY.md §8(c)):

* select_mask             — src/model.py:185-205 (threshold loops + random subsample)
* head3d                  — src/model.py:207-234 (post-MLP activations, 3D mode)
* quaternion_matrix_ref   — src/model.py:378-403 (as written: [1][1] = 1 + q00 - q00 and
                            [1][0] = q12 - q30, i.e. not a rotation matrix)
* quaternion_from_matrix  — src/model.py:406-421 (float64 eigh of the 4x4 K / 3)
* pose_transform_3d       — src/model.py:258-298
"""
import numpy as np
import torch


def select_mask(v0: torch.Tensor, mask_threshold: float, prob_threshold: float, delta: float,
                min_n: int, max_n: int):
    """Returns (mask [M] bool, mt: float, probs [M]) exactly as the reference loops do."""
    mt = mask_threshold
    probs = torch.sigmoid(v0 - mt)
    pt = prob_threshold
    mask = probs > pt
    while mask.sum() > max_n:
        mt += delta
        probs = torch.sigmoid(v0 - mt)
        mask = probs > pt
    while mask.sum() < min_n:
        mt -= delta
        probs = torch.sigmoid(v0 - mt)
        mask = probs > pt
    if mask.sum() > max_n:
        indices = torch.nonzero(mask, as_tuple=True)[0]
        rand_idx = torch.randperm(len(indices))[:max_n].to(mask.device)
        keep = indices[rand_idx]
        mask[:] = False
        mask[keep] = True
    return mask, mt, probs


def head3d(net_out, probs_sel, scale, grid_sel, prob_threshold, color_clip, voxel_size):
    """src/model.py:213-234 after the MLP; probs_sel = probs[mask]."""
    pt = prob_threshold
    quats, scales, opacities, colors, delta_means = torch.split(net_out, (4, 3, 1, 3, 3), dim=1)
    colors = torch.sigmoid(colors).clamp(color_clip[0], color_clip[1])
    log_scales = scales + scale[0]
    logit_opacities = torch.logit(((1 / (1 - pt)) * (probs_sel - pt)).clamp(1e-6, 1.0 - 1e-6)).unsqueeze(-1)
    means = grid_sel + 2 * voxel_size * torch.tanh(delta_means)
    return torch.cat([means, log_scales, quats, colors, logit_opacities], dim=1)


def quaternion_matrix_ref(quats):
    b = quats.shape[0]
    eps = 4 * np.finfo(float).eps
    quats = quats.clone().double()
    n = torch.sum(quats ** 2, dim=1)
    mask = n < eps
    n[mask] = 1.0
    quats = quats * torch.sqrt(2.0 / n).unsqueeze(1)
    outer = torch.einsum("bi,bj->bij", quats, quats)
    eye = torch.eye(4, dtype=torch.float64, device=quats.device)
    res = eye.unsqueeze(0).repeat(b, 1, 1)
    res[:, 0, 0] = res[:, 0, 0] - outer[:, 2, 2] - outer[:, 3, 3]
    res[:, 0, 1] = outer[:, 1, 2] - outer[:, 3, 0]
    res[:, 0, 2] = outer[:, 1, 3] + outer[:, 2, 0]
    res[:, 1, 0] = outer[:, 1, 2] - outer[:, 3, 0]
    res[:, 1, 1] = res[:, 1, 1] + outer[:, 0, 0] - outer[:, 0, 0]
    res[:, 1, 2] = outer[:, 2, 3] - outer[:, 1, 0]
    res[:, 2, 0] = outer[:, 1, 3] - outer[:, 2, 0]
    res[:, 2, 1] = outer[:, 2, 3] + outer[:, 1, 0]
    res[:, 2, 2] = res[:, 2, 2] - outer[:, 1, 1] - outer[:, 2, 2]
    res[mask] = eye
    return res.to(torch.float32)


def quaternion_from_matrix(mats):
    mats = mats.double()
    m00, m01, m02 = mats[:, 0, 0], mats[:, 0, 1], mats[:, 0, 2]
    m10, m11, m12 = mats[:, 1, 0], mats[:, 1, 1], mats[:, 1, 2]
    m20, m21, m22 = mats[:, 2, 0], mats[:, 2, 1], mats[:, 2, 2]
    K = torch.stack([
        torch.stack([m00 - m11 - m22, m01 + m10, m02 + m20, m21 - m12], 1),
        torch.stack([m01 + m10, m11 - m00 - m22, m12 + m21, m02 - m20], 1),
        torch.stack([m02 + m20, m12 + m21, m22 - m00 - m11, m10 - m01], 1),
        torch.stack([m21 - m12, m02 - m20, m10 - m01, m00 + m11 + m22], 1),
    ], 1)
    K = K / 3.0
    _, V = torch.linalg.eigh(K)
    quats = V[:, :, -1]
    quats = quats[:, [3, 0, 1, 2]]
    mask = quats[:, 0] < 0
    quats = torch.where(mask[:, None], -quats, quats)
    return quats.to(torch.float32)


def pose_transform_3d(params, angle, p_3d):
    means = params[:, 0:3]
    log_scales = params[:, 3:6]
    quats = params[:, 6:10]
    colors = params[:, 10:13]
    logit_op = params[:, 13:14]
    c, s = np.cos(angle), np.sin(angle)
    rot_mat = torch.tensor([[c, -s, 0], [s, c, 0], [0, 0, 1]]).to(means.device, torch.float32)
    p3 = p_3d.to(means.device) if isinstance(p_3d, torch.Tensor) else torch.tensor(p_3d).to(means.device, torch.float32)
    means = means @ rot_mat.T + p3
    rot_mat_2 = torch.tensor([[c, -s, 0, 0], [s, c, 0, 0], [0, 0, 1, 0], [0, 0, 0, 1]]).to(quats.device)
    r = quaternion_matrix_ref(quats)
    r = torch.einsum("ij,bjk->bik", rot_mat_2.to(torch.float32), r)
    quats = quaternion_from_matrix(r)
    return torch.cat([means, log_scales, quats, colors, logit_op], dim=1)
