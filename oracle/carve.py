"""CPU/torch restatement of the reference shape carver — TEST INFRASTRUCTURE ONLY (the
checker for gsr.carve; never imported by the product path).

Restates src/shape_carver.py (not importable here: torch_scatter is absent, SURVEY.md §8(c);
parity pinned by source reading):
* get_volume_torch :16-54, project_points_torch :57-103, sample_nearest_pixels_torch :106-129
* ray_cast_visibility_torch :132-204 — torch_scatter.scatter_min restated with scatter_reduce
  ('amin'), argmin ties to the lowest source index (torch_scatter's CPU order)
* project_points_torch_single_cam :207-235, compute_voxel_colors_torch :238-301 (including
  its `_, H, W, _ = images.shape` read of a [C,3,H,W] tensor)
* ShapeCarver.forward :322-366 (both branches), get_grid_points :369-374
* adjust_principal_points_to_seed (src/shape_carving.py:173-245), restated below in numpy
"""
import numpy as np
import torch


def project_points_torch(points, K, E):
    N = points.shape[0]
    ph = torch.cat([points, torch.ones(N, 1, dtype=points.dtype)], -1).unsqueeze(0).transpose(1, 2)
    cam = (E @ ph).transpose(1, 2)[..., :3].transpose(1, 2)
    pix = (K @ cam).transpose(1, 2)
    return pix[..., :2] / (pix[..., 2:3] + 1e-8)


def sample_nearest_pixels_torch(images, coords):
    n_cameras, c, h, w = images.shape
    x = coords[..., 0].round().long().clamp(min=0, max=w - 1)
    y = coords[..., 1].round().long().clamp(min=0, max=h - 1)
    cam = torch.arange(n_cameras)[:, None]
    return images[cam, :, y, x].permute(0, 2, 1)      # [C, c, N] (advanced indexing puts [C,N] first)


def get_volume_torch(images, K, E, grid_points):
    n1, n2, n3 = grid_points.shape[:3]
    coords = project_points_torch(grid_points.reshape(-1, 3), K, E)
    sampled = sample_nearest_pixels_torch(images, coords)
    return sampled.mean(dim=0).permute(1, 0).reshape(-1, n1, n2, n3)


def project_points_torch_single_cam(points, K, E):
    N = points.shape[0]
    ph = torch.cat([points, torch.ones(N, 1, dtype=points.dtype)], -1)
    cam = (E @ ph.T).T[:, :3]
    pix = (K @ cam.transpose(0, 1)).transpose(0, 1)
    return pix[:, :2] / pix[:, 2:3].clamp(min=1e-8)


def scatter_min(src, index, out):
    """torch_scatter.scatter_min(src, index, out=out) on 1-D tensors -> (out, argmin)."""
    N = src.shape[0]
    out = out.clone().scatter_reduce_(0, index, src, "amin", include_self=True)
    cand = torch.where(src == out[index], torch.arange(N), torch.full_like(index, N))
    arg = torch.full(out.shape, N, dtype=torch.long).scatter_reduce_(0, index, cand, "amin", include_self=True)
    return out, arg


def ray_cast_visibility_torch(grid_points, K, E, image_height, image_width):
    C = K.shape[0]
    N = grid_points.shape[0]
    vis = torch.zeros(C, N, dtype=torch.bool)
    R = E[:, :3, :3]
    t = E[:, :3, 3]
    cam_pos = -torch.einsum("cij,cj->ci", R.permute(0, 2, 1), t)
    for c in range(C):
        dist = (grid_points - cam_pos[c]).norm(dim=-1)
        pc = project_points_torch_single_cam(grid_points, K[c], E[c])
        px = pc[:, 0].round().long().clamp(0, image_width - 1)
        py = pc[:, 1].round().long().clamp(0, image_height - 1)
        pidx = py * image_width + px
        init = dist.new_full((image_height * image_width,), float("inf"))
        out, arg = scatter_min(dist, pidx, init)
        vis[c, (torch.arange(N) == arg[pidx]) & (out[pidx] < float("inf"))] = True
    return vis


def compute_voxel_colors_torch(grid_points, images, K, E, nonvisible_weight=0.25):
    C = images.shape[0]
    _, H, W, _ = images.shape                  # as in the reference: H <- 3, W <- image height
    vis = ray_cast_visibility_torch(grid_points, K, E, H, W)
    coords = torch.stack([project_points_torch_single_cam(grid_points, K[c], E[c]) for c in range(C)], 0)
    sampled = sample_nearest_pixels_torch(images, coords)           # [C, 3, n]
    w = torch.where(vis, torch.tensor(1.0), torch.tensor(nonvisible_weight))
    wn = w / w.sum(dim=0, keepdim=True).clamp(min=1e-8)
    return (wn[:, None] * sampled).sum(dim=0)                      # [3, n]


def get_grid_points(grid, center, angle):
    c, s = np.cos(angle), np.sin(angle)
    rot = torch.tensor([[c, -s, 0], [s, c, 0], [0, 0, 1]]).to(torch.float32)
    return torch.einsum("abci,ji->abcj", grid, rot) + center.view(1, 1, 1, 3)


def adjust_principal_points_to_seed(masks, Ks, extrinsics):
    """src/shape_carving.py:173-245: medoid per view (np.nonzero, float64 means, argmin of the
    squared distance), DLT triangulation of the seed, principal points moved so that the seed
    projects through each medoid.  masks [V,H,W] numpy; Ks [V,3,3], extrinsics [V,4,4] numpy."""
    V = masks.shape[0]
    med = []
    for i in range(V):
        ys, xs = np.nonzero(masks[i])
        if xs.size == 0:
            raise ValueError(f"Mask {i} is empty")
        cy, cx = ys.mean(), xs.mean()
        j = np.argmin((ys - cy) ** 2 + (xs - cx) ** 2)
        med.append((xs[j], ys[j]))
    med = np.array(med, dtype=np.float64)
    Ps = np.stack([Ks[i] @ np.concatenate([extrinsics[i][:3, :3], extrinsics[i][:3, 3:]], axis=1)
                   for i in range(V)], axis=0)
    A = np.vstack([r for i in range(V) for r in (med[i, 0] * Ps[i][2] - Ps[i][0], med[i, 1] * Ps[i][2] - Ps[i][1])])
    _, _, Vt = np.linalg.svd(A)
    Xh = Vt[-1]
    Xh /= Xh[3]
    X = Xh[:3]
    new = Ks.copy()
    for i in range(V):
        Xc = extrinsics[i][:3, :3] @ X + extrinsics[i][:3, 3]
        new[i, 0, 2] = med[i, 0] - Ks[i, 0, 0] * (Xc[0] / Xc[2])
        new[i, 1, 2] = med[i, 1] - Ks[i, 1, 1] * (Xc[1] / Xc[2])
    return new, X, med


def shape_carver_forward(grid, K, E, mask, rgb, center, angle, fill=0.45, K_mask=None):
    """ShapeCarver.forward; K_mask = the adapted intrinsics of the adaptive branch (the mask
    volume uses them, the colours keep K), with center = the triangulated seed."""
    C = K.shape[0]
    g = get_grid_points(grid, center, angle)
    n1, n2, n3 = g.shape[:3]
    mv = get_volume_torch(mask, K if K_mask is None else K_mask, E, g)
    out = 0.0
    for thresh in [1, (C - 1) / C]:
        b = (mv >= thresh).flatten()
        means = g.reshape(-1, 3)[b]
        colors = compute_voxel_colors_torch(means, rgb, K, E)
        vol = fill * torch.ones((4, n1 * n2 * n3), dtype=torch.float32)
        vol[0] = b.to(torch.float32)
        vol[1:, b] = colors
        out = out + vol.view(4, n1, n2, n3) / 2
    return out
