"""ORACLE (test infrastructure only) — CPU restatement of the reference 3D render path.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module, and only as the checker.  The product path never imports it.

Reference call site being restated: ``GaussianRenderer3D.render``
(src/gaussian_renderer.py:157-211) → ``gsplat.rendering.rasterization`` with
``packed=False``, ``backgrounds=bg[None]`` and gsplat defaults (near 0.01, far 1e10,
radius_clip 0, eps2d 0.3, tile 16, "classic", absgrad False).

gsplat is a third-party dependency ABSENT from /root/reference and from this container;
its version is unpinned (``gsplat>=0.1.0``, requirements.txt:10; environment.yml:26).  The
arithmetic below restates gsplat's published "classic" algorithm —
the 1.5.x line by default (torch 2.9 env, environment.yml:12), with the ≤1.4 isotropic
radius rule selectable:

* activations (adapter, restated exactly)     src/gaussian_renderer.py:183-193
* projection (A.1): R(q) from the re-normalised (w,x,y,z) quaternion, Σ = R S Sᵀ Rᵀ,
  world→camera, perspective Jacobian with FOV-clamped tx/ty, eps2d blur, conic = inv(cov2d),
  near/far cull, det ≤ 0 cull, radius rule, radius_clip cull, off-screen cull.
* binning (A.2): tile rect [floor((x−r)/16), ceil((x+r)/16)) clamped to the grid per axis,
  list order (camera, tile, depth float bits, flatten id c·N+n) — what a stable radix sort
  of gsplat's 64-bit keys over emission order yields.
* raster fwd (A.3), strictly sequential in fp32 per pixel (centre +0.5):
  σ = ½(A dx² + C dy²) + B dx dy; α = min(0.999, o e^{−σ}); skip σ<0 or α<1/255;
  stop before a Gaussian when T(1−α) ≤ 1e-4; rgb = Σ c α T + T bg; alpha = 1 − T.
* raster bwd (A.4): analytic derivative of the above with the same discrete decisions,
  derived independently here and checked in float64 against autograd of a per-pixel
  restatement (tests/test_oracle3d.py).  Projection and activation derivatives come from
  torch autograd through the restated formulas.

Parity status: the 2D path is pinned by reference fixtures; this 3D path has NO fixture
from gsplat itself (unavailable offline) — "parity unpinned" against gsplat; only the
adapter (tests/golden/ref3d_adapter.npz) and internal known-answer tests pin it.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch

__all__ = [
    "Ref3D", "activations3d", "quat_to_rotmat", "project3d", "isect_tiles",
    "raster3d_fwd", "raster3d_bwd", "render3d", "render3d_pixelloop", "tie_flags",
]


class Ref3D:
    TILE = 16
    ALPHA_THRESHOLD = 1.0 / 255.0
    ALPHA_MAX = 0.999
    T_MIN = 1e-4
    NEAR = 0.01
    FAR = 1e10
    EPS2D = 0.3
    RADIUS_CLIP = 0.0
    EXTEND_MAX = 3.33
    RADIUS_OPACITY_AABB = 0     # gsplat >= 1.5: per-axis, opacity-aware bounding box
    RADIUS_ISOTROPIC_3SIGMA = 1  # gsplat <= 1.4: ceil(3 sqrt(lambda_max))


def activations3d(params: torch.Tensor):
    """src/gaussian_renderer.py:183-193."""
    means = params[:, 0:3]
    scales = torch.exp(params[:, 3:6])
    q = params[:, 6:10]
    quats = q / (q.norm(dim=-1, keepdim=True) + 1e-8)
    colors = torch.clamp(params[:, 10:13], 0.0, 1.0)
    opac = torch.sigmoid(params[:, 13:14]).squeeze(-1)
    return means, quats, scales, colors, opac


def quat_to_rotmat(q: torch.Tensor) -> torch.Tensor:
    """(w,x,y,z) → R, re-normalised (gsplat normalises its quaternion input again)."""
    q = q * torch.rsqrt((q * q).sum(-1, keepdim=True))
    w, x, y, z = q.unbind(-1)
    r00 = 1 - 2 * (y * y + z * z)
    r01 = 2 * (x * y - w * z)
    r02 = 2 * (x * z + w * y)
    r10 = 2 * (x * y + w * z)
    r11 = 1 - 2 * (x * x + z * z)
    r12 = 2 * (y * z - w * x)
    r20 = 2 * (x * z - w * y)
    r21 = 2 * (y * z + w * x)
    r22 = 1 - 2 * (x * x + y * y)
    return torch.stack([torch.stack([r00, r01, r02], -1),
                        torch.stack([r10, r11, r12], -1),
                        torch.stack([r20, r21, r22], -1)], -2)


@dataclass
class Projection:
    means2d: torch.Tensor   # [C,N,2]  (differentiable)
    conics: torch.Tensor    # [C,N,3]  (A,B,C) of inv(cov2d) (differentiable)
    depths: torch.Tensor    # [C,N]    (no grad)
    radii: torch.Tensor     # [C,N,2]  int32, 0 = culled
    valid: torch.Tensor     # [C,N]    bool


def project3d(means, quats, scales, opac, viewmats, Ks, width, height,
              near=Ref3D.NEAR, far=Ref3D.FAR, radius_clip=Ref3D.RADIUS_CLIP,
              eps2d=Ref3D.EPS2D, radius_mode=Ref3D.RADIUS_OPACITY_AABB) -> Projection:
    """SURVEY.md Appendix A.1, batched over C cameras."""
    dt = means.dtype
    R = quat_to_rotmat(quats)                              # [N,3,3]
    M = R * scales[:, None, :]                             # R diag(s)
    cov = M @ M.transpose(-1, -2)                          # [N,3,3]
    Rv = viewmats[:, :3, :3].to(dt)                        # [C,3,3]
    tv = viewmats[:, :3, 3].to(dt)                         # [C,3]
    mc = torch.einsum("cij,nj->cni", Rv, means) + tv[:, None, :]     # [C,N,3]
    covc = torch.einsum("cij,njk,clk->cnil", Rv, cov, Rv)            # Rv Σ Rvᵀ
    x, y, z = mc.unbind(-1)
    fx = Ks[:, 0, 0].to(dt)[:, None]
    fy = Ks[:, 1, 1].to(dt)[:, None]
    cx = Ks[:, 0, 2].to(dt)[:, None]
    cy = Ks[:, 1, 2].to(dt)[:, None]
    tan_fovx = 0.5 * width / fx
    tan_fovy = 0.5 * height / fy
    lim_x_pos = (width - cx) / fx + 0.3 * tan_fovx
    lim_x_neg = cx / fx + 0.3 * tan_fovx
    lim_y_pos = (height - cy) / fy + 0.3 * tan_fovy
    lim_y_neg = cy / fy + 0.3 * tan_fovy
    rz = 1.0 / z
    rz2 = rz * rz
    tx = z * torch.minimum(lim_x_pos, torch.maximum(-lim_x_neg, x * rz))
    ty = z * torch.minimum(lim_y_pos, torch.maximum(-lim_y_neg, y * rz))
    zero = torch.zeros_like(z)
    J = torch.stack([torch.stack([fx * rz, zero, -fx * tx * rz2], -1),
                     torch.stack([zero, fy * rz, -fy * ty * rz2], -1)], -2)  # [C,N,2,3]
    cov2d = J @ covc @ J.transpose(-1, -2)                               # [C,N,2,2]
    mean2d = torch.stack([fx * x * rz + cx, fy * y * rz + cy], -1)
    c00 = cov2d[..., 0, 0] + eps2d
    c01 = cov2d[..., 0, 1]
    c10 = cov2d[..., 1, 0]
    c11 = cov2d[..., 1, 1] + eps2d
    det = c00 * c11 - c01 * c10
    with torch.no_grad():
        valid = (z >= near) & (z <= far) & (det > 0)
    safe_det = torch.where(valid, det, torch.ones_like(det))
    inv_det = 1.0 / safe_det
    conics = torch.stack([c11 * inv_det, -c01 * inv_det, c00 * inv_det], -1)
    with torch.no_grad():
        c00d, c11d, detd = c00.detach(), c11.detach(), det.detach()
        if radius_mode == Ref3D.RADIUS_OPACITY_AABB:
            op = opac.detach().to(torch.float32)[None, :].expand_as(c00d)
            thr = torch.tensor(Ref3D.ALPHA_THRESHOLD, dtype=torch.float32)
            valid = valid & (op >= thr)
            ratio = torch.clamp(op / thr, min=1.0)
            extend = torch.clamp(torch.sqrt(2.0 * torch.log(ratio)), max=Ref3D.EXTEND_MAX).to(dt)
            rx = torch.ceil(extend * torch.sqrt(torch.clamp(c00d, min=0)))
            ry = torch.ceil(extend * torch.sqrt(torch.clamp(c11d, min=0)))
            valid = valid & ~((rx <= radius_clip) & (ry <= radius_clip))
        else:
            b = 0.5 * (c00d + c11d)
            v1 = b + torch.sqrt(torch.clamp(b * b - detd, min=0.01))
            r = torch.ceil(3.0 * torch.sqrt(v1))
            rx, ry = r, r
            valid = valid & ~(r <= radius_clip)
        mx, my = mean2d.detach().unbind(-1)
        offscreen = (mx + rx <= 0) | (mx - rx >= width) | (my + ry <= 0) | (my - ry >= height)
        valid = valid & ~offscreen
        valid = valid & torch.isfinite(mx) & torch.isfinite(my)
        radii = torch.stack([rx, ry], -1)
        radii = torch.where(valid[..., None], radii, torch.zeros_like(radii)).to(torch.int32)
    return Projection(mean2d, conics, z.detach(), radii, valid)


def isect_tiles(means2d, radii, depths, width, height, tile=Ref3D.TILE, depth_order=True, band=None):
    """SURVEY.md Appendix A.2.  Returns (tile_offsets [C*T+1] int64, ids [I] int64).

    ids are flatten ids c*N+n; list order within a tile is (depth float bits, c*N+n) when
    ``depth_order`` (3D), else parameter index order (2D).  ``band`` = (y0, y1) restricts
    binning to those tile rows, counted over the C cameras' rows laid end to end (row r of
    camera c is global row c*th + r) -- the build's multi-GPU (view, band) sharding, not a
    reference feature; the full-image result restricted to the band is unchanged.
    """
    C, N = depths.shape
    tw = (width + tile - 1) // tile
    th = (height + tile - 1) // tile
    T = tw * th
    with torch.no_grad():
        m = means2d.detach().to(torch.float32)
        r = radii.to(torch.float32)
        t16 = torch.tensor(float(tile))
        tile_x = m[..., 0] / t16
        tile_y = m[..., 1] / t16
        trx = r[..., 0] / t16
        try_ = r[..., 1] / t16
        x0 = torch.clamp(torch.floor(tile_x - trx), min=0, max=tw).to(torch.int64)
        x1 = torch.clamp(torch.ceil(tile_x + trx), min=0, max=tw).to(torch.int64)
        y0 = torch.clamp(torch.floor(tile_y - try_), min=0, max=th).to(torch.int64)
        y1 = torch.clamp(torch.ceil(tile_y + try_), min=0, max=th).to(torch.int64)
        if band is not None:
            cam_row = torch.arange(C, dtype=torch.int64)[:, None] * th
            y0 = torch.maximum(y0, (band[0] - cam_row).clamp(0, th))
            y1 = torch.minimum(y1, (band[1] - cam_row).clamp(0, th))
        live = (radii[..., 0] > 0) | (radii[..., 1] > 0)
        wcnt = torch.where(live, (x1 - x0).clamp(min=0), torch.zeros_like(x0))
        hcnt = torch.where(live, (y1 - y0).clamp(min=0), torch.zeros_like(y0))
        cnt = (wcnt * hcnt).reshape(-1)
        total = int(cnt.sum())
        flat = torch.arange(C * N, dtype=torch.int64)
        owner = torch.repeat_interleave(flat, cnt)
        start = torch.cumsum(cnt, 0) - cnt
        local = torch.arange(total, dtype=torch.int64) - start[owner]
        wv = wcnt.reshape(-1)[owner]
        ty = y0.reshape(-1)[owner] + torch.div(local, wv.clamp(min=1), rounding_mode="floor")
        tx = x0.reshape(-1)[owner] + local % wv.clamp(min=1)
        cam = owner // N
        tile_id = cam * T + ty * tw + tx
        if depth_order:
            dbits = depths.detach().to(torch.float32).contiguous().view(torch.int32).reshape(-1)
            dbits = dbits[owner].to(torch.int64) & 0xFFFFFFFF
            key = (tile_id << 32) | dbits
        else:
            key = tile_id
        order = torch.sort(key, stable=True).indices   # emission order is by flatten id
        ids = owner[order]
        counts = torch.bincount(tile_id, minlength=C * T)
        offsets = torch.zeros(C * T + 1, dtype=torch.int64)
        offsets[1:] = torch.cumsum(counts, 0)
    return offsets, ids


def _tile_pixels(width, height, tile, tiles_idx, tw, offset):
    """Pixel coordinates for the listed tiles: (px, py, inside) each [Tn, tile*tile]."""
    t = tiles_idx
    txy = torch.stack([t % tw, t // tw], -1)
    lr = torch.arange(tile * tile)
    lx = lr % tile
    ly = lr // tile
    j = txy[:, 0:1] * tile + lx[None, :]
    i = txy[:, 1:2] * tile + ly[None, :]
    inside = (i < height) & (j < width)
    return j, i, inside


def raster3d_fwd(means2d, conics, colors, opac, bg, offsets, ids, width, height,
                 tile=Ref3D.TILE, keep_T=False):
    """Sequential fp32 front-to-back compositing.

    means2d [C,N,2], conics [C,N,3], colors [C,N,3], opac [C,N], bg [C,3].
    Returns rgb [C,H,W,3], alpha [C,H,W], last [C,H,W] (index into ``ids``, -1 if none)
    and (if keep_T) the per-step state needed by ``raster3d_bwd``.
    """
    dt = means2d.dtype
    C, N = opac.shape
    tw = (width + tile - 1) // tile
    th = (height + tile - 1) // tile
    T_ = tw * th
    P = tile * tile
    xy = means2d.detach().reshape(C * N, 2)
    con = conics.detach().reshape(C * N, 3)
    col = colors.detach().reshape(C * N, 3)
    op = opac.detach().reshape(C * N)
    counts = offsets[1:] - offsets[:-1]
    busy = torch.nonzero(counts > 0).flatten()
    rgb = torch.zeros(C, height, width, 3, dtype=dt)
    alpha = torch.zeros(C, height, width, dtype=dt)
    last = torch.full((C, height, width), -1, dtype=torch.int64)
    rgb[:] = bg.to(dt)[:, None, None, :]
    state = {"busy": busy, "steps": []}
    if busy.numel() == 0:
        return rgb, alpha, last, state
    cams = busy // T_
    tloc = busy % T_
    j, i, inside = _tile_pixels(width, height, tile, tloc, tw, 0.5)
    px = j.to(dt) + 0.5
    py = i.to(dt) + 0.5
    starts = offsets[busy]
    lens = counts[busy]
    Lmax = int(lens.max())
    Tn = busy.numel()
    Tcur = torch.ones(Tn, P, dtype=dt)
    Ccur = torch.zeros(Tn, P, 3, dtype=dt)
    done = ~inside
    lastv = torch.full((Tn, P), -1, dtype=torch.int64)
    thr = torch.tensor(Ref3D.ALPHA_THRESHOLD, dtype=dt)
    for k in range(Lmax):
        act = (k < lens)
        if not bool((act[:, None] & ~done).any()):
            break
        e = torch.where(act, starts + k, starts)          # list index
        g = ids[e]
        gx, gy = xy[g, 0][:, None], xy[g, 1][:, None]
        A, B, Cc = con[g, 0][:, None], con[g, 1][:, None], con[g, 2][:, None]
        o = op[g][:, None]
        dx = gx - px
        dy = gy - py
        sigma = 0.5 * (A * dx * dx + Cc * dy * dy) + B * dx * dy
        al = torch.clamp(o * torch.exp(-sigma), max=Ref3D.ALPHA_MAX)
        ok = act[:, None] & ~done & (sigma >= 0) & (al >= thr)
        nT = Tcur * (1.0 - al)
        stop = ok & (nT <= Ref3D.T_MIN)
        done = done | stop
        contrib = ok & ~stop
        if keep_T:
            state["steps"].append((Tcur.clone(), contrib))
        vis = torch.where(contrib, al * Tcur, torch.zeros_like(al))
        Ccur = Ccur + vis[..., None] * col[g][:, None, :]
        Tcur = torch.where(contrib, nT, Tcur)
        lastv = torch.where(contrib, e[:, None].expand_as(lastv), lastv)
    # scatter back
    for n_, (c, t) in enumerate(zip(cams.tolist(), tloc.tolist())):
        m = inside[n_]
        ii, jj = i[n_][m], j[n_][m]
        rgb[c, ii, jj] = Ccur[n_][m] + Tcur[n_][m][:, None] * bg[c].to(dt)[None, :]
        alpha[c, ii, jj] = 1.0 - Tcur[n_][m]
        last[c, ii, jj] = lastv[n_][m]
    state.update(dict(cams=cams, tloc=tloc, i=i, j=j, inside=inside, px=px, py=py,
                      starts=starts, lens=lens, Tfinal=Tcur, lastv=lastv))
    return rgb, alpha, last, state


def raster3d_bwd(means2d, conics, colors, opac, bg, offsets, ids, width, height,
                 state, v_rgb, v_alpha, tile=Ref3D.TILE):
    """Analytic backward of ``raster3d_fwd`` (derived here).

    rgb = Σ_i c_i α_i T_i + T_f bg,  alpha = 1 − T_f,  T_{i+1} = T_i (1 − α_i) over the
    contributing entries i.  With S_i = Σ_{j>i} c_j α_j T_j (suffix):
        ∂rgb/∂c_i   = α_i T_i
        ∂rgb/∂α_i   = c_i T_i − (S_i + T_f bg) / (1 − α_i)
        ∂alpha/∂α_i = T_f / (1 − α_i)
    and α = o e^{−σ} (where unclamped): ∂α/∂o = e^{−σ}, ∂α/∂σ = −α.
    Returns v_means2d [C,N,2], v_conics [C,N,3], v_colors [C,N,3], v_opac [C,N].
    """
    dt = means2d.dtype
    C, N = opac.shape
    xy = means2d.detach().reshape(C * N, 2)
    con = conics.detach().reshape(C * N, 3)
    col = colors.detach().reshape(C * N, 3)
    op = opac.detach().reshape(C * N)
    g_xy = torch.zeros(C * N, 2, dtype=dt)
    g_con = torch.zeros(C * N, 3, dtype=dt)
    g_col = torch.zeros(C * N, 3, dtype=dt)
    g_op = torch.zeros(C * N, dtype=dt)
    busy = state["busy"]
    if busy.numel() == 0:
        return (g_xy.view(C, N, 2), g_con.view(C, N, 3), g_col.view(C, N, 3), g_op.view(C, N))
    cams, i, j, inside = state["cams"], state["i"], state["j"], state["inside"]
    px, py, starts, lens = state["px"], state["py"], state["starts"], state["lens"]
    Tf = state["Tfinal"]
    Tn, P = Tf.shape
    # gather cotangents per tile pixel
    ic = i.clamp(max=height - 1)
    jc = j.clamp(max=width - 1)
    cc = cams[:, None].expand_as(ic)
    vr = v_rgb.to(dt)[cc, ic, jc] * inside[..., None]
    va = v_alpha.to(dt)[cc, ic, jc] * inside
    bgt = bg.to(dt)[cams][:, None, :]
    S = torch.zeros(Tn, P, 3, dtype=dt)
    steps = state["steps"]
    for k in range(len(steps) - 1, -1, -1):
        Tk, contrib = steps[k]
        act = (k < lens)
        e = torch.where(act, starts + k, starts)
        g = ids[e]
        gx, gy = xy[g, 0][:, None], xy[g, 1][:, None]
        A, B, Cc = con[g, 0][:, None], con[g, 1][:, None], con[g, 2][:, None]
        o = op[g][:, None]
        cg = col[g][:, None, :]
        dx = gx - px
        dy = gy - py
        sigma = 0.5 * (A * dx * dx + Cc * dy * dy) + B * dx * dy
        vis = torch.exp(-sigma)
        raw = o * vis
        al = torch.clamp(raw, max=Ref3D.ALPHA_MAX)
        m = contrib
        ra = 1.0 / (1.0 - al)
        fac = al * Tk
        v_c = torch.where(m[..., None], fac[..., None] * vr, torch.zeros_like(vr))
        v_al = (vr * (cg * Tk[..., None] - (S + Tf[..., None] * bgt) * ra[..., None])).sum(-1) \
            + va * Tf * ra
        v_al = torch.where(m, v_al, torch.zeros_like(v_al))
        unclamped = m & (raw <= Ref3D.ALPHA_MAX)
        v_sig = torch.where(unclamped, -raw * v_al, torch.zeros_like(v_al))
        v_o = torch.where(unclamped, vis * v_al, torch.zeros_like(v_al))
        v_A = 0.5 * v_sig * dx * dx
        v_B = v_sig * dx * dy
        v_C = 0.5 * v_sig * dy * dy
        v_x = v_sig * (A * dx + B * dy)
        v_y = v_sig * (B * dx + Cc * dy)
        S = S + torch.where(m[..., None], cg * fac[..., None], torch.zeros_like(S))
        gi = g.clone()
        sel = act
        g_xy.index_add_(0, gi[sel], torch.stack([v_x.sum(1), v_y.sum(1)], -1)[sel])
        g_con.index_add_(0, gi[sel], torch.stack([v_A.sum(1), v_B.sum(1), v_C.sum(1)], -1)[sel])
        g_col.index_add_(0, gi[sel], v_c.sum(1)[sel])
        g_op.index_add_(0, gi[sel], v_o.sum(1)[sel])
    return (g_xy.view(C, N, 2), g_con.view(C, N, 3), g_col.view(C, N, 3), g_op.view(C, N))


class _Raster3D(torch.autograd.Function):
    @staticmethod
    def forward(ctx, means2d, conics, colors, opac, bg, offsets, ids, width, height):
        rgb, alpha, last, state = raster3d_fwd(means2d, conics, colors, opac, bg, offsets, ids,
                                               width, height, keep_T=True)
        ctx.state = state
        ctx.meta = (offsets, ids, width, height)
        ctx.save_for_backward(means2d, conics, colors, opac, bg)
        ctx.mark_non_differentiable(last)
        return rgb, alpha, last

    @staticmethod
    def backward(ctx, v_rgb, v_alpha, _v_last):
        means2d, conics, colors, opac, bg = ctx.saved_tensors
        offsets, ids, width, height = ctx.meta
        C, H, W = v_alpha.shape if v_alpha is not None else (opac.shape[0], height, width)
        if v_rgb is None:
            v_rgb = torch.zeros(C, height, width, 3, dtype=means2d.dtype)
        if v_alpha is None:
            v_alpha = torch.zeros(C, height, width, dtype=means2d.dtype)
        g = raster3d_bwd(means2d, conics, colors, opac, bg, offsets, ids, width, height,
                         ctx.state, v_rgb, v_alpha)
        return g[0], g[1], g[2], g[3], None, None, None, None, None


def render3d(params, viewmats, Ks, width, height, background, *,
             radius_mode=Ref3D.RADIUS_OPACITY_AABB, near=Ref3D.NEAR, far=Ref3D.FAR,
             radius_clip=Ref3D.RADIUS_CLIP, eps2d=Ref3D.EPS2D, return_meta=False, activated=False, band=None):
    """Full oracle of GaussianRenderer3D.render for C cameras: rgb [C,H,W,3], alpha [C,H,W].

    Differentiable w.r.t. ``params`` ([N,14]); viewmats [C,4,4], Ks [C,3,3], background [3]
    or per-camera [C,3].  ``activated=True`` restates a direct gsplat ``rasterization`` call
    (src/model.py:339-365): the rows already hold scales, opacities and colours, and the
    quaternion is only renormalised inside the rotation (quat_to_rotmat).
    """
    if params.shape[1] != 14:
        raise ValueError(f"Expected 14 parameters per Gaussian, got {params.shape[1]}")
    dt = params.dtype
    C = viewmats.shape[0]
    if activated:
        means, scales, quats = params[:, 0:3], params[:, 3:6], params[:, 6:10]
        colors, opac = params[:, 10:13], params[:, 13]
    else:
        means, quats, scales, colors, opac = activations3d(params)
    proj = project3d(means, quats, scales, opac, viewmats, Ks, width, height, near=near, far=far,
                     radius_clip=radius_clip, eps2d=eps2d, radius_mode=radius_mode)
    offsets, ids = isect_tiles(proj.means2d, proj.radii, proj.depths, width, height, band=band)
    N = params.shape[0]
    colors_c = colors[None].expand(C, N, 3)
    opac_c = opac[None].expand(C, N)
    bg = background.to(dt).reshape(-1, 3).expand(C, 3).contiguous()
    rgb, alpha, last = _Raster3D.apply(proj.means2d, proj.conics, colors_c, opac_c, bg,
                                       offsets, ids, width, height)
    if return_meta:
        return rgb, alpha, dict(proj=proj, offsets=offsets, ids=ids, last=last)
    return rgb, alpha


def tie_flags(params, viewmats, Ks, width, height, *, margin=1e-4, radius_mode=Ref3D.RADIUS_OPACITY_AABB,
              activated=False, band=None, tile=Ref3D.TILE):
    """Where two correct fp32 implementations of A.3 may resolve a discrete decision differently.

    Walks the same lists as ``raster3d_fwd`` (same ``done`` state) and flags a pixel when any
    entry it evaluates sits within ``margin`` (relative) of a decision threshold:
      * the skip test α ≥ 1/255 (|α − 1/255| ≤ margin/255),
      * the stop test T(1 − α) ≤ 1e-4 for an entry that passes the skip (|nT − 1e-4| ≤ margin·1e-4),
      * the clamp α = min(0.999, o e^{−σ}) that switches the σ / opacity gradients off
        (|o e^{−σ} − 0.999| ≤ margin),
      * the test σ ≥ 0 (|σ| ≤ margin·(|A dx²| + |C dy²| + |2B dx dy|)/2: a pixel at the centre).
    The GPU evaluates the same formulas from its own projection (different fp32 roundings,
    exp2 with a log2(e)-scaled conic).  The fp32 oracle's own alpha near 1/255 is off its float64
    value by up to 2.9e-5 (relative) at config 1 (conic cancellation, sigma ~5.5 in the
    exponent); two fp32 implementations differ by up to twice that, hence 1e-4.

    Returns (pixels [C,H,W] bool, gaussians [N] bool, n_pixels): ``gaussians`` marks every
    Gaussian with α ≥ (1 − margin)/255 at a flagged pixel -- the entries whose gradient a flipped
    decision there can change (a skip flip moves that entry and, through T and the suffix
    colour, every other entry of the pixel; a stop flip adds or drops the entries after it).
    Tests allow an out-of-tolerance value ONLY at a flagged pixel / a marked Gaussian's row.
    """
    C, N = viewmats.shape[0], params.shape[0]
    with torch.no_grad():
        p = params.detach()
        if activated:
            means, scales, quats = p[:, 0:3], p[:, 3:6], p[:, 6:10]
            opac = p[:, 13]
        else:
            means, quats, scales, _, opac = activations3d(p)
        proj = project3d(means, quats, scales, opac, viewmats, Ks, width, height, radius_mode=radius_mode)
        offsets, ids = isect_tiles(proj.means2d, proj.radii, proj.depths, width, height, band=band)
        dt = proj.means2d.dtype
        xy = proj.means2d.reshape(C * N, 2)
        con = proj.conics.reshape(C * N, 3)
        op = opac[None].expand(C, N).reshape(C * N).to(dt)
        tw = (width + tile - 1) // tile
        th = (height + tile - 1) // tile
        T_ = tw * th
        pix = torch.zeros(C, height, width, dtype=torch.bool)
        gau = torch.zeros(N, dtype=torch.bool)
        counts = offsets[1:] - offsets[:-1]
        busy = torch.nonzero(counts > 0).flatten()
        if busy.numel() == 0:
            return pix, gau, 0
        cams, tloc = busy // T_, busy % T_
        j, i, inside = _tile_pixels(width, height, tile, tloc, tw, 0.5)
        px, py = j.to(dt) + 0.5, i.to(dt) + 0.5
        starts, lens = offsets[busy], counts[busy]
        Tn, P = busy.numel(), tile * tile
        thr = Ref3D.ALPHA_THRESHOLD

        def step(k):
            act = k < lens
            e = torch.where(act, starts + k, starts)
            g = ids[e]
            A, B, Cc = con[g, 0][:, None], con[g, 1][:, None], con[g, 2][:, None]
            dx, dy = xy[g, 0][:, None] - px, xy[g, 1][:, None] - py
            sigma = 0.5 * (A * dx * dx + Cc * dy * dy) + B * dx * dy
            mag = 0.5 * ((A * dx * dx).abs() + (Cc * dy * dy).abs()) + (B * dx * dy).abs()
            raw = op[g][:, None] * torch.exp(-sigma)
            return act, g, sigma, mag, raw, torch.clamp(raw, max=Ref3D.ALPHA_MAX)

        Tcur = torch.ones(Tn, P, dtype=dt)
        done = ~inside
        flag = torch.zeros(Tn, P, dtype=torch.bool)
        Lmax = int(lens.max())
        for k in range(Lmax):
            act, g, sigma, mag, raw, al = step(k)
            live = act[:, None] & ~done
            if not bool(live.any()):
                break
            near = ((al - thr).abs() <= margin * thr) | (sigma.abs() <= margin * mag)
            ok = live & (sigma >= 0) & (al >= thr)
            nT = Tcur * (1.0 - al)
            near = near | (ok & (((nT - Ref3D.T_MIN).abs() <= margin * Ref3D.T_MIN) |
                                 ((raw - Ref3D.ALPHA_MAX).abs() <= margin)))
            flag |= live & near
            stop = ok & (nT <= Ref3D.T_MIN)
            done = done | stop
            Tcur = torch.where(ok & ~stop, nT, Tcur)
        flag &= inside
        if bool(flag.any()):
            # the flagged pixels' walks again: every entry at or above the skip threshold (minus
            # the margin) up to the pixel's stop, and the next `extra` after it (a stop flip: the
            # other implementation stops at one of the next passing entries, T being at 1e-4)
            rows = torch.nonzero(flag.any(1)).flatten()
            fl = flag[rows]
            Tr = torch.ones(rows.numel(), P, dtype=dt)
            dn = ~inside[rows]
            after = torch.zeros(rows.numel(), P, dtype=torch.int64)
            extra = 2
            for k in range(Lmax):
                act, g, sigma, mag, raw, al = step(k)
                a_r, g_r, s_r, al_r = act[rows][:, None], g[rows], sigma[rows], al[rows]
                passing = a_r & (al_r >= (1.0 - margin) * thr)
                hit = fl & passing & (after < extra)
                sel = hit.any(1)
                if bool(sel.any()):
                    gau[(g_r[sel] % N)] = True
                after = after + (fl & passing & dn).to(torch.int64)
                ok = a_r & ~dn & (s_r >= 0) & (al_r >= thr)
                nT = Tr * (1.0 - al_r)
                stop = ok & (nT <= Ref3D.T_MIN)
                dn = dn | stop
                Tr = torch.where(ok & ~stop, nT, Tr)
                if not bool((a_r & fl & (after < extra)).any()):
                    break
            for n_ in rows.tolist():
                m = flag[n_]
                pix[int(cams[n_]), i[n_][m], j[n_][m]] = True
        return pix, gau, int(pix.sum())


def render3d_pixelloop(params, viewmats, Ks, width, height, background, **kw):
    """Tiny-scene restatement: per-pixel Python loop, fully differentiable by autograd.

    Same discrete decisions as ``raster3d_fwd`` (taken from detached values); used only to
    check the analytic backward in float64.
    """
    dt = params.dtype
    C = viewmats.shape[0]
    N = params.shape[0]
    means, quats, scales, colors, opac = activations3d(params)
    proj = project3d(means, quats, scales, opac, viewmats, Ks, width, height, **kw)
    offsets, ids = isect_tiles(proj.means2d, proj.radii, proj.depths, width, height)
    tile = Ref3D.TILE
    tw = (width + tile - 1) // tile
    th = (height + tile - 1) // tile
    rgb_rows = []
    alpha_rows = []
    for c in range(C):
        rows_c, rows_a = [], []
        for i in range(height):
            row_c, row_a = [], []
            for j in range(width):
                t = c * tw * th + (i // tile) * tw + (j // tile)
                s, e = int(offsets[t]), int(offsets[t + 1])
                T = torch.ones((), dtype=dt)
                Cc = torch.zeros(3, dtype=dt)
                for k in range(s, e):
                    g = int(ids[k])
                    n = g % N
                    xy = proj.means2d[c, n]
                    con = proj.conics[c, n]
                    dx = xy[0] - (j + 0.5)
                    dy = xy[1] - (i + 0.5)
                    sigma = 0.5 * (con[0] * dx * dx + con[2] * dy * dy) + con[1] * dx * dy
                    al = torch.clamp(opac[n] * torch.exp(-sigma), max=Ref3D.ALPHA_MAX)
                    if float(sigma.detach()) < 0 or float(al.detach()) < Ref3D.ALPHA_THRESHOLD:
                        continue
                    nT = T * (1 - al)
                    if float(nT.detach()) <= Ref3D.T_MIN:
                        break
                    Cc = Cc + colors[n] * al * T
                    T = nT
                row_c.append(Cc + T * background.to(dt))
                row_a.append(1 - T)
            rows_c.append(torch.stack(row_c))
            rows_a.append(torch.stack(row_a))
        rgb_rows.append(torch.stack(rows_c))
        alpha_rows.append(torch.stack(rows_a))
    return torch.stack(rgb_rows), torch.stack(alpha_rows)
