"""The backward's per-entry sum updates under aliasing (VERDICT r5 "what's weak" #1).

Every raster backward kernel reduces a group of 7 list entries x 9 partial sums over each 4x4 box's
lanes and then adds, box by box, each box's sums into the wave's per-entry slot in LDS
(raster.hip lw_add).  Two boxes of one wave may list the SAME entry at DIFFERENT positions of the
same group of 7 (their survivor lists differ before it), so the adds to that slot come from two
different lanes.  Round 5 batched the four boxes' reads ahead of their writes (commit 3ec9d20,
rebuilt today with -DGSR_BWD_LWPAR=1): one of the two updates was lost, and every oracle fixture
of the suite stayed green -- the lost box contributions were small (entries at box edges) or hid
inside the full-size tests' outlier allowance.  Only the 200-step fit test caught it.

These fixtures make the pattern the common case: dense overlapping clusters of Gaussians a few
pixels wide, so most entries reach several 4x4 boxes with substantial alpha, at group positions
that differ box to box.  Each is compared with the oracle with NO outlier fraction (3D: the
forward may leave the tolerance only at a discrete-decision tie the oracle flags,
oracle3d.tie_flags, and the cotangent is zero there, so every gradient element must match; 2D has
no such decisions), for every backward kernel that uses lw_add:
  * 3D k_raster_bwd (one pixel per lane, 128-entry units) and k_raster_bwd_pair3d (two pixels
    per lane), each with and without the forward's box masks, and the multi-sub-chunk form
    (256-entry units);
  * 2D k_raster2d_bwd_pair (one parameter set) and k_raster2d_bwd_frame (sets of several cameras;
    whole-list walks and the split walks of gsr_set_bwd2d_parts).
The fixture also counts, from the oracle's lists, how many (chunk, quadrant) groups hold an entry
that two boxes list at different positions of one group of 7 -- the racy pattern -- and requires
hundreds of them.  tools/race_control.sh runs this file against the -DGSR_BWD_LWPAR=1 build
(negative control: it must FAIL) and against the shipped library (it must pass);
profiles/r06_race_control.txt holds the record.
"""
import math

import pytest
import torch

from _util import assert_close, close_at_ties, grad_close, untie_cotangent

pytestmark = pytest.mark.gpu


def _cluster_scene3d(N, W, H, C, seed):
    """Clusters of Gaussians 2-5 px wide (sigma) that overlap densely: entries span 4x4 boxes."""
    from gsr.scenes import ring_cameras
    g = torch.Generator().manual_seed(seed)
    centres = (torch.rand(4, 3, generator=g) * 2 - 1) * 0.05
    p = torch.empty(N, 14)
    p[:, 0:3] = centres[torch.arange(N) % 4] + 0.02 * torch.randn(N, 3, generator=g)
    p[:, 3:6] = math.log(0.03) + torch.rand(N, 3, generator=g) * math.log(3.0)
    p[:, 6:10] = torch.randn(N, 4, generator=g)
    p[:, 10:13] = torch.rand(N, 3, generator=g)
    p[:, 13] = 1.5 * torch.randn(N, generator=g)
    V, K = ring_cameras(C, W, H)
    return p, V, K


def _racy_groups(p, V, K, W, H):
    """(chunk, quadrant) groups of the oracle's lists in which some entry is listed by two 4x4
    boxes at different positions of the same group of 7 (box lists back to front, as the kernel
    walks them; box membership approximated by alpha >= 1/255 at one of the box's pixels)."""
    from oracle import oracle3d as o
    C, N = V.shape[0], p.shape[0]
    m, q, s, col, op = o.activations3d(p)
    pr = o.project3d(m, q, s, op, V, K, W, H)
    off, ids = o.isect_tiles(pr.means2d, pr.radii, pr.depths, W, H)
    tw, th = (W + 15) // 16, (H + 15) // 16
    xy, con = pr.means2d.detach().reshape(C * N, 2), pr.conics.detach().reshape(C * N, 3)
    opc = op.detach()[None].expand(C, N).reshape(-1)
    racy = 0
    for ct in range(C * tw * th):
        a, b = int(off[ct]), int(off[ct + 1])
        if b <= a:
            continue
        t = ct % (tw * th)
        x0, y0 = 16 * (t % tw), 16 * (t // tw)
        yy, xx = torch.meshgrid(torch.arange(16) + y0 + 0.5, torch.arange(16) + x0 + 0.5, indexing="ij")
        for c0 in range(a, b, 128):
            g = ids[c0:min(b, c0 + 128)]
            dx = xy[g, 0][:, None, None] - xx[None]
            dy = xy[g, 1][:, None, None] - yy[None]
            sg = 0.5 * (con[g, 0][:, None, None] * dx * dx + con[g, 2][:, None, None] * dy * dy) \
                + con[g, 1][:, None, None] * dx * dy
            hit = opc[g][:, None, None] * torch.exp(-sg) >= 1.0 / 255.0        # [n,16,16]
            boxes = hit.view(-1, 4, 4, 4, 4).any(2).any(3)                     # [n, by, bx]
            for qy in range(2):
                for qx in range(2):
                    sub = boxes[:, 2 * qy:2 * qy + 2, 2 * qx:2 * qx + 2].reshape(-1, 4).flip(0)
                    pos = torch.cumsum(sub.to(torch.int64), 0) - 1                # back-to-front slot
                    both = sub.sum(1) >= 2
                    if not bool(both.any()):
                        continue
                    pp = torch.where(sub[both], pos[both], torch.full_like(pos[both], -1))
                    grp = torch.where(pp >= 0, pp // 7, pp)
                    for r in range(pp.shape[0]):
                        sl = [(int(grp[r, k]), int(pp[r, k] % 7)) for k in range(4) if int(pp[r, k]) >= 0]
                        if any(g1 == g2 and s1 != s2 for i, (g1, s1) in enumerate(sl) for g2, s2 in sl[i + 1:]):
                            racy += 1
                            break
    return racy


def _gpu3d(p, V, K, W, H, bg, cuda, vr, va):
    from gsr import render as R
    pg = p.to(cuda).requires_grad_(True)
    rgb, alpha = R.render3d(pg, V.to(cuda), K.to(cuda), W, H, bg.to(cuda), R.RenderOptions3D(capacity="exact"))
    torch.autograd.backward([rgb, alpha], [vr.to(cuda), va.to(cuda)])
    return rgb.detach().cpu(), alpha.detach().cpu(), pg.grad.detach().cpu()


@pytest.fixture(scope="module")
def scene3d():
    from oracle import oracle3d as o
    W, H, C = 64, 64, 2
    p, V, K = _cluster_scene3d(1500, W, H, C, 2606)
    bg = torch.tensor([0.3, 0.6, 0.9])
    g = torch.Generator().manual_seed(2607)
    vr, va = torch.randn(C, H, W, 3, generator=g), torch.randn(C, H, W, generator=g)
    tie_pix, vr, va = untie_cotangent(p, V, K, W, H, vr, va)
    po = p.clone().requires_grad_(True)
    rgb_o, a_o = o.render3d(po, V, K, W, H, bg)
    torch.autograd.backward([rgb_o, a_o], [vr, va])
    racy = _racy_groups(p, V, K, W, H)
    print(f"[race3d] {racy} (chunk, quadrant) groups with an entry at two positions of one group of 7; "
          f"{int(tie_pix.sum())} tie pixels (no cotangent)")
    return dict(p=p, V=V, K=K, W=W, H=H, bg=bg, vr=vr, va=va, rgb=rgb_o.detach(), alpha=a_o.detach(),
                grad=po.grad.detach(), tie_pix=tie_pix, racy=racy)


@pytest.mark.parametrize("layout,entries,lanes", [(1, 128, 0), (1, 128, 4), (1, 256, 0), (2, 128, 0), (2, 128, 4)],
                         ids=["k_raster_bwd", "k_raster_bwd_box_masks", "k_raster_bwd_multi", "k_raster_bwd_pair3d",
                              "k_raster_bwd_pair3d_box_masks"])
def test_race_3d(cuda, scene3d, layout, entries, lanes):
    """lanes 4: the quad forward, whose box masks the backward lists its boxes from (ABI 14);
    the fixture's small views otherwise take the 16-lane forward, which writes none."""
    from gsr import render as R
    from _util import forced_bwd_layout, forced_fwd_lanes
    s = scene3d
    assert s["racy"] >= 300, s["racy"]   # the fixture exercises the aliasing pattern
    R.set_chunk_entries("3d", entries)
    try:
        with forced_bwd_layout(layout), forced_fwd_lanes(lanes):
            rgb, alpha, grad = _gpu3d(s["p"], s["V"], s["K"], s["W"], s["H"], s["bg"], cuda, s["vr"], s["va"])
    finally:
        R.set_chunk_entries("3d", 128)
    close_at_ties(rgb, s["rgb"], s["tie_pix"], what=f"race3d rgb ({layout},{entries})")
    close_at_ties(alpha, s["alpha"], s["tie_pix"], what=f"race3d alpha ({layout},{entries})")
    grad_close(grad, s["grad"], what=f"race3d grad ({layout},{entries})")


def _cluster_scene2d(N, W, H, seed):
    g = torch.Generator().manual_seed(seed)
    centres = torch.rand(3, 2, generator=g) * torch.tensor([W * 0.6, H * 0.6]) + torch.tensor([W * 0.2, H * 0.2])
    p = torch.empty(N, 9)
    p[:, 0:2] = centres[torch.arange(N) % 3] + 6.0 * torch.randn(N, 2, generator=g)
    p[:, 2:4] = 1.0 + 0.35 * torch.randn(N, 2, generator=g)     # sigma ~1.5-5 px
    p[:, 4] = (torch.rand(N, generator=g) * 2 - 1) * math.pi
    p[:, 5:8] = torch.rand(N, 3, generator=g)
    p[:, 8] = -1.0 + 1.5 * torch.randn(N, generator=g)        # mostly translucent: long walks
    return p


def test_race_2d_single_set(cuda):
    """k_raster2d_bwd_pair (one parameter set, one camera) vs the dense reference compositor."""
    from gsr import render as R
    from oracle.oracle2d import render2d_dense
    W, H = 64, 48
    p = _cluster_scene2d(500, W, H, 2611)
    bg = torch.tensor([0.2, 0.5, 0.7])
    g = torch.Generator().manual_seed(2612)
    vr, va = torch.randn(H, W, 3, generator=g), torch.randn(H, W, generator=g)
    pg = p.to(cuda).requires_grad_(True)
    rgb, alpha = R.render2d(pg, W, H, bg.to(cuda), capacity="exact")
    torch.autograd.backward([rgb, alpha], [vr.to(cuda), va.to(cuda)])
    po = p.clone().requires_grad_(True)
    rgb_o, a_o = render2d_dense(po, W, H, bg)
    torch.autograd.backward([rgb_o, a_o], [vr, va])
    assert_close(rgb.detach().cpu(), rgb_o.detach(), what="race2d rgb")
    assert_close(alpha.detach().cpu(), a_o.detach(), what="race2d alpha")
    grad_close(pg.grad.cpu(), po.grad, what="race2d grad")


@pytest.mark.parametrize("parts_target", [0, 4608], ids=["whole_walks", "split_walks"])
def test_race_2d_frames(cuda, parts_target):
    """k_raster2d_bwd_frame: 3 frames x 2-3 cameras (each camera its own cotangent) in one
    launch sequence; each frame's gradient vs the sum of the dense oracle's per-camera gradients.
    parts_target 4608 (the binding's setting) splits each tile's walk into parts (few (set, tile)
    pairs here), 0 walks whole lists."""
    from gsr import _lib, render as R
    from oracle.oracle2d import render2d_dense
    W, H = 64, 48
    F = 3
    sets = (0, 0, 1, 1, 1, 2, 2)
    P = torch.stack([_cluster_scene2d(400, W, H, 2620 + f) for f in range(F)])
    bg = torch.tensor([0.9, 0.4, 0.1])
    g = torch.Generator().manual_seed(2630)
    Cn = len(sets)
    vr, va = torch.randn(Cn, H, W, 3, generator=g), torch.randn(Cn, H, W, generator=g)
    _lib.check(_lib.lib().gsr_set_bwd2d_parts(parts_target), "gsr_set_bwd2d_parts")
    try:
        pg = P.to(cuda).requires_grad_(True)
        rgb, alpha = R.render2d_units(pg, sets, W, H, bg.to(cuda), capacity="exact")
        torch.autograd.backward([rgb, alpha], [vr.to(cuda), va.to(cuda)])
    finally:
        _lib.check(_lib.lib().gsr_set_bwd2d_parts(_lib.BWD2D_PART_WORKGROUPS), "gsr_set_bwd2d_parts")
    for f in range(F):
        gsum = torch.zeros(400, 9)
        for u in [u for u, s in enumerate(sets) if s == f]:
            po = P[f].clone().requires_grad_(True)
            rgb_o, a_o = render2d_dense(po, W, H, bg)
            torch.autograd.backward([rgb_o, a_o], [vr[u], va[u]])
            gsum += po.grad
            assert_close(rgb.detach().cpu()[u], rgb_o.detach(), what=f"race2d frames rgb unit {u}")
        grad_close(pg.grad.cpu()[f], gsum, what=f"race2d frames grad frame {f} (parts target {parts_target})")
