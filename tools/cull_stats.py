#!/usr/bin/env python3
"""Backward work model per layout (GPU box): for a config's scene, count the survivor groups
the raster backward would walk under different (culling box, lanes-per-list) layouts.

For every active chunk (GSR_CHUNK entries before the tile's tile_end) and every box size, the
exact cull test of csrc/raster.hip::cull_keep decides which entries reach each box; a wave walks
groups of G survivors and waves whose lanes serve several boxes walk max over their boxes.
Prints groups and pair slots per layout, relative to the current one (8x8 box per wave).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pose-splatter_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def keep(rec, bx0, bx1, by0, by1):
    """cull_keep<false> on [M,12] records vs boxes (broadcast tensors)."""
    x, y, L = rec[..., 0], rec[..., 1], rec[..., 3]
    a, b, c, s1 = rec[..., 4], rec[..., 5], rec[..., 6], rec[..., 7]
    s2 = rec[..., 11]
    dxe = x - torch.minimum(torch.maximum(x, bx0), bx1)
    dye = y - torch.minimum(torch.maximum(y, by0), by1)
    dy1 = torch.minimum(torch.maximum(s1 * dxe, y - by1), y - by0)
    dx2 = torch.minimum(torch.maximum(s2 * dye, x - bx1), x - bx0)
    v1 = a * dxe * dxe + b * dxe * dy1 + c * dy1 * dy1
    v2 = a * dx2 * dx2 + b * dx2 * dye + c * dye * dye
    pd = (a > 0) & (c > 0) & (4 * a * c > b * b)
    return (L >= 0) & (~pd | (torch.minimum(v1, v2) <= L * 1.001 + 1e-3))


def main():
    from gsr import render as R
    from gsr.scenes import CONFIGS, gaussians3d, ring_cameras
    cfg = CONFIGS[int(sys.argv[1]) if len(sys.argv) > 1 else 3]
    dev = torch.device("cuda")
    p = gaussians3d(cfg.N, cfg.seed).to(dev)
    V, K = ring_cameras(cfg.views, cfg.width, cfg.height)
    _, _, b, _ = R.debug_forward3d(p, V.to(dev), K.to(dev), torch.ones(3, device=dev), cfg.width, cfg.height)
    torch.cuda.synchronize()
    rec = b.rec.view(-1, 12)
    ids = b.sorted_ids[:b.n_isect].long()
    toff = b.tile_off.long()
    tend = b.tile_end.long()
    tw, th = b.tw, b.th
    CT = b.CT
    chunk = 128
    # active entries: (tile, position) before tile_end
    starts, ends = toff[:-1], tend
    n_act = (ends - starts).clamp(min=0)
    tiles = torch.repeat_interleave(torch.arange(CT, device=dev), n_act)
    first = torch.repeat_interleave(starts, n_act)
    pos = torch.arange(int(n_act.sum()), device=dev) - torch.repeat_interleave(torch.cumsum(n_act, 0) - n_act, n_act)
    r = rec[ids[first + pos]]
    ck = pos // chunk   # chunk within the tile
    t = tiles % (tw * th)
    ty, tx = t // tw, t % tw
    walk = (ends - starts).clamp(min=0)
    lens = toff[1:] - toff[:-1]
    top = torch.topk(walk, 12)
    print("longest walks (entries read before every pixel stopped):", top.values.tolist())
    print("  their list lengths:", lens[top.indices].tolist())
    print("walk percentiles (busy tiles):", [int(torch.quantile(walk[lens > 0].float(), q)) for q in (0.5, 0.9, 0.99)])
    print(f"{cfg.name}: I={b.n_isect} I_eff={int(n_act.sum())} chunks={int(((n_act + chunk - 1) // chunk).sum())}")
    res = {}
    G = 7
    for bw, bh in [(8, 8), (4, 4), (8, 4), (4, 8), (16, 16), (16, 8)]:
        nbx, nby = 16 // bw, 16 // bh
        cnt = []
        for by in range(nby):
            for bx in range(nbx):
                x0 = (tx * 16 + bx * bw).float() + 0.5
                y0 = (ty * 16 + by * bh).float() + 0.5
                k = keep(r, x0, x0 + bw - 1, y0, y0 + bh - 1)
                # survivors per (tile, chunk, box)
                key = tiles * 4096 + ck
                u, inv = torch.unique(key, return_inverse=True)
                s = torch.zeros(u.numel(), device=dev).index_add_(0, inv, k.float())
                cnt.append(s)
        res[(bw, bh)] = torch.stack(cnt, 1)   # [units, boxes] with boxes row-major over the tile
        print(f"box {bw}x{bh}: survivors {int(res[(bw, bh)].sum())}  pixel-pairs {int(res[(bw, bh)].sum()) * bw * bh}")
    base = res[(8, 8)]
    g_base = torch.ceil(base / G).sum()
    print(f"layout A (8x8 box per wave, groups of {G}): groups {int(g_base)}")

    def rows_layout(box, boxes_per_wave_idx, G, label):
        s = res[box]
        tot = 0
        for idx in boxes_per_wave_idx:
            m = s[:, idx].max(1).values
            tot += torch.ceil(m / G).sum()
        print(f"{label}: wave-groups {int(tot)} ({float(tot / g_base):.3f} x A)")
        return tot
    # B: 4x4 boxes, one per 16-lane row, wave = one 8x8 quadrant (4 boxes)
    quads = [[(2 * qy + dy) * 4 + 2 * qx + dx for dy in (0, 1) for dx in (0, 1)] for qy in (0, 1) for qx in (0, 1)]
    rows_layout((4, 4), quads, 7, "B 4x4 per 16-lane row, 7-groups")
    rows_layout((4, 4), quads, 4, "B 4x4 per 16-lane row, 4-groups")
    # C: 8x8 boxes, two per wave (2 px per lane), halves = left/right quadrants
    rows_layout((8, 8), [[0, 1], [2, 3]], 7, "C 8x8 per 32-lane half (2 px/lane), 7-groups")
    # D: 8x8 boxes, four per wave (4 px per lane)
    rows_layout((8, 8), [[0, 1, 2, 3]], 7, "D 8x8 per 16-lane row (4 px/lane), 7-groups")
    # E: 4x8 boxes (w4 x h8), four per wave over a 16x8 half tile, 2 px/lane
    s48 = res[(4, 8)]   # boxes: nbx=4, nby=2 -> idx = by*4+bx
    rows_layout((4, 8), [[0, 1, 2, 3], [4, 5, 6, 7]], 7, "E 4x8 per 16-lane row (2 px/lane), 7-groups")
    rows_layout((8, 4), [[0, 1, 2, 3], [4, 5, 6, 7]], 7, "E' 8x4 per 16-lane row (2 px/lane), 7-groups")
    # F: 4x4 boxes, eight per wave (16x8 half tile, 8 lanes x 2 px per box); cost per group
    # ~716 VALU (14 pairs per lane) vs ~422 for B's 7 pairs
    halves = [[(2 * hy + dy) * 4 + bx for dy in (0, 1) for bx in range(4)] for hy in (0, 1)]
    gb = rows_layout((4, 4), quads, 7, "B again")
    gf = rows_layout((4, 4), halves, 7, "F 4x4, 8 boxes per wave (2 px/lane), 7-groups")
    print(f"VALU model: B {float(gb) * 422:.3e}  F {float(gf) * 716:.3e}  ratio {float(gf * 716 / (gb * 422)):.3f}")
    gf5 = rows_layout((4, 4), halves, 5, "F 5-groups")
    # G: 4x4 boxes assigned to the four waves by survivor count (sorted, 4 consecutive per wave)
    s44 = res[(4, 4)]
    srt = torch.sort(s44, 1, descending=True).values
    for G_ in (5, 6, 7, 8):
        tot = sum(torch.ceil(srt[:, 4 * w] / G_).sum() for w in range(4))
        print(f"G balanced 4x4, {G_}-groups: wave-groups {int(tot)} ({float(tot / g_base):.3f} x A), "
              f"lane-pair slots {int(tot) * G_ * 64}  (B: {int(gb) * 7 * 64})")
    for G_ in (5, 6, 8):
        rows_layout((4, 4), quads, G_, f"B {G_}-groups")
    print(f"VALU model F5 (~520/group): ratio {float(gf5 * 520 / (gb * 422)):.3f}")


if __name__ == "__main__":
    main()
