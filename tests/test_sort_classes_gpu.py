"""The per-tile sort's list-length classes at their boundaries.

gsr_bin_sort sorts each busy tile's list by one of several shapes chosen from device class
counts: one wave per list (< 1 024 entries), four lists per workgroup in 4 096-key slices,
two per workgroup in 8 192-key slices, one 1 024-thread workgroup per list, and the MSD
partition beyond the LDS image; the lazy depth order re-classifies lists longer than its
``min_len``.  Here one view holds tiles whose lists are exactly 1 023 / 1 024 / 4 095 /
4 096 / 8 191 / 8 192 entries long (plus >128 short filler lists, so the class path -- not the
split sort for few busy tiles -- runs), made of runs of Gaussians sharing one mean (equal
depths: ties broken by c*N+n across every class boundary).  Checked:
* the whole lists bit-exact against a CPU sort of (tile, depth bits, c*N+n), lazy order off;
* with the lazy order on at min_len 1 023, 4 095 and 8 192 (prefix 256): every consumed entry
  (before tile_end) is in the exact order, and rgb / alpha / v_params equal the full sort's
  bitwise;
* a capacity-bounded call of the same shape equals the exact one bitwise.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

LENGTHS = [1023, 1024, 4095, 4096, 8191, 8192, 1, 2, 17]
W, H = 256, 160          # 16 x 10 tiles
F = 100.0                # focal length (pixels); camera at the origin looking down +z


def _scene():
    """Params [N,14] (adapter layout) with LENGTHS[i] Gaussians on the centre of tile i and one
    or two on every other tile; runs of 7 share a mean (equal depths)."""
    tw = W // 16
    centres, counts = [], []
    for t in range(tw * (H // 16)):
        counts.append(LENGTHS[t] if t < len(LENGTHS) else 1 + t % 2)
        centres.append((16 * (t % tw) + 8.0, 16 * (t // tw) + 8.0))
    rows = []
    run = 0
    for (u, v), n in zip(centres, counts):
        for k in range(n):
            if k % 7 == 0:
                run += 1
            z = 2.0 + 0.01 * (run % 37)                 # runs of 7: one depth each
            rows.append([(u - W / 2) * z / F, (v - H / 2) * z / F, z])
    m = torch.tensor(rows, dtype=torch.float32)
    N = m.shape[0]
    g = torch.Generator().manual_seed(7)
    p = torch.zeros(N, 14)
    p[:, 0:3] = m
    p[:, 3:6] = -4.6 + 0.1 * torch.randn(N, 3, generator=g)     # ~0.5 px: one tile each
    p[:, 6] = 1.0
    p[:, 10:13] = torch.rand(N, 3, generator=g)
    p[:, 13] = -3.0 + 0.5 * torch.randn(N, generator=g)          # faint: lists walk far
    V = torch.eye(4)[None]
    K = torch.tensor([[F, 0.0, W / 2], [0.0, F, H / 2], [0.0, 0.0, 1.0]])[None]
    return p, V, K


def _expected(b, N):
    rect = b.rect.cpu().view(N, 2).to(torch.int64) & 0xFFFFFFFF
    x0, x1 = rect[:, 0] & 0xFFFF, rect[:, 0] >> 16
    y0, y1 = rect[:, 1] & 0xFFFF, rect[:, 1] >> 16
    cnt = b.cnt.cpu()[:N].to(torch.int64)
    depth = b.depth.cpu()[:N].contiguous().numpy().view(np.uint32).astype(np.int64)
    tw = (W + 15) // 16
    keys = []
    for n in torch.nonzero(cnt > 0).flatten().tolist():
        for ty in range(int(y0[n]), int(y1[n])):
            for tx in range(int(x0[n]), int(x1[n])):
                keys.append((ty * tw + tx, int(depth[n]), n))
    keys.sort()
    return torch.tensor([k[2] for k in keys]), torch.tensor([k[0] for k in keys])


class _lazy:
    def __init__(self, min_len, prefix):
        self.args = (min_len, prefix)

    def __enter__(self):
        from gsr import _lib
        _lib.check(_lib.lib().gsr_set_lazy_sort(*self.args), "gsr_set_lazy_sort")

    def __exit__(self, *exc):
        from gsr import _lib
        _lib.check(_lib.lib().gsr_set_lazy_sort(16384, 4096), "gsr_set_lazy_sort")


def _step(p, V, K, capacity="exact"):
    from gsr import render as R
    dev = p.device
    g = torch.Generator().manual_seed(3)
    vr = torch.randn(1, H, W, 3, generator=g).to(dev)
    va = torch.randn(1, H, W, generator=g).to(dev)
    pg = p.clone().requires_grad_(True)
    rgb, alpha = R.render3d(pg, V, K, W, H, torch.ones(3, device=dev), R.RenderOptions3D(capacity=capacity))
    torch.autograd.backward([rgb, alpha], [vr, va])
    torch.cuda.synchronize()
    return rgb.detach(), alpha.detach(), pg.grad


def test_sort_classes_at_boundaries(cuda):
    from gsr import render as R
    p, V, K = _scene()
    p, V, K = p.to(cuda), V.to(cuda), K.to(cuda)
    N = p.shape[0]
    with _lazy(0, 4096):   # lazy order off: every list sorted whole
        _, _, b, _ = R.debug_forward3d(p, V, K, torch.ones(3, device=cuda), W, H)
        lens = (b.tile_off[1:] - b.tile_off[:-1]).cpu()
        assert lens[:len(LENGTHS)].tolist() == LENGTHS, lens[:len(LENGTHS)].tolist()
        assert b.n_busy > 128, b.n_busy        # the class path, not the split sort
        ids, _ = _expected(b, N)
        I = b.n_isect
        assert I == ids.numel()
        assert torch.equal(b.sorted_ids.cpu()[:I].to(torch.int64), ids)
        ref = _step(p, V, K)
        R._size_hint.clear()
        _step(p, V, K)                              # exact: the bounds of the shape
        bd = _step(p, V, K, "bounded")
        assert R.last_stats()["_bins"].bounded
        assert all(torch.equal(x, y) for x, y in zip(ref, bd))
    for min_len in (1023, 4095, 8192):
        with _lazy(min_len, 256):
            _, _, b, _ = R.debug_forward3d(p, V, K, torch.ones(3, device=cuda), W, H)
            ids, tiles = _expected(b, N)
            te = b.tile_end.cpu().to(torch.int64)
            consumed = torch.arange(ids.numel()) < te[tiles]
            got = b.sorted_ids.cpu()[:ids.numel()].to(torch.int64)
            assert torch.equal(got[consumed], ids[consumed]), min_len
            lz = _step(p, V, K)
            assert all(torch.equal(x, y) for x, y in zip(ref, lz)), min_len
    R.check_overflow(cuda)
    R._size_hint.clear()
