"""Tolerance helpers shared by the parity tests.

An element is bad when |a-e| > atol + rtol*|e| OR when either side is non-finite (NaN/Inf never
compare close, so an all-NaN render or gradient fails every check).  Every check prints its
observed frac_bad / max_bad so drift is visible in the test log (`pytest -s` or the -v report).
"""
import torch


def close_report(actual: torch.Tensor, expected: torch.Tensor, rtol: float, atol):
    a = actual.detach().double().cpu()
    e = expected.detach().double().cpu()
    assert a.shape == e.shape, (a.shape, e.shape)
    err = (a - e).abs()
    tol = atol + rtol * e.abs()
    finite = torch.isfinite(a) & torch.isfinite(e)
    bad = ~(err <= tol) | ~finite          # NaN err compares False, so ~(err<=tol) catches it
    err_f = torch.where(finite, err, torch.full_like(err, float("inf")))
    # how far past its tolerance the worst bad element is, in units of the outlier scale
    return dict(max_err=float(err_f.max()) if err.numel() else 0.0,
                n_bad=int(bad.sum()), n=err.numel(),
                frac_bad=float(bad.double().mean()) if err.numel() else 0.0,
                max_bad=float(err_f[bad].max()) if bool(bad.any()) else 0.0,
                nonfinite=int((~finite).sum()))


def _report(what, r):
    print(f"[close] {what}: frac_bad={r['frac_bad']:.3e} ({r['n_bad']}/{r['n']}) "
          f"max_bad={r['max_bad']:.3e} max_err={r['max_err']:.3e} nonfinite={r['nonfinite']}")


def assert_close(actual, expected, rtol=1e-4, atol=1e-6, max_frac=0.0, max_outlier=None, what=""):
    r = close_report(actual, expected, rtol, atol)
    _report(what, r)
    msg = f"{what}: {r}"
    assert r["nonfinite"] == 0 or bool((torch.isfinite(actual.detach().cpu()) ==
                                        torch.isfinite(expected.detach().cpu())).all()), msg
    assert r["frac_bad"] <= max_frac, msg
    if max_frac > 0:
        # tolerated elements must still be finite and bounded: an unbounded outlier allowance
        # would let garbage (wrong sign, huge values) through at the tolerated fraction
        assert max_outlier is not None, f"{what}: max_frac > 0 needs a max_outlier bound"
    if max_outlier is not None:
        assert r["max_bad"] <= max_outlier, msg
    return r


def grad_close(actual, expected, rtol=1e-4, rel_floor=1e-5, max_frac=0.0, outlier_rel=None, what=""):
    """Elementwise |a-e| <= rtol*|e| + rel_floor*max|e[..., col]| (abs floor scaled to each
    parameter column, i.e. each of the P gradient components of an [N,P] gradient).

    With max_frac > 0 (discrete-decision ties between two correct fp32 implementations: a pixel
    where alpha>=1/255 or T<=1e-4 resolves differently), the elements outside the tolerance must
    still satisfy |a-e| <= outlier_rel * max|e[..., col]|.  Such a tie changes a Gaussian's
    gradient by at most ONE pixel's contribution (the flipped Gaussian's own alpha ~1/255 or
    T ~1e-4 term, and a (1-1/255) factor on the pixel's later contributions), which is a small
    fraction of the column's largest whole-image gradient; `outlier_rel` is that fraction."""
    e = expected.detach().double().cpu()
    if e.dim() >= 2 and e.numel():
        scale = e.abs().reshape(-1, e.shape[-1]).amax(dim=0).clamp_min(1e-30)
    else:
        scale = torch.tensor(float(e.abs().max()) if e.numel() else 1e-30).clamp_min(1e-30)
    r = close_report(actual, expected, rtol, rel_floor * scale)
    if max_frac > 0:
        assert outlier_rel is not None, f"{what}: max_frac > 0 needs outlier_rel"
    # the worst bad element relative to its column scale
    a = actual.detach().double().cpu()
    err = (a - e).abs()
    bad = ~(err <= rel_floor * scale + rtol * e.abs()) | ~torch.isfinite(a)
    rel = torch.where(bad, err / scale, torch.zeros_like(err))
    rel = torch.where(torch.isfinite(rel), rel, torch.full_like(rel, float("inf")))
    r["max_bad_rel_col"] = float(rel.max()) if rel.numel() else 0.0
    print(f"[grad] {what}: frac_bad={r['frac_bad']:.3e} ({r['n_bad']}/{r['n']}) "
          f"max_bad/col_scale={r['max_bad_rel_col']:.3e} nonfinite={r['nonfinite']}")
    msg = f"{what}: {r}"
    assert r["nonfinite"] == 0 or bool((torch.isfinite(a) == torch.isfinite(e)).all()), msg
    assert r["frac_bad"] <= max_frac, msg
    if outlier_rel is not None:
        assert r["max_bad_rel_col"] <= outlier_rel, msg
    return r


class forced_fwd_lanes:
    """Force the raster forward's layout (gsr_set_fwd_lanes) inside a with-block.  The automatic
    choice (3D: 16 lanes per pixel when at most 160 tiles are busy, else 4)
    depends on the call's busy tile count, and the layouts group the transmittance products
    differently (fp32 rounding), so bitwise comparisons between calls of different sizes (a
    batch view vs a single-view render, a band vs the full image) fix one layout."""

    def __init__(self, lanes: int):
        self.lanes = lanes

    def __enter__(self):
        from gsr import _lib
        _lib.check(_lib.lib().gsr_set_fwd_lanes(self.lanes), "gsr_set_fwd_lanes")
        return self

    def __exit__(self, *exc):
        from gsr import _lib
        _lib.check(_lib.lib().gsr_set_fwd_lanes(0), "gsr_set_fwd_lanes")
        return False


class forced_bwd_layout:
    """Force the 3D raster backward's layout (gsr_set_bwd_layout: 1 one pixel per lane, 2 two)
    inside a with-block; automatic afterwards."""

    def __init__(self, layout: int):
        self.layout = layout

    def __enter__(self):
        from gsr import _lib
        _lib.check(_lib.lib().gsr_set_bwd_layout(self.layout), "gsr_set_bwd_layout")
        return self

    def __exit__(self, *exc):
        from gsr import _lib
        _lib.check(_lib.lib().gsr_set_bwd_layout(0), "gsr_set_bwd_layout")
        return False


def close_at_ties(actual, expected, tie_pixels, rtol=1e-4, atol=1e-6, max_outlier=0.02, what=""):
    """Forward image check with per-element justification: a pixel may be outside
    |a-e| <= atol + rtol*|e| only where the oracle flags a discrete-decision tie
    (oracle3d.tie_flags), and there by at most max_outlier.  actual/expected [C,H,W] or
    [C,H,W,3]; tie_pixels [C,H,W] bool."""
    a = actual.detach().double().cpu()
    e = expected.detach().double().cpu()
    bad = ~((a - e).abs() <= atol + rtol * e.abs()) | ~torch.isfinite(a)
    if bad.dim() == tie_pixels.dim() + 1:
        bad = bad.any(-1)
    err = (a - e).abs()
    if err.dim() == tie_pixels.dim() + 1:
        err = err.amax(-1)
    unexplained = bad & ~tie_pixels
    n_bad, n_tie = int(bad.sum()), int(tie_pixels.sum())
    worst = float(err[bad].max()) if n_bad else 0.0
    print(f"[ties] {what}: {n_bad} pixels out of tolerance, all at the oracle's {n_tie} tie pixels: "
          f"{int(unexplained.sum()) == 0}; worst {worst:.3e}")
    assert int(unexplained.sum()) == 0, f"{what}: {int(unexplained.sum())} out-of-tolerance pixels at no flagged tie"
    assert worst <= max_outlier, f"{what}: a tie pixel differs by {worst} > {max_outlier}"
    return n_bad


def untie_cotangent(params, viewmats, Ks, width, height, v_rgb, v_alpha, **kw):
    """(tie pixels, v_rgb, v_alpha with zeros at them): the oracle's discrete-decision ties
    (oracle3d.tie_flags) carry no cotangent, so a decision flipped there between two correct
    fp32 implementations cannot move any gradient -- the gradients then compare with no outlier
    allowance (the full-size checks' 0.2 % allowance could hide lost updates)."""
    from oracle.oracle3d import tie_flags
    pix, _, n = tie_flags(params, viewmats, Ks, width, height, **kw)
    print(f"[ties] {n} of {pix.numel()} pixels at a discrete-decision tie: cotangent zeroed there")
    keep = (~pix).to(v_alpha.dtype)
    return pix, v_rgb * keep[..., None], v_alpha * keep
