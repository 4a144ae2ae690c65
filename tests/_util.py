"""Tolerance helpers shared by the parity tests."""
import torch


def close_report(actual: torch.Tensor, expected: torch.Tensor, rtol: float, atol: float):
    a = actual.detach().double().cpu()
    e = expected.detach().double().cpu()
    err = (a - e).abs()
    tol = atol + rtol * e.abs()
    bad = err > tol
    return dict(max_err=float(err.max()) if err.numel() else 0.0,
                n_bad=int(bad.sum()), n=err.numel(),
                frac_bad=float(bad.double().mean()) if err.numel() else 0.0,
                max_bad=float(err[bad].max()) if bool(bad.any()) else 0.0)


def assert_close(actual, expected, rtol=1e-4, atol=1e-6, max_frac=0.0, max_outlier=None, what=""):
    r = close_report(actual, expected, rtol, atol)
    msg = f"{what}: {r}"
    assert r["frac_bad"] <= max_frac, msg
    if max_outlier is not None:
        assert r["max_bad"] <= max_outlier, msg
    return r


def grad_close(actual, expected, rtol=1e-4, rel_floor=1e-5, max_frac=0.0, what=""):
    """Elementwise |a-e| <= rtol*|e| + rel_floor*max|e| (abs floor scaled to the tensor)."""
    scale = float(expected.detach().abs().max()) if expected.numel() else 0.0
    return assert_close(actual, expected, rtol=rtol, atol=rel_floor * max(scale, 1e-30),
                        max_frac=max_frac, what=what)
