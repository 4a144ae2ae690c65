"""The parity helpers themselves: non-finite values and unbounded outliers must fail."""
import pytest
import torch

from _util import assert_close, grad_close


def test_nan_render_fails():
    e = torch.rand(8, 8, 3)
    with pytest.raises(AssertionError):
        assert_close(torch.full_like(e, float("nan")), e)
    with pytest.raises(AssertionError):
        assert_close(e.clone().index_fill_(0, torch.tensor([2]), float("inf")), e, max_frac=0.5, max_outlier=1.0)


def test_nan_grad_fails():
    e = torch.randn(100, 14)
    a = e.clone()
    a[3, 4] = float("nan")
    with pytest.raises(AssertionError):
        grad_close(a, e, max_frac=0.05, outlier_rel=10.0)


def test_grad_outlier_bound():
    e = torch.randn(1000, 14)
    a = e.clone()
    a[0, 0] = -e[0, 0] + 3.0 * float(e[:, 0].abs().max())   # one garbage entry in 14k
    grad_close(e.clone(), e)                                   # exact passes
    with pytest.raises(AssertionError):
        grad_close(a, e, max_frac=2e-3, outlier_rel=0.05)
    b = e.clone()
    b[0, 0] += 0.01 * float(e[:, 0].abs().max())             # a bounded tie-flip passes
    r = grad_close(b, e, max_frac=2e-3, outlier_rel=0.05)
    assert r["n_bad"] == 1
    with pytest.raises(AssertionError):                       # max_frac without a bound
        grad_close(b, e, max_frac=2e-3)


def test_per_column_floor():
    # a small column (e.g. quaternion grads) is not hidden behind a large column's scale
    e = torch.randn(500, 2)
    e[:, 1] *= 1e-4
    a = e.clone()
    a[:, 1] += 1e-3 * 1e-4 * 5
    with pytest.raises(AssertionError):
        grad_close(a, e)
