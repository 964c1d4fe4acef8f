"""The parity helpers themselves: a NaN / inf anywhere must fail a check, never
vanish inside max() (nan > x is False) or compare below a bar."""
import numpy as np
import pytest

from _fixtures import rel_err, normwise, scalar_rel, worst_of, assert_all_within, NonFiniteError


@pytest.mark.parametrize("bad", [np.nan, np.inf, -np.inf])
def test_rel_err_and_normwise_refuse_non_finite(bad):
    a = np.ones(5)
    b = np.ones(5)
    a[2] = bad
    for f in (rel_err, normwise):
        with pytest.raises(NonFiniteError):
            f(a, b)
        with pytest.raises(NonFiniteError):
            f(b, a)
    assert np.isnan(rel_err(a, b, allow_nonfinite=True)) or np.isinf(rel_err(a, b, allow_nonfinite=True))
    with pytest.raises(NonFiniteError):
        scalar_rel(bad, 1.0)


def test_worst_of_and_assert_all_within_fail_on_nan():
    errs = {"h": 1e-7, "pos": float("nan"), "vel": 2e-7}
    assert np.isnan(worst_of(errs))
    assert max(errs.values()) < 1e-5          # the trap the helpers close
    with pytest.raises(AssertionError):
        assert_all_within(errs, 1e-5)
    with pytest.raises(AssertionError):
        assert_all_within([float("nan")], 1.0)
    assert_all_within({"h": 1e-7, "g": 0.0}, 1e-5)
    assert worst_of([1e-7, 3e-7]) == 3e-7


def test_rel_err_values():
    assert rel_err([1.0, 2.0], [1.0, 2.0]) == 0.0
    assert rel_err([1.0, 2.2], [1.0, 2.0]) == pytest.approx(0.1)
    assert normwise([3.0, 4.0], [0.0, 0.0]) > 0
    assert rel_err(np.zeros(0), np.zeros(0)) == 0.0
