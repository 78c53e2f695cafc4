"""Sparse statistics / in-place edits (reference ``utils/sparsefuncs.py``,
``sparsefuncs_fast.pyx``)."""
import numpy as np
import pytest
import scipy.sparse as sp

import sq_learn_amd.utils.sparsefuncs as Q

S = pytest.importorskip("sklearn.utils.sparsefuncs")
SF = pytest.importorskip("sklearn.utils.sparsefuncs_fast")


@pytest.fixture
def A():
    rng = np.random.RandomState(0)
    A = rng.rand(30, 8)
    A[A < 0.6] = 0
    return A


@pytest.mark.parametrize("fmt", ["csr", "csc"])
@pytest.mark.parametrize("axis", [0, 1])
def test_mean_variance(A, fmt, axis):
    A = A.copy()
    A[3, 2] = np.nan
    X = sp.csr_matrix(A) if fmt == "csr" else sp.csc_matrix(A)
    rng = np.random.RandomState(1)
    for w in (None, rng.rand(X.shape[axis])):
        a = S.mean_variance_axis(X, axis, weights=w, return_sum_weights=True)
        b = Q.mean_variance_axis(X, axis, weights=w, return_sum_weights=True)
        for x, y in zip(a, b):
            np.testing.assert_allclose(x, y, equal_nan=True)
    m = X.shape[1 - axis]
    lm, lv, ln = rng.rand(m), rng.rand(m), np.full(m, 5.0)
    a = S.incr_mean_variance_axis(X, axis=axis, last_mean=lm.copy(), last_var=lv.copy(),
                                  last_n=ln.copy())
    b = Q.incr_mean_variance_axis(X, axis=axis, last_mean=lm, last_var=lv, last_n=ln)
    for x, y in zip(a, b):
        np.testing.assert_allclose(x, y, equal_nan=True)
    # a feature whose running count is 0 takes the new batch statistics (the
    # reference produces NaN for it on a non-first pass)
    ln[0] = 0
    b = Q.incr_mean_variance_axis(X, axis=axis, last_mean=lm, last_var=lv, last_n=ln)
    assert np.isfinite(b[1][0]) or np.isnan(Q.mean_variance_axis(X, axis)[1][0])


@pytest.mark.parametrize("fmt", ["csr", "csc"])
def test_inplace_ops_and_minmax(A, fmt):
    X = sp.csr_matrix(A) if fmt == "csr" else sp.csc_matrix(A)
    rng = np.random.RandomState(2)
    for ax in (0, 1):
        for x, y in zip(S.min_max_axis(X, ax), Q.min_max_axis(X, ax)):
            np.testing.assert_allclose(x, y)
    for f, args in [("inplace_swap_row", (2, 7)), ("inplace_swap_row", (9, 1)),
                    ("inplace_swap_column", (1, 5)), ("inplace_column_scale", (rng.rand(8),)),
                    ("inplace_row_scale", (rng.rand(30),))]:
        X1, X2 = X.copy(), X.copy()
        getattr(S, f)(X1, *args)
        getattr(Q, f)(X2, *args)
        np.testing.assert_allclose(X1.toarray(), X2.toarray())


def test_counts_median_norms(A):
    X = sp.csr_matrix(A)
    w = np.random.RandomState(3).rand(30)
    for ax in (None, 0, 1):
        np.testing.assert_allclose(S.count_nonzero(X, axis=ax, sample_weight=w),
                                   Q.count_nonzero(X, axis=ax, sample_weight=w))
    B = sp.csc_matrix(A - 0.3 * (A > 0))
    np.testing.assert_allclose(S.csc_median_axis_0(B), Q.csc_median_axis_0(B))
    np.testing.assert_allclose(SF.csr_row_norms(X), Q.csr_row_norms(X))
    for f in ("inplace_csr_row_normalize_l1", "inplace_csr_row_normalize_l2"):
        X1, X2 = X.copy(), X.copy()
        getattr(SF, f)(X1)
        getattr(Q, f)(X2)
        np.testing.assert_allclose(X1.toarray(), X2.toarray())
    o1, o2 = np.zeros((5, 8)), np.zeros((5, 8))
    SF.assign_rows_csr(X, np.array([3, 1, 4]), np.array([0, 2, 4]), o1)
    Q.assign_rows_csr(X, np.array([3, 1, 4]), np.array([0, 2, 4]), o2)
    np.testing.assert_allclose(o1, o2)
    with pytest.raises(TypeError):
        Q.mean_variance_axis(A, 0)
    with pytest.raises(ValueError):
        Q.mean_variance_axis(X, 2)
