"""Sparse-matrix statistics and in-place edits (reference
``utils/sparsefuncs.py`` + ``utils/sparsefuncs_fast.pyx``).

Everything is vectorised over the CSR/CSC index arrays (``bincount`` on the
compressed axis, ``repeat`` of indptr to expand row ids), so there is no
per-row interpreter loop; NaNs are skipped like the reference's fast
routines."""

import numpy as np
import scipy.sparse as sp

__all__ = ["csr_row_norms", "mean_variance_axis", "incr_mean_variance_axis",
           "inplace_csr_column_scale", "inplace_csr_row_scale", "inplace_column_scale",
           "inplace_row_scale", "inplace_swap_row", "inplace_swap_column", "inplace_swap_row_csr",
           "inplace_swap_row_csc", "min_max_axis", "count_nonzero", "csc_median_axis_0",
           "inplace_csr_row_normalize_l1", "inplace_csr_row_normalize_l2", "assign_rows_csr"]


def _raise_typeerror(X):
    raise TypeError("Expected a CSR or CSC sparse matrix, got %s." % (
        X.format if sp.issparse(X) else type(X)))


def _raise_error_wrong_axis(axis):
    if axis not in (0, 1):
        raise ValueError("Unknown axis value: %d. Use 0 for rows, or 1 for columns" % axis)


def _major_ids(X):
    """Index along the compressed axis of every stored entry."""
    return np.repeat(np.arange(len(X.indptr) - 1), np.diff(X.indptr))


def csr_row_norms(X):
    """Squared L2 norm of every row of a CSR matrix."""
    X = sp.csr_matrix(X)
    return np.bincount(_major_ids(X), X.data.astype(np.float64) ** 2, minlength=X.shape[0])


def _mean_var_minor(X, weights):
    """Mean / variance along the compressed (major) axis, i.e. per minor
    index (columns of CSR, rows of CSC), NaNs ignored."""
    n_major, n_minor = (X.shape[0], X.shape[1]) if X.format == "csr" else (X.shape[1],
                                                                            X.shape[0])
    w = np.ones(n_major) if weights is None else np.asarray(weights, dtype=np.float64)
    data = X.data.astype(np.float64)
    we = w[_major_ids(X)]
    nan = np.isnan(data)
    nan_w = np.bincount(X.indices[nan], we[nan], minlength=n_minor)
    sum_w = w.sum() - nan_w
    d, ix, we = data[~nan], X.indices[~nan], we[~nan]
    s = np.bincount(ix, we * d, minlength=n_minor)
    with np.errstate(divide="ignore", invalid="ignore"):
        mean = s / sum_w
        nz_w = np.bincount(ix, we, minlength=n_minor)
        var = np.bincount(ix, we * (d - mean[ix]) ** 2, minlength=n_minor)
        var += (sum_w - nz_w) * mean ** 2
        var /= sum_w
    return mean, var, sum_w


def mean_variance_axis(X, axis, weights=None, return_sum_weights=False):
    """Per-column (axis=0) or per-row (axis=1) mean and variance."""
    _raise_error_wrong_axis(axis)
    if not sp.issparse(X) or X.format not in ("csr", "csc"):
        _raise_typeerror(X)
    if (X.format == "csr") == (axis == 0):
        out = _mean_var_minor(X, weights)
    else:
        out = _mean_var_minor(X.tocsc() if X.format == "csr" else X.tocsr(), weights)
    return out if return_sum_weights else out[:2]


def incr_mean_variance_axis(X, *, axis, last_mean, last_var, last_n, weights=None):
    """Update running mean / variance / counts with a new sparse batch."""
    _raise_error_wrong_axis(axis)
    if not sp.issparse(X) or X.format not in ("csr", "csc"):
        _raise_typeerror(X)
    if np.size(last_n) == 1:
        last_n = np.full(np.shape(last_mean), last_n, dtype=np.float64)
    if not (np.size(last_mean) == np.size(last_var) == np.size(last_n)):
        raise ValueError("last_mean, last_var, last_n do not have the same shapes.")
    if axis == 1 and np.size(last_mean) != X.shape[0]:
        raise ValueError("If axis=1, then last_mean, last_n, last_var should be of size "
                         "n_samples {} (Got {}).".format(X.shape[0], np.size(last_mean)))
    if axis == 0 and np.size(last_mean) != X.shape[1]:
        raise ValueError("If axis=0, then last_mean, last_n, last_var should be of size "
                         "n_features {} (Got {}).".format(X.shape[1], np.size(last_mean)))
    X = X.T if axis == 1 else X
    new_mean, new_var, new_n = mean_variance_axis(X, 0, weights=weights,
                                                  return_sum_weights=True)
    last_mean = np.asarray(last_mean, dtype=np.float64)
    last_var = np.asarray(last_var, dtype=np.float64)
    last_n = np.asarray(last_n, dtype=np.float64)
    upd_n = last_n + new_n
    with np.errstate(divide="ignore", invalid="ignore"):
        last_sum = last_mean * last_n
        new_sum = new_mean * new_n
        upd_mean = (last_sum + new_sum) / upd_n
        ratio = last_n / new_n
        unnorm = last_var * last_n + new_var * new_n + \
            ratio / upd_n * (last_sum / ratio - new_sum) ** 2
    zero_last = last_n == 0
    upd_mean[zero_last] = new_mean[zero_last]
    unnorm[zero_last] = (new_var * new_n)[zero_last]
    zero_new = new_n == 0
    upd_mean[zero_new] = last_mean[zero_new]
    unnorm[zero_new] = (last_var * last_n)[zero_new]
    with np.errstate(divide="ignore", invalid="ignore"):
        upd_var = unnorm / upd_n
    return upd_mean, upd_var, upd_n


def inplace_csr_column_scale(X, scale):
    X.data *= np.asarray(scale).take(X.indices, mode="clip")


def inplace_csr_row_scale(X, scale):
    X.data *= np.repeat(np.asarray(scale), np.diff(X.indptr))


def inplace_column_scale(X, scale):
    if X.format == "csc":
        inplace_csr_row_scale(X.T, scale)
    elif X.format == "csr":
        inplace_csr_column_scale(X, scale)
    else:
        _raise_typeerror(X)


def inplace_row_scale(X, scale):
    if X.format == "csc":
        inplace_csr_column_scale(X.T, scale)
    elif X.format == "csr":
        inplace_csr_row_scale(X, scale)
    else:
        _raise_typeerror(X)


def inplace_swap_row_csc(X, m, n):
    if m < 0:
        m += X.shape[0]
    if n < 0:
        n += X.shape[0]
    mm, nn = X.indices == m, X.indices == n
    X.indices[mm] = n
    X.indices[nn] = m


def inplace_swap_row_csr(X, m, n):
    """Swap rows m and n of a CSR matrix by splicing their index / data
    segments (indptr shifted between them)."""
    if m < 0:
        m += X.shape[0]
    if n < 0:
        n += X.shape[0]
    if m == n:
        return
    if m > n:
        m, n = n, m
    p = X.indptr
    a, b, c, d = p[m], p[m + 1], p[n], p[n + 1]
    for name in ("indices", "data"):
        arr = getattr(X, name)
        arr[a:d] = np.concatenate([arr[c:d], arr[b:c], arr[a:b]])
    shift = (d - c) - (b - a)
    p[m + 1:n + 1] += shift


def _swap_rows_generic(X, m, n):
    Y = X.tolil()
    Y[[m, n]] = Y[[n, m]]
    return Y.asformat(X.format)


def inplace_swap_row(X, m, n):
    if X.format == "csc":
        inplace_swap_row_csc(X, m, n)
    elif X.format == "csr":
        inplace_swap_row_csr(X, m, n)
    else:
        _raise_typeerror(X)


def inplace_swap_column(X, m, n):
    if m < 0:
        m += X.shape[1]
    if n < 0:
        n += X.shape[1]
    if X.format == "csc":
        Y = _swap_rows_generic(X.T.tocsr(), m, n).T.tocsc()
        X.data, X.indices, X.indptr = Y.data, Y.indices, Y.indptr
    elif X.format == "csr":
        inplace_swap_row_csc(X, m, n)
    else:
        _raise_typeerror(X)


def _minor_reduce(X, ufunc):
    major = np.flatnonzero(np.diff(X.indptr))
    return major, ufunc.reduceat(X.data, X.indptr[major])


def _min_or_max_axis(X, axis, min_or_max):
    N = X.shape[axis]
    if N == 0:
        raise ValueError("zero-size array to reduction operation")
    M = X.shape[1 - axis]
    mat = X.tocsc() if axis == 0 else X.tocsr()
    mat.sum_duplicates()
    major, value = _minor_reduce(mat, min_or_max)
    not_full = np.diff(mat.indptr)[major] < N
    value[not_full] = min_or_max(value[not_full], 0)
    mask = value != 0
    major = np.compress(mask, major)
    value = np.compress(mask, value)
    res = np.zeros(M, dtype=X.dtype)
    res[major] = value
    return res


def min_max_axis(X, axis, ignore_nan=False):
    """Column-wise (axis=0) or row-wise (axis=1) minimum and maximum."""
    if not sp.issparse(X) or X.format not in ("csr", "csc"):
        _raise_typeerror(X)
    _raise_error_wrong_axis(axis)
    mn, mx = (np.fmin, np.fmax) if ignore_nan else (np.minimum, np.maximum)
    return _min_or_max_axis(X, axis, mn), _min_or_max_axis(X, axis, mx)


def count_nonzero(X, axis=None, sample_weight=None):
    """Stored-entry count, optionally weighted by row."""
    if axis == -1:
        axis = 1
    elif axis == -2:
        axis = 0
    elif X.format != "csr":
        raise TypeError("Expected CSR sparse format, got {0}".format(X.format))
    if axis is None:
        if sample_weight is None:
            return X.nnz
        return np.dot(np.diff(X.indptr), sample_weight)
    if axis == 1:
        out = np.diff(X.indptr)
        return out if sample_weight is None else out * sample_weight
    if axis == 0:
        w = None if sample_weight is None else np.repeat(sample_weight, np.diff(X.indptr))
        return np.bincount(X.indices, minlength=X.shape[1], weights=w)
    raise ValueError("Unsupported axis: {0}".format(axis))


def _get_median(data, n_zeros):
    n = len(data) + n_zeros
    if not n:
        return np.nan
    neg = np.count_nonzero(data < 0)
    mid, odd = divmod(n, 2)
    data = np.sort(data)
    if odd:
        return _get_elem_at_rank(mid, data, neg, n_zeros)
    return (_get_elem_at_rank(mid - 1, data, neg, n_zeros)
            + _get_elem_at_rank(mid, data, neg, n_zeros)) / 2.0


def _get_elem_at_rank(rank, data, n_negative, n_zeros):
    if rank < n_negative:
        return data[rank]
    if rank - n_negative < n_zeros:
        return 0
    return data[rank - n_zeros]


def csc_median_axis_0(X):
    """Median of every column of a CSC matrix (implicit zeros included)."""
    if not sp.isspmatrix_csc(X):
        raise TypeError("Expected matrix of CSC format, got %s" % X.format)
    n, d = X.shape
    med = np.zeros(d)
    for j, (a, b) in enumerate(zip(X.indptr[:-1], X.indptr[1:])):
        med[j] = _get_median(np.copy(X.data[a:b]), n - (b - a))
    return med


def inplace_csr_row_normalize_l1(X):
    s = np.bincount(_major_ids(X), np.abs(X.data), minlength=X.shape[0])
    s[s == 0] = 1.0
    X.data /= np.repeat(s, np.diff(X.indptr))


def inplace_csr_row_normalize_l2(X):
    s = np.sqrt(np.bincount(_major_ids(X), X.data ** 2, minlength=X.shape[0]))
    s[s == 0] = 1.0
    X.data /= np.repeat(s, np.diff(X.indptr))


def assign_rows_csr(X, X_rows, out_rows, out):
    """Densify rows ``X_rows`` of CSR ``X`` into ``out[out_rows]``."""
    out[out_rows] = 0
    sub = X[np.asarray(X_rows)]
    r = _major_ids(sub)
    np.add.at(out, (np.asarray(out_rows)[r], sub.indices), sub.data)
