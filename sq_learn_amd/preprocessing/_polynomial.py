"""Polynomial feature expansion (reference ``preprocessing/_data.py:
PolynomialFeatures`` and ``_csr_polynomial_expansion.pyx``).

Dense inputs (numpy or device tensors) are expanded on the data's device:
one gather + product per degree over precomputed monomial index tables, in
row chunks.  CSR inputs of degree <= 3 go through the host-native
``sqh_csr_poly`` kernel (never densified); other sparse inputs are
converted to CSR first."""

from itertools import chain, combinations, combinations_with_replacement

import numpy as np
import scipy.sparse as sp
import torch

from ..base import BaseEstimator, TransformerMixin
from ..ops import _host
from ..utils.pairwise import get_chunk_n_rows
from ..utils.validation import check_array, check_is_fitted


def _combinations(n_features, degree, interaction_only, include_bias):
    comb = combinations if interaction_only else combinations_with_replacement
    start = int(not include_bias)
    return chain.from_iterable(comb(range(n_features), i) for i in range(start, degree + 1))


def _csr_degree(X, F, d, interaction_only):
    data = np.ascontiguousarray(X.data, dtype=np.float64)
    ind = np.ascontiguousarray(X.indices, dtype=np.int32)
    ptr = np.ascontiguousarray(X.indptr, dtype=np.int64)
    n = X.shape[0]
    L = _host.lib()
    out_ptr = np.zeros(n + 1, dtype=np.int64)
    L.sqh_csr_poly(_host.ptr(data), _host.ptr(ind), _host.ptr(ptr), n, F, d,
                   int(interaction_only), _host.ptr(out_ptr), None, None)
    nnz = int(out_ptr[-1])
    oi = np.empty(max(nnz, 1), dtype=np.int64)
    od = np.empty(max(nnz, 1), dtype=np.float64)
    L.sqh_csr_poly(_host.ptr(data), _host.ptr(ind), _host.ptr(ptr), n, F, d,
                   int(interaction_only), _host.ptr(out_ptr), _host.ptr(oi), _host.ptr(od))
    comb = combinations if interaction_only else combinations_with_replacement
    n_cols = sum(1 for _ in comb(range(F), d))
    return sp.csr_matrix((od[:nnz], oi[:nnz], out_ptr), shape=(n, n_cols))


class PolynomialFeatures(TransformerMixin, BaseEstimator):
    """Monomials of the input features up to ``degree`` (optionally only
    interactions, optionally with the bias column)."""

    def __init__(self, degree=2, *, interaction_only=False, include_bias=True, order="C"):
        self.degree = degree
        self.interaction_only = interaction_only
        self.include_bias = include_bias
        self.order = order

    @property
    def powers_(self):
        check_is_fitted(self)
        combos = _combinations(self.n_features_in_, self.degree, self.interaction_only,
                               self.include_bias)
        return np.vstack([np.bincount(c, minlength=self.n_features_in_) for c in combos])

    def get_feature_names_out(self, input_features=None):
        powers = self.powers_
        if input_features is None:
            input_features = ["x%d" % i for i in range(powers.shape[1])]
        names = []
        for row in powers:
            inds = np.where(row)[0]
            if len(inds):
                names.append(" ".join("%s^%d" % (input_features[i], e) if e != 1
                                      else input_features[i] for i, e in zip(inds, row[inds])))
            else:
                names.append("1")
        return np.asarray(names, dtype=object)

    def get_feature_names(self, input_features=None):
        return list(self.get_feature_names_out(input_features))

    def fit(self, X, y=None):
        if isinstance(X, torch.Tensor):
            n_features = X.shape[1]
        elif sp.issparse(X):
            n_features = X.shape[1]
        else:
            n_features = check_array(X).shape[1]
        self.n_features_in_ = n_features
        self.n_input_features_ = n_features
        self.n_output_features_ = sum(1 for _ in _combinations(
            n_features, self.degree, self.interaction_only, self.include_bias))
        return self

    def transform(self, X):
        check_is_fitted(self)
        F = self.n_features_in_
        if sp.issparse(X):
            if X.shape[1] != F:
                raise ValueError("X shape does not match training shape")
            if self.degree < 4:
                Xc = sp.csr_matrix(X, dtype=np.float64)
                Xc.sort_indices()
                blocks = []
                if self.include_bias:
                    blocks.append(sp.csr_matrix(np.ones((Xc.shape[0], 1))))
                for d in range(1, self.degree + 1):
                    blocks.append(_csr_degree(Xc, F, d, self.interaction_only))
                return sp.hstack(blocks, format="csr").astype(X.dtype)
            # higher degrees: column products on CSC (stays sparse)
            Xc = sp.csc_matrix(X)
            cols = []
            for c in _combinations(F, self.degree, self.interaction_only, self.include_bias):
                col = sp.csc_matrix(np.ones((Xc.shape[0], 1)), dtype=Xc.dtype)
                for j in c:
                    col = col.multiply(Xc[:, j])
                cols.append(sp.csc_matrix(col))
            return sp.hstack(cols, format="csr")
        numpy_in = not isinstance(X, torch.Tensor)
        Xt = torch.as_tensor(check_array(X, dtype=[np.float64, np.float32])) if numpy_in else X
        if not Xt.is_floating_point():
            Xt = Xt.double()
        if Xt.shape[1] != F:
            raise ValueError("X shape does not match training shape")
        n = Xt.shape[0]
        out = torch.empty((n, self.n_output_features_), dtype=Xt.dtype, device=Xt.device)
        col = 0
        if self.include_bias:
            out[:, 0] = 1
            col = 1
        comb = combinations if self.interaction_only else combinations_with_replacement
        for d in range(1, self.degree + 1):
            idx = list(comb(range(F), d))
            if not idx:
                continue
            it = torch.as_tensor(idx, dtype=torch.int64, device=Xt.device)
            rows = get_chunk_n_rows(len(idx) * d * Xt.element_size())
            for s in range(0, n, rows):
                out[s:s + rows, col:col + len(idx)] = Xt[s:s + rows][:, it].prod(-1)
            col += len(idx)
        if numpy_in:
            res = out.cpu().numpy()
            return np.asfortranarray(res) if self.order == "F" else res
        return out


class SplineTransformer(TransformerMixin, BaseEstimator):
    """Univariate B-spline bases per feature (reference
    ``preprocessing/_polynomial.py:337``).

    Each column gets ``n_knots + degree - 1`` basis functions (``n_knots -
    1`` when periodic) on ``n_knots`` base knots - uniform over the column's
    range, at its quantiles, or given as an array - extended by ``degree``
    equidistant knots on each side (periodic: wrapped by one period).
    ``extrapolation`` beyond the base interval: 'constant' (the boundary
    values of the basis), 'linear' (first-order continuation of the boundary
    splines), 'continue' (the polynomial pieces continued), 'periodic' or
    'error'.  All bases of a column are evaluated at once through one
    ``BSpline`` with identity coefficients."""

    def __init__(self, n_knots=5, degree=3, *, knots="uniform", extrapolation="constant",
                 include_bias=True, order="C"):
        self.n_knots = n_knots
        self.degree = degree
        self.knots = knots
        self.extrapolation = extrapolation
        self.include_bias = include_bias
        self.order = order

    @staticmethod
    def _base_knots(X, n_knots, knots):
        if knots == "quantile":
            return np.percentile(X, 100.0 * np.linspace(0.0, 1.0, n_knots), axis=0)
        lo, hi = X.min(axis=0), X.max(axis=0)
        return lo[None, :] + (hi - lo)[None, :] * np.linspace(0.0, 1.0, n_knots)[:, None]

    def fit(self, X, y=None, sample_weight=None):
        import numbers
        from scipy.interpolate import BSpline
        X = check_array(X, dtype=np.float64)
        if X.shape[0] < 2:
            raise ValueError(f"Found array with {X.shape[0]} sample(s) while a minimum of 2 is "
                             "required.")
        n, nf = X.shape
        self.n_features_in_ = nf
        if not (isinstance(self.degree, numbers.Integral) and self.degree >= 0):
            raise ValueError("degree must be a non-negative integer.")
        deg = int(self.degree)
        if isinstance(self.knots, str):
            if self.knots not in ("uniform", "quantile"):
                raise ValueError("knots must be 'uniform', 'quantile' or an array-like.")
            if not (isinstance(self.n_knots, numbers.Integral) and self.n_knots >= 2):
                raise ValueError("n_knots must be a positive integer >= 2.")
            base = self._base_knots(X, int(self.n_knots), self.knots)
        else:
            base = check_array(self.knots, dtype=np.float64)
            if base.shape[0] < 2:
                raise ValueError("Number of knots, knots.shape[0], must be >= 2.")
            if base.shape[1] != nf:
                raise ValueError("knots.shape[1] == n_features is violated.")
            if not np.all(np.diff(base, axis=0) > 0):
                raise ValueError("knots must be sorted without duplicates.")
        if self.extrapolation not in ("error", "constant", "linear", "continue", "periodic"):
            raise ValueError("extrapolation must be one of 'error', 'constant', 'linear', "
                             "'continue' or 'periodic'.")
        if not isinstance(self.include_bias, (bool, np.bool_)):
            raise ValueError("include_bias must be bool.")
        nk = base.shape[0]
        periodic = self.extrapolation == "periodic"
        if periodic and nk <= deg:
            raise ValueError(f"Periodic splines require degree < n_knots. Got n_knots={nk} and "
                             f"degree={deg}.")
        n_spl = nk - 1 if periodic else nk + deg - 1
        if periodic:
            period = base[-1] - base[0]
            full = np.concatenate([base[nk - 1 - deg:nk - 1] - period, base,
                                   base[1:deg + 1] + period])
        else:
            step_lo = base[1] - base[0]
            step_hi = base[-1] - base[-2]
            steps = np.arange(1, deg + 1, dtype=np.float64)[:, None]
            full = np.concatenate([base[0] - steps[::-1] * step_lo, base,
                                   base[-1] + steps * step_hi])
        coef = np.eye(n_spl)
        if periodic:   # the first degree bases wrap around
            coef = np.concatenate([coef, coef[:deg]])
        ext = self.extrapolation in ("periodic", "continue")
        self.bsplines_ = [BSpline.construct_fast(np.ascontiguousarray(full[:, j]), coef, deg,
                                                 extrapolate=ext) for j in range(nf)]
        self.n_features_out_ = nf * (n_spl - (0 if self.include_bias else 1))
        return self

    def transform(self, X):
        check_is_fitted(self, "bsplines_")
        X = check_array(X)
        if X.shape[1] != self.n_features_in_:
            raise ValueError(f"X has {X.shape[1]} features, but SplineTransformer is expecting "
                             f"{self.n_features_in_} features as input.")
        dtype = X.dtype if X.dtype in (np.float32, np.float64) else np.float64
        X = X.astype(np.float64, copy=False)
        deg = int(self.degree)
        n_spl = self.bsplines_[0].c.shape[1]
        out = np.zeros((X.shape[0], X.shape[1] * n_spl), dtype=dtype, order=self.order)
        for j, spl in enumerate(self.bsplines_):
            x = X[:, j]
            blk = slice(j * n_spl, (j + 1) * n_spl)
            lo_t, hi_t = spl.t[deg], spl.t[-deg - 1]
            if self.extrapolation == "periodic":
                m = spl.t.size - deg - 1
                span = spl.t[m] - spl.t[deg]
                out[:, blk] = spl(spl.t[deg] + np.mod(x - spl.t[deg], span))
                continue
            if self.extrapolation in ("continue", "error"):
                vals = spl(x)
                if self.extrapolation == "error" and np.isnan(vals).any():
                    raise ValueError("X contains values beyond the limits of the knots.")
                out[:, blk] = vals
                continue
            inside = (x >= lo_t) & (x <= hi_t)
            out[inside, blk] = spl(x[inside])
            below, above = x < lo_t, x > hi_t
            f_lo, f_hi = spl(lo_t), spl(hi_t)
            if self.extrapolation == "constant":
                # only the boundary bases are nonzero at the interval ends
                if below.any():
                    out[below, j * n_spl:j * n_spl + deg] = f_lo[:deg]
                if above.any():
                    out[above, (j + 1) * n_spl - deg:(j + 1) * n_spl] = f_hi[n_spl - deg:]
            else:   # linear continuation of the boundary bases
                d_lo, d_hi = spl(lo_t, nu=1), spl(hi_t, nu=1)
                nb = deg + 1 if deg <= 1 else deg
                for b in range(nb):
                    if below.any():
                        out[below, j * n_spl + b] = f_lo[b] + (x[below] - lo_t) * d_lo[b]
                    if above.any():
                        c = n_spl - 1 - b
                        out[above, j * n_spl + c] = f_hi[c] + (x[above] - hi_t) * d_hi[c]
        if self.include_bias:
            return out
        keep = [c for c in range(out.shape[1]) if (c + 1) % n_spl != 0]
        return out[:, keep]

    def get_feature_names_out(self, input_features=None):
        n_spl = self.bsplines_[0].c.shape[1]
        if input_features is None:
            input_features = [f"x{i}" for i in range(self.n_features_in_)]
        return np.asarray([f"{input_features[i]}_sp_{j}" for i in range(self.n_features_in_)
                           for j in range(n_spl - 1 + int(self.include_bias))], dtype=object)

    def get_feature_names(self, input_features=None):
        return list(self.get_feature_names_out(input_features))
