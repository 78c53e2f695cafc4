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
