"""Feature hashing (reference
``feature_extraction/_hash.py`` + ``_hashing_fast.pyx``).

Token collection is Python (inputs are Python mappings / iterables); the
hashing, index folding and sign flip run in the host-native kernel
``sqh_hash_features`` (``csrc/host/hashing.cpp``)."""

import numbers

import numpy as np
import scipy.sparse as sp

from ..base import BaseEstimator, TransformerMixin
from ..ops import _host


def _hashing_transform(raw_X, n_features, dtype, alternate_sign=True, seed=0):
    names, values, indptr = [], [], [0]
    for x in raw_X:
        for f, v in x:
            if isinstance(v, str):
                f = f"{f}={v}"
                v = 1
            if v == 0:
                continue
            if isinstance(f, str):
                f = f.encode("utf-8")
            elif not isinstance(f, bytes):
                raise TypeError("feature names must be strings")
            names.append(f)
            values.append(float(v))
        indptr.append(len(names))
    n = len(names)
    offsets = np.zeros(n + 1, dtype=np.int64)
    np.cumsum([len(b) for b in names], out=offsets[1:])
    buf = np.frombuffer(b"".join(names) or b"\0", dtype=np.uint8).copy()
    vals_in = np.asarray(values, dtype=np.float64) if n else np.zeros(1)
    cols = np.empty(max(n, 1), dtype=np.int32)
    vals = np.empty(max(n, 1), dtype=np.float64)
    _host.lib().sqh_hash_features(_host.ptr(buf), _host.ptr(offsets), _host.ptr(vals_in), n,
                                  int(n_features), int(bool(alternate_sign)),
                                  int(seed) & 0xFFFFFFFF, _host.ptr(cols), _host.ptr(vals))
    indptr = np.asarray(indptr, dtype=np.int64)
    if indptr[-1] <= np.iinfo(np.int32).max:
        indptr = indptr.astype(np.int32)
    return cols[:n], indptr, vals[:n].astype(dtype)


class FeatureHasher(TransformerMixin, BaseEstimator):
    """Implements feature hashing, aka the hashing trick (reference
    ``FeatureHasher``: n_features, input_type 'dict' | 'pair' | 'string',
    dtype, alternate_sign)."""

    def __init__(self, n_features=(2 ** 20), *, input_type="dict", dtype=np.float64,
                 alternate_sign=True):
        self.dtype = dtype
        self.input_type = input_type
        self.n_features = n_features
        self.alternate_sign = alternate_sign

    @staticmethod
    def _validate_params(n_features, input_type):
        if not isinstance(n_features, numbers.Integral):
            raise TypeError("n_features must be integral, got %r (%s)."
                            % (n_features, type(n_features)))
        elif n_features < 1 or n_features >= np.iinfo(np.int32).max + 1:
            raise ValueError("Invalid number of features (%d)." % n_features)
        if input_type not in ("dict", "pair", "string"):
            raise ValueError("input_type must be 'dict', 'pair' or 'string', got %r."
                             % input_type)

    def fit(self, X=None, y=None):
        self._validate_params(self.n_features, self.input_type)
        return self

    def transform(self, raw_X):
        """raw_X: iterable over iterables of (name, value) pairs, mappings, or
        strings (by input_type) -> scipy.sparse.csr_matrix (n_samples, n_features)."""
        self._validate_params(self.n_features, self.input_type)
        raw_X = iter(raw_X)
        if self.input_type == "dict":
            raw_X = (d.items() for d in raw_X)
        elif self.input_type == "string":
            raw_X = (((f, 1) for f in x) for x in raw_X)
        indices, indptr, values = _hashing_transform(raw_X, self.n_features, self.dtype,
                                                     self.alternate_sign)
        n_samples = indptr.shape[0] - 1
        if n_samples == 0:
            raise ValueError("Cannot vectorize empty sequence.")
        X = sp.csr_matrix((values, indices, indptr), dtype=self.dtype,
                          shape=(n_samples, self.n_features))
        X.sum_duplicates()
        return X

    def _more_tags(self):
        return {"X_types": [self.input_type]}
