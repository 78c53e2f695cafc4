"""Feature-dict vectorisation (reference ``feature_extraction/_dict_vectorizer.py``):
string values one-hot encode as ``name<sep>value``, numbers pass through,
iterables of strings expand to several one-hot columns."""

from array import array
from collections.abc import Iterable, Mapping
from numbers import Number
from operator import itemgetter

import numpy as np
import scipy.sparse as sp

from ..base import BaseEstimator, TransformerMixin


class DictVectorizer(TransformerMixin, BaseEstimator):
    def __init__(self, *, dtype=np.float64, separator="=", sparse=True, sort=True):
        self.dtype = dtype
        self.separator = separator
        self.sparse = sparse
        self.sort = sort

    def _name(self, f, v):
        return "%s%s%s" % (f, self.separator, v)

    def _items(self, f, v):
        """Yield (column name, value) pairs of one mapping entry."""
        if isinstance(v, str):
            yield self._name(f, v), 1
        elif isinstance(v, Number) or v is None:
            yield f, v
        elif isinstance(v, Mapping):
            raise TypeError(f"Unsupported value type {type(v)} for {f}: {v}.\n"
                            "Mapping objects are not supported.")
        elif isinstance(v, Iterable):
            for vv in v:
                if not isinstance(vv, str):
                    raise TypeError(f"Unsupported type {type(vv)} in iterable value. "
                                    "Only iterables of string are supported.")
                yield self._name(f, vv), 1
        else:
            raise TypeError(f"Unsupported value Type {type(v)} for {f}: {v}.\n"
                            f"{type(v)} objects are not supported.")

    def fit(self, X, y=None):
        names, vocab = [], {}
        for x in X:
            for f, v in x.items():
                for name, _ in self._items(f, v):
                    if name not in vocab:
                        vocab[name] = len(names)
                        names.append(name)
        if self.sort:
            names.sort()
            vocab = {f: i for i, f in enumerate(names)}
        self.feature_names_ = names
        self.vocabulary_ = vocab
        return self

    def _transform(self, X, fitting):
        if fitting:
            names, vocab = [], {}
        else:
            names, vocab = self.feature_names_, self.vocabulary_
        X = [X] if isinstance(X, Mapping) else X
        idx, vals, indptr = array("i"), [], [0]
        for x in X:
            for f, v in x.items():
                for name, val in self._items(f, v):
                    if fitting and name not in vocab:
                        vocab[name] = len(names)
                        names.append(name)
                    if name in vocab:
                        idx.append(vocab[name])
                        vals.append(self.dtype(val))
            indptr.append(len(idx))
        if len(indptr) == 1:
            raise ValueError("Sample sequence X is empty.")
        M = sp.csr_matrix((vals, np.frombuffer(idx, dtype=np.intc), indptr),
                          shape=(len(indptr) - 1, len(vocab)), dtype=self.dtype)
        if fitting and self.sort:
            names.sort()
            remap = np.empty(len(names), dtype=np.int32)
            for new, f in enumerate(names):
                remap[new] = vocab[f]
                vocab[f] = new
            M = M[:, remap]
        if self.sparse:
            M.sort_indices()
        else:
            M = M.toarray()
        if fitting:
            self.feature_names_ = names
            self.vocabulary_ = vocab
        return M

    def fit_transform(self, X, y=None):
        return self._transform(X, fitting=True)

    def transform(self, X):
        return self._transform(X, fitting=False)

    def inverse_transform(self, X, dict_type=dict):
        names = self.feature_names_
        if sp.issparse(X):
            X = sp.csr_matrix(X)
            dicts = [dict_type() for _ in range(X.shape[0])]
            for i, j in zip(*X.nonzero()):
                dicts[i][names[j]] = X[i, j]
            return dicts
        X = np.atleast_2d(np.asarray(X))
        dicts = [dict_type() for _ in range(X.shape[0])]
        for i, d in enumerate(dicts):
            for j, v in enumerate(X[i, :]):
                if v != 0:
                    d[names[j]] = X[i, j]
        return dicts

    def get_feature_names_out(self, input_features=None):
        if any(not isinstance(n, str) for n in self.feature_names_):
            return np.asarray([str(n) for n in self.feature_names_], dtype=object)
        return np.asarray(self.feature_names_, dtype=object)

    def get_feature_names(self):
        return list(self.get_feature_names_out())

    def restrict(self, support, indices=False):
        if not indices:
            support = np.where(support)[0]
        vocab = {}
        for i in support:
            vocab[self.feature_names_[i]] = len(vocab)
        self.vocabulary_ = vocab
        self.feature_names_ = [f for f, _ in sorted(vocab.items(), key=itemgetter(1))]
        return self

    def _more_tags(self):
        return {"X_types": ["dict"]}
