"""``Pipeline`` / ``make_pipeline`` (reference ``sklearn/pipeline.py:31-700``).

Chains transformers and a final estimator; data stays on the device
between steps when the steps take and return tensors (e.g. QPCA ->
KNeighborsClassifier on an MI355X keeps the projected rows in HBM).
Nested parameters use the ``step__param`` convention.
"""

from .base import BaseEstimator, clone


class Pipeline(BaseEstimator):
    def __init__(self, steps, *, memory=None, verbose=False):
        self.steps = steps
        self.memory = memory
        self.verbose = verbose

    # ---------------------------------------------------------------- params
    def get_params(self, deep=True):
        out = {"steps": self.steps, "memory": self.memory, "verbose": self.verbose}
        if not deep:
            return out
        for name, est in self.steps:
            out[name] = est
            if hasattr(est, "get_params"):
                for k, v in est.get_params(deep=True).items():
                    out[f"{name}__{k}"] = v
        return out

    def set_params(self, **params):
        names = dict(self.steps)
        for key in list(params):
            if key in names:
                self.steps = [(n, params.pop(key) if n == key else e) for n, e in self.steps]
                names = dict(self.steps)
        for key in ("steps", "memory", "verbose"):
            if key in params:
                setattr(self, key, params.pop(key))
        nested = {}
        for key, value in params.items():
            name, delim, sub = key.partition("__")
            if not delim or name not in names:
                raise ValueError(f"Invalid parameter {key!r} for estimator {self}.")
            nested.setdefault(name, {})[sub] = value
        for name, sub in nested.items():
            names[name].set_params(**sub)
        return self

    def _validate_steps(self):
        names = [n for n, _ in self.steps]
        if len(set(names)) != len(names):
            raise ValueError(f"Names provided are not unique: {names}")
        for n in names:
            if "__" in n:
                raise ValueError(f"Estimator names must not contain __: got {n!r}")
        for _, t in self.steps[:-1]:
            if t is None or t == "passthrough":
                continue
            if not (hasattr(t, "fit") or hasattr(t, "fit_transform")) or not hasattr(t, "transform"):
                raise TypeError(f"All intermediate steps should be transformers and implement "
                                f"fit and transform or be the string 'passthrough' '{t}'")

    @property
    def named_steps(self):
        return dict(self.steps)

    @property
    def _final_estimator(self):
        est = self.steps[-1][1]
        return None if est == "passthrough" else est

    def __len__(self):
        return len(self.steps)

    def __getitem__(self, ind):
        if isinstance(ind, slice):
            return Pipeline(self.steps[ind], memory=self.memory, verbose=self.verbose)
        if isinstance(ind, str):
            return self.named_steps[ind]
        return self.steps[ind][1]

    # ------------------------------------------------------------------- fit
    def _split_params(self, fit_params):
        per = {n: {} for n, _ in self.steps}
        for k, v in fit_params.items():
            name, delim, sub = k.partition("__")
            if not delim or name not in per:
                raise ValueError(f"Pipeline.fit does not accept the {k} parameter. Use "
                                 "'stepname__parameter' for step parameters.")
            per[name][sub] = v
        return per

    def _fit_transforms(self, X, y, per):
        Xt = X
        for i, (name, t) in enumerate(self.steps[:-1]):
            if t is None or t == "passthrough":
                continue
            if hasattr(t, "fit_transform"):
                Xt = t.fit_transform(Xt, y, **per[name]) if y is not None else \
                    t.fit_transform(Xt, **per[name])
            else:
                Xt = t.fit(Xt, y, **per[name]).transform(Xt)
        return Xt

    def fit(self, X, y=None, **fit_params):
        self._validate_steps()
        per = self._split_params(fit_params)
        Xt = self._fit_transforms(X, y, per)
        final = self._final_estimator
        if final is not None:
            name = self.steps[-1][0]
            if y is None:
                final.fit(Xt, **per[name])
            else:
                final.fit(Xt, y, **per[name])
        return self

    def _transform_prefix(self, X):
        Xt = X
        for _, t in self.steps[:-1]:
            if t is None or t == "passthrough":
                continue
            Xt = t.transform(Xt)
        return Xt

    def fit_transform(self, X, y=None, **fit_params):
        self._validate_steps()
        per = self._split_params(fit_params)
        Xt = self._fit_transforms(X, y, per)
        final = self._final_estimator
        if final is None:
            return Xt
        name = self.steps[-1][0]
        if hasattr(final, "fit_transform"):
            return final.fit_transform(Xt, y, **per[name]) if y is not None else \
                final.fit_transform(Xt, **per[name])
        return final.fit(Xt, y, **per[name]).transform(Xt)

    def fit_predict(self, X, y=None, **fit_params):
        self._validate_steps()
        per = self._split_params(fit_params)
        Xt = self._fit_transforms(X, y, per)
        return self.steps[-1][1].fit_predict(Xt, y, **per[self.steps[-1][0]])

    # -------------------------------------------------------------- predict
    def predict(self, X, **kw):
        return self.steps[-1][1].predict(self._transform_prefix(X), **kw)

    def predict_proba(self, X):
        return self.steps[-1][1].predict_proba(self._transform_prefix(X))

    def decision_function(self, X):
        return self.steps[-1][1].decision_function(self._transform_prefix(X))

    def transform(self, X):
        Xt = self._transform_prefix(X)
        final = self._final_estimator
        return Xt if final is None else final.transform(Xt)

    def inverse_transform(self, X):
        Xt = X
        for _, t in reversed(self.steps):
            if t is None or t == "passthrough":
                continue
            Xt = t.inverse_transform(Xt)
        return Xt

    def score(self, X, y=None, sample_weight=None):
        Xt = self._transform_prefix(X)
        final = self.steps[-1][1]
        kw = {} if sample_weight is None else {"sample_weight": sample_weight}
        return final.score(Xt, y, **kw) if y is not None else final.score(Xt)

    @property
    def classes_(self):
        return self.steps[-1][1].classes_

    @property
    def _estimator_type(self):
        return getattr(self.steps[-1][1], "_estimator_type", None)

    def __repr__(self):
        return f"Pipeline(steps={self.steps!r})"


def _name_estimators(estimators):
    names = [type(e).__name__.lower() if not isinstance(e, str) else e for e in estimators]
    counts = {}
    for n in names:
        counts[n] = counts.get(n, 0) + 1
    seen = {}
    out = []
    for n, e in zip(names, estimators):
        if counts[n] > 1:
            seen[n] = seen.get(n, 0) + 1
            out.append((f"{n}-{seen[n]}", e))
        else:
            out.append((n, e))
    return out


def make_pipeline(*steps, memory=None, verbose=False):
    return Pipeline(_name_estimators(steps), memory=memory, verbose=verbose)


__all__ = ["Pipeline", "make_pipeline", "clone"]


from .utils.metaestimators import _BaseComposition  # noqa: E402


class FeatureUnion(_BaseComposition):
    """Concatenate the outputs of several transformers fitted on the same
    input (reference ``pipeline.py:FeatureUnion``)."""

    def __init__(self, transformer_list, *, n_jobs=None, transformer_weights=None,
                 verbose=False):
        self.transformer_list = transformer_list
        self.n_jobs = n_jobs
        self.transformer_weights = transformer_weights
        self.verbose = verbose

    def get_params(self, deep=True):
        return self._get_params("transformer_list", deep=deep)

    def set_params(self, **kwargs):
        self._set_params("transformer_list", **kwargs)
        return self

    def _iter(self):
        w = self.transformer_weights or {}
        for name, t in self.transformer_list:
            if t == "drop" or t is None:
                continue
            yield name, t, w.get(name)

    def _validate(self):
        names = [n for n, _ in self.transformer_list]
        if len(set(names)) != len(names):
            raise ValueError(f"Names provided are not unique: {names}")
        for _, t in self.transformer_list:
            if t in ("drop", "passthrough") or t is None:
                continue
            if not (hasattr(t, "fit") or hasattr(t, "fit_transform")) or not hasattr(t, "transform"):
                raise TypeError("All estimators should implement fit and transform. '%s' (type %s) "
                                "doesn't" % (t, type(t)))

    @staticmethod
    def _stack(Xs, n):
        import numpy as np
        import scipy.sparse as sp
        if not Xs:
            return np.zeros((n, 0))
        if any(sp.issparse(x) for x in Xs):
            return sp.hstack([sp.csr_matrix(x) for x in Xs]).tocsr()
        return np.hstack([np.asarray(x) for x in Xs])

    def fit(self, X, y=None, **fit_params):
        self.fit_transform(X, y, **fit_params)
        return self

    def fit_transform(self, X, y=None, **fit_params):
        import numpy as np
        self._validate()
        outs, fitted = [], []
        for name, t, w in self._iter():
            if t == "passthrough":
                out, est = np.asarray(X), "passthrough"
            else:
                est = clone(t)
                out = est.fit_transform(X, y, **fit_params) if hasattr(est, "fit_transform") \
                    else est.fit(X, y, **fit_params).transform(X)
            outs.append(out * w if w is not None else out)
            fitted.append((name, est))
        dropped = [(n, t) for n, t in self.transformer_list if t == "drop" or t is None]
        self.transformer_list = fitted + dropped if dropped else fitted
        if hasattr(X, "shape"):
            self.n_features_in_ = X.shape[1]
        return self._stack(outs, len(X) if not hasattr(X, "shape") else X.shape[0])

    def transform(self, X):
        import numpy as np
        outs = []
        for name, t, w in self._iter():
            out = np.asarray(X) if t == "passthrough" else t.transform(X)
            outs.append(out * w if w is not None else out)
        return self._stack(outs, len(X) if not hasattr(X, "shape") else X.shape[0])

    def get_feature_names_out(self, input_features=None):
        import numpy as np
        out = []
        for name, t, _ in self._iter():
            out += [f"{name}__{f}" for f in t.get_feature_names_out(input_features)]
        return np.asarray(out, dtype=object)

    @property
    def named_transformers(self):
        return dict(self.transformer_list)


def make_union(*transformers, n_jobs=None, verbose=False):
    return FeatureUnion(_name_estimators(transformers), n_jobs=n_jobs, verbose=verbose)
