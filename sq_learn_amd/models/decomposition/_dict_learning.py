"""Sparse coding and dictionary learning (reference
``decomposition/_dict_learning.py`` and ``_sparse_pca.py``, 1.0 semantics).

Design:

* ``sparse_encode`` solves one sparse problem per sample, all sharing the
  dictionary Gram matrix.  The ``lasso_cd`` path runs every sample's
  coordinate descent *together* on the device: one coordinate step updates
  that coordinate for all right-hand sides at once (a rank-1 update of the
  (n_samples, n_components) ``H = code @ Gram`` panel), each sample keeping
  its own duality-gap stopping test (reference
  ``linear_model/_cd_fast.pyx`` ``enet_coordinate_descent_gram``), so the
  codes equal the per-sample Lasso fits.  LARS / OMP reuse the Gram-domain
  solvers of ``linear_model``; thresholding is one device expression.
* The block-coordinate dictionary update (reference ``_update_dict``
  :358) keeps the residual ``R = Y - D C`` resident on the device and
  applies the per-atom rank-1 corrections there.
"""

import itertools

import numpy as np
import torch
from scipy import linalg

from ...base import BaseEstimator, TransformerMixin
from ...runtime.device import resolve_device
from ...utils.extmath import randomized_svd, row_norms, svd_flip
from ...utils.validation import check_is_fitted, check_random_state

__all__ = ["DictionaryLearning", "MiniBatchDictionaryLearning", "SparseCoder", "SparsePCA",
           "MiniBatchSparsePCA", "dict_learning", "dict_learning_online", "sparse_encode"]


def _np(X):
    if hasattr(X, "detach"):
        X = X.detach().cpu().numpy()
    return np.asarray(X, dtype=np.float64)


def _check_positive_coding(method, positive):
    if positive and method in ("omp", "lars"):
        raise ValueError("Positive constraint not supported for '{}' coding method."
                         .format(method))


def _lasso_gram_batched(G, Xy, y_norm2, alpha, init, max_iter, tol, positive, dev):
    """Coordinate descent for ``min_w 0.5||x - D^T w||^2 + alpha ||w||_1``
    for every column of ``Xy`` at once (alpha already scaled by n_features).
    Returns the (n_targets, n_components) codes."""
    k, T = Xy.shape
    Q = torch.as_tensor(G, dtype=torch.float64, device=dev)
    q = torch.as_tensor(Xy.T, dtype=torch.float64, device=dev).contiguous()   # (T, k)
    W = (torch.zeros((T, k), dtype=torch.float64, device=dev) if init is None else
         torch.as_tensor(np.array(init, dtype=np.float64).reshape(T, k), device=dev).clone())
    yn = torch.as_tensor(y_norm2, dtype=torch.float64, device=dev)
    H = W @ Q
    diag = torch.diagonal(Q)
    # zero-diagonal atoms are skipped: decided once on the host (one sync)
    # rather than per coordinate and sweep
    active_j = [j for j, v in enumerate(diag.cpu().tolist()) if v != 0.0]
    live = torch.ones(T, dtype=torch.bool, device=dev)
    tol_s = tol * yn
    d_w_tol = tol
    for it in range(max_iter):
        w_max = torch.zeros(T, dtype=torch.float64, device=dev)
        d_w_max = torch.zeros_like(w_max)
        for j in active_j:
            wj = W[:, j].clone()
            H -= wj[:, None] * Q[j][None, :]
            t = q[:, j] - H[:, j]
            nw = torch.sign(t) * torch.clamp(t.abs() - alpha, min=0) / diag[j]
            if positive:
                nw = torch.where(t < 0, torch.zeros_like(nw), nw)
            nw = torch.where(live, nw, wj)
            W[:, j] = nw
            H += nw[:, None] * Q[j][None, :]
            d_w_max = torch.maximum(d_w_max, (nw - wj).abs())
            w_max = torch.maximum(w_max, nw.abs())
        check = (w_max == 0) | (d_w_max / w_max < d_w_tol) | torch.tensor(
            it == max_iter - 1, device=dev)
        check &= live
        # duality-gap test evaluated on the device for every row (masked by
        # check): one host sync per sweep (live.any() below)
        if True:
            qw = (W * q).sum(1)
            XtA = q - H
            dn = XtA.max(1).values if positive else XtA.abs().max(1).values
            R2 = yn + (W * H).sum(1) - 2.0 * qw
            const = torch.where(dn > alpha, alpha / dn, torch.ones_like(dn))
            gap = torch.where(dn > alpha, 0.5 * (R2 + R2 * const ** 2), R2)
            gap = gap + alpha * W.abs().sum(1) - const * yn + const * qw
            live &= ~(check & (gap < tol_s))
        if not bool(live.any()):
            break
    return W.cpu().numpy()


def _sparse_encode(X, dictionary, gram, cov=None, algorithm="lasso_lars", regularization=None,
                   copy_cov=True, init=None, max_iter=1000, positive=False):
    from ..linear_model._lm_extra import _lars_gram, orthogonal_mp_gram
    n, d = X.shape
    k = dictionary.shape[0]
    if dictionary.shape[1] != d:
        raise ValueError("Dictionary and X have different numbers of features:"
                         "dictionary.shape: {} X.shape{}".format(dictionary.shape, X.shape))
    if cov is None and algorithm != "lasso_cd":
        cov = dictionary @ X.T
    _check_positive_coding(algorithm, positive)
    eps = np.finfo(np.float64).eps
    if algorithm == "lasso_lars":
        a = float(regularization) / d
        code = np.empty((n, k))
        for i in range(n):
            code[i] = _lars_gram(gram, cov[:, i], d, max_iter, a, "lasso", eps, positive,
                                 False)[2]
    elif algorithm == "lasso_cd":
        a = float(regularization) / d
        Xy = dictionary @ X.T
        code = _lasso_gram_batched(gram, Xy, (X * X).sum(1), a * d, init, max_iter, 1e-4,
                                   positive, resolve_device(None))
    elif algorithm == "lars":
        code = np.empty((n, k))
        for i in range(n):
            code[i] = _lars_gram(gram, cov[:, i], d, int(regularization), 0.0, "lar", eps,
                                 False, False)[2]
    elif algorithm == "threshold":
        code = ((np.sign(cov) * np.maximum(np.abs(cov) - regularization, 0)).T)
        if positive:
            np.clip(code, 0, None, out=code)
    elif algorithm == "omp":
        code = np.asarray(orthogonal_mp_gram(
            Gram=gram, Xy=cov, n_nonzero_coefs=int(regularization), tol=None,
            norms_squared=row_norms(X, squared=True), copy_Xy=copy_cov)).T
    else:
        raise ValueError('Sparse coding method must be "lasso_lars" "lasso_cd", "lasso", '
                         '"threshold" or "omp", got %s.' % algorithm)
    return code.reshape(n, k)


def sparse_encode(X, dictionary, *, gram=None, cov=None, algorithm="lasso_lars",
                  n_nonzero_coefs=None, alpha=None, copy_cov=True, init=None, max_iter=1000,
                  n_jobs=None, check_input=True, verbose=0, positive=False):
    """Sparse code of each row of X against the rows of ``dictionary``."""
    X = _np(X)
    dictionary = _np(dictionary)
    if X.ndim != 2 or dictionary.ndim != 2:
        raise ValueError("Expected 2D arrays")
    n, d = X.shape
    k = dictionary.shape[0]
    if gram is None and algorithm != "threshold":
        gram = dictionary @ dictionary.T
    if cov is None and algorithm != "lasso_cd":
        copy_cov = False
        cov = dictionary @ X.T
    if algorithm in ("lars", "omp"):
        reg = n_nonzero_coefs
        if reg is None:
            reg = min(max(d / 10, 1), k)
    else:
        reg = 1.0 if alpha is None else alpha
    return _sparse_encode(X, dictionary, gram, cov=cov, algorithm=algorithm,
                          regularization=reg, copy_cov=copy_cov, init=init, max_iter=max_iter,
                          positive=positive)


def _update_dict(dictionary, Y, code, verbose=False, return_r2=False, random_state=None,
                 positive=False):
    """Block-coordinate update of the (n_features, n_components) dictionary
    against Y (n_features, n_samples) and code (n_components, n_samples);
    the residual panel lives on the device."""
    rs = check_random_state(random_state)
    dev = resolve_device(None)
    D = torch.as_tensor(np.array(dictionary, dtype=np.float64), device=dev)
    C = torch.as_tensor(np.array(code, dtype=np.float64), device=dev)
    R = torch.as_tensor(np.asarray(Y, dtype=np.float64), device=dev) - D @ C
    nf = Y.shape[0]
    for j in range(C.shape[0]):
        R += D[:, j:j + 1] * C[j][None, :]
        col = R @ C[j]
        if positive:
            col = col.clamp(min=0)
        nrm = float(torch.linalg.vector_norm(col))
        if nrm < 1e-10:
            col = torch.as_tensor(rs.randn(nf), device=dev)
            if positive:
                col = col.clamp(min=0)
            C[j] = 0.0
            D[:, j] = col / torch.linalg.vector_norm(col)
        else:
            D[:, j] = col / nrm
            R -= D[:, j:j + 1] * C[j][None, :]
    out = D.cpu().numpy()
    if return_r2:
        return out, float(torch.linalg.vector_norm(R)) ** 2
    return out


def dict_learning(X, n_components, *, alpha, max_iter=100, tol=1e-8, method="lars",
                  n_jobs=None, dict_init=None, code_init=None, callback=None, verbose=False,
                  random_state=None, return_n_iter=False, positive_dict=False,
                  positive_code=False, method_max_iter=1000):
    """Alternate sparse coding and dictionary updates from an SVD start."""
    if method not in ("lars", "cd"):
        raise ValueError("Coding method %r not supported as a fit algorithm." % method)
    _check_positive_coding(method, positive_code)
    method = "lasso_" + method
    alpha = float(alpha)
    rs = check_random_state(random_state)
    X = _np(X)
    if code_init is not None and dict_init is not None:
        code = np.array(code_init, order="F")
        dictionary = _np(dict_init)
    else:
        code, S, dictionary = linalg.svd(X, full_matrices=False)
        code, dictionary = svd_flip(code, dictionary)
        dictionary = S[:, None] * dictionary
    r = len(dictionary)
    if n_components <= r:
        code = code[:, :n_components]
        dictionary = dictionary[:n_components, :]
    else:
        code = np.c_[code, np.zeros((len(code), n_components - r))]
        dictionary = np.r_[dictionary, np.zeros((n_components - r, dictionary.shape[1]))]
    errors = []
    ii = -1
    for ii in range(max_iter):
        code = sparse_encode(X, dictionary, algorithm=method, alpha=alpha, init=code,
                             positive=positive_code, max_iter=method_max_iter)
        dictionary, res = _update_dict(dictionary.T, X.T, code.T, return_r2=True,
                                       random_state=rs, positive=positive_dict)
        dictionary = dictionary.T
        errors.append(0.5 * res + alpha * np.sum(np.abs(code)))
        if ii > 0 and errors[-2] - errors[-1] < tol * errors[-1]:
            break
        if ii % 5 == 0 and callback is not None:
            callback(locals())
    if return_n_iter:
        return code, dictionary, errors, ii + 1
    return code, dictionary, errors


def _gen_batches(n, bs):
    start = 0
    for _ in range(int(n // bs)):
        yield slice(start, start + bs)
        start += bs
    if start < n:
        yield slice(start, n)


def dict_learning_online(X, n_components=2, *, alpha=1, n_iter=100, return_code=True,
                         dict_init=None, callback=None, batch_size=3, verbose=False,
                         shuffle=True, n_jobs=None, method="lars", iter_offset=0,
                         random_state=None, return_inner_stats=False, inner_stats=None,
                         return_n_iter=False, positive_dict=False, positive_code=False,
                         method_max_iter=1000):
    """Online (mini-batch) dictionary learning with the sufficient
    statistics A = sum code code^T and B = sum x code^T."""
    X = _np(X)
    if n_components is None:
        n_components = X.shape[1]
    if method not in ("lars", "cd"):
        raise ValueError("Coding method not supported as a fit algorithm.")
    _check_positive_coding(method, positive_code)
    method = "lasso_" + method
    n, d = X.shape
    alpha = float(alpha)
    rs = check_random_state(random_state)
    if dict_init is not None:
        dictionary = _np(dict_init)
    else:
        _, S, dictionary = randomized_svd(X, n_components, random_state=rs)
        dictionary = S[:, None] * dictionary
    r = len(dictionary)
    if n_components <= r:
        dictionary = dictionary[:n_components, :]
    else:
        dictionary = np.r_[dictionary, np.zeros((n_components - r, dictionary.shape[1]))]
    if shuffle:
        Xtr = X.copy()
        rs.shuffle(Xtr)
    else:
        Xtr = X
    dictionary = np.array(dictionary.T, order="F")
    batches = itertools.cycle(_gen_batches(n, batch_size))
    if inner_stats is None:
        A = np.zeros((n_components, n_components))
        B = np.zeros((d, n_components))
    else:
        A, B = inner_stats[0].copy(), inner_stats[1].copy()
    ii = iter_offset - 1
    for ii, batch in zip(range(iter_offset, iter_offset + n_iter), batches):
        xb = Xtr[batch]
        cb = sparse_encode(xb, dictionary.T, algorithm=method, alpha=alpha,
                           positive=positive_code, max_iter=method_max_iter).T
        theta = float((ii + 1) * batch_size) if ii < batch_size - 1 else \
            float(batch_size ** 2 + ii + 1 - batch_size)
        beta = (theta + 1 - batch_size) / (theta + 1)
        A *= beta
        A += cb @ cb.T
        B *= beta
        B += xb.T @ cb.T
        dictionary = _update_dict(dictionary, B, A, random_state=rs, positive=positive_dict)
        if callback is not None:
            callback(locals())
    if return_inner_stats:
        if return_n_iter:
            return dictionary.T, (A, B), ii - iter_offset + 1
        return dictionary.T, (A, B)
    if return_code:
        code = sparse_encode(X, dictionary.T, algorithm=method, alpha=alpha,
                             positive=positive_code, max_iter=method_max_iter)
        if return_n_iter:
            return code, dictionary.T, ii - iter_offset + 1
        return code, dictionary.T
    if return_n_iter:
        return dictionary.T, ii - iter_offset + 1
    return dictionary.T


class _BaseSparseCoding(TransformerMixin):
    def _transform(self, X, dictionary):
        X = _np(X)
        if X.shape[1] != dictionary.shape[1]:
            raise ValueError("X has %d features, but %s is expecting %d features as input."
                             % (X.shape[1], type(self).__name__, dictionary.shape[1]))
        ta = self.transform_alpha
        if hasattr(self, "alpha") and self.alpha != 1.0 and ta is None:
            ta = 1.0  # 1.0 semantics: transform_alpha does not default to alpha
        code = sparse_encode(X, dictionary, algorithm=self.transform_algorithm,
                             n_nonzero_coefs=self.transform_n_nonzero_coefs, alpha=ta,
                             max_iter=self.transform_max_iter, positive=self.positive_code)
        if self.split_sign:
            nk = code.shape[1]
            s = np.empty((code.shape[0], 2 * nk))
            s[:, :nk] = np.maximum(code, 0)
            s[:, nk:] = -np.minimum(code, 0)
            code = s
        return code

    def transform(self, X):
        check_is_fitted(self, "components_")
        return self._transform(X, self.components_)


class SparseCoder(_BaseSparseCoding, BaseEstimator):
    """Sparse coding against a fixed, precomputed dictionary."""

    def __init__(self, dictionary, *, transform_algorithm="omp", transform_n_nonzero_coefs=None,
                 transform_alpha=None, split_sign=False, n_jobs=None, positive_code=False,
                 transform_max_iter=1000):
        self.dictionary = dictionary
        self.transform_algorithm = transform_algorithm
        self.transform_n_nonzero_coefs = transform_n_nonzero_coefs
        self.transform_alpha = transform_alpha
        self.split_sign = split_sign
        self.n_jobs = n_jobs
        self.positive_code = positive_code
        self.transform_max_iter = transform_max_iter

    def fit(self, X, y=None):
        return self

    @property
    def components_(self):
        return self.dictionary

    def transform(self, X, y=None):
        return self._transform(X, _np(self.dictionary))

    @property
    def n_components_(self):
        return np.asarray(self.dictionary).shape[0]

    @property
    def n_features_in_(self):
        return np.asarray(self.dictionary).shape[1]

    def _more_tags(self):
        # the dictionary fixes n_features: the generic fitting checks' data
        # does not apply
        return {"requires_fit": False, "_skip_fit_checks": True}


class DictionaryLearning(_BaseSparseCoding, BaseEstimator):
    def __init__(self, n_components=None, *, alpha=1, max_iter=1000, tol=1e-8,
                 fit_algorithm="lars", transform_algorithm="omp",
                 transform_n_nonzero_coefs=None, transform_alpha=None, n_jobs=None,
                 code_init=None, dict_init=None, verbose=False, split_sign=False,
                 random_state=None, positive_code=False, positive_dict=False,
                 transform_max_iter=1000):
        self.n_components = n_components
        self.alpha = alpha
        self.max_iter = max_iter
        self.tol = tol
        self.fit_algorithm = fit_algorithm
        self.transform_algorithm = transform_algorithm
        self.transform_n_nonzero_coefs = transform_n_nonzero_coefs
        self.transform_alpha = transform_alpha
        self.n_jobs = n_jobs
        self.code_init = code_init
        self.dict_init = dict_init
        self.verbose = verbose
        self.split_sign = split_sign
        self.random_state = random_state
        self.positive_code = positive_code
        self.positive_dict = positive_dict
        self.transform_max_iter = transform_max_iter

    def fit(self, X, y=None):
        rs = check_random_state(self.random_state)
        X = _np(X)
        self.n_features_in_ = X.shape[1]
        k = X.shape[1] if self.n_components is None else self.n_components
        _, U, E, self.n_iter_ = dict_learning(
            X, k, alpha=self.alpha, tol=self.tol, max_iter=self.max_iter,
            method=self.fit_algorithm, method_max_iter=self.transform_max_iter,
            code_init=self.code_init, dict_init=self.dict_init, random_state=rs,
            return_n_iter=True, positive_dict=self.positive_dict,
            positive_code=self.positive_code)
        self.components_ = U
        self._n_features_out = U.shape[0]
        self.error_ = E
        return self


class MiniBatchDictionaryLearning(_BaseSparseCoding, BaseEstimator):
    def __init__(self, n_components=None, *, alpha=1, n_iter=1000, fit_algorithm="lars",
                 n_jobs=None, batch_size=3, shuffle=True, dict_init=None,
                 transform_algorithm="omp", transform_n_nonzero_coefs=None,
                 transform_alpha=None, verbose=False, split_sign=False, random_state=None,
                 positive_code=False, positive_dict=False, transform_max_iter=1000):
        self.n_components = n_components
        self.alpha = alpha
        self.n_iter = n_iter
        self.fit_algorithm = fit_algorithm
        self.n_jobs = n_jobs
        self.batch_size = batch_size
        self.shuffle = shuffle
        self.dict_init = dict_init
        self.transform_algorithm = transform_algorithm
        self.transform_n_nonzero_coefs = transform_n_nonzero_coefs
        self.transform_alpha = transform_alpha
        self.verbose = verbose
        self.split_sign = split_sign
        self.random_state = random_state
        self.positive_code = positive_code
        self.positive_dict = positive_dict
        self.transform_max_iter = transform_max_iter

    def fit(self, X, y=None):
        rs = check_random_state(self.random_state)
        X = _np(X)
        self.n_features_in_ = X.shape[1]
        U, (A, B), self.n_iter_ = dict_learning_online(
            X, self.n_components, alpha=self.alpha, n_iter=self.n_iter, return_code=False,
            method=self.fit_algorithm, method_max_iter=self.transform_max_iter,
            dict_init=self.dict_init, batch_size=self.batch_size, shuffle=self.shuffle,
            random_state=rs, return_inner_stats=True, return_n_iter=True,
            positive_dict=self.positive_dict, positive_code=self.positive_code)
        self.components_ = U
        self._n_features_out = U.shape[0]
        self.inner_stats_ = (A, B)
        self.iter_offset_ = self.n_iter
        self.random_state_ = rs
        return self

    def partial_fit(self, X, y=None, iter_offset=None):
        if not hasattr(self, "random_state_"):
            self.random_state_ = check_random_state(self.random_state)
        dict_init = self.components_ if hasattr(self, "components_") else self.dict_init
        stats = getattr(self, "inner_stats_", None)
        if iter_offset is None:
            iter_offset = getattr(self, "iter_offset_", 0)
        X = _np(X)
        if iter_offset == 0:
            self.n_features_in_ = X.shape[1]
        U, (A, B) = dict_learning_online(
            X, self.n_components, alpha=self.alpha, n_iter=1, method=self.fit_algorithm,
            method_max_iter=self.transform_max_iter, dict_init=dict_init, batch_size=len(X),
            shuffle=False, return_code=False, iter_offset=iter_offset,
            random_state=self.random_state_, return_inner_stats=True, inner_stats=stats,
            positive_dict=self.positive_dict, positive_code=self.positive_code)
        self.components_ = U
        self._n_features_out = U.shape[0]
        self.inner_stats_ = (A, B)
        self.iter_offset_ = iter_offset + 1
        return self


class SparsePCA(TransformerMixin, BaseEstimator):
    """Sparse principal components: dictionary learning on X^T."""

    def __init__(self, n_components=None, *, alpha=1, ridge_alpha=0.01, max_iter=1000,
                 tol=1e-8, method="lars", n_jobs=None, U_init=None, V_init=None, verbose=False,
                 random_state=None):
        self.n_components = n_components
        self.alpha = alpha
        self.ridge_alpha = ridge_alpha
        self.max_iter = max_iter
        self.tol = tol
        self.method = method
        self.n_jobs = n_jobs
        self.U_init = U_init
        self.V_init = V_init
        self.verbose = verbose
        self.random_state = random_state

    def _finish(self, Vt):
        self.components_ = Vt.T
        nrm = np.linalg.norm(self.components_, axis=1)[:, None]
        nrm[nrm == 0] = 1
        self.components_ /= nrm
        self.n_components_ = len(self.components_)
        self._n_features_out = self.n_components_

    def fit(self, X, y=None):
        rs = check_random_state(self.random_state)
        X = _np(X)
        self.n_features_in_ = X.shape[1]
        self.mean_ = X.mean(axis=0)
        X = X - self.mean_
        k = X.shape[1] if self.n_components is None else self.n_components
        code_init = self.V_init.T if self.V_init is not None else None
        dict_init = self.U_init.T if self.U_init is not None else None
        Vt, _, E, self.n_iter_ = dict_learning(
            X.T, k, alpha=self.alpha, tol=self.tol, max_iter=self.max_iter, method=self.method,
            random_state=rs, code_init=code_init, dict_init=dict_init, return_n_iter=True)
        self._finish(Vt)
        self.error_ = E
        return self

    def transform(self, X):
        from ..linear_model._ridge import ridge_regression
        check_is_fitted(self, "components_")
        X = _np(X)
        if X.shape[1] != self.n_features_in_:
            raise ValueError("X has %d features, but %s is expecting %d features as input."
                             % (X.shape[1], type(self).__name__, self.n_features_in_))
        return np.asarray(ridge_regression(self.components_.T, (X - self.mean_).T,
                                           self.ridge_alpha, solver="cholesky"))


class MiniBatchSparsePCA(SparsePCA):
    def __init__(self, n_components=None, *, alpha=1, ridge_alpha=0.01, n_iter=100,
                 callback=None, batch_size=3, verbose=False, shuffle=True, n_jobs=None,
                 method="lars", random_state=None):
        super().__init__(n_components=n_components, alpha=alpha, verbose=verbose,
                         ridge_alpha=ridge_alpha, n_jobs=n_jobs, method=method,
                         random_state=random_state)
        self.n_iter = n_iter
        self.callback = callback
        self.batch_size = batch_size
        self.shuffle = shuffle

    def fit(self, X, y=None):
        rs = check_random_state(self.random_state)
        X = _np(X)
        self.n_features_in_ = X.shape[1]
        self.mean_ = X.mean(axis=0)
        X = X - self.mean_
        k = X.shape[1] if self.n_components is None else self.n_components
        Vt, _, self.n_iter_ = dict_learning_online(
            X.T, k, alpha=self.alpha, n_iter=self.n_iter, return_code=True, dict_init=None,
            callback=self.callback, batch_size=self.batch_size, shuffle=self.shuffle,
            method=self.method, random_state=rs, return_n_iter=True)
        self._finish(Vt)
        return self
