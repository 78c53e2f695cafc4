"""Kernel SVMs with libsvm semantics (reference ``svm/_classes.py``: SVC
:445, NuSVC :677, SVR :900, NuSVR :1075, OneClassSVM :1228;
``svm/_base.py`` BaseLibSVM.fit :140-245, decision functions :402-470,
``BaseSVC.decision_function`` / ``predict`` :563-630; solver formulations of
``svm/src/libsvm/svm.cpp`` :1589-1831, one-vs-one model layout, Platt
probability estimates).

Work split (MI355X-first): the Gram / kernel matrix - the only O(n^2 d)
part - is one fp64 GEMM + epilogue on the resolved device (MFMA on the
MI355X), the SMO iterations run host-native over it
(``csrc/host/svm_smo.cpp``), and prediction kernels against the support
vectors are again device GEMMs.  Problems whose n x n kernel would exceed
``SQ_SVM_DENSE_BYTES`` (default 2 GiB: n ~ 16k) or whose input is sparse
switch to kernel rows computed on demand by the host library (dense or CSR
rows, never densified) behind an LRU cache of ``cache_size`` MB - the
reference's libsvm ``Cache`` - so the training-set size is bounded by
time, not by an n x n matrix.  ``shrinking`` follows libsvm's heuristic.
"""

import os

import numbers
import warnings

import numpy as np
import scipy.sparse as sp
import torch

from ...base import BaseEstimator, ClassifierMixin, RegressorMixin
from ...exceptions import ConvergenceWarning, NotFittedError
from ...ops import _host
from ...runtime.device import resolve_device
from ...utils.class_weight import compute_class_weight
from ...utils.validation import check_is_fitted, check_random_state


def kernel_matrix(X, Y, kernel, gamma, degree, coef0, device=None):
    """K(X, Y) in fp64 on the resolved device (returned as numpy)."""
    if callable(kernel):
        return np.asarray(kernel(X, Y), dtype=np.float64)
    if kernel == "precomputed":
        return np.asarray(X, dtype=np.float64)
    dev = resolve_device(device)
    A = torch.as_tensor(np.ascontiguousarray(X, dtype=np.float64), device=dev)
    B = A if Y is X else torch.as_tensor(np.ascontiguousarray(Y, dtype=np.float64), device=dev)
    if kernel == "linear":
        K = A @ B.T
    elif kernel == "poly":
        K = (gamma * (A @ B.T) + coef0) ** degree
    elif kernel == "sigmoid":
        K = torch.tanh(gamma * (A @ B.T) + coef0)
    elif kernel == "rbf":
        d2 = (A * A).sum(1)[:, None] + (B * B).sum(1)[None, :] - 2.0 * (A @ B.T)
        K = torch.exp(-gamma * d2.clamp_(min=0.0))
        if Y is X:
            K.fill_diagonal_(1.0)
    else:
        raise ValueError("kernel %r not supported" % (kernel,))
    return K.cpu().numpy()


_KTYPE = {"linear": 0, "poly": 1, "rbf": 2, "sigmoid": 3}


class _RowKernel:
    """Kernel of the (reordered) training rows evaluated on demand by the
    host SMO (``sqh_svm_solve_rows``): dense fp64 rows or CSR."""

    def __init__(self, X, kernel, gamma, degree, coef0, cache_mb):
        if sp.issparse(X):
            X = sp.csr_matrix(X, dtype=np.float64)
            X.sort_indices()
            self.Xd = None
            self.indptr = np.ascontiguousarray(X.indptr, dtype=np.int64)
            self.indices = np.ascontiguousarray(X.indices, dtype=np.int32)
            self.data = np.ascontiguousarray(X.data, dtype=np.float64)
        else:
            self.Xd = np.ascontiguousarray(X, dtype=np.float64)
            self.indptr = self.indices = self.data = None
        self.n, self.d = X.shape
        self.ktype = _KTYPE[kernel]
        self.gamma, self.degree, self.coef0 = float(gamma), int(degree), float(coef0)
        self.cache_bytes = int(max(float(cache_mb), 1.0) * 2 ** 20)

    def _ptrs(self):
        z = 0
        return (self.Xd.ctypes.data if self.Xd is not None else z,
                self.indptr.ctypes.data if self.indptr is not None else z,
                self.indices.ctypes.data if self.indices is not None else z,
                self.data.ctypes.data if self.data is not None else z)

    def block(self, rows, cols):
        """K[rows][:, cols] (host, OpenMP)."""
        rows = np.ascontiguousarray(rows, dtype=np.int32)
        cols = np.ascontiguousarray(cols, dtype=np.int32)
        out = np.empty((len(rows), len(cols)))
        _host.lib().sqh_svm_kernel_rows(*self._ptrs(), self.n, self.d, self.ktype, self.gamma,
                                        self.coef0, self.degree, rows.ctypes.data, len(rows),
                                        cols.ctypes.data, len(cols), out.ctypes.data)
        return out


def _solve(K, idx, y, p, C, alpha0, eps, max_iter, nu, shrinking=True):
    """One SMO sub-problem; ``K`` is the dense kernel (numpy) or a
    :class:`_RowKernel`.  Returns (alpha, rho, r, status)."""
    lib = _host.lib()
    idx = np.ascontiguousarray(idx, dtype=np.int32)
    y = np.ascontiguousarray(y, dtype=np.int8)
    p = np.ascontiguousarray(p, dtype=np.float64)
    C = np.ascontiguousarray(C, dtype=np.float64)
    alpha = np.ascontiguousarray(alpha0, dtype=np.float64).copy()
    out = np.zeros(7)
    if isinstance(K, _RowKernel):
        lib.sqh_svm_solve_rows(*K._ptrs(), K.n, K.d, K.ktype, K.gamma, K.coef0, K.degree,
                               K.cache_bytes, idx.ctypes.data, y.ctypes.data, p.ctypes.data,
                               C.ctypes.data, len(idx), float(eps), int(max_iter),
                               1 if nu else 0, int(bool(shrinking)), alpha.ctypes.data,
                               out.ctypes.data)
    else:
        K = np.ascontiguousarray(K, dtype=np.float64)
        lib.sqh_svm_solve(K.ctypes.data, K.shape[0], idx.ctypes.data, y.ctypes.data,
                          p.ctypes.data, C.ctypes.data, len(idx), float(eps), int(max_iter),
                          1 if nu else 0, int(bool(shrinking)), alpha.ctypes.data,
                          out.ctypes.data)
    return alpha, out[0], out[1], int(out[3])


def _dense_limit_bytes():
    return int(os.environ.get("SQ_SVM_DENSE_BYTES", 2 << 30))


def _ovr_decision_function(predictions, confidences, n_classes):
    n = predictions.shape[0]
    votes = np.zeros((n, n_classes))
    conf = np.zeros((n, n_classes))
    k = 0
    for i in range(n_classes):
        for j in range(i + 1, n_classes):
            conf[:, i] -= confidences[:, k]
            conf[:, j] += confidences[:, k]
            votes[predictions[:, k] == 0, i] += 1
            votes[predictions[:, k] == 1, j] += 1
            k += 1
    return votes + conf / (3 * (np.abs(conf) + 1))


def _sigmoid_train(dec, labels):
    """Platt's sigmoid fit (reference ``svm.cpp: sigmoid_train``)."""
    prior1 = float(np.sum(labels > 0))
    prior0 = float(len(labels) - prior1)
    max_iter, min_step, sigma, eps = 100, 1e-10, 1e-12, 1e-5
    hi, lo = (prior1 + 1.0) / (prior1 + 2.0), 1 / (prior0 + 2.0)
    t = np.where(labels > 0, hi, lo)
    A, B = 0.0, np.log((prior0 + 1.0) / (prior1 + 1.0))

    def fval(A, B):
        fApB = dec * A + B
        return np.sum(np.where(fApB >= 0, t * fApB + np.log1p(np.exp(-fApB)),
                               (t - 1) * fApB + np.log1p(np.exp(fApB))))

    f = fval(A, B)
    for _ in range(max_iter):
        fApB = dec * A + B
        p = np.where(fApB >= 0, np.exp(-fApB) / (1.0 + np.exp(-fApB)), 1.0 / (1 + np.exp(fApB)))
        q = 1 - p
        d2 = p * q
        h11 = sigma + np.sum(dec * dec * d2)
        h22 = sigma + np.sum(d2)
        h21 = np.sum(dec * d2)
        d1 = t - p
        g1 = np.sum(dec * d1)
        g2 = np.sum(d1)
        if abs(g1) < eps and abs(g2) < eps:
            break
        det = h11 * h22 - h21 * h21
        dA = -(h22 * g1 - h21 * g2) / det
        dB = -(-h21 * g1 + h11 * g2) / det
        gd = g1 * dA + g2 * dB
        step = 1.0
        while step >= min_step:
            nA, nB = A + step * dA, B + step * dB
            nf = fval(nA, nB)
            if nf < f + 0.0001 * step * gd:
                A, B, f = nA, nB, nf
                break
            step /= 2.0
        if step < min_step:
            break
    return A, B


def _multiclass_probability(r):
    """Pairwise coupling (reference ``svm.cpp: multiclass_probability``)."""
    k = r.shape[0]
    Q = -r * r.T
    np.fill_diagonal(Q, 0)
    np.fill_diagonal(Q, np.sum(r.T ** 2, axis=1) - np.diag(r.T ** 2))
    Q = np.zeros((k, k))
    for t in range(k):
        Q[t, t] = sum(r[j, t] ** 2 for j in range(k) if j != t)
        for j in range(k):
            if j != t:
                Q[t, j] = -r[j, t] * r[t, j]
    p = np.full(k, 1.0 / k)
    max_iter = max(100, k)
    eps = 0.005 / k
    for _ in range(max_iter):
        Qp = Q @ p
        pQp = p @ Qp
        if np.max(np.abs(Qp - pQp)) < eps:
            break
        for t in range(k):
            diff = (-Qp[t] + pQp) / Q[t, t]
            p[t] += diff
            pQp = (pQp + diff * (diff * Q[t, t] + 2 * Qp[t])) / (1 + diff) / (1 + diff)
            Qp = (Qp + diff * Q[t, :]) / (1 + diff)
            p /= (1 + diff)
    return p


class BaseLibSVM(BaseEstimator):
    _impl = None
    _sparse_kernels = ("linear", "poly", "rbf", "sigmoid", "precomputed")

    def _kernel(self, X, Y):
        return kernel_matrix(X, Y, self.kernel, self._gamma, self.degree, self.coef0,
                             getattr(self, "device", None))

    def _resolve_gamma(self, X):
        if self.kernel == "precomputed" or callable(self.kernel):
            return 0.0
        if isinstance(self.gamma, str):
            if self.gamma == "scale":
                if sp.issparse(X):
                    v = X.multiply(X).mean() - X.mean() ** 2
                else:
                    v = X.var()
                return 1.0 / (X.shape[1] * v) if v != 0 else 1.0
            if self.gamma == "auto":
                return 1.0 / X.shape[1]
            raise ValueError("When 'gamma' is a string, it should be either 'scale' or 'auto'. "
                             "Got '{}' instead.".format(self.gamma))
        return float(self.gamma)

    def _prep_X(self, X, keep_sparse=False):
        if hasattr(X, "detach"):
            X = X.detach().cpu().numpy()
        if sp.issparse(X):
            if keep_sparse:
                X = sp.csr_matrix(X, dtype=np.float64)
                X.sort_indices()
                return X
            X = X.toarray()
        return np.ascontiguousarray(X, dtype=np.float64)

    def _kernel_source(self, Xs):
        """Kernel of the training rows ``Xs`` for the SMO: the dense matrix
        (one device GEMM) when it fits ``SQ_SVM_DENSE_BYTES``, else a
        :class:`_RowKernel` (rows on demand + LRU cache of ``cache_size``
        MB); sparse input always takes the row path (never densified)."""
        n = Xs.shape[0]
        if self.kernel in _KTYPE and (sp.issparse(Xs) or 8 * n * n > _dense_limit_bytes()):
            return _RowKernel(Xs, self.kernel, self._gamma, self.degree, self.coef0,
                              getattr(self, "cache_size", 200))
        Xd = Xs.toarray() if sp.issparse(Xs) else Xs
        return self._kernel(Xd, Xd)

    def fit(self, X, y, sample_weight=None):
        rnd = check_random_state(self.random_state)
        X = self._prep_X(X, keep_sparse=self.kernel in _KTYPE)
        if X.ndim != 2:
            raise ValueError("Expected 2D array")
        n = X.shape[0]
        if self.kernel == "precomputed" and n != X.shape[1]:
            raise ValueError("Precomputed matrix must be a square matrix. Input is a {}x{} "
                             "matrix.".format(X.shape[0], X.shape[1]))
        self.n_features_in_ = X.shape[1]
        y = self._validate_targets(np.asarray(y).reshape(-1) if y is not None else None, n)
        sw = np.ones(n) if sample_weight is None else np.asarray(sample_weight, np.float64)
        if sw.shape[0] != n:
            raise ValueError("sample_weight and X have incompatible shapes")
        self._gamma = self._resolve_gamma(X)
        self._random_seed = rnd.randint(np.iinfo("i").max)
        keep = sw > 0       # the reference drops zero-weight samples before solving
        self._fit_X = X
        self._fit_libsvm(X, y, sw, keep)
        self.shape_fit_ = X.shape
        self._intercept_ = self.intercept_.copy()
        self._dual_coef_ = self.dual_coef_
        if self._impl in ("c_svc", "nu_svc") and len(self.classes_) == 2:
            self.intercept_ = -self.intercept_
            self.dual_coef_ = -self.dual_coef_
        if self.fit_status_ == 1:
            warnings.warn("Solver terminated early (max_iter=%i).  Consider pre-processing "
                          "your data with StandardScaler or MinMaxScaler." % self.max_iter,
                          ConvergenceWarning)
        return self

    def _validate_targets(self, y, n):
        self.class_weight_ = np.empty(0)
        return y.astype(np.float64)

    def _max_iter(self, l):
        return self.max_iter if self.max_iter > 0 else max(10000000, 100 * l)

    # ------------------------------------------------------- regression / 1-class
    def _fit_single(self, X, y, sw, keep):
        rows = np.where(keep)[0]
        Xk = X if self.kernel == "precomputed" else X[rows]
        K = self._kernel_source(Xk) if self.kernel != "precomputed" else X[np.ix_(rows, rows)]
        l = len(rows)
        w = sw[rows]
        ar = np.arange(l, dtype=np.int32)
        if self._impl == "one_class":
            C = w.copy()
            alpha = np.zeros(l)
            nu_l = float(np.sum(w * self.nu))
            i = 0
            while nu_l > 0 and i < l:
                alpha[i] = min(C[i], nu_l)
                nu_l -= alpha[i]
                i += 1
            a, rho, _, st = _solve(K, ar, np.ones(l), np.zeros(l), C, alpha, self.tol,
                                   self._max_iter(l), nu=False,
                                   shrinking=getattr(self, "shrinking", True))
            coef = a
        elif self._impl == "epsilon_svr":
            C = np.r_[w * self.C, w * self.C]
            idx = np.r_[ar, ar]
            yy = np.r_[np.ones(l), -np.ones(l)]
            p = np.r_[self.epsilon - y[rows], self.epsilon + y[rows]]
            a, rho, _, st = _solve(K, idx, yy, p, C, np.zeros(2 * l), self.tol,
                                   self._max_iter(2 * l), nu=False,
                                   shrinking=getattr(self, "shrinking", True))
            coef = a[:l] - a[l:]
        else:  # nu_svr
            C = np.r_[w * self.C, w * self.C]
            s = float(np.sum(w * self.C * self.nu)) / 2
            alpha2 = np.zeros(2 * l)
            for i in range(l):
                alpha2[i] = alpha2[i + l] = min(s, C[i])
                s -= alpha2[i]
            idx = np.r_[ar, ar]
            yy = np.r_[np.ones(l), -np.ones(l)]
            p = np.r_[-y[rows], y[rows]]
            a, rho, _, st = _solve(K, idx, yy, p, C, alpha2, self.tol, self._max_iter(2 * l),
                                   nu=True,
                                   shrinking=getattr(self, "shrinking", True))
            coef = a[:l] - a[l:]
        sv = np.where(coef != 0)[0]
        self.support_ = rows[sv].astype(np.int32)
        self.support_vectors_ = (X[self.support_] if self.kernel != "precomputed"
                                 else np.empty((0, 0)))
        self._n_support = np.array([0, 0], dtype=np.int32) if self._impl != "one_class" else \
            np.array([len(sv), 0], dtype=np.int32)
        self.dual_coef_ = coef[sv][None, :]
        self.intercept_ = np.array([-rho])
        self.fit_status_ = st
        self._probA = self._probB = np.empty(0)

    def _dense_decision(self, X):
        X = self._prep_X(X)
        if self.kernel == "precomputed":
            Kx = X[:, self.support_]
        else:
            if X.shape[1] != self.shape_fit_[1]:
                raise ValueError("X.shape[1] = %d should be equal to %d, the number of features "
                                 "at training time" % (X.shape[1], self.shape_fit_[1]))
            sv = self.support_vectors_
            Kx = self._kernel(X, sv.toarray() if sp.issparse(sv) else sv)
        return Kx

    @property
    def n_support_(self):
        check_is_fitted(self)
        if self._impl in ("c_svc", "nu_svc"):
            return self._n_support
        return np.array([0, 0] if self._impl != "one_class" else self._n_support)

    @property
    def coef_(self):
        if self.kernel != "linear":
            raise AttributeError("coef_ is only available when using a linear kernel")
        coef = self._get_coef()
        return coef

    def _get_coef(self):
        sv = self.support_vectors_
        if sp.issparse(sv):
            return np.asarray((sv.T @ self._dual_coef_.T).T)
        return self._dual_coef_ @ sv


class BaseSVC(ClassifierMixin, BaseLibSVM):
    def _validate_targets(self, y, n):
        cls, y_ = np.unique(y, return_inverse=True)
        self.class_weight_ = compute_class_weight(self.class_weight, classes=cls, y=y)
        if len(cls) < 2:
            raise ValueError("The number of classes has to be greater than one; got %d class"
                             % len(cls))
        self.classes_ = cls
        return y_.astype(np.float64)

    def _fit_libsvm(self, X, y, sw, keep):
        K_full = X if self.kernel == "precomputed" else None
        rows_all = np.where(keep)[0]
        yk = y[rows_all].astype(int)
        n_cls = len(self.classes_)
        groups = [rows_all[yk == c] for c in range(n_cls)]
        counts = np.array([len(g) for g in groups])
        if self._impl == "nu_svc":
            for i in range(n_cls):
                for j in range(i + 1, n_cls):
                    if self.nu * (counts[i] + counts[j]) / 2 > min(counts[i], counts[j]):
                        raise ValueError("specified nu is infeasible")
        order = np.concatenate(groups)
        Kx = order if K_full is not None else None
        K = (K_full[np.ix_(order, order)] if K_full is not None
             else self._kernel_source(X[order]))
        start = np.r_[0, np.cumsum(counts)]
        nonzero = np.zeros(len(order), dtype=bool)
        pair_coef, rhos, status = {}, [], 0
        probA, probB = [], []
        w_all = sw[order]
        for i in range(n_cls):
            for j in range(i + 1, n_cls):
                si = np.arange(start[i], start[i + 1])
                sj = np.arange(start[j], start[j + 1])
                idx = np.r_[si, sj].astype(np.int32)
                l = len(idx)
                yy = np.r_[np.ones(len(si)), -np.ones(len(sj))]
                w = w_all[idx]
                if self._impl == "c_svc":
                    C = np.r_[self.C * self.class_weight_[i] * w[:len(si)],
                              self.C * self.class_weight_[j] * w[len(si):]]
                    a, rho, _, st = _solve(K, idx, yy, -np.ones(l), C, np.zeros(l), self.tol,
                                           self._max_iter(l), nu=False,
                                           shrinking=getattr(self, "shrinking", True))
                    coef = a * yy
                else:
                    C = w.copy()
                    nu_l = float(np.sum(self.nu * C))
                    sp_, sn_ = nu_l / 2, nu_l / 2
                    alpha = np.zeros(l)
                    for t in range(l):
                        if yy[t] > 0:
                            alpha[t] = min(C[t], sp_)
                            sp_ -= alpha[t]
                        else:
                            alpha[t] = min(C[t], sn_)
                            sn_ -= alpha[t]
                    a, rho, r, st = _solve(K, idx, yy, np.zeros(l), C, alpha, self.tol,
                                           self._max_iter(l), nu=True,
                                           shrinking=getattr(self, "shrinking", True))
                    coef = a * yy / r
                    rho = rho / r
                status = max(status, st)
                if self.probability:
                    A, B = self._pair_platt(K, idx, yy, w, i, j)
                    probA.append(A)
                    probB.append(B)
                nonzero[idx[coef != 0]] = True
                pair_coef[(i, j)] = (idx, coef)
                rhos.append(rho)
        sv_pos = np.where(nonzero)[0]           # class-grouped order (libsvm model layout)
        pos_of = -np.ones(len(order), dtype=np.int64)
        pos_of[sv_pos] = np.arange(len(sv_pos))
        dual = np.zeros((n_cls - 1, len(sv_pos)))
        for (i, j), (idx, coef) in pair_coef.items():
            ni = start[i + 1] - start[i]
            for t, c in zip(idx[:ni], coef[:ni]):
                if nonzero[t]:
                    dual[j - 1, pos_of[t]] = c
            for t, c in zip(idx[ni:], coef[ni:]):
                if nonzero[t]:
                    dual[i, pos_of[t]] = c
        self.support_ = order[sv_pos].astype(np.int32)
        self.support_vectors_ = (X[self.support_] if self.kernel != "precomputed"
                                 else np.empty((0, 0)))
        cls_of_sv = np.searchsorted(start[1:], sv_pos, side="right")
        self._n_support = np.bincount(cls_of_sv, minlength=n_cls).astype(np.int32)
        self.dual_coef_ = dual
        self.intercept_ = -np.asarray(rhos, dtype=np.float64)
        self.fit_status_ = status
        self._probA = np.asarray(probA)
        self._probB = np.asarray(probB)

    def _pair_platt(self, K, idx, yy, w, i, j):
        """5-fold cross-validated decision values + sigmoid fit
        (reference ``svm_binary_svc_probability``)."""
        rs = np.random.RandomState(self._random_seed)
        l = len(idx)
        perm = rs.permutation(l)
        dec = np.zeros(l)
        nr_fold = 5
        for f in range(nr_fold):
            b, e = f * l // nr_fold, (f + 1) * l // nr_fold
            test = perm[b:e]
            train = np.r_[perm[:b], perm[e:]]
            ytr = yy[train]
            if np.all(ytr > 0) or np.all(ytr < 0):
                dec[test] = 1.0 if np.all(ytr > 0) else -1.0
                continue
            sub = idx[train]
            C = np.where(ytr > 0, self.C * self.class_weight_[i], self.C * self.class_weight_[j]) \
                if self._impl == "c_svc" else np.ones(len(train))
            if self._impl == "c_svc":
                a, rho, _, _ = _solve(K, sub, ytr, -np.ones(len(train)), C * w[train],
                                      np.zeros(len(train)), self.tol, self._max_iter(len(train)),
                                      nu=False,
                                      shrinking=getattr(self, "shrinking", True))
                coef = a * ytr
            else:
                C = w[train].copy()
                nu_l = float(np.sum(self.nu * C))
                s1, s2 = nu_l / 2, nu_l / 2
                alpha = np.zeros(len(train))
                for t in range(len(train)):
                    if ytr[t] > 0:
                        alpha[t] = min(C[t], s1)
                        s1 -= alpha[t]
                    else:
                        alpha[t] = min(C[t], s2)
                        s2 -= alpha[t]
                a, rho, r, _ = _solve(K, sub, ytr, np.zeros(len(train)), C, alpha, self.tol,
                                      self._max_iter(len(train)), nu=True,
                                      shrinking=getattr(self, "shrinking", True))
                coef = a * ytr / r
                rho = rho / r
            if isinstance(K, _RowKernel):
                nz = coef != 0
                dec[test] = K.block(idx[test], sub[nz]) @ coef[nz] - rho
            else:
                dec[test] = K[np.ix_(idx[test], sub)] @ coef - rho
        return _sigmoid_train(dec, yy)

    def _ovo_decision(self, X):
        Kx = self._dense_decision(X)
        n_cls = len(self.classes_)
        start = np.r_[0, np.cumsum(self._n_support)]
        out = np.empty((Kx.shape[0], n_cls * (n_cls - 1) // 2))
        p = 0
        for i in range(n_cls):
            for j in range(i + 1, n_cls):
                si, sj = slice(start[i], start[i + 1]), slice(start[j], start[j + 1])
                out[:, p] = (Kx[:, si] @ self._dual_coef_[j - 1, si]
                             + Kx[:, sj] @ self._dual_coef_[i, sj] + self._intercept_[p])
                p += 1
        return out

    def decision_function(self, X):
        check_is_fitted(self)
        dec = self._ovo_decision(X)
        if len(self.classes_) == 2:
            return -dec.ravel()
        if self.decision_function_shape == "ovr":
            return _ovr_decision_function(dec < 0, -dec, len(self.classes_))
        return dec

    def predict(self, X):
        check_is_fitted(self)
        if self.break_ties and self.decision_function_shape == "ovo":
            raise ValueError("break_ties must be False when decision_function_shape is 'ovo'")
        n_cls = len(self.classes_)
        if self.break_ties and self.decision_function_shape == "ovr" and n_cls > 2:
            return self.classes_.take(np.argmax(self.decision_function(X), axis=1))
        dec = self._ovo_decision(X)
        votes = np.zeros((dec.shape[0], n_cls), dtype=np.int64)
        p = 0
        for i in range(n_cls):
            for j in range(i + 1, n_cls):
                pos = dec[:, p] > 0
                votes[pos, i] += 1
                votes[~pos, j] += 1
                p += 1
        return self.classes_.take(np.argmax(votes, axis=1))

    def _check_proba(self):
        if not self.probability:
            raise AttributeError("predict_proba is not available when  probability=False")

    @property
    def predict_proba(self):
        self._check_proba()
        return self._predict_proba

    def _predict_proba(self, X):
        check_is_fitted(self)
        if self._probA.size == 0:
            raise NotFittedError("predict_proba is not available when fitted with "
                                 "probability=False")
        dec = self._ovo_decision(X)
        n_cls = len(self.classes_)
        min_prob = 1e-7
        out = np.empty((dec.shape[0], n_cls))
        for s in range(dec.shape[0]):
            r = np.zeros((n_cls, n_cls))
            p = 0
            for i in range(n_cls):
                for j in range(i + 1, n_cls):
                    fApB = dec[s, p] * self._probA[p] + self._probB[p]
                    v = (np.exp(-fApB) / (1 + np.exp(-fApB)) if fApB >= 0
                         else 1 / (1 + np.exp(fApB)))
                    v = min(max(v, min_prob), 1 - min_prob)
                    r[i, j], r[j, i] = v, 1 - v
                    p += 1
            out[s] = _multiclass_probability(r) if n_cls > 2 else [r[0, 1], r[1, 0]]
        return out

    @property
    def predict_log_proba(self):
        self._check_proba()
        return lambda X: np.log(self._predict_proba(X))

    @property
    def probA_(self):
        return self._probA

    @property
    def probB_(self):
        return self._probB

    def _get_coef(self):
        n_cls = len(self.classes_)
        if n_cls == 2:
            return self.dual_coef_ @ self.support_vectors_
        start = np.r_[0, np.cumsum(self._n_support)]
        rows = []
        for i in range(n_cls):
            for j in range(i + 1, n_cls):
                si, sj = slice(start[i], start[i + 1]), slice(start[j], start[j + 1])
                rows.append(self._dual_coef_[j - 1, si] @ self.support_vectors_[si]
                            + self._dual_coef_[i, sj] @ self.support_vectors_[sj])
        return np.asarray(rows)


def _svc_init(self, kernel, degree, gamma, coef0, tol, C, nu, shrinking, probability,
              cache_size, class_weight, verbose, max_iter, decision_function_shape,
              break_ties, random_state):
    self.kernel = kernel
    self.degree = degree
    self.gamma = gamma
    self.coef0 = coef0
    self.tol = tol
    self.shrinking = shrinking
    self.probability = probability
    self.cache_size = cache_size
    self.class_weight = class_weight
    self.verbose = verbose
    self.max_iter = max_iter
    self.decision_function_shape = decision_function_shape
    self.break_ties = break_ties
    self.random_state = random_state


class SVC(BaseSVC):
    """C-support vector classification (one-vs-one, libsvm semantics)."""
    _impl = "c_svc"

    def __init__(self, *, C=1.0, kernel="rbf", degree=3, gamma="scale", coef0=0.0,
                 shrinking=True, probability=False, tol=1e-3, cache_size=200, class_weight=None,
                 verbose=False, max_iter=-1, decision_function_shape="ovr", break_ties=False,
                 random_state=None, device=None):
        _svc_init(self, kernel, degree, gamma, coef0, tol, C, 0.0, shrinking, probability,
                  cache_size, class_weight, verbose, max_iter, decision_function_shape,
                  break_ties, random_state)
        self.C = C
        self.device = device


class NuSVC(BaseSVC):
    """Nu-support vector classification."""
    _impl = "nu_svc"

    def __init__(self, *, nu=0.5, kernel="rbf", degree=3, gamma="scale", coef0=0.0,
                 shrinking=True, probability=False, tol=1e-3, cache_size=200, class_weight=None,
                 verbose=False, max_iter=-1, decision_function_shape="ovr", break_ties=False,
                 random_state=None, device=None):
        _svc_init(self, kernel, degree, gamma, coef0, tol, 1.0, nu, shrinking, probability,
                  cache_size, class_weight, verbose, max_iter, decision_function_shape,
                  break_ties, random_state)
        self.nu = nu
        self.device = device

    C = 1.0


class SVR(RegressorMixin, BaseLibSVM):
    """Epsilon-support vector regression."""
    _impl = "epsilon_svr"
    random_state = None
    classes_ = np.empty(0)

    def __init__(self, *, kernel="rbf", degree=3, gamma="scale", coef0=0.0, tol=1e-3, C=1.0,
                 epsilon=0.1, shrinking=True, cache_size=200, verbose=False, max_iter=-1,
                 device=None):
        self.kernel = kernel
        self.degree = degree
        self.gamma = gamma
        self.coef0 = coef0
        self.tol = tol
        self.C = C
        self.epsilon = epsilon
        self.shrinking = shrinking
        self.cache_size = cache_size
        self.verbose = verbose
        self.max_iter = max_iter
        self.device = device

    def _fit_libsvm(self, X, y, sw, keep):
        self._fit_single(X, y, sw, keep)

    def predict(self, X):
        check_is_fitted(self)
        return self._dense_decision(X) @ self._dual_coef_[0] + self._intercept_[0]


class NuSVR(SVR):
    """Nu-support vector regression."""
    _impl = "nu_svr"

    def __init__(self, *, nu=0.5, C=1.0, kernel="rbf", degree=3, gamma="scale", coef0=0.0,
                 shrinking=True, tol=1e-3, cache_size=200, verbose=False, max_iter=-1,
                 device=None):
        super().__init__(kernel=kernel, degree=degree, gamma=gamma, coef0=coef0, tol=tol, C=C,
                         shrinking=shrinking, cache_size=cache_size, verbose=verbose,
                         max_iter=max_iter, device=device)
        del self.epsilon
        self.nu = nu

    epsilon = 0.0


class OneClassSVM(BaseLibSVM):
    """Unsupervised outlier detection (Schoelkopf's one-class SVM)."""
    _impl = "one_class"
    _estimator_type = "outlier_detector"
    random_state = None
    classes_ = np.empty(0)

    def __init__(self, *, kernel="rbf", degree=3, gamma="scale", coef0=0.0, tol=1e-3, nu=0.5,
                 shrinking=True, cache_size=200, verbose=False, max_iter=-1, device=None):
        self.kernel = kernel
        self.degree = degree
        self.gamma = gamma
        self.coef0 = coef0
        self.tol = tol
        self.nu = nu
        self.shrinking = shrinking
        self.cache_size = cache_size
        self.verbose = verbose
        self.max_iter = max_iter
        self.device = device

    def fit(self, X, y=None, sample_weight=None):
        super().fit(X, np.ones(self._prep_X(X).shape[0]), sample_weight=sample_weight)
        self.offset_ = -self._intercept_
        return self

    def _fit_libsvm(self, X, y, sw, keep):
        self._fit_single(X, y, sw, keep)

    def decision_function(self, X):
        check_is_fitted(self)
        return self._dense_decision(X) @ self._dual_coef_[0] + self._intercept_[0]

    def score_samples(self, X):
        return self.decision_function(X) + self.offset_

    def predict(self, X):
        return np.where(self.decision_function(X) > 0, 1, -1)

    def fit_predict(self, X, y=None):
        return self.fit(X).predict(X)


__all__ = ["SVC", "NuSVC", "SVR", "NuSVR", "OneClassSVM"]
