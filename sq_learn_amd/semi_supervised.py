"""Semi-supervised learning (reference ``semi_supervised/_label_propagation.py``
- ``BaseLabelPropagation`` :71, ``LabelPropagation`` :334,
``LabelSpreading`` :463 - and ``_self_training.py`` -
``SelfTrainingClassifier`` :19).

The dense RBF affinity (n x n) and the propagation iterations
``F <- W F`` run as fp64 matmuls on the resolved device (MI355X fp64
matrix cores); the label matrix stays resident across iterations and
only the convergence scalar comes back per step."""

import warnings
from abc import ABCMeta, abstractmethod

import numpy as np
import scipy.sparse as sp
import torch
from scipy.sparse import csgraph

from .base import BaseEstimator, ClassifierMixin, MetaEstimatorMixin, clone
from .exceptions import ConvergenceWarning
from .runtime.device import resolve_device
from .utils.metaestimators import available_if
from .utils.validation import check_is_fitted


def _dense(X):
    if sp.issparse(X):
        return X.toarray().astype(np.float64)
    return np.asarray(X.detach().cpu().numpy() if hasattr(X, "detach") else X, dtype=np.float64)


def _rbf(A, B, gamma, dev):
    a = torch.as_tensor(A, dtype=torch.float64, device=dev)
    b = torch.as_tensor(B, dtype=torch.float64, device=dev)
    d = (a * a).sum(1)[:, None] + (b * b).sum(1)[None, :] - 2.0 * a @ b.T
    d.clamp_(min=0)
    return torch.exp(-gamma * d)


class BaseLabelPropagation(ClassifierMixin, BaseEstimator, metaclass=ABCMeta):
    _variant = None

    @abstractmethod
    def _build_graph(self):
        """Affinity / Laplacian the labels propagate over."""

    def __init__(self, kernel="rbf", *, gamma=20, n_neighbors=7, alpha=1, max_iter=30, tol=1e-3,
                 n_jobs=None):
        self.max_iter = max_iter
        self.tol = tol
        self.kernel = kernel
        self.gamma = gamma
        self.n_neighbors = n_neighbors
        self.alpha = alpha
        self.n_jobs = n_jobs

    def _knn(self):
        from .neighbors import NearestNeighbors
        return NearestNeighbors(n_neighbors=self.n_neighbors)

    def _get_kernel(self, X, y=None):
        """Host or device affinity; knn kernels return a CSR connectivity
        graph (fit) or neighbour index lists (predict)."""
        if self.kernel == "rbf":
            k = _rbf(X, X if y is None else y, self.gamma, self._dev)
            return k.cpu().numpy()
        if self.kernel == "knn":
            if getattr(self, "nn_fit", None) is None:
                self.nn_fit = self._knn().fit(X)
            if y is None:
                ind = np.asarray(self.nn_fit.kneighbors(self.nn_fit_X_, self.n_neighbors,
                                                        return_distance=False))
                n = ind.shape[0]
                return sp.csr_matrix((np.ones(ind.size), ind.ravel(),
                                      np.arange(0, ind.size + 1, self.n_neighbors)), shape=(n, n))
            return np.asarray(self.nn_fit.kneighbors(y, return_distance=False))
        if callable(self.kernel):
            return self.kernel(X, X) if y is None else self.kernel(X, y)
        raise ValueError("%s is not a valid kernel. Only rbf and knn or an explicit function "
                         " are supported at this time." % self.kernel)

    def predict(self, X):
        return self.classes_[np.argmax(self.predict_proba(X), axis=1)].ravel()

    def predict_proba(self, X):
        check_is_fitted(self)
        X = _dense(X)
        W = self._get_kernel(self.X_, X)
        if self.kernel == "knn":
            P = np.array([np.sum(self.label_distributions_[w], axis=0) for w in W])
        else:
            P = np.asarray(W.T @ self.label_distributions_)
        P /= np.atleast_2d(np.sum(P, axis=1)).T
        return P

    def fit(self, X, y):
        X = _dense(X)
        y = np.asarray(y)
        self._dev = resolve_device(getattr(self, "device", None))
        self.X_ = X
        self.nn_fit = None
        self.nn_fit_X_ = X
        self.n_features_in_ = X.shape[1]
        G = self._build_graph()
        classes = np.unique(y)
        classes = classes[classes != -1]
        self.classes_ = classes
        n, nc = len(y), len(classes)
        alpha = self.alpha
        if self._variant == "spreading" and (alpha is None or alpha <= 0.0 or alpha >= 1.0):
            raise ValueError("alpha=%s is invalid: it must be inside the open interval (0, 1)"
                             % alpha)
        unlabeled = y == -1
        L = np.zeros((n, nc))
        for c in classes:
            L[y == c, classes == c] = 1
        static = L.copy()
        if self._variant == "propagation":
            static[unlabeled] = 0
        else:
            static *= 1 - alpha
        dev = self._dev
        Lt = torch.as_tensor(L, device=dev)
        St = torch.as_tensor(static, device=dev)
        Gt = (torch.as_tensor(G.toarray() if sp.issparse(G) else np.asarray(G), device=dev,
                              dtype=torch.float64))
        um = torch.as_tensor(unlabeled[:, None], device=dev)
        prev = torch.zeros_like(Lt)
        converged = False
        for self.n_iter_ in range(self.max_iter):
            if float((Lt - prev).abs().sum()) < self.tol:
                converged = True
                break
            prev = Lt
            Lt = Gt @ Lt
            if self._variant == "propagation":
                norm = Lt.sum(1, keepdim=True)
                norm[norm == 0] = 1
                Lt = Lt / norm
                Lt = torch.where(um, Lt, St)
            else:
                Lt = alpha * Lt + St
        if not converged:
            warnings.warn("max_iter=%d was reached without convergence." % self.max_iter,
                          category=ConvergenceWarning)
            self.n_iter_ += 1
        L = Lt.cpu().numpy()
        norm = np.sum(L, axis=1)[:, np.newaxis]
        norm[norm == 0] = 1
        self.label_distributions_ = L / norm
        self.transduction_ = self.classes_[np.argmax(self.label_distributions_, axis=1)].ravel()
        return self


class LabelPropagation(BaseLabelPropagation):
    """Hard-clamped label propagation over a row-normalised affinity."""

    _variant = "propagation"

    def __init__(self, kernel="rbf", *, gamma=20, n_neighbors=7, max_iter=1000, tol=1e-3,
                 n_jobs=None):
        super().__init__(kernel=kernel, gamma=gamma, n_neighbors=n_neighbors, max_iter=max_iter,
                         tol=tol, n_jobs=n_jobs, alpha=None)

    def _build_graph(self):
        if self.kernel == "knn":
            self.nn_fit = None
        A = self._get_kernel(self.X_)
        norm = np.asarray(A.sum(axis=0))
        if sp.issparse(A):
            # reference _label_propagation.py:_build_graph divides by
            # np.diag of the (1, n) normaliser, i.e. by its first entry
            A = A.tocsr().astype(np.float64)
            A.data /= np.diag(np.array(norm))
        else:
            A = A / norm[:, np.newaxis]
        return A

    def fit(self, X, y):
        return super().fit(X, y)


class LabelSpreading(BaseLabelPropagation):
    """Soft-clamped spreading over the normalised graph Laplacian."""

    _variant = "spreading"

    def __init__(self, kernel="rbf", *, gamma=20, n_neighbors=7, alpha=0.2, max_iter=30, tol=1e-3,
                 n_jobs=None):
        super().__init__(kernel=kernel, gamma=gamma, n_neighbors=n_neighbors, alpha=alpha,
                         max_iter=max_iter, tol=tol, n_jobs=n_jobs)

    def _build_graph(self):
        n = self.X_.shape[0]
        if self.kernel == "knn":
            self.nn_fit = None
        A = self._get_kernel(self.X_)
        lap = -csgraph.laplacian(A, normed=True)
        if sp.issparse(lap):
            lap = lap.tocoo()
            diag = lap.row == lap.col
            lap.data[diag] = 0.0
        else:
            lap.flat[::n + 1] = 0.0
        return lap


def _est_has(attr):
    def check(self):
        est = getattr(self, "base_estimator_", self.base_estimator)
        return hasattr(est, attr)
    return check


class SelfTrainingClassifier(MetaEstimatorMixin, ClassifierMixin, BaseEstimator):
    """Iteratively pseudo-label the confident unlabeled samples (-1)."""

    def __init__(self, base_estimator, threshold=0.75, criterion="threshold", k_best=10,
                 max_iter=10, verbose=False):
        self.base_estimator = base_estimator
        self.threshold = threshold
        self.criterion = criterion
        self.k_best = k_best
        self.max_iter = max_iter
        self.verbose = verbose

    def fit(self, X, y):
        X = X if sp.issparse(X) else np.asarray(X)
        y = np.asarray(y)
        if y.dtype.kind in "US":
            raise ValueError("y has dtype string. If you wish to predict on string targets, use "
                             "dtype object, and use -1 as the label for unlabeled samples.")
        self.base_estimator_ = clone(self.base_estimator)
        if self.max_iter is not None and self.max_iter < 0:
            raise ValueError("max_iter must be >= 0 or None, got {}".format(self.max_iter))
        if not (0 <= self.threshold < 1):
            raise ValueError("threshold must be in [0,1), got {}".format(self.threshold))
        if self.criterion not in ["threshold", "k_best"]:
            raise ValueError("criterion must be either 'threshold' or 'k_best', got {}."
                             .format(self.criterion))
        has_label = y != -1
        if np.all(has_label):
            warnings.warn("y contains no unlabeled samples", UserWarning)
        self.transduction_ = np.copy(y)
        self.labeled_iter_ = np.full_like(y, -1)
        self.labeled_iter_[has_label] = 0
        self.n_iter_ = 0
        while not np.all(has_label) and (self.max_iter is None or self.n_iter_ < self.max_iter):
            self.n_iter_ += 1
            self.base_estimator_.fit(X[has_label], self.transduction_[has_label])
            prob = np.asarray(self.base_estimator_.predict_proba(X[~has_label]))
            pred = self.base_estimator_.classes_[np.argmax(prob, axis=1)]
            mx = np.max(prob, axis=1)
            if self.criterion == "threshold":
                sel = mx > self.threshold
            else:
                k = min(self.k_best, mx.shape[0])
                sel = np.ones_like(mx, dtype=bool) if k == mx.shape[0] else \
                    np.argpartition(-mx, k)[:k]
            full = np.nonzero(~has_label)[0][sel]
            self.transduction_[full] = pred[sel]
            has_label[full] = True
            self.labeled_iter_[full] = self.n_iter_
            if full.shape[0] == 0:
                self.termination_condition_ = "no_change"
                break
        if self.n_iter_ == self.max_iter:
            self.termination_condition_ = "max_iter"
        if np.all(has_label):
            self.termination_condition_ = "all_labeled"
        self.base_estimator_.fit(X[has_label], self.transduction_[has_label])
        self.classes_ = self.base_estimator_.classes_
        if hasattr(self.base_estimator_, "n_features_in_"):
            self.n_features_in_ = self.base_estimator_.n_features_in_
        return self

    def predict(self, X):
        check_is_fitted(self)
        return self.base_estimator_.predict(X)

    @available_if(_est_has("predict_proba"))
    def predict_proba(self, X):
        check_is_fitted(self)
        return self.base_estimator_.predict_proba(X)

    @available_if(_est_has("decision_function"))
    def decision_function(self, X):
        check_is_fitted(self)
        return self.base_estimator_.decision_function(X)

    @available_if(_est_has("predict_log_proba"))
    def predict_log_proba(self, X):
        check_is_fitted(self)
        return self.base_estimator_.predict_log_proba(X)

    def score(self, X, y):
        check_is_fitted(self)
        return self.base_estimator_.score(X, y)


__all__ = ["LabelPropagation", "LabelSpreading", "SelfTrainingClassifier"]

from .utils._aliases import alias_submodules  # noqa: E402
alias_submodules(__name__, "_self_training")

from .utils._aliases import alias_reference_layout  # noqa: E402

alias_reference_layout(__name__)
