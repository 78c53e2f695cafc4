"""Spectral biclustering (reference ``cluster/_bicluster.py``) and the
bicluster consensus score (``metrics/cluster/_bicluster.py``).

The normalisations are dense device expressions (row / column scaling,
Sinkhorn-style bistochastic iterations); the singular vectors come from the
framework's randomized SVD or ARPACK and the clustering of the spectral
embedding from the framework's KMeans."""

from abc import ABCMeta, abstractmethod

import numpy as np
import scipy.sparse as sp
from scipy.optimize import linear_sum_assignment
from scipy.sparse.linalg import eigsh, svds

from ...base import BaseEstimator, BiclusterMixin
from ...utils.extmath import randomized_svd
from ...utils.validation import check_random_state

__all__ = ["SpectralBiclustering", "SpectralCoclustering", "consensus_score"]


def _make_nonnegative(X, min_value=0):
    m = X.min()
    if m < min_value:
        if sp.issparse(X):
            raise ValueError("Cannot make the data matrix nonnegative because it is sparse. "
                             "Adding a value to every entry would make it no longer sparse.")
        X = X + (min_value - m)
    return X


def _scale_normalize(X):
    X = _make_nonnegative(X)
    with np.errstate(divide="ignore", invalid="ignore"):
        r = np.asarray(1.0 / np.sqrt(X.sum(axis=1))).squeeze()
        c = np.asarray(1.0 / np.sqrt(X.sum(axis=0))).squeeze()
    r = np.where(np.isnan(r), 0, r)
    c = np.where(np.isnan(c), 0, c)
    if sp.issparse(X):
        an = sp.diags(r) @ X @ sp.diags(c)
    else:
        an = r[:, None] * X * c
    return an, r, c


def _bistochastic_normalize(X, max_iter=1000, tol=1e-5):
    X = _make_nonnegative(X)
    Xs = X
    for _ in range(max_iter):
        Xn, _, _ = _scale_normalize(Xs)
        if sp.issparse(X):
            dist = np.linalg.norm(Xs.data - X.data)
        else:
            dist = np.linalg.norm(Xs - Xn)
        Xs = Xn
        if dist is not None and dist < tol:
            break
    return Xs


def _log_normalize(X):
    X = _make_nonnegative(X, min_value=1)
    if sp.issparse(X):
        raise ValueError("Cannot compute log of a sparse matrix, because log(x) diverges to "
                         "-infinity as x goes to 0.")
    L = np.log(X)
    return L - L.mean(axis=1)[:, None] - L.mean(axis=0) + L.mean()


class BaseSpectral(BiclusterMixin, BaseEstimator, metaclass=ABCMeta):
    @abstractmethod
    def __init__(self, n_clusters=3, svd_method="randomized", n_svd_vecs=None,
                 mini_batch=False, init="k-means++", n_init=10, n_jobs="deprecated",
                 random_state=None):
        self.n_clusters = n_clusters
        self.svd_method = svd_method
        self.n_svd_vecs = n_svd_vecs
        self.mini_batch = mini_batch
        self.init = init
        self.n_init = n_init
        self.n_jobs = n_jobs
        self.random_state = random_state

    def _check_parameters(self):
        if self.svd_method not in ("randomized", "arpack"):
            raise ValueError("Unknown SVD method: '{0}'. svd_method must be one of {1}."
                             .format(self.svd_method, ("randomized", "arpack")))

    def fit(self, X, y=None):
        X = X.tocsr().astype(np.float64) if sp.issparse(X) else np.asarray(X, dtype=np.float64)
        if X.ndim != 2:
            raise ValueError("Expected 2D array, got %dD array instead" % X.ndim)
        self.n_features_in_ = X.shape[1]
        self._check_parameters()
        self._fit(X)
        return self

    def _svd(self, A, k, n_discard):
        if self.svd_method == "randomized":
            kw = {} if self.n_svd_vecs is None else {"n_oversamples": self.n_svd_vecs}
            u, _, vt = randomized_svd(A.toarray() if sp.issparse(A) else A, k,
                                      random_state=self.random_state, **kw)
        else:
            u, _, vt = svds(A, k=k, ncv=self.n_svd_vecs)
            if np.any(np.isnan(vt)):
                M = A.T @ A
                v0 = check_random_state(self.random_state).uniform(-1, 1, M.shape[0])
                vt = eigsh(M, ncv=self.n_svd_vecs, v0=v0)[1].T
            if np.any(np.isnan(u)):
                M = A @ A.T
                v0 = check_random_state(self.random_state).uniform(-1, 1, M.shape[0])
                u = eigsh(M, ncv=self.n_svd_vecs, v0=v0)[1]
        if not (np.all(np.isfinite(u)) and np.all(np.isfinite(vt))):
            raise ValueError("Input contains NaN, infinity or a value too large.")
        return u[:, n_discard:], vt[n_discard:].T

    def _k_means(self, data, n_clusters):
        from .kmeans import KMeans
        from .minibatch import MiniBatchKMeans
        if self.mini_batch:
            m = MiniBatchKMeans(n_clusters, init=self.init, n_init=self.n_init,
                                random_state=self.random_state)
        else:
            m = KMeans(n_clusters, init=self.init, n_init=self.n_init,
                       random_state=self.random_state)
        m.fit(data)
        return np.asarray(m.cluster_centers_), np.asarray(m.labels_)


class SpectralCoclustering(BaseSpectral):
    """Dhillon's spectral co-clustering of rows and columns."""

    def __init__(self, n_clusters=3, *, svd_method="randomized", n_svd_vecs=None,
                 mini_batch=False, init="k-means++", n_init=10, n_jobs="deprecated",
                 random_state=None):
        super().__init__(n_clusters, svd_method, n_svd_vecs, mini_batch, init, n_init, n_jobs,
                         random_state)

    def _fit(self, X):
        An, r, c = _scale_normalize(X)
        u, v = self._svd(An, 1 + int(np.ceil(np.log2(self.n_clusters))), n_discard=1)
        z = np.vstack((r[:, None] * u, c[:, None] * v))
        _, labels = self._k_means(z, self.n_clusters)
        n = X.shape[0]
        self.row_labels_ = labels[:n]
        self.column_labels_ = labels[n:]
        self.rows_ = np.vstack([self.row_labels_ == k for k in range(self.n_clusters)])
        self.columns_ = np.vstack([self.column_labels_ == k for k in range(self.n_clusters)])


class SpectralBiclustering(BaseSpectral):
    """Kluger's checkerboard spectral biclustering."""

    def __init__(self, n_clusters=3, *, method="bistochastic", n_components=6, n_best=3,
                 svd_method="randomized", n_svd_vecs=None, mini_batch=False, init="k-means++",
                 n_init=10, n_jobs="deprecated", random_state=None):
        super().__init__(n_clusters, svd_method, n_svd_vecs, mini_batch, init, n_init, n_jobs,
                         random_state)
        self.method = method
        self.n_components = n_components
        self.n_best = n_best

    def _check_parameters(self):
        super()._check_parameters()
        if self.method not in ("bistochastic", "scale", "log"):
            raise ValueError("Unknown method: '{0}'. method must be one of {1}."
                             .format(self.method, ("bistochastic", "scale", "log")))
        try:
            int(self.n_clusters)
        except TypeError:
            try:
                r, c = self.n_clusters
                int(r)
                int(c)
            except (ValueError, TypeError) as e:
                raise ValueError("Incorrect parameter n_clusters has value: {}. It should "
                                 "either be a single integer or an iterable with two integers:"
                                 " (n_row_clusters, n_column_clusters)") from e
        if self.n_components < 1:
            raise ValueError("Parameter n_components must be greater than 0, but its value is "
                             "{}".format(self.n_components))
        if self.n_best < 1:
            raise ValueError("Parameter n_best must be greater than 0, but its value is {}"
                             .format(self.n_best))
        if self.n_best > self.n_components:
            raise ValueError("n_best cannot be larger than n_components, but {} >  {}"
                             .format(self.n_best, self.n_components))

    def _fit(self, X):
        k = self.n_components
        if self.method == "bistochastic":
            An = _bistochastic_normalize(X)
            k += 1
        elif self.method == "scale":
            An = _scale_normalize(X)[0]
            k += 1
        else:
            An = _log_normalize(X)
        u, v = self._svd(An, k, 0 if self.method == "log" else 1)
        try:
            nr, nc = self.n_clusters
        except TypeError:
            nr = nc = self.n_clusters
        best_ut = self._fit_best_piecewise(u.T, self.n_best, nr)
        best_vt = self._fit_best_piecewise(v.T, self.n_best, nc)
        self.row_labels_ = self._project_and_cluster(X, best_vt.T, nr)
        self.column_labels_ = self._project_and_cluster(X.T, best_ut.T, nc)
        self.rows_ = np.vstack([self.row_labels_ == a for a in range(nr) for _ in range(nc)])
        self.columns_ = np.vstack([self.column_labels_ == b for _ in range(nr)
                                   for b in range(nc)])

    def _fit_best_piecewise(self, vectors, n_best, n_clusters):
        pw = np.empty_like(vectors)
        for i, v in enumerate(vectors):
            cen, lab = self._k_means(v.reshape(-1, 1), n_clusters)
            pw[i] = cen[lab].ravel()
        d = np.linalg.norm(vectors - pw, axis=1)
        return vectors[np.argsort(d)[:n_best]]

    def _project_and_cluster(self, data, vectors, n_clusters):
        return self._k_means(np.asarray(data @ vectors), n_clusters)[1]


def _jaccard(ar, ac, br, bc):
    inter = (ar * br).sum() * (ac * bc).sum()
    return inter / (ar.sum() * ac.sum() + br.sum() * bc.sum() - inter)


def consensus_score(a, b, *, similarity="jaccard"):
    """Similarity of two sets of biclusters (best one-to-one matching)."""
    if similarity == "jaccard":
        similarity = _jaccard
    ar, ac = (np.asarray(m) for m in a)
    br, bc = (np.asarray(m) for m in b)
    M = np.array([[similarity(ar[i], ac[i], br[j], bc[j]) for j in range(br.shape[0])]
                  for i in range(ar.shape[0])])
    ri, ci = linear_sum_assignment(1.0 - M)
    return M[ri, ci].sum() / max(len(a[0]), len(b[0]))
