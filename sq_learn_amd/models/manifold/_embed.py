"""Manifold learners (reference ``sklearn/manifold``): ``TSNE``
(``_t_sne.py`` + ``_utils.pyx`` perplexity search, N23), ``Isomap``
(``_isomap.py``), ``LocallyLinearEmbedding`` (``_locally_linear.py``),
``MDS`` / ``smacof`` (``_mds.py``) and ``trustworthiness``.

MI355X mapping:
* t-SNE: the perplexity binary search runs for all rows at once on the
  device.  ``method='exact'``: the O(n^2) Student-t gradient from dense
  device matmuls every iteration (n x n tiles in HBM, as the reference's
  dense P).  ``method='barnes_hut'`` (reference ``_barnes_hut_tsne.pyx``):
  the sparse k-NN P (3*perplexity neighbours) stays CSR and the gradient
  comes from the host-native Barnes-Hut kernel (``csrc/host/tsne_bh.cpp``:
  quad/oct-tree rebuilt per iteration, ``angle`` opening criterion,
  OpenMP over points, deterministic reductions) - O(n log n) time and O(n)
  memory per iteration.
* SMACOF iterations are n x n device matmuls; Isomap's geodesics use the
  framework's shortest-path kernels and device eigensolvers.
"""

import warnings

import numpy as np
import scipy.sparse as sp
import torch
from scipy import linalg
from scipy.sparse.linalg import eigsh

from ...base import BaseEstimator, TransformerMixin
from ...runtime.device import resolve_device
from ...utils.validation import check_is_fitted, check_random_state

MACHINE_EPSILON = np.finfo(np.double).eps


def _dense(X):
    if hasattr(X, "detach"):
        X = X.detach().cpu().numpy()
    return np.asarray(X.toarray() if sp.issparse(X) else X, dtype=np.float64)


def _dev():
    return resolve_device(None)


def _sqdist_t(A):
    n2 = (A * A).sum(1)
    return (n2[:, None] + n2[None, :] - 2.0 * A @ A.T).clamp_(min=0)


# --------------------------------------------------------------------- t-SNE
def _binary_search_perplexity(D, perplexity, using_neighbors):
    """Row-parallel version of the reference's per-row search
    (``manifold/_utils.pyx:_binary_search_perplexity``): identical update
    rule, every row bisects its own beta; rows stop independently."""
    dev = _dev()
    D = torch.as_tensor(np.asarray(D, dtype=np.float64), device=dev)
    n, k = D.shape
    target = np.log(perplexity)
    beta = torch.ones(n, dtype=torch.float64, device=dev)
    bmin = torch.full_like(beta, -np.inf)
    bmax = torch.full_like(beta, np.inf)
    active = torch.ones(n, dtype=torch.bool, device=dev)
    P = torch.zeros_like(D)
    diag = None
    if not using_neighbors:
        diag = torch.eye(n, dtype=torch.bool, device=dev)
    for _ in range(100):
        Pi = torch.exp(-D * beta[:, None])
        if diag is not None:
            Pi = Pi.masked_fill(diag, 0.0)
        s = Pi.sum(1)
        s = torch.where(s == 0.0, torch.full_like(s, 1e-8), s)
        Pi = Pi / s[:, None]
        ent = torch.log(s) + beta * (D * Pi).sum(1)
        diff = ent - target
        P = torch.where(active[:, None], Pi, P)
        done = diff.abs() <= 1e-5
        up = active & ~done & (diff > 0)
        dn = active & ~done & (diff <= 0)
        bmin = torch.where(up, beta, bmin)
        nb_up = torch.where(torch.isinf(bmax), beta * 2.0, (beta + bmax) / 2.0)
        bmax = torch.where(dn, beta, bmax)
        nb_dn = torch.where(torch.isinf(bmin), beta / 2.0, (beta + bmin) / 2.0)
        beta = torch.where(up, nb_up, torch.where(dn, nb_dn, beta))
        active = active & ~done
        if not bool(active.any()):
            break
    return P


def _joint_probabilities(D2, perplexity):
    P = _binary_search_perplexity(D2.astype(np.float32).astype(np.float64), perplexity, False)
    P = P + P.T
    P = P / max(float(P.sum()), MACHINE_EPSILON)
    P = P.clamp(min=MACHINE_EPSILON)
    P.fill_diagonal_(0.0)
    return P


def _joint_probabilities_nn(dist, ind, n, perplexity):
    """Symmetric sparse joint probabilities from the k-NN conditional ones
    (reference ``_t_sne.py:_joint_probabilities_nn``): CSR, kept sparse."""
    cond = _binary_search_perplexity(dist.astype(np.float32).astype(np.float64), perplexity,
                                     True).cpu().numpy()
    P = sp.csr_matrix((cond.ravel(), ind.ravel(), np.arange(0, ind.size + 1, ind.shape[1])),
                      shape=(n, n))
    P = P + P.T
    P = P / max(P.sum(), MACHINE_EPSILON)
    if not np.all(np.abs(P.data) <= 1.0):
        raise ValueError("All probabilities should be less or then equal to one")
    P = P.tocsr()
    P.sort_indices()
    return P


def _kl_grad_bh(Y, P, dof, angle, compute_error=True):
    """KL divergence and gradient with the Barnes-Hut repulsion (host
    kernel ``sqh_tsne_bh_grad``); Y: (n, dim) fp64 numpy, P: CSR."""
    from ...ops import _host
    Y = np.ascontiguousarray(Y, dtype=np.float64)
    n, dim = Y.shape
    if dim > 3:
        raise ValueError("'n_components' should be inferior to 4 for the barnes_hut algorithm "
                         "as it relies on quad-tree or oct-tree.")
    indptr = np.ascontiguousarray(P.indptr, dtype=np.int64)
    indices = np.ascontiguousarray(P.indices, dtype=np.int32)
    data = np.ascontiguousarray(P.data, dtype=np.float64)
    grad = np.empty_like(Y)
    kl = _host.lib().sqh_tsne_bh_grad(Y.ctypes.data, n, dim, indptr.ctypes.data,
                                      indices.ctypes.data, data.ctypes.data, float(angle),
                                      float(dof), int(bool(compute_error)), grad.ctypes.data)
    return (float(kl) if compute_error else None), grad


def _kl_grad(Y, P, dof, compute_error=True):
    """Exact KL(P||Q) and its gradient for the Student-t kernel."""
    D = _sqdist_t(Y)
    W = (1.0 + D / dof) ** ((dof + 1.0) / -2.0)
    W.fill_diagonal_(0.0)
    Q = (W / (2.0 * W.sum() / 2.0)).clamp(min=MACHINE_EPSILON)
    Q.fill_diagonal_(0.0)
    kl = None
    if compute_error:
        mask = P > 0
        kl = float(torch.sum(P[mask] * torch.log(P[mask].clamp(min=MACHINE_EPSILON)
                                                 / Q[mask])))
    PQd = (P - Q) * W
    g = (PQd.sum(1, keepdim=True) * Y - PQd @ Y) * (2.0 * (dof + 1.0) / dof)
    return kl, g


def _gradient_descent(Y, P, dof, it, n_iter, n_iter_check, n_iter_without_progress, momentum,
                      learning_rate, min_gain, min_grad_norm, angle=None):
    """Gradient descent with momentum and per-coordinate gains (reference
    ``_t_sne.py:_gradient_descent``).  ``angle=None``: exact gradient on the
    device tensors; otherwise Barnes-Hut on host arrays (Y numpy, P CSR)."""
    bh = angle is not None
    xp = np if bh else torch
    update = xp.zeros_like(Y)
    gains = xp.ones_like(Y)
    error = best = np.finfo(float).max
    best_iter = i = it
    for i in range(it, n_iter):
        check = (i + 1) % n_iter_check == 0
        if bh:
            kl, g = _kl_grad_bh(Y, P, dof, angle, check)
            gn = float(np.linalg.norm(g))
            inc = (update * g) < 0.0
            gains = np.maximum(np.where(inc, gains + 0.2, gains * 0.8), min_gain)
        else:
            kl, g = _kl_grad(Y, P, dof, check)
            gn = float(torch.linalg.norm(g))
            inc = (update * g) < 0.0
            gains = torch.where(inc, gains + 0.2, gains * 0.8).clamp(min=min_gain)
        g = g * gains
        update = momentum * update - learning_rate * g
        Y = Y + update
        if check:
            error = kl
            if error < best:
                best, best_iter = error, i
            elif i - best_iter > n_iter_without_progress:
                break
            if gn <= min_grad_norm:
                break
    return Y, error, i


class TSNE(BaseEstimator):
    """t-distributed stochastic neighbour embedding."""

    def __init__(self, n_components=2, *, perplexity=30.0, early_exaggeration=12.0,
                 learning_rate="warn", n_iter=1000, n_iter_without_progress=300,
                 min_grad_norm=1e-7, metric="euclidean", init="warn", verbose=0,
                 random_state=None, method="barnes_hut", angle=0.5, n_jobs=None,
                 square_distances="legacy"):
        self.n_components = n_components
        self.perplexity = perplexity
        self.early_exaggeration = early_exaggeration
        self.learning_rate = learning_rate
        self.n_iter = n_iter
        self.n_iter_without_progress = n_iter_without_progress
        self.min_grad_norm = min_grad_norm
        self.metric = metric
        self.init = init
        self.verbose = verbose
        self.random_state = random_state
        self.method = method
        self.angle = angle
        self.n_jobs = n_jobs
        self.square_distances = square_distances

    def _fit(self, X):
        init = "random" if isinstance(self.init, str) and self.init == "warn" else self.init
        lr = self.learning_rate
        if lr == "warn":
            lr = 200.0
        if self.method not in ("barnes_hut", "exact"):
            raise ValueError("'method' must be 'barnes_hut' or 'exact'")
        if self.early_exaggeration < 1.0:
            raise ValueError("early_exaggeration must be at least 1, but is {}"
                             .format(self.early_exaggeration))
        if self.n_iter < 250:
            raise ValueError("n_iter should be at least 250")
        X = X if self.metric == "precomputed" else _dense(X)
        n = X.shape[0]
        if lr == "auto":
            lr = max(n / self.early_exaggeration / 4, 50)
        self.learning_rate_ = lr
        rs = check_random_state(self.random_state)
        dev = _dev()
        if self.method == "exact":
            if self.metric == "precomputed":
                D = np.asarray(X, dtype=np.float64)
            elif self.metric == "euclidean":
                D = _sqdist_t(torch.as_tensor(X, device=dev)).cpu().numpy()
            else:
                from ...metrics import pairwise_distances
                D = np.asarray(pairwise_distances(X, metric=self.metric))
            if np.any(D < 0):
                raise ValueError("All distances should be positive, the metric given is not "
                                 "correct")
            P = _joint_probabilities(D, self.perplexity)
        else:
            from ..neighbors import NearestNeighbors
            k = min(n - 1, int(3.0 * self.perplexity + 1))
            nn = NearestNeighbors(n_neighbors=k, metric=self.metric).fit(X)
            dist, ind = nn.kneighbors(None, n_neighbors=k)
            dist = np.asarray(dist, dtype=np.float64)
            if self.metric == "euclidean":
                dist = dist ** 2
            P = _joint_probabilities_nn(dist, np.asarray(ind), n, self.perplexity)
        if isinstance(init, np.ndarray):
            Y0 = init
        elif init == "pca":
            from ..decomposition import PCA
            pca = PCA(n_components=self.n_components, svd_solver="randomized",
                      random_state=rs)
            Y0 = np.asarray(pca.fit_transform(X), dtype=np.float64)
            Y0 = Y0 / np.std(Y0[:, 0]) * 1e-4
        elif init == "random":
            Y0 = 1e-4 * rs.randn(n, self.n_components)
        else:
            raise ValueError("'init' must be 'pca', 'random', or a numpy array")
        dof = max(self.n_components - 1, 1)
        kw = dict(n_iter_check=50, min_gain=0.01, min_grad_norm=self.min_grad_norm,
                  learning_rate=lr)
        if self.method == "barnes_hut":
            if self.n_components > 3:
                raise ValueError("'n_components' should be inferior to 4 for the barnes_hut "
                                 "algorithm as it relies on quad-tree or oct-tree.")
            Y = np.array(Y0, dtype=np.float64)
            kw["angle"] = float(self.angle)
        else:
            Y = torch.as_tensor(np.asarray(Y0, dtype=np.float64), device=dev)
        Y, kl, it = _gradient_descent(Y, P * self.early_exaggeration, dof, 0, 250,
                                      n_iter_without_progress=250, momentum=0.5, **kw)
        if it < 250 or self.n_iter - 250 > 0:
            Y, kl, it = _gradient_descent(Y, P, dof, it + 1, self.n_iter,
                                          n_iter_without_progress=self.n_iter_without_progress,
                                          momentum=0.8, **kw)
        self.kl_divergence_ = kl
        self.n_iter_ = it
        self.n_features_in_ = X.shape[1]
        return Y if isinstance(Y, np.ndarray) else Y.cpu().numpy()

    def fit_transform(self, X, y=None):
        self.embedding_ = self._fit(X)
        return self.embedding_

    def fit(self, X, y=None):
        self.fit_transform(X)
        return self


def trustworthiness(X, X_embedded, *, n_neighbors=5, metric="euclidean"):
    from ...metrics import pairwise_distances
    from ..neighbors import NearestNeighbors
    if n_neighbors >= X.shape[0] / 2:
        raise ValueError("n_neighbors ({}) should be less than n_samples / 2 ({})"
                         .format(n_neighbors, X.shape[0] / 2))
    dX = np.array(pairwise_distances(X, metric=metric), dtype=np.float64)
    np.fill_diagonal(dX, np.inf)
    indX = np.argsort(dX, axis=1)
    indE = np.asarray(NearestNeighbors(n_neighbors=n_neighbors).fit(X_embedded)
                      .kneighbors(return_distance=False))
    n = X.shape[0]
    inv = np.zeros((n, n), dtype=int)
    o = np.arange(n + 1)
    inv[o[:-1, np.newaxis], indX] = o[1:]
    ranks = inv[o[:-1, np.newaxis], indE] - n_neighbors
    t = np.sum(ranks[ranks > 0])
    return 1.0 - t * (2.0 / (n * n_neighbors * (2.0 * n - 3.0 * n_neighbors - 1.0)))


# ------------------------------------------------------------------- Isomap
class Isomap(TransformerMixin, BaseEstimator):
    def __init__(self, *, n_neighbors=5, n_components=2, eigen_solver="auto", tol=0,
                 max_iter=None, path_method="auto", neighbors_algorithm="auto", n_jobs=None,
                 metric="minkowski", p=2, metric_params=None):
        self.n_neighbors = n_neighbors
        self.n_components = n_components
        self.eigen_solver = eigen_solver
        self.tol = tol
        self.max_iter = max_iter
        self.path_method = path_method
        self.neighbors_algorithm = neighbors_algorithm
        self.n_jobs = n_jobs
        self.metric = metric
        self.p = p
        self.metric_params = metric_params

    def _fit_transform(self, X):
        from ...utils.graph import graph_shortest_path
        from ..decomposition._extra import KernelPCA
        from ..neighbors import NearestNeighbors
        X = _dense(X)
        self.nbrs_ = NearestNeighbors(n_neighbors=self.n_neighbors,
                                      algorithm=self.neighbors_algorithm, metric=self.metric,
                                      p=self.p, metric_params=self.metric_params).fit(X)
        self.n_features_in_ = X.shape[1]
        self.kernel_pca_ = KernelPCA(n_components=self.n_components, kernel="precomputed",
                                     eigen_solver=self.eigen_solver, tol=self.tol,
                                     max_iter=self.max_iter)
        G = self.nbrs_.kneighbors_graph(None, self.n_neighbors, mode="distance")
        D = graph_shortest_path(G, directed=False, method=self.path_method)
        self.dist_matrix_ = np.asarray(D.detach().cpu().numpy() if hasattr(D, "detach") else D)
        K = -0.5 * self.dist_matrix_ ** 2
        self.embedding_ = self.kernel_pca_.fit_transform(K)

    def fit(self, X, y=None):
        self._fit_transform(X)
        return self

    def fit_transform(self, X, y=None):
        self._fit_transform(X)
        return self.embedding_

    def reconstruction_error(self):
        from ...preprocessing import KernelCenterer
        G = -0.5 * self.dist_matrix_ ** 2
        Gc = np.asarray(KernelCenterer().fit_transform(G))
        ev = self.kernel_pca_.eigenvalues_
        return np.sqrt(np.sum(Gc ** 2) - np.sum(ev ** 2)) / G.shape[0]

    def transform(self, X):
        check_is_fitted(self, "embedding_")
        X = _dense(X)
        d, ind = self.nbrs_.kneighbors(X, return_distance=True)
        d, ind = np.asarray(d), np.asarray(ind)
        GX = np.empty((d.shape[0], self.dist_matrix_.shape[0]))
        for i in range(d.shape[0]):
            GX[i] = np.min(self.dist_matrix_[ind[i]] + d[i][:, None], 0)
        return self.kernel_pca_.transform(-0.5 * GX ** 2)


# ---------------------------------------------------------------------- LLE
def barycenter_weights(X, Y, indices, reg=1e-3):
    X, Y = np.asarray(X, np.float64), np.asarray(Y, np.float64)
    n, k = indices.shape
    B = np.empty((n, k))
    v = np.ones(k)
    for i, ind in enumerate(indices):
        A = Y[ind]
        C = A - X[i]
        G = C @ C.T
        tr = np.trace(G)
        R = reg * tr if tr > 0 else reg
        G.flat[::k + 1] += R
        w = linalg.solve(G, v, assume_a="pos")
        B[i, :] = w / np.sum(w)
    return B


def barycenter_kneighbors_graph(X, n_neighbors, reg=1e-3, n_jobs=None):
    from ..neighbors import NearestNeighbors
    X = _dense(X)
    knn = NearestNeighbors(n_neighbors=n_neighbors + 1).fit(X)
    ind = np.asarray(knn.kneighbors(X, return_distance=False))[:, 1:]
    data = barycenter_weights(X, X, ind, reg=reg)
    n = X.shape[0]
    return sp.csr_matrix((data.ravel(), ind.ravel(), np.arange(0, n * n_neighbors + 1,
                                                               n_neighbors)), shape=(n, n))


def null_space(M, k, k_skip=1, eigen_solver="arpack", tol=1e-6, max_iter=100,
               random_state=None):
    if eigen_solver == "auto":
        eigen_solver = "arpack" if M.shape[0] > 200 and k + k_skip < 10 else "dense"
    if eigen_solver == "arpack":
        v0 = check_random_state(random_state).uniform(-1, 1, M.shape[0])
        try:
            w, V = eigsh(M, k + k_skip, sigma=0.0, tol=tol, maxiter=max_iter, v0=v0)
        except RuntimeError as e:
            raise ValueError("Error in determining null-space with ARPACK. Error message: '%s'. "
                             "Note that eigen_solver='arpack' can fail when the weight matrix is "
                             "singular or otherwise ill-behaved. In that case, eigen_solver="
                             "'dense' is recommended." % e) from e
        return V[:, k_skip:], np.sum(w[k_skip:])
    M = M.toarray() if sp.issparse(M) else M
    w, V = torch.linalg.eigh(torch.as_tensor(np.asarray(M, dtype=np.float64), device=_dev()))
    w, V = w[k_skip:k + k_skip].cpu().numpy(), V[:, k_skip:k + k_skip].cpu().numpy()
    idx = np.argsort(np.abs(w))
    return V[:, idx], np.sum(w)


def locally_linear_embedding(X, *, n_neighbors, n_components, reg=1e-3, eigen_solver="auto",
                             tol=1e-6, max_iter=100, method="standard", hessian_tol=1e-4,
                             modified_tol=1e-12, random_state=None, n_jobs=None):
    from ..neighbors import NearestNeighbors
    X = _dense(X)
    if method not in ("standard", "hessian", "modified", "ltsa"):
        raise ValueError("unrecognized method '%s'" % method)
    nbrs = NearestNeighbors(n_neighbors=n_neighbors + 1).fit(X)
    n, d = X.shape
    if n_components > d:
        raise ValueError("output dimension must be less than or equal to input dimension")
    if n_neighbors >= n:
        raise ValueError("Expected n_neighbors <= n_samples,  but n_samples = %d, "
                         "n_neighbors = %d" % (n, n_neighbors))
    dense = eigen_solver == "dense"
    if method == "standard":
        W = barycenter_kneighbors_graph(X, n_neighbors=n_neighbors, reg=reg)
        if not dense:
            Mm = sp.eye(n, format=W.format) - W
            M = (Mm.T @ Mm).tocsr()
        else:
            W = W.toarray()
            M = (W.T @ W - W.T) - W
            M.flat[::n + 1] += 1
    elif method == "hessian":
        dp = n_components * (n_components + 1) // 2
        if n_neighbors <= n_components + dp:
            raise ValueError("for method='hessian', n_neighbors must be greater than "
                             "[n_components * (n_components + 3) / 2]")
        ind = np.asarray(nbrs.kneighbors(X, n_neighbors=n_neighbors + 1,
                                         return_distance=False))[:, 1:]
        Yi = np.empty((n_neighbors, 1 + n_components + dp))
        Yi[:, 0] = 1
        M = np.zeros((n, n))
        use_svd = n_neighbors > d
        for i in range(n):
            Gi = X[ind[i]]
            Gi = Gi - Gi.mean(0)
            if use_svd:
                U = linalg.svd(Gi, full_matrices=0)[0]
            else:
                Ci = Gi @ Gi.T
                U = linalg.eigh(Ci)[1][:, ::-1]
            Yi[:, 1:1 + n_components] = U[:, :n_components]
            j = 1 + n_components
            for k in range(n_components):
                Yi[:, j:j + n_components - k] = U[:, k:k + 1] * U[:, k:n_components]
                j += n_components - k
            Q, R = linalg.qr(Yi)
            w = Q[:, n_components + 1:]
            S = w.sum(0)
            S[np.where(abs(S) < hessian_tol)] = 1
            w /= S
            nbrs_x, nbrs_y = np.meshgrid(ind[i], ind[i])
            M[nbrs_x, nbrs_y] += w @ w.T
        if not dense:
            M = sp.csr_matrix(M)
    elif method == "modified":
        if n_neighbors < n_components:
            raise ValueError("modified LLE requires n_neighbors >= n_components")
        ind = np.asarray(nbrs.kneighbors(X, n_neighbors=n_neighbors + 1,
                                         return_distance=False))[:, 1:]
        V = np.zeros((n, n_neighbors, n_neighbors))
        nev = min(d, n_neighbors)
        evals = np.zeros([n, nev])
        use_svd = n_neighbors > d
        for i in range(n):
            Xi = X[ind[i]] - X[i]
            if use_svd:
                v, s, _ = linalg.svd(Xi, full_matrices=True)
                evals[i] = s ** 2
                V[i] = v
            else:
                w_, v = linalg.eigh(Xi @ Xi.T)
                evals[i] = w_[::-1]
                V[i] = v[:, ::-1]
        reg_ = 1e-3 * evals.sum(1)
        tmp = np.einsum("ijk,j->ik", V, np.ones(n_neighbors))
        tmp[:, :nev] /= evals + reg_[:, None]
        tmp[:, nev:] /= reg_[:, None]
        w_reg = np.zeros((n, n_neighbors))
        for i in range(n):
            w_reg[i] = V[i] @ tmp[i]
        w_reg /= w_reg.sum(1)[:, None]
        rho = evals[:, n_components:].sum(1) / evals[:, :n_components].sum(1)
        eta = np.median(rho)
        s_range = np.zeros(n, dtype=int)
        ev_cum = np.cumsum(evals, 1)
        ratio = ev_cum[:, -1:] / ev_cum[:, :-1] - 1 if ev_cum.shape[1] > 1 else \
            np.zeros((n, 0))
        for i in range(n):
            s_range[i] = np.searchsorted(ratio[i, ::-1], eta) if ratio.shape[1] else 0
        s_range += n_neighbors - nev
        M = np.zeros((n, n))
        for i in range(n):
            s_i = s_range[i]
            Vi = V[i, :, n_neighbors - s_i:]
            alpha_i = np.linalg.norm(Vi.sum(0)) / np.sqrt(s_i)
            h = np.full(s_i, alpha_i) - Vi.sum(0)
            nh = np.linalg.norm(h)
            h = np.zeros(s_i) if nh < modified_tol else h / nh
            Wi = Vi - 2 * np.outer(Vi @ h, h) + (1 - alpha_i) * w_reg[i, :, None]
            nbrs_x, nbrs_y = np.meshgrid(ind[i], ind[i])
            M[nbrs_x, nbrs_y] += Wi @ Wi.T
            Wsum = Wi.sum(1)
            M[i, ind[i]] -= Wsum
            M[ind[i], i] -= Wsum
            M[i, i] += s_i
        if not dense:
            M = sp.csr_matrix(M)
    else:  # ltsa
        ind = np.asarray(nbrs.kneighbors(X, n_neighbors=n_neighbors + 1,
                                         return_distance=False))[:, 1:]
        M = np.zeros((n, n))
        use_svd = n_neighbors > d
        for i in range(n):
            Xi = X[ind[i]]
            Xi = Xi - Xi.mean(0)
            if use_svd:
                v = linalg.svd(Xi, full_matrices=True)[0]
            else:
                v = linalg.eigh(Xi @ Xi.T)[1][:, ::-1]
            Gi = np.zeros((n_neighbors, n_components + 1))
            Gi[:, 1:] = v[:, :n_components]
            Gi[:, 0] = 1.0 / np.sqrt(n_neighbors)
            GiGiT = Gi @ Gi.T
            nbrs_x, nbrs_y = np.meshgrid(ind[i], ind[i])
            M[nbrs_x, nbrs_y] -= GiGiT
            M[ind[i], ind[i]] += 1
        if not dense:
            M = sp.csr_matrix(M)
    return null_space(M, n_components, k_skip=1, eigen_solver=eigen_solver, tol=tol,
                      max_iter=max_iter, random_state=random_state)


class LocallyLinearEmbedding(TransformerMixin, BaseEstimator):

    def _more_tags(self):
        return {"_xfail_checks": {"check_transformer_general": "transform() of the training points uses the barycentric out-of-sample map, not the fitted embedding (same as the reference)"}}

    def __init__(self, *, n_neighbors=5, n_components=2, reg=1e-3, eigen_solver="auto",
                 tol=1e-6, max_iter=100, method="standard", hessian_tol=1e-4,
                 modified_tol=1e-12, neighbors_algorithm="auto", random_state=None, n_jobs=None):
        self.n_neighbors = n_neighbors
        self.n_components = n_components
        self.reg = reg
        self.eigen_solver = eigen_solver
        self.tol = tol
        self.max_iter = max_iter
        self.method = method
        self.hessian_tol = hessian_tol
        self.modified_tol = modified_tol
        self.random_state = random_state
        self.neighbors_algorithm = neighbors_algorithm
        self.n_jobs = n_jobs

    def _fit_transform(self, X):
        from ..neighbors import NearestNeighbors
        X = _dense(X)
        self.nbrs_ = NearestNeighbors(n_neighbors=self.n_neighbors,
                                      algorithm=self.neighbors_algorithm).fit(X)
        self.n_features_in_ = X.shape[1]
        rs = check_random_state(self.random_state)
        self.embedding_, self.reconstruction_error_ = locally_linear_embedding(
            X, n_neighbors=self.n_neighbors, n_components=self.n_components,
            eigen_solver=self.eigen_solver, tol=self.tol, max_iter=self.max_iter,
            method=self.method, hessian_tol=self.hessian_tol, modified_tol=self.modified_tol,
            random_state=rs, reg=self.reg)
        self._X = X

    def fit(self, X, y=None):
        self._fit_transform(X)
        return self

    def fit_transform(self, X, y=None):
        self._fit_transform(X)
        return self.embedding_

    def transform(self, X):
        check_is_fitted(self, "embedding_")
        X = _dense(X)
        ind = np.asarray(self.nbrs_.kneighbors(X, n_neighbors=self.n_neighbors,
                                               return_distance=False))
        W = barycenter_weights(X, self._X, ind, reg=self.reg)
        out = np.empty((X.shape[0], self.n_components))
        for i in range(X.shape[0]):
            out[i] = self.embedding_[ind[i]].T @ W[i]
        return out


# ---------------------------------------------------------------------- MDS
def _smacof_single(D, metric, n_components, init, max_iter, eps, rs):
    from ...isotonic import IsotonicRegression
    n = D.shape[0]
    sim_flat = ((1 - np.tri(n)) * D).ravel()
    nz = sim_flat != 0
    sim_w = sim_flat[nz]
    X = rs.rand(n * n_components).reshape((n, n_components)) if init is None else \
        np.asarray(init, dtype=np.float64)
    dev = _dev()
    Dt = torch.as_tensor(D, device=dev)
    Xt = torch.as_tensor(X, device=dev)
    ir = IsotonicRegression()
    old = None
    stress = 0.0
    for it in range(max_iter):
        dis = _sqdist_t(Xt).sqrt_()
        dis.fill_diagonal_(0.0)
        if metric:
            disp = Dt
        else:
            df = dis.cpu().numpy().ravel()
            dw = ir.fit_transform(sim_w, df[nz])
            dispf = df.copy()
            dispf[nz] = dw
            disp = torch.as_tensor(dispf.reshape(n, n), device=dev)
            disp = disp * np.sqrt((n * (n - 1) / 2) / float((disp ** 2).sum()))
        stress = float(((dis - disp) ** 2).sum()) / 2
        dis = torch.where(dis == 0, torch.full_like(dis, 1e-5), dis)
        ratio = disp / dis
        B = -ratio
        B.diagonal().add_(ratio.sum(1))
        Xt = (1.0 / n) * (B @ Xt)
        nrm = float(torch.sqrt((Xt ** 2).sum(1)).sum())
        if old is not None and (old - stress / nrm) < eps:
            break
        old = stress / nrm
    return Xt.cpu().numpy(), stress, it + 1


def smacof(dissimilarities, *, metric=True, n_components=2, init=None, n_init=8, n_jobs=None,
           max_iter=300, verbose=0, eps=1e-3, random_state=None, return_n_iter=False):
    D = np.asarray(dissimilarities, dtype=np.float64)
    if not np.allclose(D, D.T):
        raise ValueError("Array must be symmetric")
    rs = check_random_state(random_state)
    if init is not None:
        n_init = 1
    best = None
    for _ in range(n_init):
        pos, stress, it = _smacof_single(D, metric, n_components, init, max_iter, eps, rs)
        if best is None or stress < best[1]:
            best = (pos.copy(), stress, it)
    return best if return_n_iter else best[:2]


class MDS(BaseEstimator):
    def __init__(self, n_components=2, *, metric=True, n_init=4, max_iter=300, verbose=0,
                 eps=1e-3, n_jobs=None, random_state=None, dissimilarity="euclidean"):
        self.n_components = n_components
        self.dissimilarity = dissimilarity
        self.metric = metric
        self.n_init = n_init
        self.max_iter = max_iter
        self.eps = eps
        self.verbose = verbose
        self.n_jobs = n_jobs
        self.random_state = random_state

    def fit(self, X, y=None, init=None):
        self.fit_transform(X, init=init)
        return self

    def fit_transform(self, X, y=None, init=None):
        X = _dense(X)
        self.n_features_in_ = X.shape[1]
        if self.dissimilarity == "precomputed":
            self.dissimilarity_matrix_ = X
        elif self.dissimilarity == "euclidean":
            D = _sqdist_t(torch.as_tensor(X, device=_dev())).sqrt_()
            D.fill_diagonal_(0.0)
            self.dissimilarity_matrix_ = D.cpu().numpy()
        else:
            raise ValueError("Proximity must be 'precomputed' or 'euclidean'. Got %s instead"
                             % str(self.dissimilarity))
        self.embedding_, self.stress_, self.n_iter_ = smacof(
            self.dissimilarity_matrix_, metric=self.metric, n_components=self.n_components,
            init=init, n_init=self.n_init, max_iter=self.max_iter, eps=self.eps,
            random_state=self.random_state, return_n_iter=True)
        return self.embedding_


__all__ = ["TSNE", "trustworthiness", "Isomap", "LocallyLinearEmbedding",
           "locally_linear_embedding", "MDS", "smacof", "barycenter_kneighbors_graph"]
_ = warnings
