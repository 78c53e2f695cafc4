"""Spectral embedding (reference ``manifold/_spectral_embedding.py``:
``spectral_embedding`` :143, ``SpectralEmbedding`` :370).

Dense affinities (RBF / precomputed) are embedded with a full symmetric
eigendecomposition of the normalised Laplacian on the device (fp64); sparse
k-NN graphs use ARPACK shift-invert with the reference's v0 draw.  Both
end with the reference's deterministic sign flip, so the embedding is the
same up to numerical precision."""

import warnings

import numpy as np
import scipy.sparse as sp
import torch
from scipy.sparse.csgraph import connected_components
from scipy.sparse.csgraph import laplacian as csgraph_laplacian
from scipy.sparse.linalg import eigsh

from ...base import BaseEstimator
from ...runtime.device import resolve_device
from ...utils.validation import check_random_state


def _sign_flip(u):
    idx = np.argmax(np.abs(u), axis=1)
    s = np.sign(u[range(u.shape[0]), idx])
    return u * s[:, np.newaxis]


def _graph_is_connected(A):
    if sp.issparse(A):
        return connected_components(A)[0] == 1
    return connected_components(sp.csr_matrix(A))[0] == 1


def spectral_embedding(adjacency, *, n_components=8, eigen_solver=None, random_state=None,
                       eigen_tol=0.0, norm_laplacian=True, drop_first=True):
    if sp.issparse(adjacency):
        adjacency = sp.csr_matrix(adjacency, dtype=np.float64)
        if abs(adjacency - adjacency.T).max() > 1e-10:
            warnings.warn("Array is not symmetric, and will be converted to symmetric by "
                          "average with its transpose.")
            adjacency = 0.5 * (adjacency + adjacency.T)
    else:
        adjacency = np.asarray(adjacency.detach().cpu().numpy() if hasattr(adjacency, "detach")
                               else adjacency, dtype=np.float64)
        if not np.allclose(adjacency, adjacency.T):
            adjacency = 0.5 * (adjacency + adjacency.T)
    rs = check_random_state(random_state)
    n = adjacency.shape[0]
    if drop_first:
        n_components = n_components + 1
    if not _graph_is_connected(adjacency):
        warnings.warn("Graph is not fully connected, spectral embedding may not work as "
                      "expected.")
    L, dd = csgraph_laplacian(adjacency, normed=norm_laplacian, return_diag=True)
    if sp.issparse(L) and eigen_solver != "dense":
        L = L.tocoo()
        if norm_laplacian:
            diag = L.row == L.col
            L.data[diag] = 1.0
            missing = np.setdiff1d(np.arange(n), L.row[diag])
            if missing.size:
                L = sp.coo_matrix((np.r_[L.data, np.ones(missing.size)],
                                   (np.r_[L.row, missing], np.r_[L.col, missing])), shape=L.shape)
        L = -L.tocsr()
        v0 = rs.uniform(-1, 1, n)
        _, V = eigsh(L, k=n_components, sigma=1.0, which="LM", tol=eigen_tol, v0=v0)
        emb = V.T[n_components::-1]
    else:
        L = L.toarray() if sp.issparse(L) else np.array(L)
        if norm_laplacian:
            L.flat[::n + 1] = 1.0
        dev = resolve_device(None)
        w, V = torch.linalg.eigh(torch.as_tensor(L, device=dev))
        emb = V[:, :n_components].T.cpu().numpy()
        # consume the v0 draw the reference makes before ARPACK, so the
        # RandomState continues identically (e.g. into k-means)
        rs.uniform(-1, 1, n)
    if norm_laplacian:
        emb = emb / dd
    emb = _sign_flip(emb)
    return emb[1:n_components].T if drop_first else emb[:n_components].T


class SpectralEmbedding(BaseEstimator):
    """Laplacian eigenmaps."""

    def __init__(self, n_components=2, *, affinity="nearest_neighbors", gamma=None,
                 random_state=None, eigen_solver=None, n_neighbors=None, n_jobs=None):
        self.n_components = n_components
        self.affinity = affinity
        self.gamma = gamma
        self.random_state = random_state
        self.eigen_solver = eigen_solver
        self.n_neighbors = n_neighbors
        self.n_jobs = n_jobs

    def _affinity(self, X):
        if self.affinity == "precomputed":
            self.affinity_matrix_ = X
            return X
        if self.affinity == "precomputed_nearest_neighbors":
            from ..neighbors import NearestNeighbors
            nn = NearestNeighbors(n_neighbors=self.n_neighbors, metric="precomputed").fit(X)
            c = nn.kneighbors_graph(X, mode="connectivity")
            self.affinity_matrix_ = 0.5 * (c + c.T)
            return self.affinity_matrix_
        if self.affinity == "nearest_neighbors":
            from ..neighbors import kneighbors_graph
            self.n_neighbors_ = self.n_neighbors if self.n_neighbors is not None else \
                max(int(X.shape[0] / 10), 1)
            A = kneighbors_graph(X, self.n_neighbors_, include_self=True)
            self.affinity_matrix_ = 0.5 * (A + A.T)
            return self.affinity_matrix_
        if self.affinity == "rbf":
            from ...utils.pairwise import rbf_kernel
            self.gamma_ = self.gamma if self.gamma is not None else 1.0 / X.shape[1]
            K = rbf_kernel(X, gamma=self.gamma_)
            self.affinity_matrix_ = np.asarray(K.detach().cpu().numpy() if hasattr(K, "detach")
                                               else K)
            return self.affinity_matrix_
        if callable(self.affinity):
            self.affinity_matrix_ = self.affinity(X)
            return self.affinity_matrix_
        raise ValueError("%s is not a valid affinity. Expected 'precomputed', 'rbf', "
                         "'nearest_neighbors' or a callable." % self.affinity)

    def fit(self, X, y=None):
        X = np.asarray(X, dtype=np.float64) if not sp.issparse(X) else X
        self.n_features_in_ = X.shape[1]
        rs = check_random_state(self.random_state)
        A = self._affinity(X)
        self.embedding_ = spectral_embedding(A, n_components=self.n_components,
                                             eigen_solver=self.eigen_solver, random_state=rs)
        return self

    def fit_transform(self, X, y=None):
        return self.fit(X).embedding_


__all__ = ["spectral_embedding", "SpectralEmbedding"]
