"""Classical k-means on the same engine (parity oracle for delta = 0).

Reference: ``sklearn/cluster/_kmeans.py`` - ``KMeans`` (Lloyd, :383-481,
fit :842-936), ``k_means`` (:265), ``kmeans_plusplus`` (:1725).  Lloyd
semantics follow the reference exactly: strict convergence when labels stop
changing, else centre shift <= tol (tol scaled by the mean feature variance),
a final E-step when not strictly converged, inertia on the final
(labels, centres).  ``algorithm='elkan'`` runs the triangle-inequality
engine (``_elkan.py``, HIP kernel ``csrc/elkan.hip``; exact fp32/fp64
distances); 'auto' / 'full' / 'lloyd' run the fused MFMA Lloyd engine,
which on MI355X beats bounds at d >= 64.  The reference's
'auto' picks Elkan for dense data: the labels agree (both are the exact
argmin), only the cost differs.
Empty clusters are relocated to the rows farthest from their centres, like
the reference (``_k_means_fast.pyx:162-200``; per-shard top-e + one
all-gather when row-sharded).
"""

import warnings

import numpy as np
import torch

from ...base import BaseEstimator, ClusterMixin, TransformerMixin
from ...exceptions import ConvergenceWarning
from ...utils.validation import check_is_fitted, check_random_state, seed_from_random_state
from ...runtime.device import to_numpy
from ..._config import get_config
from .._data import as_data, global_mean_var, Data
from ._init import kmeans_plusplus as _kpp, kmeans_parallel as _kpar, random_init
from ._lloyd import LloydEngine
from ._elkan import ElkanEngine
from ...ops import kmeans as K


def _inertia(data, C, labels, sample_weight=None):
    X = data.X.double() if data.device.type == "cpu" else data.X.float()
    lab = labels.to(torch.int64)
    diff = X - C.to(X.dtype)[lab]
    v = (diff * diff).sum(1).double()
    if sample_weight is not None:
        v = v * sample_weight.double()
    t = v.sum().reshape(1)
    data.comm.all_reduce_(t)
    return float(t.item())


class KMeans(TransformerMixin, ClusterMixin, BaseEstimator):
    """K-Means clustering (Lloyd) with sklearn's API and semantics."""

    def __init__(self, n_clusters=8, *, init="k-means++", n_init=10, max_iter=300, tol=1e-4,
                 verbose=0, random_state=None, copy_x=True, algorithm="auto", device=None,
                 gemm_precision=None):
        self.n_clusters = n_clusters
        self.init = init
        self.n_init = n_init
        self.max_iter = max_iter
        self.tol = tol
        self.verbose = verbose
        self.random_state = random_state
        self.copy_x = copy_x
        self.algorithm = algorithm
        self.device = device
        self.gemm_precision = gemm_precision

    def _precision(self):
        return self.gemm_precision or get_config()["gemm_precision"]

    def fit(self, X, y=None, sample_weight=None):
        data = as_data(X, device=self.device, copy=self.copy_x)
        if self.n_init <= 0:
            raise ValueError(f"n_init should be > 0, got {self.n_init} instead.")
        if self.max_iter <= 0:
            raise ValueError(f"max_iter should be > 0, got {self.max_iter} instead.")
        if data.n_global < self.n_clusters:
            raise ValueError(f"n_samples={data.n_global} should be >= n_clusters={self.n_clusters}.")
        if self.algorithm not in ("auto", "full", "elkan", "lloyd"):
            raise ValueError(f"Algorithm must be 'auto', 'full' or 'elkan', got {self.algorithm} instead.")
        self.n_features_in_ = data.d
        n_init = self.n_init
        if hasattr(self.init, "__array__") and n_init != 1:
            warnings.warn("Explicit initial center position passed: performing only one init in "
                          f"KMeans instead of n_init={n_init}.", RuntimeWarning, stacklevel=2)
            n_init = 1
        rs = check_random_state(self.random_state)
        # A RandomState object must reach k-means++ unconsumed (reference
        # _kmeans.py:869 hands it straight to _init_centroids), so the
        # stochastic-layer seed is read from its state instead of drawn.
        seed = (int(rs.get_state()[1][0]) if isinstance(self.random_state, np.random.RandomState)
                else seed_from_random_state(self.random_state))
        mean, var = global_mean_var(data)
        tol = float(var.mean()) * self.tol
        Xc = data.X - mean.to(data.X.device).to(data.X.dtype) if data.X.dtype != torch.bfloat16 \
            else (data.X.float() - mean.float().to(data.device)).to(torch.bfloat16)
        dc = Data(Xc, data.n_global, data.row_offset, data.comm, data.source_kind)
        sw = None
        if sample_weight is not None:
            sw = torch.as_tensor(np.asarray(to_numpy(sample_weight), dtype=np.float64)).to(Xc.device)
        algo = self.algorithm
        if algo == "elkan" and self.n_clusters == 1:
            warnings.warn("algorithm='elkan' doesn't make sense for a single cluster. Using "
                          "'full' instead.", RuntimeWarning, stacklevel=2)
            algo = "full"
        if algo == "elkan":
            eng = ElkanEngine(Xc, self.n_clusters, sample_weight=sw, seed=seed,
                              comm=data.comm, row_offset=data.row_offset)
        else:
            eng = LloydEngine(Xc, self.n_clusters, delta=0.0, sample_weight=sw, seed=seed,
                              comm=data.comm, row_offset=data.row_offset,
                              gemm_precision=self._precision(), relocate_empty=True)
        best = None
        for r in range(n_init):
            eng.restart, eng.it = r, 0
            if isinstance(self.init, str) and self.init == "k-means++":
                C0, _ = _kpp(dc, self.n_clusters, rs, x_squared_norms=eng.xn)
            elif isinstance(self.init, str) and self.init == "k-means||":
                C0, _ = _kpar(dc, self.n_clusters, rs, x_squared_norms=eng.xn,
                              seed=int(rs.randint(2 ** 31 - 1)))
            elif isinstance(self.init, str) and self.init == "random":
                C0, _ = random_init(dc, self.n_clusters, rs)
            elif callable(self.init):
                C0 = torch.as_tensor(np.asarray(self.init(to_numpy(Xc), self.n_clusters,
                                                          random_state=rs))).to(Xc.device)
            else:
                C0 = torch.as_tensor(np.asarray(to_numpy(self.init), dtype=np.float64)).to(Xc.device) \
                    - mean.to(Xc.device)
            res = self._single(eng, dc, C0, tol, sw)
            if best is None or res[1] < best[1]:
                best = res
        labels, inertia, C, n_iter = best
        self.cluster_centers_ = to_numpy(C.double() + mean.to(C.device))
        self.labels_ = to_numpy(labels).astype(np.int32)
        self.inertia_ = inertia
        self.n_iter_ = n_iter
        distinct = len(np.unique(self.labels_))
        if data.comm.world_size == 1 and distinct < self.n_clusters:
            warnings.warn(f"Number of distinct clusters ({distinct}) found smaller than n_clusters "
                          f"({self.n_clusters}). Possibly due to duplicate points in X.",
                          ConvergenceWarning, stacklevel=2)
        return self

    def _single(self, eng, dc, C0, tol, sw):
        eng.set_centers(C0)
        labels_old = None
        strict = False
        it = 0
        for it in range(self.max_iter):
            labels, sc = eng.step()
            shift = float(sc[1].item())
            if labels_old is not None:
                changed = torch.tensor([float(not torch.equal(labels.to(torch.int64),
                                                              labels_old.to(torch.int64)))],
                                       dtype=torch.float64, device=labels.device)
                dc.comm.all_reduce_(changed, op="max")
                if changed.item() == 0.0:
                    strict = True
                    break
            if shift <= tol:
                break
            labels_old = labels.clone()
        C = eng.centers().clone()
        if not strict:
            labels, _, _ = eng.estep()
        labels = labels.clone()
        inertia = _inertia(dc, C, labels, sw)
        return labels, inertia, C, it + 1

    def _data_and_centers(self, X):
        check_is_fitted(self)
        data = as_data(X, device=self.device)
        if data.d != self.n_features_in_:
            raise ValueError(f"X has {data.d} features, but KMeans is expecting "
                             f"{self.n_features_in_} features as input.")
        return data, torch.as_tensor(self.cluster_centers_).to(data.device)

    def predict(self, X, sample_weight=None):
        data, C = self._data_and_centers(X)
        Xf = data.X.double() if data.device.type == "cpu" else data.X.float()
        D = K.distances_torch(Xf, C.to(Xf.dtype))
        return to_numpy(torch.argmin(D, 1)).astype(np.int32)

    def transform(self, X):
        data, C = self._data_and_centers(X)
        Xf = data.X.double() if data.device.type == "cpu" else data.X.float()
        return to_numpy(torch.sqrt(K.distances_torch(Xf, C.to(Xf.dtype))))

    def fit_transform(self, X, y=None, sample_weight=None):
        return self.fit(X, sample_weight=sample_weight).transform(X)

    def score(self, X, y=None, sample_weight=None):
        data, C = self._data_and_centers(X)
        Xf = data.X.double() if data.device.type == "cpu" else data.X.float()
        D = K.distances_torch(Xf, C.to(Xf.dtype))
        m = D.min(1).values.double()
        if sample_weight is not None:
            m = m * torch.as_tensor(np.asarray(sample_weight, dtype=np.float64)).to(m.device)
        return -float(m.sum())


def k_means(X, n_clusters, *, sample_weight=None, init="k-means++", n_init=10, max_iter=300,
            verbose=False, tol=1e-4, random_state=None, copy_x=True, algorithm="auto",
            return_n_iter=False, delta=None, **qkw):
    """Functional interface (reference ``_dmeans.py:265-401``): runs QMeans
    when ``delta`` is given, else KMeans."""
    if delta is not None:
        from .qmeans import QMeans
        est = QMeans(n_clusters=n_clusters, init=init, n_init=n_init, max_iter=max_iter,
                     verbose=verbose, tol=tol, random_state=random_state, copy_x=copy_x,
                     algorithm=algorithm, delta=delta, **qkw).fit(X, sample_weight=sample_weight)
    else:
        est = KMeans(n_clusters=n_clusters, init=init, n_init=n_init, max_iter=max_iter,
                     verbose=verbose, tol=tol, random_state=random_state, copy_x=copy_x,
                     algorithm=algorithm).fit(X, sample_weight=sample_weight)
    if return_n_iter:
        return est.cluster_centers_, est.labels_, est.inertia_, est.n_iter_
    return est.cluster_centers_, est.labels_, est.inertia_


def kmeans_plusplus(X, n_clusters, *, x_squared_norms=None, random_state=None,
                    n_local_trials=None):
    """Public k-means++ seeding (reference ``_kmeans.py:1725``): (centers, indices)."""
    data = as_data(X)
    rs = check_random_state(random_state)
    C, idx = _kpp(data, n_clusters, rs, n_local_trials=n_local_trials)
    return to_numpy(C), idx
