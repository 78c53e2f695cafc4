"""q-means (delta-k-means) clustering on MI355X.

Reference: ``sklearn/cluster/_dmeans.py`` class ``qMeans_`` (:833-1469) and
its Lloyd loop (:534-671), E-step (:674-777) and M-step (:780-830).

Parameters keep the reference's names and defaults.  Intentional deviations
(SURVEY.md §2.8):

* ``algorithm`` 'auto'/'full'/'lloyd'/'elkan' all run the (quantum) Lloyd
  iteration; the reference's 'auto' -> Elkan path crashes with the quantum
  kwargs (§2.8.2).
* ``predict`` / ``score`` work (the reference's raise TypeError, §2.8.3):
  ``predict(X, delta=None)`` assigns with the given band (default exact).
* empty clusters keep their previous centre instead of corrupting the
  centre array (§2.8.4); ``sample_weight`` is honoured.
* true tomography of the centres preserves their norms by default
  (``preserve_norm_tomography=True``); set it False for the reference's
  unit-norm behaviour (§2.8.12).
* no per-iteration ``print`` (§2.8.13): ``verbose`` logs structured records.
* ``multiprocess`` is accepted and ignored - every (sample, centroid) pair is
  processed by one batched GPU kernel instead of a process pool.

Framework additions: ``device``, ``gemm_precision`` ('bf16': fused bf16
MFMA kernel, d <= 256, band edge bf16-accurate; 'fp32': the certified E-step - an
fp16 MFMA filter whose error bound is certified against fp64, multi-candidate
rows re-checked in fp32/fp64, csrc/estep_f32.hip), ``compute_prelude`` (eta, mu(A),
condition number), ``ipe_Q`` (median repetitions of IPE), and
ShardedArray inputs for multi-GPU fits (one process per GPU).
"""

import warnings

import numpy as np
import torch

from ...base import BaseEstimator, ClusterMixin, TransformerMixin
from ...exceptions import ConvergenceWarning
from ...utils.validation import check_is_fitted, check_random_state, seed_from_random_state
from ...utils import tracing
from ...runtime.device import to_numpy
from ..._config import get_config
from .._data import as_data, check_n_features, global_mean_var, prelude_stats
from ...utils.checkpoint import Checkpointer, rs_state_from_tensors, rs_state_to_tensors
from ._init import kmeans_parallel, kmeans_plusplus, kmeans_plusplus_restarts, random_init
from ._lloyd import LloydEngine
from ...ops import kmeans as K
from ...quantum.fejer import median_repetitions
from ...quantum import cost_model


def _tolerance_from_var(var, tol):
    return float(var.mean()) * tol


class QMeans(TransformerMixin, ClusterMixin, BaseEstimator):
    """q-Means clustering (sklearn estimator API).

    Examples
    --------
    >>> import numpy as np
    >>> from sq_learn_amd.models.cluster import QMeans
    >>> X = np.array([[1, 2], [1, 4], [1, 0], [10, 2], [10, 4], [10, 0]])
    >>> q = QMeans(n_clusters=2, delta=0.1, random_state=0).fit(X)
    >>> sorted(np.round(q.cluster_centers_[:, 0]).tolist())
    [1.0, 10.0]
    """

    def __init__(self, n_clusters=8, *, init="k-means++", n_init=10, max_iter=300, tol=1e-4,
                 precompute_distances="deprecated", verbose=0, random_state=None, copy_x=True,
                 n_jobs="deprecated", algorithm="auto", delta=None, intermediate_error=False,
                 true_tomography=True, stop_when_reached_accuracy=True, multiprocess=False,
                 true_distance_estimate=True, device=None, gemm_precision=None,
                 compute_prelude=True, ipe_Q=None, preserve_norm_tomography=True,
                 empty_cluster="keep", failure_prob=0.0, failure_policy="ignore",
                 failure_max_attempts=3, checkpoint_dir=None, checkpoint_every=10):
        self.n_clusters = n_clusters
        self.init = init
        self.n_init = n_init
        self.max_iter = max_iter
        self.tol = tol
        self.precompute_distances = precompute_distances
        self.verbose = verbose
        self.random_state = random_state
        self.copy_x = copy_x
        self.n_jobs = n_jobs
        self.algorithm = algorithm
        self.delta = delta
        self.intermediate_error = intermediate_error
        self.true_tomography = true_tomography
        self.stop_when_reached_accuracy = stop_when_reached_accuracy
        self.multiprocess = multiprocess
        self.true_distance_estimate = true_distance_estimate
        self.device = device
        self.gemm_precision = gemm_precision
        self.compute_prelude = compute_prelude
        self.ipe_Q = ipe_Q
        self.preserve_norm_tomography = preserve_norm_tomography
        self.empty_cluster = empty_cluster
        self.failure_prob = failure_prob
        self.failure_policy = failure_policy
        self.failure_max_attempts = failure_max_attempts
        self.checkpoint_dir = checkpoint_dir
        self.checkpoint_every = checkpoint_every

    # ------------------------------------------------------------ checks
    def _check_params(self, data):
        if self.precompute_distances != "deprecated":
            warnings.warn("'precompute_distances' was deprecated in version 0.23 and will be "
                          "removed in 1.0 (renaming of 0.25). It has no effect", FutureWarning)
        if self.n_jobs != "deprecated":
            warnings.warn("'n_jobs' was deprecated in version 0.23 and will be removed in 1.0 "
                          "(renaming of 0.25).", FutureWarning)
        if self.n_init <= 0:
            raise ValueError(f"n_init should be > 0, got {self.n_init} instead.")
        if self.max_iter <= 0:
            raise ValueError(f"max_iter should be > 0, got {self.max_iter} instead.")
        if data.n_global < self.n_clusters:
            raise ValueError(f"n_samples={data.n_global} should be >= n_clusters={self.n_clusters}.")
        if self.algorithm not in ("auto", "full", "elkan", "lloyd"):
            raise ValueError(f"Algorithm must be 'auto', 'full' or 'elkan', got {self.algorithm} instead.")
        if not (hasattr(self.init, "__array__") or callable(self.init)
                or (isinstance(self.init, str) and self.init in ("k-means++", "k-means||", "random"))):
            raise ValueError("init should be either 'k-means++', 'k-means||', 'random', a ndarray or a callable, "
                             f"got '{self.init}' instead.")
        self._n_init = self.n_init
        if hasattr(self.init, "__array__") and self._n_init != 1:
            warnings.warn(f"Explicit initial center position passed: performing only one init in "
                          f"{self.__class__.__name__} instead of n_init={self._n_init}.",
                          RuntimeWarning, stacklevel=3)
            self._n_init = 1
        if self.empty_cluster not in ("keep", "zero", "relocate"):
            raise ValueError("empty_cluster must be 'keep', 'zero' or 'relocate'")
        if not 0.0 <= float(self.failure_prob) < 1.0:
            raise ValueError(f"failure_prob must be in [0, 1), got {self.failure_prob}")
        if self.failure_policy not in ("ignore", "resample"):
            raise ValueError("failure_policy must be 'ignore' or 'resample'")
        if self.failure_policy == "resample" and int(self.failure_max_attempts) < 1:
            raise ValueError("failure_max_attempts must be >= 1")

    def _delta(self):
        return 0.0 if self.delta is None else float(self.delta)

    def _precision(self):
        return self.gemm_precision or get_config()["gemm_precision"]

    def _init_centroids(self, data, init, rs, xn, mean):
        if isinstance(init, str) and init == "k-means++":
            C, _ = kmeans_plusplus(data, self.n_clusters, rs, x_squared_norms=xn)
        elif isinstance(init, str) and init == "k-means||":
            C, _ = kmeans_parallel(data, self.n_clusters, rs, x_squared_norms=xn,
                                   seed=int(rs.randint(2 ** 31 - 1)))
        elif isinstance(init, str) and init == "random":
            C, _ = random_init(data, self.n_clusters, rs)
        elif hasattr(init, "__array__") or isinstance(init, torch.Tensor):
            C = torch.as_tensor(np.asarray(to_numpy(init), dtype=np.float64)).to(data.device)
            C = C - mean.to(C.device)
        elif callable(init):
            full = data.X
            C = init(to_numpy(full), self.n_clusters, random_state=rs)
            C = torch.as_tensor(np.asarray(C, dtype=np.float64)).to(data.device)
        else:  # pragma: no cover
            raise ValueError(init)
        if C.shape != (self.n_clusters, data.d):
            raise ValueError(f"The shape of the initial centers {tuple(C.shape)} does not match the "
                             f"number of clusters {self.n_clusters} / features {data.d}.")
        return C

    # ------------------------------------------------------------------ fit
    def fit(self, X, y=None, sample_weight=None):
        """Compute q-means clustering (``_dmeans.py:1211-1325``)."""
        data = as_data(X, device=self.device, copy=self.copy_x)
        self._check_params(data)
        self.n_features_in_ = data.d
        delta = self._delta()
        if self.delta == 0:
            warnings.warn("Attention! You are running classic version of kmeans!")
            if self.intermediate_error:
                raise ValueError("intermediate_error value cannot be True if delta is zero.")
        comm = data.comm
        import time as _time
        phases = {}
        mark = [_time.perf_counter()]

        def phase(name):
            # wall-clock per fit phase (device-synchronised at the boundary)
            if data.device.type == "cuda":
                torch.cuda.synchronize(data.device)
            now = _time.perf_counter()
            phases[name] = phases.get(name, 0.0) + now - mark[0]
            mark[0] = now
        if self.compute_prelude:
            eta, mu_label, mu, cond = prelude_stats(data, 0.0, 0.1, 0.05)
            self.eta, self.muA, self.muA_norm, self.condition_number = eta, mu, mu_label, cond
        phase("prelude_s")
        rs = check_random_state(self.random_state)
        seed = seed_from_random_state(self.random_state)
        mean, var = global_mean_var(data)
        self._tol = _tolerance_from_var(var, self.tol)
        # centre the data (copy unless copy_x=False on a tensor input)
        Xc = data.X
        mean_t = mean.to(Xc.device)
        if Xc.dtype == torch.bfloat16:
            Xc = (Xc.float() - mean_t.float()).to(torch.bfloat16)
        else:
            Xc = Xc - mean_t.to(Xc.dtype)
        data_c = type(data)(Xc, data.n_global, data.row_offset, comm, data.source_kind)
        sw = None
        if sample_weight is not None:
            sw = torch.as_tensor(np.asarray(to_numpy(sample_weight), dtype=np.float64)).to(Xc.device)
            if sw.numel() != data.n_local:
                raise ValueError("sample_weight must have one weight per (local) sample")
        Q = self.ipe_Q if self.ipe_Q is not None else median_repetitions(0.1)
        tomo_kw = dict(stop_when_reached_accuracy=self.stop_when_reached_accuracy,
                       preserve_norm=self.preserve_norm_tomography)
        engine = LloydEngine(Xc, self.n_clusters, delta=delta,
                             true_distance_estimate=self.true_distance_estimate,
                             intermediate_error=self.intermediate_error,
                             true_tomography=self.true_tomography, tomography_kw=tomo_kw,
                             sample_weight=sw, seed=seed, comm=comm, row_offset=data.row_offset,
                             gemm_precision=self._precision(), ipe_Q=Q,
                             empty_policy=1 if self.empty_cluster == "zero" else 0,
                             relocate_empty=self.empty_cluster == "relocate",
                             failure_prob=float(self.failure_prob),
                             failure_attempts=(int(self.failure_max_attempts)
                                               if self.failure_policy == "resample" else 1))
        xn = engine.xn
        # iteration-level checkpoint / resume
        ckpt = Checkpointer(self.checkpoint_dir, comm, tag=type(self).__name__,
                            every=self.checkpoint_every)
        fingerprint = torch.cat([torch.tensor([float(data.n_global), float(data.d),
                                               float(self.n_clusters), float(seed % (1 << 52)),
                                               delta, float(self._n_init)], dtype=torch.float64),
                                 mean.double().cpu()])
        resume = ckpt.load()
        if resume is not None and not torch.equal(resume[0]["fingerprint"], fingerprint):
            warnings.warn("checkpoint in checkpoint_dir does not match this fit; starting over")
            resume = None
        best, start_restart = None, 0
        if resume is not None:
            st, loc = resume
            start_restart = int(st["restart"])
            if bool(st["has_best"]):
                best = (loc["best_labels"].to(data.device), float(st["best_inertia"]),
                        st["best_centers"].to(data.device), int(st["best_n_iter"]))
            rs_state_from_tensors(rs, st)
            if comm.rank == 0 and "failure_counters" in st:
                engine.failure_counters.copy_(st["failure_counters"].to(engine.device))
            self.resumed_from_ = (start_restart, int(st["it"]))
        self._ckpt_ctx = dict(ckpt=ckpt, fingerprint=fingerprint, rs=rs)
        phase("setup_s")
        # the k-means++ initialisations of every restart at once (the draws
        # in the reference order: the Lloyd loop never touches rs), one
        # device pass per centre for all restarts - also for one restart (its
        # fused passes: 0.449 vs 0.466 s sequentially at 10M x 256, k = 1024);
        # not with checkpoints (they save rs at restart boundaries)
        pre = None
        restart_inertias = []
        if (isinstance(self.init, str) and self.init == "k-means++" and resume is None
                and self._n_init - start_restart >= 1 and self.checkpoint_dir is None):
            pre = kmeans_plusplus_restarts(data_c, self.n_clusters, rs,
                                           self._n_init - start_restart)
        for restart in range(start_restart, self._n_init):
            engine.restart = restart
            engine.it = 0
            if resume is not None and restart == start_restart:
                st, loc = resume
                C0 = st["C"].to(data.device)
                engine.it = int(st["it"])
                inner = dict(best_inertia=st["r_best_inertia"], best_centers=st["r_best_centers"],
                             best_labels=loc.get("r_best_labels"), shift=float(st["shift"]),
                             engine={k[7:]: v for k, v in st.items() if k.startswith("engine_")},
                             engine_local={k[7:]: v for k, v in loc.items()
                                           if k.startswith("engine_")})
            elif pre is not None:
                C0 = pre[restart - start_restart]
                inner = None
            else:
                C0 = self._init_centroids(data_c, self.init, rs, xn, mean)
                inner = None
            phase("init_s")
            self._ckpt_ctx["outer_best"] = best
            labels, inertia, centers, n_iter = self._run_lloyd(engine, C0, resume=inner)
            phase("lloyd_s")
            restart_inertias.append(float(inertia))
            if best is None or inertia < best[1]:
                best = (labels, inertia, centers, n_iter)
        ckpt.clear()
        del self._ckpt_ctx   # holds the communicator: not estimator state
        labels, inertia, centers, n_iter = best
        cnt = engine.failure_counters.clone()
        comm.all_reduce_(cnt)
        counters = cnt.tolist()
        self.n_estimations_ = int(counters[0])
        self.n_failed_rows_ = int(counters[1])
        centers = centers.double() + mean.to(centers.device)
        self.cluster_centers_ = to_numpy(centers)
        self._labels_t = labels
        self.labels_ = to_numpy(labels).astype(np.int32)
        self.inertia_ = float(inertia)
        self.n_iter_ = int(n_iter)
        phase("finish_s")
        self.fit_phase_s_ = phases
        # the inertia each restart ended with (this run's restarts; the best
        # one is inertia_)
        self.fit_restart_inertias_ = restart_inertias
        self._mean = to_numpy(mean)
        self._engine_comm = comm
        distinct = self._count_distinct(labels, comm)
        if distinct < self.n_clusters:
            warnings.warn(f"Number of distinct clusters ({distinct}) found smaller than n_clusters "
                          f"({self.n_clusters}). Possibly due to duplicate points in X.",
                          ConvergenceWarning, stacklevel=2)
        return self

    @staticmethod
    def _count_distinct(labels, comm):
        lab = labels.to(torch.int64)
        present = torch.zeros(int(lab.max().item()) + 1 if lab.numel() else 1, dtype=torch.float64,
                              device=lab.device)
        k = present.numel()
        m = torch.tensor([k], dtype=torch.float64, device=lab.device)
        comm.all_reduce_(m, op="max")
        present = torch.zeros(int(m.item()), dtype=torch.float64, device=lab.device)
        present[lab[lab >= 0]] = 1.0
        comm.all_reduce_(present, op="max")
        return int(present.sum().item())

    def _save_checkpoint(self, engine, it, shift, best_inertia, best_centers, best_labels):
        ctx = self._ckpt_ctx
        outer = ctx.get("outer_best")
        state = dict(fingerprint=ctx["fingerprint"], restart=engine.restart, it=it + 1,
                     C=engine.centers().double(), shift=float(shift),
                     r_best_inertia=float(best_inertia), r_best_centers=best_centers.double(),
                     has_best=outer is not None,
                     best_inertia=float(outer[1]) if outer is not None else 0.0,
                     best_centers=(outer[2].double() if outer is not None
                                   else torch.zeros(1, dtype=torch.float64)),
                     best_n_iter=int(outer[3]) if outer is not None else 0,
                     **rs_state_to_tensors(ctx["rs"]))
        state.update({f"engine_{k}": v for k, v in engine.checkpoint_tensors().items()})
        cnt = engine.failure_counters.clone()
        engine.comm.all_reduce_(cnt)   # fit-wide totals, like the attributes
        state["failure_counters"] = cnt
        local = dict(r_best_labels=best_labels.to(torch.int32))
        local.update({f"engine_{k}": v for k, v in engine.checkpoint_local().items()})
        if outer is not None:
            local["best_labels"] = outer[0].to(torch.int32)
        ctx["ckpt"].save(state, local)

    def _run_lloyd(self, engine, C0, resume=None):
        """One restart of the quantum Lloyd loop (``_dmeans.py:594-671``)."""
        engine.set_centers(C0)
        log = tracing.IterationLog(type(self).__name__, self.verbose, engine.comm)
        best_inertia, best_centers, best_labels = None, None, None
        shift = 0.0
        first = 0
        if resume is not None:
            first = engine.it
            engine.restore_tensors(resume["engine"])
            engine.restore_local(resume.get("engine_local"))
            best_inertia = float(resume["best_inertia"])
            best_centers = resume["best_centers"].to(engine.device).to(engine.centers().dtype)
            best_labels = resume["best_labels"].to(engine.device)
            shift = resume["shift"]
        ckpt = getattr(self, "_ckpt_ctx", {}).get("ckpt")
        # next-iteration E-step enqueued before the scalar read (not with
        # checkpoints: a saved state must not include a speculative E-step)
        engine.pipeline = ckpt is None
        it = first - 1
        for it in range(first, self.max_iter):
            labels, sc = engine.step()
            vals = sc.tolist()  # the single D2H read of the iteration
            inertia, shift = vals[0], vals[1]
            log.record(iteration=it, inertia=inertia, shift=shift, overflow=int(vals[2]))
            if not np.isfinite(inertia) or not np.isfinite(shift):
                from ...exceptions import NumericalGuardError
                raise NumericalGuardError(f"non-finite inertia/shift at iteration {it}")
            if best_inertia is None or inertia < best_inertia:
                best_inertia = inertia
                best_centers = engine.centers().clone()
                best_labels = labels.clone()
            if shift <= self._tol:
                break
            if ckpt is not None and ckpt.due(it):
                self._save_checkpoint(engine, it, shift, best_inertia, best_centers, best_labels)
        engine.pipeline = False
        engine.drop_pending()
        it = max(it, first)
        if shift > 0:
            labels, _, inertia_t = engine.estep(best_centers)
            best_labels = labels.clone()
            it_tot = inertia_t.clone()
            engine.comm.all_reduce_(it_tot)
            best_inertia = float(it_tot.item())
            engine.set_centers(best_centers)
        self._iteration_log = log.records
        return best_labels, best_inertia, best_centers, it + 1

    # -------------------------------------------------------------- predict
    def _assign(self, X, delta):
        check_is_fitted(self)
        data = as_data(X, device=self.device)
        if data.d != self.n_features_in_:
            raise ValueError(f"X has {data.d} features, but {type(self).__name__} is expecting "
                             f"{self.n_features_in_} features as input.")
        C = torch.as_tensor(self.cluster_centers_).to(data.device)
        seed = seed_from_random_state(self.random_state)
        eng = LloydEngine(data.X, self.n_clusters, delta=delta,
                          true_distance_estimate=self.true_distance_estimate and delta > 0,
                          seed=seed, comm=data.comm, row_offset=data.row_offset,
                          gemm_precision=self._precision(),
                          ipe_Q=self.ipe_Q if self.ipe_Q is not None else median_repetitions(0.1))
        eng.restart = 0xFF
        labels, mind, inertia = eng.estep(C)
        return labels, mind, inertia, data

    def predict(self, X, sample_weight=None, delta=None):
        """Closest centre (delta=None/0) or delta-band / IPE estimate."""
        labels, _, _, _ = self._assign(X, 0.0 if delta is None else float(delta))
        return to_numpy(labels).astype(np.int32)

    def score(self, X, y=None, sample_weight=None):
        """Opposite of the inertia of X on the fitted centres."""
        labels, mind, inertia, data = self._assign(X, 0.0)
        if sample_weight is not None:
            w = torch.as_tensor(np.asarray(sample_weight, dtype=np.float64)).to(mind.device)
            val = (mind.double() * w).sum().reshape(1)
        else:
            val = inertia.double().reshape(1).clone()
        data.comm.all_reduce_(val)
        return -float(val.item())

    def transform(self, X):
        """Euclidean distances to the centres (classical path, like the reference)."""
        check_is_fitted(self)
        data = check_n_features(self, as_data(X, device=self.device))
        C = torch.as_tensor(self.cluster_centers_).to(data.device)
        Xf = data.X.double() if data.device.type == "cpu" else data.X.float()
        D = K.distances_torch(Xf, C.to(Xf.dtype))
        return to_numpy(torch.sqrt(D))

    def fit_transform(self, X, y=None, sample_weight=None):
        return self.fit(X, sample_weight=sample_weight).transform(X)

    def fit_predict(self, X, y=None, sample_weight=None):
        return self.fit(X, sample_weight=sample_weight).labels_

    # -------------------------------------------------------- cost model
    def runtime_comparison(self, n_samples, n_features, saveas=None, well_clusterable=False,
                           plot=False):
        """Quantum vs classical running time on a 100x100 (n, m) grid
        (``_dmeans.py:1412-1469``); returns (q_runtime, c_runtime)."""
        check_is_fitted(self)
        n, m = np.meshgrid(np.linspace(0, n_samples, dtype=np.int64, num=100),
                           np.linspace(0, n_features, dtype=np.int64, num=100))
        q, c = cost_model.qmeans_runtime(self.n_clusters, self.n_init, self.eta,
                                         self.condition_number, self.muA, self._delta(), n, m,
                                         well_clusterable)
        if plot:
            cost_model.plot_runtime(n, m, q, c, "k_means VS q_means", saveas)
        return q, c

    def _more_tags(self):
        return {"non_deterministic": False,
                "_xfail_checks": {"check_sample_weights_invariance":
                                  "zero sample_weight is not equivalent to removing samples"}}


# reference class name (``sklearn.cluster.qMeans_``)
qMeans_ = QMeans
