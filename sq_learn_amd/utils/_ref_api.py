"""Smaller public helpers of the reference that live in modules this package
organises differently (each is attached to its reference-layout module by
``utils._aliases.REF_NAMES``).  Host NumPy/SciPy: these are O(n) or O(d^2)
utilities, not hot paths.

Reference locations:
  * ``sklearn/utils/__init__.py`` (axis0_safe_slice, tosequence,
    indices_to_mask, check_matplotlib_support, check_pandas_support)
  * ``sklearn/metrics/pairwise.py`` (check_pairwise_arrays,
    check_paired_arrays, distance_metrics, kernel_metrics)
  * ``sklearn/metrics/cluster/_unsupervised.py`` (check_number_of_labels)
  * ``sklearn/covariance/_robust_covariance.py`` (c_step, select_candidates),
    ``_graph_lasso.py`` (alpha_max, graphical_lasso_path)
  * ``sklearn/decomposition/_nmf.py`` (norm, trace_dot)
  * ``sklearn/cluster/_dmeans.py:727-777, 2252`` (wrapper,
    labels_estimation, select_labels)
  * ``sklearn/QuantumUtility/Utility.py:405-411`` (auxiliary_fun,
    vectorize_aux_fun)
  * ``sklearn/datasets/_base.py`` (load_data), ``_species_distributions.py``
    (construct_grids), ``_twenty_newsgroups.py`` (strip_newsgroup_*),
    ``_openml.py`` (OpenMLError)
  * ``sklearn/utils/_pprint.py`` (KeyValTuple, KeyValTupleParam),
    ``_estimator_html_repr.py`` (estimator_html_repr)
"""

import csv
import html
import itertools
import random
import re
from importlib import resources  # noqa: F401  (load_data's package lookup)
from os.path import join

import numpy as np
import scipy.sparse as sp


# --------------------------------------------------------------- utils
def axis0_safe_slice(X, mask, len_mask):
    """X[mask] that returns an empty (0, n_features) array when the mask
    selects nothing (sparse X does not support empty boolean masks)."""
    if len_mask != 0:
        return X[mask, :]
    return np.zeros(shape=(0, X.shape[1]))


def tosequence(x):
    """x as an indexable sequence: ndarrays are returned as arrays, other
    sequences as is, anything else as a list."""
    if isinstance(x, np.ndarray):
        return np.asarray(x)
    from collections.abc import Sequence
    if isinstance(x, Sequence):
        return x
    return list(x)


def indices_to_mask(indices, mask_length):
    """Boolean mask of ``mask_length`` with True at ``indices``."""
    if mask_length <= np.max(indices):
        raise ValueError("mask_length must be greater than max(indices)")
    mask = np.zeros(mask_length, dtype=bool)
    mask[indices] = True
    return mask


def check_matplotlib_support(caller_name):
    try:
        import matplotlib  # noqa: F401
    except ImportError as e:
        raise ImportError(f"{caller_name} requires matplotlib. You can install matplotlib "
                          "with `pip install matplotlib`") from e


def check_pandas_support(caller_name):
    try:
        import pandas
    except ImportError as e:
        raise ImportError(f"{caller_name} requires pandas.") from e
    return pandas


# ------------------------------------------------------- metrics.pairwise
def _return_float_dtype(X, Y):
    if not sp.issparse(X) and not isinstance(X, np.ndarray):
        X = np.asarray(X)
    if Y is None:
        Y_dtype = X.dtype
    elif not sp.issparse(Y) and not isinstance(Y, np.ndarray):
        Y = np.asarray(Y)
        Y_dtype = Y.dtype
    else:
        Y_dtype = Y.dtype
    dtype = X.dtype if X.dtype == Y_dtype == np.float32 else float
    return X, Y, dtype


def check_pairwise_arrays(X, Y, *, precomputed=False, dtype=None, accept_sparse="csr",
                          force_all_finite=True, copy=False):
    """Validate X and Y (Y=None: Y is X) for a pairwise computation: 2-D,
    float (float32 kept only when both are float32), same n_features; with
    ``precomputed`` X is a distance matrix against Y's rows."""
    from .validation import check_array
    X, Y, dtype_float = _return_float_dtype(X, Y)
    if dtype is None:
        dtype = dtype_float
    kw = dict(accept_sparse=accept_sparse, dtype=dtype, copy=copy,
              force_all_finite=force_all_finite)
    if Y is X or Y is None:
        X = Y = check_array(X, **kw)
    else:
        X = check_array(X, **kw)
        Y = check_array(Y, **kw)
    if precomputed:
        if X.shape[1] != Y.shape[0]:
            raise ValueError("Precomputed metric requires shape (n_queries, n_indexed). Got "
                             f"({X.shape[0]}, {X.shape[1]}) for {Y.shape[0]} indexed.")
    elif X.shape[1] != Y.shape[1]:
        raise ValueError("Incompatible dimension for X and Y matrices: X.shape[1] == "
                         f"{X.shape[1]} while Y.shape[1] == {Y.shape[1]}")
    return X, Y


def check_paired_arrays(X, Y):
    """check_pairwise_arrays plus equal row counts (paired distances)."""
    X, Y = check_pairwise_arrays(X, Y)
    if X.shape != Y.shape:
        raise ValueError("X and Y should be of same shape. They were respectively "
                         f"{X.shape!r} and {Y.shape!r} long.")
    return X, Y


def distance_metrics():
    """The valid metric names of pairwise_distances and their functions."""
    from .pairwise import PAIRWISE_DISTANCE_FUNCTIONS
    return dict(PAIRWISE_DISTANCE_FUNCTIONS)


def kernel_metrics():
    """The valid kernel names of pairwise_kernels and their functions."""
    from .pairwise import PAIRWISE_KERNEL_FUNCTIONS
    return dict(PAIRWISE_KERNEL_FUNCTIONS)


def check_number_of_labels(n_labels, n_samples):
    """Silhouette-style scores need 2 <= n_labels <= n_samples - 1."""
    if not 1 < n_labels < n_samples:
        raise ValueError("Number of labels is %d. Valid values are 2 to n_samples - 1 "
                         "(inclusive)" % n_labels)


# --------------------------------------------------------------- covariance
def c_step(X, n_support, remaining_iterations=30, initial_estimates=None, verbose=False,
           cov_computation_method=None, random_state=None):
    """One concentration-step run of FastMCD: (location, covariance, log
    det, support mask, Mahalanobis distances)."""
    from .validation import check_random_state
    from ..covariance import _c_step
    X = np.asarray(X, dtype=np.float64)
    return _c_step(X, n_support, check_random_state(random_state),
                   remaining_iterations=remaining_iterations, initial_estimates=initial_estimates)


def select_candidates(X, n_support, n_trials, select=1, n_iter=30, verbose=False,
                      cov_computation_method=None, random_state=None):
    """The ``select`` best of ``n_trials`` c-step runs (lowest covariance
    determinant); ``n_trials`` may be a tuple of (locations, covariances)
    initial estimates.  Returns (locations, covariances, supports, dists)."""
    from .validation import check_random_state
    from ..covariance import _c_step
    X = np.asarray(X, dtype=np.float64)
    rs = check_random_state(random_state)
    if isinstance(n_trials, (int, np.integer)):
        runs = [_c_step(X, n_support, rs, remaining_iterations=n_iter) for _ in range(n_trials)]
    else:
        locs, covs = n_trials
        runs = [_c_step(X, n_support, rs, remaining_iterations=n_iter,
                        initial_estimates=(locs[j], covs[j])) for j in range(len(locs))]
    order = np.argsort([r[2] for r in runs], kind="stable")[:select]
    return (np.asarray([runs[j][0] for j in order]), np.asarray([runs[j][1] for j in order]),
            np.asarray([runs[j][3] for j in order]), np.asarray([runs[j][4] for j in order]))


def alpha_max(emp_cov):
    """Smallest alpha at which graphical lasso zeroes every off-diagonal
    entry: the largest off-diagonal |emp_cov|."""
    A = np.array(emp_cov, dtype=np.float64, copy=True)
    A.flat[:: A.shape[0] + 1] = 0
    return np.max(np.abs(A))


def graphical_lasso_path(X, alphas, cov_init=None, X_test=None, mode="cd", tol=1e-4,
                         enet_tol=1e-4, max_iter=100, verbose=False):
    """graphical_lasso along decreasing ``alphas``, each warm-started from the
    previous covariance.  Returns (covariances, precisions) and, with
    ``X_test``, the held-out log-likelihoods as a third list."""
    from ..covariance import empirical_covariance, graphical_lasso, log_likelihood
    emp_cov = empirical_covariance(X)
    covariance_ = emp_cov.copy() if cov_init is None else np.array(cov_init, copy=True)
    test_emp_cov = empirical_covariance(X_test) if X_test is not None else None
    covs, precs, scores = [], [], []
    for alpha in alphas:
        try:
            covariance_, precision_ = graphical_lasso(emp_cov, alpha=alpha, cov_init=covariance_,
                                                      mode=mode, tol=tol, enet_tol=enet_tol,
                                                      max_iter=max_iter)[:2]
            covs.append(covariance_)
            precs.append(precision_)
            if test_emp_cov is not None:
                s = log_likelihood(test_emp_cov, precision_)
        except FloatingPointError:
            s = -np.inf
            covs.append(np.nan)
            precs.append(np.nan)
        if test_emp_cov is not None:
            scores.append(s if np.isfinite(s) else -np.inf)
    if X_test is not None:
        return covs, precs, scores
    return covs, precs


# --------------------------------------------------------------- NMF
def norm(x):
    """Frobenius / l2 norm via a dot product (no copy of x)."""
    x = np.ravel(x, order="K")
    return np.sqrt(np.dot(x, x))


def trace_dot(X, Y):
    """trace(X @ Y.T) without forming the product."""
    return np.dot(np.ravel(X), np.ravel(Y))


# --------------------------------------------------------------- q-means internals
def select_labels(a):
    """A uniformly random member of the delta-band ``a`` (Python ``random``,
    the reference's own stream)."""
    return random.choice(list(a))


def wrapper(sample):
    """ipe() on an (x, y, epsilon, Q) tuple (the reference's process-pool
    task)."""
    from ..quantum.reference import ipe
    return ipe(x=sample[0], y=sample[1], epsilon=sample[2], Q=sample[3])


def labels_estimation(X, centers, delta, pool=None, true_distance_estimate=False):
    """Host delta-means label assignment of the reference (``_dmeans.py:
    732-777``): fp64 squared distances, each row's label drawn uniformly from
    its delta-band (or, with ``true_distance_estimate``, from IPE-estimated
    distances with epsilon = delta / 2, Q = 5).  Returns (labels, distances,
    inertia).  The GPU engine (``models.cluster._lloyd``) is the fast path;
    this is the reference-shaped oracle."""
    from scipy.spatial.distance import cdist
    X = np.asarray(X, dtype=np.float64)
    centers = np.asarray(centers, dtype=np.float64)
    D = np.square(cdist(X, centers, "euclidean"))
    if delta <= 0:
        lab = D.argmin(1)
        return lab, D, float(D[np.arange(len(X)), lab].sum())
    if not true_distance_estimate:
        mins = D.min(1)
        lab = [select_labels(np.where(row <= mins[e] + delta)[0]) for e, row in enumerate(D)]
        return lab, D, float(mins.sum())
    tasks = list(itertools.product(X, centers, [delta / 2], [5]))
    ips = np.array(list(pool.map(wrapper, tasks)) if pool is not None else map(wrapper, tasks),
                   dtype=np.float64).reshape(len(X), len(centers))
    xn = (X ** 2).sum(1)
    cn = (centers ** 2).sum(1)
    De = xn[:, None] + cn[None, :] - 2.0 * ips
    mins = De.min(1)
    lab = [select_labels(np.where(row <= mins[e] + delta)[0]) for e, row in enumerate(De)]
    return lab, De, float(mins.sum())


# --------------------------------------------------------------- QuantumUtility
def auxiliary_fun(q_state, i):
    """``i`` measurements of a QuantumState (tomography helper)."""
    return q_state.measure(n_times=int(i))


def vectorize_aux_fun(dic, i):
    """sqrt of the measured frequency of outcome ``i`` (0 if never seen)."""
    return np.sqrt(dic[i]) if i in dic else 0


# --------------------------------------------------------------- datasets
class OpenMLError(ValueError):
    """HTTP 412 from OpenML (no results for a query); kept for API parity -
    this package has no network access, so fetch_openml never reaches it."""


def load_data(module_path, data_file_name):
    """A packaged CSV whose header row is (n_samples, n_features,
    target names...): returns (data, target, target_names)."""
    with open(join(module_path, "data", data_file_name)) as f:
        data_file = csv.reader(f)
        temp = next(data_file)
        n_samples, n_features = int(temp[0]), int(temp[1])
        target_names = np.array(temp[2:])
        data = np.empty((n_samples, n_features))
        target = np.empty((n_samples,), dtype=int)
        for i, ir in enumerate(data_file):
            data[i] = np.asarray(ir[:-1], dtype=np.float64)
            target[i] = np.asarray(ir[-1], dtype=int)
    return data, target, target_names


def construct_grids(batch):
    """(xgrid, ygrid) cell-centre coordinates of a species-distribution
    coverage batch (x_left_lower_corner, Nx, grid_size, ...)."""
    xmin = batch.x_left_lower_corner + batch.grid_size
    xmax = xmin + (batch.Nx * batch.grid_size)
    ymin = batch.y_left_lower_corner + batch.grid_size
    ymax = ymin + (batch.Ny * batch.grid_size)
    xgrid = np.arange(xmin, xmax, batch.grid_size)
    ygrid = np.arange(ymin, ymax, batch.grid_size)
    return xgrid, ygrid


_QUOTE_RE = re.compile(r"(writes in|writes:|wrote:|says:|said:|^In article|^Quoted from|^\||^>)")


def strip_newsgroup_header(text):
    """Drop everything up to the first blank line (the message headers)."""
    _before, _blank, after = text.partition("\n\n")
    return after


def strip_newsgroup_quoting(text):
    """Drop lines that quote another message."""
    return "\n".join(line for line in text.split("\n") if not _QUOTE_RE.search(line))


def strip_newsgroup_footer(text):
    """Drop a trailing signature block (after the last line of dashes)."""
    lines = text.strip().split("\n")
    for line_num in range(len(lines) - 1, -1, -1):
        line = lines[line_num]
        if line.strip().strip("-") == "":
            break
    if line_num > 0:
        return "\n".join(lines[:line_num])
    return text


class MissingValues(tuple):
    """(nan, none): which missing-value markers a set of categories holds
    (reference ``utils/_encode.py``)."""

    def __new__(cls, nan=False, none=False):
        return super().__new__(cls, (bool(nan), bool(none)))

    nan = property(lambda self: self[0])
    none = property(lambda self: self[1])

    def to_list(self):
        out = []
        if self.none:
            out.append(None)
        if self.nan:
            out.append(np.nan)
        return out


class Sentinel:
    """Default ``out_file`` marker of export_graphviz (reference
    ``tree/_export.py``): prints as the literal default file name."""

    def __repr__(self):
        return '"tree.dot"'


# --------------------------------------------------------------- repr helpers
class KeyValTuple(tuple):
    """A (key, value) pair the estimator pretty-printer renders as k: v."""

    def __repr__(self):
        return super().__repr__()


class KeyValTupleParam(KeyValTuple):
    """A (key, value) pair rendered as k=v (estimator parameters)."""


def estimator_html_repr(estimator):
    """HTML block describing ``estimator``: nested <details> for
    meta-estimators (Pipeline steps, ColumnTransformer transformers,
    estimator / base_estimator parameters), the repr text in <pre>."""
    def block(est, name=None):
        title = html.escape(name + ": " if name else "") + html.escape(type(est).__name__)
        inner = ""
        steps = getattr(est, "steps", None) or getattr(est, "transformers", None)
        if steps:
            inner = "".join(block(s[1], str(s[0])) for s in steps
                            if not isinstance(s[1], str))
        else:
            for attr in ("estimator", "base_estimator", "final_estimator"):
                sub = getattr(est, attr, None)
                if sub is not None and hasattr(sub, "get_params"):
                    inner += block(sub, attr)
        body = f"<pre>{html.escape(repr(est))}</pre>"
        return (f"<div class='sk-item'><details><summary>{title}</summary>{body}"
                f"{inner}</details></div>")
    return f"<div class='sk-top-container'>{block(estimator)}</div>"
