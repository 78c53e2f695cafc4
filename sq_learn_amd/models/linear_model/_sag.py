"""SAG / SAGA solvers for Ridge and LogisticRegression (reference
``linear_model/_sag.py``: ``get_auto_step_size`` :20, ``sag_solver`` :89).

The epochs run in the host-native core ``csrc/host/sag.cpp`` (dense rows,
eager weight updates; see there).  The public contract is the reference's:
alpha / beta are scaled by 1 / n_samples, the step size is
``get_auto_step_size``'s, samples are drawn with replacement from a stream
seeded by ``random_state.randint(1, 2**31 - 1)`` (``make_dataset``), the
returned ``warm_start_mem`` carries the coefficients (with the intercept as
the last row when fitted) and ``n_iter_`` counts epochs.
"""

import warnings

import numpy as np
import scipy.sparse as sp

from ...exceptions import ConvergenceWarning
from ...ops import _host
from ...utils.validation import check_random_state

_LOSSES = {"log": 0, "squared": 1, "multinomial": 2}


def get_auto_step_size(max_squared_sum, alpha_scaled, loss, fit_intercept, n_samples=None,
                       is_saga=False):
    """1 / L (SAG) or 1 / (2 L + min(2 n alpha, L)) (SAGA), L the Lipschitz
    constant of the loss gradient over the rows (reference :20-86)."""
    if loss in ("log", "multinomial"):
        L = 0.25 * (max_squared_sum + int(fit_intercept)) + alpha_scaled
    elif loss == "squared":
        L = max_squared_sum + int(fit_intercept) + alpha_scaled
    else:
        raise ValueError("Unknown loss function for SAG solver, got %s instead of 'log' or "
                         "'squared'" % loss)
    if is_saga:
        mun = min(2 * n_samples * alpha_scaled, L)
        return 1.0 / (2 * L + mun)
    return 1.0 / L


def sag_solver(X, y, sample_weight=None, loss="log", alpha=1.0, beta=0.0, max_iter=1000,
               tol=0.001, verbose=0, random_state=None, check_input=True, max_squared_sum=None,
               warm_start_mem=None, is_saga=False, sparse_input=None):
    """Returns (coef_, n_iter_, warm_start_mem) like the reference.
    ``sparse_input`` (callers that densified a sparse X themselves): apply
    the sparse dataset's intercept decay; default: ``sp.issparse(X)``."""
    if warm_start_mem is None:
        warm_start_mem = {}
    if max_iter is None:
        max_iter = 1000
    # sparse input: the reference's make_dataset damps the intercept updates
    # (SPARSE_INTERCEPT_DECAY, linear_model/_base.py:206); the solver runs on
    # the dense rows with that decay
    if sparse_input is None:
        sparse_input = sp.issparse(X)
    intercept_decay = 0.01 if sparse_input else 1.0
    if sp.issparse(X):
        X = X.toarray()
    X = np.ascontiguousarray(X, dtype=np.float64)
    y = np.ascontiguousarray(np.asarray(y, dtype=np.float64).ravel())
    n, d = X.shape
    alpha_scaled = float(alpha) / n
    beta_scaled = float(beta) / n
    K = int(y.max()) + 1 if loss == "multinomial" else 1
    sw = (np.ones(n) if sample_weight is None
          else np.ascontiguousarray(np.broadcast_to(np.asarray(sample_weight, dtype=np.float64),
                                                    (n,))))
    coef_init = warm_start_mem.get("coef")
    if coef_init is None:
        coef_init = np.zeros((d, K))
    coef_init = np.array(coef_init, dtype=np.float64).reshape(-1, K)
    fit_intercept = coef_init.shape[0] == d + 1
    W = np.ascontiguousarray(coef_init[:d])
    b = np.ascontiguousarray(coef_init[d] if fit_intercept else np.zeros(K))
    rng = check_random_state(random_state)
    seed = int(rng.randint(1, np.iinfo(np.int32).max))   # make_dataset's draw
    if max_squared_sum is None:
        max_squared_sum = float(np.einsum("ij,ij->i", X, X).max()) if n else 0.0
    step = get_auto_step_size(max_squared_sum, alpha_scaled, loss, fit_intercept, n_samples=n,
                              is_saga=is_saga)
    if step * alpha_scaled == 1:
        raise ZeroDivisionError("Current sag implementation does not handle the case "
                                "step_size * alpha_scaled == 1")
    if loss not in _LOSSES:
        raise ValueError("Invalid loss parameter: got %r instead of one of %s"
                         % (loss, sorted(_LOSSES)))
    it = _host.lib().sqh_sag(X.ctypes.data, y.ctypes.data, sw.ctypes.data, n, d, K,
                             _LOSSES[loss], alpha_scaled, beta_scaled, step, int(max_iter),
                             float(tol), int(fit_intercept), intercept_decay, int(bool(is_saga)),
                             seed & 0xFFFFFFFF, W.ctypes.data, b.ctypes.data)
    if it < 0:
        raise ValueError("Floating-point under-/overflow occurred at epoch #%d. Scaling input "
                         "data with StandardScaler or MinMaxScaler might help." % (-it))
    if it == max_iter:
        warnings.warn("The max_iter was reached which means the coef_ did not converge",
                      ConvergenceWarning)
    coef_full = np.vstack([W, b[None, :]]) if fit_intercept else W
    mem = {"coef": coef_full, "num_seen": n}
    coef_ = coef_full.T if loss == "multinomial" else coef_full[:, 0]
    return coef_, it, mem


__all__ = ["sag_solver", "get_auto_step_size"]
