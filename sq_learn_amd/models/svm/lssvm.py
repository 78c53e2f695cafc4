"""Least-squares SVM classifiers: classical ``LSSVC`` and quantum-simulated
``QLSSVC``.

References: ``sklearn/svm/_classes.py:1465-1697`` (LSSVC) and
``sklearn/svm/_qSVM.py:10-404`` (QLSSVC).

The (N+1) x (N+1) system F = [[0, 1^T], [1, K + I/penalty]] is built on the
device (kernel matrix = one library GEMM + elementwise epilogue) and solved
by a symmetric eigendecomposition (QLSSVC: the reference's hermitian SVD with
optional low-rank truncation) or, for LSSVC 'cg', by batched conjugate
gradients on H = K + I/penalty.  Prediction is vectorised over test samples
(the reference loops per sample in Python).

Fixed reference defects (§2.8): ``LSSVC._cg_fit`` used the (x, info) tuple
from scipy's cg as an array and had the b / alpha formulas swapped - here
b = 1^T eta / 1^T nu, alpha = eta - nu b with H eta = y, H nu = 1, which
equals the direct solve; ``LSSVC.get_P`` used ||x_i|| in place of ||x_j||^2 -
here it uses QLSSVC's beta = sqrt((N ||x||^2 + 1) Nu).
"""

import math

import numpy as np
import torch

from ...base import BaseEstimator, ClassifierMixin
from ...utils.validation import check_is_fitted, check_array, seed_from_random_state
from ...utils import pairwise as PW
from ...utils.metrics import accuracy_score
from ...runtime.device import resolve_device, to_numpy
from ...runtime.rng import RngKey
from ...ops.random import trunc_normal_add_


class _KernelMixin:
    def _get_gamma(self, X):
        if self.gamma == "scale":
            Xn = to_numpy(X) if isinstance(X, torch.Tensor) else np.asarray(X)
            return 1.0 / (Xn.shape[1] * Xn.var())
        if self.gamma == "auto":
            return 1.0 / self.n_features_in_
        return float(self.gamma)

    def get_kernel(self, X, Y=None):
        """Kernel matrix K(X, Y) on the estimator device (tensor)."""
        dev = self._device()
        Xt = torch.as_tensor(np.asarray(to_numpy(X), dtype=np.float64), device=dev)
        Yt = None if Y is None else torch.as_tensor(np.asarray(to_numpy(Y), dtype=np.float64), device=dev)
        if self.kernel == "linear":
            return PW.linear_kernel(Xt, Yt)
        gamma = self._get_gamma(self._gamma_ref if hasattr(self, "_gamma_ref") else X)
        if self.kernel == "poly":
            return PW.polynomial_kernel(Xt, Yt, degree=self.degree, gamma=gamma, coef0=self.coef0)
        if self.kernel == "rbf":
            return PW.rbf_kernel(Xt, Yt, gamma=gamma)
        if self.kernel == "sigmoid":
            return PW.sigmoid_kernel(Xt, Yt, gamma=gamma, coef0=self.coef0)
        raise ValueError(f"unknown kernel {self.kernel!r}")

    def _device(self):
        dev = resolve_device(getattr(self, "device", None))
        return dev

    def _F(self, X):
        N = X.shape[0]
        K = self.get_kernel(X)
        dev = K.device
        F = torch.zeros((N + 1, N + 1), dtype=torch.float64, device=dev)
        F[0, 1:] = 1.0
        F[1:, 0] = 1.0
        F[1:, 1:] = K.double() + (1.0 / self.penalty) * torch.eye(N, dtype=torch.float64, device=dev)
        return F

    def get_h(self, X):
        check_is_fitted(self, "alpha_")
        Kx = self.get_kernel(self.X, X)
        return (torch.as_tensor(self.alpha_, device=Kx.device).double() @ Kx.double()
                + self.b_).cpu().numpy()

    def _gram_for_gamma(self, X):
        self._gamma_ref = np.asarray(to_numpy(X), dtype=np.float64)


class LSSVC(_KernelMixin, ClassifierMixin, BaseEstimator):
    """Classical least-squares SVM classifier (labels in {-1, +1})."""

    def _more_tags(self):
        return {"binary_only": True}


    def __init__(self, kernel="linear", penalty=0.1, degree=3, gamma="scale", coef0=0.0,
                 verbose=False, algorithm="classic", device=None, cg_tol=1e-10, cg_maxiter=1000):
        self.kernel = kernel
        self.penalty = penalty
        self.degree = degree
        self.gamma = gamma
        self.coef0 = coef0
        self.verbose = verbose
        self.algorithm = algorithm
        self.device = device
        self.cg_tol = cg_tol
        self.cg_maxiter = cg_maxiter

    def _classical_fit(self, X, y):
        F = self._F(X)
        rhs = torch.cat([torch.zeros(1, dtype=torch.float64, device=F.device),
                         torch.as_tensor(y, dtype=torch.float64, device=F.device)])
        sol = torch.linalg.pinv(F, hermitian=True) @ rhs
        return float(sol[0]), sol[1:].cpu().numpy()

    def _cg_fit(self, X, y):
        N = X.shape[0]
        H = self.get_kernel(X).double()
        H = H + (1.0 / self.penalty) * torch.eye(N, dtype=torch.float64, device=H.device)
        B = torch.stack([torch.as_tensor(y, dtype=torch.float64, device=H.device),
                         torch.ones(N, dtype=torch.float64, device=H.device)], 1)
        Z = conjugate_gradient(H, B, tol=self.cg_tol, maxiter=self.cg_maxiter)
        res = (H @ Z - B).norm() / B.norm()
        if not bool(torch.isfinite(Z).all()) or float(res) > 1e-6:
            # H is not SPD (e.g. sigmoid kernel): CG does not apply, solve directly
            Z = torch.linalg.lstsq(H, B).solution
        eta, nu = Z[:, 0], Z[:, 1]
        b = float(eta.sum() / nu.sum())
        alpha = (eta - nu * b).cpu().numpy()
        return b, alpha

    def fit(self, X, y):
        X, y = self._validate_data(X, y)
        X = np.asarray(to_numpy(X), dtype=np.float64)
        y = np.asarray(to_numpy(y), dtype=np.float64)
        self._gram_for_gamma(X)
        self.X = X
        if self.algorithm == "classic":
            self.b_, self.alpha_ = self._classical_fit(X, y)
        elif self.algorithm == "cg":
            self.b_, self.alpha_ = self._cg_fit(X, y)
        else:
            raise ValueError("Algorithm not implemented")
        self.b, self.alpha = self.b_, self.alpha_
        if self.kernel == "linear":
            self.coef_ = self.alpha_ @ X
        self.classes_ = np.array([-1.0, 1.0])
        self.is_fitted_ = True
        return self

    def decision_function(self, X):
        X = check_array(X)
        return self.get_h(X)

    def predict(self, X):
        return np.sign(self.decision_function(X))

    def get_P(self, X):
        X = np.asarray(check_array(X), dtype=np.float64)
        N = self.X.shape[0]
        h = self.get_h(X)
        Nu = self.b_ ** 2 + float(np.sum(self.alpha_ ** 2 * np.sum(self.X ** 2, 1)))
        betas = np.sqrt((N * np.sum(X ** 2, 1) + 1) * Nu)
        return 0.5 * (1 - h / betas), betas


def conjugate_gradient(A, B, tol=1e-10, maxiter=1000):
    """Batched CG for SPD A with several right-hand sides (columns of B)."""
    X = torch.zeros_like(B)
    R = B - A @ X
    P = R.clone()
    rs = (R * R).sum(0)
    b2 = (B * B).sum(0).clamp(min=1e-300)
    for _ in range(maxiter):
        AP = A @ P
        alpha = rs / (P * AP).sum(0).clamp(min=1e-300)
        X = X + P * alpha
        R = R - AP * alpha
        rs_new = (R * R).sum(0)
        if bool((rs_new <= (tol ** 2) * b2).all()):
            break
        P = R + P * (rs_new / rs.clamp(min=1e-300))
        rs = rs_new
    return X


class QLSSVC(_KernelMixin, ClassifierMixin, BaseEstimator):
    """Quantum least-squares SVM (``_qSVM.py:10-404``)."""

    def _more_tags(self):
        return {"binary_only": True}


    def __init__(self, kernel="linear", penalty=0.1, degree=3, gamma="scale", coef0=0.0,
                 verbose=False, algorithm="classic", low_rank=False, var=0.9,
                 error_type="absolute", relative_error=0.5, absolute_error=0.01, train_error=0.01,
                 random_state=None, device=None):
        if error_type not in ("absolute", "relative"):
            raise Exception(r"The error should be either 'absolute' or 'relative'")
        self.kernel = kernel
        self.penalty = penalty
        self.degree = degree
        self.gamma = gamma
        self.coef0 = coef0
        self.verbose = verbose
        self.algorithm = algorithm
        self.low_rank = low_rank
        self.var = var
        self.error_type = error_type
        self.relative_error = relative_error
        self.absolute_error = absolute_error
        self.train_error = train_error
        self.random_state = random_state
        self.device = device

    # -------------------------------------------------------------- fit
    def _classical_fit(self, y):
        """(b, alpha) = F^+ [0; y] with the optional low-rank truncation of
        the hermitian spectrum (``_qSVM.py:84-130``)."""
        F = self._F(self.X)
        lam, Qm = torch.linalg.eigh(F)
        order = torch.argsort(lam.abs(), descending=True)
        lam, Qm = lam[order], Qm[:, order]
        s = lam.abs()
        s_new = torch.zeros_like(s)
        if self.low_rank:
            if 0 <= self.var < 1.0:
                sums = float((s ** 2).sum())
                cum = torch.cumsum(s ** 2, 0) / sums
                idx = int(torch.nonzero(cum >= self.var - 1e-15)[0][0]) if bool((cum >= self.var - 1e-15).any()) else len(s) - 1
            elif self.var >= 1.0:
                idx = int(self.var) - 1
            else:
                raise Exception("QLSSVC.var shoud be greater than 0")
            s_new[:idx + 1] = s[:idx + 1]
            self.cond = float(s_new[0] / s_new[idx])
            self.normF = float(s_new[0])
        else:
            s_new = s.clone()
            self.cond = float(s[0] / s[-1])
            self.normF = float(s[0])
        self.singular_values_F_ = s_new.cpu().numpy()
        inv = torch.where(s_new > 0, 1.0 / s_new.clamp(min=1e-300), torch.zeros_like(s_new))
        sign = torch.sign(lam)
        Finv = (Qm * (inv * sign)) @ Qm.T
        rhs = torch.cat([torch.zeros(1, dtype=torch.float64, device=F.device),
                         torch.as_tensor(y, dtype=torch.float64, device=F.device)])
        sol = Finv @ rhs
        return float(sol[0]), sol[1:].cpu().numpy()

    def fit(self, X, y):
        X, y = self._validate_data(X, y)
        X = np.asarray(to_numpy(X), dtype=np.float64)
        y = np.asarray(to_numpy(y), dtype=np.float64)
        self._gram_for_gamma(X)
        self.X = X
        N = X.shape[0]
        if self.algorithm == "classic":
            self.b_, self.alpha_ = self._classical_fit(y)
        else:
            raise ValueError("Algorithm not implemented")
        self.b, self.alpha = self.b_, self.alpha_
        self.alpha_F = math.sqrt(N) + self.penalty ** -1 + float(np.linalg.norm(X, ord="fro") ** 2)
        self.Nu = self.b_ ** 2 + float(np.sum(self.alpha_ ** 2 * np.sum(X ** 2, 1)))
        if self.kernel == "linear":
            self.coef_ = self.alpha_ @ X
        self.classes_ = np.array([-1.0, 1.0])
        self.is_fitted_ = True
        self._calls = 0
        return self

    # ------------------------------------------------------------ noise
    def _noise(self, bounds):
        """One TN(-b_i, b_i) draw per element (Philox, fresh stream per call)."""
        self._calls = getattr(self, "_calls", 0) + 1
        key = RngKey(seed_from_random_state(self.random_state), "trunc_normal", self._calls)
        bounds = np.asarray(bounds, dtype=np.float64).reshape(-1)
        out = np.empty_like(bounds)
        # one stream, per-element bound: draw uniforms and map with each bound
        from ...runtime.rng import Philox
        from scipy.special import erf, erfinv
        u = Philox(key).uniform_flat(bounds.size, dtype=torch.float64).numpy()
        e = erf(bounds / np.sqrt(2.0))
        out = np.sqrt(2.0) * erfinv((2 * u - 1) * e)
        return np.clip(out, -bounds, bounds)

    def relative_error_routine(self, delta, Xmax, Xreal):
        """Iterative halving (``_qSVM.py:245-261``), vectorised over samples:
        returns (Xhat, delta_r, epsilon_abs) arrays."""
        Xmax = np.atleast_1d(np.asarray(Xmax, dtype=np.float64))
        Xreal = np.broadcast_to(np.asarray(Xreal, dtype=np.float64), Xmax.shape).copy()
        r = np.zeros_like(Xmax)
        Xr = Xmax.copy()
        Xhat = np.zeros_like(Xmax)
        eps_abs = np.zeros_like(Xmax)
        delta_r = np.zeros_like(Xmax)
        active = Xr > Xhat
        for _ in range(200):
            if not active.any():
                break
            r = np.where(active, r + 1.0, r)
            Xr = np.where(active, Xmax / 2 ** r, Xr)
            eps_abs = np.where(active, self.relative_error * Xr / 2, eps_abs)
            delta_r = np.where(active, 6 * delta / (np.pi ** 2 * r ** 2), delta_r)
            draw = Xreal + self._noise(np.where(active, eps_abs, 0.0))
            Xhat = np.where(active, draw, Xhat)
            active = Xr > Xhat
        return Xhat, delta_r, eps_abs

    # ---------------------------------------------------------- predict
    def get_betas(self, X):
        check_is_fitted(self, "alpha_")
        X = np.asarray(to_numpy(X), dtype=np.float64)
        N = len(self.X)
        return np.sqrt((N * np.sum(X ** 2, 1) + 1) * self.Nu)

    def get_h(self, X, approx=False):
        hs = super().get_h(np.asarray(to_numpy(X), dtype=np.float64))
        if approx:
            betas = self.get_betas(X)
            if self.error_type == "absolute":
                hs = hs + self._noise(np.full(hs.shape, self.absolute_error))
            else:
                _, _, ea = self.relative_error_routine(0.1, betas, np.abs(hs))
                hs = hs + self._noise(ea)
        return hs

    def get_P(self, X, approx=False):
        hs = self.get_h(X)
        beta = self.get_betas(X)
        P = 0.5 * (1 - hs / beta)
        if approx:
            if self.error_type == "absolute":
                P = P + self._noise(self.absolute_error / (2 * beta))
            else:
                _, _, ea = self.relative_error_routine(0.1, beta, np.abs(hs))
                P = P + self._noise(ea / (2 * beta))
        return P

    def predict(self, X):
        """+1 if the noisy P(x) <= 1/2 else -1 (``_qSVM.py:178-215``)."""
        check_array(X)
        check_is_fitted(self, "alpha_")
        P = self.get_P(X)
        betas = self.get_betas(X)
        if self.error_type == "absolute":
            P = P + self._noise(self.absolute_error / (2 * betas))
        else:
            h = self.get_h(X)
            _, _, ea = self.relative_error_routine(0.1, betas, np.abs(h))
            P = P + self._noise(ea / (2 * betas))
        return np.where(P <= 0.5, 1.0, -1.0)

    def classical_predict(self, X):
        check_array(X)
        return np.sign(self.get_h(X))

    def get_training_complexity(self):
        return self.cond * self.alpha_F

    def get_classification_complexity(self, X, relative_error=False):
        betas = self.get_betas(X)
        nrm = np.linalg.norm(np.append(self.b_, self.alpha_), ord=2)
        if relative_error:
            hs = np.abs(self.get_h(X))
            return (self.cond * betas * self.alpha_F) / (self.relative_error * hs * self.normF ** 2 * nrm)
        return (self.cond * betas * self.alpha_F) / (self.absolute_error * self.normF ** 2 * nrm)

    def get_approximated_hyperplane(self, x):
        beta = self.get_betas(x)
        ba = np.append(self.b_, self.alpha_)
        if self.error_type == "absolute":
            bound = self.relative_error / beta
        else:
            bound = self.relative_error * np.abs(self.get_h(x)) / beta
        bound = float(np.asarray(bound).reshape(-1)[0])
        approx = ba + self._noise(np.full(ba.shape, bound / np.sqrt(ba.size)))
        return approx[0], approx[1:] @ self.X

    def get_all_attributes(self, X):
        betas = self.get_betas(X)
        hs = self.get_h(X)
        Ps = self.get_P(X)
        rel = (self.cond * (betas - np.abs(hs)) * self.alpha_F) / (np.abs(hs) * np.sqrt(Ps))
        ab = self.cond * betas * self.alpha_F
        return betas, hs, Ps, self.cond, rel, ab

    def score(self, X, y, sample_weight=None):
        check_is_fitted(self, "alpha_")
        return accuracy_score(y, self.predict(X), sample_weight=sample_weight)
