"""Gaussian-process kernels (reference ``gaussian_process/kernels.py``).

Hyperparameters are declared per kernel and exposed in log space through
``theta`` / ``bounds`` in alphabetical order of their names (the
reference's ``dir()``-sorted convention), with analytic gradients with
respect to log-hyperparameters for every kernel except ``PairwiseKernel``
and general-nu ``Matern`` (finite differences, as the reference).
Kernel algebra: ``k1 + k2`` (Sum), ``k1 * k2`` (Product), ``k ** p``
(Exponentiation), scalars promote to ``ConstantKernel``.
"""

import math
from collections import namedtuple
from inspect import signature

import numpy as np
from scipy.spatial.distance import cdist, pdist, squareform
from scipy.special import gamma as gamma_fn
from scipy.special import kv


class Hyperparameter(namedtuple("Hyperparameter",
                                ("name", "value_type", "bounds", "n_elements", "fixed"))):
    __slots__ = ()

    def __new__(cls, name, value_type, bounds, n_elements=1, fixed=None):
        if not isinstance(bounds, str) or bounds != "fixed":
            bounds = np.atleast_2d(bounds)
            if n_elements > 1:
                if bounds.shape[0] == 1:
                    bounds = np.repeat(bounds, n_elements, 0)
                elif bounds.shape[0] != n_elements:
                    raise ValueError("Bounds on %s should have either 1 or %d dimensions. Given "
                                     "are %d" % (name, n_elements, bounds.shape[0]))
        if fixed is None:
            fixed = isinstance(bounds, str) and bounds == "fixed"
        return super().__new__(cls, name, value_type, bounds, n_elements, fixed)

    def __eq__(self, other):
        return (self.name == other.name and self.value_type == other.value_type
                and np.all(self.bounds == other.bounds) and self.n_elements == other.n_elements
                and self.fixed == other.fixed)


def _approx_fprime(xk, f, epsilon):
    f0 = f(xk)
    grad = np.zeros((f0.shape[0], f0.shape[1], len(xk)))
    ei = np.zeros(len(xk))
    for k in range(len(xk)):
        ei[k] = 1.0
        d = epsilon * ei
        grad[:, :, k] = (f(xk + d) - f0) / d[k]
        ei[k] = 0.0
    return grad


class Kernel:
    """Base class: parameter handling, theta/bounds and kernel algebra."""

    def get_params(self, deep=True):
        params = {}
        cls = self.__class__
        init = getattr(cls.__init__, "deprecated_original", cls.__init__)
        for p in signature(init).parameters.values():
            if p.name == "self" or p.kind in (p.VAR_KEYWORD, p.VAR_POSITIONAL):
                continue
            params[p.name] = getattr(self, p.name)
        return params

    def set_params(self, **params):
        if not params:
            return self
        valid = self.get_params(deep=True)
        for key, value in params.items():
            split = key.split("__", 1)
            if len(split) > 1:
                name, sub = split
                if name not in valid:
                    raise ValueError("Invalid parameter %s for kernel %s." % (name, self))
                getattr(self, name).set_params(**{sub: value})
            else:
                if key not in valid:
                    raise ValueError("Invalid parameter %s for kernel %s." % (key, self))
                setattr(self, key, value)
        return self

    def clone_with_theta(self, theta):
        from copy import deepcopy
        c = deepcopy(self)
        c.theta = theta
        return c

    @property
    def n_dims(self):
        return self.theta.shape[0]

    @property
    def hyperparameters(self):
        return [getattr(self, a) for a in dir(self) if a.startswith("hyperparameter_")]

    @property
    def theta(self):
        theta = []
        params = self.get_params()
        for hp in self.hyperparameters:
            if not hp.fixed:
                theta.append(params[hp.name])
        return np.log(np.hstack(theta)) if theta else np.array([])

    @theta.setter
    def theta(self, theta):
        params = self.get_params()
        i = 0
        for hp in self.hyperparameters:
            if hp.fixed:
                continue
            if hp.n_elements > 1:
                params[hp.name] = np.exp(theta[i:i + hp.n_elements])
                i += hp.n_elements
            else:
                params[hp.name] = np.exp(theta[i])
                i += 1
        if i != len(theta):
            raise ValueError("theta has not the correct number of entries. Should be %d; given "
                             "are %d" % (i, len(theta)))
        self.set_params(**params)

    @property
    def bounds(self):
        b = [hp.bounds for hp in self.hyperparameters if not hp.fixed]
        return np.log(np.vstack(b)) if b else np.array([]).reshape(0, 2)

    def __add__(self, b):
        return Sum(self, b if isinstance(b, Kernel) else ConstantKernel(b))

    def __radd__(self, b):
        return Sum(b if isinstance(b, Kernel) else ConstantKernel(b), self)

    def __mul__(self, b):
        return Product(self, b if isinstance(b, Kernel) else ConstantKernel(b))

    def __rmul__(self, b):
        return Product(b if isinstance(b, Kernel) else ConstantKernel(b), self)

    def __pow__(self, b):
        return Exponentiation(self, b)

    def __eq__(self, b):
        if type(self) != type(b):
            return False
        pa, pb = self.get_params(), b.get_params()
        for k in set(pa) | set(pb):
            if np.any(pa.get(k, None) != pb.get(k, None)):
                return False
        return True

    def __repr__(self):
        return "{0}({1})".format(self.__class__.__name__,
                                 ", ".join(map("{0:.3g}".format, np.exp(self.theta))))

    def diag(self, X):
        return np.diag(self(X))

    def is_stationary(self):
        return False

    @property
    def requires_vector_input(self):
        return True

    def _check_bounds_params(self):
        list_close = np.isclose(self.bounds, np.atleast_2d(self.theta).T)
        idx = 0
        for hp in self.hyperparameters:
            if hp.fixed:
                continue
            for dim in range(hp.n_elements):
                if list_close[idx, 0]:
                    import warnings
                    from ...exceptions import ConvergenceWarning
                    warnings.warn("The optimal value found for dimension %s of parameter %s is "
                                  "close to the specified lower bound %s. Decreasing the bound "
                                  "and calling fit again may find a better value."
                                  % (dim, hp.name, hp.bounds[dim][0]), ConvergenceWarning)
                elif list_close[idx, 1]:
                    import warnings
                    from ...exceptions import ConvergenceWarning
                    warnings.warn("The optimal value found for dimension %s of parameter %s is "
                                  "close to the specified upper bound %s. Increasing the bound "
                                  "and calling fit again may find a better value."
                                  % (dim, hp.name, hp.bounds[dim][1]), ConvergenceWarning)
                idx += 1


class NormalizedKernelMixin:
    def diag(self, X):
        return np.ones(X.shape[0])


class StationaryKernelMixin:
    def is_stationary(self):
        return True


class GenericKernelMixin:
    @property
    def requires_vector_input(self):
        return False


class CompoundKernel(Kernel):
    def __init__(self, kernels):
        self.kernels = kernels

    def get_params(self, deep=True):
        return dict(kernels=self.kernels)

    @property
    def theta(self):
        return np.hstack([k.theta for k in self.kernels])

    @theta.setter
    def theta(self, theta):
        k_dims = self.k1.n_dims
        for i, k in enumerate(self.kernels):
            k.theta = theta[i * k_dims:(i + 1) * k_dims]

    @property
    def k1(self):
        return self.kernels[0]

    @property
    def bounds(self):
        return np.vstack([k.bounds for k in self.kernels])

    def __call__(self, X, Y=None, eval_gradient=False):
        if eval_gradient:
            K, G = [], []
            for k in self.kernels:
                a, b = k(X, Y, eval_gradient)
                K.append(a[..., np.newaxis])
                G.append(b[..., np.newaxis])
            return np.dstack(K), np.concatenate(G, 3)
        return np.dstack([k(X, Y, eval_gradient)[..., np.newaxis] for k in self.kernels])

    def is_stationary(self):
        return np.all([k.is_stationary() for k in self.kernels])

    def diag(self, X):
        return np.vstack([k.diag(X) for k in self.kernels]).T

    @property
    def requires_vector_input(self):
        return np.any([k.requires_vector_input for k in self.kernels])


class KernelOperator(Kernel):
    def __init__(self, k1, k2):
        self.k1 = k1
        self.k2 = k2

    def get_params(self, deep=True):
        params = dict(k1=self.k1, k2=self.k2)
        if deep:
            params.update(("k1__" + k, v) for k, v in self.k1.get_params().items())
            params.update(("k2__" + k, v) for k, v in self.k2.get_params().items())
        return params

    @property
    def hyperparameters(self):
        r = [Hyperparameter("k1__" + h.name, h.value_type, h.bounds, h.n_elements)
             for h in self.k1.hyperparameters]
        r += [Hyperparameter("k2__" + h.name, h.value_type, h.bounds, h.n_elements)
              for h in self.k2.hyperparameters]
        return r

    @property
    def theta(self):
        return np.append(self.k1.theta, self.k2.theta)

    @theta.setter
    def theta(self, theta):
        n1 = self.k1.n_dims
        self.k1.theta = theta[:n1]
        self.k2.theta = theta[n1:]

    @property
    def bounds(self):
        if self.k1.bounds.size == 0:
            return self.k2.bounds
        if self.k2.bounds.size == 0:
            return self.k1.bounds
        return np.vstack((self.k1.bounds, self.k2.bounds))

    def __eq__(self, b):
        if type(self) != type(b):
            return False
        return (self.k1 == b.k1 and self.k2 == b.k2) or (self.k1 == b.k2 and self.k2 == b.k1)

    def is_stationary(self):
        return self.k1.is_stationary() and self.k2.is_stationary()

    @property
    def requires_vector_input(self):
        return self.k1.requires_vector_input or self.k2.requires_vector_input


class Sum(KernelOperator):
    def __call__(self, X, Y=None, eval_gradient=False):
        if eval_gradient:
            K1, G1 = self.k1(X, Y, eval_gradient=True)
            K2, G2 = self.k2(X, Y, eval_gradient=True)
            return K1 + K2, np.dstack((G1, G2))
        return self.k1(X, Y) + self.k2(X, Y)

    def diag(self, X):
        return self.k1.diag(X) + self.k2.diag(X)

    def __repr__(self):
        return "{0} + {1}".format(self.k1, self.k2)


class Product(KernelOperator):
    def __call__(self, X, Y=None, eval_gradient=False):
        if eval_gradient:
            K1, G1 = self.k1(X, Y, eval_gradient=True)
            K2, G2 = self.k2(X, Y, eval_gradient=True)
            return K1 * K2, np.dstack((G1 * K2[:, :, np.newaxis], G2 * K1[:, :, np.newaxis]))
        return self.k1(X, Y) * self.k2(X, Y)

    def diag(self, X):
        return self.k1.diag(X) * self.k2.diag(X)

    def __repr__(self):
        return "{0} * {1}".format(self.k1, self.k2)


class Exponentiation(Kernel):
    def __init__(self, kernel, exponent):
        self.kernel = kernel
        self.exponent = exponent

    def get_params(self, deep=True):
        params = dict(kernel=self.kernel, exponent=self.exponent)
        if deep:
            params.update(("kernel__" + k, v) for k, v in self.kernel.get_params().items())
        return params

    @property
    def hyperparameters(self):
        return [Hyperparameter("kernel__" + h.name, h.value_type, h.bounds, h.n_elements)
                for h in self.kernel.hyperparameters]

    @property
    def theta(self):
        return self.kernel.theta

    @theta.setter
    def theta(self, theta):
        self.kernel.theta = theta

    @property
    def bounds(self):
        return self.kernel.bounds

    def __eq__(self, b):
        return type(self) == type(b) and self.kernel == b.kernel and self.exponent == b.exponent

    def __call__(self, X, Y=None, eval_gradient=False):
        if eval_gradient:
            K, G = self.kernel(X, Y, eval_gradient=True)
            G = G * (self.exponent * K[:, :, np.newaxis] ** (self.exponent - 1))
            return K ** self.exponent, G
        return self.kernel(X, Y) ** self.exponent

    def diag(self, X):
        return self.kernel.diag(X) ** self.exponent

    def __repr__(self):
        return "{0} ** {1}".format(self.kernel, self.exponent)

    def is_stationary(self):
        return self.kernel.is_stationary()

    @property
    def requires_vector_input(self):
        return self.kernel.requires_vector_input


class ConstantKernel(StationaryKernelMixin, GenericKernelMixin, Kernel):
    def __init__(self, constant_value=1.0, constant_value_bounds=(1e-5, 1e5)):
        self.constant_value = constant_value
        self.constant_value_bounds = constant_value_bounds

    @property
    def hyperparameter_constant_value(self):
        return Hyperparameter("constant_value", "numeric", self.constant_value_bounds)

    def __call__(self, X, Y=None, eval_gradient=False):
        Y = X if Y is None else Y
        if eval_gradient and Y is not X:
            raise ValueError("Gradient can only be evaluated when Y is None.")
        K = np.full((_num(X), _num(Y)), self.constant_value,
                    dtype=np.array(self.constant_value).dtype)
        if eval_gradient:
            if not self.hyperparameter_constant_value.fixed:
                return K, np.full((_num(X), _num(X), 1), self.constant_value,
                                  dtype=np.array(self.constant_value).dtype)
            return K, np.empty((_num(X), _num(X), 0))
        return K

    def diag(self, X):
        return np.full(_num(X), self.constant_value, dtype=np.array(self.constant_value).dtype)

    def __repr__(self):
        return "{0:.3g}**2".format(np.sqrt(self.constant_value))


C = ConstantKernel


class WhiteKernel(StationaryKernelMixin, GenericKernelMixin, Kernel):
    def __init__(self, noise_level=1.0, noise_level_bounds=(1e-5, 1e5)):
        self.noise_level = noise_level
        self.noise_level_bounds = noise_level_bounds

    @property
    def hyperparameter_noise_level(self):
        return Hyperparameter("noise_level", "numeric", self.noise_level_bounds)

    def __call__(self, X, Y=None, eval_gradient=False):
        if Y is not None and eval_gradient:
            raise ValueError("Gradient can only be evaluated when Y is None.")
        if Y is None:
            K = self.noise_level * np.eye(_num(X))
            if eval_gradient:
                if not self.hyperparameter_noise_level.fixed:
                    return K, self.noise_level * np.eye(_num(X))[:, :, np.newaxis]
                return K, np.empty((_num(X), _num(X), 0))
            return K
        return np.zeros((_num(X), _num(Y)))

    def diag(self, X):
        return np.full(_num(X), self.noise_level, dtype=np.array(self.noise_level).dtype)

    def __repr__(self):
        return "{0}(noise_level={1:.3g})".format(self.__class__.__name__, self.noise_level)


def _num(X):
    return X.shape[0] if hasattr(X, "shape") else len(X)


def _check_ls(X, ls):
    if np.ndim(ls) > 1:
        raise ValueError("length_scale cannot be of dimension greater than 1")
    if np.ndim(ls) == 1 and X.shape[1] != ls.shape[0]:
        raise ValueError("Anisotropic kernel must have the same number of dimensions as data "
                         "(%d!=%d)" % (ls.shape[0], X.shape[1]))
    return np.squeeze(ls).astype(float)


class RBF(StationaryKernelMixin, NormalizedKernelMixin, Kernel):
    def __init__(self, length_scale=1.0, length_scale_bounds=(1e-5, 1e5)):
        self.length_scale = length_scale
        self.length_scale_bounds = length_scale_bounds

    @property
    def anisotropic(self):
        return np.iterable(self.length_scale) and len(self.length_scale) > 1

    @property
    def hyperparameter_length_scale(self):
        if self.anisotropic:
            return Hyperparameter("length_scale", "numeric", self.length_scale_bounds,
                                  len(self.length_scale))
        return Hyperparameter("length_scale", "numeric", self.length_scale_bounds)

    def __call__(self, X, Y=None, eval_gradient=False):
        X = np.atleast_2d(X)
        ls = _check_ls(X, np.asarray(self.length_scale))
        if Y is None:
            d = pdist(X / ls, metric="sqeuclidean")
            K = np.exp(-0.5 * d)
            K = squareform(K)
            np.fill_diagonal(K, 1)
        else:
            if eval_gradient:
                raise ValueError("Gradient can only be evaluated when Y is None.")
            K = np.exp(-0.5 * cdist(X / ls, Y / ls, metric="sqeuclidean"))
        if not eval_gradient:
            return K
        if self.hyperparameter_length_scale.fixed:
            return K, np.empty((X.shape[0], X.shape[0], 0))
        if not self.anisotropic or ls.shape[0] == 1:
            return K, (K * squareform(d))[:, :, np.newaxis]
        G = (X[:, np.newaxis, :] - X[np.newaxis, :, :]) ** 2 / (ls ** 2)
        return K, G * K[..., np.newaxis]

    def __repr__(self):
        if self.anisotropic:
            return "{0}(length_scale=[{1}])".format(
                self.__class__.__name__, ", ".join(map("{0:.3g}".format, self.length_scale)))
        return "{0}(length_scale={1:.3g})".format(self.__class__.__name__,
                                                   np.ravel(self.length_scale)[0])


class Matern(RBF):
    def __init__(self, length_scale=1.0, length_scale_bounds=(1e-5, 1e5), nu=1.5):
        super().__init__(length_scale, length_scale_bounds)
        self.nu = nu

    def __call__(self, X, Y=None, eval_gradient=False):
        X = np.atleast_2d(X)
        ls = _check_ls(X, np.asarray(self.length_scale))
        if Y is None:
            dists = pdist(X / ls, metric="euclidean")
        else:
            if eval_gradient:
                raise ValueError("Gradient can only be evaluated when Y is None.")
            dists = cdist(X / ls, Y / ls, metric="euclidean")
        nu = self.nu
        if nu == 0.5:
            K = np.exp(-dists)
        elif nu == 1.5:
            K = dists * math.sqrt(3)
            K = (1.0 + K) * np.exp(-K)
        elif nu == 2.5:
            K = dists * math.sqrt(5)
            K = (1.0 + K + K ** 2 / 3.0) * np.exp(-K)
        elif nu == np.inf:
            K = np.exp(-dists ** 2 / 2.0)
        else:
            K = dists.copy()
            K[K == 0.0] += np.finfo(float).eps
            tmp = math.sqrt(2 * nu) * K
            K.fill((2 ** (1.0 - nu)) / gamma_fn(nu))
            K *= tmp ** nu
            K *= kv(nu, tmp)
        if Y is None:
            K = squareform(K)
            np.fill_diagonal(K, 1)
        if not eval_gradient:
            return K
        if self.hyperparameter_length_scale.fixed:
            return K, np.empty((X.shape[0], X.shape[0], 0))
        if self.anisotropic:
            D = (X[:, np.newaxis, :] - X[np.newaxis, :, :]) ** 2 / (ls ** 2)
        else:
            D = squareform(dists ** 2)[:, :, np.newaxis]
        if nu == 0.5:
            denom = np.sqrt(D.sum(axis=2))[:, :, np.newaxis]
            with np.errstate(divide="ignore", invalid="ignore"):
                G = K[..., np.newaxis] * D / denom
            G[~np.isfinite(G)] = 0
        elif nu == 1.5:
            G = 3 * D * np.exp(-np.sqrt(3 * D.sum(-1)))[..., np.newaxis]
        elif nu == 2.5:
            tmp = np.sqrt(5 * D.sum(-1))[..., np.newaxis]
            G = 5.0 / 3.0 * D * (tmp + 1) * np.exp(-tmp)
        elif nu == np.inf:
            G = D * K[..., np.newaxis]
        else:
            def f(theta):
                return self.clone_with_theta(theta)(X, Y)
            return K, _approx_fprime(self.theta, f, 1e-10)
        if not self.anisotropic:
            return K, G[:, :].sum(-1)[:, :, np.newaxis]
        return K, G

    def __repr__(self):
        if self.anisotropic:
            return "{0}(length_scale=[{1}], nu={2:.3g})".format(
                self.__class__.__name__, ", ".join(map("{0:.3g}".format, self.length_scale)),
                self.nu)
        return "{0}(length_scale={1:.3g}, nu={2:.3g})".format(
            self.__class__.__name__, np.ravel(self.length_scale)[0], self.nu)


class RationalQuadratic(StationaryKernelMixin, NormalizedKernelMixin, Kernel):
    def __init__(self, length_scale=1.0, alpha=1.0, length_scale_bounds=(1e-5, 1e5),
                 alpha_bounds=(1e-5, 1e5)):
        self.length_scale = length_scale
        self.alpha = alpha
        self.length_scale_bounds = length_scale_bounds
        self.alpha_bounds = alpha_bounds

    @property
    def hyperparameter_length_scale(self):
        return Hyperparameter("length_scale", "numeric", self.length_scale_bounds)

    @property
    def hyperparameter_alpha(self):
        return Hyperparameter("alpha", "numeric", self.alpha_bounds)

    def __call__(self, X, Y=None, eval_gradient=False):
        if len(np.atleast_1d(self.length_scale)) > 1:
            raise AttributeError("RationalQuadratic kernel only supports isotropic version, "
                                 "please use a single scalar for length_scale")
        X = np.atleast_2d(X)
        if Y is None:
            dists = squareform(pdist(X, metric="sqeuclidean"))
            tmp = dists / (2 * self.alpha * self.length_scale ** 2)
            base = 1 + tmp
            K = base ** -self.alpha
            np.fill_diagonal(K, 1)
        else:
            if eval_gradient:
                raise ValueError("Gradient can only be evaluated when Y is None.")
            K = (1 + cdist(X, Y, metric="sqeuclidean")
                 / (2 * self.alpha * self.length_scale ** 2)) ** -self.alpha
        if not eval_gradient:
            return K
        if not self.hyperparameter_length_scale.fixed:
            lsg = (dists * K / (self.length_scale ** 2 * base))[:, :, np.newaxis]
        else:
            lsg = np.empty((K.shape[0], K.shape[1], 0))
        if not self.hyperparameter_alpha.fixed:
            ag = K * (-self.alpha * np.log(base) + dists / (2 * self.length_scale ** 2 * base))
            ag = ag[:, :, np.newaxis]
        else:
            ag = np.empty((K.shape[0], K.shape[1], 0))
        return K, np.dstack((ag, lsg))

    def __repr__(self):
        return "{0}(alpha={1:.3g}, length_scale={2:.3g})".format(
            self.__class__.__name__, self.alpha, self.length_scale)


class ExpSineSquared(StationaryKernelMixin, NormalizedKernelMixin, Kernel):
    def __init__(self, length_scale=1.0, periodicity=1.0, length_scale_bounds=(1e-5, 1e5),
                 periodicity_bounds=(1e-5, 1e5)):
        self.length_scale = length_scale
        self.periodicity = periodicity
        self.length_scale_bounds = length_scale_bounds
        self.periodicity_bounds = periodicity_bounds

    @property
    def hyperparameter_length_scale(self):
        return Hyperparameter("length_scale", "numeric", self.length_scale_bounds)

    @property
    def hyperparameter_periodicity(self):
        return Hyperparameter("periodicity", "numeric", self.periodicity_bounds)

    def __call__(self, X, Y=None, eval_gradient=False):
        X = np.atleast_2d(X)
        if Y is None:
            dists = squareform(pdist(X, metric="euclidean"))
            arg = np.pi * dists / self.periodicity
            s = np.sin(arg)
            K = np.exp(-2 * (s / self.length_scale) ** 2)
        else:
            if eval_gradient:
                raise ValueError("Gradient can only be evaluated when Y is None.")
            dists = cdist(X, Y, metric="euclidean")
            K = np.exp(-2 * (np.sin(np.pi / self.periodicity * dists) / self.length_scale) ** 2)
        if not eval_gradient:
            return K
        if not self.hyperparameter_length_scale.fixed:
            lsg = (4 / self.length_scale ** 2 * s ** 2 * K)[:, :, np.newaxis]
        else:
            lsg = np.empty((K.shape[0], K.shape[1], 0))
        if not self.hyperparameter_periodicity.fixed:
            pg = (4 * arg / self.length_scale ** 2 * np.cos(arg) * s * K)[:, :, np.newaxis]
        else:
            pg = np.empty((K.shape[0], K.shape[1], 0))
        return K, np.dstack((lsg, pg))

    def __repr__(self):
        return "{0}(length_scale={1:.3g}, periodicity={2:.3g})".format(
            self.__class__.__name__, self.length_scale, self.periodicity)


class DotProduct(Kernel):
    def __init__(self, sigma_0=1.0, sigma_0_bounds=(1e-5, 1e5)):
        self.sigma_0 = sigma_0
        self.sigma_0_bounds = sigma_0_bounds

    @property
    def hyperparameter_sigma_0(self):
        return Hyperparameter("sigma_0", "numeric", self.sigma_0_bounds)

    def __call__(self, X, Y=None, eval_gradient=False):
        X = np.atleast_2d(X)
        if Y is None:
            K = X @ X.T + self.sigma_0 ** 2
        else:
            if eval_gradient:
                raise ValueError("Gradient can only be evaluated when Y is None.")
            K = X @ Y.T + self.sigma_0 ** 2
        if not eval_gradient:
            return K
        if not self.hyperparameter_sigma_0.fixed:
            G = np.empty((K.shape[0], K.shape[1], 1))
            G[..., 0] = 2 * self.sigma_0 ** 2
            return K, G
        return K, np.empty((X.shape[0], X.shape[0], 0))

    def diag(self, X):
        return np.einsum("ij,ij->i", X, X) + self.sigma_0 ** 2

    def is_stationary(self):
        return False

    def __repr__(self):
        return "{0}(sigma_0={1:.3g})".format(self.__class__.__name__, self.sigma_0)


class PairwiseKernel(Kernel):
    def __init__(self, gamma=1.0, gamma_bounds=(1e-5, 1e5), metric="linear",
                 pairwise_kernels_kwargs=None):
        self.gamma = gamma
        self.gamma_bounds = gamma_bounds
        self.metric = metric
        self.pairwise_kernels_kwargs = pairwise_kernels_kwargs

    @property
    def hyperparameter_gamma(self):
        return Hyperparameter("gamma", "numeric", self.gamma_bounds)

    def _k(self, X, Y, gamma):
        from ...utils.pairwise import pairwise_kernels
        kw = dict(self.pairwise_kernels_kwargs or {})
        from ..decomposition._extra import _KERNEL_PARAMS
        if "gamma" in _KERNEL_PARAMS.get(self.metric, ("gamma",)) or callable(self.metric):
            kw["gamma"] = gamma
        K = pairwise_kernels(X, Y, metric=self.metric, **kw)
        return np.asarray(K.detach().cpu().numpy() if hasattr(K, "detach") else K,
                          dtype=np.float64)

    def __call__(self, X, Y=None, eval_gradient=False):
        X = np.atleast_2d(X)
        K = self._k(X, Y, self.gamma)
        if not eval_gradient:
            return K
        if self.hyperparameter_gamma.fixed:
            return K, np.empty((X.shape[0], X.shape[0], 0))
        return K, _approx_fprime(self.theta, lambda g: self._k(X, Y, np.exp(g)[0]), 1e-10)

    def diag(self, X):
        return np.apply_along_axis(self, 1, X).ravel()

    def is_stationary(self):
        return self.metric in ["rbf"]

    def __repr__(self):
        return "{0}(gamma={1}, metric={2})".format(self.__class__.__name__, self.gamma,
                                                   self.metric)


__all__ = ["Hyperparameter", "Kernel", "CompoundKernel", "Sum", "Product", "Exponentiation",
           "ConstantKernel", "WhiteKernel", "RBF", "Matern", "RationalQuadratic",
           "ExpSineSquared", "DotProduct", "PairwiseKernel", "NormalizedKernelMixin",
           "StationaryKernelMixin", "GenericKernelMixin"]
