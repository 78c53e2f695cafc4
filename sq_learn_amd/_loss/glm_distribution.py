"""Exponential dispersion models of the GLM regressors (reference
``sklearn/_loss/glm_distribution.py``): unit variance v(mu), unit deviance
d(y, mu) and its mu-derivative, summed deviances.  Host NumPy - the GLM
solvers evaluate these on O(n) vectors per L-BFGS step."""

import numbers
from abc import ABCMeta, abstractmethod

import numpy as np
from scipy.special import xlogy


class ExponentialDispersionModel(metaclass=ABCMeta):
    """Base of the Tweedie family: subclasses define ``unit_variance`` and
    ``unit_deviance``; the derivative, sums and the y-range test follow."""

    def in_y_range(self, y):
        y = np.asarray(y)
        lo, inclusive = self._lower_bound
        return np.greater_equal(y, lo) if inclusive else np.greater(y, lo)

    @abstractmethod
    def unit_variance(self, y_pred):
        """v(mu)"""

    @abstractmethod
    def unit_deviance(self, y, y_pred, check_input=False):
        """d(y, mu) >= 0, zero at y == mu"""

    def unit_deviance_derivative(self, y, y_pred):
        """d d(y, mu) / d mu = -2 (y - mu) / v(mu)"""
        return -2 * (y - y_pred) / self.unit_variance(y_pred)

    def deviance(self, y, y_pred, weights=1):
        return np.sum(weights * self.unit_deviance(y, y_pred))

    def deviance_derivative(self, y, y_pred, weights=1):
        return weights * self.unit_deviance_derivative(y, y_pred)


class TweedieDistribution(ExponentialDispersionModel):
    """Var[Y] proportional to mu^power: power 0 normal, 1 Poisson, 2 gamma,
    3 inverse Gaussian, (1, 2) compound Poisson-gamma; no distribution for
    0 < power < 1."""

    def __init__(self, power=0):
        self.power = power

    @property
    def power(self):
        return self._power

    @power.setter
    def power(self, power):
        if not isinstance(power, numbers.Real):
            raise TypeError("power must be a real number, input was {0}".format(power))
        if power <= 0:
            self._lower_bound = (-np.inf, False)
        elif 0 < power < 1:
            raise ValueError("Tweedie distribution is only defined for power<=0 and power>=1.")
        elif 1 <= power < 2:
            self._lower_bound = (0.0, True)
        else:
            self._lower_bound = (0.0, False)
        self._power = power

    def unit_variance(self, y_pred):
        return np.power(y_pred, self.power)

    def unit_deviance(self, y, y_pred, check_input=False):
        p = self.power
        y = np.asarray(y, dtype=np.float64)
        mu = np.asarray(y_pred, dtype=np.float64)
        if check_input:
            msg = ("Mean Tweedie deviance error with power={} can only be used on ".format(p))
            if p < 0:
                if np.any(mu <= 0):
                    raise ValueError(msg + "strictly positive y_pred.")
            elif p == 0:
                pass
            elif 0 < p < 1:
                raise ValueError("Tweedie deviance is only defined for power<=0 and power>=1.")
            elif 1 <= p < 2:
                if np.any(y < 0) or np.any(mu <= 0):
                    raise ValueError(msg + "non-negative y and strictly positive y_pred.")
            elif np.any(y <= 0) or np.any(mu <= 0):
                raise ValueError(msg + "strictly positive y and y_pred.")
        if p == 0:
            return (y - mu) ** 2
        if p == 1:
            return 2 * (xlogy(y, y / mu) - y + mu)
        if p == 2:
            return 2 * (np.log(mu / y) + y / mu - 1)
        return 2 * (np.power(np.maximum(y, 0), 2 - p) / ((1 - p) * (2 - p))
                    - y * np.power(mu, 1 - p) / (1 - p) + np.power(mu, 2 - p) / (2 - p))


class NormalDistribution(TweedieDistribution):
    def __init__(self):
        super().__init__(power=0)


class PoissonDistribution(TweedieDistribution):
    def __init__(self):
        super().__init__(power=1)


class GammaDistribution(TweedieDistribution):
    def __init__(self):
        super().__init__(power=2)


class InverseGaussianDistribution(TweedieDistribution):
    def __init__(self):
        super().__init__(power=3)


EDM_DISTRIBUTIONS = {"normal": NormalDistribution, "poisson": PoissonDistribution,
                     "gamma": GammaDistribution, "inverse-gaussian": InverseGaussianDistribution}
