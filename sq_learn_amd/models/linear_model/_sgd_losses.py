"""Loss-function objects of the SGD family (reference
``linear_model/_sgd_fast.pyx:38-360``: ``Hinge``, ``SquaredHinge``, ``Log``,
``ModifiedHuber``, ``SquaredLoss``, ``Huber``, ``EpsilonInsensitive``,
``SquaredEpsilonInsensitive``).

The training loops themselves run natively (``csrc/host/sgd.cpp`` evaluates
the same losses inline per sample); these objects are the public, picklable
description of a loss: ``loss(p, y)`` / ``dloss(p, y)`` (and the reference's
``py_loss`` / ``py_dloss`` names) for a prediction ``p`` and target ``y``
(+-1 for the classification losses).  ``SGDClassifier.loss_function_`` and
``SGDRegressor.loss_function_`` hold one."""

import math


class LossFunction:
    """Base class: a loss of the prediction p and the true value y."""

    def loss(self, p, y):
        raise NotImplementedError

    def dloss(self, p, y):
        raise NotImplementedError

    def py_loss(self, p, y):
        return self.loss(float(p), float(y))

    def py_dloss(self, p, y):
        return self.dloss(float(p), float(y))

    def _args(self):
        return ()

    def __reduce__(self):
        return self.__class__, self._args()

    def __repr__(self):
        return f"{self.__class__.__name__}({', '.join(repr(a) for a in self._args())})"

    def __eq__(self, other):
        return type(self) is type(other) and self._args() == other._args()

    def __hash__(self):
        return hash((type(self).__name__,) + self._args())


class Regression(LossFunction):
    """Base class of the regression losses."""


class Classification(LossFunction):
    """Base class of the classification losses (y in {-1, +1})."""


class ModifiedHuber(Classification):
    """Quadratically smoothed hinge: 0 for z = p y >= 1, (1 - z)^2 for
    -1 <= z < 1, -4 z below (Zhang 2004)."""

    def loss(self, p, y):
        z = p * y
        if z >= 1.0:
            return 0.0
        if z >= -1.0:
            return (1.0 - z) * (1.0 - z)
        return -4.0 * z

    def dloss(self, p, y):
        z = p * y
        if z >= 1.0:
            return 0.0
        if z >= -1.0:
            return 2.0 * (1.0 - z) * -y
        return -4.0 * y


class Hinge(Classification):
    """max(0, threshold - p y): threshold 1 is the SVM loss, 0 the
    perceptron's."""

    def __init__(self, threshold=1.0):
        self.threshold = float(threshold)

    def _args(self):
        return (self.threshold,)

    def loss(self, p, y):
        z = p * y
        return self.threshold - z if z <= self.threshold else 0.0

    def dloss(self, p, y):
        return -y if p * y <= self.threshold else 0.0


class SquaredHinge(Classification):
    """max(0, threshold - p y)^2."""

    def __init__(self, threshold=1.0):
        self.threshold = float(threshold)

    def _args(self):
        return (self.threshold,)

    def loss(self, p, y):
        z = self.threshold - p * y
        return z * z if z > 0 else 0.0

    def dloss(self, p, y):
        z = self.threshold - p * y
        return -2.0 * y * z if z > 0 else 0.0


class Log(Classification):
    """Logistic loss log(1 + exp(-p y)), evaluated without overflow (the
    asymptotes beyond |z| = 18)."""

    def loss(self, p, y):
        z = p * y
        if z > 18.0:
            return math.exp(-z)
        if z < -18.0:
            return -z
        return math.log1p(math.exp(-z))

    def dloss(self, p, y):
        z = p * y
        if z > 18.0:
            return math.exp(-z) * -y
        if z < -18.0:
            return -y
        return -y / (math.exp(z) + 1.0)


class SquaredLoss(Regression):
    """(p - y)^2 / 2."""

    def loss(self, p, y):
        return 0.5 * (p - y) * (p - y)

    def dloss(self, p, y):
        return p - y


class Huber(Regression):
    """Squared loss for |p - y| <= c, linear (slope c) beyond."""

    def __init__(self, c):
        self.c = float(c)

    def _args(self):
        return (self.c,)

    def loss(self, p, y):
        r = p - y
        a = abs(r)
        if a <= self.c:
            return 0.5 * r * r
        return self.c * a - 0.5 * self.c * self.c

    def dloss(self, p, y):
        r = p - y
        if abs(r) <= self.c:
            return r
        return self.c if r > 0.0 else -self.c


class EpsilonInsensitive(Regression):
    """max(0, |y - p| - epsilon) (support vector regression)."""

    def __init__(self, epsilon):
        self.epsilon = float(epsilon)

    def _args(self):
        return (self.epsilon,)

    def loss(self, p, y):
        r = abs(y - p) - self.epsilon
        return r if r > 0 else 0.0

    def dloss(self, p, y):
        if y - p > self.epsilon:
            return -1.0
        if p - y > self.epsilon:
            return 1.0
        return 0.0


class SquaredEpsilonInsensitive(Regression):
    """max(0, |y - p| - epsilon)^2."""

    def __init__(self, epsilon):
        self.epsilon = float(epsilon)

    def _args(self):
        return (self.epsilon,)

    def loss(self, p, y):
        r = abs(y - p) - self.epsilon
        return r * r if r > 0 else 0.0

    def dloss(self, p, y):
        z = y - p
        if z > self.epsilon:
            return -2.0 * (z - self.epsilon)
        if z < -self.epsilon:
            return 2.0 * (-z - self.epsilon)
        return 0.0


def make_loss(name, param=None):
    """Loss object of an SGD loss name (``param``: threshold / epsilon /
    Huber c where the loss has one)."""
    if name == "hinge":
        return Hinge(1.0 if param is None else param)
    if name == "perceptron":
        return Hinge(0.0)
    if name == "squared_hinge":
        return SquaredHinge(1.0 if param is None else param)
    if name in ("log", "log_loss"):
        return Log()
    if name == "modified_huber":
        return ModifiedHuber()
    if name in ("squared_error", "squared_loss"):
        return SquaredLoss()
    if name == "huber":
        return Huber(0.1 if param is None else param)
    if name == "epsilon_insensitive":
        return EpsilonInsensitive(0.1 if param is None else param)
    if name == "squared_epsilon_insensitive":
        return SquaredEpsilonInsensitive(0.1 if param is None else param)
    raise ValueError(f"The loss {name} is not supported.")


__all__ = ["LossFunction", "Regression", "Classification", "Hinge", "SquaredHinge", "Log",
           "ModifiedHuber", "SquaredLoss", "Huber", "EpsilonInsensitive",
           "SquaredEpsilonInsensitive"]
