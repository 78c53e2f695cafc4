"""Host NumPy pieces of the reference's MLP and GLM internals kept for API
parity (the estimators themselves train on the device):

  * ``sklearn/neural_network/_base.py``: in-place activations, their
    derivatives, the loss functions;
  * ``sklearn/neural_network/_stochastic_optimizers.py``: BaseOptimizer,
    SGDOptimizer (momentum / Nesterov, constant / invscaling / adaptive
    rates), AdamOptimizer;
  * ``sklearn/linear_model/_glm/link.py``: identity / log / logit links.
"""

import numpy as np
from scipy.special import expit, logit, xlogy


# ------------------------------------------------------------ activations
def inplace_identity(X):
    """identity: nothing to do"""


def inplace_logistic(X):
    expit(X, out=X)


def inplace_tanh(X):
    np.tanh(X, out=X)


def inplace_relu(X):
    np.maximum(X, 0, out=X)


def inplace_softmax(X):
    tmp = X - X.max(axis=1)[:, np.newaxis]
    np.exp(tmp, out=X)
    X /= X.sum(axis=1)[:, np.newaxis]


ACTIVATIONS = {"identity": inplace_identity, "tanh": inplace_tanh,
               "logistic": inplace_logistic, "relu": inplace_relu, "softmax": inplace_softmax}


def inplace_identity_derivative(Z, delta):
    """identity: the backpropagated delta is unchanged"""


def inplace_logistic_derivative(Z, delta):
    delta *= Z
    delta *= 1 - Z


def inplace_tanh_derivative(Z, delta):
    delta *= 1 - Z ** 2


def inplace_relu_derivative(Z, delta):
    delta[Z == 0] = 0


DERIVATIVES = {"identity": inplace_identity_derivative, "tanh": inplace_tanh_derivative,
               "logistic": inplace_logistic_derivative, "relu": inplace_relu_derivative}


# ------------------------------------------------------------ losses
def squared_loss(y_true, y_pred):
    """half mean squared error"""
    return ((y_true - y_pred) ** 2).mean() / 2


def log_loss(y_true, y_prob):
    """cross-entropy of one-hot / multi-label targets"""
    eps = np.finfo(y_prob.dtype).eps
    y_prob = np.clip(y_prob, eps, 1 - eps)
    if y_prob.shape[1] == 1:
        y_prob = np.append(1 - y_prob, y_prob, axis=1)
    if y_true.shape[1] == 1:
        y_true = np.append(1 - y_true, y_true, axis=1)
    return -xlogy(y_true, y_prob).sum() / y_prob.shape[0]


def binary_log_loss(y_true, y_prob):
    """binary cross-entropy"""
    eps = np.finfo(y_prob.dtype).eps
    y_prob = np.clip(y_prob, eps, 1 - eps)
    return -(xlogy(y_true, y_prob) + xlogy(1 - y_true, 1 - y_prob)).sum() / y_prob.shape[0]


LOSS_FUNCTIONS = {"squared_error": squared_loss, "log_loss": log_loss,
                  "binary_log_loss": binary_log_loss}


# ------------------------------------------------------------ optimizers
class BaseOptimizer:
    """Applies the updates of ``_get_updates`` to a list of parameter
    arrays in place."""

    def __init__(self, learning_rate_init=0.1):
        self.learning_rate_init = learning_rate_init
        self.learning_rate = float(learning_rate_init)

    def update_params(self, params, grads):
        updates = self._get_updates(grads)
        for param, update in zip((p for p in params), updates):
            param += update

    def iteration_ends(self, time_step):
        pass

    def trigger_stopping(self, msg, verbose):
        if verbose:
            print(msg + " Stopping.")
        return True


class SGDOptimizer(BaseOptimizer):
    def __init__(self, params, learning_rate_init=0.1, lr_schedule="constant", momentum=0.9,
                 nesterov=True, power_t=0.5):
        super().__init__(learning_rate_init)
        self.lr_schedule = lr_schedule
        self.momentum = momentum
        self.nesterov = nesterov
        self.power_t = power_t
        self.velocities = [np.zeros_like(p) for p in params]

    def iteration_ends(self, time_step):
        if self.lr_schedule == "invscaling":
            self.learning_rate = float(self.learning_rate_init) / (time_step + 1) ** self.power_t

    def trigger_stopping(self, msg, verbose):
        if self.lr_schedule != "adaptive":
            if verbose:
                print(msg + " Stopping.")
            return True
        if self.learning_rate <= 1e-6:
            if verbose:
                print(msg + " Learning rate too small. Stopping.")
            return True
        self.learning_rate /= 5.0
        if verbose:
            print(msg + " Setting learning rate to %f" % self.learning_rate)
        return False

    def _get_updates(self, grads):
        updates = [self.momentum * v - self.learning_rate * g
                   for v, g in zip(self.velocities, grads)]
        self.velocities = updates
        if self.nesterov:
            updates = [self.momentum * v - self.learning_rate * g
                       for v, g in zip(self.velocities, grads)]
        return updates


class AdamOptimizer(BaseOptimizer):
    def __init__(self, params, learning_rate_init=0.001, beta_1=0.9, beta_2=0.999,
                 epsilon=1e-8):
        super().__init__(learning_rate_init)
        self.beta_1 = beta_1
        self.beta_2 = beta_2
        self.epsilon = epsilon
        self.t = 0
        self.ms = [np.zeros_like(p) for p in params]
        self.vs = [np.zeros_like(p) for p in params]

    def _get_updates(self, grads):
        self.t += 1
        self.ms = [self.beta_1 * m + (1 - self.beta_1) * g for m, g in zip(self.ms, grads)]
        self.vs = [self.beta_2 * v + (1 - self.beta_2) * (g ** 2) for v, g in zip(self.vs, grads)]
        self.learning_rate = (self.learning_rate_init * np.sqrt(1 - self.beta_2 ** self.t)
                              / (1 - self.beta_1 ** self.t))
        return [-self.learning_rate * m / (np.sqrt(v) + self.epsilon)
                for m, v in zip(self.ms, self.vs)]


# ------------------------------------------------------------ GLM links
class BaseLink:
    """Link g(mu) = eta with inverse h(eta) = mu and the derivatives the
    GLM solver needs."""

    def __call__(self, y_pred):
        raise NotImplementedError

    def derivative(self, y_pred):
        raise NotImplementedError

    def inverse(self, lin_pred):
        raise NotImplementedError

    def inverse_derivative(self, lin_pred):
        raise NotImplementedError


class IdentityLink(BaseLink):
    def __call__(self, y_pred):
        return y_pred

    def derivative(self, y_pred):
        return np.ones_like(y_pred)

    def inverse(self, lin_pred):
        return lin_pred

    def inverse_derivative(self, lin_pred):
        return np.ones_like(lin_pred)


class LogLink(BaseLink):
    def __call__(self, y_pred):
        return np.log(y_pred)

    def derivative(self, y_pred):
        return 1 / y_pred

    def inverse(self, lin_pred):
        return np.exp(lin_pred)

    def inverse_derivative(self, lin_pred):
        return np.exp(lin_pred)


class LogitLink(BaseLink):
    def __call__(self, y_pred):
        return logit(y_pred)

    def derivative(self, y_pred):
        return 1 / (y_pred * (1 - y_pred))

    def inverse(self, lin_pred):
        return expit(lin_pred)

    def inverse_derivative(self, lin_pred):
        ep = expit(lin_pred)
        return ep * (1 - ep)
