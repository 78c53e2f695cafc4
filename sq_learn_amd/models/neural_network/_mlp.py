"""Multi-layer perceptrons and the Bernoulli RBM (reference
``neural_network/_multilayer_perceptron.py``, ``_stochastic_optimizers.py``,
``_base.py``, ``_rbm.py``).

The network lives on the resolved device as torch tensors (fp64 by default
for parity; ``dtype=torch.float32`` halves the traffic): forward pass,
back-propagation and the SGD / Adam updates are device kernels, while the
initialisation, mini-batch shuffles and validation splits draw from the
NumPy RandomState exactly as the reference, so the same seed trains the same
network.  L-BFGS packs the parameters and drives scipy's optimiser with
device gradients.
"""

import warnings
from abc import ABCMeta, abstractmethod

import numpy as np
import scipy.optimize
import scipy.sparse as sp
import torch

from ...base import BaseEstimator, ClassifierMixin, RegressorMixin, TransformerMixin
from ...exceptions import ConvergenceWarning
from ...runtime.device import resolve_device
from ...utils.validation import check_is_fitted, check_random_state

_STOCHASTIC = ("sgd", "adam")


def _np(X):
    if hasattr(X, "detach"):
        X = X.detach().cpu().numpy()
    return X.toarray() if sp.issparse(X) else np.asarray(X)


def _act(name, Z):
    if name == "identity":
        return Z
    if name == "logistic":
        return torch.sigmoid(Z)
    if name == "tanh":
        return torch.tanh(Z)
    if name == "relu":
        return torch.clamp(Z, min=0)
    if name == "softmax":
        return torch.softmax(Z, dim=1)
    raise ValueError(name)


def _dact(name, A, delta):
    if name == "logistic":
        return delta * A * (1 - A)
    if name == "tanh":
        return delta * (1 - A ** 2)
    if name == "relu":
        return delta.masked_fill(A == 0, 0.0)
    return delta


class _SGD:
    def __init__(self, params, lr, schedule, momentum, nesterov, power_t):
        self.learning_rate_init = lr
        self.learning_rate = float(lr)
        self.lr_schedule = schedule
        self.momentum = momentum
        self.nesterov = nesterov
        self.power_t = power_t
        self.velocities = [torch.zeros_like(p) for p in params]

    def update(self, params, grads):
        upd = [self.momentum * v - self.learning_rate * g for v, g in zip(self.velocities, grads)]
        self.velocities = upd
        if self.nesterov:
            upd = [self.momentum * v - self.learning_rate * g for v, g in zip(self.velocities,
                                                                               grads)]
        for p, u in zip(params, upd):
            p += u

    def iteration_ends(self, t):
        if self.lr_schedule == "invscaling":
            self.learning_rate = float(self.learning_rate_init) / (t + 1) ** self.power_t

    def trigger_stopping(self):
        if self.lr_schedule != "adaptive":
            return True
        if self.learning_rate <= 1e-6:
            return True
        self.learning_rate /= 5.0
        return False


class _Adam:
    def __init__(self, params, lr, b1, b2, eps):
        self.learning_rate_init = lr
        self.learning_rate = float(lr)
        self.beta_1, self.beta_2, self.epsilon = b1, b2, eps
        self.t = 0
        self.ms = [torch.zeros_like(p) for p in params]
        self.vs = [torch.zeros_like(p) for p in params]

    def update(self, params, grads):
        self.t += 1
        self.ms = [self.beta_1 * m + (1 - self.beta_1) * g for m, g in zip(self.ms, grads)]
        self.vs = [self.beta_2 * v + (1 - self.beta_2) * g * g for v, g in zip(self.vs, grads)]
        self.learning_rate = self.learning_rate_init * np.sqrt(1 - self.beta_2 ** self.t) / \
            (1 - self.beta_1 ** self.t)
        for p, m, v in zip(params, self.ms, self.vs):
            p += -self.learning_rate * m / (torch.sqrt(v) + self.epsilon)

    def iteration_ends(self, t):
        pass

    def trigger_stopping(self):
        return True


class BaseMultilayerPerceptron(BaseEstimator, metaclass=ABCMeta):
    def _device(self):
        return resolve_device(getattr(self, "device", None))

    def _t(self, a):
        return torch.as_tensor(np.ascontiguousarray(a), dtype=torch.float64,
                               device=self._device())

    def _init_coef(self, fan_in, fan_out):
        factor = 2.0 if self.activation == "logistic" else 6.0
        b = np.sqrt(factor / (fan_in + fan_out))
        c = self._random_state.uniform(-b, b, (fan_in, fan_out))
        i = self._random_state.uniform(-b, b, fan_out)
        return c, i

    def _initialize(self, y, units):
        self.n_iter_ = 0
        self.t_ = 0
        self.n_outputs_ = y.shape[1]
        self.n_layers_ = len(units)
        if not isinstance(self, ClassifierMixin):
            self.out_activation_ = "identity"
        elif self._label_binarizer.y_type_ == "multiclass":
            self.out_activation_ = "softmax"
        else:
            self.out_activation_ = "logistic"
        self._W, self._b = [], []
        for i in range(self.n_layers_ - 1):
            c, b = self._init_coef(units[i], units[i + 1])
            self._W.append(self._t(c))
            self._b.append(self._t(b))
        if self.solver in _STOCHASTIC:
            self.loss_curve_ = []
            self._no_improvement_count = 0
            if self.early_stopping:
                self.validation_scores_ = []
                self.best_validation_score_ = -np.inf
            else:
                self.best_loss_ = np.inf

    @property
    def coefs_(self):
        return [w.cpu().numpy() for w in self._W]

    @coefs_.setter
    def coefs_(self, v):
        self._W = [self._t(a) for a in v]

    @property
    def intercepts_(self):
        return [b.cpu().numpy() for b in self._b]

    @intercepts_.setter
    def intercepts_(self, v):
        self._b = [self._t(a) for a in v]

    def __getstate__(self):
        s = super().__getstate__()
        if "_W" in s:
            s["_W"] = [np.asarray(w) if not hasattr(w, "cpu") else w.cpu().numpy()
                       for w in self.__dict__["_W"]]
            s["_b"] = [np.asarray(b) if not hasattr(b, "cpu") else b.cpu().numpy()
                       for b in self.__dict__["_b"]]
        s.pop("_optimizer", None)
        return s

    def __setstate__(self, state):
        super().__setstate__(state)
        if "_W" in state:
            self._W = [self._t(w) for w in state["_W"]]
            self._b = [self._t(b) for b in state["_b"]]

    def _forward(self, X):
        acts = [X]
        for i in range(self.n_layers_ - 1):
            Z = acts[-1] @ self._W[i] + self._b[i]
            last = i + 1 == self.n_layers_ - 1
            acts.append(_act(self.out_activation_ if last else self.activation, Z))
        return acts

    def _loss(self, y, out, n):
        eps = np.finfo(np.float64).eps
        if isinstance(self, ClassifierMixin):
            p = out.clamp(eps, 1 - eps)
            if self.out_activation_ == "logistic":
                loss = -(torch.xlogy(y, p).sum() + torch.xlogy(1 - y, 1 - p).sum()) / p.shape[0]
            else:
                if p.shape[1] == 1:
                    p = torch.cat([1 - p, p], 1)
                yy = torch.cat([1 - y, y], 1) if y.shape[1] == 1 else y
                loss = -torch.xlogy(yy, p).sum() / p.shape[0]
        else:
            loss = ((y - out) ** 2).mean() / 2
        reg = sum((w * w).sum() for w in self._W)
        return loss + (0.5 * self.alpha) * reg / n

    def _backprop(self, X, y):
        n = X.shape[0]
        acts = self._forward(X)
        loss = self._loss(y, acts[-1], n)
        L = self.n_layers_ - 2
        delta = acts[-1] - y
        gW = [None] * (L + 1)
        gb = [None] * (L + 1)
        for i in range(L, -1, -1):
            gW[i] = (acts[i].T @ delta + self.alpha * self._W[i]) / n
            gb[i] = delta.mean(0)
            if i > 0:
                delta = _dact(self.activation, acts[i], delta @ self._W[i].T)
        return float(loss), gW, gb

    @abstractmethod
    def _validate(self, X, y, incremental, reset):
        """Validate X / y and encode the targets."""

    def _fit(self, X, y, incremental=False):
        hls = self.hidden_layer_sizes
        hls = [hls] if np.isscalar(hls) else list(hls)
        if any(h <= 0 for h in hls):
            raise ValueError("hidden_layer_sizes must be > 0, got %s." % hls)
        self._check_params()
        first = not hasattr(self, "_W") or (not self.warm_start and not incremental)
        X, y = self._validate(X, y, incremental, reset=first)
        n, d = X.shape
        if y.ndim == 1:
            y = y.reshape((-1, 1))
        self.n_outputs_ = y.shape[1]
        self.n_features_in_ = d
        units = [d] + hls + [self.n_outputs_]
        self._random_state = check_random_state(self.random_state)
        if not hasattr(self, "_W") or (not self.warm_start and not incremental):
            self._initialize(y, units)
        if self.solver in _STOCHASTIC:
            self._fit_stochastic(X, y, incremental)
        else:
            self._fit_lbfgs(X, y, units)
        if not all(bool(torch.isfinite(w).all()) for w in self._W + self._b):
            raise ValueError("Solver produced non-finite parameter weights. The input data may "
                             "contain large values and need to be preprocessed.")
        return self

    def _check_params(self):
        if self.max_iter <= 0:
            raise ValueError("max_iter must be > 0, got %s." % self.max_iter)
        if self.alpha < 0.0:
            raise ValueError("alpha must be >= 0, got %s." % self.alpha)
        if self.learning_rate_init <= 0.0:
            raise ValueError("learning_rate_init must be > 0, got %s." % self.learning_rate)
        if self.activation not in ("identity", "logistic", "tanh", "relu"):
            raise ValueError("The activation '%s' is not supported." % self.activation)
        if self.learning_rate not in ("constant", "invscaling", "adaptive"):
            raise ValueError("learning rate %s is not supported. " % self.learning_rate)
        if self.solver not in ("sgd", "adam", "lbfgs"):
            raise ValueError("The solver %s is not supported. " % self.solver)

    def _fit_lbfgs(self, X, y, units):
        shapes = [(units[i], units[i + 1]) for i in range(len(units) - 1)]
        sizes = [a * b for a, b in shapes] + [b for _, b in shapes]
        Xt, yt = self._t(X), self._t(y)

        def unpack(p):
            out, o = [], 0
            for s in sizes:
                out.append(p[o:o + s])
                o += s
            k = len(shapes)
            self._W = [self._t(out[i].reshape(shapes[i])) for i in range(k)]
            self._b = [self._t(out[k + i]) for i in range(k)]

        def fg(p):
            unpack(p)
            loss, gW, gb = self._backprop(Xt, yt)
            g = torch.cat([w.reshape(-1) for w in gW] + [b.reshape(-1) for b in gb])
            return loss, g.cpu().numpy()

        p0 = np.hstack([w.cpu().numpy().ravel() for w in self._W]
                       + [b.cpu().numpy().ravel() for b in self._b])
        res = scipy.optimize.minimize(fg, p0, method="L-BFGS-B", jac=True,
                                      options={"maxfun": self.max_fun, "maxiter": self.max_iter,
                                               "iprint": -1, "gtol": self.tol})
        if res.status != 0:
            warnings.warn("lbfgs failed to converge (status=%d): %s" % (res.status, res.message),
                          ConvergenceWarning)
        self.n_iter_ = min(res.nit, self.max_iter)
        self.loss_ = res.fun
        unpack(res.x)

    def _fit_stochastic(self, X, y, incremental):
        params = self._W + self._b
        if not incremental or not hasattr(self, "_optimizer"):
            if self.solver == "sgd":
                self._optimizer = _SGD(params, self.learning_rate_init, self.learning_rate,
                                       self.momentum, self.nesterovs_momentum, self.power_t)
            else:
                self._optimizer = _Adam(params, self.learning_rate_init, self.beta_1,
                                        self.beta_2, self.epsilon)
        early = self.early_stopping and not incremental
        Xv = yv = None
        if early:
            from ...model_selection import train_test_split
            strat = y if isinstance(self, ClassifierMixin) and self.n_outputs_ == 1 else None
            X, Xv, y, yv = train_test_split(X, y, random_state=self._random_state,
                                            test_size=self.validation_fraction, stratify=strat)
            if isinstance(self, ClassifierMixin):
                yv = self._label_binarizer.inverse_transform(yv)
        n = X.shape[0]
        idx = np.arange(n, dtype=int)
        bs = min(200, n) if self.batch_size == "auto" else int(np.clip(self.batch_size, 1, n))
        if self.batch_size != "auto" and (self.batch_size < 1 or self.batch_size > n):
            warnings.warn("Got `batch_size` less than 1 or larger than sample size. It is going "
                          "to be clipped")
        Xt, yt = self._t(X), self._t(y)
        for _ in range(self.max_iter):
            if self.shuffle:
                perm = np.arange(n)
                self._random_state.shuffle(perm)
                idx = idx[perm]
            it_idx = torch.as_tensor(idx, device=Xt.device)
            acc = 0.0
            for s in range(0, n, bs):
                bi = it_idx[s:s + bs]
                xb, yb = (Xt[bi], yt[bi]) if self.shuffle else (Xt[s:s + bs], yt[s:s + bs])
                loss, gW, gb = self._backprop(xb, yb)
                acc += loss * xb.shape[0]
                self._optimizer.update(params, gW + gb)
            self.n_iter_ += 1
            self.loss_ = acc / n
            self.t_ += n
            self.loss_curve_.append(self.loss_)
            self._update_no_improvement(early, Xv, yv)
            self._optimizer.iteration_ends(self.t_)
            if self._no_improvement_count > self.n_iter_no_change:
                if self._optimizer.trigger_stopping():
                    break
                self._no_improvement_count = 0
            if incremental:
                break
            if self.n_iter_ == self.max_iter:
                warnings.warn("Stochastic Optimizer: Maximum iterations (%d) reached and the "
                              "optimization hasn't converged yet." % self.max_iter,
                              ConvergenceWarning)
        if early:
            self._W = [w.clone() for w in self._best_W]
            self._b = [b.clone() for b in self._best_b]

    def _update_no_improvement(self, early, Xv, yv):
        if early:
            self.validation_scores_.append(self.score(Xv, yv))
            last = self.validation_scores_[-1]
            self._no_improvement_count = self._no_improvement_count + 1 \
                if last < self.best_validation_score_ + self.tol else 0
            if last > self.best_validation_score_:
                self.best_validation_score_ = last
                self._best_W = [w.clone() for w in self._W]
                self._best_b = [b.clone() for b in self._b]
        else:
            last = self.loss_curve_[-1]
            self._no_improvement_count = self._no_improvement_count + 1 \
                if last > self.best_loss_ - self.tol else 0
            if last < self.best_loss_:
                self.best_loss_ = last

    def _forward_fast(self, X):
        check_is_fitted(self, "_W")
        X = np.asarray(_np(X), dtype=np.float64)
        if X.shape[1] != self.n_features_in_:
            raise ValueError("X has %d features, but %s is expecting %d features as input."
                             % (X.shape[1], type(self).__name__, self.n_features_in_))
        with torch.no_grad():
            return self._forward(self._t(X))[-1].cpu().numpy()

    def fit(self, X, y):
        return self._fit(X, y, incremental=False)


class MLPClassifier(ClassifierMixin, BaseMultilayerPerceptron):
    def __init__(self, hidden_layer_sizes=(100,), activation="relu", *, solver="adam",
                 alpha=0.0001, batch_size="auto", learning_rate="constant",
                 learning_rate_init=0.001, power_t=0.5, max_iter=200, shuffle=True,
                 random_state=None, tol=1e-4, verbose=False, warm_start=False, momentum=0.9,
                 nesterovs_momentum=True, early_stopping=False, validation_fraction=0.1,
                 beta_1=0.9, beta_2=0.999, epsilon=1e-8, n_iter_no_change=10, max_fun=15000):
        self.hidden_layer_sizes = hidden_layer_sizes
        self.activation = activation
        self.solver = solver
        self.alpha = alpha
        self.batch_size = batch_size
        self.learning_rate = learning_rate
        self.learning_rate_init = learning_rate_init
        self.power_t = power_t
        self.max_iter = max_iter
        self.shuffle = shuffle
        self.random_state = random_state
        self.tol = tol
        self.verbose = verbose
        self.warm_start = warm_start
        self.momentum = momentum
        self.nesterovs_momentum = nesterovs_momentum
        self.early_stopping = early_stopping
        self.validation_fraction = validation_fraction
        self.beta_1 = beta_1
        self.beta_2 = beta_2
        self.epsilon = epsilon
        self.n_iter_no_change = n_iter_no_change
        self.max_fun = max_fun

    def _validate(self, X, y, incremental, reset):
        from ...preprocessing import LabelBinarizer
        X = np.asarray(_np(X), dtype=np.float64)
        y = np.asarray(_np(y))
        if y.ndim == 2 and y.shape[1] == 1:
            y = y.ravel()
        if (not hasattr(self, "classes_")) or (not self.warm_start and not incremental):
            self._label_binarizer = LabelBinarizer()
            self._label_binarizer.fit(y)
            self.classes_ = self._label_binarizer.classes_
        else:
            classes = np.unique(y)
            if self.warm_start and set(classes) != set(self.classes_):
                raise ValueError("warm_start can only be used where `y` has the same classes as "
                                 "in the previous call to fit. Previously got %s, `y` has %s"
                                 % (self.classes_, classes))
            if not self.warm_start and np.setdiff1d(classes, self.classes_).size:
                raise ValueError("`y` has classes not in `self.classes_`. `self.classes_` has "
                                 "%s. 'y' has %s." % (self.classes_, classes))
        y = np.asarray(self._label_binarizer.transform(y)).astype(bool).astype(np.float64)
        return X, y

    def predict(self, X):
        p = self._forward_fast(X)
        if self.n_outputs_ == 1:
            p = p.ravel()
        return self._label_binarizer.inverse_transform(p)

    def partial_fit(self, X, y, classes=None):
        if self.solver not in _STOCHASTIC:
            raise AttributeError("partial_fit is only available for stochastic optimizer. %s is "
                                 "not stochastic" % self.solver)
        if not hasattr(self, "classes_"):
            from ...preprocessing import LabelBinarizer
            if classes is None:
                raise ValueError("classes must be passed on the first call to partial_fit.")
            self._label_binarizer = LabelBinarizer()
            self._label_binarizer.fit(classes)
            self.classes_ = self._label_binarizer.classes_
            self.warm_start = self.warm_start
        return self._fit(X, y, incremental=True)

    def predict_proba(self, X):
        p = self._forward_fast(X)
        if self.n_outputs_ == 1:
            p = p.ravel()
        if p.ndim == 1:
            return np.vstack([1 - p, p]).T
        return p

    def predict_log_proba(self, X):
        return np.log(self.predict_proba(X))


class MLPRegressor(RegressorMixin, BaseMultilayerPerceptron):
    def __init__(self, hidden_layer_sizes=(100,), activation="relu", *, solver="adam",
                 alpha=0.0001, batch_size="auto", learning_rate="constant",
                 learning_rate_init=0.001, power_t=0.5, max_iter=200, shuffle=True,
                 random_state=None, tol=1e-4, verbose=False, warm_start=False, momentum=0.9,
                 nesterovs_momentum=True, early_stopping=False, validation_fraction=0.1,
                 beta_1=0.9, beta_2=0.999, epsilon=1e-8, n_iter_no_change=10, max_fun=15000):
        MLPClassifier.__init__(self, hidden_layer_sizes, activation, solver=solver, alpha=alpha,
                               batch_size=batch_size, learning_rate=learning_rate,
                               learning_rate_init=learning_rate_init, power_t=power_t,
                               max_iter=max_iter, shuffle=shuffle, random_state=random_state,
                               tol=tol, verbose=verbose, warm_start=warm_start,
                               momentum=momentum, nesterovs_momentum=nesterovs_momentum,
                               early_stopping=early_stopping,
                               validation_fraction=validation_fraction, beta_1=beta_1,
                               beta_2=beta_2, epsilon=epsilon, n_iter_no_change=n_iter_no_change,
                               max_fun=max_fun)

    def _validate(self, X, y, incremental, reset):
        X = np.asarray(_np(X), dtype=np.float64)
        y = np.asarray(_np(y), dtype=np.float64)
        if y.ndim == 2 and y.shape[1] == 1:
            y = y.ravel()
        return X, y

    def predict(self, X):
        p = self._forward_fast(X)
        return p.ravel() if p.shape[1] == 1 else p

    def partial_fit(self, X, y):
        if self.solver not in _STOCHASTIC:
            raise AttributeError("partial_fit is only available for stochastic optimizer. %s is "
                                 "not stochastic" % self.solver)
        return self._fit(X, y, incremental=True)


# --------------------------------------------------------------------- RBM
def _gen_even_slices(n, n_packs, n_samples=None):
    start = 0
    for k in range(n_packs):
        m = n // n_packs + (1 if k < n % n_packs else 0)
        if m > 0:
            end = start + m
            if n_samples is not None:
                end = min(n_samples, end)
            yield slice(start, end, None)
            start = end


class BernoulliRBM(TransformerMixin, BaseEstimator):
    """Bernoulli restricted Boltzmann machine trained with persistent
    contrastive divergence."""

    def __init__(self, n_components=256, *, learning_rate=0.1, batch_size=10, n_iter=10,
                 verbose=0, random_state=None):
        self.n_components = n_components
        self.learning_rate = learning_rate
        self.batch_size = batch_size
        self.n_iter = n_iter
        self.verbose = verbose
        self.random_state = random_state

    def _mean_hiddens(self, v):
        from scipy.special import expit
        p = np.asarray(v @ self.components_.T) + self.intercept_hidden_
        return expit(p)

    def _sample_hiddens(self, v, rng):
        p = self._mean_hiddens(v)
        return rng.random_sample(size=p.shape) < p

    def _sample_visibles(self, h, rng):
        from scipy.special import expit
        p = expit(h @ self.components_ + self.intercept_visible_)
        return rng.random_sample(size=p.shape) < p

    def _free_energy(self, v):
        return -np.asarray(v @ self.intercept_visible_).ravel() - np.logaddexp(
            0, np.asarray(v @ self.components_.T) + self.intercept_hidden_).sum(axis=1)

    def gibbs(self, v):
        check_is_fitted(self, "components_")
        if not hasattr(self, "random_state_"):
            self.random_state_ = check_random_state(self.random_state)
        h = self._sample_hiddens(v, self.random_state_)
        return self._sample_visibles(h, self.random_state_)

    def _fit(self, v, rng):
        hp = self._mean_hiddens(v)
        vn = self._sample_visibles(self.h_samples_, rng)
        hn = self._mean_hiddens(vn)
        lr = float(self.learning_rate) / v.shape[0]
        upd = np.asarray(v.T @ hp).T
        upd -= hn.T @ vn
        self.components_ += lr * upd
        self.intercept_hidden_ += lr * (hp.sum(axis=0) - hn.sum(axis=0))
        self.intercept_visible_ += lr * (np.asarray(v.sum(axis=0)).squeeze() - vn.sum(axis=0))
        hn[rng.uniform(size=hn.shape) < hn] = 1.0
        self.h_samples_ = np.floor(hn, hn)

    def partial_fit(self, X, y=None):
        X = X.tocsr() if sp.issparse(X) else np.asarray(_np(X), dtype=np.float64)
        if not hasattr(self, "random_state_"):
            self.random_state_ = check_random_state(self.random_state)
        if not hasattr(self, "components_"):
            self.components_ = np.asarray(self.random_state_.normal(
                0, 0.01, (self.n_components, X.shape[1])), order="F")
            self._n_features_out = self.components_.shape[0]
            self.n_features_in_ = X.shape[1]
        if not hasattr(self, "intercept_hidden_"):
            self.intercept_hidden_ = np.zeros(self.n_components)
        if not hasattr(self, "intercept_visible_"):
            self.intercept_visible_ = np.zeros(X.shape[1])
        if not hasattr(self, "h_samples_"):
            self.h_samples_ = np.zeros((self.batch_size, self.n_components))
        self._fit(X, self.random_state_)
        return self

    def fit(self, X, y=None):
        X = X.tocsr() if sp.issparse(X) else np.asarray(_np(X), dtype=np.float64)
        n = X.shape[0]
        self.n_features_in_ = X.shape[1]
        rng = check_random_state(self.random_state)
        self.components_ = np.asarray(rng.normal(0, 0.01, (self.n_components, X.shape[1])),
                                      order="F")
        self._n_features_out = self.components_.shape[0]
        self.intercept_hidden_ = np.zeros(self.n_components)
        self.intercept_visible_ = np.zeros(X.shape[1])
        self.h_samples_ = np.zeros((self.batch_size, self.n_components))
        nb = int(np.ceil(float(n) / self.batch_size))
        slices = list(_gen_even_slices(nb * self.batch_size, nb, n_samples=n))
        for _ in range(self.n_iter):
            for s in slices:
                self._fit(X[s], rng)
        return self

    def transform(self, X):
        check_is_fitted(self, "components_")
        X = X.tocsr() if sp.issparse(X) else np.asarray(_np(X), dtype=np.float64)
        if X.shape[1] != self.n_features_in_:
            raise ValueError("X has %d features, but BernoulliRBM is expecting %d features as "
                             "input." % (X.shape[1], self.n_features_in_))
        return self._mean_hiddens(X)

    def score_samples(self, X):
        check_is_fitted(self, "components_")
        v = X.tocsr() if sp.issparse(X) else np.asarray(_np(X), dtype=np.float64)
        rng = check_random_state(self.random_state)
        ind = (np.arange(v.shape[0]), rng.randint(0, v.shape[1], v.shape[0]))
        if sp.issparse(v):
            data = -2 * np.asarray(v[ind]).ravel() + 1
            v_ = v + sp.csr_matrix((data, ind), shape=v.shape)
        else:
            v_ = v.copy()
            v_[ind] = 1 - v_[ind]
        fe, fe_ = self._free_energy(v), self._free_energy(v_)
        return v.shape[1] * -np.logaddexp(0, -(fe_ - fe))


__all__ = ["MLPClassifier", "MLPRegressor", "BernoulliRBM"]
