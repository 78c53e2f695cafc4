"""QuantumUtility error model - exact-semantics NumPy oracle (CPU path).

Every routine of the reference's ``sklearn/QuantumUtility/Utility.py``
 with the same arguments, defaults and outcome
distributions, plus an explicit ``random_state`` so results are reproducible
(the reference mixes three unseeded generators - defect §2.8.11).

Deliberate deviations (documented):

* AE / PE draw from the Fejer law with the exact O(1) sampler of
  :mod:`.fejer` instead of enumerating all M bins (``method='exact'``
  enumerates like the reference; both have the same distribution).
* ``make_gaussian_est`` with ``noise == 0`` returns a copy instead of raising
  UnboundLocalError (``Utility.py:97-104``).
* No module side effects: no global ``warnings.simplefilter('always')``, no
  matplotlib import at module load, no ``from multiprocessing import *``
  (``Utility.py:16-23``).  Plots are produced lazily when asked for.
* ``consistent_phase_estimation`` locates the interval analytically instead
  of materialising ``np.arange(-1, 1+eps, eps)`` (2/eps floats) - the
  returned midpoint is identical.
"""

import math
import re
import warnings
from collections import Counter

import numpy as np
from scipy.special import erf, erfinv

from .fejer import (fejer_pmf, fejer_sample, ae_bins, pe_qubits, median_repetitions)

__all__ = [
    "QuantumState", "estimate_wald", "introduce_error", "introduce_error_array",
    "coupon_collect", "make_gaussian_est", "tomography", "create_rand_vec", "mu",
    "linear_search", "best_mu", "L2_tomography_fakeSign", "L2_tomogrphy_fakeSign",
    "real_tomography", "check_measure", "check_division", "amplitude_est_dist",
    "amplitude_estimation", "median_evaluation", "wrapper_phase_est_arguments",
    "unwrap_phase_est_arguments", "phase_estimation", "ipe",
    "consistent_phase_estimation", "truncated_normal", "as_generator",
    "amplitude_estimation_batch", "phase_estimation_batch",
    "consistent_phase_estimation_batch", "ipe_batch", "tomography_rows",
]


def as_generator(random_state=None):
    """numpy Generator from None / int / RandomState / Generator."""
    if isinstance(random_state, np.random.Generator):
        return random_state
    if isinstance(random_state, np.random.RandomState):
        return np.random.default_rng(random_state.randint(0, 2 ** 31 - 1))
    return np.random.default_rng(random_state)


# --------------------------------------------------------------------- Q1/Q2
class QuantumState:
    """Simulated quantum register (reference ``Utility.py:25-58``).

    ``amplitudes`` are normalised; register i is measured with probability
    amplitude_i^2.  ``measure(n)`` samples n outcomes with replacement.
    """

    def __init__(self, registers, amplitudes, random_state=None):
        self.registers = registers
        amps = np.asarray(amplitudes, dtype=np.float64)
        self.norm_factor = math.sqrt(float(np.sum(amps ** 2)))
        self.amplitudes = amps / self.norm_factor
        self.probabilities = self.amplitudes ** 2
        assert len(self.registers) == len(self.amplitudes)
        assert abs(float(self.probabilities.sum()) - 1) < 1e-10
        self._rng = as_generator(random_state)

    def measure(self, n_times=1):
        idx = self._rng.choice(len(self.probabilities), p=self.probabilities, size=n_times)
        regs = self.registers
        if isinstance(regs, np.ndarray) and regs.ndim == 1:
            return regs[idx]
        if all(np.isscalar(r) for r in regs):
            return np.asarray(regs)[idx]
        return [regs[i] for i in idx]

    def measure_counts(self, n_times):
        """Multinomial counts per register (what ``Counter(measure(n))`` gives)."""
        return self._rng.multinomial(int(n_times), self.probabilities / self.probabilities.sum())

    def get_state(self):
        return {self.registers[i]: self.probabilities[i] for i in range(len(self.registers))}


def estimate_wald(measurements):
    """Empirical frequency of each outcome (``Utility.py:61-64``)."""
    if len(measurements) and isinstance(measurements[0], np.ndarray):
        measurements = [tuple(m) for m in measurements]
    counter = Counter(np.asarray(measurements).tolist() if not isinstance(measurements, list) else measurements)
    n = len(measurements)
    return {x: counter[x] / n for x in counter}


# ----------------------------------------------------------------------- Q3
def truncated_normal(bound, size, rng):
    """Standard normal truncated to [-bound, bound] (= scipy ``truncnorm(-b, b)``).

    Inverse CDF: z = sqrt(2) erfinv(v erf(b/sqrt 2)), v ~ U(-1, 1)."""
    bound = np.asarray(bound, dtype=np.float64)
    v = rng.uniform(-1.0, 1.0, size=size)
    e = erf(bound / np.sqrt(2.0))
    z = np.sqrt(2.0) * erfinv(v * e)
    return np.clip(z, -bound, bound)


def introduce_error(value, epsilon, random_state=None):
    """value + TN(-eps, eps) draw (``Utility.py:68-69``); returns shape (1,)."""
    rng = as_generator(random_state)
    return value + truncated_normal(epsilon, 1, rng)


def introduce_error_array(array, norm_error, random_state=None):
    """Per-component TN(-e/sqrt(n), e/sqrt(n)) noise (``Utility.py:71-73``)."""
    rng = as_generator(random_state)
    array = np.asarray(array)
    size = array.shape[0]
    b = norm_error / np.sqrt(size)
    return array + truncated_normal(b, size, rng)


def coupon_collect(quantum_state):
    """Measurements until every register has been seen (``Utility.py:75-85``)."""
    seen = {v: 0 for v in quantum_state.get_state().keys()}
    counter = 0
    while sum(seen.values()) != len(seen):
        value = quantum_state.measure()[0]
        if not seen[value]:
            seen[value] = 1
        counter += 1
    return counter


def make_gaussian_est(vec, noise, random_state=None):
    """Gaussian approximation of tomography (``Utility.py:88-104``): add a
    TN(+-noise/sqrt(len)) draw to every component."""
    vec = np.asarray(vec, dtype=np.float64)
    b = noise / np.sqrt(len(vec))
    if b == 0:
        return vec.copy()
    rng = as_generator(random_state)
    return vec + truncated_normal(b, len(vec), rng)


# ----------------------------------------------------------------------- Q5
def check_measure(arr, faster_measure_increment=0):
    """Make the geomspace shot schedule strictly increasing (``Utility.py:414-422``)."""
    arr = np.array(arr, copy=True)
    incr = 5 + faster_measure_increment
    for i in range(len(arr) - 1):
        if arr[i + 1] == arr[i]:
            arr[i + 1] += incr
        if arr[i + 1] <= arr[i]:
            arr[i + 1] = arr[i] + incr
    return arr


def _tomography_shots(d, delta, norm):
    if norm == "L2":
        return int((36 * d * np.log(d)) / (delta ** 2))
    if norm == "inf":
        return int((36 * np.log(d)) / (delta ** 2))
    raise ValueError("norm must be 'L2' or 'inf'")


def _one_tomography_pass(V, n_shots, rng):
    """Algorithm 4.1 of Kerenidis-Prakash (QIPM) with n_shots measurements:
    magnitudes from |V|^2 sampling, signs from the 2d-outcome state
    1/2(V +- P).  Returns the signed estimate (``Utility.py:323-352``)."""
    d = len(V)
    pv = V ** 2
    pv = pv / pv.sum()
    counts = rng.multinomial(int(n_shots), pv)
    P = np.sqrt(counts / float(n_shots))
    amp = np.concatenate([V + P, V - P]) * 0.5
    p2 = amp ** 2
    p2 = p2 / p2.sum()
    c2 = rng.multinomial(int(n_shots), p2)
    plus = c2[:d]
    return np.where(plus > 0.4 * P ** 2 * n_shots, P, -P)


def real_tomography(V, N=None, delta=None, stop_when_reached_accuracy=True, norm="L2",
                    incremental_measure=True, faster_measure_increment=0, random_state=None):
    """Vector-state tomography (``Utility.py:259-402``).

    Returns ``{n_shots: estimate}``; with ``incremental_measure`` one entry per
    checkpoint of the geomspace(1, N, 100) schedule, stopping at the first
    checkpoint whose estimate is within ``delta`` (L2 or Linf) of the true
    (normalised) V - the reference's oracle stopping rule.
    """
    rng = as_generator(random_state)
    V = np.asarray(V, dtype=np.float64)
    nv = np.linalg.norm(V)
    if not np.isclose(nv, 1, rtol=1e-2):
        V = V / np.linalg.norm(V, ord=2)
    d = len(V)
    if N is None:
        N = _tomography_shots(d, delta, norm)
    res = {}
    if incremental_measure:
        schedule = check_measure(np.geomspace(1, N, num=100, dtype=np.int64), faster_measure_increment)
        for i in schedule:
            est = _one_tomography_pass(V, int(i), rng)
            res[int(i)] = est
            if stop_when_reached_accuracy:
                err = np.linalg.norm(V - est, ord=2 if norm == "L2" else np.inf)
                if err <= delta:
                    break
    else:
        res[int(N)] = _one_tomography_pass(V, int(N), rng)
    return res


def L2_tomography_fakeSign(V, N=None, delta=None, random_state=None):
    """Magnitudes by sampling, signs copied from V (``Utility.py:234-256``)."""
    rng = as_generator(random_state)
    V = np.asarray(V, dtype=np.float64)
    d = len(V)
    if N is None:
        N = (36 * d * np.log(d)) / (delta ** 2)
    p = V ** 2 / np.sum(V ** 2)
    counts = rng.multinomial(int(N), p)
    P = np.sqrt(counts / float(int(N)))
    return list(np.where(V < 0, -P, P))


L2_tomogrphy_fakeSign = L2_tomography_fakeSign  # reference spelling


def tomography(A, noise, true_tomography=True, stop_when_reached_accuracy=True, N=None,
               norm="L2", incremental_measure=True, faster_measure_increment=0,
               random_state=None, preserve_norm=False):
    """Tomography dispatcher (``Utility.py:107-180``).

    ``true_tomography=False``: Gaussian approximation with a Frobenius-style
    budget (matrix flattened, per-component bound noise/sqrt(rows*cols)).
    ``true_tomography=True``: :func:`real_tomography` per row; like the
    reference the estimate is a *unit* vector per row.  ``preserve_norm=True``
    (framework extension) rescales each row estimate by
    the true row norm.
    """
    assert noise >= 0
    if noise == 0:
        return A
    A = np.asarray(A, dtype=np.float64)
    rng = as_generator(random_state)
    if not true_tomography:
        flat = A.reshape(-1)
        return make_gaussian_est(flat, noise, rng).reshape(A.shape)
    rows = A if A.ndim == 2 else A[None, :]
    out = np.empty_like(rows)
    for idx in range(rows.shape[0]):
        r = real_tomography(rows[idx], delta=noise, stop_when_reached_accuracy=stop_when_reached_accuracy,
                            N=N, norm=norm, incremental_measure=incremental_measure,
                            faster_measure_increment=faster_measure_increment, random_state=rng)
        est = np.asarray(list(r.values())[-1])
        if preserve_norm:
            est = est * np.linalg.norm(rows[idx])
        out[idx] = est
    return out if A.ndim == 2 else out[0]


def tomography_rows(A, noise, **kw):
    """Alias used by the estimators: tomography of each row of A."""
    return tomography(A, noise, **kw)


def create_rand_vec(n_vec, len_vec, scale=None, type="uniform", random_state=None):
    """n_vec random unit vectors (``Utility.py:183-193``)."""
    rng = as_generator(random_state)
    out = []
    for _ in range(n_vec):
        if type == "uniform":
            v = rng.uniform(-1, 1, len_vec)
        elif type == "exp":
            v = rng.exponential(scale=scale, size=len_vec)
        else:
            raise ValueError("type must be 'uniform' or 'exp'")
        out.append(v / np.linalg.norm(v, ord=2))
    return out


# ----------------------------------------------------------------------- Q9
def _s(q, A):
    if q == 0:
        return float(np.max(np.count_nonzero(A, axis=1)))
    return float(np.max(np.sum(np.power(np.abs(A), q), axis=1)))


def mu(p, matrix):
    """mu_p(A) = sqrt(s_{2p}(A) s_{2(1-p)}(A^T)) (``Utility.py:196-212``)."""
    A = np.asarray(matrix)
    return float(np.sqrt(_s(2 * p, A) * _s(2 * (1 - p), A.T)))


def linear_search(matrix, start=0.0, end=1.0, step=0.05):
    domain = [i for i in np.arange(start, end, step)] + [end]
    values = [mu(i, matrix) for i in domain]
    best = int(np.argmin(values))
    return domain[best], values[best]


def best_mu(matrix, start=0.0, end=1.0, step=0.05):
    """min(min_p mu_p(A), ||A||_F) and a label (``Utility.py:222-231``)."""
    p, val = linear_search(matrix, start=start, end=end, step=step)
    fro = float(np.linalg.norm(matrix))
    if val <= fro:
        return f"p={p}", val
    return "Frobenius", fro


def check_division(v, n_jobs):
    """Split v work items over n_jobs (``Utility.py:425-432``, unused helper)."""
    a = float(v) / n_jobs
    d = a - int(a)
    remaining = int(round(d * n_jobs))
    vals = [int(a)] * n_jobs
    for i in range(remaining):
        vals[i] += 1
    return vals


# ---------------------------------------------------------------- Q10 / Q11
def amplitude_est_dist(w0, w1):
    """Circular distance on [0,1) (``Utility.py:435-439``)."""
    c = -np.ceil(w1 - w0)
    f = -np.floor(w1 - w0)
    return min(np.abs(c + w1 - w0), np.abs(f + w1 - w0))


def median_evaluation(func, gamma=0.1, Q=None, *args, **kwargs):
    """Median of Q evaluations (``Utility.py:534-572``)."""
    if Q is None:
        Q = median_repetitions(gamma)
    return float(np.median([func(*args, **kwargs) for _ in range(int(Q))]))


def amplitude_estimation(a, epsilon=0.01, gamma=None, M=None, nqubit=False,
                         plot_distribution=False, random_state=None, method="fast"):
    """Amplitude estimation (``Utility.py:442-531``): sample theta~ = pi j/M
    from the Fejer law centred at asin(sqrt a); return sin^2(theta~).
    ``gamma`` -> median of Q repetitions (Q=13 for gamma=0.1)."""
    rng = as_generator(random_state)
    if gamma:
        return median_evaluation(amplitude_estimation, gamma, None, a=a, epsilon=epsilon, M=M,
                                 nqubit=False, plot_distribution=plot_distribution,
                                 random_state=rng, method=method)
    if M is None:
        M = int(ae_bins(a, epsilon))
    else:
        warnings.warn("Attention! The value of M that will be considered is the one you passed. "
                      "Epsilon in this case is useless")
    n_qubits = np.ceil(np.log2(M))
    theta_a = math.asin(math.sqrt(a))
    omega = M * theta_a / np.pi
    if method == "exact":
        p = fejer_pmf(omega, M)
        j = int(rng.choice(M, p=p / p.sum()))
    else:
        j = int(fejer_sample(np.array([omega]), np.array([M]), rng)[0])
    theta_tilde = np.pi * j / M
    if plot_distribution:
        _plot_law(np.pi * np.arange(M) / M, fejer_pmf(omega, M), theta_a, epsilon)
    if nqubit:
        return theta_tilde, n_qubits, M
    return float(np.sin(theta_tilde) ** 2)


def amplitude_estimation_batch(a, epsilon, gamma=None, random_state=None, Q=None):
    """Vectorised AE over arrays ``a`` / ``epsilon`` (median-of-Q if gamma)."""
    rng = as_generator(random_state)
    a = np.asarray(a, dtype=np.float64)
    eps = np.broadcast_to(np.asarray(epsilon, dtype=np.float64), a.shape)
    M = ae_bins(a, eps)
    omega = M * np.arcsin(np.sqrt(np.clip(a, 0, 1))) / np.pi
    reps = (Q if Q is not None else median_repetitions(gamma)) if gamma else 1
    samples = np.empty((reps,) + a.shape)
    for q in range(reps):
        j = fejer_sample(omega, M, rng)
        samples[q] = np.sin(np.pi * j / M) ** 2
    return np.median(samples, axis=0) if reps > 1 else samples[0]


# ---------------------------------------------------------------------- Q15
def wrapper_phase_est_arguments(argument, type="sv"):
    """(``Utility.py:575-581``) 'sv': 2 acos(x); 'distance': asin(sqrt x)."""
    if type == "sv":
        return 2 * math.acos(argument)
    if type == "distance":
        return math.asin(np.sqrt(argument))
    raise ValueError(type)


def unwrap_phase_est_arguments(argument, eps, type="sv"):
    """(``Utility.py:584-588``) 'sv': cos(theta (eps+pi)/2); 'distance': sin^2(theta pi)."""
    if type == "sv":
        return math.cos(argument * (eps + np.pi) / 2)
    if type == "distance":
        return math.sin(argument * np.pi) ** 2
    raise ValueError(type)


# ---------------------------------------------------------------- Q12 / Q13
def phase_estimation(omega, m=None, epsilon=None, gamma=0.1, plot_distribution=False,
                     nqubit=False, random_state=None, method="fast"):
    """Phase estimation with m qubits (``Utility.py:591-694``): sample k/M,
    M = 2^m, from the Fejer law centred at M*omega."""
    assert m is not None or epsilon is not None, \
        "Attention! You need to specify the number of qubits m or the precision epsilon."
    if m is not None and nqubit:
        warnings.warn("Attention! You are specifying that you want to return also the number of "
                      "qubits used, but you are already specifying it with the m parameter.")
    if epsilon is not None:
        m = int(pe_qubits(epsilon, gamma))
    M = 2 ** int(m)
    if omega == 1 or np.isclose(omega, 1):
        return (M - 1) / M
    rng = as_generator(random_state)
    w = M * float(omega)
    if method == "exact":
        p = fejer_pmf(w, M)
        k = int(rng.choice(M, p=p / p.sum()))
    else:
        k = int(fejer_sample(np.array([w]), np.array([M]), rng)[0])
    omega_tilde = k / M
    if plot_distribution:
        _plot_law(np.arange(M) / M, fejer_pmf(w, M), omega, epsilon or 0)
    if nqubit:
        return omega_tilde, omega_tilde * M, m, M
    return omega_tilde


def phase_estimation_batch(omega, epsilon, gamma, random_state=None):
    """Vectorised PE; returns k/M per element."""
    rng = as_generator(random_state)
    omega = np.asarray(omega, dtype=np.float64)
    m = pe_qubits(np.broadcast_to(epsilon, omega.shape), gamma)
    M = (2 ** m).astype(np.int64)
    k = fejer_sample(M * omega, M, rng)
    out = k / M
    near1 = np.isclose(omega, 1) | (omega == 1)
    return np.where(near1, (M - 1) / M, out)


def _cpe_params(epsilon, gamma, n=None, shift=None):
    if n is None:
        n = int(np.ceil(np.log2(1 / epsilon)) + np.ceil(np.log2(2 + 1 / (2 * gamma))))
    C = gamma / n
    delta_prime = (epsilon * C) / 2
    L = np.floor(2 / C)
    if shift is None:
        shift = int(L / 2) + 1
    return n, delta_prime, shift


def _cpe_interval_midpoint(pe, epsilon, delta_prime, shift):
    """Midpoint of the consistent-PE interval containing ``pe`` - identical to
    bisect over np.arange(-1 - s d', 1 + eps - s d', eps) + [1 + eps - s d']."""
    start = -1 - shift * delta_prime
    stop = 1 + epsilon - shift * delta_prime
    n_ar = int(np.ceil((stop - start) / epsilon))
    pe = np.asarray(pe, dtype=np.float64)
    i = np.floor((pe - start) / epsilon).astype(np.int64) + 1   # count of grid points <= pe
    # exact numpy arange values are start + i*eps: fix off-by-one from rounding
    for _ in range(2):
        i = np.where((i > 0) & (start + (i - 1) * epsilon > pe), i - 1, i)
        i = np.where((i < n_ar) & (start + i * epsilon <= pe), i + 1, i)
    i = np.clip(i, 1, n_ar)

    def val(t):
        return np.where(t < n_ar, start + t * epsilon, stop)
    lo = val(i - 1)
    hi = val(i)
    est = (lo + hi) / 2
    return np.maximum(est, 0.0)


def consistent_phase_estimation(omega, epsilon, gamma, n=None, shift=None, random_state=None,
                                method="fast"):
    """Ta-Shma consistent phase estimation (``Utility.py:740-792``)."""
    n, dp, shift = _cpe_params(epsilon, gamma, n, shift)
    pe = phase_estimation(omega=omega, epsilon=dp, gamma=gamma, random_state=random_state,
                          method=method)
    return float(_cpe_interval_midpoint(pe, epsilon, dp, shift))


def consistent_phase_estimation_batch(omega, epsilon, gamma, random_state=None):
    """Vectorised consistent PE with scalar epsilon/gamma."""
    n, dp, shift = _cpe_params(epsilon, gamma)
    pe = phase_estimation_batch(omega, dp, gamma, random_state)
    return _cpe_interval_midpoint(pe, epsilon, dp, shift)


# ---------------------------------------------------------------------- Q14
def ipe(x, y, epsilon, Q=1, gamma=0.1, random_state=None):
    """Robust inner product estimation (``Utility.py:697-737``).  ``Q`` is
    accepted and ignored, like the reference."""
    x = np.asarray(x, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    nx2 = float(np.dot(x, x))
    ny2 = float(np.dot(y, y))
    ip = float(np.inner(x, y))
    a = (nx2 + ny2 - 2 * ip) / (2 * (nx2 + ny2))
    eps_a = epsilon * max(1, abs(ip)) / (nx2 + ny2)
    if math.isclose(a, 0.0, abs_tol=1e-15):
        a = 0
    a_tilde = amplitude_estimation(a=a, gamma=gamma, epsilon=eps_a, random_state=random_state)
    return (nx2 + ny2) * (1 - 2 * a_tilde) / 2


def ipe_batch(ip, nx2, ny2, epsilon, gamma=0.1, random_state=None):
    """Vectorised IPE from inner products and squared norms (any shapes that
    broadcast) - the oracle of the fused device kernel."""
    ip = np.asarray(ip, dtype=np.float64)
    nx2 = np.asarray(nx2, dtype=np.float64)
    ny2 = np.asarray(ny2, dtype=np.float64)
    S = nx2 + ny2
    a = (S - 2 * ip) / (2 * S)
    a = np.where(np.abs(a) <= 1e-15, 0.0, a)
    eps_a = epsilon * np.maximum(1.0, np.abs(ip)) / S
    a_t = amplitude_estimation_batch(np.clip(a, 0, 1), eps_a, gamma=gamma, random_state=random_state)
    return S * (1 - 2 * a_t) / 2


def _plot_law(x, p, centre, eps):  # pragma: no cover - interactive helper
    import matplotlib.pyplot as plt
    plt.bar(x, p, width=(x[1] - x[0]) if len(x) > 1 else 0.001)
    plt.axvline(centre, c="yellow", ls="dashed")
    plt.xlabel("outcome")
    plt.ylabel("probability")
    plt.show()
