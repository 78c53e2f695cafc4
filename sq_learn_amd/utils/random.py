"""Sampling without replacement (reference ``utils/_random.pyx:27-311``):
'auto' uses a permutation for 1% < k/n < 99%, otherwise tracking selection
(k/n < 0.2) or reservoir sampling; 'pool' keeps the reference's swap pool.
The same ``RandomState`` calls as the reference, so seeds give its draws."""

import numpy as np

from .validation import check_random_state


def _tracking_selection(n_population, n_samples, rng):
    out = np.empty(n_samples, dtype=np.int64)
    selected = set()
    for i in range(n_samples):
        j = rng.randint(n_population)
        while j in selected:
            j = rng.randint(n_population)
        selected.add(j)
        out[i] = j
    return out


def _reservoir(n_population, n_samples, rng):
    out = np.arange(n_samples, dtype=np.int64)
    for i in range(n_samples, n_population):
        j = rng.randint(0, i + 1)
        if j < n_samples:
            out[j] = i
    return out


def _pool(n_population, n_samples, rng):
    pool = np.arange(n_population, dtype=np.int64)
    out = np.empty(n_samples, dtype=np.int64)
    for i in range(n_samples):
        j = rng.randint(n_population - i)
        out[i] = pool[j]
        pool[j] = pool[n_population - i - 1]
    return out


def sample_without_replacement(n_population, n_samples, method="auto", random_state=None):
    if n_population < 0:
        raise ValueError("n_population should be greater than 0, got %s." % n_population)
    if n_samples > n_population:
        raise ValueError("n_population should be greater or equal than n_samples, got "
                         "n_samples > n_population (%s > %s)" % (n_samples, n_population))
    rng = check_random_state(random_state)
    ratio = n_samples / n_population if n_population != 0 else 1.0
    if method == "auto" and 0.01 < ratio < 0.99:
        return rng.permutation(n_population)[:n_samples]
    if method in ("auto", "tracking_selection"):
        if method == "tracking_selection" or ratio < 0.2:
            return _tracking_selection(n_population, n_samples, rng)
        return _reservoir(n_population, n_samples, rng)
    if method == "reservoir_sampling":
        return _reservoir(n_population, n_samples, rng)
    if method == "pool":
        return _pool(n_population, n_samples, rng)
    raise ValueError("Expected a method name in ('auto', 'tracking_selection', "
                     "'reservoir_sampling', 'pool'), got %s." % method)
