"""Weighted percentile (reference ``utils/stats.py:7``): lower weighted
percentile via the stable cumulative weight CDF, along axis 0 for 2-D input."""

import numpy as np


def _weighted_percentile(array, sample_weight, percentile=50):
    array = np.asarray(array)
    sample_weight = np.asarray(sample_weight, dtype=np.float64)
    n_dim = array.ndim
    if n_dim == 0:
        return array[()]
    if array.ndim == 1:
        array = array.reshape((-1, 1))
    if array.shape != sample_weight.shape and array.shape[0] == sample_weight.shape[0]:
        sample_weight = np.tile(sample_weight, (array.shape[1], 1)).T
    sorted_idx = np.argsort(array, axis=0, kind="stable")
    sorted_w = np.take_along_axis(sample_weight, sorted_idx, axis=0)
    cdf = np.cumsum(sorted_w, axis=0, dtype=np.float64)
    adjusted = percentile / 100 * cdf[-1]
    idx = np.array([np.searchsorted(cdf[:, i], adjusted[i]) for i in range(cdf.shape[1])])
    idx = np.clip(idx, 0, sorted_idx.shape[0] - 1)
    cols = np.arange(array.shape[1])
    out = array[sorted_idx[idx, cols], cols]
    return out[0] if n_dim == 1 else out
