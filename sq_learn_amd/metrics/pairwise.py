"""Reference-layout import path ``sklearn.metrics.pairwise``."""
import numpy as np

from ..utils.pairwise import *  # noqa: F401,F403
from ..utils.pairwise import euclidean_distances


def nan_euclidean_distances(X, Y=None, *, squared=False, missing_values=np.nan, copy=True):
    """Euclidean distances ignoring missing coordinates, rescaled by the
    fraction of present coordinates (reference ``metrics/pairwise.py``)."""
    X = np.array(X, dtype=np.float64, copy=True)
    same = Y is None
    Y = X if same else np.array(Y, dtype=np.float64, copy=True)
    mX = np.isnan(X) if missing_values is np.nan or missing_values != missing_values else \
        X == missing_values
    mY = mX if same else (np.isnan(Y) if missing_values != missing_values else Y == missing_values)
    X[mX] = 0
    if not same:
        Y[mY] = 0
    D = np.asarray(euclidean_distances(X, Y, squared=True), dtype=np.float64)
    D -= (X * X) @ mY.T
    D -= mX @ (Y * Y).T
    np.clip(D, 0, None, out=D)
    if same:
        np.fill_diagonal(D, 0.0)
    pX = 1 - mX
    pY = pX if same else ~mY
    cnt = pX @ pY.T
    D[cnt == 0] = np.nan
    np.maximum(1, cnt, out=cnt)
    D /= cnt
    D *= X.shape[1]
    return D if squared else np.sqrt(D, out=D)
from ..utils._ref_api import (check_paired_arrays, check_pairwise_arrays,  # noqa: E402,F401
                              distance_metrics, kernel_metrics)
