"""Device inference for tree ensembles (``csrc/forest.hip``).

``ForestTables`` uploads the concatenated node arrays of a fitted forest
once (int32 children / features, fp64 thresholds, fp64 leaf values) and is
cached on the estimator, so repeated ``predict`` calls on GPU rows only move
the rows.  CPU rows use the host-native traversal (``sqh_forest_apply``).
"""

import numpy as np
import torch

from . import _native as nat


def _dev_rows(X):
    if X.dtype != torch.float32:
        X = X.float()
    return X.contiguous()


def forest_apply(X, left, right, feat, thr, offs):
    """(n, T) int32 leaf ids of GPU rows ``X``."""
    dev = X.device
    X = _dev_rows(X)
    n, d = X.shape
    T = len(offs)
    tab = [torch.as_tensor(np.asarray(a, dtype=np.int32), device=dev) for a in (left, right, feat)]
    t_thr = torch.as_tensor(np.asarray(thr, dtype=np.float64), device=dev)
    t_off = torch.as_tensor(np.asarray(offs, dtype=np.int64), device=dev)
    out = torch.empty((n, T), dtype=torch.int32, device=dev)
    m = nat.native()
    m.forest_apply(tab[0].data_ptr(), tab[1].data_ptr(), tab[2].data_ptr(), t_thr.data_ptr(),
                   t_off.data_ptr(), T, X.data_ptr(), n, d, out.data_ptr(),
                   nat.stream_handle(dev))
    return out


class ForestTables:
    """Device copy of a forest: node tables + per-node value vectors."""

    def __init__(self, left, right, feat, thr, offs, values, device, missing_left=None):
        self.device = torch.device(device)
        i32 = lambda a: torch.as_tensor(np.asarray(a, dtype=np.int32), device=self.device)  # noqa
        self.left, self.right, self.feat = i32(left), i32(right), i32(feat)
        self.thr = torch.as_tensor(np.asarray(thr, dtype=np.float64), device=self.device)
        self.offs = torch.as_tensor(np.asarray(offs, dtype=np.int64), device=self.device)
        values = np.ascontiguousarray(values, dtype=np.float64)
        self.S = values.shape[1]
        if self.S > 32:
            raise ValueError("device forest predict supports at most 32 values per leaf")
        self.values = torch.as_tensor(values, device=self.device)
        self.missing = None
        if missing_left is not None:
            self.missing = torch.as_tensor(np.asarray(missing_left, dtype=np.uint8),
                                           device=self.device)
        self.T = len(offs)

    def predict_sum(self, X, scale=1.0):
        """(n, S) fp64 = scale * sum over trees of the leaf value vectors."""
        X = _dev_rows(X.to(self.device))
        n, d = X.shape
        out = torch.empty((n, self.S), dtype=torch.float64, device=self.device)
        nat.native().forest_predict(
            self.left.data_ptr(), self.right.data_ptr(), self.feat.data_ptr(),
            self.thr.data_ptr(), 0 if self.missing is None else self.missing.data_ptr(),
            self.offs.data_ptr(), self.T, self.values.data_ptr(), self.S, X.data_ptr(), n, d,
            float(scale), out.data_ptr(), nat.stream_handle(self.device))
        return out
