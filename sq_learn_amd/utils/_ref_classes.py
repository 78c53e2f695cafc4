"""Reference mixins kept for API parity (``sklearn/cluster/
_feature_agglomeration.py``: AgglomerationTransform)."""

import numpy as np

from ..base import TransformerMixin


class AgglomerationTransform(TransformerMixin):
    """Feature pooling by cluster label: ``transform`` reduces each cluster
    of features with ``pooling_func`` (default mean), ``inverse_transform``
    broadcasts the pooled values back to the features.  Needs ``labels_``
    (one label per feature) and optionally ``pooling_func``."""

    def transform(self, X):
        X = np.asarray(X)
        pooling = getattr(self, "pooling_func", np.mean)
        labels = np.asarray(self.labels_)
        if labels.shape[0] != X.shape[1]:
            raise ValueError("X has a different number of features than during fitting.")
        if pooling is np.mean:
            size = np.bincount(labels)
            out = np.stack([np.bincount(labels, X[i]) / size for i in range(X.shape[0])])
        else:
            out = np.stack([pooling(X[:, labels == lab], axis=1) for lab in np.unique(labels)],
                           axis=1)
        return out

    def inverse_transform(self, Xred):
        _, inverse = np.unique(self.labels_, return_inverse=True)
        return np.asarray(Xred)[..., inverse]
