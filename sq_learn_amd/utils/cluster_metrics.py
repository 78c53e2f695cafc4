"""Clustering metrics (reference ``metrics/cluster/_supervised.py``,
``_unsupervised.py`` and ``_expected_mutual_info_fast.pyx``).

Supervised scores work on the (sparse) contingency table; the expected
mutual information under the hypergeometric model - the O(R*C*N) part -
runs in the host-native library (``csrc/host/cluster_host.cpp``, OpenMP over
rows).  Silhouette / Calinski-Harabasz / Davies-Bouldin take device tensors
and compute distances in chunks with library GEMMs."""

from math import log

import numpy as np
import scipy.sparse as sp
import torch

from ..ops import _host
from ..runtime.device import to_tensor
from .pairwise import get_chunk_n_rows


def check_clusterings(labels_true, labels_pred):
    labels_true = np.asarray(labels_true)
    labels_pred = np.asarray(labels_pred)
    if labels_true.ndim != 1:
        raise ValueError("labels_true must be 1D: shape is %r" % (labels_true.shape,))
    if labels_pred.ndim != 1:
        raise ValueError("labels_pred must be 1D: shape is %r" % (labels_pred.shape,))
    if labels_true.shape[0] != labels_pred.shape[0]:
        raise ValueError("Found input variables with inconsistent numbers of samples: %r"
                         % [labels_true.shape[0], labels_pred.shape[0]])
    return labels_true, labels_pred


def _generalized_average(U, V, average_method):
    if average_method == "min":
        return min(U, V)
    if average_method == "geometric":
        return np.sqrt(U * V)
    if average_method == "arithmetic":
        return np.mean([U, V])
    if average_method == "max":
        return max(U, V)
    raise ValueError("'average_method' must be 'min', 'geometric', 'arithmetic', or 'max'")


def contingency_matrix(labels_true, labels_pred, *, eps=None, sparse=False, dtype=np.int64):
    if eps is not None and sparse:
        raise ValueError("Cannot set 'eps' when sparse=True")
    classes, class_idx = np.unique(labels_true, return_inverse=True)
    clusters, cluster_idx = np.unique(labels_pred, return_inverse=True)
    c = sp.coo_matrix((np.ones(class_idx.shape[0]), (class_idx, cluster_idx)),
                      shape=(classes.shape[0], clusters.shape[0]), dtype=dtype)
    if sparse:
        c = c.tocsr()
        c.sum_duplicates()
        return c
    c = c.toarray()
    if eps is not None:
        c = c + eps
    return c


def pair_confusion_matrix(labels_true, labels_pred):
    labels_true, labels_pred = check_clusterings(labels_true, labels_pred)
    n = np.int64(labels_true.shape[0])
    c = contingency_matrix(labels_true, labels_pred, sparse=True, dtype=np.int64)
    nk = np.ravel(c.sum(axis=1))
    ck = np.ravel(c.sum(axis=0))
    sq = (c.data ** 2).sum()
    C = np.empty((2, 2), dtype=np.int64)
    C[1, 1] = sq - n
    C[0, 1] = c.dot(ck).sum() - sq
    C[1, 0] = c.transpose().dot(nk).sum() - sq
    C[0, 0] = n ** 2 - C[0, 1] - C[1, 0] - sq
    return C


def rand_score(labels_true, labels_pred):
    C = pair_confusion_matrix(labels_true, labels_pred)
    num = C.diagonal().sum()
    den = C.sum()
    if num == den or den == 0:
        return 1.0
    return num / den


def entropy(labels):
    if len(labels) == 0:
        return 1.0
    idx = np.unique(labels, return_inverse=True)[1]
    pi = np.bincount(idx).astype(np.float64)
    pi = pi[pi > 0]
    s = np.sum(pi)
    return -np.sum((pi / s) * (np.log(pi) - log(s)))


def mutual_info_score(labels_true, labels_pred, *, contingency=None):
    if contingency is None:
        labels_true, labels_pred = check_clusterings(labels_true, labels_pred)
        contingency = contingency_matrix(labels_true, labels_pred, sparse=True)
    if isinstance(contingency, np.ndarray):
        nzx, nzy = np.nonzero(contingency)
        nz = contingency[nzx, nzy]
    elif sp.issparse(contingency):
        nzx, nzy, nz = sp.find(contingency)
    else:
        raise ValueError("Unsupported type for 'contingency': %s" % type(contingency))
    total = contingency.sum()
    pi = np.ravel(contingency.sum(axis=1))
    pj = np.ravel(contingency.sum(axis=0))
    log_c = np.log(nz)
    c_nm = nz / total
    outer = pi.take(nzx).astype(np.int64) * pj.take(nzy).astype(np.int64)
    log_outer = -np.log(outer) + log(pi.sum()) + log(pj.sum())
    mi = c_nm * (log_c - log(total)) + c_nm * log_outer
    mi = np.where(np.abs(mi) < np.finfo(mi.dtype).eps, 0.0, mi)
    return np.clip(mi.sum(), 0.0, None)


def expected_mutual_information(contingency, n_samples):
    """E[MI] of a contingency table under random permutations (host kernel)."""
    a = np.ascontiguousarray(np.ravel(contingency.sum(axis=1)), dtype=np.int64)
    b = np.ascontiguousarray(np.ravel(contingency.sum(axis=0)), dtype=np.int64)
    return float(_host.lib().sqh_expected_mutual_info(_host.ptr(a), a.size, _host.ptr(b), b.size,
                                                      int(n_samples)))


def adjusted_mutual_info_score(labels_true, labels_pred, *, average_method="arithmetic"):
    labels_true, labels_pred = check_clusterings(labels_true, labels_pred)
    n = labels_true.shape[0]
    classes = np.unique(labels_true)
    clusters = np.unique(labels_pred)
    if classes.shape[0] == clusters.shape[0] == 1 or classes.shape[0] == clusters.shape[0] == 0:
        return 1.0
    c = contingency_matrix(labels_true, labels_pred, sparse=True).astype(np.float64)
    mi = mutual_info_score(labels_true, labels_pred, contingency=c)
    emi = expected_mutual_information(c, n)
    h_true, h_pred = entropy(labels_true), entropy(labels_pred)
    den = _generalized_average(h_true, h_pred, average_method) - emi
    eps = np.finfo("float64").eps
    den = min(den, -eps) if den < 0 else max(den, eps)
    return (mi - emi) / den


def normalized_mutual_info_score(labels_true, labels_pred, *, average_method="arithmetic"):
    labels_true, labels_pred = check_clusterings(labels_true, labels_pred)
    classes = np.unique(labels_true)
    clusters = np.unique(labels_pred)
    if classes.shape[0] == clusters.shape[0] == 1 or classes.shape[0] == clusters.shape[0] == 0:
        return 1.0
    c = contingency_matrix(labels_true, labels_pred, sparse=True).astype(np.float64)
    mi = mutual_info_score(labels_true, labels_pred, contingency=c)
    h_true, h_pred = entropy(labels_true), entropy(labels_pred)
    norm = max(_generalized_average(h_true, h_pred, average_method), np.finfo("float64").eps)
    return mi / norm


def homogeneity_completeness_v_measure(labels_true, labels_pred, *, beta=1.0):
    labels_true, labels_pred = check_clusterings(labels_true, labels_pred)
    if len(labels_true) == 0:
        return 1.0, 1.0, 1.0
    hc, hk = entropy(labels_true), entropy(labels_pred)
    c = contingency_matrix(labels_true, labels_pred, sparse=True)
    mi = mutual_info_score(None, None, contingency=c)
    hom = mi / hc if hc else 1.0
    com = mi / hk if hk else 1.0
    v = 0.0 if hom + com == 0.0 else (1 + beta) * hom * com / (beta * hom + com)
    return hom, com, v


def homogeneity_score(labels_true, labels_pred):
    return homogeneity_completeness_v_measure(labels_true, labels_pred)[0]


def completeness_score(labels_true, labels_pred):
    return homogeneity_completeness_v_measure(labels_true, labels_pred)[1]


def v_measure_score(labels_true, labels_pred, *, beta=1.0):
    return homogeneity_completeness_v_measure(labels_true, labels_pred, beta=beta)[2]


def fowlkes_mallows_score(labels_true, labels_pred, *, sparse=False):
    labels_true, labels_pred = check_clusterings(labels_true, labels_pred)
    n, = labels_true.shape
    c = contingency_matrix(labels_true, labels_pred, sparse=True).astype(np.int64)
    tk = np.dot(c.data, c.data) - n
    pk = np.sum(np.asarray(c.sum(axis=0)).ravel() ** 2) - n
    qk = np.sum(np.asarray(c.sum(axis=1)).ravel() ** 2) - n
    return np.sqrt(tk / pk) * np.sqrt(tk / qk) if tk != 0.0 else 0.0


# ----------------------------------------------------------------- unsupervised
def _labels_and_X(X, labels, device=None):
    Xt = to_tensor(X, device) if not isinstance(X, torch.Tensor) else X
    if not Xt.is_floating_point() or Xt.dtype == torch.bfloat16:
        Xt = Xt.double()
    if Xt.device.type == "cpu":
        Xt = Xt.double()
    le = np.unique(np.asarray(labels), return_inverse=True)
    lab = torch.as_tensor(le[1], dtype=torch.int64, device=Xt.device)
    n_labels = len(le[0])
    n = Xt.shape[0]
    if not 1 < n_labels < n:
        raise ValueError("Number of labels is %d. Valid values are 2 to n_samples - 1 (inclusive)"
                         % n_labels)
    return Xt, lab, n_labels


def silhouette_samples(X, labels, *, metric="euclidean", device=None):
    """Per-sample silhouette coefficient; distances in GEMM chunks on the
    data's device (``metric`` 'euclidean' or 'precomputed')."""
    Xt, lab, K = _labels_and_X(X, labels, device)
    n = Xt.shape[0]
    counts = torch.bincount(lab, minlength=K).to(Xt.dtype)
    a = torch.empty(n, dtype=Xt.dtype, device=Xt.device)
    b = torch.empty(n, dtype=Xt.dtype, device=Xt.device)
    onehot = torch.nn.functional.one_hot(lab, K).to(Xt.dtype)
    rows = get_chunk_n_rows(n * Xt.element_size())
    xn = (Xt * Xt).sum(1) if metric != "precomputed" else None
    for s in range(0, n, rows):
        e = min(n, s + rows)
        if metric == "precomputed":
            D = Xt[s:e]
        else:
            D = torch.sqrt((xn[s:e, None] + xn[None, :] - 2.0 * (Xt[s:e] @ Xt.T)).clamp_(min=0))
            D[torch.arange(e - s, device=D.device), torch.arange(s, e, device=D.device)] = 0.0
        cd = D @ onehot                          # sum of distances to each cluster
        own = lab[s:e]
        intra = cd.gather(1, own[:, None])[:, 0]
        denom = (counts[own] - 1).clamp(min=1)
        a[s:e] = intra / denom
        cd = cd / counts[None, :]
        cd.scatter_(1, own[:, None], float("inf"))
        b[s:e] = cd.min(1).values
    sil = (b - a) / torch.maximum(a, b)
    sil = torch.nan_to_num(sil)
    sil = torch.where(counts[lab] > 1, sil, torch.zeros_like(sil))
    return sil.cpu().numpy()


def silhouette_score(X, labels, *, metric="euclidean", sample_size=None, random_state=None,
                     device=None):
    if sample_size is not None:
        from .validation import check_random_state
        rs = check_random_state(random_state)
        idx = rs.permutation(np.asarray(X).shape[0] if not isinstance(X, torch.Tensor)
                             else X.shape[0])[:sample_size]
        if metric == "precomputed":
            X = np.asarray(X)[idx][:, idx]
        else:
            X = X[idx]
        labels = np.asarray(labels)[idx]
    return float(np.mean(silhouette_samples(X, labels, metric=metric, device=device)))


def calinski_harabasz_score(X, labels, device=None):
    Xt, lab, K = _labels_and_X(X, labels, device)
    n = Xt.shape[0]
    mean = Xt.mean(0)
    onehot = torch.nn.functional.one_hot(lab, K).to(Xt.dtype)
    cnt = onehot.sum(0)
    cm = (onehot.T @ Xt) / cnt[:, None]
    extra = float((cnt * ((cm - mean) ** 2).sum(1)).sum())
    intra = float(((Xt - cm[lab]) ** 2).sum())
    return 1.0 if intra == 0.0 else extra * (n - K) / (intra * (K - 1.0))


def davies_bouldin_score(X, labels, device=None):
    Xt, lab, K = _labels_and_X(X, labels, device)
    onehot = torch.nn.functional.one_hot(lab, K).to(Xt.dtype)
    cnt = onehot.sum(0)
    cm = (onehot.T @ Xt) / cnt[:, None]
    dist = torch.linalg.vector_norm(Xt - cm[lab], dim=1)
    intra = (onehot.T @ dist) / cnt
    cdist = torch.cdist(cm, cm)
    if torch.allclose(intra, torch.zeros_like(intra)) or torch.allclose(cdist, torch.zeros_like(cdist)):
        return 0.0
    cdist[cdist == 0] = float("inf")
    score = (intra[:, None] + intra[None, :]) / cdist
    return float(score.max(1).values.mean())
