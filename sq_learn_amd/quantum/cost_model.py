"""Analytic quantum vs classical running-time models.

q-means (``_dmeans.py:1412-1469``) and qPCA (``_qPCA.py:1123-1316``)
formulas, evaluated on numpy grids; plotting uses matplotlib (the reference
used a MATLAB engine).
"""

import numpy as np


def qmeans_runtime(n_clusters, n_init, eta, condition_number, muA, delta, n, m,
                   well_clusterable=False):
    """Returns (q_runtime, c_runtime) on the (n, m) grid (``_dmeans.py:1437-1449``)."""
    c_runtime = n * m * n_clusters * n_init
    k = n_clusters
    if not well_clusterable:
        q = (k * m * eta * condition_number * (muA + k * eta / delta) / delta ** 2
             + (k ** 2) * (eta ** 1.5) * condition_number * muA / delta ** 2)
    else:
        q = (k ** 2) * m * (eta ** 2.5) / delta ** 3 + (k ** 2.5) * (eta ** 2) / delta ** 3
    q = q * np.ones_like(np.asarray(n, dtype=float))
    return q, c_runtime


def qpca_runtime_terms(est, n_samples, n_features, estimate_components="all"):
    """List of quantum cost terms of a fitted QPCA (``_qPCA.py:1123-1208``).

    ``est`` needs: theta_estimate, quantum_retained_variance, estimate_all,
    estimate_least_k, muA, eps, eps_theta, eta, theta (or est_theta), topk,
    topk_p, spectral_norm, delta, tomography_norm, singular_values_,
    theta_minor, least_k, least_k_p."""
    out = []
    n = np.asarray(n_samples, dtype=float)
    m = np.asarray(n_features, dtype=float)
    theta = est.theta_major if est.theta_major else getattr(est, "est_theta", 0.0)
    if est.theta_estimate:
        out.append((est.muA * np.log(est.muA / est.eps_theta) * np.log(n * m))
                   / (est.eps_theta * est.eta))
    if est.quantum_retained_variance:
        out.append(est.muA / (est.eps * est.eta) * np.ones_like(n))
    if est.estimate_all:
        k = est.topk
        logk = np.log(k) if k > 0 else 0.0
        if est.tomography_norm == "L2":
            left = (est.spectral_norm * est.muA * k * logk * n * np.log(n)) / (
                theta * np.sqrt(est.topk_p) * est.eps * est.delta ** 2)
            right = ((est.spectral_norm / theta) * (1 / np.sqrt(est.topk_p)) * (est.muA / est.eps)
                     * ((k * logk * m * np.log(m)) / est.delta ** 2))
        else:
            left = np.full(n.shape, (est.spectral_norm * est.muA * k) / (theta * est.eps * est.delta ** 2))
            right = np.full(m.shape, (est.spectral_norm * est.muA * k) / (theta * est.eps * est.delta ** 2))
        base = (est.spectral_norm * est.muA * k * logk) / (theta * np.sqrt(est.topk_p) * est.eps)
        if estimate_components == "all":
            out.append(left + right + base)
        elif estimate_components == "left_sv":
            out.append(left + base)
        elif estimate_components == "right_sv":
            out.append(right + base)
    if getattr(est, "estimate_least_k", False):
        sv = est.singular_values_
        nz = sv[~np.isclose(sv, 0)] if np.any(np.isclose(sv, 0)) else sv
        lk = est.least_k
        loglk = np.log(lk) if lk > 0 else 0.0
        if est.tomography_norm == "L2":
            left = ((est.theta_minor / nz[-1]) * (1 / np.sqrt(est.least_k_p)) * (est.muA / est.eps)
                    * ((lk * loglk * n * np.log(n)) / est.delta ** 2))
            right = ((est.theta_minor / nz[-2 if len(nz) > 1 else -1]) * (1 / np.sqrt(est.least_k_p))
                     * (est.muA / est.eps) * ((lk * loglk * m * np.log(m)) / est.delta ** 2))
        else:
            left = np.full(n.shape, (est.spectral_norm * est.muA * lk) / (est.theta_minor * est.eps * est.delta ** 2))
            right = np.full(m.shape, (est.spectral_norm * est.muA * lk) / (est.theta_minor * est.eps * est.delta ** 2))
        base = (est.theta_minor * est.muA * lk) / (nz[-2 if len(nz) > 1 else -1] * np.sqrt(est.least_k_p) * est.eps)
        if estimate_components == "all":
            out.append(left + right + base)
        elif estimate_components == "left_sv":
            out.append(left + base)
        else:
            out.append(right + base)
    return out


def plot_runtime(n, m, q_runtime, c_runtime, title, saveas=None):  # pragma: no cover - plotting
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    fig = plt.figure()
    ax = fig.add_subplot(projection="3d")
    ax.plot_wireframe(n, m, q_runtime, color="b", label="quantumRuntime")
    ax.plot_wireframe(n, m, c_runtime, color="g", label="classicRuntime")
    ax.set_xlabel("nSamples")
    ax.set_ylabel("nFeatures")
    ax.set_title(title)
    ax.legend()
    if saveas:
        fig.savefig(saveas)
    return fig
