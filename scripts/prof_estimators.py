"""Device-path workload for rocprofv3: MLP training (SGD/Adam on device),
Bayesian GMM, batched lasso sparse coding and LabelSpreading, timed per
estimator.  Usage: python scripts/prof_estimators.py"""
import json
import os
import sys
import time
import warnings

import numpy as np
import torch

warnings.filterwarnings("ignore")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _t(fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    return time.perf_counter() - t0


def main():
    from sq_learn_amd.decomposition import sparse_encode
    from sq_learn_amd.mixture import BayesianGaussianMixture
    from sq_learn_amd.neural_network import MLPClassifier
    rng = np.random.RandomState(0)
    X = rng.randn(20000, 64)
    y = (X[:, :4].sum(1) > 0).astype(int) + (X[:, 4] > 1)
    out = {}
    out["mlp_adam_256x128_5ep_s"] = _t(lambda: MLPClassifier(
        (256, 128), max_iter=5, batch_size=512, random_state=0).fit(X, y))
    out["bgmm_full_k8_s"] = _t(lambda: BayesianGaussianMixture(
        n_components=8, max_iter=50, random_state=0).fit(X[:, :16]))
    D = rng.randn(32, 64)
    D /= np.linalg.norm(D, axis=1, keepdims=True)
    out["sparse_encode_lasso_cd_5000x32_s"] = _t(lambda: sparse_encode(
        X[:5000], D, algorithm="lasso_cd", alpha=0.2))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
