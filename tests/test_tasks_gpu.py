"""Task layer on the GPU: cross-validation folds of
device estimators run as concurrent threads (HIP kernels launched from
several host threads on the rank's GPU; pinned explicitly through the
``devices`` list) and give the sequential results."""
import numpy as np
import pytest
import torch

from sq_learn_amd.cluster import KMeans
from sq_learn_amd.model_selection import cross_val_score
from sq_learn_amd.parallel.tasks import Parallel
from sq_learn_amd.utils.fixes import delayed

pytestmark = pytest.mark.gpu


def test_cross_val_kmeans_threads_match_sequential(cuda):
    rs = np.random.RandomState(0)
    X = np.concatenate([rs.randn(3000, 16) + 6 * rs.randn(1, 16) for _ in range(5)]) \
        .astype(np.float32)
    est = KMeans(n_clusters=5, n_init=1, random_state=0, device="cuda")
    seq = cross_val_score(est, X, cv=4)
    par = cross_val_score(est, X, cv=4, n_jobs=4)
    np.testing.assert_allclose(par, seq, rtol=1e-6)


def test_parallel_pinned_device_tasks(cuda):
    def work(i):
        dev = torch.cuda.current_device()
        x = torch.full((1 << 20,), float(i), device="cuda")
        return dev, float(x.sum().item())
    out = Parallel(n_jobs=4, devices=[0, 0])(delayed(work)(i) for i in range(8))
    assert [o[0] for o in out] == [0] * 8
    assert [o[1] for o in out] == [float(i) * (1 << 20) for i in range(8)]
