"""Failure-injection kernel and GPU checkpoint/resume (run on an MI355X)."""
import numpy as np
import pytest
import torch

from sq_learn_amd.ops.failure import failure_inject_
from sq_learn_amd.runtime.rng import RngKey

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("p,R,k", [(0.25, 1, 37), (0.4, 3, 1024), (0.01, 2, 5)])
def test_failure_kernel_matches_torch_twin(cuda, p, R, k):
    n = 300_007
    key = RngKey(11, "failure", 5)
    base = torch.randint(0, k, (n,), generator=torch.Generator().manual_seed(0))
    lab_g = base.to(torch.int32).to(cuda)
    cnt_g = torch.zeros(2, dtype=torch.int64, device=cuda)
    failure_inject_(lab_g, k, p, R, key, 1234, cnt_g)
    lab_c = base.clone()
    cnt_c = torch.zeros(2, dtype=torch.int64)
    failure_inject_(lab_c, k, p, R, key, 1234, cnt_c)
    torch.cuda.synchronize()
    assert torch.equal(lab_g.cpu().to(torch.int64), lab_c)
    assert cnt_g.cpu().tolist() == cnt_c.tolist()


def test_gpu_fit_checkpoint_resume(cuda, tmp_path):
    from sq_learn_amd.cluster import QMeans
    from sq_learn_amd.models.cluster._lloyd import LloydEngine
    from sq_learn_amd.utils.datasets import make_blobs
    X, _ = make_blobs(n_samples=50_000, centers=20, n_features=32, cluster_std=3.0,
                      random_state=0)
    Xt = torch.as_tensor(X, dtype=torch.float32, device=cuda)
    kw = dict(n_clusters=20, n_init=2, max_iter=8, tol=0.0, delta=0.5, random_state=1,
              true_distance_estimate=False, intermediate_error=True, true_tomography=False,
              failure_prob=0.05, checkpoint_every=2, compute_prelude=False)
    ref = QMeans(**kw).fit(Xt)
    orig = LloydEngine.step
    calls = {"n": 0}

    def crashing(self):
        calls["n"] += 1
        if calls["n"] > 11:
            raise KeyboardInterrupt
        return orig(self)

    ck = str(tmp_path / "ck")
    LloydEngine.step = crashing
    try:
        with pytest.raises(KeyboardInterrupt):
            QMeans(checkpoint_dir=ck, **kw).fit(Xt)
    finally:
        LloydEngine.step = orig
    got = QMeans(checkpoint_dir=ck, **kw).fit(Xt)
    assert got.resumed_from_[0] == 1
    np.testing.assert_array_equal(got.cluster_centers_, ref.cluster_centers_)
    np.testing.assert_array_equal(got.labels_, ref.labels_)
    assert got.n_failed_rows_ > 0
