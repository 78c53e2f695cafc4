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


@pytest.mark.parametrize("n_init", [1, 2])
def test_gpu_ipe_fit_checkpoint_resume(cuda, tmp_path, n_init):
    """IPE distances (true_distance_estimate=True, delta > 0): the label hints
    that seed each E-step's thresholds are per-rank checkpoint state and are
    reset on new centres, so a resumed fit (and every restart) repeats the
    uninterrupted one bit for bit."""
    from sq_learn_amd.cluster import QMeans
    from sq_learn_amd.models.cluster._lloyd import LloydEngine
    from sq_learn_amd.utils.datasets import make_blobs
    X, _ = make_blobs(n_samples=20_000, centers=12, n_features=24, cluster_std=2.0,
                      random_state=3)
    Xt = torch.as_tensor(X, dtype=torch.float32, device=cuda)
    kw = dict(n_clusters=12, n_init=n_init, max_iter=6, tol=0.0, delta=0.5, random_state=2,
              true_distance_estimate=True, intermediate_error=True, true_tomography=False,
              checkpoint_every=2, compute_prelude=False)
    ref = QMeans(**kw).fit(Xt)
    orig = LloydEngine.step
    calls = {"n": 0}

    def crashing(self):
        calls["n"] += 1
        if calls["n"] > 3 + 6 * (n_init - 1):
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
    assert got.resumed_from_[0] == n_init - 1
    np.testing.assert_array_equal(got.cluster_centers_, ref.cluster_centers_)
    np.testing.assert_array_equal(got.labels_, ref.labels_)


def test_ipe_hints_reset_by_new_centres(cuda):
    """set_centers clears the IPE label hints: the same (restart, iteration)
    from the same centres gives the same labels whatever ran before."""
    from sq_learn_amd.models.cluster._lloyd import LloydEngine
    from sq_learn_amd.utils.datasets import make_blobs
    X, _ = make_blobs(n_samples=30_000, centers=16, n_features=40, cluster_std=2.5,
                      random_state=5)
    Xt = torch.as_tensor(X, dtype=torch.float32, device=cuda)
    C0 = Xt[:16].clone()
    eng = LloydEngine(Xt, 16, delta=0.5, true_distance_estimate=True, intermediate_error=True,
                      seed=4)
    eng.set_centers(C0)
    first = eng.step()[0].clone()
    for _ in range(3):
        eng.step()
    eng.it = 0
    eng.set_centers(C0)
    again = eng.step()[0].clone()
    assert torch.equal(first, again)


def test_tomography_kernel_matches_law(cuda):
    """HIP tomography (K12) vs the torch implementation of the same law."""
    from sq_learn_amd.quantum import device as QD
    g = torch.Generator().manual_seed(0)
    d, rows = 64, 3000
    v = torch.randn(d, generator=g, dtype=torch.float64)
    v /= v.norm()
    A = v[None, :].repeat(rows, 1)
    key = RngKey(5, "tomography", 1)
    # fixed N (no schedule): magnitudes are unbiased, norms are exactly 1
    N = 4000
    est = QD.tomography_rows_torch(A.to(cuda), 0.3, key, N=N, incremental_measure=False)
    torch.cuda.synchronize()
    est = est.cpu()
    assert torch.allclose(est.norm(dim=1), torch.ones(rows, dtype=torch.float64), atol=1e-12)
    m2 = (est ** 2).mean(0)
    assert torch.allclose(m2, v ** 2, atol=4 * (v ** 2 / N / rows).sqrt().max().item() + 1e-4)
    big = v.abs() > 0.15
    assert (torch.sign(est[:, big]) == torch.sign(v[big])).double().mean() > 0.99
    # incremental schedule + stopping rule: errors within delta, same law as torch
    e_gpu = QD.tomography_rows_torch(A.to(cuda), 0.3, key).cpu()
    e_cpu = QD.tomography_rows_torch(A[:500], 0.3, key)
    err_g = (e_gpu - A).norm(dim=1)
    err_c = (e_cpu - A[:500]).norm(dim=1)
    assert (err_g <= 0.3 + 1e-12).double().mean() > 0.99
    assert abs(err_g.mean().item() - err_c.mean().item()) < 0.03
    # deterministic, and distinct rows get distinct draws
    e2 = QD.tomography_rows_torch(A.to(cuda), 0.3, key).cpu()
    assert torch.equal(e_gpu, e2)
    assert not torch.equal(e_gpu[0], e_gpu[1])


@pytest.mark.parametrize("delta", [0.8, 0.1])
def test_tomography_first_pass_walk_matches_all_checkpoints(cuda, monkeypatch, delta):
    """The stop rule's one-launch walk (a wave per row, checkpoints in order
    up to the first passing one) returns the all-checkpoints path's
    estimates bit for bit (same Philox words per row and checkpoint)."""
    from sq_learn_amd.quantum import device as QD
    g = torch.Generator().manual_seed(3)
    A = torch.randn(2000, 61, generator=g, dtype=torch.float64)
    A /= A.norm(dim=1, keepdim=True)
    key = RngKey(9, "tomography", 2)
    walk = QD.tomography_rows_torch(A.to(cuda), delta, key).cpu()
    monkeypatch.setenv("SQ_TOMO_ALLPAIRS", "1")
    full = QD.tomography_rows_torch(A.to(cuda), delta, key).cpu()
    assert torch.equal(walk, full)


def test_gpu_fits_are_bit_reproducible(cuda):
    """No float atomics feed any fitted quantity: two fits are identical."""
    from sq_learn_amd.cluster import QMeans
    from sq_learn_amd.decomposition import QPCA
    from sq_learn_amd.ops import linalg as L
    from sq_learn_amd.utils.datasets import make_blobs_device
    X, _ = make_blobs_device(200_000, 64, centers=50, seed=3, device=cuda, dtype=torch.bfloat16)
    kw = dict(n_clusters=50, n_init=1, max_iter=6, tol=0.0, delta=0.3, random_state=0,
              true_distance_estimate=False, intermediate_error=True, true_tomography=True)
    a = QMeans(**kw).fit(X)
    b = QMeans(**kw).fit(X)
    np.testing.assert_array_equal(a.cluster_centers_, b.cluster_centers_)
    np.testing.assert_array_equal(a.labels_, b.labels_)
    assert a.inertia_ == b.inertia_ and a.muA == b.muA
    mean = X.float().mean(0)
    assert torch.equal(L.gram_local(X, mean), L.gram_local(X, mean))
    Q = torch.randn(64, 24, device=cuda)
    assert torch.equal(L.power_iter_local(X, Q, mean), L.power_iter_local(X, Q, mean))
    p1 = QPCA(n_components=8, svd_solver="randomized", random_state=0, device=cuda).fit(X)
    p2 = QPCA(n_components=8, svd_solver="randomized", random_state=0, device=cuda).fit(X)
    np.testing.assert_array_equal(p1.singular_values_, p2.singular_values_)
