"""Long-vector tomography and the PE / CPE kernels on the device.

* ``mnom_segments_kernel`` (segmented binomial-splitting multinomial): exact
  total, chi^2 goodness of fit of the counts at n = 2e5 outcomes, independence
  of the draws from the launch chunking;
* ``tomography_long`` (qPCA left singular vectors, n >= 1e5): the error law
  against the CPU twin (numpy multinomials), the stopping rule;
* ``pe_batch_kernel`` and the device consistent phase estimation against the
  NumPy oracle's law; qPCA randomized + quantum extras end to end.
"""
import numpy as np
import pytest
import torch
from scipy import stats

from sq_learn_amd.quantum import device as QD
from sq_learn_amd.quantum import reference as Q
from sq_learn_amd.quantum.fejer import fejer_pmf
from sq_learn_amd.ops import random as R
from sq_learn_amd.runtime.rng import RngKey

pytestmark = pytest.mark.gpu


def test_mnom_segments_law_and_total(cuda):
    n = 200_000
    rng = np.random.default_rng(0)
    w = rng.exponential(size=n) ** 2
    W = torch.tensor(w[None], device=cuda)
    N = 3.0e9
    reps = 4
    cnt = QD.multinomial_long(torch.full((reps,), N, dtype=torch.float64, device=cuda), W,
                              torch.zeros(reps, dtype=torch.int64, device=cuda),
                              RngKey(1, "tomography", 0),
                              torch.arange(reps, dtype=torch.int64, device=cuda)).cpu().numpy()
    assert np.all(cnt.sum(1) == N)
    assert np.all(cnt >= 0) and np.all(cnt == np.round(cnt))
    p = w / w.sum()
    for r in range(reps):
        # pool outcomes into 200 bins of equal expected mass, chi^2 GOF
        bins = np.minimum((np.cumsum(p) * 200).astype(int), 199)
        obs = np.bincount(bins, weights=cnt[r], minlength=200)
        exp = np.bincount(bins, weights=p * N, minlength=200)
        chi2 = ((obs - exp) ** 2 / exp).sum()
        assert stats.chi2.sf(chi2, 199) > 1e-4
        # per-coordinate z-scores: counts ~ Binomial(N, p_i)
        z = (cnt[r] - N * p) / np.sqrt(N * p * (1 - p))
        assert abs(z.mean()) < 0.02 and abs(z.std() - 1) < 0.02
    assert not np.array_equal(cnt[0], cnt[1])
    # deterministic in (key, sid): a single-row launch reproduces row 2
    one = QD.multinomial_long(torch.tensor([N], dtype=torch.float64, device=cuda), W,
                              torch.zeros(1, dtype=torch.int64, device=cuda),
                              RngKey(1, "tomography", 0),
                              torch.tensor([2], dtype=torch.int64, device=cuda)).cpu().numpy()
    np.testing.assert_array_equal(one[0], cnt[2])


def test_tomography_long_matches_cpu_law(cuda):
    n = 100_000
    rng = np.random.default_rng(1)
    A = torch.tensor(rng.standard_normal((3, n)))
    Vn = (A / A.norm(dim=1, keepdim=True)).numpy()
    N = 20_000_000
    e_gpu, e_cpu = [], []
    for rep in range(8):
        g = QD.tomography_long(A.to(cuda), None, RngKey(rep, "tomography", 5), N=N,
                               incremental_measure=False).cpu().numpy()
        c = QD.tomography_long(A, None, RngKey(rep, "tomography", 6), N=N,
                               incremental_measure=False).numpy()
        e_gpu += list(np.linalg.norm(g - Vn, axis=1))
        e_cpu += list(np.linalg.norm(c - Vn, axis=1))
        assert np.allclose(np.linalg.norm(g, axis=1), 1.0, atol=0.05)
    assert stats.ks_2samp(e_gpu, e_cpu).pvalue > 1e-4
    assert abs(np.mean(e_gpu) - np.mean(e_cpu)) < 0.1 * np.mean(e_cpu)


def test_tomography_long_stopping_rule(cuda):
    n = 120_000
    rng = np.random.default_rng(2)
    A = torch.tensor(rng.standard_normal((2, n)), device=cuda)
    Vn = (A / A.norm(dim=1, keepdim=True)).cpu().numpy()
    for delta in (0.5, 0.2):
        est = QD.tomography_rows_torch(A, delta, RngKey(3, "tomography", 0)).cpu().numpy()
        err = np.linalg.norm(est - Vn, axis=1)
        assert np.all(err <= delta)
        assert np.all(err > 0.3 * delta)   # stops at the FIRST passing checkpoint


def test_pe_batch_kernel_law(cuda):
    n = 40_000
    omega, m = 0.3141, 7
    g = R.phase_estimation_batch(torch.full((n,), omega, dtype=torch.float64, device=cuda),
                                 torch.full((n,), m, dtype=torch.int32, device=cuda),
                                 RngKey(4, "pe", 0)).cpu().numpy()
    c = R.phase_estimation_batch(torch.full((2000,), omega, dtype=torch.float64),
                                 torch.full((2000,), m, dtype=torch.int32),
                                 RngKey(4, "pe", 0)).numpy()
    assert np.mean(np.isclose(g[:2000], c)) > 0.99    # same Philox streams as the CPU twin
    M = 2 ** m
    k = np.round(g * M).astype(int)
    p = fejer_pmf(M * omega, M)
    obs = np.bincount(k, minlength=M)
    exp = p * n
    big = exp >= 5
    o = np.append(obs[big], obs[~big].sum())
    e = np.append(exp[big], exp[~big].sum())
    chi2 = ((o - e) ** 2 / e).sum()
    assert stats.chi2.sf(chi2, len(e) - 1) > 1e-4


def test_consistent_pe_device_matches_oracle(cuda):
    eps, gamma = 0.02, 0.1
    om = torch.linspace(0.05, 0.95, 37, dtype=torch.float64)
    dev = QD.consistent_phase_estimation_device(om.to(cuda), eps, gamma,
                                                RngKey(5, "pe", 0)).cpu().numpy()
    ora = Q.consistent_phase_estimation_batch(om.numpy(), eps, gamma, random_state=0)
    # consistent PE returns the same interval midpoint with probability >= 1 - gamma
    assert np.mean(np.isclose(dev, ora)) > 0.85
    assert np.all(np.abs(dev - om.numpy()) <= eps + 1e-12)


def test_qpca_randomized_quantum_gpu(cuda):
    from sq_learn_amd.models.decomposition import QPCA
    rng = np.random.RandomState(0)
    Z = (rng.randn(20000, 32) @ rng.randn(32, 32)).astype(np.float32)
    q = QPCA(n_components=4, svd_solver="randomized", random_state=0, device=cuda,
             quantum_truncated=True).fit(Z, eps=1e-3, theta_major=1e-6, delta=0.2,
                                         estimate_all=True, true_tomography=True)
    L = q.estimate_left_sv
    L = L.cpu().numpy() if isinstance(L, torch.Tensor) else np.asarray(L)
    U = q.left_sv.cpu().numpy() if isinstance(q.left_sv, torch.Tensor) else np.asarray(q.left_sv)
    assert L.shape == (4, 20000)
    assert np.all(np.linalg.norm(L - U, axis=1) <= 0.2)
    np.testing.assert_allclose(q.estimate_s_values, q.singular_values_, rtol=1e-2)
