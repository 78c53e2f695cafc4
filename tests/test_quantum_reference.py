"""Distributional tests of the QuantumUtility oracle against the reference's
exact laws (SURVEY.md §4 implication 1)."""
import math

import numpy as np
import pytest
from scipy import stats

from sq_learn_amd.quantum import reference as Q
from sq_learn_amd.quantum.fejer import fejer_pmf, fejer_sample, median_repetitions, pe_qubits
from sq_learn_amd.runtime.rng import philox4x32, RngKey


def test_philox_known_answers():
    # Random123 known-answer vectors for philox4x32-10
    assert [int(v) for v in philox4x32(0, 0, 0, 0, 0, 0)] == [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]
    m = 0xffffffff
    assert [int(v) for v in philox4x32(m, m, m, m, m, m)] == [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]
    assert [int(v) for v in philox4x32(0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344,
                                       0xa4093822, 0x299f31d0)] == [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]


@pytest.mark.parametrize("omega,M", [(3.3, 10), (17.7, 100), (0.01, 64), (500.5, 1000), (123.0, 400),
                                     (99.95, 2 ** 12)])
def test_fejer_sampler_chi2(omega, M):
    rng = np.random.default_rng(0)
    p = fejer_pmf(omega, M)
    assert abs(p.sum() - 1) < 1e-9
    n = 40000
    s = fejer_sample(np.full(n, omega), np.full(n, M), rng)
    counts = np.bincount(s, minlength=M)
    exp = p * n
    # pool bins with small expectation
    order = np.argsort(-exp)
    big = exp[order] >= 5
    obs_b, exp_b = counts[order][big], exp[order][big]
    obs_r, exp_r = counts[order][~big].sum(), exp[order][~big].sum()
    obs = np.append(obs_b, obs_r) if exp_r > 0 else obs_b
    ex = np.append(exp_b, exp_r) if exp_r > 0 else exp_b
    chi2 = ((obs - ex) ** 2 / ex).sum()
    dof = len(ex) - 1
    assert stats.chi2.sf(chi2, max(dof, 1)) > 1e-4


def test_fejer_tail_is_exercised():
    rng = np.random.default_rng(1)
    M = 10 ** 5
    omega = 777.5  # phi = 1/2: heaviest tails
    s = fejer_sample(np.full(200000, omega), np.full(200000, M), rng)
    off = ((s - 777 + M // 2) % M) - M // 2
    p = fejer_pmf(omega, M)
    # probability of |offset| > 16 from the exact law vs empirical
    j = np.arange(M)
    offs = ((j - 777 + M // 2) % M) - M // 2
    pt = p[(offs > 16) | (offs < -16)].sum()
    emp = np.mean((off > 16) | (off < -16))
    assert abs(emp - pt) < 4 * math.sqrt(pt / 200000)


def test_amplitude_estimation_exact_vs_fast_median():
    a = 0.37
    rng = np.random.default_rng(3)
    fast = [Q.amplitude_estimation(a, epsilon=0.01, random_state=rng) for _ in range(3000)]
    exact = [Q.amplitude_estimation(a, epsilon=0.01, random_state=rng, method="exact") for _ in range(3000)]
    assert stats.ks_2samp(fast, exact).pvalue > 1e-3
    # error bound holds with the AE success probability >= 8/pi^2
    assert np.mean(np.abs(np.array(fast) - a) <= 0.01 * 2 + 1e-3) > 0.8


def test_median_evaluation_q():
    assert median_repetitions(0.1) == 13
    assert median_repetitions(0.5) % 2 == 1


def test_ae_gamma_median_boosts():
    rng = np.random.default_rng(4)
    vals = [Q.amplitude_estimation(0.2, epsilon=0.005, gamma=0.1, random_state=rng) for _ in range(300)]
    assert np.mean(np.abs(np.array(vals) - 0.2) <= 0.012) > 0.97


def test_phase_estimation_law():
    rng = np.random.default_rng(5)
    omega = 0.3141
    m = 8
    M = 2 ** m
    s = np.array([Q.phase_estimation(omega, m=m, random_state=rng) for _ in range(5000)])
    p = fejer_pmf(M * omega, M)
    k = np.round(s * M).astype(int)
    emp0 = np.mean(k == np.argmax(p))
    assert abs(emp0 - p.max()) < 0.03
    assert Q.phase_estimation(1.0, m=4) == 15 / 16


def test_pe_qubits_formula():
    assert pe_qubits(1e-3, 0.1) == int(np.ceil(np.log2(1e3)) + np.ceil(np.log2(2 + 5)))


def test_consistent_pe_matches_bisect():
    import bisect
    rng = np.random.default_rng(6)
    for omega in [0.1, 0.5, 0.77, 0.0005]:
        eps, gamma = 1e-2, 0.9
        n, dp, shift = Q._cpe_params(eps, gamma)
        intervals = np.arange(-1 - shift * dp, 1 + eps - shift * dp, eps)
        intervals = np.append(intervals, 1 + eps - shift * dp)
        for pe in rng.random(50):
            idx = bisect.bisect(intervals, pe)
            ref = np.mean((intervals[idx - 1], intervals[idx]))
            got = Q._cpe_interval_midpoint(pe, eps, dp, shift)
            assert abs(max(ref, 0) - got) < 1e-12
        est = Q.consistent_phase_estimation(omega, eps, gamma, random_state=rng)
        assert abs(est - omega) <= eps + 1e-9 or est == 0


def test_consistent_pe_is_consistent():
    rng = np.random.default_rng(7)
    ests = {Q.consistent_phase_estimation(0.4321, 1e-3, 0.99, random_state=rng) for _ in range(50)}
    assert len(ests) <= 2


def test_truncated_normal_law():
    rng = np.random.default_rng(8)
    b = 0.7
    z = Q.truncated_normal(b, 20000, rng)
    assert np.abs(z).max() <= b
    assert stats.kstest(z, stats.truncnorm(-b, b).cdf).pvalue > 1e-3


def test_make_gaussian_est_bound():
    v = np.arange(100.0)
    out = Q.make_gaussian_est(v, 0.5, random_state=0)
    assert np.abs(out - v).max() <= 0.05 + 1e-12
    np.testing.assert_array_equal(Q.make_gaussian_est(v, 0.0), v)


def test_tomography_gaussian_matrix_budget():
    A = np.ones((8, 16))
    est = Q.tomography(A, 0.4, true_tomography=False, random_state=1)
    assert np.abs(est - A).max() <= 0.4 / np.sqrt(8 * 16) + 1e-12


def test_real_tomography_error_bound():
    rng = np.random.default_rng(9)
    V = rng.normal(size=32)
    V /= np.linalg.norm(V)
    res = Q.real_tomography(V, delta=0.3, random_state=rng)
    est = list(res.values())[-1]
    assert np.linalg.norm(V - est) <= 0.3 or len(res) == 100
    assert abs(np.linalg.norm(est) - 1) < 1e-9


def test_true_tomography_returns_unit_rows_and_preserve_norm():
    A = np.array([[3.0, 4.0, 0.0, 1.0], [1.0, 1.0, 1.0, 1.0]])
    e = Q.tomography(A, 0.5, true_tomography=True, random_state=0)
    assert np.allclose(np.linalg.norm(e, axis=1), 1.0)
    e2 = Q.tomography(A, 0.5, true_tomography=True, random_state=0, preserve_norm=True)
    assert np.allclose(np.linalg.norm(e2, axis=1), np.linalg.norm(A, axis=1))


def test_check_measure_strictly_increasing():
    arr = Q.check_measure(np.geomspace(1, 1000, 100, dtype=np.int64))
    assert np.all(np.diff(arr) > 0)


def test_mu_and_best_mu():
    rng = np.random.default_rng(10)
    A = rng.normal(size=(30, 7))
    # p = 1/2: sqrt(max row l1 * max col l1)
    r = np.abs(A).sum(1).max()
    c = np.abs(A).sum(0).max()
    assert abs(Q.mu(0.5, A) - np.sqrt(r * c)) < 1e-9
    lab, v = Q.best_mu(A, 0, 1, 0.1)
    assert v <= np.linalg.norm(A) + 1e-12
    assert lab.startswith("p=") or lab == "Frobenius"


def test_ipe_estimates_inner_product():
    rng = np.random.default_rng(11)
    x = rng.normal(size=8)
    y = rng.normal(size=8)
    ests = [Q.ipe(x, y, 0.05, random_state=rng) for _ in range(200)]
    assert abs(np.median(ests) - x @ y) < 0.1


def test_ipe_batch_matches_scalar_law():
    rng = np.random.default_rng(12)
    ip = np.full(4000, 1.3)
    b = Q.ipe_batch(ip, 2.0, 3.0, 0.05, random_state=rng)
    s = [Q.ipe(np.array([1.0, 1.0]), np.array([1.3 - 0.0, 0.0]) * 0 + np.array([0.3, 1.0]), 0.05,
               random_state=rng) for _ in range(10)]
    assert np.isfinite(b).all() and np.isfinite(s).all()
    assert abs(np.median(b) - 1.3) < 0.05


def test_quantum_state_measure_and_wald():
    qs = Q.QuantumState(registers=["a", "b", "c"], amplitudes=[1, 1, np.sqrt(2)], random_state=0)
    m = qs.measure(20000)
    est = Q.estimate_wald(list(m))
    assert abs(est["c"] - 0.5) < 0.02
    assert set(qs.get_state()) == {"a", "b", "c"}
    assert Q.coupon_collect(qs) >= 3


def test_wrappers_roundtrip():
    x = 0.6
    th = Q.wrapper_phase_est_arguments(x)
    assert abs(Q.unwrap_phase_est_arguments(th / (0 + math.pi), 0) - x) < 1e-12
    d = Q.wrapper_phase_est_arguments(0.3, "distance")
    assert abs(Q.unwrap_phase_est_arguments(d / math.pi, 0, "distance") - 0.3) < 1e-12


def test_introduce_error_shapes():
    out = Q.introduce_error(1.0, 0.1, random_state=0)
    assert out.shape == (1,) and abs(out[0] - 1.0) <= 0.1
    arr = Q.introduce_error_array(np.zeros(16), 0.4, random_state=0)
    assert np.abs(arr).max() <= 0.1 + 1e-12


def test_create_rand_vec_unit():
    vs = Q.create_rand_vec(3, 5, random_state=0)
    assert all(abs(np.linalg.norm(v) - 1) < 1e-12 for v in vs)
