"""The quantum error model pinned to the REFERENCE's own code.

``/root/reference/sklearn/QuantumUtility/Utility.py`` is loaded with
importlib (skipped when absent) and sampled side by side with

* the NumPy oracle (:mod:`sq_learn_amd.quantum.reference`),
* the device samplers' CPU twins (:mod:`sq_learn_amd.ops.random`,
  :mod:`sq_learn_amd.quantum.device`; the same Philox streams the HIP kernels
  draw, see ``tests/test_native_random_gpu.py`` for the bit-exact twin checks).

Discrete laws (AE, PE, CPE) are compared by a two-sample chi^2 on pooled
categories, continuous ones (Gaussian tomography noise, IPE, tomography
errors) by a two-sample Kolmogorov-Smirnov test.  The reference draws from
python's ``random`` and ``np.random`` (seeded here) and, inside
``QuantumState.measure``, from an unseeded ``RandomState`` - thresholds are
p > 1e-4 so a correct law fails about once in 10^4 runs.
"""
import importlib.util
import math
import os
import random

import numpy as np
import pytest
import torch
from scipy import stats

from sq_learn_amd.quantum import reference as Q
from sq_learn_amd.quantum import device as QD
from sq_learn_amd.ops import random as R
from sq_learn_amd.runtime.rng import RngKey

REF = "/root/reference/sklearn/QuantumUtility/Utility.py"
P_MIN = 1e-4


@pytest.fixture(scope="module")
def U():
    if not os.path.exists(REF):
        pytest.skip("reference Utility.py not present")
    try:
        import matplotlib  # noqa: F401  (the reference imports pyplot at module level)
        matplotlib.use("Agg")
    except ImportError:
        pytest.skip("matplotlib missing")
    spec = importlib.util.spec_from_file_location("_ref_utility", REF)
    mod = importlib.util.module_from_spec(spec)
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        spec.loader.exec_module(mod)
    return mod


def _seed(s):
    random.seed(s)
    np.random.seed(s)


def _chi2_two_sample(a, b):
    """p-value of 'a and b come from the same discrete law' (pools rare values)."""
    a = np.round(np.asarray(a, dtype=np.float64), 12)
    b = np.round(np.asarray(b, dtype=np.float64), 12)
    vals, inv = np.unique(np.concatenate([a, b]), return_inverse=True)
    ca = np.bincount(inv[: len(a)], minlength=len(vals)).astype(float)
    cb = np.bincount(inv[len(a):], minlength=len(vals)).astype(float)
    tot = ca + cb
    big = tot >= 10
    table = np.stack([ca[big], cb[big]], 0)
    rest = np.array([[ca[~big].sum()], [cb[~big].sum()]])
    if rest.sum() > 0:
        table = np.concatenate([table, rest], 1)
    if table.shape[1] < 2:
        return 1.0
    return stats.chi2_contingency(table)[1]


# --------------------------------------------------------------- Q10 / Q11
@pytest.mark.parametrize("a,eps", [(0.3, 0.05), (0.04, 0.04), (0.81, 0.06)])
def test_amplitude_estimation_law_matches_reference(U, a, eps):
    _seed(1)
    n = 3000
    ref = [U.amplitude_estimation(a, epsilon=eps) for _ in range(n)]
    rng = np.random.default_rng(2)
    ours = [Q.amplitude_estimation(a, epsilon=eps, random_state=rng) for _ in range(n)]
    assert _chi2_two_sample(ref, ours) > P_MIN
    # device sampler (CPU twin of ae_batch_kernel: same Philox streams)
    dev = R.amplitude_estimation_batch(torch.full((n,), a, dtype=torch.float64),
                                       torch.full((n,), eps, dtype=torch.float64),
                                       RngKey(3, "ae", 0), Q=1).numpy()
    assert _chi2_two_sample(ref, dev) > P_MIN


def test_amplitude_estimation_median_matches_reference(U):
    _seed(4)
    n = 600
    a, eps = 0.37, 0.08
    ref = [U.amplitude_estimation(a, epsilon=eps, gamma=0.1) for _ in range(n)]
    rng = np.random.default_rng(5)
    ours = [Q.amplitude_estimation(a, epsilon=eps, gamma=0.1, random_state=rng) for _ in range(n)]
    assert _chi2_two_sample(ref, ours) > P_MIN
    dev = R.amplitude_estimation_batch(torch.full((n,), a, dtype=torch.float64),
                                       torch.full((n,), eps, dtype=torch.float64),
                                       RngKey(6, "ae", 0), Q=13).numpy()
    assert _chi2_two_sample(ref, dev) > P_MIN


def test_median_evaluation_q_matches_reference(U):
    calls = []
    U.median_evaluation(lambda: calls.append(1) or 0.0, gamma=0.1)
    n_ref = len(calls)
    calls.clear()
    Q.median_evaluation(lambda: calls.append(1) or 0.0, gamma=0.1)
    assert n_ref == len(calls) == 13


# ---------------------------------------------------------------- Q12 / Q13
@pytest.mark.parametrize("omega,m", [(0.3141, 6), (0.05, 7), (0.77777, 5)])
def test_phase_estimation_law_matches_reference(U, omega, m):
    _seed(7)
    n = 4000
    ref = [U.phase_estimation(omega, m=m) for _ in range(n)]
    rng = np.random.default_rng(8)
    ours = [Q.phase_estimation(omega, m=m, random_state=rng) for _ in range(n)]
    assert _chi2_two_sample(ref, ours) > P_MIN
    dev = R.phase_estimation_batch(torch.full((n,), omega, dtype=torch.float64),
                                   torch.full((n,), m, dtype=torch.int32),
                                   RngKey(9, "pe", 0)).numpy()
    assert _chi2_two_sample(ref, dev) > P_MIN


def test_phase_estimation_epsilon_qubits_match_reference(U):
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        for eps, gamma in [(0.01, 0.1), (1e-3, 0.05), (0.2, 0.3)]:
            _, _, m_ref, M_ref = U.phase_estimation(0.4, epsilon=eps, gamma=gamma, nqubit=True)
            _, _, m, M = Q.phase_estimation(0.4, epsilon=eps, gamma=gamma, nqubit=True,
                                            random_state=0)
            assert (m_ref, M_ref) == (m, M)


@pytest.mark.parametrize("omega", [0.123, 0.5, 0.9])
def test_consistent_phase_estimation_law_matches_reference(U, omega):
    import warnings
    eps, gamma = 0.05, 0.1
    _seed(10)
    n = 300
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        ref = [U.consistent_phase_estimation(omega, eps, gamma) for _ in range(n)]
    rng = np.random.default_rng(11)
    ours = [Q.consistent_phase_estimation(omega, eps, gamma, random_state=rng) for _ in range(n)]
    assert _chi2_two_sample(ref, ours) > P_MIN
    # device path: consistent PE on the PE kernel's law
    dev = QD.consistent_phase_estimation_device(torch.full((n,), omega, dtype=torch.float64),
                                                eps, gamma, RngKey(12, "pe", 0)).numpy()
    assert _chi2_two_sample(ref, dev) > P_MIN
    # consistency: the reference returns (almost) one value; so do we
    assert np.mean(np.isclose(ours, np.median(ref))) > 0.9


# ---------------------------------------------------------------------- Q14
@pytest.mark.parametrize("gamma", [None, 0.1])
def test_ipe_law_matches_reference(U, gamma):
    """gamma=None: one AE draw (the Fejer law's spread); 0.1: the reference
    default, median of 13 (concentrated on one or two values)."""
    rs = np.random.RandomState(0)
    x = rs.standard_normal(32)
    y = x + 0.3 * rs.standard_normal(32)
    eps = 0.5
    _seed(13)
    n = 1500 if gamma is None else 300
    ref = np.array([U.ipe(x, y, eps, gamma=gamma) for _ in range(n)])
    rng = np.random.default_rng(14)
    ours = np.array([Q.ipe(x, y, eps, gamma=gamma, random_state=rng) for _ in range(n)])
    # a discrete law (S (1 - 2 sin^2(pi j / M)) / 2): chi^2 on values rounded
    # past the last-ulp differences of the two formulas
    r8 = lambda v: np.round(v, 8)  # noqa: E731
    assert _chi2_two_sample(r8(ref), r8(ours)) > P_MIN
    if gamma is None:
        assert len(np.unique(r8(ref))) > 3
    # the device sampler's twin (ae_batch_kernel streams) on the same pair
    S = x @ x + y @ y
    a = torch.full((n,), (S - 2 * (x @ y)) / (2 * S), dtype=torch.float64)
    ea = torch.full((n,), eps * max(1.0, abs(x @ y)) / S, dtype=torch.float64)
    at = R.amplitude_estimation_batch(a, ea, RngKey(16, "ipe", 0), Q=1 if gamma is None else 13).numpy()
    dev = S * (1 - 2 * at) / 2
    assert _chi2_two_sample(r8(ref), r8(dev)) > P_MIN
    if gamma is not None:
        # batched oracle of the fused device kernel
        bat = Q.ipe_batch(np.full(n, x @ y), np.full(n, x @ x), np.full(n, y @ y), eps,
                          gamma=gamma, random_state=np.random.default_rng(15))
        assert _chi2_two_sample(r8(ref), r8(bat)) > P_MIN


# ------------------------------------------------------------------ Q3 / Q4
def test_gaussian_tomography_noise_matches_reference(U):
    vec = np.linspace(-1, 1, 4000)
    noise = 0.7
    np.random.seed(17)
    ref = U.make_gaussian_est(vec, noise) - vec
    ours = Q.make_gaussian_est(vec, noise, random_state=18) - vec
    assert stats.ks_2samp(ref, ours).pvalue > P_MIN
    t = torch.tensor(vec, dtype=torch.float32)
    dev = (QD.gaussian_tomography(t, noise, RngKey(19, "tomography", 0)) - t).double().numpy()
    assert stats.ks_2samp(ref, dev).pvalue > P_MIN
    b = noise / math.sqrt(len(vec))
    assert np.abs(dev).max() <= b * (1 + 1e-6)


def test_matrix_tomography_budget_matches_reference(U):
    A = np.arange(60, dtype=np.float64).reshape(6, 10) / 60
    np.random.seed(20)
    ref = U.tomography(A, 0.5, true_tomography=False) - A
    ours = Q.tomography(A, 0.5, true_tomography=False, random_state=21) - A
    assert stats.ks_2samp(ref.ravel(), ours.ravel()).pvalue > P_MIN
    assert np.abs(ref).max() <= 0.5 / math.sqrt(60) and np.abs(ours).max() <= 0.5 / math.sqrt(60)


def _tomo_errors(est_fn, V, reps):
    return np.array([np.linalg.norm(V - np.asarray(est_fn(i))) for i in range(reps)])


@pytest.mark.parametrize("d,N", [(24, 3000), (700, 40000)])
def test_real_tomography_single_pass_matches_reference(U, d, N):
    """One pass with N shots (qPCA's default: incremental_measure=False)."""
    rs = np.random.RandomState(22)
    V = rs.standard_normal(d)
    V /= np.linalg.norm(V)
    reps = 150 if d < 100 else 60
    ref = _tomo_errors(lambda i: U.real_tomography(V, N=N, incremental_measure=False)[N], V, reps)
    rng = np.random.default_rng(23)
    ours = _tomo_errors(lambda i: Q.real_tomography(V, N=N, incremental_measure=False,
                                                    random_state=rng)[N], V, reps)
    assert stats.ks_2samp(ref, ours).pvalue > P_MIN
    # device code path (long-vector algorithm for d + 1 > 512, Philox twin otherwise)
    dev = _tomo_errors(lambda i: QD.tomography_rows_torch(
        torch.tensor(V)[None], None, RngKey(24, "tomography", i), N=N, incremental_measure=False,
        stop_when_reached_accuracy=False)[0].numpy(), V, reps)
    assert stats.ks_2samp(ref, dev).pvalue > P_MIN
    # sign rule: most signs right once N >> d
    est = np.asarray(Q.real_tomography(V, N=N, incremental_measure=False, random_state=1)[N])
    big = np.abs(V) > 1 / math.sqrt(d)
    assert big.any()
    assert np.mean(np.sign(est[big]) == np.sign(V[big])) > 0.9


def test_real_tomography_stopping_rule_matches_reference(U):
    rs = np.random.RandomState(25)
    d, delta = 16, 0.3
    V = rs.standard_normal(d)
    V /= np.linalg.norm(V)
    reps = 60
    ref_n, ref_e = [], []
    for _ in range(reps):
        r = U.real_tomography(V, delta=delta)
        n_last = list(r.keys())[-1]
        ref_n.append(n_last)
        ref_e.append(np.linalg.norm(V - np.asarray(r[n_last])))
    rng = np.random.default_rng(26)
    our_n, our_e = [], []
    for _ in range(reps):
        r = Q.real_tomography(V, delta=delta, random_state=rng)
        n_last = list(r.keys())[-1]
        our_n.append(n_last)
        our_e.append(np.linalg.norm(V - np.asarray(r[n_last])))
    assert max(ref_e) <= delta and max(our_e) <= delta
    assert stats.ks_2samp(np.log(ref_n), np.log(our_n)).pvalue > P_MIN
    dev_e = [np.linalg.norm(V - QD.tomography_rows_torch(torch.tensor(V)[None], delta,
                                                         RngKey(27, "tomography", i))[0].numpy())
             for i in range(reps)]
    assert max(dev_e) <= delta


def test_fake_sign_tomography_matches_reference(U):
    rs = np.random.RandomState(28)
    V = rs.standard_normal(12)
    V /= np.linalg.norm(V)
    ref = _tomo_errors(lambda i: U.L2_tomogrphy_fakeSign(V, N=2000), V, 100)
    rng = np.random.default_rng(29)
    ours = _tomo_errors(lambda i: Q.L2_tomogrphy_fakeSign(V, N=2000, random_state=rng), V, 100)
    assert stats.ks_2samp(ref, ours).pvalue > P_MIN


# ----------------------------------------------------------------------- Q9
def test_best_mu_and_helpers_equal_reference(U):
    rs = np.random.RandomState(30)
    for shape in [(40, 7), (9, 31)]:
        A = rs.standard_normal(shape)
        A[A < -1.2] = 0.0
        assert U.best_mu(A) == Q.best_mu(A)
        assert U.best_mu(A, step=0.1)[1] == pytest.approx(Q.best_mu(A, step=0.1)[1], rel=1e-12)
    for w0, w1 in [(0.1, 0.95), (0.5, 0.5), (0.99, 0.01)]:
        assert U.amplitude_est_dist(w0, w1) == pytest.approx(Q.amplitude_est_dist(w0, w1))
    arr = np.array([1, 1, 2, 2, 2, 9, 9, 30], dtype=np.int64)
    np.testing.assert_array_equal(U.check_measure(arr.copy(), 0), Q.check_measure(arr, 0))
    for v, j in [(10, 3), (7, 7), (100, 6)]:
        assert U.check_division(v, j) == Q.check_division(v, j)
    for x in [0.1, 0.7]:
        assert U.wrapper_phase_est_arguments(x) == Q.wrapper_phase_est_arguments(x)
        assert U.wrapper_phase_est_arguments(x, "distance") == Q.wrapper_phase_est_arguments(x, "distance")
        assert U.unwrap_phase_est_arguments(x, 0.01) == Q.unwrap_phase_est_arguments(x, 0.01)


def test_introduce_error_law_matches_reference(U):
    np.random.seed(31)
    arr = np.zeros(3000)
    ref = U.introduce_error_array(arr, 2.0)
    ours = Q.introduce_error_array(arr, 2.0, random_state=32)
    assert stats.ks_2samp(ref, ours).pvalue > P_MIN
    ref1 = np.array([U.introduce_error(0.0, 0.3)[0] for _ in range(2000)])
    ours1 = np.array([Q.introduce_error(0.0, 0.3, random_state=i)[0] for i in range(2000)])
    assert stats.ks_2samp(ref1, ours1).pvalue > P_MIN


def test_quantum_state_and_coupon_match_reference(U):
    regs, amps = ["a", "b", "c"], [0.2, 0.5, 0.84]
    _seed(33)
    qs_ref = U.QuantumState(registers=regs, amplitudes=amps)
    qs = Q.QuantumState(registers=regs, amplitudes=amps, random_state=34)
    assert qs_ref.get_state() == pytest.approx(qs.get_state())
    ref = list(qs_ref.measure(6000))
    ours = list(qs.measure(6000))
    assert _chi2_two_sample([regs.index(r) for r in ref], [regs.index(r) for r in ours]) > P_MIN
    cref = [U.coupon_collect(qs_ref) for _ in range(300)]
    cours = [Q.coupon_collect(qs) for _ in range(300)]
    assert stats.ks_2samp(cref, cours).pvalue > P_MIN
