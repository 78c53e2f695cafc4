"""fp64-faithful sigma_min / condition number (reference: fp64 LAPACK SVD,
``_dmeans.py:1244-1245``) by sharded CholeskyQR2 - against numpy's SVD at
condition numbers 1e3..1e6, where the Gram eigenvalues alone lose
eps * cond^2."""
import numpy as np
import pytest
import torch

from sq_learn_amd.models._data import as_data, sigma_min
from sq_learn_amd.models.decomposition._svd import full_svd


def _matrix(n, d, cond, seed):
    rng = np.random.RandomState(seed)
    U, _ = np.linalg.qr(rng.standard_normal((n, d)))
    V, _ = np.linalg.qr(rng.standard_normal((d, d)))
    S = np.logspace(0, -np.log10(cond), d)
    return (U * S) @ V.T


@pytest.mark.parametrize("cond", [1e3, 1e6])
def test_sigma_min_matches_lapack(cond):
    X = _matrix(20000, 24, cond, 0)
    ref = np.linalg.svd(X, compute_uv=False).min()
    got = sigma_min(as_data(X, device="cpu"))
    assert abs(got - ref) <= 1e-9 * ref * cond / 1e3 + 1e-14


def test_full_svd_cholqr2_matches_lapack():
    X = _matrix(30000, 16, 1e5, 1) + 0.5
    d = as_data(X, device="cpu")
    mean = torch.tensor(X.mean(0))
    res = full_svd(d, mean, 4, method="cholqr2")
    assert res.method == "cholqr2"
    S = np.linalg.svd(X - X.mean(0), compute_uv=False)
    np.testing.assert_allclose(res.S, S, rtol=1e-9)


def test_rank_deficient_falls_back():
    rng = np.random.RandomState(2)
    A = rng.standard_normal((5000, 6))
    X = np.hstack([A, A[:, :2]])          # rank 6 of 8
    assert sigma_min(as_data(X, device="cpu")) < 1e-5


def test_single_pass_cholqr_tolerance_at_cond_100(monkeypatch):
    """cond(R1) <= 100 skips CholeskyQR2's second pass (ops.linalg.cholqr2_r):
    the singular values then carry ~eps64 cond^2 <= 2.2e-12 relative error
    and the right singular vectors ~that over the relative gap.  Pinned here
    against LAPACK at cond = 90, the worst case the shortcut accepts."""
    from sq_learn_amd.ops import linalg as L
    calls = {"n": 0}
    orig = L.gram64_local

    def counting(*a, **k):
        calls["n"] += 1
        return orig(*a, **k)

    monkeypatch.setattr(L, "gram64_local", counting)
    X = _matrix(40000, 16, 90.0, 3)
    d = as_data(X, device="cpu")
    mean = torch.zeros(16, dtype=torch.float64)
    res = full_svd(d, mean, 4, method="cholqr2")
    assert res.method == "cholqr2" and calls["n"] == 1     # one pass over X
    _, S, Vt = np.linalg.svd(X, full_matrices=False)
    np.testing.assert_allclose(res.S, S, rtol=3e-12)
    gap = np.min(np.abs(np.diff(S)) / S[:-1])
    for i in range(16):
        c = abs(float(np.dot(res.Vt[i], Vt[i])))
        assert 1.0 - c <= (3e-12 / gap) ** 2 + 1e-15
        assert np.linalg.norm(abs(res.Vt[i]) - abs(Vt[i])) <= 3e-11 / gap
