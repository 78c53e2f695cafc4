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
