"""fp64 CholeskyQR2 sigma_min and full SVD on the device (row data fp32)."""
import numpy as np
import pytest
import torch

from sq_learn_amd.models._data import as_data, sigma_min
from sq_learn_amd.models.decomposition._svd import full_svd

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("cond", [1e3, 1e6])
def test_sigma_min_gpu_matches_lapack(cuda, cond):
    rng = np.random.RandomState(0)
    n, d = 400000, 64
    U, _ = np.linalg.qr(rng.standard_normal((n, d)))
    V, _ = np.linalg.qr(rng.standard_normal((d, d)))
    S = np.logspace(0, -np.log10(cond), d)
    X32 = ((U * S) @ V.T).astype(np.float32)
    ref = np.linalg.svd(X32.astype(np.float64), compute_uv=False)
    got = sigma_min(as_data(torch.tensor(X32, device=cuda)))
    assert abs(got - ref.min()) <= 1e-8 * ref.min() * cond / 1e3
    res = full_svd(as_data(torch.tensor(X32, device=cuda)), torch.zeros(d, device=cuda), 3)
    assert res.method == "cholqr2"
    np.testing.assert_allclose(res.S, ref, rtol=1e-8 * cond / 1e3)


@pytest.mark.parametrize("d", [7, 16, 100, 256])
def test_gram64_kernel_exact(cuda, d):
    from sq_learn_amd.ops.linalg import gram64_native
    rng = np.random.RandomState(d)
    n = 50021
    X = rng.standard_normal((n, d)).astype(np.float32)
    mu = X.astype(np.float64).mean(0)
    G = gram64_native(torch.tensor(X, device=cuda), torch.tensor(mu, device=cuda)).cpu().numpy()
    Xc = X.astype(np.float64) - mu
    np.testing.assert_allclose(G, Xc.T @ Xc, rtol=1e-12, atol=1e-9)
    G64 = gram64_native(torch.tensor(Xc, device=cuda)).cpu().numpy()
    np.testing.assert_allclose(G64, Xc.T @ Xc, rtol=1e-12, atol=1e-9)


def test_gram64_kernel_bf16(cuda):
    from sq_learn_amd.ops.linalg import gram64_native
    rng = np.random.RandomState(1)
    X = torch.tensor(rng.standard_normal((30001, 128)), dtype=torch.bfloat16, device=cuda)
    Xd = X.double().cpu().numpy()
    G = gram64_native(X).cpu().numpy()
    np.testing.assert_allclose(G, Xd.T @ Xd, rtol=1e-12, atol=1e-9)
