"""fp64-MFMA tall-skinny GEMMs (csrc/tsgemm64.hip) against plain PyTorch
fp64 references of the same ops: the Gram / cross product
(A - mu_a)^T (B - mu_b) and the projection (A - mu) W, for feature counts
from 1 to 1024 (tile tails, several tile pairs), fp32 / bf16 / fp64 inputs,
row strides that defeat the vector loads, empty shards, and the chunked
accumulate mode; plus CholeskyQR2 and the randomized SVD at d = 512 / 784."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from sq_learn_amd.ops import linalg as L  # noqa: E402
from sq_learn_amd.parallel.comm import Comm  # noqa: E402


def _close(got, ref):
    torch.testing.assert_close(got.cpu(), ref, rtol=1e-12, atol=1e-10 * float(ref.abs().max() + 1))


@pytest.mark.parametrize("n,d", [(100_003, 256), (4097, 37), (9, 16), (20_000, 300),
                                 (1, 5), (30_001, 784), (5000, 1024), (0, 64)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float64])
@pytest.mark.parametrize("centred", [False, True])
def test_gram_matches_fp64(cuda, n, d, dtype, centred):
    g = torch.Generator().manual_seed(n * 7 + d)
    X = (torch.randn(n, d, generator=g) * 3 + 5).to(dtype)
    mean = X.double().mean(0) if (centred and n) else (torch.zeros(d, dtype=torch.float64) if centred else None)
    G = L.gram64_native(X.to(cuda), None if mean is None else mean.to(cuda))
    Xd = X.double() - (mean if centred else 0.0)
    ref = Xd.T @ Xd
    _close(G, ref)
    assert torch.equal(G.cpu(), G.cpu().T)


@pytest.mark.parametrize("n,da,db", [(50_001, 256, 26), (7777, 512, 64), (3000, 784, 10),
                                     (12_345, 130, 200), (100, 1024, 128), (33, 20, 300)])
@pytest.mark.parametrize("dtypes", [(torch.float32, torch.float64), (torch.bfloat16, torch.float32),
                                    (torch.float64, torch.float64)])
def test_cross_matches_fp64(cuda, n, da, db, dtypes):
    g = torch.Generator().manual_seed(n + da * 3 + db)
    A = (torch.randn(n, da, generator=g) * 2 - 1).to(dtypes[0])
    B = torch.randn(n, db, generator=g).to(dtypes[1])
    ma = A.double().mean(0)
    C = L.xtx(A.to(cuda), B.to(cuda), mean_a=ma.to(cuda))
    ref = (A.double() - ma).T @ B.double()
    _close(C, ref)


def test_strided_rows_and_accumulate(cuda):
    """Row stride > d (a column slice of a wider matrix, unaligned for the
    vector loads) and the chunked += mode used by CholeskyQR2 pass 2."""
    g = torch.Generator().manual_seed(3)
    W = torch.randn(20_000, 301, generator=g)
    A = W[:, 3:260]                                # stride 301, offset 3: scalar loads
    assert A.stride(0) == 301
    Ad = A.to(cuda)
    out = torch.zeros(257, 257, dtype=torch.float64, device=cuda)
    for s in range(0, 20_000, 7000):
        L.xtx(Ad[s:s + 7000], out=out, accumulate=True)
    ref = A.double().T @ A.double()
    _close(out, ref)


@pytest.mark.parametrize("n,d,l", [(100_003, 256, 26), (5000, 784, 784), (4097, 37, 37),
                                   (20_000, 512, 64), (1, 3, 2), (9999, 1024, 130)])
@pytest.mark.parametrize("upper", [False, True])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float64])
def test_xw_matches_fp64(cuda, n, d, l, upper, dtype):
    if upper and d != l:
        pytest.skip("triangular W is square")
    g = torch.Generator().manual_seed(n + d + l)
    A = (torch.randn(n, d, generator=g) + 1).to(dtype)
    Wm = torch.randn(d, l, generator=g, dtype=torch.float64)
    if upper:
        Wm = torch.triu(Wm)
    mu = A.double().mean(0)
    Y = L.xw(A.to(cuda), Wm.to(cuda), mean=mu.to(cuda), upper=upper)
    ref = (A.double() - mu) @ Wm
    _close(Y, ref)
    Y32 = L.xw(A.to(cuda), Wm.to(cuda), mean=mu.to(cuda), upper=upper, out_dtype=torch.float32)
    torch.testing.assert_close(Y32.cpu().double(), ref, rtol=2e-6, atol=1e-6 * float(ref.abs().max() + 1))


@pytest.mark.parametrize("d", [512, 784])
def test_cholqr2_sigma_wide(cuda, d):
    """sigma_min / sigma_max of a d = 512 / 784 matrix with cond ~1e6 to
    LAPACK fp64 precision (the q-means prelude and qPCA full path at BASELINE
    configs 2 / 4 shapes)."""
    n = 40_000
    rng = np.random.default_rng(d)
    Q1, _ = np.linalg.qr(rng.standard_normal((n, d)))
    Q2, _ = np.linalg.qr(rng.standard_normal((d, d)))
    s = np.logspace(0, -6, d)
    X = (Q1 * s) @ Q2.T
    ref = np.linalg.svd(X, compute_uv=False)
    R = L.cholqr2_r(torch.tensor(X, dtype=torch.float64, device=cuda), Comm(None))
    got = torch.linalg.svdvals(R.cpu()).numpy()
    np.testing.assert_allclose(got, ref, rtol=1e-9)


@pytest.mark.parametrize("method", ["gram", "stream"])
@pytest.mark.parametrize("d,dtype", [(512, torch.bfloat16), (784, torch.float32)])
def test_randomized_svd_wide(cuda, d, dtype, method):
    """Randomized range finder at d = 512 (BASELINE config 2 dtype) and 784:
    the top singular values of a matrix with a decaying spectrum match the
    exact fp64 SVD of the same (rounded) data, on both the Gram-domain and
    the streamed range finder."""
    from sq_learn_amd.utils.extmath import randomized_svd_distributed
    n, k = 60_000, 10
    g = torch.Generator().manual_seed(d)
    U0, _ = torch.linalg.qr(torch.randn(n, 40, generator=g, dtype=torch.float64))
    V0, _ = torch.linalg.qr(torch.randn(d, 40, generator=g, dtype=torch.float64))
    s0 = torch.logspace(2, 0, 40, dtype=torch.float64)
    X = ((U0 * s0) @ V0.T + 1e-3 * torch.randn(n, d, generator=g, dtype=torch.float64)).to(dtype)
    mu = X.double().mean(0)
    ref = torch.linalg.svdvals(X.double() - mu)[:k]
    U, s, Vt = randomized_svd_distributed(X.to(cuda), mu.to(cuda), k, Comm(None), seed=0,
                                          method=method)
    torch.testing.assert_close(s.cpu(), ref, rtol=1e-7, atol=0)
    # U^T U = I, U S Vt reconstructs the top-k part
    UtU = (U.T @ U).cpu()
    torch.testing.assert_close(UtU, torch.eye(k, dtype=torch.float64), atol=1e-9, rtol=0)
