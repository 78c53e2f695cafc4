"""fp64-MFMA Gram kernel (csrc/gram64.hip) against a plain PyTorch fp64
reference of the same op: fp32 / bf16 / fp64 input, with and without the
centring mean, odd feature counts and row counts that are not a multiple of
the 8-row (two k-step) stride."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from sq_learn_amd.ops import linalg as L  # noqa: E402


@pytest.mark.parametrize("n,d", [(100_003, 256), (4097, 37), (9, 16), (50_000, 200), (1, 5)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float64])
@pytest.mark.parametrize("centred", [False, True])
def test_gram64_matches_fp64(n, d, dtype, centred):
    g = torch.Generator().manual_seed(n * 7 + d)
    X = (torch.randn(n, d, generator=g) * 3 + 5).to(dtype)
    mean = X.double().mean(0) if centred else None
    G = L.gram64_native(X.cuda(), None if mean is None else mean.cuda())
    Xd = X.double() - (mean if centred else 0.0)
    ref = Xd.T @ Xd
    torch.testing.assert_close(G.cpu(), ref, rtol=1e-12, atol=1e-9 * float(ref.abs().max()))
    assert torch.equal(G.cpu(), G.cpu().T)
