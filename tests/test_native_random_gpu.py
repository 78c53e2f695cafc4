"""HIP stochastic kernels vs the torch/Philox reference path."""
import math

import numpy as np
import pytest
import torch

from sq_learn_amd.runtime.rng import RngKey, Philox
from sq_learn_amd.ops import random as R
from sq_learn_amd.ops import _native as nat

pytestmark = pytest.mark.gpu


def test_native_loaded(cuda):
    m = nat.native()
    assert m.__file__.endswith(".so")
    arch = m.device_arch()
    assert arch is not None and "gfx950" in arch[0]


def test_philox_uniform_bitexact(cuda):
    key = RngKey(1234, "generic", 7)
    g = R.philox_uniform((1000,), key, device=cuda, offset=13).cpu()
    c = R.philox_uniform((1000,), key, device="cpu", offset=13)
    assert torch.equal(g, c)


def test_trunc_normal_matches_cpu(cuda):
    key = RngKey(99, "trunc_normal", 3)
    x = torch.zeros(4096, dtype=torch.float32, device=cuda)
    R.trunc_normal_add_(x, 0.5, key, offset=5)
    y = torch.zeros(4096, dtype=torch.float32)
    R.trunc_normal_add_(y, 0.5, key, offset=5)
    assert torch.allclose(x.cpu(), y, atol=1e-5)
    assert float(x.abs().max()) <= 0.5


def test_normal_matches_cpu(cuda):
    key = RngKey(5, "data", 1)
    a = R.philox_normal((3000,), key, device=cuda).cpu()
    b = R.philox_normal((3000,), key, device="cpu")
    assert torch.allclose(a, b, atol=1e-4)


def test_ae_batch_distribution(cuda):
    key = RngKey(11, "ae", 0)
    a = torch.full((20000,), 0.3, dtype=torch.float64, device=cuda)
    eps = torch.full_like(a, 0.01)
    g = R.amplitude_estimation_batch(a, eps, key, Q=1).cpu().numpy()
    c = R.amplitude_estimation_batch(a.cpu()[:2000], eps.cpu()[:2000], key, Q=1).numpy()
    # same streams -> CPU twin reproduces the first 2000 device draws (rare fp32/fp64 boundary diffs)
    assert np.mean(np.isclose(g[:2000], c)) > 0.99
    assert abs(np.median(g) - 0.3) < 0.01
