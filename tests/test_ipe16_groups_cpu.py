"""The ipe16 norm-group DP (``Ipe16.group_tiles``, host library
``sqh_group_tiles``) equals the numpy formulation (``group_tiles_np``) cut
for cut: random sorted norms, duplicated values (ties), outliers, partial
last tiles, G = 1..4."""
import numpy as np
import pytest

from sq_learn_amd.ops.kmeans import Ipe16


@pytest.mark.parametrize("seed", range(40))
def test_host_group_dp_matches_numpy(seed):
    rng = np.random.default_rng(seed)
    k = int(rng.integers(1, 3000))
    nt = -(-k // 64)
    kind = seed % 4
    if kind == 0:
        cs = rng.random(k)
    elif kind == 1:
        cs = np.round(rng.random(k) * 4) / 4          # many ties
    elif kind == 2:
        cs = np.concatenate([rng.random(k - min(k, 5)), 50 + rng.random(min(k, 5))])
    else:
        cs = np.full(k, 3.0)
    cs = np.sort(cs)
    for G in range(1, min(4, nt) + 1):
        assert Ipe16.group_tiles(cs, k, nt, G) == Ipe16.group_tiles_np(cs, k, nt, G), (k, G)
