"""Skip fraction of the ipe16 row skip on the orthogonal-competitor case
(tests/test_ipe16_gpu.py _fire_case) as the competitors' distance s varies:
picks the band-edge case of tests/test_ipe16_skip_gpu.py."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "tests")))
sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))
from test_ipe16_gpu import _fire_case  # noqa: E402
from test_ipe16_skip_gpu import _two_steps  # noqa: E402

dev = torch.device("cuda")
n = 100_000
for s in (4.0, 5.0, 6.0, 7.0, 8.0, 9.0, 10.0, 12.0, 14.0, 18.0):
    x, C = _fire_case(s=s)
    X = torch.tensor(np.tile(x, (n, 1)), device=dev)
    Ct = torch.tensor(C, device=dev)
    hint = torch.zeros(n, dtype=torch.int32, device=dev)
    st = torch.zeros((2, 8), dtype=torch.int64, device=dev)
    out, _ = _two_steps(X, Ct, 0.25, 13, 8, True, hint0=hint, ht=9e-4, stats=st)
    print(s, st.tolist(), flush=True)
