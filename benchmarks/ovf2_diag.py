"""Diagnostic: rows whose label differs between the dense-row path with and
without the second (3 members per lane) 3-pass (SQ_OVF2), on the k = 6000
case of tests/test_estep_wide_gpu.py::test_large_k_filter."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from test_estep_wide_gpu import _data, _estep, _fp64_rule  # noqa: E402

n, d, k = 5000, 64, 6000
X, C = _data(n, d, k, seed=9, groups=200)
out = {}
for v in ("0", "1"):
    os.environ["SQ_OVF2"] = v
    eng, key, lab, mind, _ = _estep(X, C, 0.5)
    out[v] = (lab.clone(), eng.buf.counts.clone().cpu().tolist())
D, lab64, mn64 = _fp64_rule(X, C, 0.5, key, eng.k_pad)
print("counts off/on", out["0"][1], out["1"][1])
bad = torch.nonzero(out["1"][0] != lab64)[:, 0].tolist()
print("mismatch rows (ovf2 on):", bad[:10], "off:", torch.nonzero(out["0"][0] != lab64)[:, 0].tolist()[:10])
for r in bad[:5]:
    m = float(mn64[r])
    mem = torch.nonzero(D[r] <= m + 0.5)[:, 0].tolist()
    kap = sorted(mem, key=lambda j: (j % 32, j // 32))
    print("row", r, "band", len(mem), "ref", int(lab64[r]), "on", int(out["1"][0][r]),
          "off", int(out["0"][0][r]))
    print("  kappa order", kap)
    print("  rank ref", kap.index(int(lab64[r])) if int(lab64[r]) in kap else None,
          "rank on", kap.index(int(out["1"][0][r])) if int(out["1"][0][r]) in kap else None)
    lanes = {}
    for j in mem:
        lanes.setdefault(j % 32, []).append(j)
    print("  per lane", {l: v for l, v in sorted(lanes.items()) if len(v) > 1})
