"""Diagnostic: rows_f64 / x64 labels vs the torch fp64 band rule at large k."""
import numpy as np
import torch
from sq_learn_amd.models.cluster._lloyd import LloydEngine
from sq_learn_amd.ops import kmeans as K


def rule(X, C, delta, key, k_pad):
    D = torch.cdist(torch.from_numpy(X).double().cuda(), torch.from_numpy(C).double().cuda(),
                    compute_mode="donot_use_mm_for_euclid_dist") ** 2
    g = torch.arange(X.shape[0], dtype=torch.int64, device=D.device)
    lab, mn = K.band_select_torch(D, g, delta, key, k_pad)
    return D, lab, mn


for (n, d, k) in [(3001, 40, 20000), (3001, 40, 4000), (3001, 40, 8000), (3001, 40, 9000)]:
    rs = np.random.RandomState(k)
    X = (rs.randn(n, d) * 1.5).astype(np.float32)
    C = (X[rs.choice(n, k, replace=True)] + 0.05 * rs.randn(k, d)).astype(np.float32)
    Xt = torch.from_numpy(X).cuda()
    lab = torch.empty(n, dtype=torch.int32, device="cuda")
    mind = torch.empty(n, dtype=torch.float32, device="cuda")
    key = LloydEngine(Xt, 8, delta=0.3, seed=5)._key("band_select")
    K.rows_f64_native(Xt, torch.from_numpy(C).cuda(), lab, mind, 0.3, key, 0)
    D, lab64, mn64 = rule(X, C, 0.3, key, ((k + 63) // 64) * 64)
    bad = lab.long() != lab64
    band = (D <= (mn64 + 0.3)[:, None]).sum(1)
    inb = D.gather(1, lab.long()[:, None])[:, 0] <= mn64 + 0.3
    print(f"rows_f64 n={n} d={d} k={k}: bad={int(bad.sum())} mind_err={float(((mind.double()-mn64).abs()/mn64).max()):.2e} "
          f"label_in_band={float(inb.double().mean()):.3f} band_mean={float(band.double().mean()):.2f} band_max={int(band.max())}")
    if int(bad.sum()):
        i = int(torch.nonzero(bad)[0])
        mem = torch.nonzero(D[i] <= mn64[i] + 0.3)[:, 0].tolist()
        print("   row", i, "got", int(lab[i]), "want", int(lab64[i]), "members", mem[:40])
