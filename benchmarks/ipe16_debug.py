"""Debug: the screen's near lists against a host recomputation of the band
test (v = alpha^2 (|c|^2 - 2 x.c) in fp64 vs the rows' [vlo, vhi])."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))
from sq_learn_amd.ops import kmeans as K  # noqa: E402
from sq_learn_amd.runtime.rng import RngKey  # noqa: E402
from sq_learn_amd.utils.datasets import make_blobs_device  # noqa: E402


def main():
    n = 4096
    d = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    dev = torch.device("cuda")
    X, _ = make_blobs_device(n, d, centers=k, cluster_std=1.0, seed=1, device=dev, dtype=torch.float32)
    Xc, _ = make_blobs_device(20000, d, centers=k, cluster_std=1.0, seed=1, device=dev, dtype=torch.float32)
    C = Xc[torch.randperm(20000, generator=torch.Generator().manual_seed(0))[:k].to(dev)].contiguous()
    xn = (X.double() ** 2).sum(1).float().contiguous()
    cn = (C * C).sum(1).contiguous()
    alpha = K.choose_alpha(float(xn.max()), 0.5)
    st = K.Ipe16(X, k, K.pad_features(d), K.pad_clusters(k), alpha, dev)
    st.set_centers(C)
    D = torch.cdist(X.double(), C.double()) ** 2
    hint = D.argmin(1).to(torch.int32)
    lab = torch.empty(n, dtype=torch.int32, device=dev)
    mind = torch.empty(n, dtype=torch.float32, device=dev)
    stats = torch.zeros(8, dtype=torch.int64, device=dev)
    keys = [RngKey(1, p, 0) for p in ("ipe", "band_select", "ipe16_skip", "ipe16_row")]
    nd = {}

    def fb(rl, rc, ln, thr, hj, s, e):
        nd["n"] = ln

    st.estep(X, C, hint.clone(), xn, cn, lab, mind, 0.25, 13, *keys, 0, False, stats=stats,
             fallback=fb)
    torch.cuda.synchronize()
    print("alpha", alpha, "stats", stats.tolist(), "dense", nd)
    cnt = int(st.counts[0, 0])
    ent = st.list[:cnt].cpu().numpy()
    rows = ent >> 16
    js = ent & 0x3FFF
    fired = (ent & 0x8000) != 0
    v = alpha ** 2 * ((C.double() ** 2).sum(1)[None, :] - 2 * X.double() @ C.double().T)
    vlo = st.vlo[:n].double()[:, None]
    vhi = st.vhi[:n].double()[:, None]
    near_ref = ~((v >= vlo) & (v <= vhi))
    near_ref[torch.arange(n), hint.long()] = False
    rst = st.rst[:n].cpu().numpy()
    nr = near_ref.sum(1).cpu().numpy()
    got = np.bincount(rows[~fired], minlength=n)
    ok = rst == 0
    print(json.dumps({"rows_ok": int(ok.sum()), "near_ref_mean": float(nr[ok].mean()),
                      "near_kernel_mean": float(got[ok].mean()),
                      "rows_mismatch": int((nr[ok] != got[ok]).sum())}))
    Dl = (st.vlo[:n].double() / alpha ** 2 + xn.double()).cpu().numpy()
    Dh = (st.vhi[:n].double() / alpha ** 2 + xn.double()).cpu().numpy()
    ovf = np.where(ok & (st.rflag[:n].cpu().numpy() != 0))[0]
    print("overflow rows", len(ovf))
    for r in list(np.where(ok)[0][:4]) + list(ovf[:6]):
        dd = D[r].cpu().numpy()
        print(json.dumps({"row": int(r), "thr": float(st.thr[r]), "xn": float(xn[r]),
                          "Dl": float(Dl[r]), "Dh": float(Dh[r]), "H": float(st.H[r]),
                          "Dmin2": sorted(dd.tolist())[:4], "Dmax": float(dd.max()),
                          "near_ref": int(nr[r]), "near_kernel": int(got[r]),
                          "kernel_js": js[rows == r][:8].tolist()}))


if __name__ == "__main__":
    main()
