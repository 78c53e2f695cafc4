"""Why a row is or is not skipped by the ipe16 row skip, over a Lloyd
trajectory: per step the largest centroid shift (smax), and on a row
subsample the kept bound lb against the true smallest non-label distance,
and the two skip conditions (lb^2 >= need_lo, ub^2 <= need_hi) evaluated
from the step's own bands (rows the sweep saw)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))
from sq_learn_amd.models._data import Data, gather_rows  # noqa: E402
from sq_learn_amd.models.cluster._lloyd import LloydEngine  # noqa: E402
from sq_learn_amd.parallel.comm import Comm  # noqa: E402
from sq_learn_amd.utils.datasets import make_blobs_device  # noqa: E402


def q(t, ps=(0.01, 0.1, 0.5, 0.9)):
    t = t.float()
    t = t[torch.isfinite(t)]
    if t.numel() == 0:
        return []
    return [round(float(v), 3) for v in torch.quantile(t, torch.tensor(ps, device=t.device))]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2_000_000
    d = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    k = int(sys.argv[3]) if len(sys.argv) > 3 else 1024
    steps = int(sys.argv[4]) if len(sys.argv) > 4 else 8
    seed = 2024
    dev = torch.device("cuda")
    X, _ = make_blobs_device(n, d, centers=k, cluster_std=1.0, seed=seed, device=dev,
                             dtype=torch.float32)
    C0 = gather_rows(Data(X, n, 0, Comm(None), "sharded"),
                     np.random.RandomState(seed).choice(n, k, replace=False))
    eng = LloydEngine(X, k, delta=0.5, true_distance_estimate=True, intermediate_error=True,
                      true_tomography=False, seed=seed, comm=Comm(None), gemm_precision="fp32")
    eng.set_centers(C0)
    eng.ipe16_stats = torch.zeros(8, dtype=torch.int64, device=dev)
    sub = torch.arange(0, n, max(1, n // 20000), device=dev)[:20000]
    prev_skip = None
    for s in range(steps):
        C = eng.centers().clone().double()
        st0 = getattr(eng, "_ipe16", None)
        lb_before = st0.lb[sub].double().clone() if st0 is not None else None
        eng.ipe16_stats.zero_()
        lab, sc = eng.step()
        sc.tolist()
        st = eng._ipe16
        skipped = st.rflag[sub] == 2
        lab_s = lab[sub].long()
        hint = eng._ipe_lab[eng._ipe_cur ^ 1][sub].long()
        Xs = X[sub].double()
        D = (Xs * Xs).sum(1)[:, None] + (C * C).sum(1)[None, :] - 2.0 * Xs @ C.T
        Dn = D.clone()
        Dn[torch.arange(len(sub), device=dev), lab_s] = float("inf")
        dmin = Dn.min(1).values.clamp_min(0).sqrt()
        lbv = st.lb[sub].double()
        swept = st.rflag[sub] != 2
        a2 = st.alpha ** 2
        vlo = st.vlo[sub].double()[:, :st.G]
        vhi = st.vhi[sub].double()[:, :st.G]
        need_lo = (vlo.max(1).values) / a2 + (X[sub].double() ** 2).sum(1)
        need_hi = (vhi.min(1).values) / a2 + (X[sub].double() ** 2).sum(1)
        dh = D.gather(1, hint.clamp_min(0)[:, None])[:, 0].clamp_min(0).sqrt()
        ub = dh + st.Rc[hint.clamp_min(0)].double().amax(1)
        mwv = st.mw[hint.clamp_min(0)].double() - dh
        # per-group upper condition (need_hi per group vs dh + Rc[hint][g])
        Rcg = st.Rc[hint.clamp_min(0)].double()[:, :st.G]
        up_ok = ((dh[:, None] + Rcg) ** 2 <= vhi / a2 + (X[sub].double() ** 2).sum(1)[:, None]).all(1)
        lbb = lb_before if lb_before is not None else lbv
        lo_ok = (lbb - float(st.smax)).clamp_min(0) ** 2 >= need_lo
        sw = ~skipped
        fails = {"swept": int(sw.sum()),
                 "lo_fail_only": float((sw & ~lo_ok & up_ok).double().sum() / max(int(sw.sum()), 1)),
                 "up_fail_only": float((sw & lo_ok & ~up_ok).double().sum() / max(int(sw.sum()), 1)),
                 "both_fail": float((sw & ~lo_ok & ~up_ok).double().sum() / max(int(sw.sum()), 1)),
                 "neither_fail": float((sw & lo_ok & up_ok).double().sum() / max(int(sw.sum()), 1)),
                 "up_ratio_q(swept)": q(((dh[:, None] + Rcg).amax(1) ** 2 /
                                        (vhi / a2 + (X[sub].double() ** 2).sum(1)[:, None]).amin(1))[sw])}
        mw_ok = mwv.clamp_min(0) ** 2 >= need_lo
        trans = {}
        if prev_skip is not None:
            for nm, m in (("after_skip", prev_skip), ("after_sweep", ~prev_skip)):
                trans[nm] = {"rows": int(m.sum()), "skip_now": float(skipped[m].double().mean()),
                             "lo_ok": float(lo_ok[m].double().mean()),
                             "mw_ok": float(mw_ok[m].double().mean()),
                             "up_ok": float(up_ok[m].double().mean()),
                             "lbe_minus_needlo_q": q((lbv - float(st.smax) - need_lo.clamp_min(0).sqrt())[m])}
        prev_skip = skipped
        rec = {"step": s, "smax": float(st.smax), "skipped": int(eng.ipe16_stats[7]),
               "trans": trans, "fails": fails,
               "Rc_q": q(st.Rc[:k]), "lb_over_true_q": q((lbv / dmin)[lbv > 0]),
               "lb_zero_frac": float((lbv == 0).double().mean()),
               "lb_q": q(lbv), "dmin_q": q(dmin),
               "swept_need_lo_sqrt_q": q(need_lo[swept].clamp_min(0).sqrt()),
               "swept_lb_minus_needlo_q": q((lbv - need_lo.clamp_min(0).sqrt())[swept]),
               "swept_ub_q": q(ub[swept]), "swept_need_hi_sqrt_q": q(need_hi[swept].clamp_min(0).sqrt()),
               "lab_eq_hint": float((lab_s == hint).double().mean()),
               "mw_minus_dh_q": q(mwv), "n_wild": st.n_wild,
               "lbdecayed_minus_needlo_q(swept)": q((lbv - float(st.smax) - need_lo.clamp_min(0).sqrt())[swept])}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
