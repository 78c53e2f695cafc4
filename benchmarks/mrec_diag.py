"""Multi-candidate row records: how many steady-state multi rows could be
certified WITHOUT reading the row, under three bounds on the gap change
g_j = D_j - D_a (a = argmin) between Lloyd iterations (fp64, sampled rows):
  tri  : the triangle bound (sqrt(D_a) + s_a)^2 + delta < (sqrt(D_o) - max s_o)^2
  pair : g_j + dnu + 2 c_a.dw - 2 sqrt(D_a)|dw| > delta   (dw = shift_a - shift_j)
  proj : as pair, with dw split along w = c_a - c_j (x.w known from g_j)
and the truth (band still {a}).  Usage: python benchmarks/mrec_diag.py"""
import os
import sys
import json
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["SQ_MULTI_RECORDS"] = "0"


def main():
    from sq_learn_amd.utils.datasets import make_blobs_device
    from sq_learn_amd.models.cluster._lloyd import LloydEngine
    import numpy as np
    n = int(os.environ.get("ROWS", "10000000"))
    d, k, delta = 256, 1024, 0.5
    dev = torch.device("cuda", 0)
    X, _ = make_blobs_device(n, d, centers=1024, cluster_std=1.0, seed=0, device=dev,
                             dtype=torch.float32)
    rs = np.random.RandomState(0)
    C0 = X[torch.from_numpy(rs.choice(n, k, replace=False)).to(dev)]
    eng = LloydEngine(X, k, delta=delta, intermediate_error=True, seed=0)
    eng.set_centers(C0)
    for _ in range(8):
        eng.step()
    out = {}
    H = 4
    Cs = []
    for h in range(H + 1):
        Cs.append(eng.centers().double().clone())
        if h == 0:
            lab, mind, _ = eng._estep(eng._key("band_select"))
            torch.cuda.synchronize()
            m = int(eng.buf.counts[2].item())
            rows = eng.buf.multi_rows[:m].clone()
            cand = eng.buf.multi_cand[rows].clone()
            eng._pending = None
        eng.step()
    torch.cuda.synchronize()
    out["multi_rows"] = m
    sel = torch.randperm(m, device=dev)[:200000]
    rows, cand = rows[sel], cand[sel]
    c_r = cand[:, 0].clamp(0, 16)
    out["frac_two_cand"] = float((c_r == 2).double().mean())
    x = X[rows].double()
    nmax = int(c_r.max())
    J = cand[:, 1:1 + nmax].long()
    valid = torch.arange(nmax, device=dev)[None, :] < c_r[:, None]
    J = torch.where(valid, J, J[:, :1])

    def dists(C):
        return ((x[:, None, :] - C[J]) ** 2).sum(-1)
    D0 = dists(Cs[0])
    Dm = torch.where(valid, D0, torch.full_like(D0, float("inf")))
    ai = Dm.argmin(1)
    a = J.gather(1, ai[:, None])[:, 0]
    Da = Dm.gather(1, ai[:, None])[:, 0]
    other = valid & (torch.arange(nmax, device=dev)[None, :] != ai[:, None])
    g0 = torch.where(other, Dm - Da[:, None], torch.full_like(Dm, float("inf")))
    single = g0.min(1).values > delta          # band {a} at t
    out["band_single_frac"] = float(single.double().mean())
    res = {}
    for h in range(1, H + 1):
        C1 = Cs[h]
        Dh = dists(C1)
        gh = torch.where(other, Dh - Dh.gather(1, ai[:, None]), torch.full_like(Dh, float("inf")))
        truth = single & (gh.min(1).values > delta)
        # cumulative per-step shift norms (the ring of prefix sums)
        sh = sum(((Cs[t + 1] - Cs[t]) ** 2).sum(1).sqrt() for t in range(h))
        sa = sh[a]
        so = torch.where(other, sh[J], torch.zeros_like(Dh)).max(1).values
        lo = torch.where(other, Dm, torch.full_like(Dm, float("inf"))).min(1).values.sqrt()
        tri = single & ((Da.sqrt() + sa) ** 2 + delta < (lo - so).clamp(min=0) ** 2)
        # pair bound with the total displacement since t
        ca0, cj0 = Cs[0][a][:, None, :], Cs[0][J]
        ca1, cj1 = C1[a][:, None, :], C1[J]
        w0 = ca0 - cj0
        dw = (ca1 - ca0) - (cj1 - cj0)
        dnu = ((cj1 ** 2).sum(-1) - (ca1 ** 2).sum(-1)) - ((cj0 ** 2).sum(-1) - (ca0 ** 2).sum(-1))
        ra = Da.sqrt()[:, None]
        dwn = dw.norm(dim=-1)
        pair_lo = g0 + dnu + 2 * (ca0 * dw).sum(-1) - 2 * ra * dwn
        pair = single & torch.where(other, pair_lo > delta, torch.ones_like(other)).all(1)
        # projection: dw = beta w0 + dw_perp; x.w0 = (g0 - nu0)/2 exactly
        nu0 = (cj0 ** 2).sum(-1) - (ca0 ** 2).sum(-1)
        ww = (w0 ** 2).sum(-1).clamp(min=1e-300)
        beta = (dw * w0).sum(-1) / ww
        dperp = dw - beta[..., None] * w0
        xw = (g0.clamp(max=1e30) - nu0) / 2
        proj_lo = g0 + dnu + 2 * beta * xw + 2 * (ca0 * dperp).sum(-1) - 2 * ra * dperp.norm(dim=-1)
        proj = single & torch.where(other, proj_lo > delta, torch.ones_like(other)).all(1)
        res[h] = {"truth": float(truth.double().mean()), "tri": float(tri.double().mean()),
                  "pair": float(pair.double().mean()), "proj": float(proj.double().mean()),
                  "med_shift_a": float(sa.median()), "med_dw": float(dwn[other].median()),
                  "med_dperp": float(dperp.norm(dim=-1)[other].median())}
    out["steps"] = res
    g = g0[other]
    out["gap_quantiles"] = [float(q) for q in torch.quantile(g[:100000].float(), torch.tensor(
        [0.05, 0.25, 0.5, 0.75, 0.95], device=dev))]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
