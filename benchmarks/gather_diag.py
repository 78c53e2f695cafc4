"""Gather cost of the multi rows on the headline data: torch index_select of
the rows listed by the filter (fp16 512 B and fp32 1 KiB rows) vs the same
bytes read contiguously - is the screen bound by the row gather itself?"""
import os
import sys
import json
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def main():
    from sq_learn_amd.utils.datasets import make_blobs_device
    from sq_learn_amd.models.cluster._lloyd import LloydEngine
    import numpy as np
    n, d, k = 10_000_000, 256, 1024
    dev = torch.device("cuda", 0)
    X, _ = make_blobs_device(n, d, centers=1024, cluster_std=1.0, seed=0, device=dev,
                             dtype=torch.float32)
    rs = np.random.RandomState(0)
    C0 = X[torch.from_numpy(rs.choice(n, k, replace=False)).to(dev)]
    eng = LloydEngine(X, k, delta=0.5, intermediate_error=True, seed=0)
    eng.set_centers(C0)
    for _ in range(12):
        eng.step()
    torch.cuda.synchronize()
    nb = int(eng.buf.counts[5].item())
    idx = (eng.rows_b[:nb] & ((1 << 56) - 1)).clone()
    idx_sorted, _ = torch.sort(idx)
    out = {"rows_b": nb}
    Xh = eng.Xh16
    out["gather_f16_us"] = timeit(lambda: torch.index_select(Xh, 0, idx))
    out["gather_f16_sorted_us"] = timeit(lambda: torch.index_select(Xh, 0, idx_sorted))
    out["gather_f32_us"] = timeit(lambda: torch.index_select(X, 0, idx))
    out["contig_f16_us"] = timeit(lambda: Xh[:nb].clone())
    out["contig_f32_us"] = timeit(lambda: X[:nb].clone())
    rnd = torch.randint(0, n, (nb,), device=dev)
    out["gather_f16_random_us"] = timeit(lambda: torch.index_select(Xh, 0, rnd))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
