"""Timings of the fp64-MFMA tall-skinny kernels (csrc/tsgemm64.hip) on the
BASELINE shapes: Gram of 10M x 256 fp32 (CholeskyQR2 pass 1), cross product
X^T Y (power iteration, l = 26), X W (l = 26 and the d x d triangular
R1^-1 of CholeskyQR2 pass 2), 1M x 512 bf16 and 70k x 784.
python benchmarks/tsgemm_bench.py [--reps R]"""
import argparse
import time

import torch

from sq_learn_amd.ops import linalg as L


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    for n, d, dt in [(10_000_000, 256, torch.float32), (1_000_000, 512, torch.bfloat16),
                     (70_000, 784, torch.float32)]:
        X = torch.randn(n, d, device=dev, generator=g).to(dt)
        mu = X[:1000].double().mean(0)
        l = 26
        Z = torch.randn(d, l, device=dev, dtype=torch.float64, generator=g)
        Y = torch.randn(n, l, device=dev, dtype=torch.float64, generator=g)
        W = torch.triu(torch.randn(d, d, device=dev, dtype=torch.float64, generator=g))
        Yd = torch.empty(n, d, device=dev, dtype=torch.float64)
        res = {}
        res["gram"] = (timed(lambda: L.xtx(X, mean_a=mu), a.reps), n * d * d)          # ~n d^2 flops (upper)
        res["xty_l26"] = (timed(lambda: L.xtx(X, Y, mean_a=mu), a.reps), 2 * n * d * l)
        res["xw_l26"] = (timed(lambda: L.xw(X, Z, mean=mu), a.reps), 2 * n * d * l)
        res["xw_tri"] = (timed(lambda: L.xw(X, W, mean=mu, upper=True, out=Yd), a.reps), n * d * d)
        res["cholqr2_sigma"] = (timed(lambda: L.cholqr2_r(X, _Comm(), mu), max(1, a.reps // 2)), 3 * n * d * d)
        for k, (t, fl) in res.items():
            print(f"{n}x{d} {str(dt)[6:]} {k}: {t * 1e3:.2f} ms  {fl / t / 1e12:.1f} TFLOP/s", flush=True)
        del X, Y, Yd


class _Comm:
    world_size = 1

    def all_reduce_(self, t, op="sum"):
        return t


if __name__ == "__main__":
    main()
