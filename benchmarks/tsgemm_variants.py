"""Variant sweep of csrc/tsgemm64.hip (build-time knobs SQ_TS_WPE /
SQ_TS_PK32 / SQ_TS_PREFETCH): each variant is compiled (on the host, before
the GPU run: --build) into benchmarks/_tsv/<name>.so and timed through ctypes on
the BASELINE shapes.
python benchmarks/tsgemm_variants.py --build   (CPU: hipcc)
python benchmarks/tsgemm_variants.py            (GPU: time every built variant)"""
import argparse
import ctypes
import glob
import os
import subprocess
import sys
import time

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
SRC = os.path.join(ROOT, "sq_learn_amd", "csrc", "tsgemm64.hip")
OUT = os.path.join(ROOT, "benchmarks", "_tsv")   # not under ./build (gpurun-ignored)
VARIANTS = {
    "base": {},
    "wpe2": {"SQ_TS_WPE": 2},
    "pk16": {"SQ_TS_PK32": 0},
    "nopf": {"SQ_TS_PREFETCH": 0},
    "wpe2_pk16": {"SQ_TS_WPE": 2, "SQ_TS_PK32": 0},
}


def build():
    os.makedirs(OUT, exist_ok=True)
    for name, defs in VARIANTS.items():
        d = [f"-D{k}={v}" for k, v in defs.items()]
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
               "-shared", *d, SRC, "-o", os.path.join(OUT, name + ".so")]
        subprocess.check_call(cmd)
        print("built", name, flush=True)


def run():
    import torch
    sys.path.insert(0, ROOT)
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev).cuda_stream
    g = torch.Generator(device=dev).manual_seed(0)
    shapes = [(10_000_000, 256, torch.float32, 0), (1_000_000, 512, torch.bfloat16, 2)]
    for so in sorted(glob.glob(os.path.join(OUT, "*.so"))):
        lib = ctypes.CDLL(so)
        name = os.path.basename(so)[:-3]
        for n, d, dt, code in shapes:
            X = torch.randn(n, d, device=dev, generator=g).to(dt)
            Y = torch.empty(n, d, device=dev, dtype=torch.float64)
            W = torch.triu(torch.randn(d, d, device=dev, dtype=torch.float64, generator=g))
            mu = X[:1000].double().mean(0)
            C = torch.zeros(d, d, dtype=torch.float64, device=dev)
            splits = 8 * max(1, -(-1024 // 3) // 8) if d == 256 else 8 * max(1, -(-1024 // 10) // 8)
            part = torch.empty(splits * 64 * 128 * 128, dtype=torch.float64, device=dev)
            P = ctypes.c_void_p
            L = ctypes.c_longlong

            def gram():
                rc = lib.sq_xtx(P(X.data_ptr()), code, L(X.stride(0)), P(mu.data_ptr()), d,
                                P(X.data_ptr()), code, L(X.stride(0)), P(mu.data_ptr()), d, L(n), 1,
                                splits, P(part.data_ptr()), P(C.data_ptr()), 0, P(st))
                assert rc == 0, rc

            def xw():
                rc = lib.sq_xw(P(X.data_ptr()), code, L(X.stride(0)), P(mu.data_ptr()), L(n), d,
                               P(W.data_ptr()), L(W.stride(0)), d, 1, P(Y.data_ptr()), 1,
                               L(Y.stride(0)), P(st))
                assert rc == 0, rc

            for fname, fn in (("gram", gram), ("xw_tri", xw)):
                fn()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(5):
                    fn()
                torch.cuda.synchronize()
                ms = (time.perf_counter() - t0) / 5 * 1e3
                print(f"{name:10s} {n}x{d} {fname}: {ms:.2f} ms  {n * d * d / ms / 1e9:.1f} TFLOP/s",
                      flush=True)
            del X, Y


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    a = ap.parse_args()
    build() if a.build else run()
