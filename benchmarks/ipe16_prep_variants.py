"""Where ipe16_prep_kernel's time goes: timing-only variant libraries built
with SQ_IPE16_DIAG bits (csrc/ipe16.hip: 1 no hint sampler, 2 no fire
listing, 4 no fired-pair evaluation, 8 one band for all groups, 16 no
near-pair flush in the sweep, 32 no far-minimum upkeep - results not the
law's), each the production objects relinked with one recompiled
ipe16.hip.

    python benchmarks/ipe16_prep_variants.py --build    (CPU)
    scripts/gpu_prepvar.sh                              (GPU: rocprof per variant)"""
import os
import shutil
import subprocess
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
OUT = os.path.join(ROOT, "benchmarks", "_ipev")
VARIANTS = {"d0": 0, "d16": 16, "d32": 32, "d48": 48}


def build():
    sys.path.insert(0, ROOT)
    from sq_learn_amd import _build as B
    B.build()
    os.makedirs(OUT, exist_ok=True)
    objs = sorted(os.path.join(B.BUILD, f) for f in os.listdir(B.BUILD) if f.endswith(".o"))
    for name, bits in VARIANTS.items():
        obj = os.path.join(OUT, f"ipe16_{name}.o")
        subprocess.check_call([B.HIPCC, "-std=c++17", "-fPIC", f"--offload-arch={B.ARCH}", "-I", B.CSRC,
                               "-O3", f"-DSQ_IPE16_DIAG={bits}", "-c",
                               os.path.join(B.CSRC, "ipe16.hip"), "-o", obj])
        link = [o for o in objs if not os.path.basename(o).startswith("ipe16.hip")] + [obj]
        subprocess.check_call([B.HIPCC, "-shared", "-fPIC", f"--offload-arch={B.ARCH}", "-o",
                               os.path.join(OUT, name + ".so")] + link)
        os.remove(obj)
        print("built", name, flush=True)


if __name__ == "__main__":
    if "--build" in sys.argv:
        build()
