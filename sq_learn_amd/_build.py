"""In-tree build of the native HIP layer (``sq_learn_amd/_C*.so``).

Plays the role of the reference's Cython/numpy.distutils build
(``sklearn/_build_utils/__init__.py:38-76``, ``openmp_helpers.py``): every
``csrc/*.hip`` translation unit is compiled by ``hipcc --offload-arch=gfx950``
(CDNA4 only - no multi-arch fatbins, no CUDA/hipify layer) and linked with
the CPython-API marshalling module ``csrc/module.cpp`` into one extension
that lives next to this file (so it travels with the repo snapshot to GPU
boxes and is what the python processes load).

Usage: ``python -m sq_learn_amd._build [--force] [--jobs N] [--debug]``.

The host-native library (``csrc/host/*.cpp``: hashing, isotonic PAVA, graph
searches, svmlight parsing, DBSCAN expansion, ...) is built alongside with
the host C++ compiler into ``_sq_host.so`` (``build_host``).

Tuning variants (kernel experiments only): ``--define NAME=VALUE ... --out
PATH.so`` builds a separately named extension with extra preprocessor
definitions; ``SQ_NATIVE_VARIANT=PATH.so`` makes the loader use it.
"""

import argparse
import contextlib
import fcntl
import os
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.environ.get("SQ_CSRC_DIR", os.path.join(HERE, "csrc"))   # override: A/B kernel variants
BUILD = os.path.join(HERE, "..", "build", "sq_native")
ARCH = os.environ.get("SQ_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def ext_path():
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return os.path.join(HERE, "_C" + suffix)


def _sources():
    hips = sorted(f for f in os.listdir(CSRC) if f.endswith(".hip"))
    headers = sorted(f for f in os.listdir(CSRC) if f.endswith(".h"))
    return hips, headers


def _newest(paths):
    return max((os.path.getmtime(p) for p in paths), default=0.0)


def needs_build():
    out = ext_path()
    if not os.path.exists(out):
        return True
    hips, headers = _sources()
    srcs = [os.path.join(CSRC, f) for f in hips + headers + ["module.cpp"]] + [__file__]
    return _newest(srcs) > os.path.getmtime(out)


@contextlib.contextmanager
def _build_lock(name):
    """Cross-process build lock (``build/<name>.lock``): pytest-xdist workers,
    gloo test ranks and torchrun ranks all call ``build()`` on first use; only
    one compiles, the others wait and then see a fresh library."""
    os.makedirs(os.path.join(HERE, "..", "build"), exist_ok=True)
    fd = os.open(os.path.join(HERE, "..", "build", name + ".lock"), os.O_CREAT | os.O_RDWR, 0o644)
    try:
        fcntl.flock(fd, fcntl.LOCK_EX)
        yield
    finally:
        fcntl.flock(fd, fcntl.LOCK_UN)
        os.close(fd)


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("native build failed:\n" + " ".join(cmd) + "\n" + r.stdout)
    return r.stdout


def build(force=False, jobs=None, debug=False, verbose=False, defines=(), out=None):
    """Compile and link the extension; returns its path."""
    variant = out is not None
    out = out or ext_path()
    if not variant and not force and not needs_build():
        return out
    with _build_lock("sq_native"):
        # another process may have finished the same build while we waited
        if not variant and not force and not needs_build():
            return out
        return _build_locked(out, variant, jobs, debug, verbose, defines)


def _build_locked(out, variant, jobs, debug, verbose, defines):
    bdir = BUILD if not variant else os.path.join(
        BUILD, "variant_" + os.path.splitext(os.path.basename(out))[0])
    os.makedirs(bdir, exist_ok=True)
    hips, _ = _sources()
    opt = ["-O0", "-g"] if debug else ["-O3"]
    common = [HIPCC, "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-I", CSRC,
              "-Wno-unused-result", "-Wno-unused-command-line-argument"] + opt
    common += ["-D" + d for d in defines]
    py_inc = sysconfig.get_paths()["include"]
    jobs = jobs or int(os.environ.get("MAX_JOBS", min(8, os.cpu_count() or 4)))

    def compile_one(src):
        obj = os.path.join(bdir, src + ".o")
        cmd = common + ["-c", os.path.join(CSRC, src), "-o", obj]
        if src == "module.cpp":
            cmd = [HIPCC, "-std=c++17", "-fPIC", "-O2", "-I", py_inc, "-c",
                   os.path.join(CSRC, src), "-o", obj]
        log = _run(cmd)
        if verbose and log.strip():
            print(log)
        return obj

    units = hips + ["module.cpp"]
    with ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(compile_one, units))
    tmp = f"{out}.{os.getpid()}.tmp"
    _run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", tmp] + objs)
    os.replace(tmp, out)
    return out


HOST_SRC = os.path.join(CSRC, "host")
CXX = os.environ.get("CXX", "g++")


def host_path():
    return os.path.join(HERE, "_sq_host.so")


def _host_sources():
    return sorted(os.path.join(HOST_SRC, f) for f in os.listdir(HOST_SRC)
                  if f.endswith((".cpp", ".h")))


def host_needs_build():
    out = host_path()
    return not os.path.exists(out) or _newest(_host_sources() + [__file__]) > os.path.getmtime(out)


def build_host(force=False, debug=False, sanitize=None, out=None):
    """Host-native library (``csrc/host/*.cpp`` -> ``_sq_host.so``, loaded
    with ctypes): C++17 + OpenMP, no HIP dependency.

    ``sanitize="address,undefined"`` builds an instrumented copy (default
    ``build/_sq_host_asan.so``, never the in-tree library) for CPU race /
    memory checks: load it with ``SQ_HOST_LIB=<path>`` and
    ``LD_PRELOAD=$(g++ -print-file-name=libasan.so)``
    (``scripts/host_asan.sh`` runs the host-native tests that way)."""
    if sanitize and out is None:
        out = os.path.join(HERE, "..", "build", "_sq_host_asan.so")
    out = out or host_path()
    if not force and not sanitize and not host_needs_build():
        return out
    with _build_lock("sq_host"):
        if not force and not sanitize and not host_needs_build():
            return out
        srcs = [f for f in _host_sources() if f.endswith(".cpp")]
        opt = ["-O0", "-g"] if debug else ["-O3"]
        if sanitize:
            opt = ["-O1", "-g", "-fno-omit-frame-pointer", f"-fsanitize={sanitize}"]
        tmp = f"{out}.{os.getpid()}.tmp"
        _run([CXX, "-std=c++17", "-fPIC", "-shared", "-fopenmp", "-I", HOST_SRC] + opt + srcs
             + ["-o", tmp])
        os.replace(tmp, out)
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("--jobs", type=int, default=None)
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--define", action="append", default=[])
    ap.add_argument("--out", default=None)
    ap.add_argument("--host-sanitize", default=None,
                    help="build only an instrumented host library, e.g. address,undefined")
    a = ap.parse_args(argv)
    if a.host_sanitize:
        print(build_host(force=True, sanitize=a.host_sanitize, out=a.out))
        return 0
    path = build(force=a.force, jobs=a.jobs, debug=a.debug, verbose=a.verbose,
                 defines=a.define, out=a.out)
    if a.out is None:
        print(build_host(force=a.force, debug=a.debug))
    print(path)


if __name__ == "__main__":
    sys.exit(main())
