"""``show_versions`` (reference ``utils/_show_versions.py``): system, Python
dependency and - the MI355X part - ROCm / GPU / native-extension
information, for bug reports."""

import importlib
import platform
import sys


def _sys_info():
    return {"python": sys.version.replace("\n", " "), "executable": sys.executable,
            "machine": platform.platform()}


def _deps_info():
    out = {}
    for mod in ("sq_learn_amd", "pip", "setuptools", "numpy", "scipy", "torch", "joblib",
                "threadpoolctl", "pandas", "matplotlib"):
        try:
            m = importlib.import_module(mod)
            out[mod] = getattr(m, "__version__", "unknown")
        except ImportError:
            out[mod] = None
    return out


def _gpu_info():
    info = {}
    try:
        import torch
        info["hip"] = getattr(torch.version, "hip", None)
        n = torch.cuda.device_count()
        info["gpus"] = n
        if n and torch.cuda.is_available():
            p = torch.cuda.get_device_properties(0)
            info["gpu0"] = f"{p.name} ({getattr(p, 'gcnArchName', '?')}, " \
                           f"{p.total_memory / 2**30:.0f} GiB, {p.multi_processor_count} CUs)"
    except Exception as e:  # pragma: no cover
        info["error"] = repr(e)
    try:
        from .._build import ext_path, host_path
        import os
        info["native_hip_extension"] = ext_path() if os.path.exists(ext_path()) else None
        info["native_host_library"] = host_path() if os.path.exists(host_path()) else None
    except Exception:  # pragma: no cover
        pass
    return info


def show_versions():
    """Print system, dependency and GPU / native-library information."""
    for title, d in (("System", _sys_info()), ("Python dependencies", _deps_info()),
                     ("GPU / native", _gpu_info())):
        print(f"\n{title}:")
        for k, v in d.items():
            print(f"{k:>24}: {v}")
