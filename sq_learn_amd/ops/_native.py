"""Loader for the in-tree native extension ``sq_learn_amd._C``.

Policy (task contract): on a GPU tensor every op runs its HIP kernel; if the
extension is missing or stale it is (re)built in-tree on first use, and if
that fails the op raises - it never silently falls back to a torch
implementation on the device.  CPU tensors use the torch reference path of
each op (tests, the CPU oracle, gloo multi-process tests).
"""

import importlib
import importlib.util
import os
import threading

import torch

_lock = threading.Lock()
_mod = None
_err = None

DT_F32, DT_F64, DT_BF16 = 0, 1, 2


def _load():
    global _mod, _err
    with _lock:
        if _mod is not None:
            return _mod
        from .. import _build
        try:
            variant = os.environ.get("SQ_NATIVE_VARIANT")
            if variant:
                # kernel-tuning experiments: a separately built extension
                spec = importlib.util.spec_from_file_location("sq_learn_amd._C", variant)
                _mod = importlib.util.module_from_spec(spec)
                spec.loader.exec_module(_mod)
                return _mod
            if os.environ.get("SQ_NO_AUTOBUILD", "0") != "1" and _build.needs_build():
                _build.build()
            _mod = importlib.import_module("sq_learn_amd._C")
        except Exception as e:  # pragma: no cover - exercised on broken installs
            _err = e
            raise
        return _mod


def native():
    """The extension module (builds it if needed); raises if unavailable."""
    if _mod is not None:
        return _mod
    return _load()


def available():
    try:
        native()
        return True
    except Exception:
        return False


def use_native(*tensors):
    """True when the op must take the HIP path (any tensor on a GPU)."""
    return any(isinstance(t, torch.Tensor) and t.is_cuda for t in tensors)


def stream_handle(device=None):
    """Handle of the current torch stream of ``device`` for a native launch,
    with ``device`` made the calling thread's current device first: a
    default stream's handle is 0 (the null stream), which HIP resolves
    against the CURRENT device, so launching for ``cuda:1`` from a thread
    whose current device is 0 would run on the wrong GPU.  (The HIP current
    device is per thread: the task layer's per-GPU worker threads and
    ``torch.cuda.device`` contexts are unaffected elsewhere.)"""
    fast = _fast_stream_fns()
    if fast is not None:
        # one C call for the device, one for the raw stream handle (no
        # torch.cuda.Stream object): this runs before every native launch,
        # ~20 per Lloyd step, and the N = 8 per-rank step is ~0.2 ms
        getdev, raw = fast
        cur = getdev()
        if device is None:
            return raw(cur)
        dev = device if isinstance(device, torch.device) else torch.device(device)
        if dev.type != "cuda":
            return raw(cur)
        idx = dev.index if dev.index is not None else cur
        if idx != cur:
            torch.cuda.set_device(idx)
        return raw(idx)
    if device is not None:
        dev = torch.device(device)
        if dev.type == "cuda":
            idx = dev.index if dev.index is not None else torch.cuda.current_device()
            if idx != torch.cuda.current_device():
                torch.cuda.set_device(idx)
            return torch.cuda.current_stream(idx).cuda_stream
    return torch.cuda.current_stream(device).cuda_stream


_FAST_STREAM = None


def _fast_stream_fns():
    """(current device, raw current stream of a device) as direct torch C
    calls, once CUDA is initialised; None before (or without them)."""
    global _FAST_STREAM
    if _FAST_STREAM is None:
        getdev = getattr(torch._C, "_cuda_getDevice", None)
        raw = getattr(torch._C, "_cuda_getCurrentRawStream", None)
        if getdev is None or raw is None or not torch.cuda.is_initialized():
            return None
        _FAST_STREAM = (getdev, raw)
    return _FAST_STREAM


def ptr(t):
    return 0 if t is None else t.data_ptr()


def dtype_code(t):
    if t.dtype == torch.float32:
        return DT_F32
    if t.dtype == torch.float64:
        return DT_F64
    if t.dtype == torch.bfloat16:
        return DT_BF16
    raise TypeError(f"unsupported dtype {t.dtype} for native op")


def loaded_path():
    m = native()
    return getattr(m, "__file__", None)
