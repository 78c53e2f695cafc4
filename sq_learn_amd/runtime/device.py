"""Device / dtype resolution and host<->device conversion.

The MI355X counterpart of the reference's ``utils/_openmp_helpers.pyx:18-61``
(effective thread count): here the parallel resource is the HIP device of the
current rank (one process per GPU, ``LOCAL_RANK`` selects it) and the data
layout policy (bf16 storage for the big row matrices, fp32 for the small
replicated state, fp64 on the CPU oracle path).
"""

import os

import numpy as np
import torch

from .._config import get_config

_DTYPES = {
    "float64": torch.float64, "fp64": torch.float64, "double": torch.float64,
    "float32": torch.float32, "fp32": torch.float32, "float": torch.float32,
    "bfloat16": torch.bfloat16, "bf16": torch.bfloat16,
    "float16": torch.float16, "fp16": torch.float16,
}


def gpu_available():
    return torch.cuda.is_available()


def local_rank():
    return int(os.environ.get("LOCAL_RANK", "0"))


def resolve_device(device=None):
    """Return the torch.device estimators should compute on.

    ``device=None`` uses the global config ('auto' -> the rank's GPU when
    one is visible, otherwise the CPU).
    """
    if isinstance(device, torch.device):
        return device
    if device is None:
        device = get_config()["device"]
    if device == "auto":
        if gpu_available():
            n = torch.cuda.device_count()
            return torch.device("cuda", local_rank() % max(n, 1))
        return torch.device("cpu")
    if device in ("cuda", "gpu", "hip"):
        return torch.device("cuda", local_rank() % max(torch.cuda.device_count(), 1))
    return torch.device(device)


def resolve_dtype(dtype):
    if dtype is None:
        return None
    if isinstance(dtype, torch.dtype):
        return dtype
    if isinstance(dtype, str):
        return _DTYPES[dtype]
    return {np.float64: torch.float64, np.float32: torch.float32,
            np.float16: torch.float16}[np.dtype(dtype).type]


def is_tensor(x):
    return isinstance(x, torch.Tensor)


def to_tensor(x, device=None, dtype=None, copy=False):
    """Convert numpy / list / tensor to a torch tensor on ``device``."""
    device = resolve_device(device)
    dtype = resolve_dtype(dtype)
    if isinstance(x, torch.Tensor):
        t = x
        if dtype is not None and t.dtype != dtype:
            t = t.to(dtype)
            copy = False
        if t.device != device:
            t = t.to(device)
            copy = False
        return t.clone() if copy else t
    arr = np.asarray(x)
    if any(st < 0 for st in arr.strides):
        arr = np.ascontiguousarray(arr)   # torch rejects negative strides
    if dtype is None:
        if arr.dtype.kind in "fc":
            dtype = resolve_dtype(arr.dtype) if arr.dtype in (np.float32, np.float64, np.float16) else torch.float64
        elif arr.dtype.kind == "b":
            dtype = torch.bool
        elif arr.dtype.kind in "iu":
            dtype = torch.int64
        else:
            dtype = torch.float64
    t = torch.as_tensor(arr, dtype=dtype)
    if t.device != device:
        t = t.to(device, non_blocking=False)
    elif copy:
        t = t.clone()
    return t


def to_numpy(x):
    """Convert a tensor (any device, any float dtype) to a numpy array."""
    if isinstance(x, torch.Tensor):
        t = x.detach()
        if t.dtype in (torch.bfloat16, torch.float16):
            t = t.float()
        return t.cpu().numpy()
    return np.asarray(x)


def compute_dtype_for(data_dtype, device):
    """Accumulation dtype for reductions over rows: fp64 on the CPU oracle
    path for float64 inputs, fp32 otherwise (MI355X fp64 is 1/2 rate VALU and
    has no bf16-class MFMA, so GPU accumulation stays fp32)."""
    if device.type == "cpu" and data_dtype == torch.float64:
        return torch.float64
    return torch.float32


def synchronize(device=None):
    device = resolve_device(device)
    if device.type == "cuda":
        torch.cuda.synchronize(device)
