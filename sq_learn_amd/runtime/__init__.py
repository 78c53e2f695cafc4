"""Runtime layer: device/dtype policy, counter-based RNG keys, HIP graph
capture helpers, tracing."""

from .device import (resolve_device, resolve_dtype, to_tensor, to_numpy,
                     gpu_available, local_rank, synchronize, compute_dtype_for)
from .rng import Philox, RngKey, philox4x32, uniform_from_u32

__all__ = ["resolve_device", "resolve_dtype", "to_tensor", "to_numpy",
           "gpu_available", "local_rank", "synchronize", "compute_dtype_for",
           "Philox", "RngKey", "philox4x32", "uniform_from_u32"]
