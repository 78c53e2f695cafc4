"""MurmurHash3 (x86, 32-bit) - reference ``utils/murmurhash.pyx``
(``murmurhash3_32``), computed by the host-native library
(``csrc/host/hashing.cpp``)."""

import numpy as np

from ..ops import _host


def _pack_strings(items):
    bs = [s.encode("utf-8") if isinstance(s, str) else bytes(s) for s in items]
    offsets = np.zeros(len(bs) + 1, dtype=np.int64)
    np.cumsum([len(b) for b in bs], out=offsets[1:])
    buf = np.frombuffer(b"".join(bs) or b"\0", dtype=np.uint8).copy()
    return buf, offsets


def murmurhash3_32(key, seed=0, positive=False):
    """32-bit hash of an int32 / str / bytes key or an array of them.

    Returns int32 (``positive=False``) or uint32 bit patterns as Python ints
    for scalar keys, numpy arrays for array keys (reference semantics)."""
    L = _host.lib()
    seed = int(seed) & 0xFFFFFFFF
    scalar = isinstance(key, (int, np.integer, str, bytes))
    if isinstance(key, (int, np.integer)):
        arr = np.asarray([key], dtype=np.int32)
    elif isinstance(key, (str, bytes)):
        arr = np.asarray([key], dtype=object)
    else:
        arr = np.asarray(key)
        if arr.dtype not in (np.int32, object) and arr.dtype.kind not in "US":
            raise TypeError(f"key.dtype should be int32, got {arr.dtype}")
    out = np.empty(arr.shape, dtype=np.uint32)
    flat = out.reshape(-1)
    if arr.dtype == np.int32:
        a = np.ascontiguousarray(arr.reshape(-1))
        L.sqh_murmur_i32(_host.ptr(a), a.size, seed, _host.ptr(flat))
    else:
        buf, off = _pack_strings(arr.reshape(-1).tolist())
        L.sqh_murmur_bytes(_host.ptr(buf), _host.ptr(off), len(off) - 1, seed, _host.ptr(flat))
    res = out if positive else out.view(np.int32)
    if scalar:
        return int(res.reshape(-1)[0])
    return res
