"""Counter-based random numbers (Philox4x32-10) shared by the CPU and HIP paths.

The reference draws its noise from three unrelated generators: NumPy's global
state via ``scipy.stats.truncnorm`` (``Utility.py:68-104``), Python's
``random`` module (``Utility.py:508, 653``; ``_dmeans.py:2252-2257``) and a
fresh unseeded ``np.random.RandomState()`` per measurement
(``Utility.py:53``).  That makes results irreproducible and impossible to
shard.  Here every random draw is a pure function

    value = f(Philox4x32_10(counter, key))

where ``key`` is the 64-bit seed and ``counter`` packs (stream id, global
element index).  The HIP kernels (``csrc/philox.h``) implement the identical
function, so CPU tests, single-GPU runs and row-sharded multi-GPU runs draw
the *same* numbers for the same global element (SURVEY.md §2.6 C8, §7.4
"shard-invariant reproducibility").

This module is the torch (CPU or device) implementation; int64 arithmetic
holds the uint32 lanes.
"""

import hashlib

import torch

M0 = 0xD2511F53
M1 = 0xCD9E8D57
W0 = 0x9E3779B9
W1 = 0xBB67AE85
MASK32 = 0xFFFFFFFF

# Stream purposes (upper 16 bits of the 64-bit stream id).  Each stochastic
# operation of the framework gets its own purpose so draws never collide.
PURPOSE = {
    "generic": 0x0000,
    "trunc_normal": 0x0001,
    "band_select": 0x0002,   # random key for uniform delta-band / tie selection
    "ae": 0x0003,            # amplitude estimation samples
    "pe": 0x0004,            # phase estimation samples
    "tomography": 0x0005,    # multinomial shots
    "failure": 0x0006,       # failure-probability Bernoulli draws
    "init": 0x0007,          # centroid initialisation
    "data": 0x0008,          # synthetic data generators
    "gaussian": 0x0009,      # plain normal draws (randomized SVD test matrix)
    "ipe": 0x000A,           # inner product estimation
    "ipe_skip": 0x000B,      # IPE hazard budgets / thinning of the pruned screen
    "kmpp": 0x000C,          # reserved: k-means++ device streams
    "ipe16_skip": 0x000D,    # certified fp16 IPE screen: stream budgets / thinning
    "ipe16_row": 0x000E,     # certified fp16 IPE screen: per-row budget minimum
}


def _mulhilo(a, b):
    """(hi, lo) 32-bit halves of the 64-bit product a*b, a,b < 2**32 (int64)."""
    b_lo = b & 0xFFFF
    b_hi = b >> 16
    t1 = a * b_lo
    t2 = a * b_hi
    mid = t1 + ((t2 & 0xFFFF) << 16)
    lo = mid & MASK32
    hi = (t2 >> 16) + (mid >> 32)
    return hi & MASK32, lo


def philox4x32(c0, c1, c2, c3, k0, k1, rounds=10):
    """Philox4x32 with ``rounds`` rounds on int64 tensors holding uint32 values.

    Any argument may be a python int or a tensor; tensors broadcast.
    Returns four int64 tensors of uint32 values.
    """
    def as_t(v, like):
        if isinstance(v, torch.Tensor):
            return v.to(torch.int64)
        return torch.full_like(like, int(v) & MASK32)

    like = None
    for v in (c0, c1, c2, c3):
        if isinstance(v, torch.Tensor):
            like = v.to(torch.int64)
            break
    if like is None:
        like = torch.zeros((), dtype=torch.int64)
    shape = torch.broadcast_shapes(*[v.shape for v in (c0, c1, c2, c3) if isinstance(v, torch.Tensor)] or [()])
    like = torch.zeros(shape, dtype=torch.int64, device=like.device)
    x0, x1, x2, x3 = (as_t(v, like).expand(shape) for v in (c0, c1, c2, c3))
    k0 = int(k0) & MASK32
    k1 = int(k1) & MASK32
    for r in range(rounds):
        if r:
            k0 = (k0 + W0) & MASK32
            k1 = (k1 + W1) & MASK32
        hi0, lo0 = _mulhilo(torch.full_like(x0, M0), x0)
        hi1, lo1 = _mulhilo(torch.full_like(x2, M1), x2)
        x0, x1, x2, x3 = (hi1 ^ x1 ^ k0), lo1, (hi0 ^ x3 ^ k1), lo0
    return x0, x1, x2, x3


def uniform_from_u32(x, dtype=torch.float32):
    """Map uint32 (int64 tensor) to a uniform in the open interval (0, 1)."""
    return (((x >> 8).to(torch.float64) + 0.5) * (1.0 / 16777216.0)).to(dtype)


def seed_to_key(seed):
    """Map an arbitrary python seed (int / None / str) to a 64-bit Philox key."""
    if seed is None:
        from .._config import get_config
        seed = get_config()["seed"]
    if isinstance(seed, (int,)) and 0 <= seed < (1 << 64):
        s = seed
    else:
        s = int.from_bytes(hashlib.sha256(repr(seed).encode()).digest()[:8], "little")
    return s & MASK32, (s >> 32) & MASK32


class RngKey:
    """A (seed, stream) pair: the identity of one reproducible random stream.

    ``stream`` is a 64-bit integer; its upper 16 bits hold the purpose code
    (see :data:`PURPOSE`), the lower 48 bits an operation-specific id such as
    ``(restart << 24) | iteration``.
    """

    __slots__ = ("k0", "k1", "stream")

    def __init__(self, seed=None, purpose="generic", sub=0):
        self.k0, self.k1 = seed_to_key(seed)
        self.stream = ((PURPOSE[purpose] & 0xFFFF) << 48) | (int(sub) & ((1 << 48) - 1))

    def derive(self, purpose=None, sub=None):
        other = RngKey.__new__(RngKey)
        other.k0, other.k1 = self.k0, self.k1
        p = (self.stream >> 48) if purpose is None else PURPOSE[purpose]
        s = (self.stream & ((1 << 48) - 1)) if sub is None else int(sub)
        other.stream = ((p & 0xFFFF) << 48) | (s & ((1 << 48) - 1))
        return other

    @property
    def s0(self):
        return self.stream & MASK32

    @property
    def s1(self):
        return (self.stream >> 32) & MASK32

    def as_tuple(self):
        """(k0, k1, s0, s1) - the scalar arguments the HIP kernels take."""
        return self.k0, self.k1, self.s0, self.s1

    def __repr__(self):
        return f"RngKey(key=0x{self.k1:08x}{self.k0:08x}, stream=0x{self.stream:016x})"


class Philox:
    """Vectorised Philox draws keyed by global element indices (torch)."""

    def __init__(self, key: RngKey):
        self.key = key

    def u32x4(self, index):
        """Four uint32 words per element of the int64 ``index`` tensor."""
        index = index.to(torch.int64)
        lo = index & MASK32
        hi = (index >> 32) & MASK32
        return philox4x32(lo, hi, self.key.s0, self.key.s1, self.key.k0, self.key.k1)

    def uniform(self, index, n=1, dtype=torch.float32):
        """``n`` (<=4) uniforms in (0,1) per index; returns list of tensors."""
        words = self.u32x4(index)
        return [uniform_from_u32(w, dtype) for w in words[:n]]

    def uniform_flat(self, numel, offset=0, device="cpu", dtype=torch.float32):
        """``numel`` uniforms for flat element ids offset..offset+numel-1.

        Element e uses word (e % 4) of the Philox block e // 4, so the
        values are independent of how the range is split (sharding).
        """
        start = offset // 4
        stop = (offset + numel + 3) // 4
        idx = torch.arange(start, stop, dtype=torch.int64, device=device)
        w = self.u32x4(idx)
        allw = torch.stack(w, dim=1).reshape(-1)
        first = offset - start * 4
        return uniform_from_u32(allw[first:first + numel], dtype)

    def normal_flat(self, numel, offset=0, device="cpu", dtype=torch.float32):
        """Standard normals for flat element ids (Box-Muller on word pairs).

        Element e uses block e // 2 (words 0,1 -> radius/angle); word 2/3
        unused so that the mapping is a function of e alone.
        """
        idx = torch.arange(offset, offset + numel, dtype=torch.int64, device=device)
        blk = idx >> 1
        w0, w1, _, _ = self.u32x4(blk)
        u1 = uniform_from_u32(w0, torch.float64)
        u2 = uniform_from_u32(w1, torch.float64)
        r = torch.sqrt(-2.0 * torch.log(u1))
        ang = 2.0 * torch.pi * u2
        z = torch.where((idx & 1) == 0, r * torch.cos(ang), r * torch.sin(ang))
        return z.to(dtype)
