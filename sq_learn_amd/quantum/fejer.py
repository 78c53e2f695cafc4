"""Exact O(1)-expected samplers for the Fejer-kernel outcome laws of
amplitude estimation (AE) and phase estimation (PE).

Reference semantics (``Utility.py:442-531`` AE, ``:591-694`` PE): with M
outcome bins and the true value placed at the real position ``omega`` (in
units of bins: ``omega = M*asin(sqrt(a))/pi`` for AE, ``omega = M*w`` for PE)
the reference enumerates all M bins, computes

    p_j = | sin(M*Delta_j*pi) / (M*sin(Delta_j*pi)) |^2 ,  Delta_j = circular
          distance between j/M and omega/M,

(``p_j = 1`` when ``Delta_j == 0``) and draws one bin with ``random.choices``.
That costs O(M) per draw (M = 2^17 for the qPCA precisions: 0.13 s per
singular value).

Because ``M*Delta_j = +-(j - omega) (mod M)``, the numerator is the constant
``sin^2(pi*phi)`` with ``phi = frac(omega)``, so with ``l = j - floor(omega)``

    P(l) = sin^2(pi*phi) / (M^2 sin^2(pi*(l - phi)/M)),   sum_l P(l) = 1,

over one period ``l - phi in (-M/2, M/2]``.  We sample it exactly:

1. inverse-CDF walk over the 2W+1 most likely offsets 0, 1, -1, 2, -2, ...
   (they carry >= 1 - 2/(pi^2 W) of the mass);
2. otherwise rejection sampling on the two tails with the telescoping
   proposal q(z) = 1/(z-1/2) - 1/(z+1/2) (exact discrete inverse CDF),
   acceptance 4(z^2-1/4)/(M^2 sin^2(pi z/M)) in [0.40, 1].

Same algorithm in the HIP kernels (``csrc/fejer.h``); tests check it against
full enumeration with chi-square (tests/test_quantum_reference.py).
"""

import numpy as np

WALK = 16          # offsets walked on each side before the tail sampler
SMALL_M = 2 * WALK + 4   # at or below this M the whole period is enumerated


def fejer_pmf(omega, M):
    """Full probability vector over the M bins (the reference's law), float64.

    Used by tests and for tiny M."""
    j = np.arange(M, dtype=np.float64)
    w0 = j / M
    w1 = omega / M
    diff = w1 - w0
    c = -np.ceil(diff)
    f = -np.floor(diff)
    dist = np.minimum(np.abs(c + diff), np.abs(f + diff))
    with np.errstate(divide="ignore", invalid="ignore"):
        p = np.abs(np.sin(M * dist * np.pi) / (M * np.sin(dist * np.pi))) ** 2
    p = np.where(dist == 0, 1.0, p)
    return p


def _walk_offsets(n_terms):
    """0, 1, -1, 2, -2, ... (n_terms values)."""
    out = np.zeros(n_terms, dtype=np.int64)
    for t in range(1, n_terms):
        out[t] = (t + 1) // 2 if t % 2 == 1 else -(t // 2)
    return out


def fejer_sample(omega, M, rng):
    """Sample one bin index in [0, M) per element of ``omega`` (vectorised).

    ``omega`` and ``M`` broadcast; ``rng`` is a numpy Generator.
    """
    omega = np.asarray(omega, dtype=np.float64)
    M = np.broadcast_to(np.asarray(M, dtype=np.int64), omega.shape).copy()
    omega = np.broadcast_to(omega, M.shape).copy()
    flat_o = omega.reshape(-1)
    flat_M = M.reshape(-1)
    out = np.empty(flat_o.shape, dtype=np.int64)

    small = flat_M <= SMALL_M
    if small.any():
        for i in np.nonzero(small)[0]:
            p = fejer_pmf(flat_o[i], int(flat_M[i]))
            cdf = np.cumsum(p)
            u = rng.random() * cdf[-1]
            out[i] = min(int(np.searchsorted(cdf, u, side="right")), int(flat_M[i]) - 1)
    big = ~small
    if big.any():
        o = flat_o[big]
        Mb = flat_M[big].astype(np.float64)
        fl = np.floor(o)
        phi = o - fl
        s = np.sin(np.pi * phi) ** 2
        offs = _walk_offsets(2 * WALK + 1)                       # [T]
        x = offs[None, :] - phi[:, None]                          # [B, T]
        den = np.sin(np.pi * x / Mb[:, None])
        with np.errstate(divide="ignore", invalid="ignore"):
            p = s[:, None] / (Mb[:, None] ** 2 * den ** 2)
        p = np.where(den == 0, 1.0, p)
        cdf = np.cumsum(p, axis=1)
        u = rng.random(o.shape[0])
        k = (cdf < u[:, None]).sum(axis=1)                        # first idx with cdf >= u
        in_walk = k < offs.shape[0]
        ell = np.where(in_walk, offs[np.minimum(k, offs.shape[0] - 1)], 0)
        if (~in_walk).any():
            idx = np.nonzero(~in_walk)[0]
            ell[idx] = _tail_sample(phi[idx], Mb[idx], rng)
        out[big] = np.mod(fl.astype(np.int64) + ell, flat_M[big])
    return out.reshape(omega.shape)


def _tail_sample(phi, M, rng):
    """Rejection sampler for offsets with |l| > WALK (see module doc)."""
    n = phi.shape[0]
    res = np.zeros(n, dtype=np.int64)
    pending = np.arange(n)
    l_R = np.floor(phi + M / 2.0)
    l_L = l_R - M + 1.0
    # right tail z = l - phi, l in [W+1, l_R]; left tail z = phi - l, l in [l_L, -W-1]
    zR0 = WALK + 1 - phi
    nR = np.maximum(l_R - WALK, 0.0)
    zL0 = WALK + 1 + phi
    nL = np.maximum(-WALK - l_L, 0.0)
    SR = np.where(nR > 0, 1.0 / (zR0 - 0.5) - 1.0 / (zR0 + nR - 0.5), 0.0)
    SL = np.where(nL > 0, 1.0 / (zL0 - 0.5) - 1.0 / (zL0 + nL - 0.5), 0.0)
    for _ in range(10000):
        if pending.size == 0:
            break
        ph = phi[pending]
        Mp = M[pending]
        sr, sl = SR[pending], SL[pending]
        u_side = rng.random(pending.size) * (sr + sl)
        right = u_side < sr
        z0 = np.where(right, zR0[pending], zL0[pending])
        S = np.where(right, sr, sl)
        cnt = np.where(right, nR[pending], nL[pending])
        v = rng.random(pending.size)
        R = 1.0 / (z0 - 0.5) - v * S
        i = np.ceil(1.0 / R - 0.5 - z0)
        i = np.clip(i, 0, np.maximum(cnt - 1, 0))
        z = z0 + i
        acc = 4.0 * (z * z - 0.25) / (Mp ** 2 * np.sin(np.pi * z / Mp) ** 2)
        ok = rng.random(pending.size) < acc
        ell = np.where(right, np.round(z + ph), np.round(ph - z)).astype(np.int64)
        res[pending[ok]] = ell[ok]
        pending = pending[~ok]
    return res


def ae_bins(a, epsilon=None, M=None):
    """Number of AE bins (reference ``Utility.py:483-486``)."""
    if M is None:
        epsilon = np.asarray(epsilon, dtype=np.float64)
        return np.ceil((np.pi / (2 * epsilon)) * (1 + np.sqrt(1 + 4 * epsilon))).astype(np.int64)
    return np.asarray(M, dtype=np.int64)


def pe_qubits(epsilon, gamma):
    """m = ceil(log2(1/eps)) + ceil(log2(2 + 1/(2 gamma))) (Nielsen-Chuang 5.35,
    reference ``Utility.py:635``)."""
    return (np.ceil(np.log2(1.0 / np.asarray(epsilon, dtype=np.float64)))
            + np.ceil(np.log2(2 + 1.0 / (2 * np.asarray(gamma, dtype=np.float64))))).astype(np.int64)


def median_repetitions(gamma):
    """Q of median evaluation (reference ``Utility.py:564-568``): odd ceil of
    ln(1/gamma) / (2 (8/pi^2 - 1/2)^2); gamma=0.1 -> 13."""
    z = np.log(1.0 / gamma) / (2 * (8 / np.pi ** 2 - 0.5) ** 2)
    Q = int(np.ceil(z))
    if Q % 2 == 0:
        Q += 1
    return Q
