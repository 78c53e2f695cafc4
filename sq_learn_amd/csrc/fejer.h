// Exact O(1)-expected Fejer-kernel sampler for amplitude / phase estimation.
// Same algorithm as sq_learn_amd/quantum/fejer.py (see its docstring):
//   P(l) = sin^2(pi phi) / (M^2 sin^2(pi (l - phi) / M)),  phi = frac(omega)
//   1) inverse-CDF walk over l = 0, 1, -1, 2, -2, ... (|l| <= WALK),
//      sines by angle-addition recurrence (no transcendental per step);
//   2) tails by rejection with the telescoping proposal 1/(z-1/2)-1/(z+1/2).
// Random words come from Philox blocks (sample id s, block b): counter
// (s_lo, s_hi | b << 16, stream_lo, stream_hi) so every sample owns 2^16
// independent blocks.
#pragma once
#include "common.h"

namespace sq {

constexpr int kFejerWalk = 16;
constexpr int kFejerSmallM = 2 * kFejerWalk + 4;

struct WordStream {
  RngKey key;
  uint64_t s;
  uint32_t b = 0;
  u4 cur;
  int used = 4;
  SQ_DEV WordStream(const RngKey& k, uint64_t sid) : key(k), s(sid) {}
  SQ_DEV uint32_t next() {
    if (used == 4) {
      cur = philox4x32_10((uint32_t)s, ((uint32_t)(s >> 32) & 0xFFFFu) | (b << 16),
                          key.s0, key.s1, key.k0, key.k1);
      ++b;
      used = 0;
    }
    uint32_t w = used == 0 ? cur.x : (used == 1 ? cur.y : (used == 2 ? cur.z : cur.w));
    ++used;
    return w;
  }
  SQ_DEV double u() { return u01d(next()); }
};

// The per-law setup (phi, sin^2(pi phi), the walk's rotation constants) is
// computed once; sample() then costs the walk (plus rare tail rejections).
// fejer_sample() below = FejerLaw(omega, M).sample(ws): identical words and
// results to the CPU twin (ops/random.py fejer_sample_torch).
struct FejerLaw {
  double omega, phi, Md;
  long long M, base;
  float s, sa, ca, sb, cb, inv_m2;
  SQ_DEV FejerLaw(double omega_, long long M_) : omega(omega_), M(M_) {
    const double PI = 3.14159265358979323846;
    const double fl = floor(omega);
    phi = omega - fl;
    Md = (double)M;
    base = (long long)fl;
    s = 0.f; sa = ca = sb = cb = inv_m2 = 0.f;
    if (phi == 0.0) return;
    s = (float)sin(PI * phi);
    s = s * s;
    if (M <= kFejerSmallM) return;
    const float alpha = (float)(PI / Md);
    const float beta = (float)(PI * phi / Md);
    __sincosf(beta, &sb, &cb);
    __sincosf(alpha, &sa, &ca);
    inv_m2 = (float)(1.0 / (Md * Md));
  }
  // pmf of the walk offset l (bin base + l) given sin(l alpha - beta)
  SQ_DEV float walk_term(float sn) const { return s * inv_m2 / (sn * sn); }
  // offset of a draw conditioned on |l| > kFejerWalk (rejection, telescoping proposal)
  SQ_DEV long long tail_ell(WordStream& ws) const {
    const double PI = 3.14159265358979323846;
    long long ell = 0;
    double lR = floor(phi + Md / 2.0);
    double lL = lR - Md + 1.0;
    double zR0 = kFejerWalk + 1 - phi, nR = fmax(lR - kFejerWalk, 0.0);
    double zL0 = kFejerWalk + 1 + phi, nL = fmax(-kFejerWalk - lL, 0.0);
    double SR = nR > 0 ? 1.0 / (zR0 - 0.5) - 1.0 / (zR0 + nR - 0.5) : 0.0;
    double SL = nL > 0 ? 1.0 / (zL0 - 0.5) - 1.0 / (zL0 + nL - 0.5) : 0.0;
    for (int it = 0; it < 4096; ++it) {
      bool right = ws.u() * (SR + SL) < SR;
      double z0 = right ? zR0 : zL0, S = right ? SR : SL, cnt = right ? nR : nL;
      double R = 1.0 / (z0 - 0.5) - ws.u() * S;
      double i = ceil(1.0 / R - 0.5 - z0);
      i = fmin(fmax(i, 0.0), fmax(cnt - 1.0, 0.0));
      double z = z0 + i;
      double sn = sin(PI * z / Md);
      double accp = 4.0 * (z * z - 0.25) / (Md * Md * sn * sn);
      if (ws.u() < accp) {
        ell = right ? (long long)llround(z + phi) : (long long)llround(phi - z);
        break;
      }
    }
    return ell;
  }
  SQ_DEV long long bin_of(long long ell) const {
    long long j = (base + ell) % M;
    if (j < 0) j += M;
    return j;
  }
  // returns the sampled bin in [0, M)
  SQ_DEV long long sample(WordStream& ws) const {
    const double PI = 3.14159265358979323846;
    if (phi == 0.0) {  // the true value sits on a bin: p = 1 there
      long long j = base % M; if (j < 0) j += M; return j;
    }
    if (M <= kFejerSmallM) {
      // enumerate the whole period: bins j = 0..M-1, inverse CDF
      double u = ws.u();
      double acc = 0.0;
      long long pick = M - 1;
      double tot = 0.0;
      for (long long j = 0; j < M; ++j) {
        double d = (double)j - omega;
        double sn = sin(PI * d / Md);
        tot += (sn == 0.0) ? 1.0 : (double)s / (Md * Md * sn * sn);
      }
      u *= tot;
      for (long long j = 0; j < M; ++j) {
        double d = (double)j - omega;
        double sn = sin(PI * d / Md);
        acc += (sn == 0.0) ? 1.0 : (double)s / (Md * Md * sn * sn);
        if (acc >= u) { pick = j; break; }
      }
      return pick;
    }
    // ---- walk
    float u = (float)ws.u();
    // l = 0 : sin(-beta)
    float den = sb * sb;
    float acc = s * inv_m2 / den;
    long long ell = 0;
    bool found = acc >= u;
    float st = 0.f, ct = 1.f;  // sin/cos(t*alpha)
    for (int t = 1; t <= kFejerWalk && !found; ++t) {
      float nst = st * ca + ct * sa;
      float nct = ct * ca - st * sa;
      st = nst; ct = nct;
      float sp = st * cb - ct * sb;  // sin(t*alpha - beta)   (l = +t)
      acc += s * inv_m2 / (sp * sp);
      if (acc >= u) { ell = t; found = true; break; }
      float sm = st * cb + ct * sb;  // -sin(-t*alpha - beta) (l = -t)
      acc += s * inv_m2 / (sm * sm);
      if (acc >= u) { ell = -t; found = true; break; }
    }
    if (!found) ell = tail_ell(ws);
    long long j = (base + ell) % M;
    if (j < 0) j += M;
    return j;
  }
};

SQ_DEV long long fejer_sample(double omega, long long M, WordStream& ws) {
  return FejerLaw(omega, M).sample(ws);
}

// amplitude estimation of a in [0,1] with M bins: returns sin^2(pi j / M)
SQ_DEV double ae_sample(double a, long long M, WordStream& ws) {
  const double PI = 3.14159265358979323846;
  double omega = (double)M * asin(sqrt(fmin(fmax(a, 0.0), 1.0))) / PI;
  long long j = fejer_sample(omega, M, ws);
  double sv = sin(PI * (double)j / (double)M);
  return sv * sv;
}

SQ_DEV long long ae_bins(double eps) {
  const double PI = 3.14159265358979323846;
  return (long long)ceil((PI / (2.0 * eps)) * (1.0 + sqrt(1.0 + 4.0 * eps)));
}

// small odd-length median (Q <= 31) by insertion sort in registers
template <int QMAX>
SQ_DEV double median_of(double* v, int Q) {
  for (int i = 1; i < Q; ++i) {
    double x = v[i]; int j = i - 1;
    while (j >= 0 && v[j] > x) { v[j + 1] = v[j]; --j; }
    v[j + 1] = x;
  }
  return (Q & 1) ? v[Q / 2] : 0.5 * (v[Q / 2 - 1] + v[Q / 2]);
}

}  // namespace sq
