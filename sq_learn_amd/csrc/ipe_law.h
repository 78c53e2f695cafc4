// Shared device code of the IPE E-step kernels (csrc/ipe.hip: the fp32
// row-group kernel; csrc/ipe16.hip: the certified fp16 screen): the exact
// median-of-Q amplitude-estimation samplers, the pruned exact branch, the
// hazard bound of one pair and the initial hazard budgets.  See ipe.hip for
// the law (reference QuantumUtility/Utility.py:442-572, 697-737).
#pragma once
#include "common.h"
#include "band.h"
#include "fejer.h"

namespace sq {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr double binom_c(int n, int i) {
  double c = 1.0;
  for (int t = 1; t <= i; ++t) c = c * (double)(n - i + t) / (double)t;
  return c;
}

// Q (median repetitions) up to 31: Utility.py:534-572's Q for gamma down to
// ~1e-4; the draw path keeps the kIpeKeep smallest circular distances (the
// median of Q <= 31 draws is the (Q/2)-th of them)
constexpr int kIpeMaxQ = 31;
constexpr int kIpeKeep = 16;
static_assert(kIpeMaxQ / 2 + 1 <= kIpeKeep, "the median must be among the kept draws");
constexpr int kIpeWalkM = 128;

// binomial coefficients C(n, i), n < 32 (uniform indices: scalar loads)
static __constant__ double kBinom[32][32] = {
#define C_(n, i) ((i) > (n) ? 0.0 : binom_c(n, i))
#define R8(n, b) C_(n, b), C_(n, b + 1), C_(n, b + 2), C_(n, b + 3), C_(n, b + 4), C_(n, b + 5), \
                 C_(n, b + 6), C_(n, b + 7)
#define R(n) {R8(n, 0), R8(n, 8), R8(n, 16), R8(n, 24)}
    R(0),  R(1),  R(2),  R(3),  R(4),  R(5),  R(6),  R(7),  R(8),  R(9),  R(10),
    R(11), R(12), R(13), R(14), R(15), R(16), R(17), R(18), R(19), R(20), R(21),
    R(22), R(23), R(24), R(25), R(26), R(27), R(28), R(29), R(30), R(31)
#undef R
#undef R8
#undef C_
};

// P(Binomial(Q, F) >= h) = F^h sum_{m=0}^{Q-h} C(Q, h+m) F^m G^(Q-h-m),
// G = 1 - F: a homogeneous Horner scheme (one mul + one fma per term, all
// terms positive: no cancellation, no division)
SQ_DEV double binom_upper_tail(double F, int Q, int h) {
  if (F <= 0.0) return 0.0;
  if (F >= 1.0) return 1.0;
  const double G = 1.0 - F;
  const int nt = Q - h;
  double b = kBinom[Q][Q];
  double gp = 1.0;
  for (int m = nt - 1; m >= 0; --m) {
    gp *= G;
    b = fma(b, F, kBinom[Q][h + m] * gp);
  }
  double fh = 1.0;
  for (int i = 0; i < h; ++i) fh *= F;
  return fh * b;
}

// 1 / x to full fp64 precision: v_rcp_f64 + two Newton steps (the IEEE
// division sequence is ~3x longer)
SQ_DEV double rcp64(double x) {
  double r = __builtin_amdgcn_rcp(x);
  double e = fma(-x, r, 1.0);
  r = fma(r, e, r);
  e = fma(-x, r, 1.0);
  return fma(r, e, r);
}

// The median of Q (odd) iid draws T_1..T_Q with CDF F is F^-1(U_(h)), h =
// (Q + 1) / 2, U_(h) the h-th order statistic of Q uniforms ~ Beta(h, h):
// P(U_(h) <= x) = G(x) = P(Binomial(Q, x) >= h).  One uniform u gives
// x* = G^-1(u), after which the draw is ONE inverse-CDF walk of F to x* - no
// per-draw sorting (Utility.py:534-572's median over Q repetitions, exact
// law).

// exact draw of the median of Q (odd) iid AE estimates for small M: the
// value classes t = min(j, M - j) in increasing sin^2 order, their masses
// p(t) + p(M - t) accumulated until F(t) >= x* (fp64 angle-addition
// recurrence, no transcendental per step).  F(t) >= x* = G^-1(u) iff
// G(F(t)) >= u (G increasing), so the walk tests G(F(t)) >= u directly: one
// binomial tail per class step instead of a Newton solve for x* (~5-8 tail
// + density evaluations and a division per lane, divergent) - the walk to
// the median's class is short (its value is near the pair's a).
SQ_DEV double ae_median_walk(double omega, long long M, int Q, double u) {
  const double PI = 3.14159265358979323846;
  const double fl = floor(omega);
  const double phi = omega - fl;
  const double Md = (double)M;
  if (phi == 0.0) {   // all draws land on the true bin
    long long j = (long long)fl % M;
    if (j < 0) j += M;
    const double v = sin(PI * (double)j / Md);
    return v * v;
  }
  const int h = (Q + 1) / 2;
  const double sp = sin(PI * phi);
  const double num = sp * sp / (Md * Md);
  const double alpha = PI / Md, beta = PI * omega / Md;
  double sa, ca, sb, cb;
  sincos(alpha, &sa, &ca);
  sincos(beta, &sb, &cb);
  const long long tmax = M / 2;
  double st = 0.0, ct = 1.0;   // sin / cos(t alpha)
  double F = 0.0;
  double v = 0.0;
  for (long long t = 0; t <= tmax; ++t) {
    const double sm = st * cb - ct * sb;   // sin(t alpha - beta): bin t
    double mass = num * rcp64(sm * sm);
    if (t != 0 && 2 * t != M) {
      const double spl = st * cb + ct * sb;   // sin(t alpha + beta): bin M - t
      mass += num * rcp64(spl * spl);
    }
    F += mass;
    v = st * st;
    if (binom_upper_tail(F, Q, h) >= u) return v;
    const double nst = st * ca + ct * sa;
    ct = ct * ca - st * sa;
    st = nst;
  }
  return v;
}

// median of Q Fejer draws (any Q <= kIpeMaxQ, any M).  The Q draws are one
// inverse-CDF pass: their uniforms are generated already SORTED (sequential
// order statistics u_(i+1) = 1 - (1 - u_(i)) V^(1/(Q-i))), so a single
// central-out walk over l = 0, 1, -1, ..., +-kFejerWalk hands every draw its
// bin; the draws whose uniform lies beyond the walk's mass are drawn from the
// tail law (given how many fall there, they are iid from it - the multiset,
// and so the median, has exactly the law of Q independent draws).  Each
// draw's circular bin distance is bubbled into a sorted register array.
// The bin distances are integers: with M < 2^31 (every pair of realistic
// data - the caller decides per wave) they are kept as uint32 (one register,
// full-rate v_min_u32 / v_max_u32 compare-exchanges) instead of fp64.
SQ_DEV uint32_t ce_lo(uint32_t a, uint32_t b) { return min(a, b); }
SQ_DEV uint32_t ce_hi(uint32_t a, uint32_t b) { return max(a, b); }
SQ_DEV double ce_lo(double a, double b) { return fmin(a, b); }
SQ_DEV double ce_hi(double a, double b) { return fmax(a, b); }

template <typename K>
SQ_DEV void insert_sorted(K (&c)[kIpeKeep], K x) {
#pragma unroll
  for (int i = 0; i < kIpeKeep; ++i) {
    const K lo = ce_lo(c[i], x);
    x = ce_hi(c[i], x);
    c[i] = lo;
  }
}

template <typename K>
SQ_DEV double ae_median_draws(double omega, long long M, int Q, WordStream& ws) {
  const double PI = 3.14159265358979323846;
  const FejerLaw law(omega, M);   // per-pair setup shared by the Q draws
  K c[kIpeKeep];   // the kIpeKeep smallest so far, ascending
#pragma unroll
  for (int i = 0; i < kIpeKeep; ++i) c[i] = sizeof(K) == 4 ? (K)0xFFFFFFFFu : (K)1e300;
  auto circ = [&](long long j) -> K { return (K)(j < M - j ? j : M - j); };
  if (law.phi == 0.0 || M <= kFejerSmallM) {
#pragma nounroll
    for (int q = 0; q < Q; ++q) insert_sorted(c, circ(law.sample(ws)));
  } else {
    int got = 0;
    float om = 1.0f;   // 1 - u_(got+1)
    auto next_u = [&]() -> float {
      const float V = u01(ws.next());
      om *= __expf(__logf(V) / (float)(Q - got));
      return 1.0f - om;
    };
    float un = next_u();
    float acc = law.walk_term(law.sb);   // l = 0: sin(-beta)^2
    while (got < Q && un <= acc) {
      insert_sorted(c, circ(law.bin_of(0)));
      ++got;
      if (got < Q) un = next_u();
    }
    float st = 0.f, ct = 1.f;
    for (int t = 1; t <= kFejerWalk && got < Q; ++t) {
      const float nst = st * law.ca + ct * law.sa;
      const float nct = ct * law.ca - st * law.sa;
      st = nst;
      ct = nct;
      acc += law.walk_term(st * law.cb - ct * law.sb);   // l = +t
      while (got < Q && un <= acc) {
        insert_sorted(c, circ(law.bin_of(t)));
        ++got;
        if (got < Q) un = next_u();
      }
      acc += law.walk_term(st * law.cb + ct * law.sb);   // l = -t
      while (got < Q && un <= acc) {
        insert_sorted(c, circ(law.bin_of(-t)));
        ++got;
        if (got < Q) un = next_u();
      }
    }
#pragma nounroll
    for (; got < Q; ++got) insert_sorted(c, circ(law.bin_of(law.tail_ell(ws))));
  }
  double m1 = 0.0, m0 = 0.0;
#pragma unroll
  for (int i = 0; i < kIpeKeep; ++i) {
    if (i == Q / 2) m1 = (double)c[i];
    if (i == Q / 2 - 1) m0 = (double)c[i];
  }
  const double v1 = sin(PI * m1 / (double)M);
  if (Q & 1) return v1 * v1;
  const double v0 = sin(PI * m0 / (double)M);
  return 0.5 * (v0 * v0 + v1 * v1);
}

SQ_DEV float ipe_distance(float ipf, double nx2, double ny2, double eps, int Q, const RngKey& key,
                          unsigned long long sid) {
  const double ip = (double)ipf;
  const double S = nx2 + ny2;
  if (!(S > 0.0)) return 0.0f;
  double a = (S - 2.0 * ip) / (2.0 * S);
  if (fabs(a) <= 1e-15) a = 0.0;
  a = fmin(fmax(a, 0.0), 1.0);
  const double eps_a = eps * fmax(1.0, fabs(ip)) / S;
  long long M = ae_bins(eps_a);
  if (M > (1LL << 40)) M = 1LL << 40;
  if (M < 1) M = 1;
  const double PI = 3.14159265358979323846;
  const double omega = (double)M * asin(sqrt(a)) / PI;
  WordStream ws(key, sid);
  double at;
  if ((Q & 1) && M <= kIpeWalkM) {
    const uint32_t w0 = ws.next(), w1 = ws.next();
    const double u = ((double)(((unsigned long long)w0 << 21) ^ (unsigned long long)(w1 >> 11)) + 0.5) *
                     (1.0 / 9007199254740992.0);
    at = ae_median_walk(omega, M, Q, u);
  } else {
    // wave-uniform choice of the key type (same draws, same law either way)
    if (__ballot(M >= (1LL << 31)) == 0ull)
      at = ae_median_draws<uint32_t>(omega, M, Q, ws);
    else
      at = ae_median_draws<double>(omega, M, Q, ws);
  }
  return (float)(2.0 * S * at);
}

// ---------------------------------------------------------------- pruning
// A pair can change a row's label only if its estimate D~ is <= a value
// some other pair of the row actually drew, thr.  For odd Q the median's
// value class t (values increase with t = min(j, M - j)) is <= t_b =
// max{t : D~(t) <= thr} iff at least h = (Q+1)/2 of the Q draws fall in L =
// {bins of class <= t_b}: P(in L) = pi_L = P(Bin(Q, p_L) >= h), p_L the
// Fejer mass of L.  Every bin of L lies >= m = omega - t_b bins from omega,
// and the Fejer pmf is sin^2(pi phi) / (M^2 sin^2(pi delta / M)) <= 1 /
// (4 delta^2) (Jordan), so p_L <= pbar = (1/m + 1/m^2) / 2 and pi_L <= pibar =
// P(Bin(Q, pbar) >= h).  Given u uniform on [0, b) with b >= pibar, the pair
// loses when u >= pibar; otherwise p_L and pi_L are summed exactly, u >= pi_L
// loses, and u < pi_L gives the number c >= h of draws in L (P(C = c | C >=
// h), inverted with the same u) and the median = the h-th smallest of c iid
// draws from the Fejer law restricted to L: F_L^-1(p_L V), V ~ Beta(h, c - h
// + 1) from a fresh uniform.  Exact law of "D~ if <= thr" (ipe_pruned_exact).

// x = G^-1(u), G(x) = P(Bin(c, x) >= h): the h-th order statistic of c uniforms
SQ_DEV double order_stat_inv(double u, int c, int h) {
  if (c == 1) return u;
  double cq = (double)c;                  // c C(c-1, h-1)
  for (int i = 1; i < h; ++i) cq = cq * (double)(c - i) / (double)i;
  double lo = 0.0, hi = 1.0;
  const double mean = (double)h / (c + 1.0);
  const double sd = sqrt(mean * (1.0 - mean) / (c + 2.0));
  double x = mean + 1.4142135623730951 * sd * (double)erfinvf((float)(2.0 * u - 1.0));
  x = fmin(fmax(x, 1e-12), 1.0 - 1e-12);
  for (int it = 0; it < 60; ++it) {
    const double g = binom_upper_tail(x, c, h) - u;
    if (g > 0.0) hi = x; else lo = x;
    double dens = cq;
    for (int i = 0; i < h - 1; ++i) dens *= x;
    for (int i = 0; i < c - h; ++i) dens *= 1.0 - x;
    double xn = dens > 0.0 ? x - g / dens : 0.5 * (lo + hi);
    if (!(xn > lo && xn < hi)) xn = 0.5 * (lo + hi);
    const bool done = fabs(xn - x) <= 1e-15 * fmax(fmin(x, 1.0 - x), 1e-300) || hi - lo <= 1e-16;
    x = xn;
    if (done) break;
  }
  return x;
}

// the rare branch of the pruned sampler (u < pibar): exact p_L, pi_L, c and
// the restricted-law median by class walks (fp64 angle-addition recurrence)
SQ_DEV float ipe_pruned_exact(double ip, double S, double eps, int Q, float thr, double u,
                              WordStream& ws) {
  const double PI = 3.14159265358979323846;
  double a = (S - 2.0 * ip) / (2.0 * S);
  if (fabs(a) <= 1e-15) a = 0.0;
  a = fmin(fmax(a, 0.0), 1.0);
  const double eps_a = eps * fmax(1.0, fabs(ip)) / S;
  long long M = ae_bins(eps_a);
  if (M > (1LL << 40)) M = 1LL << 40;
  if (M < 1) M = 1;
  const double Md = (double)M;
  const double omega = Md * asin(sqrt(a)) / PI;
  const double fl = floor(omega);
  const double phi = omega - fl;
  const float INF = __builtin_inff();
  if (phi == 0.0) {   // point mass on the class of bin floor(omega)
    long long j = (long long)fl % M;
    if (j < 0) j += M;
    const long long t = j < M - j ? j : M - j;
    const double s = sin(PI * (double)t / Md);
    const float v = (float)(2.0 * S * s * s);
    return v <= thr ? v : INF;
  }
  const double sp = sin(PI * phi);
  const double num = sp * sp / (Md * Md);
  double sa, ca, sb, cb;
  sincos(PI / Md, &sa, &ca);
  sincos(PI * omega / Md, &sb, &cb);
  const long long tmax = M / 2;
  const int h = (Q + 1) / 2;
  // pass 1: p_L = mass of the classes whose value is <= thr
  double st = 0.0, ct = 1.0, F = 0.0;
  long long tb = -1;
  for (long long t = 0; t <= tmax; ++t) {
    if ((float)(2.0 * S * st * st) > thr) break;
    const double sm = st * cb - ct * sb;
    double mass = num / (sm * sm);
    if (t != 0 && 2 * t != M) {
      const double spl = st * cb + ct * sb;
      mass += num / (spl * spl);
    }
    F += mass;
    tb = t;
    const double nst = st * ca + ct * sa;
    ct = ct * ca - st * sa;
    st = nst;
  }
  if (tb < 0) return INF;
  const double pL = fmin(F, 1.0);
  if (!(u < binom_upper_tail(pL, Q, h))) return INF;
  // c = number of draws in L given >= h of them: P(C >= c) > u >= P(C >= c + 1)
  int c = h;
  {
    const double q = 1.0 - pL;
    double tail = 0.0;
    for (int cc = Q; cc >= h; --cc) {
      double pm = 1.0;   // C(Q, cc) pL^cc q^(Q - cc)
      for (int i = 0; i < cc; ++i) pm *= pL * (double)(Q - i) / (double)(i + 1);
      for (int i = 0; i < Q - cc; ++i) pm *= q;
      tail += pm;
      if (tail > u) { c = cc; break; }
    }
  }
  const uint32_t w0 = ws.next(), w1 = ws.next();
  const double u2 = ((double)(((unsigned long long)w0 << 21) ^ (unsigned long long)(w1 >> 11)) + 0.5) *
                    (1.0 / 9007199254740992.0);
  const double target = pL * order_stat_inv(u2, c, h);
  // pass 2: the restricted-law inverse CDF
  st = 0.0; ct = 1.0; F = 0.0;
  double v = 0.0;
  for (long long t = 0; t <= tb; ++t) {
    const double sm = st * cb - ct * sb;
    double mass = num / (sm * sm);
    if (t != 0 && 2 * t != M) {
      const double spl = st * cb + ct * sb;
      mass += num / (spl * spl);
    }
    F += mass;
    v = st * st;
    if (F >= target) break;
    const double nst = st * ca + ct * sa;
    ct = ct * ca - st * sa;
    st = nst;
  }
  return (float)(2.0 * S * v);
}

// ------------------------------------------------- hazard-budget screening
// Every pair of a row is screened against the row's FIXED threshold thr =
// the sampled estimate of its hint pair (the exact-distance argmin of pass
// 1, or the previous iteration's label).  pibar_j (above) bounds the
// probability that pair j's estimate reaches thr; instead of one uniform per
// pair (u < pibar_j), the pairs of one stream (row g, centroid class
// (j / 16) mod 4, j mod 16: the pairs one lane sweeps for that row, in tile
// order) form a sequence of independent Bernoulli(b_j) events,
// b_j = 1 - exp(-H_j), H_j = ceil(2^32 * pu_j (1 + 2^-10)) 2^-32 >= -log(1 - pu_j),
// pu_j >= pibar_j the fp32 union bound: one Exp(1) budget per stream, spent
// by the integer hazards H_j, fires at the pair where it runs out
// (memoryless: exactly the Bernoulli(b_j) law per pair).  A fired pair is
// thinned: u = U b_j, U uniform -> u is uniform on [0, b_j), so u >= pibar
// loses and u < pibar runs the exact branch above (u uniform on [0, pi_L)
// given u < pi_L: the exact law of "D~ if <= thr").  A far pair costs the
// fp32 bound and an integer subtract; fires are rare (sum of hazards <<
// 1 per stream), and a new budget is drawn only after one.  The outcome of
// each pair depends on (thr, its stream) only - never on the order in which
// the lanes' queues drain - so labels are identical however the rows are
// grouped into workgroups or sharded over ranks.

struct IpeScreen {
  float kq;       // (1 - 3e-6) / (sqrt(2) eps), rounded down (the m margin folded in)
  float smax;     // 6e10 eps, rounded down: S / max(1, |ip|) < smax keeps M below its cap
  float cqh;      // 1.0002 C(Q, h), rounded up (the pu margin folded in)
  float hf;       // h = (Q + 1) / 2
  uint32_t cap;   // initial budgets' cap (units 2^-32): 2^23 per pair of a stream
  double ucap;    // exp(-cap 2^-32): U <= ucap -> the capped budget
};

// upper bound on sqrt(x (1 + 2^-23)) (the class-value rounding of thr)
SQ_DEV float ipe_sthr(float x) { return __builtin_amdgcn_sqrtf(x) * 1.000001f; }

// The fp32 hazard of one pair against thr (sthr = ipe_sthr(thr)):
// true -> hq = its integer hazard (units 2^-32) and pbar; false -> the pair
// needs the full sampler (D~ competitive with thr, degenerate a, huge walk).
//   S = |x|^2 + |c|^2, D = S - 2 ip = 2 S a;  asin(y) - asin(x) >= y - x, so
//   every bin t of a class with value <= thr lies m >= (M / pi)(sqrt a - sqrt r)
//   >= sqrt(S) (sqrt D - sqrt thr') / (sqrt2 eps max(1, |ip|)) bins below omega
//   (M >= pi / eps_a = pi S / (eps max(1, |ip|)));  D >= S 2^-12 keeps the
//   fp32 relative error of D below 7.4e-4 (the sqrt(D) margin 4.9e-4 covers
//   its half); every other product carries its ulps in the 3e-6 margin.
SQ_DEV bool ipe_hazard(float ip, float nx2, float ny2, float sthr, float kt, const IpeScreen& sc,
                       uint32_t& hq, float& pbar) {
#pragma clang fp contract(off)   // the drain recomputes hq bit for bit
  // straight-line (every lane evaluates everything; the conditions are
  // combined at the end): no divergent exits in the tile epilogue.  Every
  // constant margin is folded into a per-launch (sc) or per-row (kt =
  // 1.571 sthr) factor.
  const float S = nx2 + ny2;
  const float D = fmaf(-2.0f, ip, S);
  const bool c1 = (D >= S * 2.44140625e-4f) & (D <= S * 1.998046875f);
  const float sD = __builtin_amdgcn_sqrtf(fmaxf(D, 0.0f)) * (1.0f - 4.8828125e-4f);
  const float ra = __builtin_amdgcn_rcpf(fmaxf(1.0f, fabsf(ip)));
  const float P = __builtin_amdgcn_sqrtf(S) * ra * sc.kq;
  const float m = (sD - sthr) * P;
  // t_b <= M sqrt(r) / 2, M <= pi / eps_a + pi + 1: the exact branch's walk
  const float tcap = fmaf(kt, P, 2.2f);
  // M below its 2^40 cap
  const bool c2 = (m >= 3.0f) & (tcap <= 1048576.0f) & (S * ra < sc.smax);
  // pb >= (r + r^2) / 2 (r = 1 / m): one rounded fma, the rcp's ulp and the
  // product's rounding inside the 2.4e-5 factor
  const float rm = __builtin_amdgcn_rcpf(fmaxf(m, 3.0f));
  // (rm <= 1/3 always: pb < 0.23, no clamp to 1)
  const float pb = fmaf(rm, rm, rm) * 0.500012f;
  // C(Q, h) pbar^h = C(Q, h) 2^(h log2 pbar): v_log / v_exp (1 ulp each;
  // |h log2 pbar| < 2^8 puts the exponent's error below 2^-14 relative to
  // pw... covered 30x by the 2e-4 margin in cqh); an underflow to 0 still
  // gives hq = 1 >= 2^32 pibar
  const float pu = sc.cqh * __builtin_amdgcn_exp2f(sc.hf * __builtin_amdgcn_logf(pb));
  // -log(1 - pu) <= pu (1 + pu) <= pu (1 + 2^-10): 2^32 H < 2^22.01, so 256
  // pairs of one stream never exhaust a capped (2^31) budget
  const bool c3 = pu < 9.765625e-4f;
  // (hq is only spent when c3 holds: no clamp; v_cvt saturates otherwise)
  hq = (uint32_t)(pu * (1.001f * 4294967296.0f)) + 1u;
  pbar = pb;
  return c1 & c2 & c3;
}

SQ_DEV float ipe_kt(float sthr) { return 1.571f * sthr; }

SQ_DEV bool ipe_hazard(float ip, float nx2, float ny2, float sthr, const IpeScreen& sc,
                       uint32_t& hq, float& pbar) {
  return ipe_hazard(ip, nx2, ny2, sthr, ipe_kt(sthr), sc, hq, pbar);
}

// 53-bit uniform in (0, 1) from two words
SQ_DEV double u53(uint32_t w0, uint32_t w1) {
  return ((double)(((unsigned long long)w0 << 21) ^ (unsigned long long)(w1 >> 11)) + 0.5) *
         (1.0 / 9007199254740992.0);
}

// an Exp(1) budget in units of 2^-32, capped at 2^31 (= E >= 1/2: more than
// 256 capped hazards can spend)
SQ_DEV uint32_t ipe_budget(uint32_t w0, uint32_t w1) {
  const double U = u53(w0, w1);
  if (U <= 0.6065306597126334) return 0x80000000u;   // exp(-1/2)
  return (uint32_t)(-log(U) * 4294967296.0);
}

// The initial budgets of a lane's streams: rows gb[t] + i (i < 4, the NG
// groups' first rows of one parity), class / column cls.  Rows 2m and 2m + 1
// take words (0, 1) / (2, 3) of one Philox block (stream 64 (2m) + cls,
// block 0; a fire's redraws use odd blocks) - half the Philox rounds, each
// stream's words still a function of (key, stream) only.  A stream spends at
// most (its pairs) x (2^-10 (1.001) + 2^-32) < cap 2^-32 (cap = 2^23 per
// pair), so a budget E >= cap never runs out - exactly as an uncapped one:
// only the ~3 % with U > exp(-cap 2^-32) need -log U, and those logs are
// lane-compacted (one fp64 log per round, each lane's next pending budget).
template <int NG>
SQ_DEV void ipe_initial_budgets(const RngKey& key, const long long (&gb)[NG], int cls,
                                const IpeScreen& sc, u32x4 (&bud)[NG]) {
  double U[NG][4];
  const bool odd = (gb[0] & 1) != 0;   // wave-uniform
#pragma unroll
  for (int t = 0; t < NG; ++t) {
    auto block = [&](long long row) -> u4 {
      WordStream ws(key, (unsigned long long)row * 64ull + (unsigned long long)cls);
      u4 w;
      w.x = ws.next();
      w.y = ws.next();
      w.z = ws.next();
      w.w = ws.next();
      return w;
    };
    if (!odd) {
      const u4 a = block(gb[t]), c = block(gb[t] + 2);
      U[t][0] = u53(a.x, a.y);
      U[t][1] = u53(a.z, a.w);
      U[t][2] = u53(c.x, c.y);
      U[t][3] = u53(c.z, c.w);
    } else {
      const u4 a = block(gb[t] - 1), c = block(gb[t] + 1), e = block(gb[t] + 3);
      U[t][0] = u53(a.z, a.w);
      U[t][1] = u53(c.x, c.y);
      U[t][2] = u53(c.z, c.w);
      U[t][3] = u53(e.x, e.y);
    }
  }
  uint32_t pend = 0u;
#pragma unroll
  for (int t = 0; t < NG; ++t) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      bud[t][i] = sc.cap;
      pend |= U[t][i] > sc.ucap ? 1u << (4 * t + i) : 0u;
    }
  }
  while (__ballot(pend != 0u) != 0ull) {
    const int b = pend ? __builtin_ctz(pend) : 0;
    double u = 0.5;
#pragma unroll
    for (int t = 0; t < NG; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) u = b == 4 * t + i ? U[t][i] : u;
    const uint32_t v = (uint32_t)(-log(u) * 4294967296.0);
#pragma unroll
    for (int t = 0; t < NG; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) bud[t][i] = (pend && b == 4 * t + i) ? v : bud[t][i];
    pend &= pend - 1u;
  }
}

// The same budgets for arbitrary rows (list mode): row g takes words (0, 1)
// of block (g, cls) when g is even, words (2, 3) of block (g - 1, cls) when
// odd - exactly ipe_initial_budgets' pairing, one block per row.
template <int NG>
SQ_DEV void ipe_initial_budgets_rows(const RngKey& key, const long long (&gr)[NG][4], int cls,
                                     const IpeScreen& sc, u32x4 (&bud)[NG]) {
  double U[NG][4];
#pragma unroll
  for (int t = 0; t < NG; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const long long g = gr[t][i];
      WordStream ws(key, (unsigned long long)(g & ~1LL) * 64ull + (unsigned long long)cls);
      const uint32_t w0 = ws.next(), w1 = ws.next(), w2 = ws.next(), w3 = ws.next();
      U[t][i] = (g & 1) ? u53(w2, w3) : u53(w0, w1);
    }
  uint32_t pend = 0u;
#pragma unroll
  for (int t = 0; t < NG; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      bud[t][i] = sc.cap;
      pend |= U[t][i] > sc.ucap ? 1u << (4 * t + i) : 0u;
    }
  while (__ballot(pend != 0u) != 0ull) {
    const int b = pend ? __builtin_ctz(pend) : 0;
    double u = 0.5;
#pragma unroll
    for (int t = 0; t < NG; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) u = b == 4 * t + i ? U[t][i] : u;
    const uint32_t v = (uint32_t)(-log(u) * 4294967296.0);
#pragma unroll
    for (int t = 0; t < NG; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) bud[t][i] = (pend && b == 4 * t + i) ? v : bud[t][i];
    pend &= pend - 1u;
  }
}

SQ_DEV bool ipe_better(float ob, uint32_t ok, int oj, float b, uint32_t kk, int jj) {
  return ob < b || (ob == b && (ok < kk || (ok == kk && oj < jj)));
}

}  // namespace sq
