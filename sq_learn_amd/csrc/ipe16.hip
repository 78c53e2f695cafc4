// Certified fp16 screen of the IPE E-step of q-means ("l2-sampled" distance
// estimates, the reference DEFAULT: sklearn/cluster/_dmeans.py:753-772 ->
// QuantumUtility/Utility.py:697-737).  Same law as ipe.hip,
// without an fp32 inner product per (row, centroid) pair.
//
// The estimator (ipe.hip header): D~ = 2 S a~, a~ the median of Q amplitude
// estimations of a = (S - 2 ip) / (2 S), S = |x|^2 + |c|^2; label = argmin_j D~.
// As in ipe.hip every row first samples its HINT pair (the previous labels,
// or an approximate argmin) in full: thr = D~_hint.  Every other pair can only
// matter if its estimate falls at or below thr, and its probability of doing
// so is bounded by the Fejer tail at m = (sqrt(D) - sqrt(thr)) sqrt(S) /
// (sqrt2 eps max(1, |ip|)) bins (ipe_hazard).  Here that bound is taken PER
// ROW over a distance band instead of per pair:
//
//  * prep (one lane per row): the hint's exact inner product (the canonical
//    fp32 dot below), thr, and a band [Dl, Dh] of squared distances such that
//    every pair whose fp32 law distance lies in it passes ipe_hazard with
//    hazard <= H_row (a rigorous fp64 bound over S in [Smin, Smax] of the
//    row, every fp32 rounding of the screen covered), translated into the
//    certified fp16 filter's units (estep_f32.hip estep_x64: v = alpha^2
//    (|c|^2 - 2 x.c) with the per-row error bound E_i): far iff
//    Vlo <= v <= Vhi;
//  * sweep (fp16 v_mfma_f32_32x32x16_f16 over the fp16 copy of alpha x, the
//    estep_x64 tile ring): a pair is FAR (per-pair cost: one med3 and one
//    compare) or NEAR (appended to its row's LDS list).  Far pairs never read
//    their inner product: each fires with probability 1 - exp(-H_row),
//    independently (the memoryless budget construction of ipe.hip), so the
//    fire positions are known in advance - prep draws them per row (a
//    binomial count, then a uniform subset of the pairs) and evaluates the
//    fired pairs itself;
//  * near kernel: every listed pair gets the canonical fp32 inner product;
//    a near pair is sampled in full (ipe_distance, the pair's own Philox
//    stream), a fired far pair is thinned to the exact law of "D~ if <= thr"
//    (u = U (1 - exp(-H_row)) < pibar: ipe_pruned_exact); results merge into
//    the row's (D~, tie key | j) by one 64-bit atomicMin;
//  * rows with more than kCapR listed pairs ("dense": no usable band, or a
//    crowded threshold) are left to the fp32 row-group kernel of ipe.hip in
//    list mode, with the same hint and threshold.
// Every decision is a function of the row, its hint, the centroids and the
// Philox keys (global row index): labels do not depend on blocking, list
// order or the number of ranks.
//
// The canonical inner product of a pair (the one the law uses - the reference
// uses np.inner in fp64; any fixed fp32 order is within ~d 2^-24 |x||c|):
// lane c16 of a 16-lane group sums f = c16, c16 + 16, ... by fmaf in order,
// then an xor tree over the 16 lanes (ipe_hint_kernel's order).
#include "ipe_law.h"
#include <cmath>
#include <utility>

namespace sq {
namespace i16 {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// Timing-only variant builds (benchmarks/ipe16_prep_variants.py): bits of
// SQ_IPE16_DIAG drop parts of prep - 1: the hint's sampler (thr = the fp32
// distance), 2: the budget / fire listing, 4: the fired pairs' evaluation,
// 8: the per-group bands (group 0's for all), 16: the sweep's near-pair
// flush (flagged values dropped), 32: the sweep's far-minimum upkeep.
// Results are NOT the law's;
// never set in the production build.
#ifndef SQ_IPE16_DIAG
#define SQ_IPE16_DIAG 0
#endif

constexpr int kTileN = 64;    // centroids per LDS tile (estep_x64 operand)
constexpr int kNW = 4;        // waves per workgroup (one per SIMD)
constexpr int kRS = 2;        // row sets of 32 per wave
constexpr int kRows = kNW * 32 * kRS;   // 256 rows per block
constexpr int kRing = 3;      // centroid-tile LDS slots
constexpr int kCapR = 64;     // listed pairs per row (more: dense)
constexpr int kNLS = kCapR + 2;   // LDS row stride of the lists (uint16): no bank aliasing
constexpr int kMaxG = 4;      // centroid groups (tiles sorted by |c|^2): one band per group
constexpr int kFireCap = 7;   // listed fires per row (more: dense); [0] of a row's record = count

SQ_DEV float vmin(float a, float b) {
  float r;
  asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
SQ_DEV float and_or(float a, uint32_t m, uint32_t q) {
  float r;
  asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(m), "v"(q));
  return r;
}
SQ_DEV float vmed3(float a, float b, float c) {
  float r;
  asm("v_med3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

template <typename F, int... I>
SQ_DEV void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
SQ_DEV void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// the row-sorted packed best: (D~ bits, tie key with the centroid in its low
// 14 bits) - one u64 min orders by (D~, random key), like ipe_better
SQ_DEV unsigned long long pack_best(float dt, const RngKey& tie, long long g, int j) {
  const uint32_t tk = (band_key(tie, g, (uint32_t)j) & ~0x3FFFu) | (uint32_t)j;
  return ((unsigned long long)__float_as_uint(dt) << 32) | (unsigned long long)tk;
}

// canonical fp32 inner products of B (row, centroid) pairs (stride-1, d <=
// 16 U values) by the 16 lanes c16 = 0..15 of a group, every lane returning
// the totals: lane c16 sums f = c16, c16 + 16, ... by fmaf in order (zeros
// past d add +0), then an xor tree over the 16 lanes.  All B pairs' loads
// are issued before the first fma (one memory latency per batch, not one
// per pair).
// (U > 16, wide rows: 16 values per pair at a time, the same fmaf order)
template <int U, int B>
SQ_DEV void canon_dot_batch(const float* const (&xp)[B], const float* const (&cp)[B], int d,
                            int c16, float (&out)[B]) {
  constexpr int UC = U < 16 ? U : 16;
  static_assert(U % UC == 0, "chunked canonical dot");
  float s[B];
#pragma unroll
  for (int b = 0; b < B; ++b) s[b] = 0.0f;
  for (int u0 = 0; u0 < U; u0 += UC) {
    float xv[B][UC], cv[B][UC];
#pragma unroll
    for (int b = 0; b < B; ++b)
#pragma unroll
      for (int u = 0; u < UC; ++u) {
        const int f = c16 + 16 * (u0 + u);
        xv[b][u] = f < d ? xp[b][f] : 0.0f;
        cv[b][u] = f < d ? cp[b][f] : 0.0f;
      }
#pragma unroll
    for (int b = 0; b < B; ++b)
#pragma unroll
      for (int u = 0; u < UC; ++u) s[b] = fmaf(xv[b][u], cv[b][u], s[b]);
  }
#pragma unroll
  for (int b = 0; b < B; ++b) {
    float t = s[b];
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) t += __shfl_xor(t, o, 64);
    out[b] = t;
  }
}

// the next float above x (finite x)
SQ_DEV float f32_up(float x) {
  if (x == 0.0f) return 1.401298464e-45f;
  const uint32_t b = __float_as_uint(x);
  return __uint_as_float(x > 0.0f ? b + 1u : b - 1u);
}

struct Cut {
  float vlo, vhi, H;
  int ok;
};

struct CutParams {
  double alpha, Ch, sub_rel, mt, min_width;
  int d;
  // per-launch constants of row_cut (host: cut_constants): the per-row
  // band then costs 6 fp64 sqrt and 2 divisions per group instead of 8
  // sqrt, 8 divisions and a pow
  double c, inv_c, kqm, mt_e, a, inv2a, mtk, klo, khi;
  float Hf;
  int band_ok;
};

// The row's exact squared norm range [x2lo, x2hi] (fp32 |x|^2 with its
// summation error) and the fp16 filter's error bound E on
// v = alpha^2 (|c|^2 - 2 x.c) (estep_x64's per-row bound).
struct RowErr {
  double x2lo, x2hi, E;
};
SQ_DEV RowErr row_err(float nx2f, const CutParams& cp) {
  const double u = 0x1p-24;
  const double nx2 = nx2f;
  RowErr r;
  r.x2lo = nx2 * (1.0 - (cp.d + 2) * u);
  r.x2hi = nx2 * (1.0 + (cp.d + 2) * u);
  const double xsv = cp.alpha * sqrt(r.x2hi) * (1.0 + 0x1p-16);
  r.E = (1.0625 * 0x1p-10 * xsv * cp.Ch + 0x1p-15 * (0.25 * cp.Ch * cp.Ch + xsv * cp.Ch) +
         cp.sub_rel * (xsv + cp.Ch)) * (1.0 + 1e-6);
  return r;
}

// fp64 -> fp32 rounded down / up (finite x)
SQ_DEV float f32_dn(double x) {
  float f = (float)x;
  if ((double)f > x) f = -f32_up(-f);
  return f;
}
SQ_DEV float f32_upd(double x) {
  float f = (float)x;
  if ((double)f < x) f = f32_up(f);
  return f;
}

// Lower bound on sqrt(D) of a pair from its canonical fp32 inner product
// (law D vs exact D within (3 d + 64) 2^-24 S, as in row_cut).
SQ_DEV float pair_dist_lo(float ip, float nx2, float ny2, int d) {
  const double S = (double)nx2 + (double)ny2;
  const double D = S - 2.0 * (double)ip - (3.0 * d + 64.0) * 0x1p-24 * S * (1.0 + 1e-6);
  return D > 0.0 ? f32_dn(sqrt(D) * (1.0 - 1e-12)) : 0.0f;
}

// The row's far band (see the header).  For a pair at law distance D with
// S in [Smin, Smax] and ip = (S - D) / 2 (fp32 rounding folded in), the
// screen's bin distance is m = (c sqrt(D) - sthr) kq sqrt(S) /
// max(1, |ip|); for fixed D, sqrt(S) / max(1, |S - D| / 2) is unimodal in S,
// so its minimum is at Smin or Smax, and for each endpoint the set of y =
// sqrt(D) with m >= m_t is an interval with closed-form ends (one quadratic
// below S, one above).  The band is the intersection of the two intervals
// and of ipe_hazard's other conditions; its hazard bound is pu(m_t).  All in
// fp64, with margins covering every fp32 rounding of ipe_hazard.
SQ_DEV Cut row_cut(float nx2f, float sthrf, float ktf, float Sminf, float Smaxf, const IpeScreen& sc,
                   const CutParams& cp) {
  Cut out{__builtin_inff(), -__builtin_inff(), 0.0f, 0};
  if (!cp.band_ok) return out;                                        // c2, c3 (m_t, pu)
  const double Smin = Sminf, Smax = Smaxf, kq = sc.kq, kt = ktf;
  const double sthr = (double)sthrf * (1.0 + 1e-7);
  if (!(Smin > 0.0) || !(sthr < 1e300)) return out;
  const double rSmin = sqrt(Smin), rSmax = sqrt(Smax);
  const double Pmax = kq * rSmax * (1.0 + 1e-5);
  if (!(kt * Pmax + 2.2 <= 1048576.0 * (1.0 - 1e-6))) return out;    // walk cap (c2)
  if (!(Smax * (1.0 + 1e-5) < (double)sc.smax)) return out;           // M cap (c2)
  // sqrt(Smax 2^-12 (1 + 1e-5)) and sqrt(Smin 1.998046875 (1 - 1e-5)) (c1)
  // as products with constants (the few-ulp differences are inside the
  // 1e-9 margins below)
  double ylo = rSmax * cp.klo;
  double yhi = rSmin * cp.khi;
  // |ip| <= |S - D| / 2 (1 + 1e-6) + 1e-6 S: m >= mt  <=>
  //   kqm sqrt(S) (c y - sthr) >= mt max(1, |S - y^2| (1 + 1e-6) / 2 + 1e-6 S)
  const double a = cp.a;
  for (int side = 0; side < 2; ++side) {
    const double S = side ? Smax : Smin;
    const double rS = side ? rSmax : rSmin;
    const double B = 2.0 * cp.kqm * rS * cp.c;
    const double C0 = 2.0 * cp.kqm * rS * sthr;
    const double sl = 2e-6 * cp.mt_e * S;
    // max(1, .) = 1 part: c y - sthr >= mt / (kqm rS)
    const double y0 = (cp.mtk / rS + sthr) * cp.inv_c;
    // below S: a y^2 + B y - (a S + sl + C0) >= 0
    const double cA = a * S + sl + C0;
    const double yA = (-B + sqrt(B * B + 4.0 * a * cA)) * cp.inv2a;
    // above S: a y^2 - B y + (C0 + sl - a S) <= 0
    const double dB = B * B - 4.0 * a * (C0 + sl - a * S);
    if (!(dB >= 0.0)) return out;
    const double sdB = sqrt(dB);
    const double yB = (B + sdB) * cp.inv2a;
    const double yBm = (B - sdB) * cp.inv2a;
    // m >= mt on {y >= yA} (below-S branch) intersected with [yBm, yB]
    ylo = fmax(ylo, fmax(y0, fmax(yA, yBm)) * (1.0 + 1e-9));
    yhi = fmin(yhi, yB * (1.0 - 1e-9));
  }
  if (!(ylo <= yhi)) return out;
  const double Dl = ylo * ylo, Dh = yhi * yhi;
  // a sliver of a band (a row whose threshold sits among the other
  // centroids) would list most of its pairs: dense from the start
  if (Dh - Dl < cp.min_width * Dl) return out;
  // -> fp16 filter units: v = alpha^2 (D - |x|^2) +- E
  const double errD = (3.0 * cp.d + 64.0) * 0x1p-24 * Smax;           // law D vs exact D
  const RowErr re = row_err(nx2f, cp);
  const double a2 = cp.alpha * cp.alpha;
  const double vlo = a2 * (Dl + errD - re.x2lo) + re.E;
  const double vhi = a2 * (Dh - errD - re.x2hi) - re.E;
  float flo = (float)vlo, fhi = (float)vhi;
  if ((double)flo < vlo) flo = f32_up(flo);
  if ((double)fhi > vhi) fhi = -f32_up(-fhi);
  if (!(flo <= fhi)) return out;
  out.vlo = flo;
  out.vhi = fhi;
  out.H = cp.Hf;   // depends on m_t only
  out.ok = 1;
  return out;
}

// row_cut's per-launch constants (the margins of the per-row version they
// replace: c, kqm, mt's (1 + 1e-6); pu(m_t) and H >= -log(1 - pu) rounded up)
static void cut_constants(CutParams& cp, const IpeScreen& sc) {
  const double e1 = 1.0 + 1e-6;
  cp.c = (1.0 - 4.8828125e-4) * (1.0 - 1e-6);   // sD = sqrt(D) (1 - 2^-11), rounded
  cp.inv_c = (1.0 / cp.c) * (1.0 + 1e-15);
  cp.kqm = (double)sc.kq * (1.0 - 3e-5);         // sqrt / rcp / products of P and m
  cp.mt_e = cp.mt * (1.0 + 1e-6);
  cp.a = cp.mt_e * e1;
  cp.inv2a = (1.0 / (2.0 * cp.a)) * (1.0 + 1e-15);
  cp.mtk = cp.mt_e / cp.kqm * (1.0 + 1e-15);
  cp.klo = sqrt(0x1p-12 * (1.0 + 1e-5)) * (1.0 + 1e-15);
  cp.khi = sqrt(1.998046875 * (1.0 - 1e-5)) * (1.0 - 1e-15);
  const double m = cp.mt;
  const double r = (1.0 / m) * (1.0 + 1e-5);
  const double pb = (r + r * r) * 0.500012 * (1.0 + 1e-5);
  const double pu = (double)sc.cqh * pow(pb, (double)sc.hf) * (1.0 + 2e-3);
  cp.band_ok = (m >= 3.0 && pu < 9.765625e-4 * (1.0 - 1e-6)) ? 1 : 0;   // c2, c3
  const double H = pu * (1.0 + pu) * (1.0 + 1e-6);                       // >= -log(1 - pu)
  float Hf = (float)H;
  if ((double)Hf < H) Hf = std::nextafter(Hf, 1e30f);
  cp.Hf = Hf;
}

// ------------------------------------------------------------------ prep
// Per row: the hint pair in full (thr), the far band, the row's budget
// draw.  Outputs (row-indexed, local rows): thr / hj (ipe.hip's ext_thr /
// ext_hj: the dense fallback reuses them), vlo / vhi / H, rM (min of the 32
// stream budgets when it can run out within the row, else -1), rst (1: no
// usable band or hint - dense), best (the hint's packed estimate).
//
// Row skip (lb given).  lb[r] is a lower bound on |x - c_j| for every
// centroid j other than the row's label of the previous E-step (= this
// step's hint), at that step's centres; moved by the largest centroid shift
// since (Hamerly).  With ub = |x - c_hint| + max_j |c_hint - c_j| an upper
// bound on every other distance, a row whose [lb^2, ub^2] lies inside
// EVERY group's far band - with the fp16 filter's error E and the |x|^2
// range folded in, i.e. where the sweep would provably classify every
// non-hint pair far - needs no sweep: its only listed pairs would be its
// fires (prep's own list, the hint's dropped).  Prep finishes such a row
// itself: canonical fp32 dots of its fired pairs, the near kernel's
// thinning of a fired far pair (same streams, same arithmetic), the packed
// minimum -> labels / mind; so the labels are bit-identical with the skip
// on or off.  Every other row goes to the sweep's row list.
struct PrepArgs {
  const float* X;
  long long ldx;
  const float* C;
  const int* hint;
  const float* xn;
  const float* cn;
  float* thr;
  int* hj;
  float* vlo;
  float* vhi;
  float* H;
  unsigned char* rst;
  unsigned long long* best;
  uint16_t* rfire;          // [n][8]: count, then up to kFireCap fired pairs (j | 0x8000)
  const float* gS;          // [G][2] min / max |c|^2 of each centroid group
  int G;
  long long n;
  int d, k;
  double eps;
  int Q;
  RngKey key, tie, bkey, skey;
  long long row_offset;
  IpeScreen sc;
  CutParams cp;
  unsigned long long* stats;
  // row skip / bound upkeep (lb == nullptr: off)
  float* lb;                // [n] lower bound on sqrt(D) to every non-label centroid
  int lb_ok;                // lb is relative to `hint` (the previous labels)
  const float* smax;        // [1] tau: the largest shift of a non-wild centroid since
                            //     lb's centres (rounded up; the W largest are "wild")
  const float* Rc;          // [k][4] max over group g of |c_l - c_j| (rounded up)
  const float* mw;          // [k] min over the wild j != l of |c_l - c_j| (rounded down)
  float* lbo;               // [n] x2lo - E / alpha^2: the sweep's v -> D lower bound
  float* dhint;             // [n] lower bound on sqrt(D) of the hint pair
  int* rows;                // rows left to the sweep (all of them when lb is off)
  int* rows_count;
  int* labels;              // skipped rows' results
  float* mind;
  unsigned char* rflag;     // skipped rows: 2 (finalize leaves them)
  float* ea2;               // [n] E / alpha^2 (the sweep's pair certificate)
};

template <int KU>
__global__ void __launch_bounds__(256) ipe16_prep_kernel(PrepArgs a) {
  constexpr int kWF = 64 * kFireCap;   // a wave's fired pairs of skipped rows
  __shared__ float sip[256];
  __shared__ int slab[256];
  __shared__ float red[2][4];
  __shared__ uint32_t fpair[4][kWF];   // (lane << 16) | j
  __shared__ float fip[4][kWF];
  __shared__ unsigned long long sbest[256];
  __shared__ float s_t[256], s_H[256];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c16 = lane & 15, q4 = lane >> 4;
  // min / max of the centroid norms (S range of every pair of a row)
  float mn = __builtin_inff(), mx = 0.0f;
  for (int j = threadIdx.x; j < a.k; j += 256) {
    mn = fminf(mn, a.cn[j]);
    mx = fmaxf(mx, a.cn[j]);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    mn = fminf(mn, __shfl_xor(mn, o, 64));
    mx = fmaxf(mx, __shfl_xor(mx, o, 64));
  }
  if (lane == 0) {
    red[0][wave] = mn;
    red[1][wave] = mx;
  }
  const long long rb = (long long)blockIdx.x * 256 + wave * 64;
  // the wave's 64 hint pairs, 4 per lane group: rows 16 g + 4 b + q4
  constexpr int B = 4;
#pragma unroll 1
  for (int g = 0; g < 4; ++g) {
    const float* xp[B];
    const float* cp_[B];
    int lb[B];
#pragma unroll
    for (int b = 0; b < B; ++b) {
      const long long r = rb + 16 * g + 4 * b + q4;
      const int l = r < a.n ? a.hint[r] : -1;
      const bool ok = r < a.n && l >= 0 && l < a.k;
      lb[b] = ok ? l : -2;
      xp[b] = a.X + (size_t)(ok ? r : 0) * a.ldx;
      cp_[b] = a.C + (size_t)(ok ? l : 0) * a.d;
    }
    float sv[B];
    canon_dot_batch<KU, B>(xp, cp_, a.d, c16, sv);
    if (c16 == 0) {
#pragma unroll
      for (int b = 0; b < B; ++b) {
        const int x = 16 * g + 4 * b + q4;
        sip[wave * 64 + x] = sv[b];
        slab[wave * 64 + x] = lb[b];
      }
    }
  }
  __syncthreads();
  const float cmin = fminf(fminf(red[0][0], red[0][1]), fminf(red[0][2], red[0][3]));
  const float cmax = fmaxf(fmaxf(red[1][0], red[1][1]), fmaxf(red[1][2], red[1][3]));
  (void)cmin;
  const long long r = rb + lane;
  uint32_t st_flag = 0, st_dense = 0, st_skip = 0, st_exact = 0, st_full = 0;
  // C^ = 2 alpha max_j |c_j| of the fp16 filter's bound, from the largest
  // fp32 norm widened by its summation error
  CutParams cp = a.cp;
  cp.Ch = 2.0 * cp.alpha * sqrt((double)cmax * (1.0 + (cp.d + 2) * 0x1p-24)) * (1.0 + 0x1p-16);
  const double a2 = cp.alpha * cp.alpha;
  bool skip = false;
  int nfs = 0;                 // fired pairs prep finishes itself (skipped rows)
  uint16_t fire[kFireCap];
  int l = -2;
  float t = __builtin_inff();
  float lbe_f = 0.0f, dh_lo = 0.0f;
  long long g = 0;
  if (r < a.n) {
    l = slab[threadIdx.x];
    g = a.row_offset + r;
    const float nx2 = a.xn[r];
    Cut cut{-__builtin_inff(), __builtin_inff(), 0.0f, 0};
    int nf = 0;
    float glo[kMaxG], ghi[kMaxG];
    int nok = 0;
    if (l >= 0) {
#if SQ_IPE16_DIAG & 1
      t = fmaxf(nx2 + a.cn[l] - 2.0f * sip[threadIdx.x], 0.0f);
#else
      t = ipe_distance(sip[threadIdx.x], (double)nx2, (double)a.cn[l], a.eps, a.Q, a.key,
                       (unsigned long long)g * (unsigned long long)a.k + (unsigned long long)l);
#endif
      const float sthr = ipe_sthr(t);
      // one band per centroid group (its own S range: the groups are
      // contiguous in |c|^2); a group without a band lists all its pairs
      for (int q = 0; q < a.G; ++q) {
#if SQ_IPE16_DIAG & 8
        const Cut cq = row_cut(nx2, sthr, ipe_kt(sthr), nx2 + a.gS[0], nx2 + a.gS[2 * a.G - 1],
                               a.sc, cp);
#else
        const Cut cq = row_cut(nx2, sthr, ipe_kt(sthr), nx2 + a.gS[2 * q], nx2 + a.gS[2 * q + 1],
                               a.sc, cp);
#endif
        // (no band: [+inf, +inf] - med3(v, +inf, +inf) != v, every pair near;
        // an inverted interval would make med3 return v: far)
        glo[q] = cq.ok ? cq.vlo : __builtin_inff();
        ghi[q] = cq.ok ? cq.vhi : __builtin_inff();
        if (cq.ok) {
          cut = cq;   // H depends on m_t only: the same for every group
          ++nok;
        }
      }
      cut.ok = nok > 0;
    }
    if (cut.ok) {
      // Each far pair fires with probability b = 1 - exp(-H), independently
      // (a stream spending H per pair from a memoryless Exp(1) budget):
      // the row's fires are N ~ Binomial(k, b) by inversion (P(0) =
      // exp(-k H), P(n + 1) / P(n) = (k - n) / (n + 1) (e^H - 1)) and, given
      // N, a uniform N-subset of the k pairs (Lemire integers, duplicates
      // redrawn) - one exp and ~N Philox words per row, no per-fire log.
      // More than kFireCap fires: the row is dense.
      const double H = (double)cut.H;
      if (!(SQ_IPE16_DIAG & 2)) {
        WordStream ws(a.bkey, (unsigned long long)g);
        const uint32_t w0 = ws.next(), w1 = ws.next();
        const double u = u53(w0, w1);
        double pn = exp(-(double)a.k * H);
        double cdf = pn;
        const double rat = expm1(H);
        int N = 0;
        while (u > cdf && N <= kFireCap) {
          pn *= (double)(a.k - N) / (double)(N + 1) * rat;
          cdf += pn;
          ++N;
        }
        const uint32_t km = (uint32_t)a.k;
        const uint32_t kthr = (uint32_t)(-km) % km;
        for (int e = 0; e < N && e < kFireCap; ++e) {
          uint32_t j = 0;
          bool dup = true;
          while (dup) {
            uint32_t wv = ws.next();
            unsigned long long xm = (unsigned long long)wv * km;
            while ((uint32_t)xm < kthr) {
              wv = ws.next();
              xm = (unsigned long long)wv * km;
            }
            j = (uint32_t)(xm >> 32);
            dup = false;
            for (int f = 0; f < e; ++f) dup = dup || (fire[f] & 0x3FFFu) == j;
          }
          fire[e] = (uint16_t)(j | 0x8000u);
        }
        nf = N;
      }
      st_flag = nf > 0 ? 1 : 0;
      if (nf > kFireCap) cut.ok = 0;   // a row this hot: dense
    }
    const RowErr re = row_err(nx2, cp);
    a.ea2[r] = f32_upd(re.E / a2);
    if (a.lb && l >= 0) {
      const double S = (double)nx2 + (double)a.cn[l];
      const double errH = (3.0 * cp.d + 64.0) * 0x1p-24 * S * (1.0 + 1e-6);
      const double Dc = S - 2.0 * (double)sip[threadIdx.x];
      dh_lo = Dc - errH > 0.0 ? f32_dn(sqrt(Dc - errH) * (1.0 - 1e-12)) : 0.0f;
      if (a.lb_ok && cut.ok && nok == a.G) {
        // non-wild centroids moved by <= tau since the bound; the wild ones
        // by the triangle inequality through the hint's centre
        const double dhi0 = sqrt(fmax(Dc + errH, 0.0)) * (1.0 + 1e-12);
        const double lbe = fmin((double)a.lb[r] - (double)a.smax[0], (double)a.mw[l] - dhi0);
        if (lbe > 0.0) {
          // every non-hint pair provably far in the sweep: its exact D in
          // [need_lo, need_hi] of its group puts v = alpha^2 (D - |x|^2) +- E
          // inside [vlo, vhi]
          double need_lo = -__builtin_inf();
          for (int q = 0; q < a.G; ++q) need_lo = fmax(need_lo, ((double)glo[q] + re.E) / a2 + re.x2hi);
          need_lo += 1e-12 * fabs(need_lo);
          // upper side per group: |x - c_j| <= |x - c_hint| + |c_hint - c_j|
          const double dhi = sqrt(fmax(Dc + errH, 0.0)) * (1.0 + 1e-12);
          bool up = true;
          for (int q = 0; q < a.G; ++q) {
            const double nh = ((double)ghi[q] - re.E) / a2 + re.x2lo;
            const double ub = dhi + (double)a.Rc[4 * l + q];
            up = up && ub * ub * (1.0 + 1e-12) <= nh - 1e-12 * fabs(nh);
          }
          skip = lbe * lbe * (1.0 - 1e-12) >= need_lo && up;
          lbe_f = f32_dn(lbe);
        }
      }
      if (!skip) a.lbo[r] = f32_dn(re.x2lo - re.E / a2);
      if (!skip) a.dhint[r] = dh_lo;
    }
    // every row's fired pairs are finished here (the row's X was just read
    // for the hint pair): a fire on the hint is void (dense rows: the
    // fallback samples the whole row)
    if (cut.ok && !(SQ_IPE16_DIAG & 4))
      for (int e = 0; e < nf; ++e)
        if ((fire[e] & 0x3FFF) != l) fire[nfs++] = fire[e];
    if (skip || nfs > 0) {
      s_t[threadIdx.x] = t;
      s_H[threadIdx.x] = cut.H;
    }
    if (skip) {
      st_skip = 1;
    } else {
      if (!cut.ok) {
        // dense: every pair "far" in the sweep (no list traffic), the whole
        // row to the fp32 kernel
        cut.vlo = -__builtin_inff();
        cut.vhi = __builtin_inff();
        st_dense = 1;
      }
      if (l >= 0 && nfs == 0) a.best[r] = pack_best(t, a.tie, g, l);
      a.thr[r] = t;
      a.hj[r] = l >= 0 ? l : -2;
      for (int q = 0; q < a.G; ++q) {
        a.vlo[r * kMaxG + q] = cut.ok ? glo[q] : -__builtin_inff();
        a.vhi[r * kMaxG + q] = cut.ok ? ghi[q] : __builtin_inff();
      }
      a.H[r] = cut.H;
      a.rst[r] = cut.ok ? 0 : 1;

    }
  }
  // the sweep's row list (one atomic per wave)
  {
    const bool lst = r < a.n && !skip;
    const unsigned long long m = __ballot(lst);
    int base = 0;
    if (lane == 0 && m) base = atomicAdd(a.rows_count, __popcll(m));
    base = __shfl(base, 0, 64);
    if (lst) a.rows[base + __popcll(m & ((1ull << lane) - 1ull))] = (int)r;
  }
  if (__ballot(skip || nfs > 0) != 0ull) {
    // the rows' fired pairs: canonical dots 16 at a time (4 per 16-lane
    // group, the rows' X just read), then one lane per pair
    int incl = nfs;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int v = __shfl_up(incl, o, 64);
      if (lane >= o) incl += v;
    }
    const int tot = __shfl(incl, 63, 64);
    for (int e = 0; e < nfs; ++e) fpair[wave][incl - nfs + e] = ((uint32_t)lane << 16) | (fire[e] & 0x3FFFu);
    if (skip || nfs > 0) sbest[threadIdx.x] = pack_best(t, a.tie, g, l);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll 1
    for (int base = 0; base < tot; base += 16) {
      const float* xp[B];
      const float* cp_[B];
#pragma unroll
      for (int b = 0; b < B; ++b) {
        const int e = base + 4 * b + q4;
        const uint32_t pr = e < tot ? fpair[wave][e] : fpair[wave][0];
        xp[b] = a.X + (size_t)(rb + (pr >> 16)) * a.ldx;
        cp_[b] = a.C + (size_t)(pr & 0xFFFFu) * a.d;
      }
      float sv[B];
      canon_dot_batch<KU, B>(xp, cp_, a.d, c16, sv);
      if (c16 == 0) {
#pragma unroll
        for (int b = 0; b < B; ++b) {
          const int e = base + 4 * b + q4;
          if (e < tot) fip[wave][e] = sv[b];
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // a fired pair: its exact hazard (canonical inner product) certifies it
    // far - P(D~ <= thr) <= pibar <= 1 - exp(-H_row) - and it is thinned
    // (the thinning word of the stream's fire block, the exact branch), or
    // it is sampled in full (ipe16_near_kernel's rule for a fired near pair;
    // a band-far pair is certified by construction)
    for (int e = lane; e < tot; e += 64) {
      const uint32_t pr = fpair[wave][e];
      const int ln = (int)(pr >> 16), j = (int)(pr & 0xFFFFu);
      const long long rr = rb + ln;
      const long long gg = a.row_offset + rr;
      const float ip = fip[wave][e];
      const float nx2 = a.xn[rr], ny2 = a.cn[j];
      const float tt = s_t[wave * 64 + ln];
      uint32_t hq = 0;
      float pbar = 1.0f;
      const bool ok = ipe_hazard(ip, nx2, ny2, ipe_sthr(tt), a.sc, hq, pbar);
      const int h = (a.Q + 1) / 2;
      const double pib = ok ? binom_upper_tail((double)pbar, a.Q, h) * (1.0 + 1e-12) : 1.0;
      const double beff = -expm1(-(double)s_H[wave * 64 + ln]);
      float dt = __builtin_inff();
      if (ok && pib <= beff) {
        WordStream ws(a.skey, (unsigned long long)gg * 32ull + (unsigned long long)(j & 31));
        ws.b = (uint32_t)(2 + 2 * (j >> 5));
        (void)ws.next();
        (void)ws.next();
        const uint32_t w2 = ws.next(), w3 = ws.next();
        const double u = u53(w2, w3) * beff;
        if (u < pib) {
          ++st_exact;
          dt = ipe_pruned_exact((double)ip, (double)nx2 + (double)ny2, a.eps, a.Q, tt, u, ws);
        }
      } else {
        ++st_full;
        dt = ipe_distance(ip, (double)nx2, (double)ny2, a.eps, a.Q, a.key,
                          (unsigned long long)gg * (unsigned long long)a.k + (unsigned long long)j);
      }
      if (dt < __builtin_inff()) atomicMin(&sbest[wave * 64 + ln], pack_best(dt, a.tie, gg, j));
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (skip) {
      const unsigned long long bb = sbest[threadIdx.x];
      const int lab = (int)(bb & 0x3FFFu);
      a.labels[r] = lab;
      a.mind[r] = __uint_as_float((uint32_t)(bb >> 32));
      a.rflag[r] = 2;
      // the bound for the next step (relative to this label): the hint
      // joins the non-label set when the label moved
      a.lb[r] = lab == l ? lbe_f : fminf(lbe_f, dh_lo);
    } else if (nfs > 0) {
      // the near kernel merges the sweep's near pairs into this
      a.best[r] = sbest[threadIdx.x];
    }
  }
  if (a.stats) {
    uint32_t f = st_flag, dn = st_dense, sk = st_skip, ex = st_exact, fu = st_full;
    uint32_t nfired = (uint32_t)nfs;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      f += (uint32_t)__shfl_xor((int)f, o, 64);
      dn += (uint32_t)__shfl_xor((int)dn, o, 64);
      sk += (uint32_t)__shfl_xor((int)sk, o, 64);
      ex += (uint32_t)__shfl_xor((int)ex, o, 64);
      fu += (uint32_t)__shfl_xor((int)fu, o, 64);
      nfired += (uint32_t)__shfl_xor((int)nfired, o, 64);
    }
    if (lane == 0) {
      atomicAdd(a.stats + 4, (unsigned long long)f);
      atomicAdd(a.stats + 5, (unsigned long long)dn);
      if (sk) atomicAdd(a.stats + 7, (unsigned long long)sk);
      if (ex) atomicAdd(a.stats + 2, (unsigned long long)ex);
      if (fu) atomicAdd(a.stats + 6, (unsigned long long)fu);
      if (nfired) atomicAdd(a.stats + 1, (unsigned long long)nfired);
    }
  }
}

// ------------------------------------------------------------------ pair certificate
// A pair the row's group band flags near may still be provably far: its own
// S = |x|^2 + |c|^2 (not the group's range) and the inner-product interval
// the fp16 value v = alpha^2 (|c|^2 - 2 x.c) +- E gives.  With ip_c the
// canonical fp32 inner product (the law's), 2 ip_c lies in cv +- w,
// cv = |c|^2 - v / alpha^2, w = (d + 2) u |c|^2 (fp32 |c|^2) + E / alpha^2
// (fp16 filter) + d u S (canonical dot) + the fp32 roundings here; so the
// law's D = S - 2 ip_c >= S - cv - w and ipe_hazard's bin distance
// m >= (sqrt(D_lo) (1 - 2^-11) - sthr) sqrt(S) kq / max(1, |ip|_max).  When
// that is >= m_t (the row's band hazard: pu(m) <= pu(m_t) <= 1 - exp(-H))
// and a = D / 2S stays inside ipe_hazard's range over the whole interval,
// the pair's P(D~ <= thr) is covered by its stream's budget exactly like a
// band-far pair's: it is not listed (a fire on it stays a plain fired pair,
// thinned with its exact hazard by the near kernel).
struct CertParams {
  float inv_a2;   // 1 / alpha^2 (a power of two)
  float kq;       // IpeScreen::kq
  float mt;       // m_t of the band hazard
  float smax;     // IpeScreen::smax
  float du;       // d 2^-24
};

SQ_DEV bool cert_far(float v, float ny2, float nx2, float sthr, float ea2, const CertParams& p) {
  constexpr float u = 5.9604645e-8f;   // 2^-24
  const float S = nx2 + ny2;
  const float vs = v * p.inv_a2;
  const float cv = ny2 - vs;
  const float w = (p.du * (ny2 + S) + 2.0f * u * ny2 + ea2 + 4.0f * u * (fabsf(ny2) + fabsf(vs))) *
                  1.001f;
  const float Dlo = (S - cv - w) - 4.0f * u * (S + fabsf(cv) + w);
  const float Dhi = (S - cv + w) + 4.0f * u * (S + fabsf(cv) + w);
  const float aip = fmaxf(1.0f, 0.5f * (fabsf(cv) + w) * 1.0001f);
  // (v_sqrt_f32: 1 ulp, inside the 1e-5 factors; m >= m_t as a product)
  const float rS = __builtin_amdgcn_sqrtf(S);
  const float num = __builtin_amdgcn_sqrtf(fmaxf(Dlo, 0.0f)) * ((1.0f - 4.8828125e-4f) * (1.0f - 1e-5f)) -
                    sthr;
  const float kt = 1.571f * sthr;
  return (Dlo >= S * (2.44140625e-4f * 1.0001f)) & (Dhi <= S * (1.998046875f * 0.9999f)) &
         (num > 0.0f) & (num * rS * p.kq * (1.0f - 1e-5f) >= p.mt * 1.0001f * aip) &
         (fmaf(kt, rS * p.kq * 1.00001f, 2.2f) <= 1048576.0f * 0.9999f) & (S < p.smax * 0.9999f);
}

// ------------------------------------------------------------------ sweep
// estep_x64's sweep (persistent workgroups of 4 waves x 2 row sets x 32
// rows, the wave's fp16 A fragments resident in VGPRs, 64-centroid tiles
// through a 3-slot LDS ring by LDS-DMA with counted vmcnt) with an IPE
// epilogue.  Register i of a lane (half, r32) holds row (i & 3) + 8 (i >> 2)
// + 4 half of its row set, column 64 t + 32 h + r32.
//  ARGMIN: hint = approximate argmin of v (packed (t, h, r32) in the low
//          14 mantissa bits; any hint is exact for the law);
//  screen: far iff med3(v, vlo, vhi) == v; near pairs -> the row's LDS list.
struct SweepArgs {
  const _Float16* Xh;       // [n][d_pad] fp16(alpha x)
  const _Float16* C;        // estep_x64 operand (hi region used)
  const float* vlo;
  const float* vhi;
  const unsigned char* rst;
  const uint16_t* rfire;    // prep's fired pairs per row
  const int* perm;          // operand column (sorted by |c|^2) -> centroid id
  int G;
  int gb[3];                 // first tile of groups 1..3 (n_tiles: none)
  const int* hj;            // hints (prep's)
  int* hint_out;            // ARGMIN output
  unsigned long long* list; // (row << 16) | j | fired << 15
  int* list_count;
  long long* dense_rows;
  int* dense_count;
  unsigned char* rflag;     // 1: dense (fallback), written per row
  long long n;
  int k, k_pad;
  long long row_offset;
  unsigned long long* stats;
  // list mode (screen): the rows prep left to the sweep, positions [0, *rows_count)
  const int* rows;
  const int* rows_count;
  // bound upkeep (screen, lb given): lb[r] <- sqrt of min over the row's far
  // values v / alpha^2 + lbo[r] (a lower bound on D of every far pair); the
  // near kernel folds in the listed pairs, finalize the hint
  float* lb;
  const float* lbo;
  double inv_a2;
  // the pair certificate of near-flagged pairs (cert_far)
  const float* cns;         // [k_pad] fp32 |c|^2 (the law's) by operand column
  const float* xn;          // [n] fp32 |x|^2
  const float* thr;         // [n] the hint's estimate
  const float* ea2;         // [n] E / alpha^2 (rounded up)
  CertParams cert;
  // wide rows (GV): the pass values of every position, [n][k_pad] in the
  // accumulator layout, from ipe16_values_kernel (the same MFMA sequence)
  const float* V;
};

template <int KSD, bool ARGMIN, bool LB, bool GV = false>
__global__ void __launch_bounds__(kNW * 64) ipe16_sweep_kernel(SweepArgs a) {
  constexpr int KT = KSD + 1;                 // data k-steps + the norm step
  constexpr int SLOT = KT * 2048;
  constexpr int TILE_STRIDE = (2 * KSD + 1) * 2048;
  constexpr int PIECES = SLOT / 1024;
  constexpr int PPW = (PIECES + kNW - 1) / kNW;
  constexpr int DX = KSD * 16;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  auto buf = [&](int g) -> unsigned char* { return smem + (g % kRing) * SLOT; };
  uint16_t* nl = reinterpret_cast<uint16_t*>(smem + (GV ? 0 : kRing * SLOT));   // [kRows][kNLS]
  int* ncnt = reinterpret_cast<int*>(nl + kRows * kNLS);                  // [kRows]
  int* shint = ncnt + kRows;                                              // [kRows]
  float* sband = reinterpret_cast<float*>(shint + kRows);                 // [kRows][G][2]
  float* sfm = sband + kRows * kMaxG * 2;                                 // [kRows]
  float* s_nx2 = sfm + kRows;                                             // [kRows]
  float* s_sthr = s_nx2 + kRows;                                          // [kRows]
  float* s_ea2 = s_sthr + kRows;                                          // [kRows]
  float* s_lbo = s_ea2 + kRows;                                           // [kRows]
  int* s_rr = reinterpret_cast<int*>(s_lbo + kRows);                      // [kRows] row | rst << 31

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r32 = lane & 31;
  const int half = lane >> 5;
  // positions [0, n): rows 0.. n - 1, or list entries (screen in list mode)
  const long long n = a.rows ? (long long)*a.rows_count : a.n;
  auto R = [&](long long p) -> long long { return a.rows ? (long long)a.rows[p] : p; };
  const int n_tiles = a.k_pad / kTileN;
  const long long nblk = (n + kRows - 1) / kRows;
  long long blk = blockIdx.x;
  if (blk >= nblk) return;
  int qbits = 1;
  while ((1 << qbits) < 2 * n_tiles) ++qbits;
  const uint32_t keep = ~((1u << (qbits + 5)) - 1u);

  auto stage = [&](int U) {
    if constexpr (GV) return;
    const int t = U % n_tiles;
    const unsigned char* tile = reinterpret_cast<const unsigned char*>(a.C) + (size_t)t * TILE_STRIDE;
    unsigned char* dst = buf(U);
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int p = wave + kNW * i < PIECES ? wave + kNW * i : PIECES - 1;
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(tile + p * 1024 + lane * 16),
          (__attribute__((address_space(3))) void*)(dst + p * 1024), 16, 0, 0);
    }
  };
  auto sync_tile = [&]() {
    if constexpr (GV) return;
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PPW) : "memory");
    __builtin_amdgcn_s_barrier();
  };
  // rows of the block: set st of wave w, row rl of the set's 32
  auto row_of = [&](long long b, int st, int rl) -> long long {
    return b * kRows + (wave * kRS + st) * 32 + rl;
  };
  f16x8 ah[kRS][KSD];
  auto load_a = [&](long long b) {
    if constexpr (GV) return;
#pragma unroll
    for (int st = 0; st < kRS; ++st) {
      long long r = row_of(b, st, r32);
      r = R(r < n ? r : n - 1);
      const _Float16* xr = a.Xh + (size_t)r * DX + half * 8;
#pragma unroll
      for (int ks = 0; ks < KSD; ++ks) ah[st][ks] = *reinterpret_cast<const f16x8*>(xr + ks * 16);
    }
  };
  f16x8 aug = (f16x8)0;
  if (half == 0) { aug[0] = aug[1] = aug[2] = (_Float16)1.0f; }
  const int lane_off = (half * 64 + r32) * 16;
  auto frag = [&](const unsigned char* cur, int g) -> f16x8 {
    return *reinterpret_cast<const f16x8*>(cur + lane_off + (g / KT) * 512 + (g % KT) * 2048);
  };
  // per-lane state: the 16 rows' band edges per set (screen) / running
  // packed minima (argmin); the near bits of the last epilogue
  // lower band edge per register (row); the upper edge per row set: the
  // smallest of the lane half's 16 rows (a row with a higher edge flags a
  // few more pairs, which the pair certificate then clears) - 30 VGPRs for
  // the bound upkeep
  float lo[kRS][16], hi[kRS];
  // (screen, LB) per register the minimum far value: the row's bound upkeep
  float fm[kRS][LB ? 16 : 1];
  // near bits of the last epilogue (bit 16 st + i: register (st, i)); rows
  // whose list is full are muted (dense: no more pushes from this lane)
  uint32_t nb = 0, mute = 0;
  auto rl_of = [&](int i) { return (i & 3) + 8 * (i >> 2) + 4 * half; };
  // one value of the previous half-tile (o), half-tile index q = 2 t + h
  auto epi = [&](int st, int i, float v, uint32_t q) {
    if constexpr (ARGMIN) {
      lo[st][i] = vmin(lo[st][i], and_or(v, keep, (q << 5) | (uint32_t)r32));
    } else {
      const bool far = (v >= lo[st][i]) & (v <= hi[st]);
      nb |= far ? 0u : (1u << (16 * st + i));
      if constexpr (LB && !(SQ_IPE16_DIAG & 32)) fm[st][i] = vmin(fm[st][i], far ? v : __builtin_inff());
    }
  };
  typedef f32x16 Acc[kRS];
  constexpr int PFD = 2, NB = PFD + 1;
  f16x8 bq[NB];
  auto pass = [&](auto H_, const unsigned char* cur, Acc& acc, const Acc& o, uint32_t qo,
                  bool do_epi) {
    constexpr int h = decltype(H_)::value;
    if constexpr (GV) {
      // this half-tile's values (half-tile index qo + 1) of the block's rows,
      // then the previous half-tile's epilogue
      const int col = 32 * (int)(qo + 1u) + r32;
#pragma unroll
      for (int st = 0; st < kRS; ++st)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          long long p = row_of(blk, st, rl_of(i));
          p = p < n ? p : n - 1;
          acc[st][i] = a.V[(size_t)p * a.k_pad + col];
        }
      if (do_epi) {
#pragma unroll
        for (int e = 0; e < 16 * kRS; ++e) epi(e / 16, e % 16, o[e / 16][e % 16], qo);
      }
      return;
    }
#pragma unroll
    for (int st = 0; st < kRS; ++st) acc[st] = (f32x16){0};
#pragma unroll
    for (int ks = 0; ks < KT; ++ks) {
      const int g = h * KT + ks;
      if (g + PFD < 2 * KT) bq[(g + PFD) % NB] = frag(cur, g + PFD);
#pragma unroll
      for (int st = 0; st < kRS; ++st)
        acc[st] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ks < KSD ? ah[st][ks] : aug, bq[g % NB],
                                                         acc[st], 0, 0, 0);
      if (do_epi) {
#pragma unroll
        for (int e = (ks * 16 * kRS) / KT; e < ((ks + 1) * 16 * kRS) / KT; ++e)
          epi(e / 16, e % 16, o[e / 16][e % 16], qo);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  // near pairs of the half-tile just screened (operand column jp): each lane
  // walks its set bits (the hint, co-located centroids, padding)
  // (o: the accumulators of that half-tile, still live; jc / ny2: its
  // lane column's centroid and |c|^2, loaded a tile ahead - a global load
  // here would wait for the in-flight tile DMA as well)
  auto flush_near = [&](long long b, int jc, float ny2, const Acc& o) {
    if constexpr (!ARGMIN) {
      if (SQ_IPE16_DIAG & 16) nb = 0;
      nb &= ~mute;
      if (__ballot(nb != 0u) != 0ull) {
#pragma unroll
        for (int st = 0; st < kRS; ++st) {
          uint32_t m = (nb >> (16 * st)) & 0xFFFFu;
          while (m) {
            const int i = __builtin_ctz(m);
            m &= m - 1u;
            const int rb = (wave * kRS + st) * 32 + rl_of(i);
            if (jc >= 0 && jc != shint[rb] && row_of(b, st, rl_of(i)) < n) {
              // the flagged value: a branch-free select of register i
              float v = o[st][0];
#pragma unroll
              for (int e = 1; e < 16; ++e) v = i == e ? o[st][e] : v;
              if (!cert_far(v, ny2, s_nx2[rb], s_sthr[rb], s_ea2[rb], a.cert)) {
                const int s = atomicAdd(&ncnt[rb], 1);
                if (s < kCapR) nl[rb * kNLS + s] = (uint16_t)(jc | 0x4000);
                else mute |= 1u << (16 * st + i);   // the row is dense
              }
            }
          }
        }
      }
      nb = 0;
    }
  };

  // the lane's 32 rows' band edges of centroid group q.  A row without a
  // band in a group wider than one tile is dense right away (muted, its count
  // past the cap): certifying 64+ pairs per tile would only delay that (the
  // first steps after a random init); in a one-tile group - the DP
  // grouping's outlying norms - its pairs go through the certificate
  auto load_bands = [&](int q) {
    if constexpr (!ARGMIN) {
      const int qs = q == 0 ? 0 : a.gb[q - 1];
      const int qe = q == 3 ? n_tiles : (a.gb[q] < n_tiles ? a.gb[q] : n_tiles);
      const bool wide = qe - qs > 1;
#pragma unroll
      for (int st = 0; st < kRS; ++st)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int rb = (wave * kRS + st) * 32 + rl_of(i);
          const int e = rb * kMaxG + q;
          lo[st][i] = sband[2 * e];
          hi[st] = i == 0 ? sband[2 * e + 1] : fminf(hi[st], sband[2 * e + 1]);
          if (wide && lo[st][i] == __builtin_inff()) {
            mute |= 1u << (16 * st + i);
            ncnt[rb] = kCapR + 1;
          }
        }
    }
  };
  auto group_of = [&](int t) { return (t >= a.gb[0]) + (t >= a.gb[1]) + (t >= a.gb[2]); };

  int U = 0;
  if constexpr (!GV) {
    stage(0);
    stage(1);
    load_a(blk);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }

  for (; blk < nblk; blk += gridDim.x) {
    // ---- block prologue: the rows' band edges, hints, listed fires
    if constexpr (ARGMIN) {
#pragma unroll
      for (int st = 0; st < kRS; ++st)
#pragma unroll
        for (int i = 0; i < 16; ++i) lo[st][i] = __builtin_inff();
    } else {
      mute = 0;
      if constexpr (LB) {
#pragma unroll
        for (int st = 0; st < kRS; ++st)
#pragma unroll
          for (int i = 0; i < 16; ++i) fm[st][i] = __builtin_inff();
      }
      // the rows' hints, norms, thresholds and bands (thread t: row t; a
      // row past n: all far).  The row id first, then every load of the row
      // in flight together (one wait instead of one per load); prep
      // finishes the fires, so the lists start empty
      static_assert(kRows == kNW * 64, "one row per thread");
      {
        const int t = tid;
        const long long p = blk * kRows + t;
        const bool pv = p < n;
        const long long r = pv ? R(p) : 0;
        const int hj = a.hj[r];
        const float xn = a.xn[r], th = a.thr[r], e2 = a.ea2[r];
        const unsigned char rs = a.rst[r];
        const float lo_r = (LB && a.lb) ? a.lbo[r] : 0.0f;
        float blo[kMaxG], bhi[kMaxG];
#pragma unroll
        for (int q = 0; q < kMaxG; ++q) {
          const bool v = pv && q < a.G;
          blo[q] = v ? a.vlo[r * kMaxG + q] : -__builtin_inff();
          bhi[q] = v ? a.vhi[r * kMaxG + q] : __builtin_inff();
        }
        shint[t] = pv ? hj : -1;
        s_nx2[t] = xn;
        s_sthr[t] = ipe_sthr(th);
        s_ea2[t] = e2;
        s_lbo[t] = lo_r;
        s_rr[t] = (int)r | (rs != 0 ? (int)0x80000000u : 0);
        ncnt[t] = 0;
#pragma unroll
        for (int q = 0; q < kMaxG; ++q) {
          sband[2 * (t * kMaxG + q)] = blo[q];
          sband[2 * (t * kMaxG + q) + 1] = bhi[q];
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      load_bands(0);
    }
    // ---- the sweep: half 0 of tile t (epilogue of tile t - 1's half 1),
    // half 1 (epilogue of half 0), one ring slot per tile
    f32x16 cA[kRS], cB[kRS];
    // the lane columns' centroids / norms of the two flushes of a tile
    auto colc = [&](int jp, int& jc, float& ny2) {
      if constexpr (!ARGMIN) {
        jc = jp < a.k ? a.perm[jp] : -1;
        ny2 = a.cns[jp];
      }
    };
    int jcA = -1, jcB = -1;
    float nyA = 0.0f, nyB = 0.0f;
    for (int t = 0; t < n_tiles; ++t) {
      if (t > 0) colc(64 * (t - 1) + 32 + r32, jcA, nyA);
      colc(64 * t + r32, jcB, nyB);
      stage(U + kRing - 1);
      if constexpr (!GV) {
#pragma unroll
        for (int j = 0; j < PFD; ++j) bq[j] = frag(buf(U), j);
      }
      pass(std::integral_constant<int, 0>{}, buf(U), cA, cB, (uint32_t)(2 * t - 1), t > 0);
      flush_near(blk, jcA, nyA, cB);
      // tile t's values (epilogues from the next pass on) use its group's bands
      if (t > 0 && group_of(t) != group_of(t - 1)) load_bands(group_of(t));
      pass(std::integral_constant<int, 1>{}, buf(U), cB, cA, (uint32_t)(2 * t), true);
      flush_near(blk, jcB, nyB, cA);
      sync_tile();
      ++U;
    }
    colc(64 * (n_tiles - 1) + 32 + r32, jcA, nyA);
    load_a(blk + gridDim.x);   // clamped rows: unconditional
#pragma unroll
    for (int st = 0; st < kRS; ++st)
#pragma unroll
      for (int i = 0; i < 16; ++i) epi(st, i, cB[st][i], (uint32_t)(2 * n_tiles - 1));
    flush_near(blk, jcA, nyA, cB);

    if constexpr (ARGMIN) {
      // row minimum over the 32 lanes of each half: the packed value holds
      // the tile-half index and the lane column
#pragma unroll
      for (int st = 0; st < kRS; ++st)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          float v = lo[st][i];
#pragma unroll
          for (int o = 1; o < 32; o <<= 1) v = vmin(v, __shfl_xor(v, o, 64));
          if (r32 == i) {
            const long long r = row_of(blk, st, rl_of(i));
            if (r < n) {
              const uint32_t p = __float_as_uint(v);
              const uint32_t q = (p >> 5) & ((1u << qbits) - 1u);
              const int j = (int)((q >> 1) * kTileN + (q & 1u) * 32u + (p & 31u));
              a.hint_out[r] = a.perm[j < a.k ? j : 0];
            }
          }
        }
    } else {
      // the rows' minimum far values (over the 32 columns of a half)
      if constexpr (LB) {
#pragma unroll
        for (int st = 0; st < kRS; ++st)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            float v = fm[st][i];
#pragma unroll
            for (int o = 1; o < 32; o <<= 1) v = vmin(v, __shfl_xor(v, o, 64));
            if (r32 == i) sfm[(wave * kRS + st) * 32 + rl_of(i)] = v;
          }
      }
      // ---- flush the block's lists: dedupe fires against near pairs and the
      // hint, dense rows to the fallback list, the rest compacted to the
      // global pair list (one atomic per wave)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      const int t = tid;   // kRows == 256 threads: one row each
      const long long p = blk * kRows + t;
      const int rrw = s_rr[t];   // (the prologue's row id and dense flag)
      const long long r = p < n ? (long long)(rrw & 0x7FFFFFFF) : 0;
      int c = 0;
      bool dense = false;
      uint16_t* row_l = nl + t * kNLS;
      if (p < n) {
        c = ncnt[t];
        dense = c > kCapR || rrw < 0;
        if (dense) {
          c = 0;
        } else {
          // a fire on the hint is void; a fire on a near pair is merged into
          // its entry (bit 15): the near kernel decides from the pair's exact
          // hazard whether it is sampled in full or treated as far
          const int hj = shint[t];
          int w = 0;
          for (int e = 0; e < c; ++e) {
            const uint16_t v = row_l[e];
            bool drop = false;
            if (v & 0x8000) {
              const int j = v & 0x3FFF;
              drop = j == hj;
              for (int f = 0; f < c && !drop; ++f)
                if (row_l[f] == (uint16_t)(j | 0x4000)) {
                  row_l[f] = (uint16_t)(j | 0xC000);
                  drop = true;
                }
            }
            if (!drop) row_l[w++] = v;
          }
          c = w;
        }
        a.rflag[r] = dense ? 1 : 0;
        if (LB && a.lb) {
          // far pairs: exact D >= v / alpha^2 + x2lo - E / alpha^2 (lbo);
          // a dense row (fallback) keeps no bound
          const float fmv = sfm[t];
          float lbv = 0.0f;
          if (!dense) {
            const double D = (double)fmv * a.inv_a2 + (double)s_lbo[t];
            lbv = fmv == __builtin_inff() ? fmv : (D > 0.0 ? f32_dn(sqrt(D) * (1.0 - 1e-12)) : 0.0f);
          }
          a.lb[r] = lbv;
        }
      }
      // wave scan of the counts
      int incl = c;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int v = __shfl_up(incl, o, 64);
        if (lane >= o) incl += v;
      }
      const int wtot = __shfl(incl, 63, 64);
      int base = 0;
      if (lane == 63 && wtot > 0) base = atomicAdd(a.list_count, wtot);
      base = __shfl(base, 63, 64);
      const unsigned long long rr = (unsigned long long)r << 16;
      for (int e = 0; e < c; ++e) a.list[base + incl - c + e] = rr | (unsigned long long)row_l[e];
      const unsigned long long dm = __ballot(dense);
      if (dm) {
        int db = 0;
        if (lane == 0) db = atomicAdd(a.dense_count, __popcll(dm));
        db = __shfl(db, 0, 64);
        if (dense) a.dense_rows[db + __popcll(dm & ((1ull << lane) - 1ull))] = r;
      }
      if (a.stats) {
        uint32_t nfire = 0, nnear = 0;
        for (int e = 0; e < c; ++e) {
          if (row_l[e] & 0x4000) ++nnear; else ++nfire;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
          nfire += (uint32_t)__shfl_xor((int)nfire, o, 64);
          nnear += (uint32_t)__shfl_xor((int)nnear, o, 64);
        }
        if (lane == 0) {
          atomicAdd(a.stats + 0, (unsigned long long)nnear);
          atomicAdd(a.stats + 1, (unsigned long long)nfire);
          atomicAdd(a.stats + 3, (unsigned long long)__popcll(dm));
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ------------------------------------------------------------------ values
// Wide rows (d_pad > 256: the A fragments of a row set no longer fit in
// VGPRs next to the sweep's epilogue state): the sweep's pass values are
// computed here first - per wave 32 positions x one 64-centroid tile, the
// SAME operands in the same k-step order through the same MFMA from zero, so
// every value equals the resident-fragment sweep's bit for bit - and the
// GV sweep reads them instead of running its MFMAs.  V [n][k_pad] fp32, in
// the accumulator layout (register i of lane (half, r32): row (i & 3) +
// 8 (i >> 2) + 4 half of the wave's 32, column 64 t + 32 h + r32).
struct ValuesArgs {
  const _Float16* Xh;
  const _Float16* C;
  const int* rows;          // list mode: positions -> rows
  const int* rows_count;
  long long n;              // positions (upper bound in list mode)
  int ksd, k_pad;
  float* V;
};
__global__ void __launch_bounds__(256) ipe16_values_kernel(ValuesArgs a) {
  const long long n = a.rows ? (long long)*a.rows_count : a.n;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r32 = lane & 31, half = lane >> 5;
  const long long p0 = ((long long)blockIdx.x * 4 + wave) * 32;
  if (p0 >= n) return;
  const int t = blockIdx.y;
  const long long p = p0 + r32 < n ? p0 + r32 : n - 1;
  const long long r = a.rows ? (long long)a.rows[p] : p;
  const int KT = a.ksd + 1;
  const _Float16* xr = a.Xh + (size_t)r * (a.ksd * 16) + half * 8;
  const unsigned char* tile = reinterpret_cast<const unsigned char*>(a.C) +
                              (size_t)t * (2 * a.ksd + 1) * 2048 + (half * 64 + r32) * 16;
  f16x8 aug = (f16x8)0;
  if (half == 0) { aug[0] = aug[1] = aug[2] = (_Float16)1.0f; }
  f32x16 c0 = (f32x16){0}, c1 = (f32x16){0};
  for (int ks = 0; ks < KT; ++ks) {
    const f16x8 av = ks < a.ksd ? *reinterpret_cast<const f16x8*>(xr + ks * 16) : aug;
    const f16x8 b0 = *reinterpret_cast<const f16x8*>(tile + ks * 2048);
    const f16x8 b1 = *reinterpret_cast<const f16x8*>(tile + 512 + ks * 2048);
    c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(av, b0, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(av, b1, c1, 0, 0, 0);
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const long long q = p0 + (i & 3) + 8 * (i >> 2) + 4 * half;
    if (q < n) {
      float* vr = a.V + (size_t)q * a.k_pad + 64 * t + r32;
      vr[0] = c0[i];
      vr[32] = c1[i];
    }
  }
}

// ------------------------------------------------------------------ near
// The listed pairs: 16 lanes per canonical dot (4 pairs at a time per wave,
// 64 per round), then one lane per pair samples and merges.
struct NearArgs {
  const unsigned long long* list;
  const int* list_count;
  const float* X;
  long long ldx;
  const float* C;
  const float* xn;
  const float* cn;
  const float* thr;
  const float* H;
  unsigned long long* best;
  int d, k;
  double eps;
  int Q;
  RngKey key, tie, skey;
  long long row_offset;
  IpeScreen sc;
  unsigned long long* stats;
  float* lb;                // bound upkeep: every listed pair is a non-hint pair
};

template <int KU>
__global__ void __launch_bounds__(256) ipe16_near_kernel(NearArgs a) {
  __shared__ float sip[256];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c16 = lane & 15, q4 = lane >> 4;
  const long long cnt = *a.list_count;
  uint32_t st_exact = 0, st_full = 0;
  for (long long base = ((long long)blockIdx.x * 4 + wave) * 64; base < cnt;
       base += (long long)gridDim.x * 256) {
    constexpr int B = 4;
#pragma unroll 1
    for (int g = 0; g < 4; ++g) {
      const float* xp[B];
      const float* cp_[B];
#pragma unroll
      for (int b = 0; b < B; ++b) {
        const long long e = base + 16 * g + 4 * b + q4;
        long long r = 0;
        int j = 0;
        if (e < cnt) {
          const unsigned long long ent = a.list[e];
          r = (long long)(ent >> 16);
          j = (int)(ent & 0x3FFFu);
        }
        xp[b] = a.X + (size_t)r * a.ldx;
        cp_[b] = a.C + (size_t)j * a.d;
      }
      float sv[B];
      canon_dot_batch<KU, B>(xp, cp_, a.d, c16, sv);
      if (c16 == 0) {
#pragma unroll
        for (int b = 0; b < B; ++b) sip[wave * 64 + 16 * g + 4 * b + q4] = sv[b];
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const long long e = base + lane;
    if (e < cnt) {
      const unsigned long long ent = a.list[e];
      const long long r = (long long)(ent >> 16);
      const int j = (int)(ent & 0x3FFFu);
      const bool fired = (ent & 0x8000u) != 0;
      const bool near = (ent & 0x4000u) != 0;
      const long long g = a.row_offset + r;
      const float ip = sip[threadIdx.x];
      const float nx2 = a.xn[r], ny2 = a.cn[j];
      const float t = a.thr[r];
      float dt = __builtin_inff();
      if (a.lb) atomicMin(reinterpret_cast<unsigned int*>(a.lb + r),
                          __float_as_uint(pair_dist_lo(ip, nx2, ny2, a.d)));
      // the pair's exact hazard (canonical inner product): a near pair the
      // row's band could not certify may still be far - ipe_hazard passes and
      // its bound P(D~ <= thr) <= pibar <= 1 - exp(-H_row) - and then it is a
      // far pair of its stream like the others (fired: thinned; else nothing)
      uint32_t hq = 0;
      float pbar = 1.0f;
      const bool ok = ipe_hazard(ip, nx2, ny2, ipe_sthr(t), a.sc, hq, pbar);
      const int h = (a.Q + 1) / 2;
      const double pib = ok ? binom_upper_tail((double)pbar, a.Q, h) * (1.0 + 1e-12) : 1.0;
      const double beff = -expm1(-(double)a.H[r]);
      const bool far = !near || (ok && pib <= beff);
      if (!far) {
        ++st_full;
        dt = ipe_distance(ip, (double)nx2, (double)ny2, a.eps, a.Q, a.key,
                          (unsigned long long)g * (unsigned long long)a.k + (unsigned long long)j);
      } else if (fired) {
        WordStream ws(a.skey, (unsigned long long)g * 32ull + (unsigned long long)(j & 31));
        ws.b = (uint32_t)(2 + 2 * (j >> 5));
        (void)ws.next();
        (void)ws.next();                     // words 0, 1: the stream's next budget (prep)
        const uint32_t w2 = ws.next(), w3 = ws.next();
        const double u = u53(w2, w3) * beff;
        if (u < pib) {
          ++st_exact;
          dt = ipe_pruned_exact((double)ip, (double)nx2 + (double)ny2, a.eps, a.Q, t, u, ws);
        }
      }
      if (dt < __builtin_inff()) atomicMin(a.best + r, pack_best(dt, a.tie, g, j));
    }
    __builtin_amdgcn_wave_barrier();
  }
  if (a.stats) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      st_exact += (uint32_t)__shfl_xor((int)st_exact, o, 64);
      st_full += (uint32_t)__shfl_xor((int)st_full, o, 64);
    }
    if (lane == 0 && st_exact) atomicAdd(a.stats + 2, (unsigned long long)st_exact);
    if (lane == 0 && st_full) atomicAdd(a.stats + 6, (unsigned long long)st_full);
  }
}

// labels / mind of the rows the screen resolved (dense rows: the fallback)
// (skipped rows: prep's own; lb given: a row whose label left its hint
// adds the hint pair to its non-label bound)
__global__ void __launch_bounds__(256) ipe16_finalize_kernel(const unsigned long long* best,
                                                            const unsigned char* rflag,
                                                            int* labels, float* mind,
                                                            long long n, const int* hj, float* lb,
                                                            const float* dhint) {
  const long long r = (long long)blockIdx.x * 256 + threadIdx.x;
  if (r >= n || rflag[r]) return;
  const unsigned long long b = best[r];
  const int lab = (int)(b & 0x3FFFu);
  labels[r] = lab;
  mind[r] = __uint_as_float((uint32_t)(b >> 32));
  if (lb && lab != hj[r]) lb[r] = fminf(lb[r], dhint[r]);
}

// ------------------------------------------------------------------ skip bounds
// The row skip's per-step centroid quantities (ops.kmeans.Ipe16._skip_bounds
// in three launches instead of ~45 small torch ops - each ~8 us of launch
// gap, and each distinct torch kernel 30-130 ms of lazy loading at its first
// use).  G = C C^T (fp64, the caller's GEMM), nrm = |c|^2.
// |c|^2 is G's diagonal, the margin 1e-12 max |c|^2 (each workgroup takes the
// max itself: no host read).
//  1. per centroid a (one workgroup): Dlo / Dhi of every pair from the
//     expansion with its margin (as the torch version), the nearest other
//     centroid nn[a] (Dlo), and a's shift sh[a] since the previous centres;
//  2. one workgroup: the median of nn (bitonic sort in LDS), the wild count
//     W = clamp(#{sh > 0.01 median}, n_wild, k / 2) and tau = the (W+1)-th
//     largest shift -> smax (rounded up);
//  3. per centroid a: mw[a] = min over the wild j != a of Dlo (rounded down),
//     Rc[a][g] = max over norm group g (operand columns) of Dhi (rounded up).
struct BoundsArgs {
  const float* C;
  const float* Cprev;     // nullable: no shifts (first call)
  const double* G;        // [k][k]
  const int* perm;        // operand column -> centroid
  int k, d, Gn, n_wild;
  int gs[4];              // first tile of each group
  double mrel;            // margin / max |c|^2
  double* sh;             // [k] work
  double* nn;             // [k] work
  double* tau;            // [1] work
  int* wild_n;            // [1] out
  float* smax;            // [1] out
  float* mw;              // [k] out
  float* Rc;              // [k][4] out
};
SQ_DEV double sb_d2(const BoundsArgs& a, int i, int j) {
  return (a.G[(size_t)i * (a.k + 1)] + a.G[(size_t)j * (a.k + 1)]) - 2.0 * a.G[(size_t)i * a.k + j];
}
SQ_DEV double sb_lo(double D2, double marg) { return sqrt(fmax(D2 - marg, 0.0)) * (1.0 - 1e-9); }
SQ_DEV double sb_hi(double D2, double marg) { return sqrt(fmax(D2 + marg, 0.0)) * (1.0 + 1e-9); }
SQ_DEV double wave_max_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  return v;
}
// the margin, in every thread of a 256-thread block
SQ_DEV double sb_margin(const BoundsArgs& a, double* red4) {
  double m = 0.0;
  for (int j = threadIdx.x; j < a.k; j += 256) m = fmax(m, a.G[(size_t)j * (a.k + 1)]);
  m = wave_max_d(m);
  if ((threadIdx.x & 63) == 0) red4[threadIdx.x >> 6] = m;
  __syncthreads();
  return a.mrel * fmax(fmax(red4[0], red4[1]), fmax(red4[2], red4[3]));
}
SQ_DEV double wave_min_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o, 64));
  return v;
}
SQ_DEV double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__global__ void __launch_bounds__(256) skip_bounds_rows_kernel(BoundsArgs a) {
  __shared__ double red[3][4];
  const int i = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const double marg = sb_margin(a, red[2]);
  double m = __builtin_inf();
  for (int j = tid; j < a.k; j += 256)
    if (j != i) m = fmin(m, sb_lo(sb_d2(a, i, j), marg));
  double s2 = 0.0;
  if (a.Cprev)
    for (int f = tid; f < a.d; f += 256) {
      const double dd = (double)a.C[(size_t)i * a.d + f] - (double)a.Cprev[(size_t)i * a.d + f];
      s2 += dd * dd;
    }
  m = wave_min_d(m);
  s2 = wave_sum_d(s2);
  if (lane == 0) {
    red[0][wave] = m;
    red[1][wave] = s2;
  }
  __syncthreads();
  if (tid == 0) {
    a.nn[i] = fmin(fmin(red[0][0], red[0][1]), fmin(red[0][2], red[0][3]));
    a.sh[i] = sqrt((red[1][0] + red[1][1]) + (red[1][2] + red[1][3])) * (1.0 + 1e-9);
  }
}
constexpr int kSbMaxK = 4096;
SQ_DEV void lds_bitonic(double* v, int np2) {
  for (int size = 2; size <= np2; size <<= 1)
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      __syncthreads();
      for (int t = threadIdx.x; t < np2 / 2; t += blockDim.x) {
        const int lo = 2 * t - (t & (stride - 1));
        const int hi = lo + stride;
        const bool asc = (lo & size) == 0;
        const double x = v[lo], y = v[hi];
        if ((x > y) == asc) {
          v[lo] = y;
          v[hi] = x;
        }
      }
    }
  __syncthreads();
}
__global__ void __launch_bounds__(1024) skip_bounds_tau_kernel(BoundsArgs a) {
  __shared__ double v[kSbMaxK];
  __shared__ int cnt;
  int np2 = 1;
  while (np2 < a.k) np2 <<= 1;
  for (int j = threadIdx.x; j < np2; j += blockDim.x) v[j] = j < a.k ? a.nn[j] : __builtin_inf();
  if (threadIdx.x == 0) cnt = 0;
  lds_bitonic(v, np2);
  const double tgt = 0.01 * v[(a.k - 1) / 2];
  __syncthreads();
  int c = 0;
  for (int j = threadIdx.x; j < a.k; j += blockDim.x) c += a.sh[j] > tgt ? 1 : 0;
  atomicAdd(&cnt, c);
  // descending shifts: ascending sort of -sh
  for (int j = threadIdx.x; j < np2; j += blockDim.x) v[j] = j < a.k ? -a.sh[j] : __builtin_inf();
  lds_bitonic(v, np2);
  if (threadIdx.x == 0) {
    const int W0 = a.n_wild < a.k ? a.n_wild : a.k;
    int W = cnt;
    W = W < W0 ? W0 : W;
    const int half = a.k / 2 > 1 ? a.k / 2 : 1;
    W = W > half ? half : W;
    W = W > a.k - 1 ? a.k - 1 : W;
    const double t = a.k > W0 ? -v[W] : 0.0;
    a.tau[0] = t;
    a.wild_n[0] = W;
    a.smax[0] = (float)(t * (1.0 + 0x1p-20));
  }
}
__global__ void __launch_bounds__(256) skip_bounds_cols_kernel(BoundsArgs a) {
  __shared__ double red[6][4];
  const int i = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const double marg = sb_margin(a, red[5]);
  const double tau = a.Cprev ? a.tau[0] : __builtin_inf();
  double mw = __builtin_inf();
  double rc[4] = {0.0, 0.0, 0.0, 0.0};
  for (int c = tid; c < a.k; c += 256) {
    const int j = a.perm[c];
    const double D2 = sb_d2(a, i, j);
    if (j != i && a.Cprev && a.sh[j] > tau) mw = fmin(mw, sb_lo(D2, marg));
    const int t = c >> 6;
    const int g = (t >= a.gs[1] && a.Gn > 1) + (t >= a.gs[2] && a.Gn > 2) + (t >= a.gs[3] && a.Gn > 3);
    const double h = sb_hi(D2, marg);
#pragma unroll
    for (int q = 0; q < 4; ++q) rc[q] = q == g ? fmax(rc[q], h) : rc[q];
  }
  mw = wave_min_d(mw);
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) rc[q] = fmax(rc[q], __shfl_xor(rc[q], o, 64));
  if (lane == 0) {
    red[0][wave] = mw;
#pragma unroll
    for (int q = 0; q < 4; ++q) red[1 + q][wave] = rc[q];
  }
  __syncthreads();
  if (tid == 0) {
    const double m = fmin(fmin(red[0][0], red[0][1]), fmin(red[0][2], red[0][3]));
    a.mw[i] = (float)(m * (1.0 - 0x1p-20));
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const double r = fmax(fmax(red[1 + q][0], red[1 + q][1]), fmax(red[1 + q][2], red[1 + q][3]));
      a.Rc[(size_t)i * 4 + q] = q < a.Gn ? (float)(r * (1.0 + 0x1p-20)) : 0.0f;
    }
  }
}

}  // namespace i16
}  // namespace sq

using namespace sq;
using namespace sq::i16;

template <int KSD, bool ARGMIN, bool LB, bool GV = false>
static int launch_sweep(const SweepArgs& a, hipStream_t st) {
  constexpr int SLOT = (KSD + 1) * 2048;
  const size_t lds = (GV ? 0 : kRing * (size_t)SLOT) + (size_t)kRows * kNLS * 2 + 2 * kRows * 4 +
                     (size_t)kRows * kMaxG * 2 * 4 + (size_t)kRows * 6 * 4;
  auto kern = ipe16_sweep_kernel<KSD, ARGMIN, LB, GV>;
  static int attr = 0;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    // the tile ring counts its own vmcnt: a register spill (scratch memory
    // ops between the DMA and its wait) would break that count
    hipFuncAttributes fa;
    attr = (hipFuncGetAttributes(&fa, (const void*)kern) == hipSuccess && fa.localSizeBytes > 0) ? 2 : 1;
  }
  if (attr == 2) return (int)hipErrorNotSupported;
  static int resident = 0;
  if (resident == 0) {
    int dev = 0, cus = 0, per_cu = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)kern, kNW * 64, lds);
    resident = (cus > 0 ? cus : 256) * (per_cu > 0 ? per_cu : 1);
  }
  const long long nblk = (a.n + kRows - 1) / kRows;
  const unsigned grid = (unsigned)(nblk < resident ? nblk : resident);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(kNW * 64), lds, st, a);
  return (int)hipGetLastError();
}

static IpeScreen make_screen(int k, double eps, int Q) {
  IpeScreen sc;
  const int h = (Q + 1) / 2;
  double cq = 1.0;
  for (int i = 0; i < h; ++i) cq = cq * (double)(Q - i) / (double)(i + 1);
  sc.hf = (float)h;
  sc.cqh = (float)(cq * (1.0002 * (1.0 + 1e-6)));
  sc.kq = (float)((1.0 - 3e-6) * (1.0 - 1e-6) / (1.4142135623730951 * eps));
  sc.smax = (float)(6.0e10 * eps * (1.0 - 1e-6));
  sc.cap = (uint32_t)(((k + 63) / 64) * (1u << 23));
  sc.ucap = exp(-(double)sc.cap * 0x1p-32);
  return sc;
}

static RngKey key_at(const long long* ia, int i) {
  return RngKey{(uint32_t)ia[i], (uint32_t)ia[i + 1], (uint32_t)ia[i + 2], (uint32_t)ia[i + 3]};
}

extern "C" {

// One call per phase (op), arguments in host arrays (ia: integers and device
// pointers, da: doubles) so the binding stays one signature:
//   op 0 prep, 1 argmin sweep, 2 screen sweep, 3 near, 4 finalize.
// ia layout (all ops): [0] X, [1] ldx, [2] C fp32, [3] Xh fp16, [4] C_op,
//   [5] hint in, [6] hint out (argmin), [7] xn, [8] cn, [9] thr, [10] hj,
//   [11] vlo, [12] vhi, [13] H, [14] rfire, [15] rst, [16] best, [17] list,
//   [18] list_count, [19] dense_rows, [20] dense_count, [21] rflag,
//   [22] labels, [23] mind, [24] stats, [25] n, [26] d, [27] d_pad, [28] k,
//   [29] k_pad, [30] Q, [31] row_offset, [32..35] key, [36..39] tie,
//   [40..43] skey, [44..47] bkey, [48] perm (operand column -> centroid),
//   [49] group |c|^2 ranges [G][2], [50] G, [51] lb (0: no row skip / bound
//   upkeep), [52] lb valid (skip allowed), [53] smax [1], [54] Rc [k],
//   [55] lbo, [56] dhint, [57] sweep rows, [58] sweep row count, [59] ea2,
//   [60] |c|^2 by operand column [k_pad], [61..63] first tile of groups 1..3,
//   [64] mw [k] (row skip: nearest wild centroid), [65] V (0: the sweep's own
//   MFMAs; required for d_pad > 256), [66] rows of V
// da: [0] eps, [1] alpha, [2] m_t, [3] min band width (relative to Dl)
int sq_ipe16(int op, const long long* ia, const double* da, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (op == 5) {
    // skip bounds (own layout): ia [0] C fp32 [k][d], [1] C_prev (0: none),
    // [2] G = C C^T fp64 [k][k], [4] perm int32, [5] k, [6] d,
    // [7] G groups, [8] n_wild, [9..12] first tile of groups 0..3, [13] sh,
    // [14] nn (fp64 [k] work), [15] tau (fp64 [1]), [16] wild count (int32
    // [1]), [17] smax, [18] mw, [19] Rc [k][4]; da [0] the D2 margin relative to max |c|^2
    BoundsArgs b;
    b.C = (const float*)ia[0];
    b.Cprev = (const float*)ia[1];
    b.G = (const double*)ia[2];
    b.perm = (const int*)ia[4];
    b.k = (int)ia[5];
    b.d = (int)ia[6];
    b.Gn = (int)ia[7];
    b.n_wild = (int)ia[8];
    for (int q = 0; q < 4; ++q) b.gs[q] = (int)ia[9 + q];
    b.sh = (double*)ia[13];
    b.nn = (double*)ia[14];
    b.tau = (double*)ia[15];
    b.wild_n = (int*)ia[16];
    b.smax = (float*)ia[17];
    b.mw = (float*)ia[18];
    b.Rc = (float*)ia[19];
    b.mrel = da[0];
    if (b.k < 1 || b.k > kSbMaxK || b.d < 1 || b.Gn < 1 || b.Gn > 4 || !b.C || !b.G ||
        !b.perm || !b.sh || !b.nn || !b.tau || !b.wild_n || !b.smax || !b.mw || !b.Rc)
      return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(skip_bounds_rows_kernel, dim3(b.k), dim3(256), 0, st, b);
    if (b.Cprev) hipLaunchKernelGGL(skip_bounds_tau_kernel, dim3(1), dim3(1024), 0, st, b);
    hipLaunchKernelGGL(skip_bounds_cols_kernel, dim3(b.k), dim3(256), 0, st, b);
    return (int)hipGetLastError();
  }
  const long long n = ia[25];
  if (n <= 0) return 0;
  const int d = (int)ia[26], d_pad = (int)ia[27], k = (int)ia[28], k_pad = (int)ia[29];
  const int Q = (int)ia[30];
  const double eps = da[0];
  if (Q < 1 || Q > kIpeMaxQ || !(Q & 1) || k < 1 || k > 16384 || k_pad % 64 || k_pad < k ||
      d < 1 || d > d_pad || d_pad % 16 || d_pad > 1024 || (d_pad > 256 && !ia[65]) ||
      !(eps > 0.0) || ia[50] < 1 ||
      ia[50] > kMaxG || ia[50] > k_pad / 64)
    return (int)hipErrorInvalidValue;
  auto P = [&](int i) -> void* { return (void*)(intptr_t)ia[i]; };
  const IpeScreen sc = make_screen(k, eps, Q);
  if (op == 0) {
    PrepArgs a;
    a.X = (const float*)P(0);
    a.ldx = ia[1];
    a.C = (const float*)P(2);
    a.hint = (const int*)P(5);
    a.xn = (const float*)P(7);
    a.cn = (const float*)P(8);
    a.thr = (float*)P(9);
    a.hj = (int*)P(10);
    a.vlo = (float*)P(11);
    a.vhi = (float*)P(12);
    a.H = (float*)P(13);
    a.rfire = (uint16_t*)P(14);
    a.rst = (unsigned char*)P(15);
    a.best = (unsigned long long*)P(16);
    a.gS = (const float*)P(49);
    a.G = (int)ia[50];
    a.n = n;
    a.d = d;
    a.k = k;
    a.eps = eps;
    a.Q = Q;
    a.key = key_at(ia, 32);
    a.tie = key_at(ia, 36);
    a.bkey = key_at(ia, 44);
    a.skey = key_at(ia, 40);
    a.row_offset = ia[31];
    a.sc = sc;
    // the fp16 filter's error-bound constants (estep_x64)
    a.cp.alpha = da[1];
    a.cp.Ch = 0.0;   // per block, from the centroid norms
    a.cp.sub_rel = 0x1p-21 * sqrt((double)d_pad);
    a.cp.mt = da[2];
    a.cp.min_width = da[3];
    a.cp.d = d;
    cut_constants(a.cp, sc);
    a.stats = (unsigned long long*)P(24);
    a.lb = (float*)P(51);
    a.lb_ok = (int)ia[52];
    a.smax = (const float*)P(53);
    a.Rc = (const float*)P(54);
    a.mw = (const float*)P(64);
    a.lbo = (float*)P(55);
    a.dhint = (float*)P(56);
    a.rows = (int*)P(57);
    a.rows_count = (int*)P(58);
    a.labels = (int*)P(22);
    a.mind = (float*)P(23);
    a.rflag = (unsigned char*)P(21);
    a.ea2 = (float*)P(59);
    if (!a.ea2 || !a.rows || !a.rows_count ||
        (a.lb && (!a.lbo || !a.dhint || (a.lb_ok && (!a.smax || !a.Rc || !a.mw)))))
      return (int)hipErrorInvalidValue;
    const dim3 pg((unsigned)((n + 255) / 256));
    switch (d_pad) {
#define CASE(KSD)                                                               \
  case KSD * 16:                                                                \
    hipLaunchKernelGGL(ipe16_prep_kernel<KSD>, pg, dim3(256), 0, st, a); break;
      CASE(1) CASE(2) CASE(4) CASE(8) CASE(16)
#undef CASE
      default:   // wide rows: chunked canonical dots (zeros past d add +0)
        hipLaunchKernelGGL(ipe16_prep_kernel<64>, pg, dim3(256), 0, st, a);
    }
    return (int)hipGetLastError();
  }
  if (op == 1 || op == 2) {
    SweepArgs a;
    a.Xh = (const _Float16*)P(3);
    a.C = (const _Float16*)P(4);
    a.vlo = (const float*)P(11);
    a.vhi = (const float*)P(12);
    a.rfire = (const uint16_t*)P(14);
    a.rst = (const unsigned char*)P(15);
    a.hj = (const int*)P(10);
    a.perm = (const int*)P(48);
    a.G = (int)ia[50];
    for (int q = 0; q < 3; ++q) a.gb[q] = (int)ia[61 + q];
    a.hint_out = (int*)P(6);
    a.list = (unsigned long long*)P(17);
    a.list_count = (int*)P(18);
    a.dense_rows = (long long*)P(19);
    a.dense_count = (int*)P(20);
    a.rflag = (unsigned char*)P(21);
    a.n = n;
    a.k = k;
    a.k_pad = k_pad;
    a.row_offset = ia[31];
    a.stats = (unsigned long long*)P(24);
    const bool am = op == 1;
    // the argmin sweep (hints) runs over all rows; the screen over prep's list
    a.rows = am ? nullptr : (const int*)P(57);
    a.rows_count = am ? nullptr : (const int*)P(58);
    a.lb = am ? nullptr : (float*)P(51);
    a.lbo = (const float*)P(55);
    a.inv_a2 = 1.0 / (da[1] * da[1]);
    a.cns = (const float*)P(60);
    a.xn = (const float*)P(7);
    a.thr = (const float*)P(9);
    a.ea2 = (const float*)P(59);
    a.cert.inv_a2 = (float)a.inv_a2;
    a.cert.kq = sc.kq;
    a.cert.mt = (float)da[2];
    a.cert.smax = sc.smax;
    a.cert.du = (float)d * 0x1p-24f;
    if (!am && (!a.rows || !a.ea2 || !a.cns || (double)a.cert.inv_a2 != a.inv_a2))
      return (int)hipErrorInvalidValue;
    a.V = (const float*)P(65);
    if (a.V) {
      // wide rows (or forced): the values first, then the sweep without MFMA;
      // ia[66] = the rows V holds (>= the positions of this launch)
      if (ia[66] < n) return (int)hipErrorInvalidValue;
      ValuesArgs v;
      v.Xh = a.Xh;
      v.C = a.C;
      v.rows = a.rows;
      v.rows_count = a.rows_count;
      v.n = n;
      v.ksd = d_pad / 16;
      v.k_pad = k_pad;
      v.V = (float*)P(65);
      hipLaunchKernelGGL(ipe16_values_kernel, dim3((unsigned)((n + 127) / 128), (unsigned)(k_pad / 64)),
                         dim3(256), 0, st, v);
      return am ? launch_sweep<1, true, false, true>(a, st)
                : (a.lb ? launch_sweep<1, false, true, true>(a, st)
                        : launch_sweep<1, false, false, true>(a, st));
    }
    switch (d_pad) {
#define CASE(KSD)                                                                  \
  case KSD * 16:                                                                   \
    return am ? launch_sweep<KSD, true, false>(a, st)                                \
              : (a.lb ? launch_sweep<KSD, false, true>(a, st)                      \
                      : launch_sweep<KSD, false, false>(a, st));
      CASE(1) CASE(2) CASE(4) CASE(8) CASE(16)
#undef CASE
      default:
        return (int)hipErrorInvalidValue;
    }
  }
  if (op == 3) {
    NearArgs a;
    a.list = (const unsigned long long*)P(17);
    a.list_count = (const int*)P(18);
    a.X = (const float*)P(0);
    a.ldx = ia[1];
    a.C = (const float*)P(2);
    a.xn = (const float*)P(7);
    a.cn = (const float*)P(8);
    a.thr = (const float*)P(9);
    a.H = (const float*)P(13);
    a.best = (unsigned long long*)P(16);
    a.d = d;
    a.k = k;
    a.eps = eps;
    a.Q = Q;
    a.key = key_at(ia, 32);
    a.tie = key_at(ia, 36);
    a.skey = key_at(ia, 40);
    a.row_offset = ia[31];
    a.sc = sc;
    a.stats = (unsigned long long*)P(24);
    a.lb = (float*)P(51);
    static int grid = 0;
    if (grid == 0) {
      int dev = 0, cus = 0;
      (void)hipGetDevice(&dev);
      (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
      grid = 8 * (cus > 0 ? cus : 256);
    }
    switch (d_pad) {
#define CASE(KSD)                                                                             \
  case KSD * 16:                                                                              \
    hipLaunchKernelGGL(ipe16_near_kernel<KSD>, dim3((unsigned)grid), dim3(256), 0, st, a); break;
      CASE(1) CASE(2) CASE(4) CASE(8) CASE(16)
#undef CASE
      default:   // wide rows
        hipLaunchKernelGGL(ipe16_near_kernel<64>, dim3((unsigned)grid), dim3(256), 0, st, a);
    }
    return (int)hipGetLastError();
  }
  if (op == 4) {
    hipLaunchKernelGGL(ipe16_finalize_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                       (const unsigned long long*)P(16), (const unsigned char*)P(21), (int*)P(22),
                       (float*)P(23), n, (const int*)P(10), (float*)P(51), (const float*)P(56));
    return (int)hipGetLastError();
  }
  return (int)hipErrorInvalidValue;
}

}  // extern "C"
