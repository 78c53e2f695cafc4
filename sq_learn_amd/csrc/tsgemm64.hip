// Tall-skinny fp64 GEMMs on the matrix cores (v_mfma_f64_16x16x4_f64) for
// any feature count: the linear algebra of the qPCA / q-means preludes
//  at the reference's fp64 LAPACK
// precision (``_qPCA.py:581``, ``utils/extmath.py:161-242``,
// ``_dmeans.py:1244-1245``).
//
//   xtx : C = (A - mu_a)^T (B - mu_b) over the rows; A n x da, B n x db
//         (B = A: the symmetric Gram, upper tile pairs only).  Split-K over
//         row ranges; every workgroup writes its partial tile, and
//         xtx_finalize sums the partials in a fixed order (deterministic,
//         no float atomics) into C (+= for chunked callers).
//   xw  : Y = (A - mu) W; A n x d, W d x l fp64 (upper-triangular W: the
//         k-loop of column tile J stops at its last column).  Output fp64
//         or fp32.
//
// One workgroup = 8 waves on a TM x TN output tile, TM = 64 WM, TN = 32 WN:
// wave w owns a (16 WM) x (16 WN) sub-tile (wm = w & 3, wn = w >> 2), WM x WN
// accumulators of 16 x 16.  Operands are staged through LDS as CENTRED
// fp64 panels of 16 k-rows (k = data rows for xtx, features for xw): panel
// row stride TM + 16 doubles, so the two 16-lane halves of a ds_read_b64
// lane group (k-rows q and q + 1) land on disjoint banks.  The next panel
// is loaded from global memory into registers while the MFMAs consume the
// current one (double-buffered LDS, one barrier per panel).  fp32 / bf16
// inputs are widened exactly; products and sums are fp64.
// f64 MFMA operands: lane l holds A[i = l & 15][k = l >> 4] and
// B[k = l >> 4][j = l & 15]; C/D: lane l, register r -> (row (l >> 4) + 4 r,
// col l & 15).
#include "common.h"
#include <type_traits>

namespace sq {

typedef double f64x4 __attribute__((ext_vector_type(4)));

SQ_DEV double widen(float v) { return (double)v; }
SQ_DEV double widen(double v) { return v; }
SQ_DEV double widen(uint16_t v) { return (double)bf16_to_f32(v); }

constexpr int kPK = 16;      // k-rows per LDS panel (4 MFMA k-steps)
constexpr int kThreads = 512;
// build-time knobs for the variant sweep (benchmarks/tsgemm_variants.py)
#ifndef SQ_TS_WPE
#define SQ_TS_WPE 4          // min waves per SIMD (4: 128 VGPRs, 2 workgroups per CU)
#endif
#ifndef SQ_TS_PK32
#define SQ_TS_PK32 1         // 32-row panels for fp32-staged operands
#endif
#ifndef SQ_TS_PREFETCH
#define SQ_TS_PREFETCH 1     // next k-step's LDS operands read before this step's MFMAs
#endif

// LDS storage of a panel element: fp32 / bf16 inputs are kept as raw fp32
// (exact), fp64 inputs as fp64; the centring happens at operand read
template <typename T> struct Store { using type = float; };
template <> struct Store<double> { using type = double; };

// the MFMAs of one 16-k-row panel pair: As[k][lda_s], Bs[k][ldb_s]; each
// operand is widened and centred (per-lane column mean, in registers)
template <int PK, int WM, int WN, typename SA, typename SB>
SQ_DEV void panel_mfma(const SA* __restrict__ As, const SB* __restrict__ Bs, int lda_s, int ldb_s,
                       int wm, int wn, int lane, const double (&ma)[WM], const double (&mb)[WN],
                       f64x4 (&acc)[WM][WN], int kvalid) {
  const int c16 = lane & 15, q4 = lane >> 4;
  const SA* pa = As + q4 * lda_s + wm * WM * 16 + c16;
  const SB* pb = Bs + q4 * ldb_s + wn * WN * 16 + c16;
  // the raw operands of k-step kk + 1 are read from LDS before the MFMAs of
  // k-step kk are issued (their latency hides behind those MFMAs)
  SA ra[WM];
  SB rb[WN];
#pragma unroll
  for (int i = 0; i < WM; ++i) ra[i] = pa[i * 16];
#pragma unroll
  for (int j = 0; j < WN; ++j) rb[j] = pb[j * 16];
#pragma unroll
  for (int kk = 0; kk < PK / 4; ++kk) {
    if (!SQ_TS_PREFETCH && kk > 0) {
#pragma unroll
      for (int i = 0; i < WM; ++i) ra[i] = pa[(4 * kk) * lda_s + i * 16];
#pragma unroll
      for (int j = 0; j < WN; ++j) rb[j] = pb[(4 * kk) * ldb_s + j * 16];
    }
    // k-rows past the split's end hold 0, which centring would turn into
    // -mu: their A operand is forced to 0 so they add nothing (a select,
    // no exec-mask branch in the loop)
    const double kv = 4 * kk + q4 < kvalid ? 1.0 : 0.0;
    double a[WM], b[WN];
#pragma unroll
    for (int i = 0; i < WM; ++i) a[i] = ((double)ra[i] - ma[i]) * kv;
#pragma unroll
    for (int j = 0; j < WN; ++j) b[j] = (double)rb[j] - mb[j];
    if (SQ_TS_PREFETCH && kk + 1 < PK / 4) {
#pragma unroll
      for (int i = 0; i < WM; ++i) ra[i] = pa[(4 * (kk + 1)) * lda_s + i * 16];
#pragma unroll
      for (int j = 0; j < WN; ++j) rb[j] = pb[(4 * (kk + 1)) * ldb_s + j * 16];
    }
#pragma unroll
    for (int i = 0; i < WM; ++i)
#pragma unroll
      for (int j = 0; j < WN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i], b[j], acc[i][j], 0, 0, 0);
  }
}

// ------------------------------------------------------------------ xtx
// Panel of 16 data rows x TC columns of M (row-major, ld) in LDS S[k][TC+16]
// (row stride = 16 mod 32 elements: conflict-free operand reads).
//  * fp32 / bf16: thread t -> row t / (TC/V), V consecutive columns (one
//    16-B / 8-B global load), stored with one V-wide ds_write (lanes
//    contiguous: conflict-free);
//  * fp64: thread t -> row t / 32, columns (t % 32) + 32 e (8-B loads, a
//    wave reads 256 contiguous bytes per row; ds_write_b64 lanes contiguous).
template <typename T, int TC, bool VEC, int PK = kPK>
struct RowPanel {
  using S = typename Store<T>::type;
  static constexpr bool F64 = sizeof(T) == 8;
  static_assert(!F64 || PK == 16, "fp64 panels: 32 threads per 16-row panel row");
  static constexpr int V = (PK * TC) / kThreads;   // 1, 2, 4 (8 for 32-row fp32 panels)
  static constexpr int TPR = F64 ? 32 : TC / V;     // threads per panel row
  static constexpr int LD = TC + 16;
  S v[V];
  SQ_DEV void load(const T* __restrict__ M, long long ld, long long r, long long r_end, int c0,
                   int ncols) {
    const int t = threadIdx.x;
    const long long row = r + t / TPR;
    const T* p = M + (size_t)(row < r_end ? row : r) * ld;
    const bool rok = row < r_end;
    if constexpr (F64) {
#pragma unroll
      for (int e = 0; e < V; ++e) {
        const int col = c0 + (t % 32) + 32 * e;
        v[e] = rok && col < ncols ? p[col] : 0.0;
      }
    } else {
      const int col = c0 + (t % TPR) * V;
      const int lim = rok ? ncols - col : 0;
      if (VEC && V == 8 && lim >= 8) {
        if constexpr (sizeof(T) == 4) {
          const float4 x = *reinterpret_cast<const float4*>(p + col);
          const float4 y = *reinterpret_cast<const float4*>(p + col + 4);
          v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
          v[4] = y.x; v[5] = y.y; v[6] = y.z; v[7] = y.w;
          return;
        } else {
          const uint4 x = *reinterpret_cast<const uint4*>(p + col);
          const uint32_t w4[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[2 * e] = bf16_to_f32((uint16_t)(w4[e] & 0xFFFFu));
            v[2 * e + 1] = bf16_to_f32((uint16_t)(w4[e] >> 16));
          }
          return;
        }
      }
      if (VEC && V == 4 && lim >= 4) {
        if constexpr (sizeof(T) == 4) {
          const float4 x = *reinterpret_cast<const float4*>(p + col);
          v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
          return;
        } else {
          const uint2 x = *reinterpret_cast<const uint2*>(p + col);
          v[0] = bf16_to_f32((uint16_t)(x.x & 0xFFFFu));
          v[1] = bf16_to_f32((uint16_t)(x.x >> 16));
          v[2] = bf16_to_f32((uint16_t)(x.y & 0xFFFFu));
          v[3] = bf16_to_f32((uint16_t)(x.y >> 16));
          return;
        }
      }
#pragma unroll
      for (int e = 0; e < V; ++e) v[e] = e < lim ? (float)widen(p[col + e]) : 0.0f;
    }
  }
  SQ_DEV void store(S* __restrict__ dst) const {
    const int t = threadIdx.x;
    if constexpr (F64) {
#pragma unroll
      for (int e = 0; e < V; ++e) dst[(t / 32) * LD + (t % 32) + 32 * e] = v[e];
    } else if constexpr (V == 8) {
      float* q = dst + (t / TPR) * LD + (t % TPR) * 8;
      *reinterpret_cast<float4*>(q) = make_float4(v[0], v[1], v[2], v[3]);
      *reinterpret_cast<float4*>(q + 4) = make_float4(v[4], v[5], v[6], v[7]);
    } else if constexpr (V == 4) {
      *reinterpret_cast<float4*>(dst + (t / TPR) * LD + (t % TPR) * 4) =
          make_float4(v[0], v[1], v[2], v[3]);
    } else if constexpr (V == 2) {
      *reinterpret_cast<float2*>(dst + (t / TPR) * LD + (t % TPR) * 2) = make_float2(v[0], v[1]);
    } else {
      dst[(t / TPR) * LD + t % TPR] = v[0];
    }
  }
};

template <typename TA, typename TB, int WM, int WN, bool SYM, bool VEC>
__global__ void __launch_bounds__(kThreads, SQ_TS_WPE) xtx_kernel(
    const TA* __restrict__ A, long long lda, const double* __restrict__ mua, int da,
    const TB* __restrict__ B, long long ldb, const double* __restrict__ mub, int db, long long n,
    int n_splits, int n_pairs, int ntb, double* __restrict__ part) {
  constexpr int TM = 64 * WM, TN = 32 * WN;
  // 32-row panels when both operands stage as fp32 (half the barriers per
  // MFMA; 74 KiB of LDS), 16 for fp64 operands
  constexpr int PK = (SQ_TS_PK32 && sizeof(TA) < 8 && sizeof(TB) < 8) ? 32 : 16;
  using PA = RowPanel<TA, TM, VEC, PK>;
  using PB = RowPanel<TB, TN, VEC, PK>;
  using SA = typename PA::S;
  using SB = typename PB::S;
  __shared__ __attribute__((aligned(16))) SA As[2][PK * PA::LD];
  __shared__ __attribute__((aligned(16))) SB Bs[2][PK * PB::LD];
  // XCD-aware item: the 8 XCDs take splits s = xcd mod 8, so every tile pair
  // of a split (the same rows) runs in one XCD's L2
  const int b = blockIdx.x;
  const int xcd = b & 7, idx = b >> 3;
  const int s = 8 * (idx / n_pairs) + xcd;
  const int p = idx % n_pairs;
  int I, J;
  if (SYM) {   // upper pairs (I <= J), row-major over I
    I = 0;
    int rem = p, row_len = ntb;
    while (rem >= row_len) { rem -= row_len; ++I; --row_len; }
    J = I + rem;
  } else {
    I = p / ntb;
    J = p % ntb;
  }
  const bool diag = SYM && I == J;
  const int wv = threadIdx.x >> 6;
  const bool below = diag && (wv & 3) * WM > (wv >> 2) * WN + WN - 1;   // wave-uniform
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = w & 3, wn = w >> 2;
  const int c16 = lane & 15, q4 = lane >> 4;
  const long long per = (n + n_splits - 1) / n_splits;
  const long long r_begin = (long long)s * per;
  const long long r_end = r_begin + per < n ? r_begin + per : n;
  const int a0 = I * TM, b0 = J * TN;
  // the column means of this lane's operand columns (constant over the
  // rows), staged through LDS and read into registers before any panel load
  // is in flight (a global load here would make the compiler drain the
  // prefetch queue - vmcnt(0) - inside the MFMA loop)
  __shared__ double smu[TM + TN];
  for (int c = threadIdx.x; c < TM + TN; c += kThreads) {
    const int ca = a0 + c, cb = b0 + c - TM;
    smu[c] = c < TM ? (mua && ca < da ? mua[ca] : 0.0) : (mub && cb < db ? mub[cb] : 0.0);
  }
  __syncthreads();
  double ma[WM], mb[WN];
#pragma unroll
  for (int i = 0; i < WM; ++i) ma[i] = smu[(wm * WM + i) * 16 + c16];
#pragma unroll
  for (int j = 0; j < WN; ++j) mb[j] = smu[TM + (wn * WN + j) * 16 + c16];
  f64x4 acc[WM][WN];
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j) acc[i][j] = (f64x4){0.0, 0.0, 0.0, 0.0};
  PA pa;
  PB pb;
  const TB* Bsrc = SYM ? (const TB*)A : B;
  const long long ldbs = SYM ? lda : ldb;
  const int npan = r_end > r_begin ? (int)((r_end - r_begin + PK - 1) / PK) : 0;
  if (npan > 0) {
    pa.load(A, lda, r_begin, r_end, a0, da);
    if (!diag) pb.load(Bsrc, ldbs, r_begin, r_end, b0, db);
    pa.store(As[0]);
    if (!diag) pb.store(Bs[0]);
  }
  __syncthreads();
  for (int st = 0; st < npan; ++st) {
    const int cur = st & 1;
    const bool more = st + 1 < npan;
    if (more) {   // next panel: global -> registers, in flight during the MFMAs
      const long long r = r_begin + (long long)(st + 1) * PK;
      pa.load(A, lda, r, r_end, a0, da);
      if (!diag) pb.load(Bsrc, ldbs, r, r_end, b0, db);
    }
    // SYM diagonal tile: B = the A panel (SYM: TA == TB and TM == TN, one
    // inlined copy of the MFMA loop with a runtime operand source); the
    // waves whose whole sub-tile lies below the diagonal skip the MFMAs (the
    // finalize reads the upper triangle only)
    const SB* bsrc = diag ? (const SB*)As[cur] : Bs[cur];
    const long long left = r_end - (r_begin + (long long)st * PK);
    if (!below)
      panel_mfma<PK, WM, WN>(As[cur], bsrc, PA::LD, PB::LD, wm, wn, lane, ma, mb, acc,
                             left < PK ? (int)left : PK);
    if (more) {
      pa.store(As[cur ^ 1]);
      if (!diag) pb.store(Bs[cur ^ 1]);
    }
    __syncthreads();
  }
  // partial tile (TM x TN) of item (s, p)
  double* out = part + ((size_t)s * n_pairs + p) * (TM * TN);
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        out[((wm * WM + i) * 16 + q4 + 4 * r) * TN + (wn * WN + j) * 16 + c16] = acc[i][j][r];
}

// C[i][j] (+)= sum over splits of the partial tiles; SYM also writes the
// mirror C[j][i].  A workgroup takes 64 consecutive elements of C; its 4
// waves sum the splits s = g mod 4 (coalesced 64-element rows of the
// partials), combined in LDS in the fixed order ((g0 + g1) + g2) + g3.
__global__ void __launch_bounds__(256) xtx_finalize_kernel(const double* __restrict__ part,
                                                           int n_splits, int n_pairs, int TM,
                                                           int TN, int ntb, int da, int db,
                                                           int sym, int accumulate,
                                                           double* __restrict__ C) {
  __shared__ double red[4][64];
  const int g = threadIdx.x >> 6, el = threadIdx.x & 63;
  const long long e = (long long)blockIdx.x * 64 + el;
  const bool live = e < (long long)da * db;
  const int i = live ? (int)(e / db) : 0, j = live ? (int)(e % db) : 0;
  const bool want = live && !(sym && i > j);
  double sum = 0.0;
  size_t off = 0;
  if (want) {
    const int I = i / TM, J = j / TN;
    const int p = sym ? I * ntb - I * (I - 1) / 2 + (J - I) : I * ntb + J;
    off = (size_t)p * TM * TN + (size_t)(i - I * TM) * TN + (j - J * TN);
    const size_t stride = (size_t)n_pairs * TM * TN;
#pragma unroll 8
    for (int s = g; s < n_splits; s += 4) sum += part[(size_t)s * stride + off];
  }
  red[g][el] = sum;
  __syncthreads();
  if (g == 0 && want) {
    double t = ((red[0][el] + red[1][el]) + red[2][el]) + red[3][el];
    if (accumulate) t += C[(size_t)i * db + j];
    C[(size_t)i * db + j] = t;
    if (sym && i != j) C[(size_t)j * db + i] = t;
  }
}

// ------------------------------------------------------------------- xw
// A panel: TM data rows x 16 features, centred fp64 in LDS S[row][18]
// (operand reads: lanes 0-15 = 16 rows at one k -> row * 18 mod 32 spreads
// them over the even 2-dword slots, k + 1 the odd ones: conflict-free);
// thread t -> row t / 4, features (t % 4) * 4 .. + 4 (TM = 128)
constexpr int kLDK = 18;
template <typename T, int TM, bool VEC>
struct ColPanel {
  static constexpr int V = (kPK * TM) / kThreads;   // 4 (TM 128)
  static constexpr int TPR = kPK / V;
  double v[V];
  SQ_DEV void load(const T* __restrict__ A, long long lda, const double* __restrict__ mu,
                   long long r0, long long n, int k0, int d) {
    const int t = threadIdx.x;
    const long long row = r0 + t / TPR;
    const int col = k0 + (t % TPR) * V;
    const int lim = row < n ? d - col : 0;
    const T* p = A + (size_t)(row < n ? row : r0) * lda + col;
    bool done = false;
    if constexpr (VEC && V == 4) {
      if (lim >= 4) {
        if constexpr (sizeof(T) == 4) {
          const float4 x = *reinterpret_cast<const float4*>(p);
          v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
        } else if constexpr (sizeof(T) == 8) {
          const double2 x0 = *reinterpret_cast<const double2*>(p);
          const double2 x1 = *reinterpret_cast<const double2*>(p + 2);
          v[0] = x0.x; v[1] = x0.y; v[2] = x1.x; v[3] = x1.y;
        } else {
          const uint2 x = *reinterpret_cast<const uint2*>(p);
          v[0] = bf16_to_f32((uint16_t)(x.x & 0xFFFFu));
          v[1] = bf16_to_f32((uint16_t)(x.x >> 16));
          v[2] = bf16_to_f32((uint16_t)(x.y & 0xFFFFu));
          v[3] = bf16_to_f32((uint16_t)(x.y >> 16));
        }
        done = true;
      }
    }
    if (!done) {
#pragma unroll
      for (int e = 0; e < V; ++e) v[e] = e < lim ? widen(p[e]) : 0.0;
    }
    if (mu) {
#pragma unroll
      for (int e = 0; e < V; ++e)
        if (e < lim) v[e] -= mu[col + e];
    }
  }
  SQ_DEV void store(double* __restrict__ S) const {
    const int t = threadIdx.x;
#pragma unroll
    for (int e = 0; e < V; e += 2)
      *reinterpret_cast<double2*>(S + (t / TPR) * kLDK + (t % TPR) * V + e) = make_double2(v[e], v[e + 1]);
  }
};

// operand reads of the xw A panel: A[i = row][k] = S[row][k]
template <int WM, int WN>
SQ_DEV void panel_mfma_xw(const double* __restrict__ As, const double* __restrict__ Ws, int ldw_s,
                          int wm, int wn, int lane, f64x4 (&acc)[WM][WN]) {
  const int c16 = lane & 15, q4 = lane >> 4;
#pragma unroll
  for (int kk = 0; kk < kPK / 4; ++kk) {
    double a[WM], b[WN];
#pragma unroll
    for (int i = 0; i < WM; ++i) a[i] = As[((wm * WM + i) * 16 + c16) * kLDK + 4 * kk + q4];
#pragma unroll
    for (int j = 0; j < WN; ++j) b[j] = Ws[(4 * kk + q4) * ldw_s + (wn * WN + j) * 16 + c16];
#pragma unroll
    for (int i = 0; i < WM; ++i)
#pragma unroll
      for (int j = 0; j < WN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i], b[j], acc[i][j], 0, 0, 0);
  }
}

template <typename T, typename TO, int WM, int WN, bool VEC>
__global__ void __launch_bounds__(kThreads, SQ_TS_WPE) xw_kernel(
    const T* __restrict__ A, long long lda, const double* __restrict__ mu, long long n, int d,
    const double* __restrict__ W, long long ldw, int l, int upper, TO* __restrict__ Y,
    long long ldy) {
  constexpr int TM = 64 * WM, TN = 32 * WN;
  using PW = RowPanel<double, TN, false>;   // W panel: 16 k-rows x TN columns (ldw any)
  __shared__ __attribute__((aligned(16))) double As[2][TM * kLDK];
  __shared__ __attribute__((aligned(16))) double Ws[2][kPK * PW::LD];
  const long long r0 = (long long)blockIdx.x * TM;
  const int c0 = blockIdx.y * TN;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = w & 3, wn = w >> 2;
  f64x4 acc[WM][WN];
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j) acc[i][j] = (f64x4){0.0, 0.0, 0.0, 0.0};
  // upper-triangular W: rows k > last column of the tile are zero
  const int kend = upper ? (c0 + TN < d ? c0 + TN : d) : d;
  const int npan = (kend + kPK - 1) / kPK;
  ColPanel<T, TM, VEC> pa;
  PW pw;
  pa.load(A, lda, mu, r0, n, 0, kend);
  pw.load(W, ldw, 0, kend, c0, l);
  pa.store(As[0]);
  pw.store(Ws[0]);
  __syncthreads();
  for (int st = 0; st < npan; ++st) {
    const int cur = st & 1;
    const bool more = st + 1 < npan;
    if (more) {
      pa.load(A, lda, mu, r0, n, (st + 1) * kPK, kend);
      pw.load(W, ldw, (st + 1) * kPK, kend, c0, l);
    }
    panel_mfma_xw<WM, WN>(As[cur], Ws[cur], PW::LD, wm, wn, lane, acc);
    if (more) {
      pa.store(As[cur ^ 1]);
      pw.store(Ws[cur ^ 1]);
    }
    __syncthreads();
  }
  const int c16 = lane & 15, q4 = lane >> 4;
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const long long row = r0 + (wm * WM + i) * 16 + q4 + 4 * r;
        const int col = c0 + (wn * WN + j) * 16 + c16;
        if (row < n && col < l) Y[(size_t)row * ldy + col] = (TO)acc[i][j][r];
      }
}

}  // namespace sq

using namespace sq;

namespace {

// WN from the output width: 32-column tiles for thin outputs (power
// iteration, l <= 32), 64 for <= 64, else 128
int pick_wn(int cols) { return cols <= 32 ? 1 : (cols <= 64 ? 2 : 4); }

template <typename TA, typename TB, int WN, bool SYM>
int launch_xtx_t(const void* A, long long lda, const double* mua, int da, const void* B,
                 long long ldb, const double* mub, int db, long long n, int n_splits, double* part,
                 bool vec, hipStream_t st) {
  constexpr int WM = 2;
  constexpr int TM = 64 * WM, TN = 32 * WN;
  const int nta = (da + TM - 1) / TM, ntb = (db + TN - 1) / TN;
  const int n_pairs = SYM ? nta * (nta + 1) / 2 : nta * ntb;
  const dim3 grid((unsigned)(n_splits * n_pairs));
#define GO(V)                                                                                   \
  hipLaunchKernelGGL((xtx_kernel<TA, TB, WM, WN, SYM, V>), grid, dim3(kThreads), 0, st,         \
                     (const TA*)A, lda, mua, da, (const TB*)B, ldb, mub, db, n, n_splits,       \
                     n_pairs, SYM ? nta : ntb, part)
  if (vec) GO(true); else GO(false);
#undef GO
  return (int)hipGetLastError();
}

template <typename TA, typename TB, bool SYM>
int launch_xtx_w(int wn, const void* A, long long lda, const double* mua, int da, const void* B,
                 long long ldb, const double* mub, int db, long long n, int n_splits,
                 double* part, bool vec, hipStream_t st) {
  if constexpr (SYM) {
    return launch_xtx_t<TA, TB, 4, true>(A, lda, mua, da, B, ldb, mub, db, n, n_splits, part, vec, st);
  } else {
  switch (wn) {
    case 1: return launch_xtx_t<TA, TB, 1, false>(A, lda, mua, da, B, ldb, mub, db, n, n_splits, part, vec, st);
    case 2: return launch_xtx_t<TA, TB, 2, false>(A, lda, mua, da, B, ldb, mub, db, n, n_splits, part, vec, st);
    default: return launch_xtx_t<TA, TB, 4, false>(A, lda, mua, da, B, ldb, mub, db, n, n_splits, part, vec, st);
  }
  }
}

template <typename TA>
int launch_xtx_b(int tb, int wn, bool sym, const void* A, long long lda, const double* mua,
                 int da, const void* B, long long ldb, const double* mub, int db, long long n,
                 int n_splits, double* part, bool vec, hipStream_t st) {
  if (sym) return launch_xtx_w<TA, TA, true>(wn, A, lda, mua, da, A, lda, mua, da, n, n_splits, part, vec, st);
  switch (tb) {
    case 0: return launch_xtx_w<TA, float, false>(wn, A, lda, mua, da, B, ldb, mub, db, n, n_splits, part, vec, st);
    case 1: return launch_xtx_w<TA, double, false>(wn, A, lda, mua, da, B, ldb, mub, db, n, n_splits, part, vec, st);
    default: return launch_xtx_w<TA, uint16_t, false>(wn, A, lda, mua, da, B, ldb, mub, db, n, n_splits, part, vec, st);
  }
}

template <typename T, typename TO, int WN>
int launch_xw_t(const void* A, long long lda, const double* mu, long long n, int d,
                const double* W, long long ldw, int l, int upper, void* Y, long long ldy,
                bool vec, hipStream_t st) {
  constexpr int WM = 2;
  constexpr int TM = 64 * WM, TN = 32 * WN;
  const dim3 grid((unsigned)((n + TM - 1) / TM), (unsigned)((l + TN - 1) / TN));
#define GO(V)                                                                                 \
  hipLaunchKernelGGL((xw_kernel<T, TO, WM, WN, V>), grid, dim3(kThreads), 0, st, (const T*)A, \
                     lda, mu, n, d, W, ldw, l, upper, (TO*)Y, ldy)
  if (vec) GO(true); else GO(false);
#undef GO
  return (int)hipGetLastError();
}

template <typename T, typename TO>
int launch_xw_w(int wn, const void* A, long long lda, const double* mu, long long n, int d,
                const double* W, long long ldw, int l, int upper, void* Y, long long ldy,
                bool vec, hipStream_t st) {
  switch (wn) {
    case 1: return launch_xw_t<T, TO, 1>(A, lda, mu, n, d, W, ldw, l, upper, Y, ldy, vec, st);
    case 2: return launch_xw_t<T, TO, 2>(A, lda, mu, n, d, W, ldw, l, upper, Y, ldy, vec, st);
    default: return launch_xw_t<T, TO, 4>(A, lda, mu, n, d, W, ldw, l, upper, Y, ldy, vec, st);
  }
}

template <typename T>
int launch_xw_o(int to, int wn, const void* A, long long lda, const double* mu, long long n, int d,
                const double* W, long long ldw, int l, int upper, void* Y, long long ldy,
                bool vec, hipStream_t st) {
  if (to == 1) return launch_xw_w<T, double>(wn, A, lda, mu, n, d, W, ldw, l, upper, Y, ldy, vec, st);
  return launch_xw_w<T, float>(wn, A, lda, mu, n, d, W, ldw, l, upper, Y, ldy, vec, st);
}

bool aligned(const void* p, long long ld, int esz) {
  // 4-element vector loads: base and row stride 4-element aligned
  return ((uintptr_t)p % (4 * esz)) == 0 && ld % 4 == 0;
}

int esize(int code) { return code == 1 ? 8 : (code == 2 ? 2 : 4); }

}  // namespace

extern "C" {

// geometry of an xtx call: tile sizes, pair count (the host sizes `part`)
int sq_xtx_geometry(int da, int db, int sym, int* TM, int* TN, int* n_pairs) {
  const int wn = sym ? 4 : pick_wn(db);
  *TM = 128;
  *TN = 32 * wn;
  if (sym) *TN = 128;
  const int nta = (da + 127) / 128, ntb = (db + *TN - 1) / *TN;
  *n_pairs = sym ? nta * (nta + 1) / 2 : nta * ntb;
  return 0;
}

// dtype codes: 0 fp32, 1 fp64, 2 bf16.  sym: B ignored (B = A).
// n_splits must be a multiple of 8; part holds n_splits * n_pairs * TM * TN.
int sq_xtx(const void* A, int ta, long long lda, const void* mua, int da, const void* B, int tb,
           long long ldb, const void* mub, int db, long long n, int sym, int n_splits, void* part,
           void* C, int accumulate, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (da < 1 || db < 1 || n < 0 || n_splits < 8 || n_splits % 8 || lda < da || (!sym && ldb < db))
    return (int)hipErrorInvalidValue;
  if (sym) db = da;
  int TM, TN, np;
  sq_xtx_geometry(da, db, sym, &TM, &TN, &np);
  const int wn = TN / 32;
  const bool vec = aligned(A, lda, esize(ta)) && (sym || aligned(B, ldb, esize(tb)));
  int rc;
  switch (ta) {
    case 0: rc = launch_xtx_b<float>(tb, wn, sym, A, lda, (const double*)mua, da, B, ldb, (const double*)mub, db, n, n_splits, (double*)part, vec, st); break;
    case 1: rc = launch_xtx_b<double>(tb, wn, sym, A, lda, (const double*)mua, da, B, ldb, (const double*)mub, db, n, n_splits, (double*)part, vec, st); break;
    default: rc = launch_xtx_b<uint16_t>(tb, wn, sym, A, lda, (const double*)mua, da, B, ldb, (const double*)mub, db, n, n_splits, (double*)part, vec, st); break;
  }
  if (rc) return rc;
  const int ntb = sym ? (da + TM - 1) / TM : (db + TN - 1) / TN;
  const long long tot = (long long)da * db;
  hipLaunchKernelGGL(xtx_finalize_kernel, dim3((unsigned)((tot + 63) / 64)), dim3(256), 0, st,
                     (const double*)part, n_splits, np, TM, TN, ntb, da, db, sym, accumulate,
                     (double*)C);
  return (int)hipGetLastError();
}

// Y = (A - mu) W; W d x l fp64 (ldw), upper: W upper triangular; to: 0 fp32, 1 fp64
int sq_xw(const void* A, int ta, long long lda, const void* mu, long long n, int d, const void* W,
          long long ldw, int l, int upper, void* Y, int to, long long ldy, void* stream) {
  if (n <= 0) return 0;
  if (d < 1 || l < 1 || lda < d || ldw < l || ldy < l) return (int)hipErrorInvalidValue;
  const int wn = pick_wn(l);
  const bool vec = aligned(A, lda, esize(ta));
  hipStream_t st = (hipStream_t)stream;
  switch (ta) {
    case 0: return launch_xw_o<float>(to, wn, A, lda, (const double*)mu, n, d, (const double*)W, ldw, l, upper, Y, ldy, vec, st);
    case 1: return launch_xw_o<double>(to, wn, A, lda, (const double*)mu, n, d, (const double*)W, ldw, l, upper, Y, ldy, vec, st);
    default: return launch_xw_o<uint16_t>(to, wn, A, lda, (const double*)mu, n, d, (const double*)W, ldw, l, upper, Y, ldy, vec, st);
  }
}

}  // extern "C"
