// Row statistics for the qPCA / q-means preludes on
// gfx950 (the Gram / power-iteration GEMMs live in tsgemm64.hip).
//
// mu_sums    : all exponents of the mu(A) p-grid in one pass per 512-column
//              block (row power sums -> max, column power sums)
//              (Utility.py:196-231).
// row_norms  : ||x_i||^2 for bf16/fp32 rows.
#include "common.h"
#include <type_traits>

namespace sq {

typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(2))) float f32x2;   // packed fp32 (v_pk_*_f32)

template <typename T> SQ_DEV float ld1(const T* p, size_t i);
template <> SQ_DEV float ld1<float>(const float* p, size_t i) { return p[i]; }
template <> SQ_DEV float ld1<uint16_t>(const uint16_t* p, size_t i) { return bf16_to_f32(p[i]); }

// ------------------------------------------------------------------ mu
// Power sums of |a|^q for a p-grid of exponents (mu(A), Utility.py:196-231):
// rowmax[i] = max_r sum_c |a_rc|^q_i, colsum[i][c] = sum_r |a_rc|^q_i.
// Lanes own 8 consecutive columns; LPR = ceil(d/8) (power of two) lanes per
// row, so a wave covers 64/LPR rows at once (no idle lanes for d < 256).
// One v_log per element, one v_exp per (element, exponent); row sums by
// log2(LPR) xor-shuffles; column sums reduced in LDS per workgroup and
// written as per-WG partials, summed by mu_colsum_kernel in a fixed order
// (no float atomics: deterministic).  ``mean`` (fp32 [d_total], nullable):
// the power sums of |a - mean| (the centred matrix without a centred copy).
constexpr int MUQ = 12;

template <typename T>
SQ_DEV void ld8raw(const T* p, bool full, int valid, float v[8]);
template <>
SQ_DEV void ld8raw<uint16_t>(const uint16_t* p, bool full, int valid, float v[8]) {
  if (full) {
    uint4 u = *reinterpret_cast<const uint4*>(p);
    uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[2 * e] = __uint_as_float(w[e] << 16);
      v[2 * e + 1] = __uint_as_float(w[e] & 0xFFFF0000u);
    }
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = e < valid ? bf16_to_f32(p[e]) : 0.f;
  }
}
template <>
SQ_DEV void ld8raw<float>(const float* p, bool full, int valid, float v[8]) {
  if (full) {
    float4 a = *reinterpret_cast<const float4*>(p);
    float4 b = *reinterpret_cast<const float4*>(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = e < valid ? p[e] : 0.f;
  }
}

// Transposing butterfly over the LPR (>= 16) lanes of a row: 16 values per
// lane in, the LPR-lane sum of value butterfly_index(lane) out in v[0].  A
// halving step at lane bit o (while more than one value is left) keeps the
// upper half of the values on lanes with the bit set, the lower half on the
// others, and adds the partner's copy of the kept half; the remaining steps
// (LPR > 16) add the partner's single value.
template <int LPR>
SQ_DEV int butterfly_index(int lane) {
  int j = 0;
#pragma unroll
  for (int s = 0, o = LPR / 2, c = 16; o >= 1; ++s, o >>= 1) {
    if (c > 1 && o >= LPR / 16) {
      if (lane & o) j += c / 2;
      c /= 2;
    }
  }
  return j;
}

// The butterfly partner at lane bit O
// (measured: DPP moves for the low bits - quad_perm / row mirrors, with
// their VALU-to-DPP wait states - made the kernel 2.3x slower than
// ds_bpermute at 10M x 256)
template <int O>
SQ_DEV float xpart(float x) {
  return __shfl_xor(x, O, 64);
}

template <int LPR>
SQ_DEV void rowsum_butterfly(float (&v)[16], int lane) {
  // halving steps on the high lane bits (LPR/2 down to LPR/16), then plain
  // adds on the low bits
  auto halve = [&](auto C_, auto O_) {
    constexpr int c = decltype(C_)::value, o = decltype(O_)::value;
    const bool hi = (lane & o) != 0;
#pragma unroll
    for (int t = 0; t < c / 2; ++t) {
      const float send = hi ? v[t] : v[t + c / 2];
      const float keep = hi ? v[t + c / 2] : v[t];
      v[t] = keep + xpart<o>(send);
    }
  };
  halve(std::integral_constant<int, 16>{}, std::integral_constant<int, LPR / 2>{});
  halve(std::integral_constant<int, 8>{}, std::integral_constant<int, LPR / 4>{});
  halve(std::integral_constant<int, 4>{}, std::integral_constant<int, LPR / 8>{});
  halve(std::integral_constant<int, 2>{}, std::integral_constant<int, LPR / 16>{});
  if constexpr (LPR >= 64) v[0] += xpart<LPR / 32>(v[0]);
  if constexpr (LPR >= 32) v[0] += xpart<1>(v[0]);
}

// d > 512: one launch per 512-column block (col0); the row power sums of the
// earlier blocks are carried in rowacc[nq][n] and the maxima taken by the
// last block (final = 1).
// ARITH: the exponents are the arithmetic grid 0, qstep, 2 qstep, ... (the
// p-grid of mu(A)).  Every exponent slot is computed (slots >= nq are
// dropped at the end): one basic block per row step, no per-exponent branch.
template <typename T, int LPR, bool ARITH>
__global__ void __launch_bounds__(256) mu_sums_kernel(
    const T* __restrict__ X, long long ldx, int col0, int d_total, const float* __restrict__ qs,
    int nq, float* __restrict__ rowmax, float* __restrict__ part, float* __restrict__ rowacc,
    int final, long long n, int d, long long rows_per_wg, const float* __restrict__ mean,
    float qstep) {
  constexpr int RPW = 64 / LPR;              // rows per wave step
  __shared__ float red[256 * 8];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int vl = lane % LPR;                  // column group of this lane
  const int sg = (wave * 64 + lane) / LPR;    // row slot within the WG (0 .. 4*RPW-1)
  const int c0 = vl * 8;
  const bool vec = ((ldx % 8) == 0) && ((col0 % 8) == 0) && (c0 + 8 <= d);
  const int valid = d - c0;
  // this lane's 8 column means (0 without a mean)
  float mu8[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) mu8[e] = (mean && c0 + e < d) ? mean[col0 + c0 + e] : 0.f;
  float q[MUQ];
#pragma unroll
  for (int i = 0; i < MUQ; ++i) q[i] = i < nq ? qs[i] : 0.f;
  f32x2 cs[MUQ][4];   // column sums, packed pairs of the lane's 8 columns
  float rmax[MUQ];
  // (LPR >= 16) the exponent whose row sums this lane ends with, and the
  // lane bits that hold duplicates of it (the butterfly's plain steps)
  float rmax1 = 0.f;
  const int rjl = butterfly_index<LPR>(lane);
  constexpr int rj_dup = LPR > 16 ? (LPR / 16 - 1) : 0;
#pragma unroll
  for (int i = 0; i < MUQ; ++i) {
    rmax[i] = 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e) cs[i][e] = (f32x2){0.f, 0.f};
  }
  const long long r_beg = (long long)blockIdx.x * rows_per_wg;
  const long long r_end = min(n, r_beg + rows_per_wg);
  // the next row step's 8 values are loaded before this step's arithmetic
  // (the loop is otherwise one dependent load per step: latency-bound)
  float vn[8];
  auto load8 = [&](long long rr, float (&dst)[8]) {
    if (c0 < d && rr < r_end) ld8raw<T>(X + (size_t)rr * ldx + col0 + c0, vec, valid, dst);
    else {
#pragma unroll
      for (int e = 0; e < 8; ++e) dst[e] = 0.f;
    }
  };
  load8(r_beg + sg, vn);
  for (long long r = r_beg + sg; r < r_end; r += 4 * RPW) {
    float v[8], lg[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = vn[e];
    load8(r + 4 * RPW, vn);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = e < valid ? fabsf(v[e] - mu8[e]) : 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) lg[e] = __builtin_amdgcn_logf(v[e]);   // log2, -inf at 0
    // qstep > 0: q_i = i qstep - one exp2 per element, then |a|^(i qstep) by
    // successive products (<= MUQ roundings, ~1e-6 relative)
    // (arithmetic grid: packed pairs - one v_pk_mul / v_pk_add per 2 columns)
    f32x2 tb[4], cur[4];
    if constexpr (ARITH) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        tb[e] = (f32x2){__builtin_amdgcn_exp2f(qstep * lg[2 * e]),
                        __builtin_amdgcn_exp2f(qstep * lg[2 * e + 1])};
        cur[e] = tb[e];
      }
    }
    // per exponent: the lane's column sums and its partial row sum (LPR >=
    // 16: collected for the butterfly; else reduced right away)
    float rsv[LPR >= 16 ? 16 : 1];
#pragma unroll
    for (int i = 0; i < (LPR >= 16 ? 16 : 1); ++i) rsv[i] = 0.f;
#pragma unroll
    for (int i = 0; i < MUQ; ++i) {
      {
        f32x2 rs2 = (f32x2){0.f, 0.f};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          // |a|^0 counts nonzeros; exp2(q * -inf) = 0 for q > 0
          f32x2 pw;
          if constexpr (ARITH) {
            if (i == 0) {
              pw = (f32x2){v[2 * e] != 0.f ? 1.f : 0.f, v[2 * e + 1] != 0.f ? 1.f : 0.f};
            } else {
              if (i > 1) cur[e] *= tb[e];
              pw = cur[e];
            }
          } else {
            pw.x = q[i] == 0.f ? (v[2 * e] != 0.f ? 1.f : 0.f)
                               : __builtin_amdgcn_exp2f(q[i] * lg[2 * e]);
            pw.y = q[i] == 0.f ? (v[2 * e + 1] != 0.f ? 1.f : 0.f)
                               : __builtin_amdgcn_exp2f(q[i] * lg[2 * e + 1]);
          }
          cs[i][e] += pw;
          rs2 += pw;
        }
        float rs = rs2.x + rs2.y;
        if constexpr (LPR >= 16) {
          rsv[i] = rs;
        } else {
#pragma unroll
          for (int o = 1; o < LPR; o <<= 1) rs += __shfl_xor(rs, o, 64);
          if (rowacc && i < nq) {   // column blocks: carry the row sum to the next block
            rs += rowacc[(size_t)i * n + r];
            if (!final && vl == 0) rowacc[(size_t)i * n + r] = rs;
          }
          rmax[i] = fmaxf(rmax[i], rs);
        }
      }
    }
    if constexpr (LPR >= 16) {
      // the row sums of all exponents at once: a transposing butterfly over
      // the LPR lanes of the row - each halving step keeps half of the
      // values (by the lane bit) and adds the partner's copy of them, so 16
      // values cost 16 lane exchanges instead of 16 log2(LPR); each lane ends
      // with the full row sum of ONE exponent (rs_j, j = rjl)
      rowsum_butterfly<LPR>(rsv, lane);
      float rs = rsv[0];
      if (rjl < nq) {
        if (rowacc) {   // column blocks: carry the row sum to the next block
          rs += rowacc[(size_t)rjl * n + r];
          if (!final && (lane & rj_dup) == 0) rowacc[(size_t)rjl * n + r] = rs;
        }
        rmax1 = fmaxf(rmax1, rs);
      }
    }
  }
  // row maxima: one atomic per exponent per wave (max is order-independent)
  if constexpr (LPR >= 16) {
    // lanes holding the same exponent: those differing in the bits the
    // butterfly did not halve on (rj_dup) and in the row-slot bits
    float m = rmax1;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1)
      if ((o & rj_dup) || o >= LPR) m = fmaxf(m, __shfl_xor(m, o, 64));
    if (final && rjl < nq && (lane & (rj_dup | ~(LPR - 1) & 63)) == 0) atomic_max_pos(&rowmax[rjl], m);
  } else {
#pragma unroll
    for (int i = 0; i < MUQ; ++i) {
      if (i < nq && final) {
        float m = rmax[i];
#pragma unroll
        for (int o = LPR; o < 64; o <<= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
        if (lane == 0) atomic_max_pos(&rowmax[i], m);
      }
    }
  }
  // column sums: reduce the 4*RPW row slots sharing a column group in LDS
  // (a constant trip count with unconditional barriers, so the loop unrolls:
  // a runtime-indexed cs would live in scratch)
#pragma unroll
  for (int i = 0; i < MUQ; ++i) {
    if (i < nq) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        red[tid * 8 + 2 * e] = cs[i][e].x;
        red[tid * 8 + 2 * e + 1] = cs[i][e].y;
      }
    }
    __syncthreads();
    if (i < nq && sg == 0) {     // threads 0..LPR-1: one per column group
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      for (int s2 = 0; s2 < 4 * RPW; ++s2) {
        const int t = s2 * LPR + vl;
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += red[t * 8 + e];
      }
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (c0 + e < d) part[((size_t)blockIdx.x * nq + i) * d_total + col0 + c0 + e] = acc[e];
    }
    __syncthreads();
  }
}

// colsum[i][c] = sum over WGs of part[wg][i][c] (fixed order)
__global__ void __launch_bounds__(256) mu_colsum_kernel(const float* __restrict__ part, int wgs,
                                                        int nq, int d, float* __restrict__ colsum) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= nq * d) return;
  float s = 0.f;
  for (int w = 0; w < wgs; ++w) s += part[(size_t)w * nq * d + idx];
  colsum[idx] = s;
}

template <typename T>
__global__ void __launch_bounds__(256) row_norms_kernel(const T* __restrict__ X, float* __restrict__ out,
                                                        long long n, int d) {
  // 16-byte vector loads; 4 rows per wave when d <= 128 elements-per-16B*16
  const int lane = threadIdx.x & 63;
  const long long r = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= n) return;
  constexpr int V = 16 / sizeof(T);
  const T* row = X + (size_t)r * d;
  float s = 0.f;
  const bool aligned = ((d * sizeof(T)) % 16 == 0);
  if (aligned) {
    for (int c = lane * V; c < d; c += 64 * V) {
      uint4 u = *reinterpret_cast<const uint4*>(row + c);
      uint32_t w[4] = {u.x, u.y, u.z, u.w};
      if constexpr (sizeof(T) == 2) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float lo = __uint_as_float(w[i] << 16), hi = __uint_as_float(w[i] & 0xFFFF0000u);
          s += lo * lo + hi * hi;
        }
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) { float v = __uint_as_float(w[i]); s += v * v; }
      }
    }
  } else {
    for (int c = lane; c < d; c += 64) {
      float v = ld1<T>(X, (size_t)r * d + c);
      s += v * v;
    }
  }
  s = wave_sum(s);
  if (lane == 0) out[r] = s;
}


// Column sums and sums of squares in fp64 (global_mean_var): one thread per
// column (a wave reads 64 consecutive features of a row), 8 rows in flight
// per thread; per-workgroup partials part[b][2 d] over the fixed row
// partition, summed in a fixed order by the caller (deterministic).
template <typename T>
__global__ void __launch_bounds__(256) col_moments_kernel(const T* __restrict__ X, long long ldx,
                                                          long long n, int d, long long rpw,
                                                          double* __restrict__ part) {
  const long long r0 = (long long)blockIdx.x * rpw;
  const long long r1 = min(n, r0 + rpw);
  for (int c = threadIdx.x; c < d; c += 256) {
    double s = 0.0, ss = 0.0;
    long long r = r0;
    for (; r + 8 <= r1; r += 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = ld1<T>(X, (size_t)(r + u) * ldx + c);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        s += (double)v[u];
        ss = fma((double)v[u], (double)v[u], ss);
      }
    }
    for (; r < r1; ++r) {
      const double v = (double)ld1<T>(X, (size_t)r * ldx + c);
      s += v;
      ss = fma(v, v, ss);
    }
    part[(size_t)blockIdx.x * 2 * d + c] = s;
    part[(size_t)blockIdx.x * 2 * d + d + c] = ss;
  }
}

}  // namespace sq

using namespace sq;

extern "C" {

// qstep > 0: the exponents are exactly 0, qstep, 2 qstep, ... (qs[i] = i qstep)
int sq_mu_sums(const void* X, int xdtype, long long ldx, const void* qs, int nq, void* rowmax,
               void* colsum, void* part, int part_wgs, void* rowacc, long long n, int d,
               const void* mean, float qstep, void* stream) {
  if (n <= 0) return 0;
  if (nq > MUQ || part_wgs < 1 || ldx < d || (d > 512 && !rowacc)) return (int)hipErrorInvalidValue;
  long long wgs = min((long long)part_wgs, max(1LL, (n + 255) / 256));
  long long rpw = (n + wgs - 1) / wgs;
  wgs = (n + rpw - 1) / rpw;
  hipStream_t st = (hipStream_t)stream;
  for (int col0 = 0; col0 < d; col0 += 512) {
    const int dc = d - col0 < 512 ? d - col0 : 512;
    const int final = col0 + 512 >= d;
    float* racc = d > 512 ? (float*)rowacc : nullptr;
    int lpr = 1;
    while (lpr * 8 < dc) lpr <<= 1;
#define MU_CASE(T, L)                                                                          \
  case L:                                                                                      \
    if (qstep > 0.f)                                                                           \
      hipLaunchKernelGGL((mu_sums_kernel<T, L, true>), dim3((unsigned)wgs), dim3(256), 0, st,  \
                         (const T*)X, ldx, col0, d, (const float*)qs, nq, (float*)rowmax,      \
                         (float*)part, racc, final, n, dc, rpw, (const float*)mean, qstep);    \
    else                                                                                       \
    hipLaunchKernelGGL((mu_sums_kernel<T, L, false>), dim3((unsigned)wgs), dim3(256), 0, st,   \
                       (const T*)X, ldx, col0, d, (const float*)qs, nq, (float*)rowmax,        \
                       (float*)part, racc, final, n, dc, rpw, (const float*)mean, qstep);      \
    break;
    if (xdtype == 0) {
      switch (lpr) { MU_CASE(float, 1) MU_CASE(float, 2) MU_CASE(float, 4) MU_CASE(float, 8)
                     MU_CASE(float, 16) MU_CASE(float, 32) MU_CASE(float, 64)
                     default: return (int)hipErrorInvalidValue; }
    } else if (xdtype == 2) {
      switch (lpr) { MU_CASE(uint16_t, 1) MU_CASE(uint16_t, 2) MU_CASE(uint16_t, 4)
                     MU_CASE(uint16_t, 8) MU_CASE(uint16_t, 16) MU_CASE(uint16_t, 32)
                     MU_CASE(uint16_t, 64) default: return (int)hipErrorInvalidValue; }
    } else {
      return (int)hipErrorInvalidValue;
    }
#undef MU_CASE
  }
  hipLaunchKernelGGL(mu_colsum_kernel, dim3((unsigned)((nq * d + 255) / 256)), dim3(256), 0, st,
                     (const float*)part, (int)wgs, nq, d, (float*)colsum);
  return (int)hipGetLastError();
}

// part fp64 [part_wgs][2 d], zero-initialised by the caller (the first wgs <= part_wgs rows
// are written)
int sq_col_moments(const void* X, int xdtype, long long ldx, long long n, int d, void* part,
                   int part_wgs, void* stream) {
  if (n <= 0 || d <= 0) return 0;
  if (part_wgs < 1 || ldx < d) return (int)hipErrorInvalidValue;
  long long wgs = min((long long)part_wgs, max(1LL, (n + 255) / 256));
  const long long rpw = (n + wgs - 1) / wgs;
  wgs = (n + rpw - 1) / rpw;
  hipStream_t st = (hipStream_t)stream;
  if (xdtype == 0)
    hipLaunchKernelGGL(col_moments_kernel<float>, dim3((unsigned)wgs), dim3(256), 0, st,
                       (const float*)X, ldx, n, d, rpw, (double*)part);
  else if (xdtype == 2)
    hipLaunchKernelGGL(col_moments_kernel<uint16_t>, dim3((unsigned)wgs), dim3(256), 0, st,
                       (const uint16_t*)X, ldx, n, d, rpw, (double*)part);
  else
    return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}

int sq_row_norms(const void* X, int xdtype, void* out, long long n, int d, void* stream) {
  if (n <= 0) return 0;
  unsigned grid = (unsigned)((n + 3) / 4);
  hipStream_t st = (hipStream_t)stream;
  if (xdtype == 0)
    hipLaunchKernelGGL(row_norms_kernel<float>, dim3(grid), dim3(256), 0, st, (const float*)X,
                       (float*)out, n, d);
  else if (xdtype == 2)
    hipLaunchKernelGGL(row_norms_kernel<uint16_t>, dim3(grid), dim3(256), 0, st,
                       (const uint16_t*)X, (float*)out, n, d);
  else
    return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}

}  // extern "C"
