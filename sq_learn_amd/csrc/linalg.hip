// Tall-skinny linear algebra for qPCA / q-means preludes (SURVEY.md §2.6
// K13-K15) on gfx950.
//
// gram       : G += (X-mu)^T (X-mu) over a row range, exact fp32 MFMA
//              (v_mfma_f32_16x16x4_f32); one pass over X, centring fused into
//              the LDS staging; upper-triangular 64x64 output tiles, split-K
//              over row ranges, per-split partial tiles summed in a fixed
//              order (no float atomics: deterministic).
// power_iter : Z += (X-mu)^T ((X-mu) Q) fused - the randomized range-finder
//              power iteration reads X once per iteration; Y never touches HBM
//              (phase 1 Y = Xc Q per wave -> LDS, phase 2 Z += Xc^T Y).
// mu_sums    : all exponents of the mu(A) p-grid in one pass
//              (row power sums -> max, column power sums) (Utility.py:196-231).
// row_norms  : ||x_i||^2 for bf16/fp32 rows.
#include "common.h"

namespace sq {

typedef __attribute__((ext_vector_type(4))) float f32x4;

template <typename T> SQ_DEV float ld1(const T* p, size_t i);
template <> SQ_DEV float ld1<float>(const float* p, size_t i) { return p[i]; }
template <> SQ_DEV float ld1<uint16_t>(const uint16_t* p, size_t i) { return bf16_to_f32(p[i]); }

// ------------------------------------------------------------------ gram
// tile 64x64 of G (features a0.., b0..), 4 waves each 32x32 (2x2 blocks 16x16)
// rows staged RS at a time: LDS A[RS][64+1], B[RS][64+1] fp32 (centred)
constexpr int GT = 64;
constexpr int GRS = 64;

template <typename T> SQ_DEV void ld4(const T* p, float v[4]);
template <> SQ_DEV void ld4<float>(const float* p, float v[4]) {
  float4 a = *reinterpret_cast<const float4*>(p);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
}
template <> SQ_DEV void ld4<uint16_t>(const uint16_t* p, float v[4]) {
  uint2 u = *reinterpret_cast<const uint2*>(p);
  v[0] = __uint_as_float(u.x << 16); v[1] = __uint_as_float(u.x & 0xFFFF0000u);
  v[2] = __uint_as_float(u.y << 16); v[3] = __uint_as_float(u.y & 0xFFFF0000u);
}

// G (upper tiles, then mirrored on the host) = sum over splits, fixed order
__global__ void __launch_bounds__(256) gram_reduce_kernel(const float* __restrict__ part,
                                                          int splits, int tiles, int side, int d,
                                                          float* __restrict__ G) {
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long long)tiles * GT * GT) return;
  const int tile0 = (int)(idx / (GT * GT));
  const int e = (int)(idx % (GT * GT));
  int tile = tile0, ta = 0;
  while (tile >= side - ta) { tile -= side - ta; ++ta; }
  const int tb = ta + tile;
  const int ra = ta * GT + e / GT, cb = tb * GT + e % GT;
  if (ra >= d || cb >= d) return;
  float s = 0.f;
  for (int sp = 0; sp < splits; ++sp) s += part[((size_t)sp * tiles + tile0) * GT * GT + e];
  G[(size_t)ra * d + cb] = s;
}

template <typename T>
__global__ void __launch_bounds__(256) gram_kernel(const T* __restrict__ X, float* __restrict__ part,
                                                   const float* __restrict__ mean, long long n,
                                                   int d, int n_tiles_side, long long rows_per_split) {
  const bool vec4 = (d % 4) == 0;
  __shared__ float As[GRS][GT + 1];
  __shared__ float Bs[GRS][GT + 1];
  // decode upper-triangular tile id
  int tile = blockIdx.x;
  int ta = 0;
  while (tile >= n_tiles_side - ta) { tile -= n_tiles_side - ta; ++ta; }
  int tb = ta + tile;
  const int a0 = ta * GT, b0 = tb * GT;
  const long long r_beg = (long long)blockIdx.y * rows_per_split;
  const long long r_end = min(n, r_beg + rows_per_split);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wa = (wave >> 1) * 32, wb = (wave & 1) * 32;
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  for (long long r = r_beg; r < r_end; r += GRS) {
    // stage: 4 consecutive features per thread (vector loads when aligned)
    for (int e = tid * 4; e < GRS * GT; e += 256 * 4) {
      const int rr = e / GT, c = e % GT;
      const long long row = r + rr;
      float va[4] = {0.f, 0.f, 0.f, 0.f}, vb[4] = {0.f, 0.f, 0.f, 0.f};
      if (row < r_end) {
        const T* xr = X + (size_t)row * d;
        if (vec4 && a0 + c + 4 <= d) {
          ld4<T>(xr + a0 + c, va);
#pragma unroll
          for (int q = 0; q < 4; ++q) va[q] -= mean[a0 + c + q];
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q)
            if (a0 + c + q < d) va[q] = ld1<T>(xr, a0 + c + q) - mean[a0 + c + q];
        }
        if (vec4 && b0 + c + 4 <= d) {
          ld4<T>(xr + b0 + c, vb);
#pragma unroll
          for (int q = 0; q < 4; ++q) vb[q] -= mean[b0 + c + q];
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q)
            if (b0 + c + q < d) vb[q] = ld1<T>(xr, b0 + c + q) - mean[b0 + c + q];
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) { As[rr][c + q] = va[q]; Bs[rr][c + q] = vb[q]; }
    }
    __syncthreads();
#pragma unroll 4
    for (int k = 0; k < GRS; k += 4) {
      const int kr = k + (lane >> 4);
      float av[2], bv[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) av[i] = As[kr][wa + i * 16 + (lane & 15)];
#pragma unroll
      for (int j = 0; j < 2; ++j) bv[j] = Bs[kr][wb + j * 16 + (lane & 15)];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i], bv[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }
  // C/D map 16x16: col = lane&15, row = (lane>>4)*4 + reg
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        // per-split partial tile (no atomics); gram_reduce_kernel sums the
        // splits in a fixed order -> deterministic Gram matrix
        const int la = wa + i * 16 + (lane >> 4) * 4 + g;
        const int lb = wb + j * 16 + (lane & 15);
        part[(((size_t)blockIdx.y * gridDim.x + blockIdx.x) * GT + la) * GT + lb] = acc[i][j][g];
      }
}

// ------------------------------------------------------------ power_iter
// 64 rows per step: wave w computes Y[16w..16w+15][0..l) = Xc Q, writes LDS;
// then wave w accumulates Z[f in group w][0..l) += Xc^T Y over the 64 rows.
template <typename T, int DP, int LP>
__global__ void __launch_bounds__(256, 1) power_iter_kernel(
    const T* __restrict__ X, const float* __restrict__ Q, float* __restrict__ Z,
    const float* __restrict__ mean, long long n, int d, int l, long long rows_per_wg) {
  constexpr int RS = 64;
  constexpr int XP = DP + 1;           // padded row (bank-conflict-free column reads)
  constexpr int YP = LP + 1;
  constexpr int FB = DP / 16 / 4;      // f-blocks (16 wide) per wave
  constexpr int LB = LP / 16;          // l-blocks per wave
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* Xs = sm;                      // [RS][XP]
  float* Qs = Xs + RS * XP;            // [DP][LP]
  float* Ys = Qs + DP * LP;            // [RS][YP]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int e = tid; e < DP * LP; e += 256) {
    int f = e / LP, c = e % LP;
    Qs[e] = (f < d && c < l) ? Q[(size_t)f * l + c] : 0.f;
  }
  f32x4 z[FB][LB];
#pragma unroll
  for (int i = 0; i < FB; ++i)
#pragma unroll
    for (int j = 0; j < LB; ++j) z[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const long long r_beg = (long long)blockIdx.x * rows_per_wg;
  const long long r_end = min(n, r_beg + rows_per_wg);
  for (long long r = r_beg; r < r_end; r += RS) {
    __syncthreads();
    for (int e = tid; e < RS * DP; e += 256) {
      int rr = e / DP, c = e % DP;
      long long row = r + rr;
      float v = 0.f;
      if (row < r_end && c < d) v = ld1<T>(X, (size_t)row * d + c) - mean[c];
      Xs[rr * XP + c] = v;
    }
    __syncthreads();
    // phase 1: Y[16 rows of wave][LP]
    {
      f32x4 y[LB];
#pragma unroll
      for (int j = 0; j < LB; ++j) y[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
      const int yr = wave * 16 + (lane & 15);
      for (int k = 0; k < DP; k += 4) {
        const int kf = k + (lane >> 4);
        float av = Xs[yr * XP + kf];
#pragma unroll
        for (int j = 0; j < LB; ++j) {
          float bv = Qs[kf * LP + j * 16 + (lane & 15)];
          y[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, y[j], 0, 0, 0);
        }
      }
#pragma unroll
      for (int j = 0; j < LB; ++j)
#pragma unroll
        for (int g = 0; g < 4; ++g)
          Ys[(wave * 16 + (lane >> 4) * 4 + g) * YP + j * 16 + (lane & 15)] = y[j][g];
    }
    __syncthreads();
    // phase 2: Z[f][c] += sum_rows Xc[row][f] Y[row][c]
    for (int k = 0; k < RS; k += 4) {
      const int kr = k + (lane >> 4);
      float bv[LB];
#pragma unroll
      for (int j = 0; j < LB; ++j) bv[j] = Ys[kr * YP + j * 16 + (lane & 15)];
#pragma unroll
      for (int i = 0; i < FB; ++i) {
        float av = Xs[kr * XP + (wave * FB + i) * 16 + (lane & 15)];
#pragma unroll
        for (int j = 0; j < LB; ++j)
          z[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv[j], z[i][j], 0, 0, 0);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < FB; ++i)
#pragma unroll
    for (int j = 0; j < LB; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        int f = (wave * FB + i) * 16 + (lane >> 4) * 4 + g;
        int c = j * 16 + (lane & 15);
        // per-WG partial (no atomics): summed in a fixed order by pi_reduce_kernel
        if (f < d && c < l) Z[((size_t)blockIdx.x * d + f) * l + c] = z[i][j][g];
      }
}

__global__ void __launch_bounds__(256) pi_reduce_kernel(const float* __restrict__ part, int wgs,
                                                        int dl, float* __restrict__ Z) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= dl) return;
  float s = 0.f;
  for (int w = 0; w < wgs; ++w) s += part[(size_t)w * dl + idx];
  Z[idx] = s;
}

// ------------------------------------------------------------------ mu
// Power sums of |a|^q for a p-grid of exponents (mu(A), Utility.py:196-231):
// rowmax[i] = max_r sum_c |a_rc|^q_i, colsum[i][c] = sum_r |a_rc|^q_i.
// Lanes own 8 consecutive columns; LPR = ceil(d/8) (power of two) lanes per
// row, so a wave covers 64/LPR rows at once (no idle lanes for d < 256).
// One v_log per element, one v_exp per (element, exponent); row sums by
// log2(LPR) xor-shuffles; column sums reduced in LDS per workgroup and
// written as per-WG partials, summed by mu_colsum_kernel in a fixed order
// (no float atomics: deterministic).
constexpr int MUQ = 12;

template <typename T>
SQ_DEV void ld8abs(const T* p, bool full, int valid, float v[8]);
template <>
SQ_DEV void ld8abs<uint16_t>(const uint16_t* p, bool full, int valid, float v[8]) {
  if (full) {
    uint4 u = *reinterpret_cast<const uint4*>(p);
    uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[2 * e] = fabsf(__uint_as_float(w[e] << 16));
      v[2 * e + 1] = fabsf(__uint_as_float(w[e] & 0xFFFF0000u));
    }
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = e < valid ? fabsf(bf16_to_f32(p[e])) : 0.f;
  }
}
template <>
SQ_DEV void ld8abs<float>(const float* p, bool full, int valid, float v[8]) {
  if (full) {
    float4 a = *reinterpret_cast<const float4*>(p);
    float4 b = *reinterpret_cast<const float4*>(p + 4);
    v[0] = fabsf(a.x); v[1] = fabsf(a.y); v[2] = fabsf(a.z); v[3] = fabsf(a.w);
    v[4] = fabsf(b.x); v[5] = fabsf(b.y); v[6] = fabsf(b.z); v[7] = fabsf(b.w);
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = e < valid ? fabsf(p[e]) : 0.f;
  }
}

template <typename T, int LPR>
__global__ void __launch_bounds__(256) mu_sums_kernel(
    const T* __restrict__ X, const float* __restrict__ qs, int nq, float* __restrict__ rowmax,
    float* __restrict__ part, long long n, int d, long long rows_per_wg) {
  constexpr int RPW = 64 / LPR;              // rows per wave step
  __shared__ float red[256 * 8];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int vl = lane % LPR;                  // column group of this lane
  const int sg = (wave * 64 + lane) / LPR;    // row slot within the WG (0 .. 4*RPW-1)
  const int c0 = vl * 8;
  const bool vec = ((d % 8) == 0) && (c0 + 8 <= d);
  const int valid = d - c0;
  float q[MUQ];
#pragma unroll
  for (int i = 0; i < MUQ; ++i) q[i] = i < nq ? qs[i] : 0.f;
  float cs[MUQ][8], rmax[MUQ];
#pragma unroll
  for (int i = 0; i < MUQ; ++i) {
    rmax[i] = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) cs[i][e] = 0.f;
  }
  const long long r_beg = (long long)blockIdx.x * rows_per_wg;
  const long long r_end = min(n, r_beg + rows_per_wg);
  for (long long r = r_beg + sg; r < r_end; r += 4 * RPW) {
    float v[8], lg[8];
    if (c0 < d) ld8abs<T>(X + (size_t)r * d + c0, vec, valid, v);
    else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = 0.f;
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) lg[e] = __builtin_amdgcn_logf(v[e]);   // log2, -inf at 0
#pragma unroll
    for (int i = 0; i < MUQ; ++i) {
      if (i < nq) {
        float rs = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          // |a|^0 counts nonzeros; exp2(q * -inf) = 0 for q > 0
          const float pw = q[i] == 0.f ? (v[e] != 0.f ? 1.f : 0.f)
                                        : __builtin_amdgcn_exp2f(q[i] * lg[e]);
          cs[i][e] += pw;
          rs += pw;
        }
#pragma unroll
        for (int o = 1; o < LPR; o <<= 1) rs += __shfl_xor(rs, o, 64);
        rmax[i] = fmaxf(rmax[i], rs);
      }
    }
  }
  // row maxima: one atomic per exponent per wave (max is order-independent)
#pragma unroll
  for (int i = 0; i < MUQ; ++i) {
    if (i < nq) {
      float m = rmax[i];
#pragma unroll
      for (int o = LPR; o < 64; o <<= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
      if (lane == 0) atomic_max_pos(&rowmax[i], m);
    }
  }
  // column sums: reduce the 4*RPW row slots sharing a column group in LDS
  for (int i = 0; i < nq; ++i) {
#pragma unroll
    for (int e = 0; e < 8; ++e) red[tid * 8 + e] = cs[i][e];
    __syncthreads();
    if (sg == 0) {               // threads 0..LPR-1: one per column group
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      for (int s2 = 0; s2 < 4 * RPW; ++s2) {
        const int t = s2 * LPR + vl;
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += red[t * 8 + e];
      }
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (c0 + e < d) part[((size_t)blockIdx.x * nq + i) * d + c0 + e] = acc[e];
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

}  // namespace sq

using namespace sq;

template <typename T, int DP, int LP>
static int launch_pi(const void* X, const void* Q, void* Z, const void* mean, long long n, int d,
                     int l, void* part, int part_wgs, hipStream_t st) {
  size_t lds = ((size_t)64 * (DP + 1) + (size_t)DP * LP + (size_t)64 * (LP + 1)) * 4;
  auto kern = power_iter_kernel<T, DP, LP>;
  hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  long long wgs = min((long long)part_wgs, max(1LL, (n + 1023) / 1024));
  long long rpw = ((n + wgs - 1) / wgs + 63) / 64 * 64;
  wgs = (n + rpw - 1) / rpw;
  hipLaunchKernelGGL(kern, dim3((unsigned)wgs), dim3(256), lds, st, (const T*)X, (const float*)Q,
                     (float*)part, (const float*)mean, n, d, l, rpw);
  hipLaunchKernelGGL(pi_reduce_kernel, dim3((unsigned)((d * l + 255) / 256)), dim3(256), 0, st,
                     (const float*)part, (int)wgs, d * l, (float*)Z);
  return (int)hipGetLastError();
}

extern "C" {

int sq_gram_bf16(const void* X, int xdtype, void* G, const void* mean, long long n, int d,
                 void* part, long long part_cap, void* stream) {
  if (n <= 0) return 0;
  int side = (d + GT - 1) / GT;
  int tiles = side * (side + 1) / 2;
  int splits = (int)max(1LL, min(2048LL / tiles, (n + 4095) / 4096));
  splits = (int)min((long long)splits, max(1LL, part_cap / ((long long)tiles * GT * GT)));
  long long rps = ((n + splits - 1) / splits + GRS - 1) / GRS * GRS;
  splits = (int)((n + rps - 1) / rps);
  if ((long long)splits * tiles * GT * GT > part_cap) return (int)hipErrorInvalidValue;
  dim3 grid(tiles, splits);
  hipStream_t st = (hipStream_t)stream;
  if (xdtype == 0)
    hipLaunchKernelGGL(gram_kernel<float>, grid, dim3(256), 0, st, (const float*)X, (float*)part,
                       (const float*)mean, n, d, side, rps);
  else if (xdtype == 2)
    hipLaunchKernelGGL(gram_kernel<uint16_t>, grid, dim3(256), 0, st, (const uint16_t*)X,
                       (float*)part, (const float*)mean, n, d, side, rps);
  else
    return (int)hipErrorInvalidValue;
  long long tot = (long long)tiles * GT * GT;
  hipLaunchKernelGGL(gram_reduce_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st,
                     (const float*)part, splits, tiles, side, d, (float*)G);
  return (int)hipGetLastError();
}

int sq_power_iter(const void* X, int xdtype, const void* Q, void* Z, const void* mean, long long n,
                  int d, int l, void* part, int part_wgs, void* stream) {
  if (n <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (l > 64 || d > 256 || part_wgs < 1) return (int)hipErrorInvalidValue;
  int DP = d <= 64 ? 64 : (d <= 128 ? 128 : 256);
  int LP = l <= 16 ? 16 : (l <= 32 ? 32 : 64);
#define PI_CASE(TT, D_, L_) \
  if (DP == D_ && LP == L_) return launch_pi<TT, D_, L_>(X, Q, Z, mean, n, d, l, part, part_wgs, st);
  if (xdtype == 0) {
    PI_CASE(float, 64, 16) PI_CASE(float, 64, 32) PI_CASE(float, 64, 64)
    PI_CASE(float, 128, 16) PI_CASE(float, 128, 32) PI_CASE(float, 128, 64)
    PI_CASE(float, 256, 16) PI_CASE(float, 256, 32) PI_CASE(float, 256, 64)
  } else if (xdtype == 2) {
    PI_CASE(uint16_t, 64, 16) PI_CASE(uint16_t, 64, 32) PI_CASE(uint16_t, 64, 64)
    PI_CASE(uint16_t, 128, 16) PI_CASE(uint16_t, 128, 32) PI_CASE(uint16_t, 128, 64)
    PI_CASE(uint16_t, 256, 16) PI_CASE(uint16_t, 256, 32) PI_CASE(uint16_t, 256, 64)
  }
#undef PI_CASE
  return (int)hipErrorInvalidValue;
}

int sq_mu_sums(const void* X, int xdtype, const void* qs, int nq, void* rowmax, void* colsum,
               void* part, int part_wgs, long long n, int d, void* stream) {
  if (n <= 0) return 0;
  if (nq > MUQ || d > 256 || part_wgs < 1) return (int)hipErrorInvalidValue;
  long long wgs = min((long long)part_wgs, max(1LL, (n + 255) / 256));
  long long rpw = (n + wgs - 1) / wgs;
  wgs = (n + rpw - 1) / rpw;
  hipStream_t st = (hipStream_t)stream;
  int lpr = 1;
  while (lpr * 8 < d) lpr <<= 1;
#define MU_CASE(T, L)                                                                          \
  case L:                                                                                      \
    hipLaunchKernelGGL((mu_sums_kernel<T, L>), dim3((unsigned)wgs), dim3(256), 0, st,          \
                       (const T*)X, (const float*)qs, nq, (float*)rowmax, (float*)part, n, d,  \
                       rpw);                                                                   \
    break;
  if (xdtype == 0) {
    switch (lpr) { MU_CASE(float, 1) MU_CASE(float, 2) MU_CASE(float, 4) MU_CASE(float, 8)
                   MU_CASE(float, 16) MU_CASE(float, 32) default: return (int)hipErrorInvalidValue; }
  } else if (xdtype == 2) {
    switch (lpr) { MU_CASE(uint16_t, 1) MU_CASE(uint16_t, 2) MU_CASE(uint16_t, 4)
                   MU_CASE(uint16_t, 8) MU_CASE(uint16_t, 16) MU_CASE(uint16_t, 32)
                   default: return (int)hipErrorInvalidValue; }
  } else {
    return (int)hipErrorInvalidValue;
  }
#undef MU_CASE
  hipLaunchKernelGGL(mu_colsum_kernel, dim3((unsigned)((nq * d + 255) / 256)), dim3(256), 0, st,
                     (const float*)part, (int)wgs, nq, d, (float*)colsum);
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
