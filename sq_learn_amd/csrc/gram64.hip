// fp64 Gram on the matrix cores: G = (X - mu)^T (X - mu) accumulated with
// v_mfma_f64_16x16x4_f64 (the reference's fp64 LAPACK
// precision for sigma_min, the condition number and the qPCA spectrum,
// ``_dmeans.py:1244-1245``, ``_qPCA.py:581``).  The building block of the
// sharded CholeskyQR2 in ops/linalg.py (pass 1 on X, pass 2 on X R1^-1).
//
// X is fp32 / bf16 (products of their values are exact in fp64) or fp64; d <= 256
// (padded to a multiple of 16: NB column blocks, NB (NB + 1) / 2 upper
// 16 x 16 blocks of G).  A workgroup of 8 waves streams its contiguous row
// range in k-steps of 4 rows; the 16-column fragment of block b for the
// k-step - lane l: X[r0 + (l >> 4)][16 b + (l & 15)] - is BOTH the A operand
// (A[i][k] = X[r0+k][16 bi + i]) of block row bi and the B operand of block
// column bj; a wave loads its fragments of a k-step (L1/L2: the 8 waves
// read the same rows) and runs its NB + 1 block MFMAs on them; the second
// wave of each SIMD covers the load latency of the first.
// Each workgroup writes its partial upper blocks; the host side sums the
// partials in a fixed order (deterministic).  f64 C/D layout: lane l,
// register r -> (row (l >> 4) + 4 r, col l & 15).
#include "common.h"
#include <type_traits>

namespace sq {

typedef double f64x4 __attribute__((ext_vector_type(4)));

SQ_DEV double to_f64(float v) { return (double)v; }
SQ_DEV double to_f64(double v) { return v; }
SQ_DEV double to_f64(uint16_t v) { return (double)bf16_to_f32(v); }   // bf16 bits

// Block assignment: wave w < ceil(NB/2) owns upper-block rows w and NB-1-w
// (NB - w + w + 1 = NB + 1 blocks; the middle row of odd NB once): slot t <
// NB - w is block (w, w + t), slot t >= NB - w is block (NB-1-w, t - 1).
// The A operand of a slot is one of two row fragments (a wave-uniform
// select), its B operand the fragment of the slot's column block, loaded
// straight from memory (runtime column, no register-array indexing).
template <typename T, int NB, bool HAS_MU>
__global__ void __launch_bounds__(512) gram64_kernel(const T* __restrict__ X, long long ldx,
                                                     const double* __restrict__ mu, long long n,
                                                     int d, double* __restrict__ part) {
  constexpr int SLOTS = NB + 1;
  constexpr int NBLK = NB * (NB + 1) / 2;
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int c16 = lane & 15, q4 = lane >> 4;
  // the mean in LDS (read per MFMA operand by the two-k-step path: 2 x 17
  // fp64 registers saved), filled before any wave leaves
  __shared__ double smu[16 * NB];
  if (HAS_MU) {
    for (int c = threadIdx.x; c < 16 * NB; c += blockDim.x) smu[c] = c < d ? mu[c] : 0.0;
    __syncthreads();
  }
  if (w >= (NB + 1) / 2) return;   // wave-uniform; no block barrier below
  const int i1 = w, i2 = NB - 1 - w;
  const int n1 = NB - w;                         // slots of row i1
  const int nslot = (i1 == i2) ? n1 : SLOTS;     // odd NB: middle row once
  const long long per = (n + gridDim.x - 1) / gridDim.x;
  const long long r_begin = (long long)blockIdx.x * per;
  const long long r_end = r_begin + per < n ? r_begin + per : n;
  auto colblk = [&](int t) { return t < n1 ? w + t : t - 1; };
  f64x4 acc[SLOTS];
#pragma unroll
  for (int t = 0; t < SLOTS; ++t) acc[t] = (f64x4){0.0, 0.0, 0.0, 0.0};
  // the raw values of TWO k-steps are loaded together (8 rows in flight per
  // wave; fp32 / bf16 input: 2 x 19 raw fp32 registers - the fp64 copies of
  // both would not fit 2 waves / SIMD) and widened / centred right before
  // their MFMAs; no runtime-indexed register arrays (those live in scratch)
  using R = typename std::conditional<sizeof(T) == 8, double, float>::type;
  R rA[SLOTS], rB[SLOTS], a1A, a2A, a1B, a2B;
  for (long long r0 = r_begin; r0 < r_end; r0 += 8) {
    const long long ra = r0 + q4, rb = r0 + 4 + q4;
    const bool okA = ra < r_end, okB = rb < r_end;
    const T* xa = X + (size_t)(okA ? ra : r_begin) * ldx;
    const T* xb = X + (size_t)(okB ? rb : r_begin) * ldx;
#pragma unroll
    for (int t = 0; t < SLOTS; ++t) {
      const int col = 16 * colblk(t) + c16;
      const bool live = t < nslot && col < d;
      rA[t] = live && okA ? (R)to_f64(xa[col]) : (R)0;
      rB[t] = live && okB ? (R)to_f64(xb[col]) : (R)0;
    }
    const int c1 = 16 * i1 + c16, c2 = 16 * i2 + c16;
    a1A = c1 < d && okA ? (R)to_f64(xa[c1]) : (R)0;
    a2A = c2 < d && okA ? (R)to_f64(xa[c2]) : (R)0;
    a1B = c1 < d && okB ? (R)to_f64(xb[c1]) : (R)0;
    a2B = c2 < d && okB ? (R)to_f64(xb[c2]) : (R)0;
    {
      const double fa1 = okA && c1 < d ? (double)a1A - (HAS_MU ? smu[c1] : 0.0) : 0.0;
      const double fa2 = okA && c2 < d ? (double)a2A - (HAS_MU ? smu[c2] : 0.0) : 0.0;
#pragma unroll
      for (int t = 0; t < SLOTS; ++t) {
        if (t < nslot) {
          const double a = t < n1 ? fa1 : fa2;
          const int cb = 16 * colblk(t) + c16;
          const double b = okA && cb < d ? (double)rA[t] - (HAS_MU ? smu[cb] : 0.0) : 0.0;
          acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[t], 0, 0, 0);
        }
      }
    }
    {
      const double fa1 = okB && c1 < d ? (double)a1B - (HAS_MU ? smu[c1] : 0.0) : 0.0;
      const double fa2 = okB && c2 < d ? (double)a2B - (HAS_MU ? smu[c2] : 0.0) : 0.0;
#pragma unroll
      for (int t = 0; t < SLOTS; ++t) {
        if (t < nslot) {
          const double a = t < n1 ? fa1 : fa2;
          const int cb = 16 * colblk(t) + c16;
          const double b = okB && cb < d ? (double)rB[t] - (HAS_MU ? smu[cb] : 0.0) : 0.0;
          acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[t], 0, 0, 0);
        }
      }
    }
  }
  // partial upper blocks of this workgroup: block (bi, bj) at linear id
  // bi * NB - bi (bi - 1) / 2 + (bj - bi)
  double* out = part + (size_t)blockIdx.x * NBLK * 256;
#pragma unroll
  for (int t = 0; t < SLOTS; ++t) {
    if (t < nslot) {
      const int bi = t < n1 ? i1 : i2;
      const int bj = colblk(t);
      const int id = bi * NB - bi * (bi - 1) / 2 + (bj - bi);
#pragma unroll
      for (int r = 0; r < 4; ++r) out[(size_t)id * 256 + (q4 + 4 * r) * 16 + c16] = acc[t][r];
    }
  }
}

}  // namespace sq

using namespace sq;

template <typename T>
static int launch_gram64(const T* X, long long ldx, const double* mu, long long n, int d,
                         double* part, int grid, hipStream_t st) {
  const int nb = (d + 15) / 16;
  switch (nb) {
#define CASE(NB)                                                                        \
  case NB:                                                                              \
    if (mu)                                                                             \
      hipLaunchKernelGGL((gram64_kernel<T, NB, true>), dim3(grid), dim3(512), 0, st, X, ldx, \
                         mu, n, d, part);                                               \
    else                                                                                \
      hipLaunchKernelGGL((gram64_kernel<T, NB, false>), dim3(grid), dim3(512), 0, st, X,     \
                         ldx, mu, n, d, part);                                          \
    break;
    CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8)
    CASE(9) CASE(10) CASE(11) CASE(12) CASE(13) CASE(14) CASE(15) CASE(16)
#undef CASE
    default:
      return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

// dtype: 0 fp32, 1 fp64, 2 bf16
extern "C" int sq_gram64(const void* X, int is_f64, long long ldx, const void* mu, long long n,
                         int d, void* part, int grid, void* stream) {
  if (n <= 0) return 0;
  if (d < 1 || d > 256 || grid < 1 || ldx < d) return (int)hipErrorInvalidValue;
  if (is_f64 == 2)
    return launch_gram64((const uint16_t*)X, ldx, (const double*)mu, n, d, (double*)part, grid,
                         (hipStream_t)stream);
  if (is_f64)
    return launch_gram64((const double*)X, ldx, (const double*)mu, n, d, (double*)part, grid,
                         (hipStream_t)stream);
  return launch_gram64((const float*)X, ldx, (const double*)mu, n, d, (double*)part, grid,
                       (hipStream_t)stream);
}
