// Non-GEMM pairwise reductions (reference
// ``metrics/_pairwise_fast.pyx``: ``_chi2_kernel_fast``; the
// ``pairwise_distances`` manhattan / chebyshev / minkowski metrics).
//
//   op 0  L1          sum |x - y|
//   op 1  additive chi2   -sum (x - y)^2 / (x + y)   (terms with x + y = 0 skipped)
//   op 2  chebyshev   max |x - y|
//   op 3  minkowski   (sum |x - y|^p)^(1/p)
//
// These are elementwise-then-reduce over the feature axis, so no MFMA: a
// register-blocked tile kernel.  A 256-thread workgroup owns a 64 x 64 output
// tile; X and Y rows are staged through LDS 32 features at a time (row-major
// with one padding column, so the per-thread column reads are conflict-free),
// and each thread accumulates a 4 x 4 sub-block in registers.
#include "common.h"

namespace sq {

constexpr int PT = 64;   // output tile edge
constexpr int PK = 32;   // features per LDS stage

template <typename T, int OP>
__device__ __forceinline__ T pw_term(T x, T y, T p) {
  if constexpr (OP == 0) return fabs(x - y);
  if constexpr (OP == 1) {
    const T s = x + y;
    return s != T(0) ? -(x - y) * (x - y) / s : T(0);
  }
  if constexpr (OP == 2) return fabs(x - y);
  return pow(fabs(x - y), p);
}

template <typename T, int OP>
__global__ void __launch_bounds__(256) pairwise_tile_kernel(const T* __restrict__ X,
                                                            const T* __restrict__ Y,
                                                            T* __restrict__ out, int n, int m,
                                                            int d, T p) {
  __shared__ T xs[PT][PK + 1];
  __shared__ T ys[PT][PK + 1];
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const int i0 = blockIdx.y * PT, j0 = blockIdx.x * PT;
  T acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = T(0);
  for (int k0 = 0; k0 < d; k0 += PK) {
    for (int t = threadIdx.x; t < PT * PK; t += 256) {
      const int r = t / PK, c = t % PK;
      const int gi = i0 + r, gj = j0 + r, gk = k0 + c;
      xs[r][c] = (gi < n && gk < d) ? X[(size_t)gi * d + gk] : T(0);
      ys[r][c] = (gj < m && gk < d) ? Y[(size_t)gj * d + gk] : T(0);
    }
    __syncthreads();
    const int kk = min(PK, d - k0);
    for (int c = 0; c < kk; ++c) {
      T xv[4], yv[4];
#pragma unroll
      for (int a = 0; a < 4; ++a) xv[a] = xs[ty + 16 * a][c];
#pragma unroll
      for (int b = 0; b < 4; ++b) yv[b] = ys[tx + 16 * b][c];
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const T v = pw_term<T, OP>(xv[a], yv[b], p);
          if constexpr (OP == 2)
            acc[a][b] = fmax(acc[a][b], v);
          else
            acc[a][b] += v;
        }
    }
    __syncthreads();
  }
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const int gi = i0 + ty + 16 * a;
    if (gi >= n) continue;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int gj = j0 + tx + 16 * b;
      if (gj >= m) continue;
      T v = acc[a][b];
      if constexpr (OP == 3) v = pow(v, T(1) / p);
      out[(size_t)gi * m + gj] = v;
    }
  }
}

template <typename T>
static int launch_pairwise(const void* X, const void* Y, void* out, int n, int m, int d, int op,
                           double p, hipStream_t s) {
  dim3 grid((unsigned)((m + PT - 1) / PT), (unsigned)((n + PT - 1) / PT));
  const T pp = (T)p;
  switch (op) {
    case 0: hipLaunchKernelGGL((pairwise_tile_kernel<T, 0>), grid, dim3(256), 0, s, (const T*)X, (const T*)Y, (T*)out, n, m, d, pp); break;
    case 1: hipLaunchKernelGGL((pairwise_tile_kernel<T, 1>), grid, dim3(256), 0, s, (const T*)X, (const T*)Y, (T*)out, n, m, d, pp); break;
    case 2: hipLaunchKernelGGL((pairwise_tile_kernel<T, 2>), grid, dim3(256), 0, s, (const T*)X, (const T*)Y, (T*)out, n, m, d, pp); break;
    case 3: hipLaunchKernelGGL((pairwise_tile_kernel<T, 3>), grid, dim3(256), 0, s, (const T*)X, (const T*)Y, (T*)out, n, m, d, pp); break;
    default: return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

}  // namespace sq

using namespace sq;

// dtype 0 = fp32, 1 = fp64; X (n, d), Y (m, d) row-major, out (n, m)
extern "C" int sq_pairwise_reduce(const void* X, const void* Y, void* out, int n, int m, int d,
                                  int op, double p, int dtype, void* stream) {
  if (n <= 0 || m <= 0) return 0;
  if (d < 0 || op < 0 || op > 3) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == 0) return launch_pairwise<float>(X, Y, out, n, m, d, op, p, s);
  if (dtype == 1) return launch_pairwise<double>(X, Y, out, n, m, d, op, p, s);
  return (int)hipErrorInvalidValue;
}
