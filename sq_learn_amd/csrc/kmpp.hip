// Greedy k-means++ trial pass (reference sklearn/cluster/
// _kmeans.py:153-247 and _dmeans.py:153-247): for the t candidate centres of
// one step, every row's squared distance to each candidate and the t trial
// potentials  sum_i w_i min(closest_i, |x_i - c_t|^2)  in ONE pass over X.
//
// The step is HBM-bound (k - 1 sequential passes over the whole matrix, t
// <= 16 candidates, 2 t flops per loaded byte), so the kernel is shaped for
// the stream: a wave owns 64 rows (one per lane for the arithmetic), loads
// them as coalesced 32-feature tiles (8 rows x 128 B per load instruction,
// next tile prefetched into registers while the current one is consumed)
// and transposes them through its own LDS slot; the candidates are
// wave-uniform (scalar loads / SGPR operands), direct-form fp32
// distances sum_f (x_f - c_f)^2 (no |x|^2 + |c|^2 - 2 x.c cancellation), fp64
// potential partials per block in a fixed order (deterministic), and the
// distances written transposed D[t][n] so the caller picks the winning
// trial's column contiguously.  Replaces a library GEMM + ~6 torch
// elementwise passes over [n, t] temporaries per centre.
#include "common.h"

namespace sq {

constexpr int kKppTile = 32;          // features per staged tile (128 B of a row)
constexpr int kKppStride = 36;        // LDS row stride in floats (16-B aligned, skewed banks)

template <int TMAX>
__global__ void __launch_bounds__(256) kmpp_trials_kernel(
    const float* __restrict__ X, long long ldx, int d, long long n, int t,
    const float* __restrict__ cand, const double* __restrict__ closest,
    const double* __restrict__ w, float* __restrict__ D, double* __restrict__ part) {
  __shared__ double red[4][TMAX];
  __shared__ __attribute__((aligned(16))) float tile[4][64 * kKppStride];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float* my = tile[wave];
  double pot[TMAX];
#pragma unroll
  for (int j = 0; j < TMAX; ++j) pot[j] = 0.0;
  const long long nblk = (n + 63) / 64;                      // 64-row groups, one per wave pass
  const long long wstride = (long long)gridDim.x * 4;
  const int ntiles = (d + kKppTile - 1) / kKppTile;
  // coalesced tile load: lane -> (row r0 + 8 q + (lane >> 3), 16-B chunk lane & 7)
  const int lrow = lane >> 3, lchunk = lane & 7;
  float4 nxt[8];
  auto load_tile = [&](long long r0, int tix) {
    const int f = tix * kKppTile + lchunk * 4;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      long long r = r0 + q * 8 + lrow;
      r = r < n ? r : n - 1;
      nxt[q] = f < d ? *reinterpret_cast<const float4*>(X + r * ldx + f)
                     : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  long long g = (long long)blockIdx.x * 4 + wave;
  if (g < nblk) load_tile(g * 64, 0);
  for (; g < nblk; g += wstride) {
    const long long r0 = g * 64;
    const long long i = r0 + lane;
    float acc[TMAX];
#pragma unroll
    for (int j = 0; j < TMAX; ++j) acc[j] = 0.0f;
    for (int tix = 0; tix < ntiles; ++tix) {
      // stage the landed tile (in-order LDS within the wave: no barrier)
#pragma unroll
      for (int q = 0; q < 8; ++q)
        *reinterpret_cast<float4*>(my + (q * 8 + lrow) * kKppStride + lchunk * 4) = nxt[q];
      // prefetch the next tile (or the next row group's first tile)
      if (tix + 1 < ntiles) load_tile(r0, tix + 1);
      else if (g + wstride < nblk) load_tile((g + wstride) * 64, 0);
      const int f0 = tix * kKppTile;
      const int fl = min(kKppTile, d - f0);
#pragma unroll
      for (int c4 = 0; c4 < kKppTile / 4; ++c4) {
        if (c4 * 4 >= fl) break;
        const float4 x4 = *reinterpret_cast<const float4*>(my + lane * kKppStride + c4 * 4);
        const int f = f0 + c4 * 4;
#pragma unroll
        for (int j = 0; j < TMAX; ++j) {
          if (j < t) {
            const float* c = cand + (size_t)j * d + f;
            float e = x4.x - c[0];
            acc[j] = fmaf(e, e, acc[j]);
            e = x4.y - c[1];
            acc[j] = fmaf(e, e, acc[j]);
            e = x4.z - c[2];
            acc[j] = fmaf(e, e, acc[j]);
            e = x4.w - c[3];
            acc[j] = fmaf(e, e, acc[j]);
          }
        }
      }
    }
    if (i < n) {
      const double cl = closest[i];
      const double wi = w ? w[i] : 1.0;
#pragma unroll
      for (int j = 0; j < TMAX; ++j) {
        if (j < t) {
          D[(size_t)j * n + i] = acc[j];
          pot[j] += wi * fmin(cl, (double)acc[j]);
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < TMAX; ++j) {
    const double s = wave_sum(pot[j]);
    if (lane == 0) red[wave][j] = s;
  }
  __syncthreads();
  if (threadIdx.x < t)
    part[(size_t)blockIdx.x * t + threadIdx.x] =
        ((red[0][threadIdx.x] + red[1][threadIdx.x]) + red[2][threadIdx.x]) + red[3][threadIdx.x];
}

}  // namespace sq

using namespace sq;

extern "C" {

// X fp32 [n][ldx] (d <= ldx, d % 4 == 0, 16-B aligned rows), cand fp32 [t][d],
// closest fp64 [n], w fp64 [n] or null, D fp32 [t][n], part fp64 [grid][t]
// with grid = sq_kmpp_grid(n).  part rows are summed by the caller.
int sq_kmpp_grid(long long n) {
  const long long b = (n + 255) / 256;     // 4 waves x 64 rows per block pass
  return (int)(b < 2048 ? (b > 0 ? b : 1) : 2048);
}

int sq_kmpp_trials(const void* X, long long ldx, int d, long long n, int t, const void* cand,
                   const void* closest, const void* w, void* D, void* part, void* stream) {
  if (n <= 0) return 0;
  if (t <= 0 || t > 16 || d <= 0 || (d & 3) || ldx < d || (ldx & 3)) return (int)hipErrorInvalidValue;
  const int grid = sq_kmpp_grid(n);
  hipStream_t st = (hipStream_t)stream;
#define LAUNCH(TM)                                                                              \
  hipLaunchKernelGGL(kmpp_trials_kernel<TM>, dim3(grid), dim3(256), 0, st, (const float*)X,   \
                     ldx, d, n, t, (const float*)cand, (const double*)closest,                 \
                     (const double*)w, (float*)D, (double*)part)
  if (t <= 4) LAUNCH(4);
  else if (t <= 8) LAUNCH(8);
  else LAUNCH(16);
#undef LAUNCH
  return (int)hipGetLastError();
}

}  // extern "C"
