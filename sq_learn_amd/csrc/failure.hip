// Simulated algorithmic failure: each row's quantum
// distance estimation fails with probability p.  With R attempts (R = 1:
// policy 'ignore'; R > 1: 'resample' - repeat the estimation until it
// succeeds, at most R times) a row is corrupted only when every attempt
// fails, and then its label is replaced by an outlier: a uniformly random
// centroid.  Attempt r of global row g uses Philox word g*R + r of `key`,
// the outlier label word g of `key2`, so the outcome is independent of the
// sharding and bit-identical to the torch twin (ops/kmeans.py
// failure_inject_torch).  counters[0] += attempts made, counters[1] +=
// corrupted rows (wave-reduced, one 64-bit atomic per wave per counter).
#include "common.h"

namespace sq {

__global__ void __launch_bounds__(256) failure_inject_kernel(
    int* __restrict__ labels, long long n, int k, float p, int R, RngKey key, RngKey key2,
    long long row_offset, unsigned long long* __restrict__ counters, float* __restrict__ lb,
    float* __restrict__ corr, float* __restrict__ mind, const float* __restrict__ X, long long ldx,
    const float* __restrict__ C, int ldc, int d) {
  unsigned long long attempts = 0, corrupted = 0;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const unsigned long long g = (unsigned long long)(row_offset + i);
    int r = 0;
    bool ok = false;
    for (; r < R; ++r) {
      if (u01(key.word(g * (unsigned long long)R + r)) >= p) { ok = true; break; }
    }
    attempts += (unsigned long long)(ok ? r + 1 : R);
    if (!ok) {
      int lab = (int)(u01(key2.word(g)) * (float)k);
      lab = lab < k ? lab : k - 1;
      const int old = labels[i];
      labels[i] = lab;
      ++corrupted;
      if (lb) lb[i] = 0.0f;
      if ((corr || mind) && old >= 0 && old < k && old != lab) {
        const float* x = X + i * ldx;
        const float* co = C + (size_t)old * ldc;
        const float* cn = C + (size_t)lab * ldc;
        double d_old = 0.0, d_new = 0.0;
        for (int f = 0; f < d; ++f) {
          const double a = (double)x[f] - (double)co[f], b = (double)x[f] - (double)cn[f];
          d_old = fma(a, a, d_old);
          d_new = fma(b, b, d_new);
        }
        if (corr) corr[i] += (float)(d_old - d_new);
        // a single-candidate row's min distance is filled later from its
        // label (mind < 0): keep the E-step's minimum instead
        if (mind && mind[i] < 0.0f) mind[i] = (float)d_old;
      }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    attempts += __shfl_xor(attempts, o, 64);
    corrupted += __shfl_xor(corrupted, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    if (attempts) atomicAdd(&counters[0], attempts);
    if (corrupted) atomicAdd(&counters[1], corrupted);
  }
}

}  // namespace sq

using namespace sq;

extern "C" int sq_failure_inject(void* labels, long long n, int k, double p, int R, unsigned k0,
                                 unsigned k1, unsigned s0, unsigned s1, unsigned t0, unsigned t1,
                                 unsigned u0, unsigned u1, long long row_offset, void* counters,
                                 void* lb, void* corr, void* mind, const void* X, long long ldx,
                                 const void* C, int ldc, int d, void* stream) {
  if (n <= 0) return 0;
  if (R < 1 || k < 1 || ((corr || mind) && (!X || !C || ldx < d || ldc < d)))
    return (int)hipErrorInvalidValue;
  RngKey key{k0, k1, s0, s1}, key2{t0, t1, u0, u1};
  long long blocks = (n + 255) / 256;
  unsigned grid = (unsigned)(blocks < 4096 ? blocks : 4096);
  hipLaunchKernelGGL(failure_inject_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                     (int*)labels, n, k, (float)p, R, key, key2, row_offset,
                     (unsigned long long*)counters, (float*)lb, (float*)corr, (float*)mind,
                     (const float*)X, ldx,
                     (const float*)C, ldc, d);
  return (int)hipGetLastError();
}
