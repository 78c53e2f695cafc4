// Stochastic layer kernels: counter-based Philox
// draws keyed by global element index, fused with the operation that
// consumes them, so no random tensor is ever materialised and every rank of
// a row-sharded job draws identical numbers for the same global element.
#include "common.h"
#include "fejer.h"

namespace sq {

// x[i] += TN(-b, b) for flat element ids offset+i   (K11; Utility.py:88-104)
template <typename T>
__global__ void __launch_bounds__(256) trunc_normal_add_kernel(
    T* __restrict__ x, long long n, float b, float erf_b, RngKey key, unsigned long long offset) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  long long stride = (long long)gridDim.x * blockDim.x;
  for (; i < n; i += stride) {
    uint32_t w = key.word(offset + (unsigned long long)i);
    float z = trunc_normal(w, b, erf_b);
    if constexpr (sizeof(T) == 8) x[i] = x[i] + (double)z;
    else x[i] = x[i] + z;
  }
}

// out[i] = mean + std * N(0,1) for flat element ids offset+i.
// element e: block e>>1, words (x,y) -> Box-Muller, even -> cos, odd -> sin
template <typename T>
__global__ void __launch_bounds__(256) philox_normal_kernel(
    T* __restrict__ out, long long n, float mean, float stdv, RngKey key, unsigned long long offset) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  long long stride = (long long)gridDim.x * blockDim.x;
  for (; i < n; i += stride) {
    unsigned long long e = offset + (unsigned long long)i;
    u4 blk = key.block(e >> 1);
    float u1 = u01(blk.x), u2 = u01(blk.y);
    float r = sqrtf(-2.0f * logf(u1));
    float s, c; sincosf(6.28318530717958647f * u2, &s, &c);
    float z = (e & 1) ? r * s : r * c;
    float v = mean + stdv * z;
    if constexpr (sizeof(T) == 2) {
      reinterpret_cast<uint16_t*>(out)[i] = f32_to_bf16_rne(v);
    } else {
      out[i] = (T)v;
    }
  }
}

// uniform (0,1) for flat ids
__global__ void __launch_bounds__(256) philox_uniform_kernel(
    float* __restrict__ out, long long n, RngKey key, unsigned long long offset) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  long long stride = (long long)gridDim.x * blockDim.x;
  for (; i < n; i += stride) out[i] = u01(key.word(offset + (unsigned long long)i));
}

// Batched amplitude estimation (K9): out[i] = median over Q of AE(a[i], eps[i])
// Sample id of repetition q of element i: (offset + i) * Q + q.
__global__ void __launch_bounds__(256) ae_batch_kernel(
    const double* __restrict__ a, const double* __restrict__ eps, double* __restrict__ out,
    long long n, int Q, RngKey key, unsigned long long offset) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  long long M = ae_bins(eps[i]);
  double v[31];
  for (int q = 0; q < Q; ++q) {
    WordStream ws(key, ((offset + (unsigned long long)i) * (unsigned long long)Q) + q);
    v[q] = ae_sample(a[i], M, ws);
  }
  out[i] = Q == 1 ? v[0] : median_of<31>(v, Q);
}

// Batched phase estimation: out[i] = k/M, M = 2^m[i], centre omega[i] in [0,1)
__global__ void __launch_bounds__(256) pe_batch_kernel(
    const double* __restrict__ omega, const int* __restrict__ m, double* __restrict__ out,
    long long n, RngKey key, unsigned long long offset) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  long long M = 1LL << m[i];
  double w = omega[i];
  if (w == 1.0 || fabs(w - 1.0) <= 1e-8 + 1e-5) { out[i] = (double)(M - 1) / (double)M; return; }
  WordStream ws(key, offset + (unsigned long long)i);
  long long k = fejer_sample((double)M * w, M, ws);
  out[i] = (double)k / (double)M;
}

}  // namespace sq

using namespace sq;

static inline int grid_for(long long n, int block = 256, int cap = 2048 * 4) {
  long long g = (n + block - 1) / block;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return (int)g;
}

extern "C" {

int sq_trunc_normal_add(void* x, int dtype, long long n, double b, unsigned k0, unsigned k1,
                        unsigned s0, unsigned s1, unsigned long long offset, void* stream) {
  if (n <= 0) return 0;
  RngKey key{k0, k1, s0, s1};
  float erf_b = erff((float)b * 0.70710678118654752f);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == 0)
    hipLaunchKernelGGL(trunc_normal_add_kernel<float>, dim3(grid_for(n)), dim3(256), 0, st,
                       (float*)x, n, (float)b, erf_b, key, offset);
  else
    hipLaunchKernelGGL(trunc_normal_add_kernel<double>, dim3(grid_for(n)), dim3(256), 0, st,
                       (double*)x, n, (float)b, erf_b, key, offset);
  return (int)hipGetLastError();
}

int sq_philox_normal(void* out, int dtype, long long n, double mean, double stdv, unsigned k0,
                     unsigned k1, unsigned s0, unsigned s1, unsigned long long offset, void* stream) {
  if (n <= 0) return 0;
  RngKey key{k0, k1, s0, s1};
  hipStream_t st = (hipStream_t)stream;
  if (dtype == 0)
    hipLaunchKernelGGL(philox_normal_kernel<float>, dim3(grid_for(n)), dim3(256), 0, st,
                       (float*)out, n, (float)mean, (float)stdv, key, offset);
  else if (dtype == 1)
    hipLaunchKernelGGL(philox_normal_kernel<double>, dim3(grid_for(n)), dim3(256), 0, st,
                       (double*)out, n, (float)mean, (float)stdv, key, offset);
  else
    hipLaunchKernelGGL(philox_normal_kernel<__hip_bfloat16>, dim3(grid_for(n)), dim3(256), 0, st,
                       (__hip_bfloat16*)out, n, (float)mean, (float)stdv, key, offset);
  return (int)hipGetLastError();
}

int sq_philox_uniform(void* out, long long n, unsigned k0, unsigned k1, unsigned s0, unsigned s1,
                      unsigned long long offset, void* stream) {
  if (n <= 0) return 0;
  RngKey key{k0, k1, s0, s1};
  hipLaunchKernelGGL(philox_uniform_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream,
                     (float*)out, n, key, offset);
  return (int)hipGetLastError();
}

int sq_ae_batch(const void* a, const void* eps, void* out, long long n, int Q, unsigned k0,
                unsigned k1, unsigned s0, unsigned s1, unsigned long long offset, void* stream) {
  if (n <= 0) return 0;
  if (Q < 1 || Q > 31) return -1;
  RngKey key{k0, k1, s0, s1};
  hipLaunchKernelGGL(ae_batch_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, (const double*)a, (const double*)eps, (double*)out, n, Q,
                     key, offset);
  return (int)hipGetLastError();
}

int sq_pe_batch(const void* omega, const void* m, void* out, long long n, unsigned k0, unsigned k1,
                unsigned s0, unsigned s1, unsigned long long offset, void* stream) {
  if (n <= 0) return 0;
  RngKey key{k0, k1, s0, s1};
  hipLaunchKernelGGL(pe_batch_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, (const double*)omega, (const int*)m, (double*)out, n, key,
                     offset);
  return (int)hipGetLastError();
}

}  // extern "C"
