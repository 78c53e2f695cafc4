// Decision-forest inference on gfx950 (SURVEY.md N13/N17 prediction paths:
// reference ``tree/_tree.pyx`` Tree.apply / predict, ``ensemble/_forest.py``
// averaging, ``_hist_gradient_boosting/_predictor.pyx``).
//
// Trees are flattened into struct-of-arrays node tables (int32 children /
// feature, fp64 thresholds so the comparison ``(double)x <= threshold`` is the
// host builder's exactly); all trees of a forest share one table with
// per-tree node offsets.  Rows are float32 row-major.
//
// * forest_apply_kernel: one lane per (row, tree) pair -> leaf id.  Grid
//   covers n * T lanes (>> 256 CUs for any realistic batch).
// * forest_predict_kernel: one lane per row walks every tree and accumulates
//   the leaf value vectors in registers (S <= 32 outputs/classes) - no n x T
//   leaf-id intermediate in HBM; optional NaN routing (missing_left) for the
//   histogram-GBDT predictors.
#include "common.h"

namespace sq {

__global__ void forest_apply_kernel(const int* __restrict__ left, const int* __restrict__ right,
                                    const int* __restrict__ feature,
                                    const double* __restrict__ thr,
                                    const long long* __restrict__ offs, int T,
                                    const float* __restrict__ X, long long n, int d,
                                    int* __restrict__ out) {
  long long g = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n * (long long)T) return;
  long long i = g / T;
  int t = (int)(g - i * T);
  const float* xi = X + i * d;
  const long long base = offs[t];
  int node = 0;
  while (left[base + node] != -1) {
    const long long q = base + node;
    node = ((double)xi[feature[q]] <= thr[q]) ? left[q] : right[q];
  }
  out[g] = node;
}

template <int S>
__global__ void forest_predict_kernel(const int* __restrict__ left, const int* __restrict__ right,
                                      const int* __restrict__ feature,
                                      const double* __restrict__ thr,
                                      const unsigned char* __restrict__ missing_left,
                                      const long long* __restrict__ offs, int T,
                                      const double* __restrict__ value, int s_act,
                                      const float* __restrict__ X, long long n, int d,
                                      double scale, double* __restrict__ out) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float* xi = X + i * d;
  double acc[S];
#pragma unroll
  for (int s = 0; s < S; ++s) acc[s] = 0.0;
  for (int t = 0; t < T; ++t) {
    const long long base = offs[t];
    int node = 0;
    while (left[base + node] != -1) {
      const long long q = base + node;
      const float xv = xi[feature[q]];
      bool go_left;
      if (missing_left != nullptr && xv != xv) go_left = missing_left[q] != 0;
      else go_left = (double)xv <= thr[q];
      node = go_left ? left[q] : right[q];
    }
    const double* v = value + (base + node) * (long long)s_act;
#pragma unroll
    for (int s = 0; s < S; ++s)
      if (s < s_act) acc[s] += v[s];
  }
#pragma unroll
  for (int s = 0; s < S; ++s)
    if (s < s_act) out[i * s_act + s] = acc[s] * scale;
}

}  // namespace sq

using namespace sq;

extern "C" int sq_forest_apply(const void* left, const void* right, const void* feature,
                               const void* thr, const void* offs, int T, const void* X,
                               long long n, int d, void* out, void* stream) {
  if (n <= 0 || T <= 0) return 0;
  const long long lanes = n * (long long)T;
  const int bs = 256;
  hipLaunchKernelGGL(forest_apply_kernel, dim3((unsigned)((lanes + bs - 1) / bs)), dim3(bs), 0,
                     (hipStream_t)stream, (const int*)left, (const int*)right,
                     (const int*)feature, (const double*)thr, (const long long*)offs, T,
                     (const float*)X, n, d, (int*)out);
  return (int)hipGetLastError();
}

// value: (total_nodes, s_act) fp64; out: (n, s_act) = scale * sum_t value[leaf_t]
extern "C" int sq_forest_predict(const void* left, const void* right, const void* feature,
                                 const void* thr, const void* missing_left, const void* offs,
                                 int T, const void* value, int s_act, const void* X, long long n,
                                 int d, double scale, void* out, void* stream) {
  if (n <= 0) return 0;
  if (s_act <= 0 || s_act > 32) return (int)hipErrorInvalidValue;
  const int bs = 128;
  dim3 grid((unsigned)((n + bs - 1) / bs));
  hipStream_t st = (hipStream_t)stream;
#define SQ_FP(SV)                                                                              \
  hipLaunchKernelGGL((forest_predict_kernel<SV>), grid, dim3(bs), 0, st, (const int*)left,     \
                     (const int*)right, (const int*)feature, (const double*)thr,              \
                     (const unsigned char*)missing_left, (const long long*)offs, T,           \
                     (const double*)value, s_act, (const float*)X, n, d, scale, (double*)out)
  if (s_act <= 1) SQ_FP(1);
  else if (s_act <= 4) SQ_FP(4);
  else if (s_act <= 8) SQ_FP(8);
  else if (s_act <= 16) SQ_FP(16);
  else SQ_FP(32);
#undef SQ_FP
  return (int)hipGetLastError();
}
