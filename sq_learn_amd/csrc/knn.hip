// Brute-force k-NN selection: per query row, the kk
// smallest distances of a distance tile produced by the library GEMM.
// One wave per row; each lane keeps a sorted register list of its columns'
// best KMAX, then the 64 lists are merged by kk rounds of wave-wide argmin.
#include "common.h"

namespace sq {

constexpr int KMAX = 32;

__global__ void __launch_bounds__(256) knn_topk_kernel(const float* __restrict__ D,
                                                       float* __restrict__ outd,
                                                       long long* __restrict__ outi, long long m,
                                                       int nref, long long ldD, int kk,
                                                       long long col_offset) {
  const int lane = threadIdx.x & 63;
  const long long r = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= m) return;
  float bv[KMAX];
  int bi[KMAX];
#pragma unroll
  for (int i = 0; i < KMAX; ++i) { bv[i] = __builtin_inff(); bi[i] = 0x7FFFFFFF; }
  const float* row = D + r * ldD;
  for (int j = lane; j < nref; j += 64) {
    float v = row[j];
    if (v < bv[kk - 1] || (v == bv[kk - 1] && j < bi[kk - 1])) {
      // insertion into the sorted list (static indices -> registers)
      float cv = v; int ci = j;
#pragma unroll
      for (int i = 0; i < KMAX; ++i) {
        if (i < kk) {
          bool lt = cv < bv[i] || (cv == bv[i] && ci < bi[i]);
          float tv = bv[i]; int ti = bi[i];
          bv[i] = lt ? cv : tv; bi[i] = lt ? ci : ti;
          cv = lt ? tv : cv; ci = lt ? ti : ci;
        }
      }
    }
  }
  // merge: kk rounds; the lane owning the wave minimum pops its head
  for (int t = 0; t < kk; ++t) {
    float v = bv[0]; int ix = bi[0];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      float ov = __shfl_xor(v, o, 64);
      int oi = __shfl_xor(ix, o, 64);
      if (ov < v || (ov == v && oi < ix)) { v = ov; ix = oi; }
    }
    if (lane == 0) {
      outd[r * kk + t] = v;
      outi[r * kk + t] = ix == 0x7FFFFFFF ? -1 : (long long)ix + col_offset;
    }
    if (bi[0] == ix && bv[0] == v) {
#pragma unroll
      for (int i = 0; i < KMAX - 1; ++i) { bv[i] = bv[i + 1]; bi[i] = bi[i + 1]; }
      bv[KMAX - 1] = __builtin_inff(); bi[KMAX - 1] = 0x7FFFFFFF;
    }
  }
}

}  // namespace sq

using namespace sq;

extern "C" int sq_knn_topk(const void* D, void* outd, void* outi, long long m, int nref,
                           long long ldD, int kk, long long col_offset, void* stream) {
  if (m <= 0) return 0;
  if (kk < 1 || kk > KMAX) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(knn_topk_kernel, dim3((unsigned)((m + 3) / 4)), dim3(256), 0,
                     (hipStream_t)stream, (const float*)D, (float*)outd, (long long*)outi, m, nref,
                     ldD, kk, col_offset);
  return (int)hipGetLastError();
}
