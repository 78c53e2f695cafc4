// Row-gather microbenchmark: what does reading the fp16 rows (512 B) of a
// multi-row list cost on its own?  n = 10M rows x 256 halves; the list holds
// 1.14M rows (every ~9th row, in the bounds filter's (tid, p) chunk order).
// Variants: rows per wave step (LPR lanes per row) x loads in flight.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
#include <random>

#define CK(x) do { hipError_t e = (x); if (e) { printf("err %d line %d\n", (int)e, __LINE__); return 1; } } while (0)

template <int LPR, int DEPTH>
__global__ void __launch_bounds__(256) gather(const uint4* __restrict__ X, const long long* __restrict__ list,
                                             long long cnt, float* __restrict__ out) {
  constexpr int RPW = 64 / LPR;
  constexpr int V = 32 / LPR;   // uint4 per lane per row (512 B rows)
  const int lane = threadIdx.x & 63, sub = lane & (LPR - 1), r = lane / LPR;
  const long long gw = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const long long nw = (long long)gridDim.x * 4;
  const long long per = ((cnt + nw - 1) / nw + RPW * DEPTH - 1) / (RPW * DEPTH) * (RPW * DEPTH);
  const long long b0 = gw * per, b1 = min(cnt, b0 + per);
  float acc = 0.f;
  for (long long e = b0; e < b1; e += RPW * DEPTH) {
    uint4 v[DEPTH][V];
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      const long long ee = min(e + d * RPW + r, b1 - 1);
      const long long g = list[ee];
#pragma unroll
      for (int q = 0; q < V; ++q) v[d][q] = X[g * 32 + q * LPR + sub];
    }
#pragma unroll
    for (int d = 0; d < DEPTH; ++d)
#pragma unroll
      for (int q = 0; q < V; ++q) acc += __uint_as_float(v[d][q].x ^ v[d][q].y ^ v[d][q].z ^ v[d][q].w);
  }
  if (acc == 1.2345f) out[0] = acc;
}

// + NC candidate rows per list row from a small table (the shift operand:
// L2 hits), ids from a per-row record
template <int NC>
__global__ void __launch_bounds__(256) gather_cand(const uint4* __restrict__ X, const long long* __restrict__ list,
                                                  long long cnt, const uint4* __restrict__ T, const int* __restrict__ ids,
                                                  float* __restrict__ out) {
  const int lane = threadIdx.x & 63, sub = lane & 31, r = lane >> 5;
  const long long gw = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const long long nw = (long long)gridDim.x * 4;
  const long long per = ((cnt + nw - 1) / nw + 7) / 8 * 8;
  const long long b0 = gw * per, b1 = min(cnt, b0 + per);
  float acc = 0.f;
  for (long long e = b0; e < b1; e += 8) {
    uint4 v[4], c[4][NC > 0 ? NC : 1];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const long long ee = min(e + d * 2 + r, b1 - 1);
      const long long g = list[ee];
      v[d] = X[g * 32 + sub];
#pragma unroll
      for (int k = 0; k < NC; ++k) c[d][k] = T[(size_t)ids[(g & 1023) * 4 + k] * 32 + sub];
    }
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      acc += __uint_as_float(v[d].x ^ v[d].w);
#pragma unroll
      for (int k = 0; k < NC; ++k) acc += __uint_as_float(c[d][k].x ^ c[d][k].w);
    }
  }
  if (acc == 1.2345f) out[0] = acc;
}

__global__ void contig(const uint4* __restrict__ X, long long n16, float* out) {
  float acc = 0.f;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (long long)gridDim.x * blockDim.x) {
    const uint4 v = X[i];
    acc += __uint_as_float(v.x ^ v.y ^ v.z ^ v.w);
  }
  if (acc == 1.2345f) out[0] = acc;
}

template <class F>
float timeit(F f) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  f(); hipDeviceSynchronize();
  hipEventRecord(a);
  for (int i = 0; i < 10; ++i) f();
  hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  return ms * 100.f;   // us per call
}

int main() {
  const long long n = 10000000, cnt_target = 1140000;
  uint4* X; long long* L; float* out;
  CK(hipMalloc(&X, n * 512));
  CK(hipMemset(X, 1, n * 512));
  CK(hipMalloc(&out, 4));
  // the filter's order: chunks of 8192 rows, entry order (tid, p) -> row c0 + p * 256 + tid
  std::mt19937 rng(1);
  std::vector<long long> h;
  for (long long c0 = 0; c0 < n; c0 += 8192)
    for (int t = 0; t < 256; ++t)
      for (int p = 0; p < 32; ++p) {
        const long long i = c0 + p * 256 + t;
        if (i < n && (rng() % 1000) < 114) h.push_back(i);
      }
  const long long cnt = (long long)h.size();
  std::vector<long long> hs(h); std::sort(hs.begin(), hs.end());
  CK(hipMalloc(&L, cnt * 8));
  long long* Ls; CK(hipMalloc(&Ls, cnt * 8));
  CK(hipMemcpy(L, h.data(), cnt * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(Ls, hs.data(), cnt * 8, hipMemcpyHostToDevice));
  printf("list %lld rows (%.1f MB of rows)\n", cnt, cnt * 512 / 1e6);
  printf("contig read of the same bytes: %.1f us\n", timeit([&] { contig<<<4096, 256>>>(X, cnt * 32, out); }));
  for (int grid : {1024, 2048, 4096}) {
    printf("grid %d: LPR32 d1 %.1f  d2 %.1f  d4 %.1f | LPR16 d1 %.1f d2 %.1f d4 %.1f | LPR8 d2 %.1f | sorted LPR32 d2 %.1f\n", grid,
           timeit([&] { gather<32, 1><<<grid, 256>>>(X, L, cnt, out); }),
           timeit([&] { gather<32, 2><<<grid, 256>>>(X, L, cnt, out); }),
           timeit([&] { gather<32, 4><<<grid, 256>>>(X, L, cnt, out); }),
           timeit([&] { gather<16, 1><<<grid, 256>>>(X, L, cnt, out); }),
           timeit([&] { gather<16, 2><<<grid, 256>>>(X, L, cnt, out); }),
           timeit([&] { gather<16, 4><<<grid, 256>>>(X, L, cnt, out); }),
           timeit([&] { gather<8, 2><<<grid, 256>>>(X, L, cnt, out); }),
           timeit([&] { gather<32, 2><<<grid, 256>>>(X, Ls, cnt, out); }));
  }
  // candidate table: 1024 rows x 512 B, ids: 400 hot rows
  uint4* T; int* ids;
  CK(hipMalloc(&T, 1024 * 512));
  CK(hipMemset(T, 2, 1024 * 512));
  std::vector<int> hid(4096);
  for (auto& v : hid) v = (int)(rng() % 400);
  CK(hipMalloc(&ids, 4096 * 4));
  CK(hipMemcpy(ids, hid.data(), 4096 * 4, hipMemcpyHostToDevice));
  for (int grid : {1024, 2048}) {
    printf("grid %d with candidate rows: NC0 %.1f  NC1 %.1f  NC2 %.1f  NC4 %.1f\n", grid,
           timeit([&] { gather_cand<0><<<grid, 256>>>(X, L, cnt, T, ids, out); }),
           timeit([&] { gather_cand<1><<<grid, 256>>>(X, L, cnt, T, ids, out); }),
           timeit([&] { gather_cand<2><<<grid, 256>>>(X, L, cnt, T, ids, out); }),
           timeit([&] { gather_cand<4><<<grid, 256>>>(X, L, cnt, T, ids, out); }));
  }
  return 0;
}
