// Elkan k-means assignment: triangle-inequality bounds
// for the classical ``KMeans(algorithm='elkan')``.
//
// Reference semantics (``cluster/_k_means_elkan.pyx``): ``init_bounds_dense``
// (:33-101) and ``_update_chunk_dense`` (:336-409), with the bound update of
// ``elkan_iter_chunked_dense`` (:282-317) moved to the front of the next
// assignment (same arithmetic: lower -= shift[j] clamped at 0, upper +=
// shift[label]).  Per row the candidate centres are visited in index order
// and the running (label, upper) pair is updated exactly as the reference's
// sequential loop does, so labels and bounds follow the same recurrence.
//
// MI355X mapping: one wave per row (grid-stride over rows).  The row's
// lower bounds live in a wave-private LDS slice for the duration of the row
// (read once, written once: 2*k*sizeof(T) bytes of HBM traffic per row and
// iteration, the bound-update pass of the reference fused in).  Candidate
// tests run 64 centres per ballot; each surviving centre's Euclidean
// distance is a cooperative wave dot product (lanes over features, x held in
// registers, butterfly reduce), so a row that needs one distance costs one
// coalesced centre-row read instead of a lane-serial d-loop.  Rows whose
// upper bound is below half the distance to their nearest other centre skip
// all distance work (Elkan's lemma 1).
#include "common.h"

namespace sq {

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <typename T>
__device__ __forceinline__ T wave_allsum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <typename T, int NT>
__device__ __forceinline__ T row_distance(const T (&x)[NT], const T* __restrict__ c, int d,
                                          int lane) {
  T acc = 0;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int f = lane + 64 * t;
    if (f < d) {
      const T df = x[t] - c[f];
      acc += df * df;
    }
  }
  return sqrt(wave_allsum(acc));
}

// init != 0: initial bounds (reference init_bounds_dense): label starts at 0
// with lower bounds zero, every centre j is tested against upper > hcc[label, j].
template <typename T, int NT>
__global__ void __launch_bounds__(256) elkan_kernel(
    const T* __restrict__ X, const T* __restrict__ C, const T* __restrict__ hcc,
    const T* __restrict__ snext, const T* __restrict__ shift, int* __restrict__ labels,
    T* __restrict__ upper, T* __restrict__ lower, long long n, int d, int k, int init) {
  extern __shared__ unsigned char smem_raw[];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wpb = blockDim.x >> 6;
  T* l = reinterpret_cast<T*>(smem_raw) + (size_t)wave * k;
  const long long stride = (long long)gridDim.x * wpb;
  for (long long i = (long long)blockIdx.x * wpb + wave; i < n; i += stride) {
    const T* xr = X + i * (long long)d;
    T* lr = lower + i * (long long)k;
    T x[NT];
    bool have_x = false;
    auto load_x = [&]() {
      if (have_x) return;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int f = lane + 64 * t;
        x[t] = f < d ? xr[f] : T(0);
      }
      have_x = true;
    };
    int label;
    T u;
    bool tight;
    if (init) {
      for (int j = lane; j < k; j += 64) l[j] = T(0);
      label = 0;
      load_x();
      u = row_distance(x, C, d, lane);
      wave_sync();
      if (lane == 0) l[0] = u;
      tight = true;
    } else {
      label = labels[i];
      u = upper[i] + shift[label];
      for (int j = lane; j < k; j += 64) {
        const T v = lr[j] - shift[j];
        l[j] = v > T(0) ? v : T(0);
      }
      tight = false;
    }
    wave_sync();
    if (init || u > snext[label]) {
      int last = init ? 0 : -1;
      for (int j0 = 0; j0 < k; j0 += 64) {
        const int j = j0 + lane;
        while (true) {
          const bool c = j < k && j > last && j != label && u > l[j] &&
                         u > hcc[(long long)label * k + j];
          const unsigned long long m = __ballot(c);
          if (!m) break;
          const int jb = j0 + (int)__ffsll((long long)m) - 1;
          load_x();
          if (!tight) {
            u = row_distance(x, C + (long long)label * d, d, lane);
            wave_sync();
            if (lane == 0) l[label] = u;
            wave_sync();
            tight = true;
          }
          const T lj = l[jb];
          const T hj = hcc[(long long)label * k + jb];
          if (u > lj || u > hj) {
            const T dj = row_distance(x, C + (long long)jb * d, d, lane);
            wave_sync();
            if (lane == 0) l[jb] = dj;
            if (dj < u) {
              label = jb;
              u = dj;
            }
          }
          last = jb;
          wave_sync();
        }
      }
    }
    wave_sync();
    for (int j = lane; j < k; j += 64) lr[j] = l[j];
    if (lane == 0) {
      labels[i] = label;
      upper[i] = u;
    }
    wave_sync();
  }
}

template <typename T, int NT>
static int launch_elkan(const void* X, const void* C, const void* hcc, const void* snext,
                        const void* shift, void* labels, void* upper, void* lower, long long n,
                        int d, int k, int init, hipStream_t stream) {
  const size_t row_bytes = (size_t)k * sizeof(T);
  int wpb = 4;
  while (wpb > 1 && row_bytes * wpb > 65536) wpb >>= 1;
  if (row_bytes * wpb > 65536) return (int)hipErrorInvalidValue;
  long long blocks = (n + wpb - 1) / wpb;
  const unsigned grid = (unsigned)(blocks < 16384 ? blocks : 16384);
  hipLaunchKernelGGL((elkan_kernel<T, NT>), dim3(grid), dim3(64 * wpb), row_bytes * wpb, stream,
                     (const T*)X, (const T*)C, (const T*)hcc, (const T*)snext, (const T*)shift,
                     (int*)labels, (T*)upper, (T*)lower, n, d, k, init);
  return (int)hipGetLastError();
}

template <typename T>
static int dispatch_elkan(const void* X, const void* C, const void* hcc, const void* snext,
                          const void* shift, void* labels, void* upper, void* lower, long long n,
                          int d, int k, int init, hipStream_t s) {
  if (d <= 64) return launch_elkan<T, 1>(X, C, hcc, snext, shift, labels, upper, lower, n, d, k, init, s);
  if (d <= 128) return launch_elkan<T, 2>(X, C, hcc, snext, shift, labels, upper, lower, n, d, k, init, s);
  if (d <= 256) return launch_elkan<T, 4>(X, C, hcc, snext, shift, labels, upper, lower, n, d, k, init, s);
  if (d <= 512) return launch_elkan<T, 8>(X, C, hcc, snext, shift, labels, upper, lower, n, d, k, init, s);
  if (d <= 1024) return launch_elkan<T, 16>(X, C, hcc, snext, shift, labels, upper, lower, n, d, k, init, s);
  return (int)hipErrorInvalidValue;
}

}  // namespace sq

using namespace sq;

// dtype: 0 = fp32, 1 = fp64 (X, C, hcc, snext, shift, upper, lower share it)
extern "C" int sq_elkan_step(const void* X, const void* C, const void* hcc, const void* snext,
                             const void* shift, void* labels, void* upper, void* lower,
                             long long n, int d, int k, int dtype, int init, void* stream) {
  if (n <= 0) return 0;
  if (k < 1 || d < 1) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == 0)
    return dispatch_elkan<float>(X, C, hcc, snext, shift, labels, upper, lower, n, d, k, init, s);
  if (dtype == 1)
    return dispatch_elkan<double>(X, C, hcc, snext, shift, labels, upper, lower, n, d, k, init, s);
  return (int)hipErrorInvalidValue;
}
