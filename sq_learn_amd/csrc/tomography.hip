// Shot-based vector tomography (Kerenidis-Prakash QIPM Alg. 4.1; reference
// Utility.py:259-402) for a batch of rows, on the device.
//
// For every (row, checkpoint t) pair one wave runs the two measurement
// rounds of the algorithm with N_t shots each:
//   1. magnitudes: counts ~ Multinomial(N_t, v_i^2); P_i = sqrt(c_i / N_t)
//   2. signs:      plus ~ Multinomial(N_t, {((v_i + P_i)/2)^2}_i + remainder);
//                  est_i = P_i if plus_i > 0.4 P_i^2 N_t else -P_i
// The multinomials are sampled by binary splitting over a padded outcome
// tree (M - 1 binomials, log2(M) levels; lanes own the nodes of a level), so
// a wave needs no sequential pass over the d outcomes.  Binomials use
// inversion for small means and BTRS (Hormann 1993) otherwise, in fp64, with
// Philox words keyed by (row, t, round, node, trial): the outcome is a pure
// function of the key, identical on every rank (centroid tomography is
// replicated) and across the two launch modes below.
//   mode 0: err[row][t] = ||v - est||_2 (or _inf) for every checkpoint;
//   mode 1: est of checkpoint first[row] written to out[row][:].
// The host picks first[row] = the first checkpoint with err <= delta (the
// reference's stopping rule) between the two launches.
#include "common.h"

namespace sq {

constexpr int kTomoMaxM = 512;   // padded outcomes (d + 1 <= 512)

SQ_DEV double u01_53(const RngKey& key, unsigned long long ctr, int w) {
  u4 b = key.block(ctr);
  uint32_t x = w == 0 ? b.x : b.z;
  uint32_t y = w == 0 ? b.y : b.w;
  return ((double)(((unsigned long long)x << 21) ^ (unsigned long long)(y >> 11)) + 0.5) *
         (1.0 / 9007199254740992.0);
}

// Binomial(n, p) with n < 2^52, p in [0, 1]; ctr selects an independent
// stream of Philox blocks (2 uniforms per block).
SQ_DEV double binomial(double n, double p, const RngKey& key, unsigned long long ctr) {
  if (n <= 0.0 || p <= 0.0) return 0.0;
  if (p >= 1.0) return n;
  const bool flip = p > 0.5;
  const double pp = flip ? 1.0 - p : p;
  double k;
  if (n * pp < 12.0) {
    // inversion: walk the pmf from 0 (expected ~ n p + 1 steps)
    const double q = 1.0 - pp;
    const double s = pp / q;
    const double a = (n + 1.0) * s;
    double r = pow(q, n);
    double u = u01_53(key, ctr << 6, 0);
    k = 0.0;
    int guard = 0;
    while (u > r && guard < 4096) {
      u -= r;
      k += 1.0;
      r *= (a / k - s);
      ++guard;
    }
    if (k > n) k = n;
  } else {
    // BTRS transformed rejection
    const double q = 1.0 - pp;
    const double spq = sqrt(n * pp * q);
    const double b = 1.15 + 2.53 * spq;
    const double a = -0.0873 + 0.0248 * b + 0.01 * pp;
    const double c = n * pp + 0.5;
    const double vr = 0.92 - 4.2 / b;
    const double alpha = (2.83 + 5.1 / b) * spq;
    const double lpq = log(pp / q);
    const double m = floor((n + 1.0) * pp);
    const double h = lgamma(m + 1.0) + lgamma(n - m + 1.0);
    k = c;
    // trial t uses Philox block (ctr << 6) + t: words (x, y) -> U, (z, w) -> V
    // (acceptance > 0.9 per trial: 63 trials are never exhausted in practice)
    for (int trial = 0; trial < 63; ++trial) {
      const unsigned long long tc = (ctr << 6) + (unsigned long long)trial;
      const double U = u01_53(key, tc, 0) - 0.5;
      const double V = u01_53(key, tc, 1);
      const double us = 0.5 - fabs(U);
      k = floor((2.0 * a / us + b) * U + c);
      if (k < 0.0 || k > n) continue;
      if (us >= 0.07 && V <= vr) break;
      const double lv = log(V * alpha / (a / (us * us) + b));
      if (lv <= h - lgamma(k + 1.0) - lgamma(n - k + 1.0) + (k - m) * lpq) break;
    }
  }
  return flip ? n - k : k;
}

// Multinomial counts over the outcomes whose probabilities' prefix sums are
// pre[0..M] (pre[0] = 0, pre[M] = total), N shots, into cnt[0..M).  The wave
// shares lvl[] (scratch, M doubles).  Node (level l, index i) covers
// [i * M >> l, (i + 1) * M >> l).
SQ_DEV void multinomial_tree(const double* pre, int M, double N, double* cnt, double* lvl,
                             const RngKey& key, unsigned long long ctr_base, int lane) {
  if (lane == 0) lvl[0] = N;
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  int nodes = 1;
  for (int width = M; width > 1; width >>= 1, nodes <<= 1) {
    // children of node i are written to cnt[] then copied back to lvl[]
    for (int i = lane; i < nodes; i += 64) {
      const int lo = i * width, mid = lo + width / 2, hi = lo + width;
      const double tot = pre[hi] - pre[lo];
      const double left = pre[mid] - pre[lo];
      const double n = lvl[i];
      double nl = 0.0;
      if (n > 0.0 && tot > 0.0) {
        const double pl = left / tot;
        nl = binomial(n, pl < 0.0 ? 0.0 : (pl > 1.0 ? 1.0 : pl), key,
                      ctr_base + (unsigned long long)(nodes + i));
      }
      cnt[2 * i] = nl;
      cnt[2 * i + 1] = n - nl;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    for (int i = lane; i < 2 * nodes; i += 64) lvl[i] = cnt[i];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  }
  // leaves now in cnt[0..M)
}

// 4 waves per workgroup.  mode 0: one (row, checkpoint) pair per wave (the
// checkpoint's error); mode 1: one row per wave at checkpoint first[row];
// mode 2 (stop at the first passing checkpoint): one row per wave walks its
// checkpoints in order and keeps the estimate of the first whose error is
// <= stop_err (else the last) - the same Philox words per (row, checkpoint)
// as modes 0 + 1, so the same result, with only the checkpoints up to the
// first passing one evaluated.
__global__ void __launch_bounds__(256) tomography_kernel(
    const double* __restrict__ V, int r, int d, const long long* __restrict__ sched, int T,
    int mode, const int* __restrict__ first, double* __restrict__ err, double* __restrict__ out,
    int norm_inf, RngKey key, long long row_offset, double stop_err) {
  extern __shared__ __attribute__((aligned(16))) double tsm[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long long pair = (long long)blockIdx.x * 4 + w;
  const long long npairs = mode == 0 ? (long long)r * T : (long long)r;
  if (pair >= npairs) return;
  const int row = (int)(mode == 0 ? pair / T : pair);
  const int t_first = mode == 0 ? (int)(pair % T) : (mode == 1 ? first[row] : 0);
  const int t_last = mode == 2 ? T - 1 : t_first;
  for (int t = t_first; t <= t_last; ++t) {
  int M = 1;
  while (M < d + 1) M <<= 1;
  double* pre = tsm + (size_t)w * (4 * kTomoMaxM + 2);     // M + 1
  double* cnt = pre + kTomoMaxM + 1;                         // M
  double* lvl = cnt + kTomoMaxM;                             // M
  double* est = lvl + kTomoMaxM;                             // d
  const double* v = V + (size_t)row * d;
  const double N = (double)sched[t];
  const unsigned long long g = (unsigned long long)(row_offset + row);
  const unsigned long long base = ((g * (unsigned long long)T + t) * 2ull) << 20;

  // ---- round 1: magnitudes, p_i = v_i^2 (normalised)
  for (int i = lane; i <= M; i += 64) {
    // exclusive prefix computed serially per lane-chunk below
    pre[i] = 0.0;
  }
  __builtin_amdgcn_wave_barrier();
  if (lane == 0) {
    double s = 0.0;
    for (int i = 0; i < M; ++i) {
      pre[i] = s;
      s += i < d ? v[i] * v[i] : 0.0;
    }
    pre[M] = s;
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  multinomial_tree(pre, M, N, cnt, lvl, key, base, lane);
  for (int i = lane; i < d; i += 64) est[i] = sqrt(cnt[i] / N);   // P_i
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");

  // ---- round 2: signs; outcomes 0..d-1 = plus_i, outcome d = remainder
  if (lane == 0) {
    double s = 0.0, z = 0.0;
    for (int i = 0; i < d; ++i) {
      const double ap = 0.5 * (v[i] + est[i]), am = 0.5 * (v[i] - est[i]);
      z += ap * ap + am * am;
    }
    for (int i = 0; i < M; ++i) {
      pre[i] = s;
      double pi = 0.0;
      if (i < d) {
        const double ap = 0.5 * (v[i] + est[i]);
        pi = ap * ap / z;
      } else if (i == d) {
        pi = 1.0 - s;
        if (pi < 0.0) pi = 0.0;
      }
      s += pi;
    }
    pre[M] = s;
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  multinomial_tree(pre, M, N, cnt, lvl, key, base + (1ull << 20), lane);
  double e = 0.0;
  for (int i = lane; i < d; i += 64) {
    const double P = est[i];
    const double s = cnt[i] > 0.4 * P * P * N ? P : -P;
    if (mode != 0) out[(size_t)row * d + i] = s;
    const double df = v[i] - s;
    e = norm_inf ? fmax(e, fabs(df)) : e + df * df;
  }
  if (mode != 1) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const double x = __shfl_xor(e, o, 64);
      e = norm_inf ? fmax(e, x) : e + x;
    }
    const double ev = norm_inf ? e : sqrt(e);
    if (mode == 0 && lane == 0) err[(size_t)row * T + t] = ev;
    if (mode == 2 && ev <= stop_err) break;   // wave-uniform (the reduced error)
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  }
}

// ---------------------------------------------------------------------------
// Multinomial over LONG outcome vectors (the left singular vectors of qPCA
// have n = 1e6..1e7 coordinates, row-sharded over the ranks; SURVEY.md K12,
// reference Utility.py:313-352 applied at _qPCA.py:1059-1063).
//
// The outcome axis is cut into segments of <= kSegP outcomes.  One workgroup
// draws the counts of one segment given the segment's total count: the
// segment's weights go to an LDS heap (mass[P + i] = w_i, mass[i] =
// mass[2i] + mass[2i + 1], pairwise fp64 sums), then the count heap is split
// top-down, cnt[2i] ~ Binomial(cnt[i], mass[2i] / mass[i]), one tree level
// per step with a thread per node.  The host recursion (quantum/device.py
// multinomial_long) draws the segment totals the same way one level up from
// the segments' masses, so any length is a few launches of O(length) work.
// Draws are keyed by (sid[b], segment, tree level, node): a pure function of
// the key, independent of launch geometry and of the checkpoint chunking.
constexpr int kSegP = 2048;

__global__ void __launch_bounds__(256) mnom_segments_kernel(
    const double* __restrict__ W, long long ldw, const long long* __restrict__ wrow, long long m,
    int nseg, const double* __restrict__ Nseg, double* __restrict__ cnt, long long ldc,
    RngKey key, const long long* __restrict__ sid, int level) {
  __shared__ double mass[2 * kSegP];
  __shared__ double cn[2 * kSegP];
  const long long s = blockIdx.x;          // b * nseg + j
  const long long b = s / nseg;
  const int j = (int)(s % nseg);
  const long long lo = (long long)j * kSegP;
  const int len = (int)min((long long)kSegP, m - lo);
  int P = 1;
  while (P < len) P <<= 1;
  const double* w = W + (size_t)wrow[b] * ldw + lo;
  for (int i = threadIdx.x; i < P; i += blockDim.x) {
    const double v = i < len ? w[i] : 0.0;
    mass[P + i] = v > 0.0 ? v : 0.0;
  }
  __syncthreads();
  for (int width = P >> 1; width >= 1; width >>= 1) {
    for (int i = width + threadIdx.x; i < 2 * width; i += blockDim.x)
      mass[i] = mass[2 * i] + mass[2 * i + 1];
    __syncthreads();
  }
  if (threadIdx.x == 0) cn[1] = Nseg[s];
  __syncthreads();
  const unsigned long long seg_ctr =
      ((((unsigned long long)sid[b] * (unsigned long long)nseg + (unsigned long long)j) << 4) |
       (unsigned long long)(level & 15)) << 12;
  for (int width = 1; width < P; width <<= 1) {
    for (int i = width + threadIdx.x; i < 2 * width; i += blockDim.x) {
      const double n = cn[i], tot = mass[i], left = mass[2 * i];
      double nl = 0.0;
      if (n > 0.0 && tot > 0.0) {
        const double pl = left / tot;
        nl = binomial(n, pl < 0.0 ? 0.0 : (pl > 1.0 ? 1.0 : pl), key, seg_ctr | (unsigned long long)i);
      }
      cn[2 * i] = nl;
      cn[2 * i + 1] = n - nl;
    }
    __syncthreads();
  }
  double* out = cnt + (size_t)b * ldc + lo;
  for (int i = threadIdx.x; i < len; i += blockDim.x) out[i] = cn[P + i];
}

}  // namespace sq

using namespace sq;

extern "C" int sq_tomography(const void* V, int r, int d, const void* sched, int T, int mode,
                             const void* first, void* err, void* out, int norm_inf, unsigned k0,
                             unsigned k1, unsigned s0, unsigned s1, long long row_offset,
                             void* stream, double stop_err) {
  if (r <= 0) return 0;
  if (d < 1 || d + 1 > kTomoMaxM || T < 1) return (int)hipErrorInvalidValue;
  RngKey key{k0, k1, s0, s1};
  const long long npairs = mode == 0 ? (long long)r * T : (long long)r;
  const size_t lds = 4 * (size_t)(4 * kTomoMaxM + 2) * sizeof(double);   // 64 KiB
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)tomography_kernel,
                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  hipLaunchKernelGGL(tomography_kernel, dim3((unsigned)((npairs + 3) / 4)), dim3(256), lds,
                     (hipStream_t)stream, (const double*)V, r, d, (const long long*)sched, T,
                     mode, (const int*)first, (double*)err, (double*)out, norm_inf, key,
                     row_offset, stop_err);
  return (int)hipGetLastError();
}

extern "C" int sq_mnom_segments(const void* W, long long ldw, const void* wrow, long long m,
                                long long B, const void* Nseg, void* cnt, long long ldc,
                                unsigned k0, unsigned k1, unsigned s0, unsigned s1,
                                const void* sid, int level, void* stream) {
  if (B <= 0 || m <= 0) return 0;
  const long long nseg = (m + kSegP - 1) / kSegP;
  if (nseg > (1LL << 30) || B * nseg > (1LL << 31) - 1) return (int)hipErrorInvalidValue;
  RngKey key{k0, k1, s0, s1};
  hipLaunchKernelGGL(mnom_segments_kernel, dim3((unsigned)(B * nseg)), dim3(256), 0,
                     (hipStream_t)stream, (const double*)W, ldw, (const long long*)wrow, m,
                     (int)nseg, (const double*)Nseg, (double*)cnt, ldc, key,
                     (const long long*)sid, level);
  return (int)hipGetLastError();
}
