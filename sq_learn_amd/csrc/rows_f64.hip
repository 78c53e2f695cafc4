// Exact fp64 E-step over a list of rows on the fp64 matrix cores (SURVEY.md
// §2.6 K1/K2, reference ``sklearn/cluster/_dmeans.py:736-751``: scipy's fp64
// ``cdist`` squared, then the delta-band rule).  Serves
//   * the overflow rows of the fp32-faithful 3-pass kernel and the dense rows
//     of the certified filter at d_pad > 256 (rows whose band edge is crowded
//     beyond what the fp16 filter separates) - device-driven list + count;
//   * every row of the engines that have no fp16 filter (d_pad > 1024, the
//     generic GPU engine) - the identity list.
// One workgroup = 4 waves = one group of 16 rows; the waves split the
// centroid tiles of 16 (t = wave, wave + 4, ...).
//
// Pass 1: D64_ij = |x_i|^2 + |c_j|^2 - 2 x_i.c_j with x.c on
//   v_mfma_f64_16x16x4_f64 (products of fp32 values are exact in fp64), the
//   norms from the same operand values in the same k order; per row the
//   minimum over j and per (row, tile) the minimum rounded down to fp32 (LDS).
// Pass 2: the candidates C_i = {j : D64_ij <= min_i + delta + 4 E_i}, with
//   E_i = (d + 3) 2^-51 (|x_i| + max_j |c_j|)^2 >= |D64 - D| and >= the error
//   of the direct form, go to a per-row LDS list (tiles whose minimum is
//   above every row's threshold are skipped).
// Band: the candidates' distances are recomputed in scipy cdist's direct form
//   sum_f (x_f - c_f)^2 (fp64; 16 lanes per candidate); min, band, kappa-rank
//   pick (band.h's rule) over them - every centroid outside C_i is provably
//   outside the band of the direct-form distances, so the label is the fp64
//   band rule of the re-check kernels.  A row with more than kRfCap
//   candidates (a band wider than 64 centroids) takes the exact direct-form
//   scan over all k (band_pick_wave).
// Outputs per row: label, mind = min distance, corr = mind - d(label) (the
// incremental M-step's correction) and ub = |x - c_label| (Hamerly).
#include "common.h"
#include "band.h"

namespace sq {

typedef double f64x4r __attribute__((ext_vector_type(4)));
constexpr int kRfCap = 64;       // candidates per row kept in LDS
constexpr int kRfTminMax = 512;  // tiles whose per-row minima fit the LDS (k <= 8192)

template <bool V4>
__global__ void __launch_bounds__(256) rows_f64_kernel(
    const float* __restrict__ X, long long ldx, const float* __restrict__ C, long long ldc, int d,
    int k, const long long* __restrict__ rows, const int* __restrict__ count, long long n_direct,
    long long cap, int* __restrict__ labels, float* __restrict__ mind, float* __restrict__ corr,
    float* __restrict__ ub, double delta, RngKey key, long long row_offset) {
  __shared__ double smin[4][16];
  __shared__ double scm[4];
  __shared__ int ccnt[16];
  __shared__ int cidx[16][kRfCap];
  __shared__ double cdd[16][kRfCap];
  __shared__ float tmin[16][kRfTminMax];
  __shared__ double sxn[16], sthr[16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int q = lane >> 4, c16 = lane & 15;
  const long long cnt = rows ? min((long long)*count, cap) : n_direct;
  const int nt = (k + 15) >> 4;
  const bool use_tmin = nt <= kRfTminMax;
  const int dsteps = (d + 15) >> 4;
  const double ebase = (double)(d + 3) * 0x1p-51;
  for (long long g0 = (long long)blockIdx.x * 16; g0 < cnt; g0 += (long long)gridDim.x * 16) {
    auto row_of = [&](int i) -> long long {
      const long long e = min(g0 + i, cnt - 1);
      return rows ? rows[e] : e;
    };
    const float* xr = X + (size_t)row_of(c16) * ldx;   // A operand: row c16
    // distance tile t for rows q + 4 rr, column 16 t + c16 (+inf past k);
    // xi[rr] = |x_{q+4rr}|^2, cn = |c_{16t+c16}|^2, xo = |x_{c16}|^2
    auto tileD = [&](int t, double (&D)[4], double (&xi)[4], double& cn, double& xo) {
      const int j = 16 * t + c16;
      const bool jv = j < k;
      const float* cr = C + (size_t)(jv ? j : 0) * ldc;
      f64x4r acc = {0.0, 0.0, 0.0, 0.0};
      double xs = 0.0, cs = 0.0;
      for (int st = 0; st < dsteps; ++st) {
        const int f = 16 * st + 4 * q;
        double a[4], b[4];
        if (V4 && f + 3 < d) {
          const float4 av = *reinterpret_cast<const float4*>(xr + f);
          const float4 bv = jv ? *reinterpret_cast<const float4*>(cr + f)
                               : make_float4(0.f, 0.f, 0.f, 0.f);
          a[0] = av.x; a[1] = av.y; a[2] = av.z; a[3] = av.w;
          b[0] = bv.x; b[1] = bv.y; b[2] = bv.z; b[3] = bv.w;
        } else {
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            a[s] = f + s < d ? (double)xr[f + s] : 0.0;
            b[s] = (jv && f + s < d) ? (double)cr[f + s] : 0.0;
          }
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[s], b[s], acc, 0, 0, 0);
          xs = fma(a[s], a[s], xs);
          cs = fma(b[s], b[s], cs);
        }
      }
      xs += __shfl_xor(xs, 16, 64);
      xs += __shfl_xor(xs, 32, 64);
      cs += __shfl_xor(cs, 16, 64);
      cs += __shfl_xor(cs, 32, 64);
      cn = cs;
      xo = xs;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        xi[rr] = __shfl(xs, q + 4 * rr, 64);   // lane q + 4rr holds row q + 4rr's norm
        D[rr] = jv ? xi[rr] + cs - 2.0 * acc[rr] : __builtin_inf();
      }
    };

    // ---- pass 1: row minima, per-tile minima, max centroid norm
    if (tid < 16) ccnt[tid] = 0;
    double mn[4] = {__builtin_inf(), __builtin_inf(), __builtin_inf(), __builtin_inf()};
    double cm = 0.0;
    for (int t = wave; t < nt; t += 4) {
      double D[4], xi[4], cn, xo;
      tileD(t, D, xi, cn, xo);
      if (t == 0 && lane < 16) sxn[lane] = xo;   // (wave 0) the 16 row norms
      if (16 * t + c16 < k) cm = fmax(cm, cn);
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        double v = D[rr];
        mn[rr] = fmin(mn[rr], v);
        if (use_tmin) {
#pragma unroll
          for (int o = 1; o < 16; o <<= 1) v = fmin(v, __shfl_xor(v, o, 64));
          if (c16 == 0) tmin[q + 4 * rr][t] = __double2float_rd(v);
        }
      }
    }
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) mn[rr] = fmin(mn[rr], __shfl_xor(mn[rr], o, 64));
      if (c16 == 0) smin[wave][q + 4 * rr] = mn[rr];
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) cm = fmax(cm, __shfl_xor(cm, o, 64));
    if (lane == 0) scm[wave] = cm;
    __syncthreads();
    const double cmax = sqrt(fmax(fmax(scm[0], scm[1]), fmax(scm[2], scm[3])));
    auto rmin = [&](int i) {
      return fmin(fmin(smin[0][i], smin[1][i]), fmin(smin[2][i], smin[3][i]));
    };

    // ---- pass 2: candidate lists (thresholds per row in LDS)
    if (tid < 16) {
      const double sx = sqrt(fmax(sxn[tid], 0.0)) + cmax;
      sthr[tid] = rmin(tid) + delta + 4.0 * ebase * sx * sx;
    }
    __syncthreads();
    for (int t = wave; t < nt; t += 4) {
      // skip a tile whose minimum is above the threshold of all 16 rows
      if (use_tmin && !__any((double)tmin[c16][t] <= sthr[c16])) continue;   // wave-uniform
      double D[4], xi[4], cn, xo;
      tileD(t, D, xi, cn, xo);
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int i = q + 4 * rr;
        if (D[rr] <= sthr[i] && g0 + i < cnt) {
          const int s = atomicAdd(&ccnt[i], 1);
          if (s < kRfCap) cidx[i][s] = 16 * t + c16;
        }
      }
    }
    __syncthreads();

    // ---- band: wave w resolves rows w, w + 4, w + 8, w + 12
    for (int i = wave; i < 16; i += 4) {
      if (g0 + i >= cnt) break;   // wave-uniform
      const long long r = row_of(i);
      const float* xrow = X + (size_t)r * ldx;
      const int nc = ccnt[i];
      auto direct = [&](int j) -> double {   // 16 lanes per candidate (group q)
        const float* cr = C + (size_t)j * ldc;
        double s = 0.0;
        for (int f = 4 * c16; f < d; f += 64) {
          if (V4 && f + 3 < d) {
            const float4 xv = *reinterpret_cast<const float4*>(xrow + f);
            const float4 cv = *reinterpret_cast<const float4*>(cr + f);
            const double e0 = (double)xv.x - (double)cv.x, e1 = (double)xv.y - (double)cv.y;
            const double e2 = (double)xv.z - (double)cv.z, e3 = (double)xv.w - (double)cv.w;
            s = fma(e0, e0, fma(e1, e1, fma(e2, e2, fma(e3, e3, s))));
          } else {
            for (int u = 0; u < 4 && f + u < d; ++u) {
              const double e = (double)xrow[f + u] - (double)cr[f + u];
              s = fma(e, e, s);
            }
          }
        }
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) s += __shfl_xor(s, o, 64);
        return s;
      };
      int pick = 0;
      double mdd = 0.0, dpick = 0.0;
      if (nc <= kRfCap) {
        for (int base = 0; base < nc; base += 4) {   // 4 candidates per round
          const int cl = base + q;
          const int j = cl < nc ? cidx[i][cl] : cidx[i][0];
          const double dd = direct(j);
          if (c16 == 0 && cl < nc) cdd[i][cl] = dd;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        const bool mine = lane < nc;
        const int jm = mine ? cidx[i][lane] : 0;
        const double dm = mine ? cdd[i][lane] : __builtin_inf();
        mdd = dm;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) mdd = fmin(mdd, __shfl_xor(mdd, o, 64));
        const bool inb = mine && dm <= mdd + delta;
        const int b = __popcll(__ballot(inb));
        const int kme = inb ? (((jm & 31) << 20) | (jm >> 5)) : 0x7fffffff;
        int rank = 0;
        for (int tt = 0; tt < nc; ++tt) rank += __shfl(kme, tt, 64) < kme ? 1 : 0;
        const int rsel = band_rank(band_u(key, row_offset + r), b > 0 ? b : 1);
        const unsigned long long pm = __ballot(inb && rank == rsel);
        const int pl = pm ? __ffsll((long long)pm) - 1 : 0;
        pick = __shfl(jm, pl, 64);
        dpick = __shfl(dm, pl, 64);
      } else {
        // a band wider than kRfCap: exact direct-form scan over all k, one
        // lane per centroid (rare: > 64 centroids within delta of the min)
        auto dlane = [&](int j) -> double {
          const float* cr = C + (size_t)j * ldc;
          double s = 0.0;
          for (int f = 0; f < d; ++f) {
            const double e = (double)xrow[f] - (double)cr[f];
            s = fma(e, e, s);
          }
          return s;
        };
        double m = __builtin_inf();
        for (int j = lane; j < k; j += 64) m = fmin(m, dlane(j));
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) m = fmin(m, __shfl_xor(m, o, 64));
        mdd = m;
        pick = band_pick_wave(dlane, k, m + delta, band_u(key, row_offset + r), lane);
        if (pick < 0) pick = 0;
        dpick = dlane(pick);
      }
      if (lane == 0) {
        labels[r] = pick;
        mind[r] = (float)mdd;
        if (corr) corr[r] = (float)(mdd - dpick);
        if (ub) ub[r] = (float)sqrt(dpick) * (1.0f + 0x1p-20f);
      }
    }
    __syncthreads();   // LDS lists reused by the next group
  }
}

}  // namespace sq

using namespace sq;

extern "C" {

// rows/count: device list of row indices and its length (capped at cap);
// rows == null: every row 0 .. n_direct-1.  X fp32 [.][ldx], C fp32 [k][ldc]
// (d used columns of each).  grid: workgroups (each one 16-row group at a time).
int sq_rows_f64(const void* X, long long ldx, const void* C, long long ldc, int d, int k,
                const void* rows, const void* count, long long n_direct, long long cap,
                void* labels, void* mind, void* corr, void* ub, double delta, unsigned k0,
                unsigned k1, unsigned s0, unsigned s1, long long row_offset, int grid,
                void* stream) {
  if (d <= 0 || k <= 0 || ldx < d || ldc < d || grid <= 0) return (int)hipErrorInvalidValue;
  if (rows == nullptr && n_direct <= 0) return 0;
  if (rows != nullptr && (count == nullptr || cap <= 0)) return cap <= 0 ? 0 : (int)hipErrorInvalidValue;
  RngKey key{k0, k1, s0, s1};
  const bool v4 = (d % 4 == 0) && (ldx % 4 == 0) && (ldc % 4 == 0) &&
                  ((uintptr_t)X % 16 == 0) && ((uintptr_t)C % 16 == 0);
  hipStream_t st = (hipStream_t)stream;
  if (v4)
    hipLaunchKernelGGL(rows_f64_kernel<true>, dim3((unsigned)grid), dim3(256), 0, st,
                       (const float*)X, ldx, (const float*)C, ldc, d, k, (const long long*)rows,
                       (const int*)count, n_direct, cap, (int*)labels, (float*)mind, (float*)corr,
                       (float*)ub, delta, key, row_offset);
  else
    hipLaunchKernelGGL(rows_f64_kernel<false>, dim3((unsigned)grid), dim3(256), 0, st,
                       (const float*)X, ldx, (const float*)C, ldc, d, k, (const long long*)rows,
                       (const int*)count, n_direct, cap, (int*)labels, (float*)mind, (float*)corr,
                       (float*)ub, delta, key, row_offset);
  return (int)hipGetLastError();
}

}  // extern "C"
