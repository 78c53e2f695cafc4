// Exact accelerated greedy k-means++ (reference
// sklearn/cluster/_kmeans.py:153-247 and _dmeans.py:153-247).
//
// One step = t candidate centres sampled from the current potential, the t
// trial potentials sum_i w_i min(closest_i, |x_i - c_j|^2), the best trial
// kept.  The step used to be one full pass over X (k - 1 passes of 10 GB at
// 10M x 256).  Here a row is read only when a candidate can improve it:
//
//  1. triangle screen (kmpp_screen_kernel): each row keeps its nearest chosen
//     centre a(i) and closest_i = |x_i - C_a|^2.  |c_j - C_a|^2 > 4.01 closest_i
//     proves |x_i - c_j| > |x_i - C_a| (with the fp32 rounding of both sides
//     covered), so min(closest_i, D_ij) = closest_i without reading the row.
//     Rows with a trial left go to the survivor list;
//  2. certified int8 bound (kmpp_bound_kernel): survivors are read from an
//     int8 copy (per-row scale s_i, stored error norm e_i >= |x_i - x~_i|);
//     the candidates are int8 too, as two terms (c~ = s_c (q1 + q2 / 254),
//     error norm ec_j >= |c_j - c~_j|), so <q_i, q1_j> and <q_i, q2_j> are
//     EXACT int32 MFMA dot products (v_mfma_i32_16x16x64_i8, 16 rows x 16
//     trials per instruction) and |x_i - c_j| >= |x~_i - c~_j| - e_i - ec_j
//     with |x~ - c~|^2 = s^2 |q|^2 + |c~|^2 - 2 s <q, c~> evaluated in fp64
//     (rounding covered); trials still undecided send the row on;
//  3. exact pass (kmpp_exact_kernel): the fp32 direct-form distances
//     sum_f (x_f - c_f)^2 (no norm-expansion cancellation) of the remaining
//     rows; a trial that improves a row (D_ij < closest_i) records D_ij and
//     adds w_i (closest_i - D_ij) to its per-block improvement sum.
//
// Potentials are fixed point: a row's potential is q_i = rint(w_i closest_i
// scale) with one global power-of-two scale chosen so the total stays below
// 2^53, so every sum of q's is an exact fp64 integer: the trial potentials
// P - Delta_j (Delta_j = the improvement sums), the per-block totals and the
// in-block prefix of the two-level sampler (kmpp_pick_kernel: block by
// prefix over the block totals, then row by a workgroup scan of that block)
// are order-independent - the same ids with or without the screens, on any
// number of ranks.  The best trial's improvements are applied lazily (the
// next screen / pick reads the improving rows' D from the mask), so no pass
// touches rows that did not change.
#include "common.h"

namespace sq {

constexpr int kKppTile = 32;          // fp32 features per staged tile (128 B of a row)
constexpr int kKppInitGrid = 16384;   // workgroups of the first-centre pass
constexpr int kKppStride = 36;        // LDS row stride in floats (16-B aligned, skewed banks)

SQ_DEV double kpp_q(float v, double wi, double scale) { return rint((double)v * wi * scale); }

// ------------------------------------- first centre (+ the int8 copy)
// 16 lanes per row (4 rows per wave; float4 loads, 256 contiguous bytes per
// row and instruction): closest_i = |x_i - c0|^2 (fp32, fixed lane-tree
// order), nearest_i = 0, the per-block max of w_i closest_i (the caller
// turns the global max into the fixed-point scale); with Xq: the row's int8
// copy in the same pass - q = rint(x / s) (s = max|x| / 127), e = |x - s q|
// rounded up, q2 = |q|^2 (exact int), features d .. dq-1 zero.  (d, ldx
// multiples of 4.)
__global__ void __launch_bounds__(256) kmpp_init_kernel(
    const float* __restrict__ X, long long ldx, int d, long long n, const float* __restrict__ c0,
    const double* __restrict__ w, float* __restrict__ closest, int* __restrict__ nearest,
    double* __restrict__ bmax, int8_t* __restrict__ Xq, int dq, float* __restrict__ srow,
    float* __restrict__ erow, int* __restrict__ q2row) {
  __shared__ double red[4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int sub = lane & 15;
  const long long i0 = ((long long)blockIdx.x * 4 + wave) * 4 + (lane >> 4);
  const long long stride = (long long)gridDim.x * 16;
  double m = 0.0;
  for (long long ib = i0 - (lane >> 4); ib < n; ib += stride) {   // wave-uniform bound
    const long long i = ib + (lane >> 4);
    const bool ok = i < n;
    const float* x = X + (ok ? i : 0) * ldx;
    float acc = 0.0f, mx = 0.0f;
    for (int f = 4 * sub; f < d; f += 64) {
      const float4 v = *reinterpret_cast<const float4*>(x + f);
      const float4 c = *reinterpret_cast<const float4*>(c0 + f);
      float e = v.x - c.x;
      acc = fmaf(e, e, acc);
      e = v.y - c.y;
      acc = fmaf(e, e, acc);
      e = v.z - c.z;
      acc = fmaf(e, e, acc);
      e = v.w - c.w;
      acc = fmaf(e, e, acc);
      mx = fmaxf(fmaxf(mx, fmaxf(fabsf(v.x), fabsf(v.y))), fmaxf(fabsf(v.z), fabsf(v.w)));
    }
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) {
      acc += __shfl_xor(acc, o, 64);
      mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    }
    if (ok && sub == 0) {
      closest[i] = acc;
      nearest[i] = 0;
    }
    if (ok) m = fmax(m, (double)acc * (w ? w[i] : 1.0));
    if (Xq) {
      const float s = mx > 0.0f ? mx / 127.0f : 1.0f;
      double e2 = 0.0;
      int q2 = 0;
      for (int f = 4 * sub; f < dq; f += 64) {
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (f < d) v = *reinterpret_cast<const float4*>(x + f);
        const float vv[4] = {v.x, v.y, v.z, v.w};
        uint32_t pk = 0;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          int q = 0;
          if (f + u < d) {
            q = (int)fminf(fmaxf(rintf(vv[u] / s), -127.0f), 127.0f);
            const double r = (double)vv[u] - (double)s * (double)q;
            e2 += r * r;
            q2 += q * q;
          }
          pk |= ((uint32_t)(uint8_t)(int8_t)q) << (8 * u);
        }
        if (ok) *reinterpret_cast<uint32_t*>(Xq + i * dq + f) = pk;
      }
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) {
        e2 += __shfl_xor(e2, o, 64);
        q2 += __shfl_xor(q2, o, 64);
      }
      if (ok && sub == 0) {
        srow[i] = s;
        erow[i] = (float)(sqrt(e2) * (1.0 + 1e-6)) * 1.000001f;
        q2row[i] = q2;
      }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmax(m, __shfl_xor(m, o, 64));
  if (lane == 0) red[wave] = m;
  __syncthreads();
  if (threadIdx.x == 0) bmax[blockIdx.x] = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
}

// block b of the fixed row partition (rows [b R, b R + R)): exact fixed-point total
__global__ void __launch_bounds__(256) kmpp_block_totals_kernel(
    const float* __restrict__ closest, const double* __restrict__ w, long long n, long long R,
    double scale, double* __restrict__ block_tot) {
  __shared__ double red[256];
  const long long r0 = (long long)blockIdx.x * R;
  const long long r1 = r0 + R < n ? r0 + R : n;
  double s = 0.0;
  for (long long i = r0 + threadIdx.x; i < r1; i += 256) s += kpp_q(closest[i], w ? w[i] : 1.0, scale);
  red[threadIdx.x] = s;
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if (threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
    __syncthreads();
  }
  if (threadIdx.x == 0) block_tot[blockIdx.x] = red[0];
}

// ------------------------------------------- candidate-centre distances
// blocks 0 .. t-1: candidate j = blockIdx.x -> its two-term int8 copy
// (candq[j], candq[16 + j], zero padded to dq) and cinfo[j]; blocks t ..:
// one wave per chosen centre m < c -> ccmin[m] = min_j |cand_j - C_m|^2
// (NaN-propagating: a NaN keeps every row of centre m live); the whole grid
// zeroes delta_part and the list counters.
SQ_DEV void kmpp_cc_body(int blk, int nblk, 
    const float* __restrict__ cand, const float* __restrict__ C, int c, int d, int t,
    float* __restrict__ ccmin, double* __restrict__ cinfo, int8_t* __restrict__ candq, int dq,
    double* __restrict__ delta_part, long long ndp, int* __restrict__ counters) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long long gid = (long long)blk * 256 + threadIdx.x;
  const long long gsz = (long long)nblk * 256;
  for (long long e = gid; e < ndp; e += gsz) delta_part[e] = 0.0;
  if (gid < 4) counters[gid] = 0;
  if ((int)blk >= t) {
    const int m = 4 * ((int)blk - t) + wave;
    if (m >= c) return;
    const float* cm = C + (size_t)m * d;
    float mn = __builtin_inff();
    for (int j = 0; j < t; ++j) {
      const float* cj = cand + (size_t)j * d;
      float acc = 0.0f;
      for (int f = lane; f < d; f += 64) {
        const float e = cj[f] - cm[f];
        acc = fmaf(e, e, acc);
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
      mn = (acc != acc || acc < mn) ? acc : mn;
    }
    if (lane == 0) ccmin[m] = mn;
    return;
  }
  const int j = blk;
  const float* cj = cand + (size_t)j * d;
  {
    // two-term int8 candidate: y = c / s_c, q1 = rint(y), q2 = rint(254 (y - q1)),
    // c~ = s_c (q1 + q2 / 254); cinfo[j] = (s_c, ec >= |c - c~|, |c~|^2, 0) fp64
    __shared__ float redf[4];
    __shared__ double redd[2][4];
    float mx = 0.0f;
    for (int f = threadIdx.x; f < d; f += 256) mx = fmaxf(mx, fabsf(cj[f]));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    if (lane == 0) redf[wave] = mx;
    __syncthreads();
    mx = fmaxf(fmaxf(redf[0], redf[1]), fmaxf(redf[2], redf[3]));
    const double sc = mx > 0.0f ? (double)mx / 127.0 : 1.0;
    double er = 0.0, c2 = 0.0;
    for (int f = threadIdx.x; f < dq; f += 256) {
      int q1 = 0, q2 = 0;
      if (f < d) {
        const double y = (double)cj[f] / sc;
        q1 = (int)fmin(fmax(rint(y), -127.0), 127.0);
        q2 = (int)fmin(fmax(rint((y - (double)q1) * 254.0), -127.0), 127.0);
        const double ct = sc * ((double)q1 + (double)q2 / 254.0);
        er += ((double)cj[f] - ct) * ((double)cj[f] - ct);
        c2 += ct * ct;
      }
      candq[(size_t)j * dq + f] = (int8_t)q1;
      candq[(size_t)(16 + j) * dq + f] = (int8_t)q2;
    }
    er = wave_sum(er);
    c2 = wave_sum(c2);
    if (lane == 0) { redd[0][wave] = er; redd[1][wave] = c2; }
    __syncthreads();
    if (threadIdx.x == 0) {
      const double e = (redd[0][0] + redd[0][1]) + (redd[0][2] + redd[0][3]);
      const double q = (redd[1][0] + redd[1][1]) + (redd[1][2] + redd[1][3]);
      cinfo[j * 4 + 0] = sc;
      cinfo[j * 4 + 1] = sqrt(e) * (1.0 + 1e-12) + 1e-12 * sqrt(q);
      cinfo[j * 4 + 2] = q;
      cinfo[j * 4 + 3] = 0.0;
    }
  }
}

// Row lists are per-block segments: block b of the fixed partition owns
// list[b R, b R + count[b]) (no global atomics - a single list counter for
// 10M rows serialised ~156k wave atomics per pass).  Append of this lane's
// item when ``take``: one LDS atomic per wave.
SQ_DEV void seg_append(bool take, int value, int* __restrict__ seg, int* lcnt) {
  const unsigned long long b = __ballot(take);
  if (b == 0ull) return;
  const int lane = threadIdx.x & 63;
  int base = 0;
  if (lane == 0) base = atomicAdd(lcnt, (int)__popcll(b));
  base = __shfl(base, 0, 64);
  if (take) {
    const unsigned long long below = b & ((1ull << lane) - 1ull);
    seg[base + (int)__popcll(below)] = value;
  }
}

// ---------------------------------------------------- 1. triangle screen
// lazy update of the previous step's winner (best_prev < 0: none), mask_out
// cleared, rows with a live trial appended to this block's segment of surv
// (prune) or of exact (!prune); scount / ecount[b] = the segment length.
SQ_DEV void kmpp_screen_body(int blk, 
    float* __restrict__ closest, int* __restrict__ nearest,
    const uint16_t* __restrict__ mask_prev, const float* __restrict__ Dprev,
    const int* __restrict__ best_prev, int c_prev, const float* __restrict__ ccmin, long long n,
    long long R, uint16_t* __restrict__ mask_out, int* __restrict__ surv,
    int* __restrict__ exact, int* __restrict__ scount, int* __restrict__ ecount, int prune) {
  __shared__ int lcnt;
  const int bp = best_prev ? *best_prev : -1;
  const long long r0 = (long long)blk * R;
  const long long r1 = r0 + R < n ? r0 + R : n;
  int* seg = (prune ? surv : exact) + r0;
  if (threadIdx.x == 0) lcnt = 0;
  __syncthreads();
  for (long long i0 = r0; i0 < r1; i0 += 256) {
    const long long i = i0 + threadIdx.x;
    bool live = false;
    if (i < r1) {
      float cl = closest[i];
      int a = nearest[i];
      if (bp >= 0 && ((mask_prev[i] >> bp) & 1u)) {
        cl = Dprev[(size_t)bp * n + i];
        a = c_prev;
        closest[i] = cl;
        nearest[i] = a;
      }
      mask_out[i] = 0;
      if (!prune) {
        live = true;
      } else if (cl > 0.0f) {
        live = !(ccmin[a] > 4.01f * cl);   // some trial within 2 sqrt(closest) of C_a
      }
    }
    seg_append(live, (int)i, seg, &lcnt);
  }
  __syncthreads();
  if (threadIdx.x == 0) (prune ? scount : ecount)[blk] = lcnt;
}

// ------------------------------------------------ 2. certified int8 bound
typedef int kpp_v4i __attribute__((ext_vector_type(4)));

// <q_row, q1_j> and <q_row, q2_j> for the 16 rows of a group (row slot =
// lane & 15, -1: none) and the 16 trial slots: lane l supplies 16 bytes of
// row (l & 15) and of trial (l & 15) at k-block l >> 4 of every 64-feature
// step; out: lane l = trial l & 15, rows 4 (l >> 4) + i
SQ_DEV void kpp_i8_dots(const int8_t* __restrict__ Xq, int dq, int row,
                        const int8_t* __restrict__ cb, int lane, kpp_v4i& hi, kpp_v4i& lo) {
  const int c16 = lane & 15, kb = lane >> 4;
  hi = kpp_v4i{0, 0, 0, 0};
  lo = kpp_v4i{0, 0, 0, 0};
  const int8_t* xr = Xq + (size_t)(row >= 0 ? row : 0) * dq + 16 * kb;
  const int8_t* b1 = cb + (size_t)c16 * dq + 16 * kb;
  const int8_t* b2 = cb + (size_t)(16 + c16) * dq + 16 * kb;
  for (int s = 0; s < dq; s += 64) {
    kpp_v4i a = kpp_v4i{0, 0, 0, 0};
    if (row >= 0) a = *reinterpret_cast<const kpp_v4i*>(xr + s);
    const kpp_v4i bh = *reinterpret_cast<const kpp_v4i*>(b1 + s);
    const kpp_v4i bl = *reinterpret_cast<const kpp_v4i*>(b2 + s);
    hi = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, bh, hi, 0, 0, 0);
    lo = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, bl, lo, 0, 0, 0);
  }
}

// Each wave takes two 16-row groups per iteration: both groups' row ids,
// then their int8 rows (NS 16-byte loads per lane each, NS = dq / 64 known
// at compile time up to dq = 256) and per-row scalars are all in flight
// before the MFMAs - the row gathers, not the int8 MFMAs, bound this pass.
template <int NS>
SQ_DEV void kmpp_bound_body(int blk, 
    const int8_t* __restrict__ Xq, int dq, const float* __restrict__ srow,
    const float* __restrict__ erow, const int* __restrict__ q2row,
    const float* __restrict__ closest, const int8_t* __restrict__ candq,
    const double* __restrict__ cinfo, int t, int d, long long R, const int* __restrict__ surv,
    const int* __restrict__ scount, int* __restrict__ exact, int* __restrict__ ecount) {
  extern __shared__ __attribute__((aligned(16))) int8_t cb[];   // [2][16][dq]
  __shared__ int lcnt;
  for (int e = threadIdx.x * 16; e < 32 * dq; e += 256 * 16)
    *reinterpret_cast<uint4*>(cb + e) = *reinterpret_cast<const uint4*>(candq + e);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c16 = lane & 15, kb = lane >> 4;
  const long long r0 = (long long)blk * R;
  const int cnt = scount[blk];
  const int* sseg = surv + r0;
  int* eseg = exact + r0;
  if (threadIdx.x == 0) lcnt = 0;
  __syncthreads();
  // the exact pass's fp32 direct-form D carries <= 3 (d + 2) u relative error
  const float lim_rel = 1.0f + 3.0f * (float)(d + 2) * 5.9604645e-08f + 1e-6f;
  const bool jv = c16 < t;
  // the trial's scale and error norm, rounded UP to fp32 (they only enter as
  // magnitudes of upper-bounded terms); |c~|^2 to nearest (its rounding is
  // inside the 1e-6 absolute-sum margin below)
  const float sc = jv ? (float)cinfo[c16 * 4 + 0] * (1.0f + 1.2e-7f) : 1.0f;
  const float ec = jv ? (float)cinfo[c16 * 4 + 1] * (1.0f + 1.2e-7f) : 0.0f;
  const float cc2 = jv ? (float)cinfo[c16 * 4 + 2] : 0.0f;
  const int nsd = NS > 0 ? NS : dq / 64;
  const int8_t* b1 = cb + (size_t)c16 * dq + 16 * kb;
  const int8_t* b2 = cb + (size_t)(16 + c16) * dq + 16 * kb;
  // the row ids of the next iteration are fetched one iteration ahead
  int nrow[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int e = wave * 32 + 16 * h + c16;
    nrow[h] = e < cnt ? sseg[e] : -1;
  }
  for (int g0 = wave * 32; g0 < cnt; g0 += 128) {
    int row[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      row[h] = nrow[h];
      const int e = g0 + 128 + 16 * h + c16;
      nrow[h] = e < cnt ? sseg[e] : -1;
    }
    // per-row scalars of the lane's row slot c16 (all 4 lane copies load them)
    float rs[2], re_[2], rcl[2];
    int rq2[2];
    kpp_v4i hi[2], lo[2];
    if constexpr (NS > 0) {
      kpp_v4i a[2][NS > 0 ? NS : 1];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int8_t* xr = Xq + (size_t)(row[h] >= 0 ? row[h] : 0) * dq + 16 * kb;
#pragma unroll
        for (int s4 = 0; s4 < NS; ++s4)
          a[h][s4] = row[h] >= 0 ? *reinterpret_cast<const kpp_v4i*>(xr + 64 * s4)
                                 : kpp_v4i{0, 0, 0, 0};
        const int rr = row[h] >= 0 ? row[h] : 0;
        rs[h] = srow[rr];
        re_[h] = erow[rr];
        rq2[h] = q2row[rr];
        rcl[h] = closest[rr];
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        hi[h] = kpp_v4i{0, 0, 0, 0};
        lo[h] = kpp_v4i{0, 0, 0, 0};
#pragma unroll
        for (int s4 = 0; s4 < NS; ++s4) {
          const kpp_v4i bh = *reinterpret_cast<const kpp_v4i*>(b1 + 64 * s4);
          const kpp_v4i bl = *reinterpret_cast<const kpp_v4i*>(b2 + 64 * s4);
          hi[h] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[h][s4], bh, hi[h], 0, 0, 0);
          lo[h] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[h][s4], bl, lo[h], 0, 0, 0);
        }
      }
    } else {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int rr = row[h] >= 0 ? row[h] : 0;
        rs[h] = srow[rr];
        re_[h] = erow[rr];
        rq2[h] = q2row[rr];
        rcl[h] = closest[rr];
        kpp_i8_dots(Xq, dq, row[h], cb, lane, hi[h], lo[h]);
      }
    }
    (void)nsd;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      unsigned long long bal[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int src = 4 * kb + i;   // the row slot of result register i
        const int rr = __shfl(row[h], src, 64);
        const float s = __shfl(rs[h], src, 64);
        const float er = __shfl(re_[h], src, 64);
        const float q2 = (float)__shfl(rq2[h], src, 64);
        const float cl = __shfl(rcl[h], src, 64);
        bool need = false;
        if (jv && rr >= 0) {
          // fp32 with rigorous margins: every term below carries <= 7 u of
          // relative rounding (the int32 dots and |q|^2 convert exactly below
          // 2^24, within u above; the sum Ihi + Ilo / 254 rounds relative to
          // itself), so |Dq_fl - Dq| <= 1e-6 (A + |c~|^2 + 2 |dot|)
          const float A = s * s * q2;
          const float dot = s * sc * ((float)hi[h][i] + (float)lo[h][i] * (1.0f / 254.0f));
          const float Dq = (A + cc2) - 2.0f * dot;
          const float Dlb = Dq - 1e-6f * (A + cc2 + 2.0f * fabsf(dot));
          float lb = 0.0f;
          if (Dlb > 0.0f) {
            const float r = __builtin_amdgcn_sqrtf(Dlb) * (1.0f - 1e-6f) - er - ec;
            lb = r > 0.0f ? r * r * (1.0f - 1e-6f) : 0.0f;
          }
          need = !(lb > cl * lim_rel);
        }
        bal[i] = __ballot(need);
      }
      // row slot c16 (lanes < 16): rows 4 q + i live in lanes [16 q, 16 q + 16) of bal[i]
      const int q = c16 >> 2, ii = c16 & 3;
      const unsigned long long bi = ii == 0 ? bal[0] : ii == 1 ? bal[1] : ii == 2 ? bal[2] : bal[3];
      const bool take = lane < 16 && row[h] >= 0 && ((bi >> (16 * q)) & 0xFFFFull) != 0ull;
      seg_append(take, row[h], eseg, &lcnt);
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) ecount[blk] = lcnt;
}

// test hook: out[r][j] = <q_r, q1_j>, out[n + r][j]... (int32 [2][n][16]) for rows 0..n-1
__global__ void __launch_bounds__(64) kmpp_dots_kernel(const int8_t* __restrict__ Xq, int dq,
                                                       long long n,
                                                       const int8_t* __restrict__ candq,
                                                       int* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) int8_t cb[];
  for (int e = threadIdx.x * 16; e < 32 * dq; e += 64 * 16)
    *reinterpret_cast<uint4*>(cb + e) = *reinterpret_cast<const uint4*>(candq + e);
  __syncthreads();
  const int lane = threadIdx.x;
  const long long g0 = (long long)blockIdx.x * 16;
  const long long r = g0 + (lane & 15);
  kpp_v4i hi, lo;
  kpp_i8_dots(Xq, dq, r < n ? (int)r : -1, cb, lane, hi, lo);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const long long rr = g0 + 4 * (lane >> 4) + i;
    if (rr < n) {
      out[rr * 16 + (lane & 15)] = hi[i];
      out[(n + rr) * 16 + (lane & 15)] = lo[i];
    }
  }
}

// ------------------------------------------------------- 3. exact pass
// One lane per row (64 rows per wave pass), rows staged through LDS in
// 32-feature tiles (8 lanes x 16 B per row, the next tile's loads in flight
// during the current tile's FMAs); a row improved by trial j records D_ij
// and its fixed-point improvement, summed per lane, per wave, then per block
// (exact integers: any order) and STORED as delta_part[block][j] - one write
// per block instead of one fp64 atomic per improved (row, trial).
template <int TMAX>
SQ_DEV void kmpp_exact_body(int blk, 
    const float* __restrict__ X, long long ldx, int d, long long n, int t,
    const float* __restrict__ cand, const float* __restrict__ closest,
    const double* __restrict__ w, double scale, const int* __restrict__ exact,
    const int* __restrict__ ecount, uint16_t* __restrict__ mask_out, float* __restrict__ Dout,
    double* __restrict__ delta_part, long long R) {
  __shared__ __attribute__((aligned(16))) float tile[4][64 * kKppStride];
  __shared__ double dred[4][TMAX];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float* my = tile[wave];
  const int cnt = ecount[blk];
  const int* eseg = exact + (long long)blk * R;
  const long long nb = (cnt + 63) / 64;
  const int ntiles = (d + kKppTile - 1) / kKppTile;
  const int lrow = lane >> 3, lchunk = lane & 7;
  double dsum[TMAX];
#pragma unroll
  for (int j = 0; j < TMAX; ++j) dsum[j] = 0.0;
  for (long long b = wave; b < nb; b += 4) {
    const long long e = b * 64 + lane;
    const int row = e < cnt ? eseg[e] : -1;
    int rq[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) rq[q] = __shfl(row, q * 8 + lrow, 64);
    float4 v[8];
    auto fetch = [&](int tix) {
      const int f = tix * kKppTile + lchunk * 4;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        v[q] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (rq[q] >= 0 && f < d) v[q] = *reinterpret_cast<const float4*>(X + (size_t)rq[q] * ldx + f);
      }
    };
    float acc[TMAX];
#pragma unroll
    for (int j = 0; j < TMAX; ++j) acc[j] = 0.0f;
    fetch(0);
    for (int tix = 0; tix < ntiles; ++tix) {
      // stage: row slot q * 8 + (lane >> 3), 16-B chunk lane & 7
#pragma unroll
      for (int q = 0; q < 8; ++q)
        *reinterpret_cast<float4*>(my + (q * 8 + lrow) * kKppStride + lchunk * 4) = v[q];
      if (tix + 1 < ntiles) fetch(tix + 1);
      const int f0 = tix * kKppTile;
      // the row's 32 features in registers, then trial by trial: a trial's
      // 32 wave-uniform features are two 64-byte scalar loads (one wait per
      // trial, not one per 4 features); a short last tile is zero padded on
      // both sides (adds 0), so the fmaf chain per trial stays sequential
      float xv[kKppTile];
#pragma unroll
      for (int c4 = 0; c4 < kKppTile / 4; ++c4) {
        const float4 x4 = *reinterpret_cast<const float4*>(my + lane * kKppStride + c4 * 4);
        xv[4 * c4] = x4.x;
        xv[4 * c4 + 1] = x4.y;
        xv[4 * c4 + 2] = x4.z;
        xv[4 * c4 + 3] = x4.w;
      }
      const bool full_tile = f0 + kKppTile <= d;
#pragma unroll
      for (int j = 0; j < TMAX; ++j) {
        if (j < t) {
          const float* c = cand + (size_t)j * d + f0;   // wave-uniform: scalar loads
          if (full_tile) {
#pragma unroll
            for (int u = 0; u < kKppTile; ++u) {
              const float ev = xv[u] - c[u];
              acc[j] = fmaf(ev, ev, acc[j]);
            }
          } else {
            for (int u = 0; u < d - f0; ++u) {
              const float ev = xv[u] - c[u];
              acc[j] = fmaf(ev, ev, acc[j]);
            }
          }
        }
      }
    }
    if (row >= 0) {
      const float cl = closest[row];
      const double wi = w ? w[row] : 1.0;
      const double qcl = kpp_q(cl, wi, scale);
      uint32_t m = 0;
#pragma unroll
      for (int j = 0; j < TMAX; ++j) {
        if (j < t && acc[j] < cl) {
          m |= 1u << j;
          Dout[(size_t)j * n + row] = acc[j];
          dsum[j] += qcl - kpp_q(acc[j], wi, scale);
        }
      }
      mask_out[row] = (uint16_t)m;
    }
  }
#pragma unroll
  for (int j = 0; j < TMAX; ++j) {
    const double s = wave_sum(dsum[j]);
    if (lane == 0) dred[wave][j] = s;
  }
  __syncthreads();
  if (threadIdx.x < t && threadIdx.x < TMAX) {
    const int j = threadIdx.x;
    delta_part[(long long)blk * t + j] = (dred[0][j] + dred[1][j]) + (dred[2][j] + dred[3][j]);
  }
}

// -------------------------------------------------- two-level sampling
// One workgroup per value v: the first row (in row order) whose inclusive
// fixed-point prefix reaches v - np.searchsorted(stable_cumsum, v) on the
// current potentials (after the winning trial of mask / D / best).
SQ_DEV void kmpp_pick_body(int blk, 
    const double* __restrict__ block_tot, int G, long long R, long long n,
    const double* __restrict__ vals, const float* __restrict__ closest,
    const uint16_t* __restrict__ mask, const float* __restrict__ D, const int* __restrict__ best,
    const double* __restrict__ w, double scale, long long* __restrict__ pos,
    const float* __restrict__ X, long long ldx, int d, float* __restrict__ cands,
    long long* __restrict__ cand_ids, long long row_offset, long long n_global) {
  __shared__ double sc[256];
  __shared__ long long found;
  __shared__ double base;
  const double v = vals[blk];
  const int tid = threadIdx.x;
  const int bp = best ? *best : -1;
  // ---- block: per-thread chunk sums, WG exclusive scan, first crossing
  const int chunk = (G + 255) / 256;
  const int g0 = min(G, tid * chunk), g1 = min(G, g0 + chunk);
  double s = 0.0;
  for (int g = g0; g < g1; ++g) s += block_tot[g];
  sc[tid] = s;
  if (tid == 0) found = (long long)G - 1;
  __syncthreads();
  for (int o = 1; o < 256; o <<= 1) {   // Hillis-Steele inclusive scan (exact integers)
    const double a = tid >= o ? sc[tid - o] : 0.0;
    __syncthreads();
    sc[tid] += a;
    __syncthreads();
  }
  const double excl = sc[tid] - s;   // exclusive prefix of this thread's chunk
  double run = excl;
  long long hit = -1;
  for (int g = g0; g < g1; ++g) {
    run += block_tot[g];
    if (run >= v) { hit = g; break; }
  }
  if (hit >= 0) atomicMin(&found, hit);
  __syncthreads();
  const long long bsel = found;
  // exclusive prefix of the chosen block: from the thread whose chunk holds it
  if (bsel >= g0 && bsel < g1) {
    double p = excl;
    for (long long g = g0; g < bsel; ++g) p += block_tot[g];
    base = p;
  }
  __syncthreads();
  const double resid = v - base;
  // ---- row within the block
  const long long r0 = bsel * R;
  const long long r1 = r0 + R < n ? r0 + R : n;
  const long long rchunk = (r1 - r0 + 255) / 256;
  const long long a0 = min(r1, r0 + tid * rchunk), a1 = min(r1, a0 + rchunk);
  auto qrow = [&](long long i) -> double {
    float cl = closest[i];
    if (bp >= 0 && ((mask[i] >> bp) & 1u)) cl = D[(size_t)bp * n + i];
    return kpp_q(cl, w ? w[i] : 1.0, scale);
  };
  s = 0.0;
  for (long long i = a0; i < a1; ++i) s += qrow(i);
  __syncthreads();
  sc[tid] = s;
  if (tid == 0) found = r1 > r0 ? r1 - 1 : (n > 0 ? n - 1 : 0);
  __syncthreads();
  for (int o = 1; o < 256; o <<= 1) {
    const double a = tid >= o ? sc[tid - o] : 0.0;
    __syncthreads();
    sc[tid] += a;
    __syncthreads();
  }
  run = sc[tid] - s;
  hit = -1;
  for (long long i = a0; i < a1; ++i) {
    run += qrow(i);
    if (run >= resid) { hit = i; break; }
  }
  if (hit >= 0) atomicMin(&found, hit);
  __syncthreads();
  if (tid == 0) pos[blk] = found;
  if (cands) {
    // the candidate row itself (and its global id), clamped to the shard
    const long long r = found < 0 ? 0 : (found > n - 1 ? n - 1 : found);
    for (int f = tid; f < d; f += 256) cands[(size_t)blk * d + f] = X[(size_t)r * ldx + f];
    if (tid == 0) {
      const long long g = r + row_offset;
      cand_ids[blk] = g < 0 ? 0 : (g > n_global - 1 ? n_global - 1 : g);
    }
  }
}

// ------------------------------------------- winner of one centre (1 rank)
// Delta_j = sum over blocks of delta_part[b][j] (exact integers), the trial
// potentials P - Delta_j, the first minimal one wins (torch.argmin's rule):
// P, the block totals, centres[c], ids[c], the lazily applied winner and the
// next centre's sampling values draws_next * P - one launch instead of the
// host-side chain of small tensor ops.
SQ_DEV void kmpp_finish_body(
    const double* __restrict__ delta_part, int G, int t, double* __restrict__ block_tot,
    double* __restrict__ P, const double* __restrict__ draws_next, double* __restrict__ vals,
    const float* __restrict__ cands, const long long* __restrict__ cand_ids, int d,
    float* __restrict__ centers, long long* __restrict__ ids, int c, int* __restrict__ best_out) {
  __shared__ double red[64][16];
  __shared__ double dj[16];
  __shared__ int sb;
  __shared__ double sP;
  const int tid = threadIdx.x, j = tid & 15, g = tid >> 4;
  double s = 0.0;
  if (j < t) {
#pragma unroll 8
    for (int b = g; b < G; b += 64) s += delta_part[(size_t)b * t + j];
  }
  red[g][j] = s;
  __syncthreads();
  if (tid < t) {
    double a = 0.0;
    for (int q = 0; q < 64; ++q) a += red[q][tid];
    dj[tid] = a;
  }
  __syncthreads();
  if (tid == 0) {
    const double p0 = *P;
    int bj = 0;
    double bv = p0 - dj[0];
    for (int q = 1; q < t; ++q) {
      const double v = p0 - dj[q];
      if (v < bv) { bv = v; bj = q; }
    }
    sb = bj;
    sP = bv;
    *P = bv;
    *best_out = bj;
    ids[c] = cand_ids[bj];
  }
  __syncthreads();
  const int bj = sb;
  if (draws_next && tid < t) vals[tid] = draws_next[tid] * sP;
  for (int b = tid; b < G; b += 1024) block_tot[b] -= delta_part[(size_t)b * t + bj];
  for (int f = tid; f < d; f += 1024) centers[(size_t)c * d + f] = cands[(size_t)bj * d + f];
}


// ---------------------------------------------- single-restart kernels
__global__ void __launch_bounds__(256) kmpp_cc_kernel(
    const float* __restrict__ cand, const float* __restrict__ C, int c, int d, int t,
    float* __restrict__ ccmin, double* __restrict__ cinfo, int8_t* __restrict__ candq, int dq,
    double* __restrict__ delta_part, long long ndp, int* __restrict__ counters) {
  kmpp_cc_body(blockIdx.x, gridDim.x, cand, C, c, d, t, ccmin, cinfo, candq, dq, delta_part, ndp,
               counters);
}
__global__ void __launch_bounds__(256) kmpp_screen_kernel(
    float* __restrict__ closest, int* __restrict__ nearest, const uint16_t* __restrict__ mask_prev,
    const float* __restrict__ Dprev, const int* __restrict__ best_prev, int c_prev,
    const float* __restrict__ ccmin, long long n, long long R, uint16_t* __restrict__ mask_out,
    int* __restrict__ surv, int* __restrict__ exact, int* __restrict__ scount,
    int* __restrict__ ecount, int prune) {
  kmpp_screen_body(blockIdx.x, closest, nearest, mask_prev, Dprev, best_prev, c_prev, ccmin, n, R,
                   mask_out, surv, exact, scount, ecount, prune);
}
template <int NS>
__global__ void __launch_bounds__(256) kmpp_bound_kernel(
    const int8_t* __restrict__ Xq, int dq, const float* __restrict__ srow,
    const float* __restrict__ erow, const int* __restrict__ q2row,
    const float* __restrict__ closest, const int8_t* __restrict__ candq,
    const double* __restrict__ cinfo, int t, int d, long long R, const int* __restrict__ surv,
    const int* __restrict__ scount, int* __restrict__ exact, int* __restrict__ ecount) {
  kmpp_bound_body<NS>(blockIdx.x, Xq, dq, srow, erow, q2row, closest, candq, cinfo, t, d, R, surv,
                      scount, exact, ecount);
}
template <int TMAX>
__global__ void __launch_bounds__(256) kmpp_exact_kernel(
    const float* __restrict__ X, long long ldx, int d, long long n, int t,
    const float* __restrict__ cand, const float* __restrict__ closest,
    const double* __restrict__ w, double scale, const int* __restrict__ exact,
    const int* __restrict__ ecount, uint16_t* __restrict__ mask_out, float* __restrict__ Dout,
    double* __restrict__ delta_part, long long R) {
  kmpp_exact_body<TMAX>(blockIdx.x, X, ldx, d, n, t, cand, closest, w, scale, exact, ecount,
                        mask_out, Dout, delta_part, R);
}
__global__ void __launch_bounds__(256) kmpp_pick_kernel(
    const double* __restrict__ block_tot, int G, long long R, long long n,
    const double* __restrict__ vals, const float* __restrict__ closest,
    const uint16_t* __restrict__ mask, const float* __restrict__ D, const int* __restrict__ best,
    const double* __restrict__ w, double scale, long long* __restrict__ pos,
    const float* __restrict__ X, long long ldx, int d, float* __restrict__ cands,
    long long* __restrict__ cand_ids, long long row_offset, long long n_global) {
  kmpp_pick_body(blockIdx.x, block_tot, G, R, n, vals, closest, mask, D, best, w, scale, pos, X,
                 ldx, d, cands, cand_ids, row_offset, n_global);
}
__global__ void __launch_bounds__(1024) kmpp_finish_kernel(
    const double* __restrict__ delta_part, int G, int t, double* __restrict__ block_tot,
    double* __restrict__ P, const double* __restrict__ draws_next, double* __restrict__ vals,
    const float* __restrict__ cands, const long long* __restrict__ cand_ids, int d,
    float* __restrict__ centers, long long* __restrict__ ids, int c, int* __restrict__ best_out) {
  kmpp_finish_body(delta_part, G, t, block_tot, P, draws_next, vals, cands, cand_ids, d, centers,
                   ids, c, best_out);
}

// ---------------------------------------------- batched restarts
// NR independent k-means++ runs (the restarts of one fit, their draws taken
// up front in the reference's order) advance through their centres in
// lockstep, one launch per phase for all of them.  Per-restart state through
// a device table [NR][kKppNF] of pointers (and the fixed-point scale); the
// rows (X, its int8 copy) are shared.  The row passes (screen / bound /
// exact) order their workgroups row block first, restart second, so the NR
// restarts' workgroups of one row block run side by side and a row two of
// them need is read from HBM once (the L2 / MALL serves the rest).
constexpr int kKppNF = 32;
enum KppField {
  F_CLOSEST = 0, F_NEAREST, F_MASK0, F_MASK1, F_D0, F_D1, F_SURV, F_EXACT, F_SCOUNT, F_ECOUNT,
  F_CC, F_CINFO, F_CANDQ, F_DELTA, F_BTOT, F_POS, F_CANDS, F_CANDIDS, F_CENTERS, F_IDS, F_P,
  F_VALS, F_DRAWS, F_BEST, F_COUNTERS, F_SCALE
};
struct KppArgs {
  const long long* tab;
  int nr;
  const float* X;
  long long ldx;
  int d;
  long long n;
  int t, k, dq;
  const int8_t* Xq;
  const float* srow;
  const float* erow;
  const int* q2row;
  const double* w;
  long long R;
  int G;
  int c, c_prev, cur, prune;
  long long row_offset, n_global, doff, ndp;
  int per;   // workgroups per restart of the cc phase
  // fused screen / bound (ops 7, 8): the union of the restarts' survivors
  int* useg;          // per-block segments of row ids (any restart live)
  uint16_t* umask;    // the restarts live for useg[i] (bit r)
  int* ucount;        // [G] segment lengths
  int tp;             // trial columns per restart (t rounded up to a power of two)
};
// Row-pass workgroup -> (row block b, restart r), XCD-aware: workgroups are
// dealt to the 8 XCDs round robin (id % 8), so the nr restarts of row block
// b take ids with the same residue - one XCD, one L2 for that block's rows
// (read by nr workgroups close in time).  Grid: ceil(G / 8) * 8 * nr.
SQ_DEV bool kpp_decode(int id, int nr, int G, int& b, int& r) {
  const int x = id & 7, q = id >> 3;
  b = (q / nr) * 8 + x;
  r = q % nr;
  return b < G;
}
template <typename P_>
SQ_DEV P_ kf(const KppArgs& a, int r, int f) {
  return reinterpret_cast<P_>(a.tab[(size_t)r * kKppNF + f]);
}
SQ_DEV double kscale(const KppArgs& a, int r) {
  return __longlong_as_double(a.tab[(size_t)r * kKppNF + F_SCALE]);
}

__global__ void __launch_bounds__(256) kmpp_cc_batch_kernel(KppArgs a) {
  const int r = blockIdx.x / a.per, b = blockIdx.x % a.per;
  kmpp_cc_body(b, a.per, kf<const float*>(a, r, F_CANDS), kf<const float*>(a, r, F_CENTERS), a.c,
               a.d, a.t, kf<float*>(a, r, F_CC), kf<double*>(a, r, F_CINFO),
               kf<int8_t*>(a, r, F_CANDQ), a.dq, kf<double*>(a, r, F_DELTA), a.ndp,
               kf<int*>(a, r, F_COUNTERS));
}
__global__ void __launch_bounds__(256) kmpp_screen_batch_kernel(KppArgs a) {
  int b, r;
  if (!kpp_decode(blockIdx.x, a.nr, a.G, b, r)) return;
  const int prev = 1 - a.cur;
  kmpp_screen_body(b, kf<float*>(a, r, F_CLOSEST), kf<int*>(a, r, F_NEAREST),
                   kf<const uint16_t*>(a, r, F_MASK0 + prev), kf<const float*>(a, r, F_D0 + prev),
                   a.c_prev >= 0 ? kf<const int*>(a, r, F_BEST) : nullptr, a.c_prev,
                   kf<const float*>(a, r, F_CC), a.n, a.R, kf<uint16_t*>(a, r, F_MASK0 + a.cur),
                   kf<int*>(a, r, F_SURV), kf<int*>(a, r, F_EXACT), kf<int*>(a, r, F_SCOUNT),
                   kf<int*>(a, r, F_ECOUNT), a.prune);
}
template <int NS>
__global__ void __launch_bounds__(256) kmpp_bound_batch_kernel(KppArgs a) {
  int b, r;
  if (!kpp_decode(blockIdx.x, a.nr, a.G, b, r)) return;
  kmpp_bound_body<NS>(b, a.Xq, a.dq, a.srow, a.erow, a.q2row, kf<const float*>(a, r, F_CLOSEST),
                      kf<const int8_t*>(a, r, F_CANDQ), kf<const double*>(a, r, F_CINFO), a.t, a.d,
                      a.R, kf<const int*>(a, r, F_SURV), kf<const int*>(a, r, F_SCOUNT),
                      kf<int*>(a, r, F_EXACT), kf<int*>(a, r, F_ECOUNT));
}
template <int TMAX>
__global__ void __launch_bounds__(256) kmpp_exact_batch_kernel(KppArgs a) {
  int b, r;
  if (!kpp_decode(blockIdx.x, a.nr, a.G, b, r)) return;
  kmpp_exact_body<TMAX>(b, a.X, a.ldx, a.d, a.n, a.t, kf<const float*>(a, r, F_CANDS),
                        kf<const float*>(a, r, F_CLOSEST), a.w, kscale(a, r),
                        kf<const int*>(a, r, F_EXACT), kf<const int*>(a, r, F_ECOUNT),
                        kf<uint16_t*>(a, r, F_MASK0 + a.cur), kf<float*>(a, r, F_D0 + a.cur),
                        kf<double*>(a, r, F_DELTA), a.R);
}
__global__ void __launch_bounds__(256) kmpp_pick_batch_kernel(KppArgs a) {
  const int r = blockIdx.x / a.t, b = blockIdx.x % a.t;
  const int prev = 1 - a.cur;
  kmpp_pick_body(b, kf<const double*>(a, r, F_BTOT), a.G, a.R, a.n, kf<const double*>(a, r, F_VALS),
                 kf<const float*>(a, r, F_CLOSEST), kf<const uint16_t*>(a, r, F_MASK0 + prev),
                 kf<const float*>(a, r, F_D0 + prev),
                 a.c_prev >= 0 ? kf<const int*>(a, r, F_BEST) : nullptr, a.w, kscale(a, r),
                 kf<long long*>(a, r, F_POS), a.X, a.ldx, a.d, kf<float*>(a, r, F_CANDS),
                 kf<long long*>(a, r, F_CANDIDS), a.row_offset, a.n_global);
}
__global__ void __launch_bounds__(1024) kmpp_finish_batch_kernel(KppArgs a) {
  const int r = blockIdx.x;
  const double* dr = kf<const double*>(a, r, F_DRAWS);
  kmpp_finish_body(kf<const double*>(a, r, F_DELTA), a.G, a.t, kf<double*>(a, r, F_BTOT),
                   kf<double*>(a, r, F_P), a.doff >= 0 ? dr + a.doff : nullptr,
                   kf<double*>(a, r, F_VALS), kf<const float*>(a, r, F_CANDS),
                   kf<const long long*>(a, r, F_CANDIDS), a.d, kf<float*>(a, r, F_CENTERS),
                   kf<long long*>(a, r, F_IDS), a.c, kf<int*>(a, r, F_BEST));
}

// ---------------------------------------------- fused restart passes
// The per-restart bound pass reads every survivor's int8 row once per
// restart: NR x ~50 % of X per centre step, and the restarts' workgroups of
// one row block do not meet in L2 (measured: 0.487 -> 0.451 s per restart
// only).  The fused passes read a row ONCE per step for all restarts:
//  7. screen: one workgroup per row block walks its rows for every restart
//     (the lazy winner update and the triangle test of kmpp_screen_body,
//     unchanged) and lists the rows live in ANY restart, with the bit mask
//     of the restarts they are live in;
//  8. bound: the listed rows' int8 copies meet every restart's trials in one
//     MFMA sweep - the nr x t trial columns side by side (tp = t rounded up
//     to a power of two columns per restart, so a 16-column MFMA block holds
//     whole restarts) - and each (row, restart) pair live in the mask takes
//     the certified test of kmpp_bound_body; undecided rows go to that
//     restart's exact segment.  The same rows reach each restart's exact
//     pass as in the per-restart passes (set equality; the exact pass's
//     block sums are order-free), so the ids are unchanged.
SQ_DEV int seg_append_pos(bool take, int value, int* __restrict__ seg, int* lcnt) {
  const unsigned long long b = __ballot(take);
  if (b == 0ull) return -1;
  const int lane = threadIdx.x & 63;
  int base = 0;
  if (lane == 0) base = atomicAdd(lcnt, (int)__popcll(b));
  base = __shfl(base, 0, 64);
  if (!take) return -1;
  const int p = base + (int)__popcll(b & ((1ull << lane) - 1ull));
  seg[p] = value;
  return p;
}

// The restarts' pointers, staged once per workgroup in LDS and moved to
// SGPRs at each use (reading them from the pointer table in the row loop
// re-loads them after every global store - the compiler cannot rule out
// that a store aliases the table - and a lane-varying table read puts a
// dependent load in front of every row access).
template <typename P_>
SQ_DEV P_ uni_ptr(unsigned long long v) {
  const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)v);
  const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(v >> 32));
  return reinterpret_cast<P_>(((unsigned long long)hi << 32) | lo);
}
enum ScrPtr { S_CL = 0, S_NEAR, S_MPREV, S_DPREV, S_MCUR, S_CC, S_BP, S_NP };

__global__ void __launch_bounds__(256) kmpp_screen_fused_kernel(KppArgs a) {
  __shared__ int lcnt;
  __shared__ unsigned long long sp[16][S_NP];
  const int blk = blockIdx.x;
  const int prev = 1 - a.cur;
  const long long r0 = (long long)blk * a.R;
  const long long r1 = r0 + a.R < a.n ? r0 + a.R : a.n;
  if (threadIdx.x == 0) lcnt = 0;
  if (threadIdx.x < a.nr) {
    const int r = threadIdx.x;
    sp[r][S_CL] = (unsigned long long)a.tab[(size_t)r * kKppNF + F_CLOSEST];
    sp[r][S_NEAR] = (unsigned long long)a.tab[(size_t)r * kKppNF + F_NEAREST];
    sp[r][S_MPREV] = (unsigned long long)a.tab[(size_t)r * kKppNF + F_MASK0 + prev];
    sp[r][S_DPREV] = (unsigned long long)a.tab[(size_t)r * kKppNF + F_D0 + prev];
    sp[r][S_MCUR] = (unsigned long long)a.tab[(size_t)r * kKppNF + F_MASK0 + a.cur];
    sp[r][S_CC] = (unsigned long long)a.tab[(size_t)r * kKppNF + F_CC];
    sp[r][S_BP] = (unsigned long long)(long long)(a.c_prev >= 0 ? *kf<const int*>(a, r, F_BEST) : -1);
  }
  __syncthreads();
  for (long long i0 = r0; i0 < r1; i0 += 256) {
    const long long i = i0 + threadIdx.x;
    unsigned bits = 0;
    if (i < r1) {
      // four restarts at a time: their loads first (no store in between:
      // all in flight), then the lazy winner's rows, the stores and the
      // triangle tests
      for (int r4 = 0; r4 < a.nr; r4 += 4) {
        float cl[4];
        int c[4];
        unsigned mp[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int r = r4 + u;
          if (r < a.nr) {
            const int bp = (int)(long long)sp[r][S_BP];
            cl[u] = uni_ptr<const float*>(sp[r][S_CL])[i];
            c[u] = uni_ptr<const int*>(sp[r][S_NEAR])[i];
            mp[u] = bp >= 0 ? uni_ptr<const uint16_t*>(sp[r][S_MPREV])[i] : 0u;
          }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int r = r4 + u;
          if (r < a.nr) {
            const int bp = (int)(long long)sp[r][S_BP];
            if (bp >= 0 && ((mp[u] >> bp) & 1u)) {
              cl[u] = uni_ptr<const float*>(sp[r][S_DPREV])[(size_t)bp * a.n + i];
              c[u] = a.c_prev;
              uni_ptr<float*>(sp[r][S_CL])[i] = cl[u];
              uni_ptr<int*>(sp[r][S_NEAR])[i] = c[u];
            }
            uni_ptr<uint16_t*>(sp[r][S_MCUR])[i] = 0;
            if (cl[u] > 0.0f && !(uni_ptr<const float*>(sp[r][S_CC])[c[u]] > 4.01f * cl[u]))
              bits |= 1u << r;
          }
        }
      }
    }
    const int p = seg_append_pos(bits != 0u, (int)i, a.useg + r0, &lcnt);
    if (p >= 0) a.umask[r0 + p] = (uint16_t)bits;
  }
  __syncthreads();
  if (threadIdx.x == 0) a.ucount[blk] = lcnt;
}

// kScol: trial columns (nr x tp <= 128); LDS: the two-term int8 trials
// [2][kScol][dq] and per column (s_c, ec, |c~|^2)
constexpr int kScol = 128;
// Exact pass, batched restarts (op 9): one lane per (row, trial) instead of
// one lane per row - the per-block exact lists are short (~1-5 % of a
// block's rows), so a lane per row left most of each wave idle and each
// trial's candidate features came through the scalar cache, which the
// restarts' different candidates thrash.  Here the block's candidates sit in
// LDS ([t][d + 4] fp32, padded rows: conflict-free 16-B reads), RW = 256 / tp
// rows at a time are staged ([RW][d + 4]; the next RW rows' loads in flight
// during the current FMAs), and lane (row slot s, trial j) runs the SAME
// sequential fmaf chain over f = 0 .. d - 1 as kmpp_exact_body - identical
// D, masks and improvement sums.  d <= 256.
constexpr int kExRowsMax = 32;
__global__ void __launch_bounds__(256) kmpp_exact2_batch_kernel(KppArgs a) {
  int blk, r;
  if (!kpp_decode(blockIdx.x, a.nr, a.G, blk, r)) return;
  extern __shared__ __attribute__((aligned(16))) float exs[];
  __shared__ double dred[4][16];
  const int d = a.d, ds = a.d + 4, t = a.t, tp = a.tp;
  const int RW = 256 / tp < kExRowsMax ? 256 / tp : kExRowsMax;
  float* cs = exs;                    // [t][ds]
  float* xs = exs + (size_t)t * ds;   // [RW][ds]
  const float* cand = kf<const float*>(a, r, F_CANDS);
  const float* closest = kf<const float*>(a, r, F_CLOSEST);
  uint16_t* mask_out = kf<uint16_t*>(a, r, F_MASK0 + a.cur);
  float* Dout = kf<float*>(a, r, F_D0 + a.cur);
  const double scale = kscale(a, r);
  const int cnt = kf<const int*>(a, r, F_ECOUNT)[blk];
  const int* eseg = kf<const int*>(a, r, F_EXACT) + (long long)blk * a.R;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int d4 = d >> 2;
  for (int e = tid; e < t * d4; e += 256) {
    const int j = e / d4, f4 = e % d4;
    *reinterpret_cast<float4*>(cs + (size_t)j * ds + 4 * f4) =
        *reinterpret_cast<const float4*>(cand + (size_t)j * d + 4 * f4);
  }
  const int rs = tid / tp, j = tid % tp;
  double dsum = 0.0;
  // row staging: RW d4 float4 per chunk, kExRowsMax * 64 / 256 = 8 per thread at most
  constexpr int kPer = kExRowsMax * 64 / 256;
  float4 v[kPer];
  auto fetch = [&](int c0) {
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int e = tid + 256 * i;
      v[i] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (e < RW * d4) {
        const int s = e / d4, f4 = e % d4;
        const int p = c0 + s;
        if (p < cnt) v[i] = *reinterpret_cast<const float4*>(a.X + (size_t)eseg[p] * a.ldx + 4 * f4);
      }
    }
  };
  fetch(0);
  for (int c0 = 0; c0 < cnt; c0 += RW) {
    __syncthreads();   // the previous chunk's reads of xs are done (and cs staged)
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int e = tid + 256 * i;
      if (e < RW * d4) *reinterpret_cast<float4*>(xs + (size_t)(e / d4) * ds + 4 * (e % d4)) = v[i];
    }
    __syncthreads();
    if (c0 + RW < cnt) fetch(c0 + RW);
    const int p = rs < RW ? c0 + rs : cnt;
    const bool live = p < cnt && j < t;
    float acc = 0.0f;
    if (live) {
      const float* xr = xs + (size_t)rs * ds;
      const float* cr = cs + (size_t)j * ds;
      for (int f = 0; f < d; f += 4) {
        const float4 x4 = *reinterpret_cast<const float4*>(xr + f);
        const float4 c4 = *reinterpret_cast<const float4*>(cr + f);
        float ev = x4.x - c4.x;
        acc = fmaf(ev, ev, acc);
        ev = x4.y - c4.y;
        acc = fmaf(ev, ev, acc);
        ev = x4.z - c4.z;
        acc = fmaf(ev, ev, acc);
        ev = x4.w - c4.w;
        acc = fmaf(ev, ev, acc);
      }
    }
    const int row = p < cnt ? eseg[p] : 0;
    uint32_t m = 0;
    if (live) {
      const float cl = closest[row];
      if (acc < cl) {
        const double wi = a.w ? a.w[row] : 1.0;
        m = 1u << j;
        Dout[(size_t)j * a.n + row] = acc;
        dsum += kpp_q(cl, wi, scale) - kpp_q(acc, wi, scale);
      }
    }
    // the row's mask over its tp lanes
    for (int o = 1; o < tp; o <<= 1) m |= (uint32_t)__shfl_xor((int)m, o, 64);
    if (j == 0 && p < cnt) mask_out[row] = (uint16_t)m;
  }
  // improvement sums per trial (exact integers: any order)
  for (int o = tp; o < 64; o <<= 1) dsum += __shfl_xor(dsum, o, 64);
  if (lane < tp) dred[wave][lane] = dsum;
  __syncthreads();
  if (tid < t) {
    double* dp = kf<double*>(a, r, F_DELTA);
    dp[(long long)blk * t + tid] = (dred[0][tid] + dred[1][tid]) + (dred[2][tid] + dred[3][tid]);
  }
}

// Exact pass over (row, trial) PAIRS (op 10, after the fused bound): the
// bound leaves ~1-2 of a listed row's t trials undecided, and records them
// (the entry's trial mask, in the restart's surv segment); the lane-per-
// (row, trial) pass above computed all t.  Here each wave expands 64 list
// entries into their undecided pairs (wave scan of the mask popcounts) and
// runs one lane per pair: the row straight from global memory (float4, a
// few loads ahead), the trial's features from LDS, the same sequential
// fmaf chain - identical D for every pair it computes; a decided trial
// provably does not improve its row, so the masks, D and block sums equal
// the full pass's (mask bits set by 32-bit atomicOr: the screen cleared
// every row's mask; the per-trial sums by LDS fp64 atomics of exact
// fixed-point integers).
template <int U>
__global__ void __launch_bounds__(256) kmpp_exact3_batch_kernel(KppArgs a) {
  int blk, r;
  if (!kpp_decode(blockIdx.x, a.nr, a.G, blk, r)) return;
  extern __shared__ __attribute__((aligned(16))) float exs3[];
  __shared__ double dsum[16];
  __shared__ int srow[4][64];
  __shared__ uint16_t spair[4][64 * 16];
  const int d = a.d, ds = a.d + 4, t = a.t;
  float* cs = exs3;                    // [t][ds]
  const float* cand = kf<const float*>(a, r, F_CANDS);
  const float* closest = kf<const float*>(a, r, F_CLOSEST);
  uint16_t* mask_out = kf<uint16_t*>(a, r, F_MASK0 + a.cur);
  float* Dout = kf<float*>(a, r, F_D0 + a.cur);
  const double scale = kscale(a, r);
  const int cnt = kf<const int*>(a, r, F_ECOUNT)[blk];
  const int* eseg = kf<const int*>(a, r, F_EXACT) + (long long)blk * a.R;
  const int* mseg = kf<const int*>(a, r, F_SURV) + (long long)blk * a.R;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int d4 = d >> 2;
  for (int e = tid; e < t * d4; e += 256) {
    const int j = e / d4, f4 = e % d4;
    *reinterpret_cast<float4*>(cs + (size_t)j * ds + 4 * f4) =
        *reinterpret_cast<const float4*>(cand + (size_t)j * d + 4 * f4);
  }
  if (tid < 16) dsum[tid] = 0.0;
  __syncthreads();
  for (int e0 = wave * 64; e0 < cnt; e0 += 256) {
    const int e = e0 + lane;
    const int row = e < cnt ? eseg[e] : -1;
    const unsigned m = e < cnt ? (unsigned)mseg[e] & ((1u << t) - 1u) : 0u;
    const int np = __popc(m);
    int incl = np;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int v = __shfl_up(incl, o, 64);
      if (lane >= o) incl += v;
    }
    const int tot = __shfl(incl, 63, 64);
    srow[wave][lane] = row;
    {
      int w = incl - np;
      unsigned mm = m;
      while (mm) {
        const int j = __builtin_ctz(mm);
        mm &= mm - 1u;
        spair[wave][w++] = (uint16_t)((lane << 4) | j);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (int b = 0; b < tot; b += 64) {
      const bool live = b + lane < tot;
      const uint16_t pr = live ? spair[wave][b + lane] : (uint16_t)0;
      const int rr = srow[wave][pr >> 4];
      const int j = pr & 15;
      float acc = 0.0f;
      if (live) {
        const float* xr = a.X + (size_t)rr * a.ldx;
        const float* cr = cs + (size_t)j * ds;
        // (U: float4 row loads in flight)
        for (int f0 = 0; f0 < d; f0 += 4 * U) {
          float4 xv[U];
#pragma unroll
          for (int u = 0; u < U; ++u)
            xv[u] = f0 + 4 * u < d ? *reinterpret_cast<const float4*>(xr + f0 + 4 * u)
                                   : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
          for (int u = 0; u < U; ++u) {
            if (f0 + 4 * u < d) {
              const float4 c4 = *reinterpret_cast<const float4*>(cr + f0 + 4 * u);
              float ev = xv[u].x - c4.x;
              acc = fmaf(ev, ev, acc);
              ev = xv[u].y - c4.y;
              acc = fmaf(ev, ev, acc);
              ev = xv[u].z - c4.z;
              acc = fmaf(ev, ev, acc);
              ev = xv[u].w - c4.w;
              acc = fmaf(ev, ev, acc);
            }
          }
        }
        const float cl = closest[rr];
        if (acc < cl) {
          const double wi = a.w ? a.w[rr] : 1.0;
          Dout[(size_t)j * a.n + rr] = acc;
          atomicOr(reinterpret_cast<unsigned int*>(mask_out + (rr & ~1)), (1u << j) << (16 * (rr & 1)));
          atomicAdd(&dsum[j], kpp_q(cl, wi, scale) - kpp_q(acc, wi, scale));
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
  __syncthreads();
  if (tid < t) kf<double*>(a, r, F_DELTA)[(long long)blk * t + tid] = dsum[tid];
}

constexpr int kBfThreads = 512;   // 8 waves share one staging of the trials
template <int NS>
__global__ void __launch_bounds__(kBfThreads) kmpp_bound_fused_kernel(KppArgs a) {
  constexpr int DQ = NS * 64;
  constexpr int NWV = kBfThreads / 64;
  // dynamic LDS: [2][ncb 16][CS] int8 (sized to the columns in use:
  // occupancy).  A ds_read_b128 lane group reads 8 columns at one offset,
  // which a DQ (multiple of 256 B) stride put on one bank slot - 8-way
  // conflicts, ~10 LDS cycles per read in the PMC.  NS = 4 (16 pieces per
  // column): piece p of column c is stored at p ^ (c & 15), so the group's
  // two 8-lane halves (kb 0 / 1, complementary c16 sets) hit 16 distinct
  // slots; other NS: a 16-B pad per column
  constexpr int CS = NS == 4 ? DQ : DQ + 16;
  auto swz = [](int p, int c) { return NS == 4 ? (p ^ (c & 15)) : p; };
  extern __shared__ __attribute__((aligned(16))) int8_t cbs[];
  __shared__ float cpar[kScol][3];
  __shared__ int lcnt[16];
  __shared__ float sclo[NWV * 16 * 17];   // row stride 17: no ds_write_b32 bank aliasing
  __shared__ unsigned long long spc[16], spe[16], sps[16];   // closest / exact / surv
  const int blk = blockIdx.x;
  const int tp = a.tp, t = a.t, nr = a.nr;
  if (threadIdx.x < nr) {
    spc[threadIdx.x] = (unsigned long long)a.tab[(size_t)threadIdx.x * kKppNF + F_CLOSEST];
    spe[threadIdx.x] = (unsigned long long)a.tab[(size_t)threadIdx.x * kKppNF + F_EXACT];
    sps[threadIdx.x] = (unsigned long long)a.tab[(size_t)threadIdx.x * kKppNF + F_SURV];
  }
  const int ncol = nr * tp, ncb = (ncol + 15) / 16;
  auto cb = [&](int hl, int col) -> int8_t* { return cbs + ((size_t)hl * ncb * 16 + col) * CS; };
  // stage every restart's trials: column c = r tp + j (j >= t: zero)
  for (int e = threadIdx.x; e < 2 * ncb * 16 * (DQ / 16); e += kBfThreads) {
    const int hl = e / (ncb * 16 * (DQ / 16));
    const int rem = e % (ncb * 16 * (DQ / 16));
    const int col = rem / (DQ / 16), piece = rem % (DQ / 16);
    const int r = col / tp, j = col % tp;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (r < nr && j < t)
      v = *reinterpret_cast<const uint4*>(kf<const int8_t*>(a, r, F_CANDQ) +
                                          ((size_t)(hl * 16 + j) * a.dq + piece * 16));
    *reinterpret_cast<uint4*>(cb(hl, col) + swz(piece, col) * 16) = v;
  }
  for (int col = threadIdx.x; col < ncb * 16; col += kBfThreads) {
    const int r = col / tp, j = col % tp;
    const bool jv = r < nr && j < t;
    const double* ci = jv ? kf<const double*>(a, r, F_CINFO) + j * 4 : nullptr;
    // scale and error norm rounded UP to fp32, |c~|^2 to nearest (kmpp_bound_body)
    cpar[col][0] = jv ? (float)ci[0] * (1.0f + 1.2e-7f) : 1.0f;
    cpar[col][1] = jv ? (float)ci[1] * (1.0f + 1.2e-7f) : 0.0f;
    cpar[col][2] = jv ? (float)ci[2] : 0.0f;
  }
  if (threadIdx.x < 16) lcnt[threadIdx.x] = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c16 = lane & 15, kb = lane >> 4;
  const long long r0 = (long long)blk * a.R;
  const int cnt = a.ucount[blk];
  const int* useg = a.useg + r0;
  const uint16_t* umask = a.umask + r0;
  const float lim_rel = 1.0f + 3.0f * (float)(a.d + 2) * 5.9604645e-08f + 1e-6f;
  const int rpb = 16 / tp;   // restarts per 16-column block
  // one group ahead in registers: the group's row ids / masks, int8 rows,
  // per-row scalars and the rows' closest values of the restarts they are
  // live in (lane (kb, c16): restarts kb, kb + 4, kb + 8, kb + 12 of row
  // slot c16); the current group's closest values go through LDS
  float* scl = sclo + wave * 16 * 17;   // [16 row slots][16 restarts (+1 pad)]
  int nrow = -1;
  unsigned nbits = 0u;
  kpp_v4i nav[NS];
  float nrs = 0.f, nre = 0.f, ncl[4];
  int nq2 = 0;
  // the list entries (row id, restart mask) run one group further ahead:
  // the row loads of group g + 1 need them, and waiting for them right
  // before issuing those loads exposed a full memory latency per group
  int irow = -1;
  unsigned ibits = 0u;
  auto load_ids = [&](int g) {
    const int e = g + c16;
    irow = e < cnt ? useg[e] : -1;
    ibits = e < cnt ? umask[e] : 0u;
  };
  auto prefetch = [&]() {
    nrow = irow;
    nbits = ibits;
    const int rr0 = nrow >= 0 ? nrow : 0;
    const int8_t* xr = a.Xq + (size_t)rr0 * a.dq + 16 * kb;
#pragma unroll
    for (int s4 = 0; s4 < NS; ++s4)
      nav[s4] = nrow >= 0 ? *reinterpret_cast<const kpp_v4i*>(xr + 64 * s4) : kpp_v4i{0, 0, 0, 0};
    nrs = a.srow[rr0];
    nre = a.erow[rr0];
    nq2 = a.q2row[rr0];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int rr = kb + 4 * u;
      ncl[u] = (nrow >= 0 && rr < nr && ((nbits >> rr) & 1u))
                   ? reinterpret_cast<const float*>(spc[rr])[nrow] : 0.0f;
    }
  };
  load_ids(wave * 16);
  prefetch();
  load_ids(wave * 16 + 16 * NWV);
  for (int g0 = wave * 16; g0 < cnt; g0 += 16 * NWV) {
    const int row = nrow;
    const unsigned bits = nbits;
    kpp_v4i av[NS];
#pragma unroll
    for (int s4 = 0; s4 < NS; ++s4) av[s4] = nav[s4];
    const float rs = nrs, re_ = nre;
    const int rq2 = nq2;
#pragma unroll
    for (int u = 0; u < 4; ++u) scl[c16 * 17 + kb + 4 * u] = ncl[u];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    prefetch();
    load_ids(g0 + 32 * NWV);
    // restarts live in any row of the group
    unsigned gbits = row >= 0 ? bits : 0u;
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) gbits |= (unsigned)__shfl_xor((int)gbits, o, 64);
    gbits = (unsigned)__builtin_amdgcn_readfirstlane((int)gbits);
    // the row of each result register (row slot 4 kb + i) and its scalars,
    // the same for every column block
    int rrv[4];
    unsigned rbv[4];
    float sv[4], erv[4], Av[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int src = 4 * kb + i;
      rrv[i] = __shfl(row, src, 64);
      rbv[i] = (unsigned)__shfl((int)bits, src, 64);
      sv[i] = __shfl(rs, src, 64);
      erv[i] = __shfl(re_, src, 64);
      const float q2 = (float)__shfl(rq2, src, 64);
      Av[i] = sv[i] * sv[i] * q2;
    }
    for (int cbk = 0; cbk < ncb; ++cbk) {
      const unsigned bm = ((1u << rpb) - 1u) << (cbk * rpb);
      if (!(gbits & bm)) continue;
      kpp_v4i hi = kpp_v4i{0, 0, 0, 0}, lo = kpp_v4i{0, 0, 0, 0};
#pragma unroll
      for (int s4 = 0; s4 < NS; ++s4) {
        const int pc = swz(4 * s4 + kb, c16) * 16;
        const kpp_v4i bh = *reinterpret_cast<const kpp_v4i*>(cb(0, cbk * 16 + c16) + pc);
        const kpp_v4i bl = *reinterpret_cast<const kpp_v4i*>(cb(1, cbk * 16 + c16) + pc);
        hi = __builtin_amdgcn_mfma_i32_16x16x64_i8(av[s4], bh, hi, 0, 0, 0);
        lo = __builtin_amdgcn_mfma_i32_16x16x64_i8(av[s4], bl, lo, 0, 0, 0);
      }
      const int col = cbk * 16 + c16;
      const int r = col / tp, j = col % tp;
      const bool jv = r < nr && j < t;
      const float sc = cpar[col][0], ec = cpar[col][1], cc2 = cpar[col][2];
      unsigned long long bal[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int src = 4 * kb + i;   // the row slot of result register i
        const int rr = rrv[i];
        const float s = sv[i], er = erv[i], A = Av[i];
        bool need = false;
        if (jv && rr >= 0 && ((rbv[i] >> r) & 1u)) {
          const float cl = scl[src * 17 + r];
          const float dot = s * sc * ((float)hi[i] + (float)lo[i] * (1.0f / 254.0f));
          const float Dq = (A + cc2) - 2.0f * dot;
          const float Dlb = Dq - 1e-6f * (A + cc2 + 2.0f * fabsf(dot));
          float lb = 0.0f;
          if (Dlb > 0.0f) {
            const float rt = __builtin_amdgcn_sqrtf(Dlb) * (1.0f - 1e-6f) - er - ec;
            lb = rt > 0.0f ? rt * rt * (1.0f - 1e-6f) : 0.0f;
          }
          need = !(lb > cl * lim_rel);
        }
        bal[i] = __ballot(need);
      }
      // row slot c16 (lanes < 16): rows 4 q + i live in lanes [16 q, 16 q + 16) of bal[i];
      // restart p of this block: lanes [p tp, p tp + tp) of that 16-lane group
      const int q = c16 >> 2, ii = c16 & 3;
      const unsigned long long bi = ii == 0 ? bal[0] : ii == 1 ? bal[1] : ii == 2 ? bal[2] : bal[3];
      const unsigned tmask = tp >= 16 ? 0xFFFFu : ((1u << tp) - 1u);
      for (int p = 0; p < rpb; ++p) {
        const int rp = cbk * rpb + p;
        if (rp >= nr) break;
        const unsigned tm = ((unsigned)(bi >> (16 * q + p * tp))) & tmask;
        const bool take = lane < 16 && row >= 0 && tm != 0u;
        const int pos = seg_append_pos(take, row, uni_ptr<int*>(spe[rp]) + r0, &lcnt[rp]);
        // the undecided trials of the entry (the surv segments are free in
        // the fused passes): op 10 computes only those
        if (pos >= 0) uni_ptr<int*>(sps[rp])[r0 + pos] = (int)tm;
      }
    }
  }
  __syncthreads();
  if (threadIdx.x < nr) kf<int*>(a, threadIdx.x, F_ECOUNT)[blk] = lcnt[threadIdx.x];
}

}  // namespace sq

using namespace sq;

extern "C" {

static int kpp_grid(long long n) {
  const long long b = (n + 255) / 256;
  return (int)(b < 2048 ? (b > 0 ? b : 1) : 2048);
}

// closest fp32 [n], nearest int32 [n], bmax fp64 [sq_kmpp_grid(-1) = kKppInitGrid] for
// sq_kmpp_init; sq_kmpp_grid(n >= 0): the workgroups of the per-block passes
int sq_kmpp_grid(long long n) { return n < 0 ? kKppInitGrid : kpp_grid(n); }

// Xq (nullable) int8 [n][dq] (dq = d rounded up to 64), srow / erow fp32 [n], q2row int32 [n]
int sq_kmpp_init(const void* X, long long ldx, int d, long long n, const void* c0, const void* w,
                 void* closest, void* nearest, void* bmax, void* Xq, int dq, void* srow,
                 void* erow, void* q2row, void* stream) {
  if (n <= 0) return 0;
  if (d <= 0 || (d & 3) || ldx < d || (ldx & 3) || (Xq && (dq < d || (dq & 63))))
    return (int)hipErrorInvalidValue;
  // 16 lanes per row: enough waves in flight to cover the row loads' latency
  // (bmax holds kKppInitGrid entries; the caller takes their max)
  const long long gb = (n + 15) / 16;   // 16 rows per workgroup pass
  const int grid = (int)(gb < kKppInitGrid ? gb : kKppInitGrid);
  hipLaunchKernelGGL(kmpp_init_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                     (const float*)X, ldx, d, n, (const float*)c0, (const double*)w,
                     (float*)closest, (int*)nearest, (double*)bmax, (int8_t*)Xq, dq,
                     (float*)srow, (float*)erow, (int*)q2row);
  return (int)hipGetLastError();
}

int sq_kmpp_block_totals(const void* closest, const void* w, long long n, long long R, int G,
                         double scale, void* block_tot, void* stream) {
  if (G <= 0) return 0;
  hipLaunchKernelGGL(kmpp_block_totals_kernel, dim3(G), dim3(256), 0, (hipStream_t)stream,
                     (const float*)closest, (const double*)w, n, R, scale, (double*)block_tot);
  return (int)hipGetLastError();
}

// cc: ccmin fp32 [>= c] (ldcc: its capacity)
int sq_kmpp_cc(const void* cand, const void* C, int c, int d, int t, void* cc, int ldcc,
               void* cinfo, void* candq, int dq, void* delta_part, long long ndp, void* counters,
               void* stream) {
  if (t < 1 || t > 16 || c < 0 || c > ldcc || dq < d || (dq & 63)) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(kmpp_cc_kernel, dim3(t + (c + 3) / 4), dim3(256), 0, (hipStream_t)stream,
                     (const float*)cand, (const float*)C, c, d, t, (float*)cc, (double*)cinfo,
                     (int8_t*)candq, dq, (double*)delta_part, ndp, (int*)counters);
  return (int)hipGetLastError();
}

// G blocks of R rows (G R >= n); scount / ecount int [G]
int sq_kmpp_screen(void* closest, void* nearest, const void* mask_prev, const void* Dprev,
                   const void* best_prev, int c_prev, const void* cc, int ldcc, int t, long long n,
                   long long R, int G, void* mask_out, void* surv, void* exact, void* scount,
                   void* ecount, int prune, void* stream) {
  if (n <= 0) return 0;
  if (t < 1 || t > 16 || R <= 0 || G <= 0 || (long long)G * R < n) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(kmpp_screen_kernel, dim3(G), dim3(256), 0, (hipStream_t)stream,
                     (float*)closest, (int*)nearest, (const uint16_t*)mask_prev,
                     (const float*)Dprev, (const int*)best_prev, c_prev, (const float*)cc, n,
                     R, (uint16_t*)mask_out, (int*)surv, (int*)exact, (int*)scount,
                     (int*)ecount, prune);
  return (int)hipGetLastError();
}

// candq int8 [2][16][dq] (trial slots >= t zero), cinfo fp64 [t][4]
int sq_kmpp_bound(const void* Xq, int dq, const void* srow, const void* erow, const void* xq2,
                  const void* closest, const void* candq, const void* cinfo, int t, int d,
                  long long n, long long R, int G, const void* surv, const void* scount,
                  void* exact, void* ecount, void* stream) {
  if (n <= 0) return 0;
  if (t < 1 || t > 16 || (dq & 63) || dq < d || R <= 0 || G <= 0 || 32 * dq > 65536)
    return (int)hipErrorInvalidValue;
#define LAUNCH(NS)                                                                              \
  hipLaunchKernelGGL(kmpp_bound_kernel<NS>, dim3(G), dim3(256), (size_t)32 * dq,                \
                     (hipStream_t)stream, (const int8_t*)Xq, dq, (const float*)srow,            \
                     (const float*)erow, (const int*)xq2, (const float*)closest,                \
                     (const int8_t*)candq, (const double*)cinfo, t, d, R, (const int*)surv,     \
                     (const int*)scount, (int*)exact, (int*)ecount)
  switch (dq / 64) {
    case 1: LAUNCH(1); break;
    case 2: LAUNCH(2); break;
    case 3: LAUNCH(3); break;
    case 4: LAUNCH(4); break;
    default: LAUNCH(0); break;
  }
#undef LAUNCH
  return (int)hipGetLastError();
}

int sq_kmpp_dots(const void* Xq, int dq, long long n, const void* candq, void* out, void* stream) {
  if (n <= 0) return 0;
  if ((dq & 63) || 32 * dq > 65536) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(kmpp_dots_kernel, dim3((unsigned)((n + 15) / 16)), dim3(64), (size_t)32 * dq,
                     (hipStream_t)stream, (const int8_t*)Xq, dq, n, (const int8_t*)candq,
                     (int*)out);
  return (int)hipGetLastError();
}

int sq_kmpp_exact(const void* X, long long ldx, int d, long long n, int t, const void* cand,
                  const void* closest, const void* w, double scale, const void* exact,
                  const void* ecount, void* mask_out, void* Dout, void* delta_part, long long R,
                  int G, void* stream) {
  if (n <= 0) return 0;
  if (t < 1 || t > 16 || d <= 0 || (d & 3) || ldx < d || (ldx & 3) || R <= 0 || G <= 0)
    return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
#define LAUNCH(TM)                                                                              \
  hipLaunchKernelGGL(kmpp_exact_kernel<TM>, dim3(G), dim3(256), 0, st, (const float*)X, ldx,    \
                     d, n, t, (const float*)cand, (const float*)closest, (const double*)w,     \
                     scale, (const int*)exact, (const int*)ecount, (uint16_t*)mask_out,        \
                     (float*)Dout, (double*)delta_part, R)
  if (t <= 4) LAUNCH(4);
  else if (t <= 8) LAUNCH(8);
  else LAUNCH(16);
#undef LAUNCH
  return (int)hipGetLastError();
}

// cands (nullable): also copy the picked rows (fp32 [t][d]) and their global ids (int64 [t])
int sq_kmpp_pick(const void* block_tot, int G, long long R, long long n, const void* vals, int t,
                 const void* closest, const void* mask, const void* D, const void* best,
                 const void* w, double scale, void* pos, const void* X, long long ldx, int d,
                 void* cands, void* cand_ids, long long row_offset, long long n_global,
                 void* stream) {
  if (t < 1 || G < 1 || n <= 0 || (cands && (!X || !cand_ids || d < 1 || ldx < d)))
    return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(kmpp_pick_kernel, dim3(t), dim3(256), 0, (hipStream_t)stream,
                     (const double*)block_tot, G, R, n, (const double*)vals,
                     (const float*)closest, (const uint16_t*)mask, (const float*)D,
                     (const int*)best, (const double*)w, scale, (long long*)pos, (const float*)X,
                     ldx, d, (float*)cands, (long long*)cand_ids, row_offset, n_global);
  return (int)hipGetLastError();
}

int sq_kmpp_finish(const void* delta_part, int G, int t, void* block_tot, void* P,
                   const void* draws_next, void* vals, const void* cands, const void* cand_ids,
                   int d, void* centers, void* ids, int c, void* best_out, void* stream) {
  if (t < 1 || t > 16 || G < 1 || d < 1 || c < 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(kmpp_finish_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream,
                     (const double*)delta_part, G, t, (double*)block_tot, (double*)P,
                     (const double*)draws_next, (double*)vals, (const float*)cands,
                     (const long long*)cand_ids, d, (float*)centers, (long long*)ids, c,
                     (int*)best_out);
  return (int)hipGetLastError();
}

// Batched restarts: op 1 cc, 2 screen, 3 bound, 4 exact, 5 pick, 6 finish.
// ia: [0] table (device int64 [nr][32]), [1] nr, [2] X, [3] ldx, [4] d,
// [5] n, [6] t, [7] k, [8] dq, [9] Xq, [10] srow, [11] erow, [12] q2row,
// [13] w, [14] R, [15] G, [16] c (centre being chosen), [17] c_prev (the
// lazily applied winner's centre, -1: none), [18] cur (mask / D pair this
// step writes), [19] prune, [20] row_offset, [21] n_global, [22] draws
// offset of the next centre (elements, -1: last centre), [23] delta_part
// entries per restart; ops 7 (fused screen) / 8 (fused bound): [24] useg
// (int32 [G R]), [25] umask (uint16 [G R]), [26] ucount (int32 [G]), [27] tp.
int sq_kmpp_batch(int op, const long long* ia, void* stream) {
  KppArgs a;
  a.tab = (const long long*)ia[0];
  a.nr = (int)ia[1];
  a.X = (const float*)ia[2];
  a.ldx = ia[3];
  a.d = (int)ia[4];
  a.n = ia[5];
  a.t = (int)ia[6];
  a.k = (int)ia[7];
  a.dq = (int)ia[8];
  a.Xq = (const int8_t*)ia[9];
  a.srow = (const float*)ia[10];
  a.erow = (const float*)ia[11];
  a.q2row = (const int*)ia[12];
  a.w = (const double*)ia[13];
  a.R = ia[14];
  a.G = (int)ia[15];
  a.c = (int)ia[16];
  a.c_prev = (int)ia[17];
  a.cur = (int)ia[18];
  a.prune = (int)ia[19];
  a.row_offset = ia[20];
  a.n_global = ia[21];
  a.doff = ia[22];
  a.ndp = ia[23];
  a.per = 1;
  a.useg = (int*)ia[24];
  a.umask = (uint16_t*)ia[25];
  a.ucount = (int*)ia[26];
  a.tp = (int)ia[27];
  hipStream_t st = (hipStream_t)stream;
  if (!a.tab || a.nr < 1 || a.nr > 64 || a.t < 1 || a.t > 16 || a.n <= 0 || a.d < 1 ||
      (a.d & 3) || a.ldx < a.d || (a.ldx & 3) || a.R <= 0 || a.G <= 0 ||
      (long long)a.G * a.R < a.n || (a.cur & ~1))
    return (int)hipErrorInvalidValue;
  const unsigned rows_grid = (unsigned)((long long)((a.G + 7) / 8) * 8 * a.nr);
  switch (op) {
    case 1: {
      if (a.c < 0 || a.c > a.k || a.dq < a.d || (a.dq & 63)) return (int)hipErrorInvalidValue;
      a.per = a.t + (a.c + 3) / 4;
      hipLaunchKernelGGL(kmpp_cc_batch_kernel, dim3((unsigned)(a.per * a.nr)), dim3(256), 0, st, a);
      break;
    }
    case 2:
      hipLaunchKernelGGL(kmpp_screen_batch_kernel, dim3(rows_grid), dim3(256), 0, st, a);
      break;
    case 3: {
      if (!a.Xq || (a.dq & 63) || a.dq < a.d || 32 * a.dq > 65536) return (int)hipErrorInvalidValue;
#define LAUNCH(NS)                                                                              \
  hipLaunchKernelGGL(kmpp_bound_batch_kernel<NS>, dim3(rows_grid), dim3(256), (size_t)32 * a.dq, st, a)
      switch (a.dq / 64) {
        case 1: LAUNCH(1); break;
        case 2: LAUNCH(2); break;
        case 3: LAUNCH(3); break;
        case 4: LAUNCH(4); break;
        default: LAUNCH(0); break;
      }
#undef LAUNCH
      break;
    }
    case 4:
      if (a.t <= 4) hipLaunchKernelGGL(kmpp_exact_batch_kernel<4>, dim3(rows_grid), dim3(256), 0, st, a);
      else if (a.t <= 8) hipLaunchKernelGGL(kmpp_exact_batch_kernel<8>, dim3(rows_grid), dim3(256), 0, st, a);
      else hipLaunchKernelGGL(kmpp_exact_batch_kernel<16>, dim3(rows_grid), dim3(256), 0, st, a);
      break;
    case 5:
      hipLaunchKernelGGL(kmpp_pick_batch_kernel, dim3((unsigned)(a.t * a.nr)), dim3(256), 0, st, a);
      break;
    case 6:
      if (a.c < 0) return (int)hipErrorInvalidValue;
      hipLaunchKernelGGL(kmpp_finish_batch_kernel, dim3((unsigned)a.nr), dim3(1024), 0, st, a);
      break;
    case 10: {
      // exact pass over the fused bound's undecided pairs: d <= 256
      if (a.d > 256 || !a.prune) return (int)hipErrorInvalidValue;
      const size_t lds = (size_t)a.t * (a.d + 4) * sizeof(float);
      // 16 float4 row loads in flight per lane (10M x 256, k = 1024, 10
      // restarts: 4 / 8 / 16 -> 0.229 / 0.221 / 0.218 s per restart)
      hipLaunchKernelGGL(kmpp_exact3_batch_kernel<16>, dim3(rows_grid), dim3(256), lds, st, a);
      break;
    }
    case 9: {
      // exact pass, lane per (row, trial): d <= 256, tp a power of two >= t
      if (a.d > 256 || a.tp < a.t || a.tp > 16 || (a.tp & (a.tp - 1))) return (int)hipErrorInvalidValue;
      const int RW = 256 / a.tp < kExRowsMax ? 256 / a.tp : kExRowsMax;
      const size_t lds = (size_t)(a.t + RW) * (a.d + 4) * sizeof(float);
      hipLaunchKernelGGL(kmpp_exact2_batch_kernel, dim3(rows_grid), dim3(256), lds, st, a);
      break;
    }
    case 7:
    case 8: {
      // fused passes: <= 16 restarts (uint16 masks), nr tp <= kScol columns, dq <= 256
      if (!a.useg || !a.umask || !a.ucount || a.nr > 16 || a.tp < a.t || a.tp > 16 ||
          (a.tp & (a.tp - 1)) || a.nr * a.tp > kScol || !a.prune)
        return (int)hipErrorInvalidValue;
      if (op == 7) {
        hipLaunchKernelGGL(kmpp_screen_fused_kernel, dim3((unsigned)a.G), dim3(256), 0, st, a);
        break;
      }
      if (!a.Xq || (a.dq & 63) || a.dq < a.d || a.dq > 256) return (int)hipErrorInvalidValue;
      const size_t lds = (size_t)2 * ((a.nr * a.tp + 15) / 16) * 16 * (a.dq == 256 ? 256 : a.dq + 16);
      // (the padded columns can pass 64 KiB at kScol columns)
#define LAUNCH(NS)                                                                               \
  do {                                                                                           \
    static bool attr = false;                                                                    \
    if (!attr) {                                                                                 \
      (void)hipFuncSetAttribute((const void*)kmpp_bound_fused_kernel<NS>,                        \
                                hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024);        \
      attr = true;                                                                               \
    }                                                                                            \
    hipLaunchKernelGGL(kmpp_bound_fused_kernel<NS>, dim3((unsigned)a.G), dim3(kBfThreads), lds, \
                       st, a);                                                                   \
  } while (0)
      switch (a.dq / 64) {
        case 1: LAUNCH(1); break;
        case 2: LAUNCH(2); break;
        case 3: LAUNCH(3); break;
        default: LAUNCH(4); break;
      }
#undef LAUNCH
      break;
    }
    default:
      return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

}  // extern "C"
