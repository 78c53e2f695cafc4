// fp32-faithful fused q-means E-step on gfx950 (SURVEY.md §2.6 K1/K2,
// reference ``sklearn/cluster/_dmeans.py:736-751``: fp64 ``cdist`` squared,
// then the delta-band {j : D_ij <= min_i + delta}).
//
// Arithmetic.  gfx950 has no xf32 MFMA and the exact fp32 MFMA runs at 1/16
// of the fp16 rate, so the products are formed from an fp16 hi/lo split:
//   x^ = alpha x = xh + xl,   c^ = -2 alpha c = ch + cl      (fp16 each)
//   x^.c^ ~= xh.ch + xh.cl + xl.ch                            (3 MFMA passes)
// alpha is a power of two chosen on the host so that alpha^2 max||x||^2 <=
// 2^13: every fp16 piece is in range, products of fp16 pieces are exact in
// fp32 and the accumulation is fp32 (v_mfma_f32_32x32x16_f16).  The split
// represents each operand to 2^-22 relative (2^-25 absolute for entries far
// below the row scale) and the dropped xl.cl term is 2^-22 relative, i.e. the
// result has the error profile of an fp32 GEMM (error ~ 2^-24 sqrt(K) of the
// partial sums), unlike the bf16 kernel (2^-9 per operand).  The centroid
// norm alpha^2 ||c||^2 rides in an augmented k-step as a 3-way fp16 split
// against the constant A fragment [1, 1, 1, 0 ...], so the accumulator holds
//   D'~ = alpha^2 (||c||^2 - 2 x.c)       (the row-constant ||x||^2 is added
// only to the reported minimum: the band test needs no cancellation with it)
// and the band threshold is compared in the same scaled units (delta alpha^2,
// exact: alpha is a power of two).
//
// Selection.  No index packing: every lane keeps the 3 smallest values of its
// columns (j = lane mod 32 of every tile, 2 per tile) with the indices of the
// two smallest in separate registers (8 VALU per value, hidden under the 6
// MFMAs of each k-step).  After the sweep the 32 lanes sharing a row merge
// their (min, 2nd, argmin) by a transposed reduce-scatter; rows whose 2nd
// value is inside the band are resolved from the per-lane top-2 lists in
// kappa order (band.h); a lane whose 3rd value is inside the band could hide
// a 4th member -> the row goes to the overflow list and is re-done exactly in
// fp64 by the rows kernel (csrc/rows_f64.hip: fp64-MFMA candidates, then
// sum of (x - c)^2 - cdist's own formula).
//
// Layout.  One workgroup = 4 waves (one per SIMD, up to 512 registers) x 32
// rows; each wave keeps its 32 rows as fp16 hi/lo A fragments in VGPRs for the
// whole centroid sweep (X is read from HBM once per iteration, as fp32, and
// split in registers).  Centroid tiles of 64 stream through a 2-deep LDS ring
// by LDS-DMA (global_load_lds, 16 B per lane); a tile is [hi chunks (d/8 + 2,
// incl. the norm chunk)][lo chunks (d/8)] of [64 centroids][8 fp16], so every
// B-fragment read is base + immediate and conflict-free.  Persistent grid; the
// next block's rows are loaded while the merge / band resolution runs and the
// epilogue of tile t runs in the MFMA shadow of tile t+1.
#include "common.h"
#include "band.h"
#include <utility>

namespace sq {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kTileN = 64;          // centroids per LDS tile
constexpr int kMaxCand = 16;        // candidates per multi row (fp64 re-check list)

SQ_DEV float vmin(float a, float b) {
  float r;
  asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
// (bits(a) & m) | q in ONE VALU op (v_and_or_b32; the compiler emits an and
// plus an or3 that it pairs across values)
SQ_DEV float and_or(float a, uint32_t m, uint32_t q) {
  float r;
  asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(m), "v"(q));   // one SGPR per VOP3 on gfx9
  return r;
}
SQ_DEV float vmed3(float a, float b, float c) {
  float r;
  asm("v_med3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// TOP = 2: per lane the two smallest values are band members, a 3rd in the
// band -> overflow.  TOP = 3 (the overflow rows of a TOP = 2 pass, in list
// mode): three members per lane, a 4th -> overflow; its rows are loaded at
// the block start instead of prefetched (the longer lists need the
// registers).
#ifndef SQ_SPLIT_ACC_ALL
#define SQ_SPLIT_ACC_ALL 1   // 0: one accumulator in the two-member pass (measured slower overall)
#endif
template <int KSD, int TOP = 2>
__global__ void __launch_bounds__(256, 1) estep_f32_kernel(
    const float* __restrict__ X, const _Float16* __restrict__ C, const float* __restrict__ xn,
    int* __restrict__ labels, float* __restrict__ mind, long long* __restrict__ ovf_rows,
    int* __restrict__ ovf_count, double* __restrict__ part, long long n, int k_pad, float alpha,
    float inv_alpha2, float delta_s, RngKey key, long long row_offset, int ovf_cap,
    const long long* __restrict__ rlist, const int* __restrict__ rcount,
    const float* __restrict__ cmax2_p, long long* __restrict__ mrows, int* __restrict__ mcand,
    int* __restrict__ multi_count, unsigned char* __restrict__ xflag, long long mcap) {
  // list mode (rlist != null): the rows are rlist[0 .. *rcount) - the dense
  // rows handed over by the certified filter kernel (estep_x64_kernel)
  // cmax2_p (max_j alpha^2 ||c_j||^2, nullable): the band decisions are made
  // only where the fp32-faithful values are provably on one side of the
  // band edge.  A row with a tracked value within 2 E of it is settled in
  // fp64: its candidates (every tracked value <= edge + 2 E; complete when
  // no lane's last tracked value is that low) go to the multi list for the
  // fp64 re-check (recheck_rows_kernel, launched after this pass), else the
  // row overflows to the exact rows kernel.  E bounds |D'~ - alpha^2 D'|:
  // the hi/lo split drops <= 3 2^-22 |x^| |c^|; the fp32 accumulation of the
  // DX hi.hi products and 16 norm pieces adds <= (DX + 16) 2^-24, the two
  // cross-term accumulators (terms <= 2^-10 of them) <= 2 DX 2^-34 and the
  // final sum 2^-24, of the sum of their magnitudes <= 2 |x^| C + C^2
  // (C = max alpha ||c||).
  const float Cm = cmax2_p ? sqrtf(*cmax2_p) * (1.0f + 0x1p-16f) : 0.0f;
  // (SPLIT_ACC: the cross terms in their own accumulators - the tighter
  // bound.  The two-member pass then spills (its registers also hold the
  // next block's prefetched rows: 1.10 vs 0.63 ms on the hard regime's 214K
  // dense rows), but with one accumulator there its wider window sends more
  // rows on: hard regime 6.33 vs 5.78 ms per step)
  constexpr bool SPLIT_ACC = SQ_SPLIT_ACC_ALL || TOP == 3;
  constexpr float kEps3 =
      SPLIT_ACC ? (3.0f * 0x1p-22f + (KSD * 16 + 18.0f) * 0x1p-24f + 2.0f * KSD * 16 * 0x1p-34f) *
                      1.0625f
                : (3.0f * 0x1p-22f + (3.0f * KSD * 16 + 48.0f) * 0x1p-24f) * 1.0625f;
  if (rlist) n = min(n, (long long)*rcount);
  auto map_row = [&](long long r) -> long long { return rlist ? rlist[r] : r; };
  constexpr int NW = 4;
  constexpr int DX = KSD * 16;                 // fp32 row length (padded features)
  constexpr int HI_BYTES = (KSD + 1) * 2048;   // data chunks + norm chunk pair
  constexpr int TILE_BYTES = HI_BYTES + KSD * 2048;
  constexpr int PIECES = TILE_BYTES / 1024;
  constexpr int ROWS = NW * 32;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  auto buf = [&](int g) -> unsigned char* { return smem + (g & 1) * TILE_BYTES; };

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r32 = lane & 31;
  const int half = lane >> 5;
  const int n_tiles = k_pad / kTileN;
  const long long nblk = (n + ROWS - 1) / ROWS;
  long long blk = blockIdx.x;
  if (blk >= nblk) return;

  auto stage = [&](int G) {
    const int t = G % n_tiles;
    const unsigned char* tile = reinterpret_cast<const unsigned char*>(C) + (size_t)t * TILE_BYTES;
    unsigned char* dst = buf(G);
    for (int p = wave; p < PIECES; p += NW) {
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(tile + p * 1024 + lane * 16),
          (__attribute__((address_space(3))) void*)(dst + p * 1024), 16, 0, 0);
    }
  };

  // ---- A operand: 32 rows of this wave, fp32 from HBM, split in registers
  f16x8 ah[KSD], al[KSD];
  float4 raw[KSD][2];
  auto load_raw = [&](long long b) {
    const long long r = b * ROWS + wave * 32 + r32;
    const float* xr = X + (size_t)map_row(r < n ? r : n - 1) * DX + half * 8;
#pragma unroll
    for (int ks = 0; ks < KSD; ++ks) {
      raw[ks][0] = *reinterpret_cast<const float4*>(xr + ks * 16);
      raw[ks][1] = *reinterpret_cast<const float4*>(xr + ks * 16 + 4);
    }
  };
  auto split = [&]() {
#pragma unroll
    for (int ks = 0; ks < KSD; ++ks) {
      const float v[8] = {raw[ks][0].x, raw[ks][0].y, raw[ks][0].z, raw[ks][0].w,
                          raw[ks][1].x, raw[ks][1].y, raw[ks][1].z, raw[ks][1].w};
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float s = v[e] * alpha;                  // exact (power of two)
        const _Float16 h = (_Float16)s;
        ah[ks][e] = h;
        al[ks][e] = (_Float16)(s - (float)h);          // s - h exact in fp32
      }
    }
  };
  f16x8 aug = (f16x8)0;
  if (half == 0) { aug[0] = aug[1] = aug[2] = (_Float16)1.0f; }

  static_assert(TOP == 2 || TOP == 3, "two or three members per lane");
  constexpr bool PREFETCH = TOP == 2;
  // per-lane top-(TOP + 1) values and the indices of the TOP smallest
  float m1[16], m2[16], m3[16], m4[TOP == 3 ? 16 : 1];
  int i1[16], i2[16], i3[TOP == 3 ? 16 : 1];

  const int lane_off = (half * 64 + r32) * 16;
  auto ldb = [&](const unsigned char* p) -> f16x8 { return *reinterpret_cast<const f16x8*>(p); };

  auto tile_step = [&](const unsigned char* cur, f32x16& n0, f32x16& n1, bool do_mfma,
                       const f32x16& o0, const f32x16& o1, int t_prev, bool do_epi) {
    const int j0 = t_prev * kTileN + r32;
    const int j1 = j0 + 32;
    auto ins = [&](int i, float v, int j) {
      // values, not references, in the selects: a select of two array
      // elements becomes a select of addresses and spills the arrays
      const float q1 = m1[i], q2 = m2[i];
      const int a1 = i1[i], a2 = i2[i];
      const bool lt1 = v < q1, lt2 = v < q2;
      const int b2 = lt2 ? j : a2;
      if constexpr (TOP == 3) {
        const float q3 = m3[i];
        const int a3 = i3[i];
        const bool lt3 = v < q3;
        m4[i] = vmed3(q3, v, m4[i]);
        i3[i] = lt2 ? a2 : (lt3 ? j : a3);
      }
      m3[i] = vmed3(q2, v, m3[i]);
      m2[i] = vmed3(q1, v, q2);
      m1[i] = vmin(q1, v);
      i2[i] = lt1 ? a1 : b2;
      i1[i] = lt1 ? j : a1;
    };
    auto epi_row = [&](int i) {
      ins(i, o0[i], j0);
      ins(i, o1[i], j1);
    };
    if (do_mfma) {
      // the hi.hi products and the norm step in acc, the two cross terms
      // (~2^-11 of them) in their own accumulators: the rounding error of the
      // large partial sums comes from d_pad + 16 adds, not 3 d_pad + 48
      f32x16 acc0 = {0}, acc1 = {0}, acl0 = {0}, acl1 = {0};
      const unsigned char* hb = cur + lane_off;
      const unsigned char* lb = cur + HI_BYTES + lane_off;
      f16x8 bh0[2], bh1[2], bl0[2], bl1[2];
      bh0[0] = ldb(hb);
      bh1[0] = ldb(hb + 512);
      bl0[0] = ldb(lb);
      bl1[0] = ldb(lb + 512);
#pragma unroll
      for (int ks = 0; ks < KSD; ++ks) {
        const int c = ks & 1, nx = c ^ 1;
        bh0[nx] = ldb(hb + (ks + 1) * 2048);           // ks + 1 == KSD: the norm chunk
        bh1[nx] = ldb(hb + (ks + 1) * 2048 + 512);
        if (ks + 1 < KSD) {
          bl0[nx] = ldb(lb + (ks + 1) * 2048);
          bl1[nx] = ldb(lb + (ks + 1) * 2048 + 512);
        }
        acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[ks], bh0[c], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[ks], bh1[c], acc1, 0, 0, 0);
        if constexpr (SPLIT_ACC) {
          acl0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[ks], bl0[c], acl0, 0, 0, 0);
          acl1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[ks], bl1[c], acl1, 0, 0, 0);
          acl0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[ks], bh0[c], acl0, 0, 0, 0);
          acl1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[ks], bh1[c], acl1, 0, 0, 0);
        } else {
          acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[ks], bl0[c], acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[ks], bl1[c], acc1, 0, 0, 0);
          acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[ks], bh0[c], acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[ks], bh1[c], acc1, 0, 0, 0);
        }
        if (do_epi) {
#pragma unroll
          for (int i = (ks * 16) / KSD; i < ((ks + 1) * 16) / KSD; ++i) epi_row(i);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(aug, bh0[KSD & 1], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(aug, bh1[KSD & 1], acc1, 0, 0, 0);
      if constexpr (SPLIT_ACC) {
        n0 = acc0 + acl0;
        n1 = acc1 + acl1;
      } else {
        n0 = acc0;
        n1 = acc1;
      }
    } else if (do_epi) {
#pragma unroll
      for (int i = 0; i < 16; ++i) epi_row(i);
    }
  };
  auto sync_tile = [&]() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  };
  // merge two (min, 2nd, argmin) triples; ties of the min keep the smaller index
  auto merge = [](float& a1, float& a2, int& ai, float b1, float b2, int bi) {
    const float lo2 = vmin(a2, b2);
    const bool tb = b1 < a1 || (b1 == a1 && bi < ai);
    a2 = vmed3(a1, b1, lo2);
    a1 = vmin(a1, b1);
    ai = tb ? bi : ai;
  };

  int G = 0;
  stage(0);
  load_raw(blk);
  sync_tile();
  split();
  double my_inertia = 0.0;

  for (; blk < nblk; blk += gridDim.x) {
    const long long row0 = blk * ROWS + wave * 32;
    if constexpr (!PREFETCH) {
      if (blk != (long long)blockIdx.x) {   // the first block's rows came with the prologue
        load_raw(blk);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        split();
      }
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      m1[i] = m2[i] = m3[i] = __builtin_inff();
      i1[i] = i2[i] = 0;
      if constexpr (TOP == 3) {
        m4[i] = __builtin_inff();
        i3[i] = 0;
      }
    }
    f32x16 pA0, pA1, pB0, pB1;
    stage(G + 1);
    tile_step(buf(G), pA0, pA1, true, pA0, pA1, 0, false);
    sync_tile();
    int t = 0;
    while (true) {
      if (t + 1 >= n_tiles) {
        if constexpr (PREFETCH) load_raw(blk + gridDim.x);   // clamped rows: unconditional
        tile_step(smem, pB0, pB1, false, pA0, pA1, t, true);
        break;
      }
      stage(G + 2);
      tile_step(buf(G + 1), pB0, pB1, true, pA0, pA1, t, true);
      sync_tile();
      ++t;
      ++G;
      if (t + 1 >= n_tiles) {
        if constexpr (PREFETCH) load_raw(blk + gridDim.x);
        tile_step(smem, pA0, pA1, false, pB0, pB1, t, true);
        break;
      }
      stage(G + 2);
      tile_step(buf(G + 1), pA0, pA1, true, pB0, pB1, t, true);
      sync_tile();
      ++t;
      ++G;
    }
    ++G;

    // ---- transposed reduce-scatter merge of the 32 lanes of each half: a
    // lane ends with the row-global (min, 2nd, argmin) of row r32 >> 1
    float R1[16], R2[16];
    int RI[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) { R1[i] = m1[i]; R2[i] = m2[i]; RI[i] = i1[i]; }
#pragma unroll
    for (int o = 16, c = 8; o >= 2; o >>= 1, c >>= 1) {
      const bool hi = (r32 & o) != 0;
#pragma unroll
      for (int j = 0; j < c; ++j) {
        const float ra = R1[j], rb = R1[c + j], sa = R2[j], sb = R2[c + j];
        const int ia = RI[j], ib = RI[c + j];
        const float s1 = hi ? ra : rb, s2 = hi ? sa : sb;
        const int si = hi ? ia : ib;
        float k1 = hi ? rb : ra, k2 = hi ? sb : sa;
        int ki = hi ? ib : ia;
        merge(k1, k2, ki, __shfl_xor(s1, o, 64), __shfl_xor(s2, o, 64), __shfl_xor(si, o, 64));
        R1[j] = k1;
        R2[j] = k2;
        RI[j] = ki;
      }
    }
    float q1 = R1[0], q2 = R2[0];
    int qi = RI[0];
    merge(q1, q2, qi, __shfl_xor(R1[0], 1, 64), __shfl_xor(R2[0], 1, 64), __shfl_xor(RI[0], 1, 64));

    const int irow = r32 >> 1;
    const int rloc = (irow & 3) + 8 * (irow >> 2) + 4 * half;
    const long long grow_local = row0 + rloc;
    const bool owner = ((r32 & 1) == 0) && grow_local < n;
    const float thr = q1 + delta_s;
    const long long gmap = owner ? map_row(grow_local) : 0;
    const float xnv = owner ? xn[gmap] : 0.0f;
    // 2 E of this row (the edge moves with q1's own error too)
    const float e2 = cmax2_p ? 2.0f * kEps3 * (2.0f * alpha * sqrtf(xnv) * Cm + Cm * Cm) : 0.0f;
    // 2nd value within 2 E of the edge: membership undecidable here
    const bool unc = cmax2_p && fabsf(q2 - thr) <= e2;
    const bool band2 = q2 <= thr && !unc;
    if (owner) {
      const float dist = fmaxf(xnv + q1 * inv_alpha2, 0.0f);
      mind[gmap] = dist;
      if (!band2 && !unc) labels[gmap] = qi;
      my_inertia += (double)dist;
    }
    // rows with >= 2 band members: the rank rule over the per-lane top-2
    // lists; lane r32 holds the columns j = r32 mod 32, so (lane, index)
    // order is kappa order.  A lane whose 3rd value is in the band -> overflow.
    // Rows near the edge (unc, or a tracked value within 2 E): fp64 below.
    const unsigned long long slow = __ballot(owner && (band2 || unc));
    if (slow) {
      const float urow = band_u(key, row_offset + gmap);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const unsigned long long sel = slow & ((1ull << (2 * i)) | (1ull << (32 + 2 * i)));
        if (!sel) continue;
        const int src = 32 * half + 2 * i;
        const bool mine = (slow >> src) & 1ull;
        const float thr_i = __shfl(thr, src, 64);
        const float u_i = __shfl(urow, src, 64);
        const float e2_i = __shfl(e2, src, 64);
        const bool unc_i = __shfl(unc ? 1 : 0, src, 64) != 0;
        const long long g_i = __shfl(gmap, src, 64);
        const int c1 = (mine && m1[i] <= thr_i) ? 1 : 0;
        const int c2 = (mine && m2[i] <= thr_i) ? 1 : 0;
        int c3 = 0;
        bool v3;
        // certified mode: a tracked value within 2 E of the edge; the
        // candidates (tracked values <= edge + 2 E, in index order) and
        // whether a lane's last tracked value is that low (list incomplete)
        const float lim = thr_i + e2_i;
        bool nr = fabsf(m1[i] - thr_i) <= e2_i || fabsf(m2[i] - thr_i) <= e2_i ||
                  fabsf(m3[i] - thr_i) <= e2_i;
        int cc = (m1[i] <= lim ? 1 : 0) + (m2[i] <= lim ? 1 : 0);
        bool last_in;
        if constexpr (TOP == 3) {
          c3 = (mine && m3[i] <= thr_i) ? 1 : 0;
          v3 = mine && m4[i] <= thr_i;
          nr = nr || fabsf(m4[i] - thr_i) <= e2_i;
          cc += m3[i] <= lim ? 1 : 0;
          last_in = m4[i] <= lim;
        } else {
          v3 = mine && m3[i] <= thr_i;
          last_in = m3[i] <= lim;
        }
        const bool row_unc =
            cmax2_p && mine &&
            (unc_i || ((__ballot(mine && nr) >> (32 * half)) & 0xFFFFFFFFull) != 0ull);
        const int cl = c1 + c2 + c3;
        // inclusive prefixes of member / candidate counts over the 32 lanes
        // of this half
        int incl = cl, cinc = cc;
#pragma unroll
        for (int o = 1; o < 32; o <<= 1) {
          const int v = __shfl_up(incl, o, 32);
          const int w = __shfl_up(cinc, o, 32);
          if (r32 >= o) {
            incl += v;
            cinc += w;
          }
        }
        const int ctot = __shfl(cinc, 32 * half + 31, 64);
        const bool untr = ((__ballot(mine && last_in) >> (32 * half)) & 0xFFFFFFFFull) != 0ull;
        // near the edge with a complete list of 2..kMaxCand candidates: fp64
        // re-check of the candidates (multi list), otherwise overflow
        const bool to_multi = row_unc && mrows && !untr && ctot >= 2 && ctot <= kMaxCand;
        if (to_multi) {
          int* mc = mcand + g_i * (kMaxCand + 1);
          const int b0 = 1 + cinc - cc;
          if (cc > 0) mc[b0] = i1[i];
          if (cc > 1) mc[b0 + 1] = i2[i];
          if constexpr (TOP == 3) {
            if (cc > 2) mc[b0 + 2] = i3[i];
          }
        }
        const int total = __shfl(incl, 32 * half + 31, 64);
        const bool ovf = ((__ballot(v3) >> (32 * half)) & 0xFFFFFFFFull) != 0ull;
        const int r = band_rank(u_i, total > 0 ? total : 1);
        // the lane whose [incl - cl, incl) range holds rank r supplies the
        // member: its (r - (incl - cl))-th in ascending index order
        const bool hit = cl > 0 && r >= incl - cl && r < incl;
        int myj;
        if constexpr (TOP == 3) {
          // the lane's members in index (kappa) order
          const int x1 = i1[i];
          const int x2 = cl >= 2 ? i2[i] : 0x7fffffff, x3 = cl >= 3 ? i3[i] : 0x7fffffff;
          const int s_lo = min(x1, min(x2, x3)), s_hi = max(x1, max(x2, x3));
          const int s_mid = (int)((unsigned)x1 + (unsigned)x2 + (unsigned)x3 - (unsigned)s_lo -
                                  (unsigned)s_hi);   // (used for cl == 3 only)
          const int kk = r - (incl - cl);
          myj = kk == 0 ? s_lo : (kk == 1 ? (cl == 2 ? min(max(x1, x2), s_hi) : s_mid) : s_hi);
        } else {
          const int x1 = i1[i], x2 = i2[i];
          const int lo_j = min(x1, x2), hi_j = max(x1, x2);
          myj = cl == 1 ? x1 : (r - (incl - cl) == 0 ? lo_j : hi_j);
        }
        const unsigned long long hb = __ballot(hit) >> (32 * half);
        const int pl = hb ? __ffsll((long long)hb) - 1 : 0;
        const int jsel = __shfl(myj, 32 * half + pl, 64);
        if (mine && r32 == 2 * i) {
          const long long g = gmap;
          bool to_ovf = ovf;
          if (row_unc) {
            to_ovf = false;
            if (to_multi) {
              const long long slot = atomicAdd(multi_count, 1);
              if (slot < mcap) {
                mrows[slot] = g;
                if (xflag) xflag[slot] = 1;
                mcand[g * (kMaxCand + 1)] = ctot;
                labels[g] = -1;
              } else {
                to_ovf = true;
              }
            } else if (ctot == 1 && !untr) {
              labels[g] = qi;   // every other value certainly beyond the edge
            } else {
              to_ovf = true;
            }
          }
          if (to_ovf) {
            const int slot = atomicAdd(ovf_count, 1);
            if (slot < ovf_cap) ovf_rows[slot] = g;
            labels[g] = -1;
          } else if (!row_unc) {
            labels[g] = jsel;
          }
        }
      }
    }
    if constexpr (PREFETCH) {
      if (blk + gridDim.x < nblk) split();
    }
  }
  my_inertia = wave_sum(my_inertia);
  if (lane == 0) part[(size_t)blockIdx.x * NW + wave] = my_inertia;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ---------------------------------------------------------------------------
// estep_x64: certified filter + exact fp64 re-check (the default GPU E-step).
//
// One MFMA pass on the fp16 HI pieces only (xh . ch + the norm step) gives
// D'~ with a RIGOROUS per-row error bound
//   |D'~_ij - alpha^2 D'_ij| <= E_i = 1.0625 2^-10 |x^_i| C^        (fp16 rounding of both operands)
//                                   + 2^(qbits-23) M_i               (index packed in the low bits)
//                                   + 2^-15 M_i                      (fp32 accumulation, <= 2^15 adds)
//                                   + 2^-21 sqrt(d) (|x^_i| + C^)    (fp16 subnormal pieces)
// with |x^_i| = alpha |x_i|, C^ = max_j |c^_j| = 2 alpha max_j |c_j| and
// M_i = C^^2 / 4 + |x^_i| C^ >= every partial sum.  Every centroid that can
// be the row minimum or a band member then satisfies D'~ <= T_i = min D'~ +
// delta alpha^2 + 2 E_i (a candidate).  Each lane keeps the 3 smallest packed
// values of its columns; after the sweep the candidates (at most 2 per lane)
// go to an LDS list and their distances are recomputed EXACTLY in fp64 from
// the fp32 rows and centroids (sum_f (x_f - c_f)^2, scipy cdist's formula),
// so the label is the reference's fp64 delta-band rule, bit for bit:
//   * 1 candidate   : it is the argmin and the whole band - label known, the
//                     min distance is left to the M-step (mind = -1 marker:
//                     the segmented reduce computes |x - c_label|^2 in fp64
//                     while it streams the row anyway);
//   * 2..16         : fp64 re-check here, min, band, kappa-rank pick, exact
//                     mind.  The (row, candidate) pairs of the wave are
//                     flattened and 8 lanes compute one pair (32 features
//                     each, every load of the round in flight at once);
//   * more, or a lane whose 3rd value is a candidate ("dense" rows, where the
//     band edge is crowded beyond what one fp16 pass can separate): the row
//     goes to a device list for the fp32-faithful 3-pass kernel
//     (estep_f32_kernel in list mode).
// The A operand is the fp16 hi copy of the rows (alpha x rounded once at
// setup, 2 B per value: the same HBM stream as the bf16 kernel) and the next
// block's fragments are loaded right after the last MFMA of a block, so their
// latency hides behind the epilogue, the candidate extraction and the
// re-check.  4 waves (1 per SIMD: 512 registers, no spills) x 32 rows per
// workgroup share each staged
// tile; only the HI region of each operand tile is staged (34 KiB per slot at
// d = 256).
// Gap record of a multi-candidate row whose band the fp32 screen (or the gap
// screen) certified as {argmin} in iteration rec_it (csrc: recheck_fast_kernel,
// gap_screen_kernel): the argmin's squared distance da, the gaps
// g[c] = D(cand c) - da of its c_r <= kGapCand candidates (mcand order; 0 for
// the argmin's slot), one error bound err covering da and every g[c], and the
// candidates themselves (16-bit fields, k <= 16384):
//   ids[0] = j0 | slot << 14 | j1 << 16 | (c_r - 1) << 30,  ids[1] = j2 | j3 << 16
constexpr int kGapCand = 4;
struct __align__(16) GapRec {
  float da, err;
  float g[kGapCand];
  unsigned ids[2];
};
#ifndef SQ_X64_NW
#define SQ_X64_NW 4
#endif
constexpr int kX64Waves = SQ_X64_NW;   // waves per workgroup (8: 2 per SIMD, spills)
#ifndef SQ_X64_RING
#define SQ_X64_RING 3
#endif
#ifndef SQ_X64_PIN
#define SQ_X64_PIN 1
#endif
constexpr int kX64Ring = SQ_X64_RING;  // centroid-tile LDS slots (3: 2 tiles in flight)

// Diagnostic build only (-DSQ_X64_STAMP=1, a variant library): per-wave
// s_memtime sums of the kernel's phases go to a buffer of their own (never an
// output), read back by sq_x64_stamps().  [wave][0 total, 1 sweep, 2 tile-sync
// waits, 3 first-tile sync of a block (row-operand loads), 4 row-set epilogue,
// 5 blocks, 6 stage() issue, 7 epilogue up to the candidate lists, 8 A-load
// issue at block end]
#ifndef SQ_X64_STAMP
#define SQ_X64_STAMP 0
#endif
#if SQ_X64_STAMP
constexpr int kStampWaves = 8192;
constexpr int kStampN = 12;
__device__ unsigned long long g_x64_stamps[kStampWaves * kStampN];
#define SQ_STAMP_NOW() __builtin_amdgcn_s_memtime()
#endif

// Tile geometry of the certified filter: a 64-centroid tile is KT = KSD + 1
// k-steps (d_pad / 16 data steps + the norm step) of 2 KiB each.  Up to
// d_pad = 256 a whole tile is one LDS ring slot; above, the tile is staged in
// NS sub-tiles of at most 24 k-steps (48 KiB) so the 3-slot ring stays within
// the 160 KiB LDS at every d_pad <= 1024, and the accumulation of a tile spans
// NS slots (one counted-vmcnt barrier each).  The A operand (the wave's 32
// rows, d_pad / 4 fp16x2 registers) stays resident for the whole sweep.
template <int KSD>
struct X64Geom {
  static constexpr int KT = KSD + 1;
  static constexpr int NS = (KT + 23) / 24;
  static constexpr int SK = (KT + NS - 1) / NS;    // k-steps per slot
  static constexpr int SLOT = SK * 2048;           // bytes per LDS slot
};

// Row sets of 32 per wave: 2 (64 rows share each staged B fragment - half
// the L2 -> LDS staging per row, which bounds the d <= 256 sweep) while the
// A fragments fit the registers; 1 above d_pad = 256.
#ifndef SQ_X64_RS
#define SQ_X64_RS 2
#endif
#ifndef SQ_X64_PFD
#define SQ_X64_PFD 2   // B-fragment read distance of the row-set sweep (k-steps)
#endif
template <int KSD>
struct X64RowSets {
  static constexpr int value = KSD <= 16 ? SQ_X64_RS : 1;
};

template <typename F, int... I>
SQ_DEV void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
SQ_DEV void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

template <int KSD, int RS>
__global__ void __launch_bounds__(kX64Waves * 64) estep_x64_kernel(
    const _Float16* __restrict__ Xh, const float* __restrict__ X, const _Float16* __restrict__ C,
    const float* __restrict__ Cm, const float* __restrict__ xn, const float* __restrict__ cmax2_p,
    int* __restrict__ labels, float* __restrict__ mind, long long* __restrict__ dense_rows,
    int* __restrict__ dense_count, long long* __restrict__ mrows, int* __restrict__ mcand,
    int* __restrict__ multi_count, long long n, int k_pad, float alpha, float delta_s,
    RngKey key, long long row_offset, int dense_cap, int qbits, const long long* __restrict__ rlist,
    const int* __restrict__ rcount, float* __restrict__ ub, float* __restrict__ lb,
    int* __restrict__ mflag) {
  constexpr int NW = kX64Waves;
  constexpr int DX = KSD * 16;
  using GEO = X64Geom<KSD>;
  constexpr int KT = GEO::KT, NS = GEO::NS, SK = GEO::SK, SLOT = GEO::SLOT;
  constexpr int TILE_STRIDE = (2 * KSD + 1) * 2048;
  constexpr int PIECES = SLOT / 1024;           // 1 KiB LDS-DMA pieces per slot
  constexpr int ROWS = NW * 32 * RS;              // RS sets of 32 rows per wave
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int RING = kX64Ring;                // LDS slots
  constexpr int PPW = (PIECES + NW - 1) / NW;   // glds per wave per stage (uniform: counted vmcnt)
  auto buf = [&](int g) -> unsigned char* { return smem + (g % RING) * SLOT; };
  int* cand_all = reinterpret_cast<int*>(smem + RING * SLOT);        // [NW][RS][32][kMaxCand]
  int* cnt_all = cand_all + NW * RS * 32 * kMaxCand;                  // [NW][RS][32], then [NW][64] dump slots

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r32 = lane & 31;
  const int half = lane >> 5;
  const int n_tiles = k_pad / kTileN;
  // list mode (rlist != null): the rows to process are rlist[0 .. *rcount)
  // (the rows the Hamerly bounds could not prune); positions map to rows
  const long long ne = rlist ? min((long long)*rcount, n) : n;
  auto row_at = [&](long long pos) -> long long {
    const long long q = pos < ne ? pos : ne - 1;
    return rlist ? rlist[q] : q;
  };
  const long long nblk = (ne + ROWS - 1) / ROWS;
  long long blk = blockIdx.x;
  if (blk >= nblk) return;
  const uint32_t qmask = (1u << qbits) - 1u;
  const uint32_t keep = ~qmask;
  // rigorous bound constants (fp32, rounded up by the 1.0625 / 1+2^-16 factors)
  const float Ch = 2.0f * sqrtf(*cmax2_p) * (1.0f + 0x1p-16f);
  const float pack_rel = ldexpf(1.0f, qbits - 23) + 0x1p-15f;
  const float sub_rel = 0x1p-21f * sqrtf((float)DX);

  // unit U = sub-tile U % NS of tile (U / NS) % n_tiles (the sequence runs on
  // across row blocks: the next block's first tiles are staged during the
  // current block's last ones)
  auto stage = [&](int U) {
    const int t = (NS == 1 ? U : U / NS) % n_tiles;
    const int sub = NS == 1 ? 0 : U % NS;
    const int npc = 2 * min(SK, KT - sub * SK);   // valid pieces of this sub-tile
    const unsigned char* tile = reinterpret_cast<const unsigned char*>(C) + (size_t)t * TILE_STRIDE +
                                (size_t)sub * SLOT;
    unsigned char* dst = buf(U);
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      // every wave issues PPW loads (the surplus repeat the last piece: same
      // bytes to the same LDS slot) so one counted vmcnt fits all waves
      const int p = wave + NW * i < npc ? wave + NW * i : npc - 1;
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(tile + p * 1024 + lane * 16),
          (__attribute__((address_space(3))) void*)(dst + p * 1024), 16, 0, 0);
    }
  };

  // the wave's RS sets of 32 rows share every B fragment (register blocking:
  // the staged centroid tiles are read once per 32 RS rows)
  f16x8 ah[RS][KSD];
  auto load_a = [&](long long b) {
#pragma unroll
    for (int st = 0; st < RS; ++st) {
      const long long r = row_at(b * ROWS + (wave * RS + st) * 32 + r32);
      const _Float16* xr = Xh + (size_t)r * DX + half * 8;
#pragma unroll
      for (int ks = 0; ks < KSD; ++ks) ah[st][ks] = *reinterpret_cast<const f16x8*>(xr + ks * 16);
    }
  };
  f16x8 aug = (f16x8)0;
  if (half == 0) { aug[0] = aug[1] = aug[2] = (_Float16)1.0f; }
  // |x|^2 of the row whose reduced minimum this lane ends with (rl_own of
  // each row set), loaded with the block's A operand so the epilogue does not
  // wait on a dependent global load
  const int rl_lane = ((r32 >> 1) & 3) + 8 * ((r32 >> 1) >> 2) + 4 * half;
  float xn_cur[RS], xn_nxt[RS];
  auto load_xn = [&](long long b, float (&dst)[RS]) {
#pragma unroll
    for (int st = 0; st < RS; ++st) dst[st] = xn[row_at(b * ROWS + (wave * RS + st) * 32 + rl_lane)];
  };

  float m1[RS][16], m2[RS][16], m3[RS][16];
  const int lane_off = (half * 64 + r32) * 16;
  auto ldb = [&](const unsigned char* p) -> f16x8 { return *reinterpret_cast<const f16x8*>(p); };
  auto ins = [&](int st, int i, float v, uint32_t q) {
    const float p = and_or(v, keep, q);   // (v & keep) | q: the tile index in the low bits
    const float a1 = m1[st][i], a2 = m2[st][i];
    m3[st][i] = vmed3(a2, p, m3[st][i]);
    m2[st][i] = vmed3(a1, p, a2);
    m1[st][i] = vmin(a1, p);
  };
  typedef f32x16 Acc[RS][2];
  // k-steps [S SK, min((S+1) SK, KT)) of the current tile from the slot at
  // cur, with the epilogue rows of the previous tile (o0 / o1, tile t_prev)
  // spread over the tile's KT k-steps
  auto sub_step = [&](auto S_, const unsigned char* cur, Acc& acc, const Acc& o, int t_prev,
                      bool do_epi) {
    constexpr int S = decltype(S_)::value;
    constexpr int K0 = S * SK, K1 = (S + 1) * SK < KT ? (S + 1) * SK : KT;
    const uint32_t q0 = (uint32_t)(t_prev * 2), q1 = q0 + 1u;
    const unsigned char* hb = cur + lane_off;
    f16x8 b0[2], b1[2];
    b0[0] = ldb(hb);
    b1[0] = ldb(hb + 512);
#pragma unroll
    for (int ks = K0; ks < K1; ++ks) {
      const int c = (ks - K0) & 1, nx = c ^ 1;
      if (ks + 1 < K1) {
        b0[nx] = ldb(hb + (ks + 1 - K0) * 2048);
        b1[nx] = ldb(hb + (ks + 1 - K0) * 2048 + 512);
      }
#pragma unroll
      for (int st = 0; st < RS; ++st) {
        const f16x8 A = ks < KSD ? ah[st][ks] : aug;
        acc[st][0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A, b0[c], acc[st][0], 0, 0, 0);
        acc[st][1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A, b1[c], acc[st][1], 0, 0, 0);
      }
      if (do_epi) {
        // the previous tile's RS x 16 rows, spread evenly over the KT k-steps
#pragma unroll
        for (int e = (ks * 16 * RS) / KT; e < ((ks + 1) * 16 * RS) / KT; ++e) {
          ins(e / 16, e % 16, o[e / 16][0][e % 16], q0);
          ins(e / 16, e % 16, o[e / 16][1][e % 16], q1);
        }
      }
#if SQ_X64_PIN
      __builtin_amdgcn_sched_barrier(0);
#endif
    }
  };
  auto epi_all = [&](const Acc& o, int t_prev) {
    const uint32_t q0 = (uint32_t)(t_prev * 2), q1 = q0 + 1u;
#pragma unroll
    for (int st = 0; st < RS; ++st)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        ins(st, i, o[st][0][i], q0);
        ins(st, i, o[st][1][i], q1);
      }
  };
  // RING == 2: the tile staged in this step must land before the barrier
  // (vmcnt(0)).  RING == 3: staging runs two tiles ahead and the barrier
  // only retires the tile staged one step earlier - vmcnt(PPW) leaves this
  // step's glds in flight across the raw s_barrier (no __syncthreads: its
  // fence would drain them).
#if SQ_X64_STAMP
  unsigned long long st_sync = 0, st_sync0 = 0, st_post = 0, st_sweep = 0, st_blocks = 0;
  unsigned long long st_stage = 0, st_cand = 0, st_aload = 0, st_rmin = 0, st_cl = 0, st_ub = 0;
  const unsigned long long st_t0 = SQ_STAMP_NOW();
  bool st_first = true;
#endif
  auto sync_tile = [&]() {
#if SQ_X64_STAMP
    const unsigned long long sa = SQ_STAMP_NOW();
#endif
    if constexpr (RING == 2) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PPW) : "memory");
    }
    __builtin_amdgcn_s_barrier();
#if SQ_X64_STAMP
    const unsigned long long sw = SQ_STAMP_NOW() - sa;
    st_sync += sw;
    if (st_first) st_sync0 += sw;
    st_first = false;
#endif
  };

  // one tile = NS sub-steps, each: stage the unit RING - 1 ahead, MFMAs on
  // the current unit, retire the next one (counted vmcnt + raw barrier)
  int U = 0;
  auto tile = [&](Acc& acc, const Acc& o, int t_prev, bool do_epi) {
    // accumulates straight into the destination set (its previous contents
    // were the epilogue input of the tile before: consumed)
#pragma unroll
    for (int st = 0; st < RS; ++st) acc[st][0] = acc[st][1] = (f32x16){0};
    static_for<NS>([&](auto S_) {
      stage(U + RING - 1);
      sub_step(S_, buf(U), acc, o, t_prev, do_epi);
      sync_tile();
      ++U;
    });
  };

  stage(0);
  if constexpr (RING == 3) stage(1);
  load_a(blk);
  load_xn(blk, xn_cur);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  for (; blk < nblk; blk += gridDim.x) {
#pragma unroll
    for (int st = 0; st < RS; ++st)
#pragma unroll
      for (int i = 0; i < 16; ++i) m1[st][i] = m2[st][i] = m3[st][i] = __builtin_inff();
    if constexpr (RS == 1) {
      Acc pA, pB;
      tile(pA, pA, 0, false);
      int t = 0;
      while (true) {
        if (t + 1 >= n_tiles) {
          load_a(blk + gridDim.x);   // clamped rows: unconditional (no phi on ah)
          load_xn(blk + gridDim.x, xn_nxt);
          epi_all(pA, t);
          break;
        }
        tile(pB, pA, t, true);
        ++t;
        if (t + 1 >= n_tiles) {
          load_a(blk + gridDim.x);
          load_xn(blk + gridDim.x, xn_nxt);
          epi_all(pB, t);
          break;
        }
        tile(pA, pB, t, true);
        ++t;
      }
    } else {
      // RS row sets: each staged tile is swept one column half at a time
      // (both row sets per B fragment); the half just finished is inserted
      // during the next half's MFMAs - two RS x 16-register accumulator sets
      // live instead of four
      f32x16 cA[RS], cB[RS];
      // B fragments stream through a ring of PFD + 1 registers, PFD k-steps
      // ahead of their MFMAs (one k-step of cover - a single MFMA pair - left
      // the ds_read_b128 latency exposed at every k-step); the two column
      // halves of a tile are one stream of 2 KT fragments, so the second
      // half's first reads are in flight during the first half's last MFMAs
      constexpr int PFD = SQ_X64_PFD;
      constexpr int NB = PFD + 1;
      f16x8 bq[NB];
      auto frag = [&](const unsigned char* cur, int g) -> f16x8 {
        return ldb(cur + lane_off + (g / KT) * 512 + (g % KT) * 2048);
      };
      auto pass = [&](auto H_, const unsigned char* cur, f32x16 (&acc)[RS],
                      const f32x16 (&o)[RS], uint32_t qo, bool do_epi) {
        constexpr int h = decltype(H_)::value;
#pragma unroll
        for (int st = 0; st < RS; ++st) acc[st] = (f32x16){0};
#pragma unroll
        for (int ks = 0; ks < KT; ++ks) {
          const int g = h * KT + ks;
          if (g + PFD < 2 * KT) bq[(g + PFD) % NB] = frag(cur, g + PFD);
#pragma unroll
          for (int st = 0; st < RS; ++st)
            acc[st] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ks < KSD ? ah[st][ks] : aug,
                                                             bq[g % NB], acc[st], 0, 0, 0);
          if (do_epi) {
#pragma unroll
            for (int e = (ks * 16 * RS) / KT; e < ((ks + 1) * 16 * RS) / KT; ++e)
              ins(e / 16, e % 16, o[e / 16][e % 16], qo);
          }
#if SQ_X64_PIN
          __builtin_amdgcn_sched_barrier(0);
#endif
        }
      };
      auto drain = [&](const f32x16 (&o)[RS], uint32_t qo) {
#pragma unroll
        for (int st = 0; st < RS; ++st)
#pragma unroll
          for (int i = 0; i < 16; ++i) ins(st, i, o[st][i], qo);
      };
      static_assert(NS == 1, "row sets need whole tiles per LDS slot");
#if SQ_X64_STAMP
      const unsigned long long sw0 = SQ_STAMP_NOW();
      st_first = true;
      ++st_blocks;
#endif
      for (int t = 0; t < n_tiles; ++t) {
#if SQ_X64_STAMP
        const unsigned long long sg0 = SQ_STAMP_NOW();
#endif
        stage(U + RING - 1);
#if SQ_X64_STAMP
        st_stage += SQ_STAMP_NOW() - sg0;
#endif
        // half 0 of tile t (with the previous tile's half 1), then half 1
        // (with this tile's half 0); packed index q = 2 t + half
#pragma unroll
        for (int j = 0; j < PFD; ++j) bq[j] = frag(buf(U), j);
        pass(std::integral_constant<int, 0>{}, buf(U), cA, cB, (uint32_t)(2 * t - 1), t > 0);
        pass(std::integral_constant<int, 1>{}, buf(U), cB, cA, (uint32_t)(2 * t), true);
        sync_tile();
        ++U;
      }
#if SQ_X64_STAMP
      const unsigned long long sl0 = SQ_STAMP_NOW();
#endif
      load_a(blk + gridDim.x);   // clamped rows: unconditional
      load_xn(blk + gridDim.x, xn_nxt);
#if SQ_X64_STAMP
      st_aload += SQ_STAMP_NOW() - sl0;
#endif
      drain(cB, (uint32_t)(2 * n_tiles - 1));
#if SQ_X64_STAMP
      st_sweep += SQ_STAMP_NOW() - sw0;
#endif
    }
#if SQ_X64_STAMP
    const unsigned long long sp0 = SQ_STAMP_NOW();
#endif

    // ---- per row set: row minimum, candidates, bounds, classification (a
    // runtime loop: one copy of the code; the set's top-3 lists are selected
    // by value into ms1..ms3 - compile-time register indices only)
#pragma nounroll
    for (int st = 0; st < RS; ++st) {
#if SQ_X64_STAMP
    const unsigned long long sc0 = SQ_STAMP_NOW();
#endif
    const long long row0 = blk * ROWS + (wave * RS + st) * 32;
    int* cand = cand_all + (wave * RS + st) * 32 * kMaxCand;
    int* cnt = cnt_all + (wave * RS + st) * 32;
    float ms1[16], ms2[16], ms3[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      ms1[i] = m1[0][i]; ms2[i] = m2[0][i]; ms3[i] = m3[0][i];
#pragma unroll
      for (int o = 1; o < RS; ++o) {
        const float a1 = m1[o][i], a2 = m2[o][i], a3 = m3[o][i];
        ms1[i] = st == o ? a1 : ms1[i];
        ms2[i] = st == o ? a2 : ms2[i];
        ms3[i] = st == o ? a3 : ms3[i];
      }
    }

    // ---- row minimum (packed) by the transposed reduce-scatter: lane r32
    // even ends with the min of row irow = r32 >> 1 of its half
    auto row_min = [&](float (&R)[16]) -> float {
#pragma unroll
      for (int o = 16, c = 8; o >= 2; o >>= 1, c >>= 1) {
        const bool hi = (r32 & o) != 0;
#pragma unroll
        for (int j = 0; j < c; ++j) {
          // values first, then the selects: a select of two array elements
          // becomes a select of addresses (runtime-indexed register array)
          const float lo_v = R[j], hi_v = R[c + j];
          const float keepv = hi ? hi_v : lo_v, sendv = hi ? lo_v : hi_v;
          R[j] = vmin(keepv, __shfl_xor(sendv, o, 64));
        }
      }
      return vmin(R[0], __shfl_xor(R[0], 1, 64));
    };
    float R[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) R[i] = ms1[i];
    const float rmin = row_min(R);
    const int irow = r32 >> 1;
    const int rl_own = (irow & 3) + 8 * (irow >> 2) + 4 * half;
    float xn_own = xn_cur[0];
#pragma unroll
    for (int o = 1; o < RS; ++o) xn_own = st == o ? xn_cur[o] : xn_own;
    const float xsv = alpha * sqrtf(xn_own) * (1.0f + 0x1p-16f);
    const float prod = xsv * Ch;
    const float mag = 0.25f * Ch * Ch + prod;
    const float E = 1.0625f * 0x1p-10f * prod + pack_rel * mag + sub_rel * (xsv + Ch);
    const float T_own = __uint_as_float(__float_as_uint(rmin) & keep) + delta_s + 2.0f * E;

    // ---- candidates -> LDS list of their row (C/D layout: register i of this
    // lane is row (i & 3) + 8 (i >> 2) + 4 half, column class r32)
#if SQ_X64_STAMP
    const unsigned long long sc1 = SQ_STAMP_NOW();
    st_rmin += sc1 - sc0;
#endif
    float nc[16];   // per register: this lane's smallest NON-candidate value
    // the 16 row thresholds of this lane's registers: all 16 reads in flight
    // before the first use (one LDS latency, not 16 in a chain)
    float Tr[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) Tr[i] = __shfl(T_own, 32 * half + 2 * i, 64);
    // per-lane dump slot: the list / count stores below are unconditional
    // (a lane with nothing to store writes here) - no exec-mask branches
    int* const sink = cnt_all + NW * RS * 32 + wave * 64 + lane;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float T = Tr[i];
      nc[i] = ms1[i] > T ? ms1[i] : (ms2[i] > T ? ms2[i] : ms3[i]);
      const int rl = (i & 3) + 8 * (i >> 2) + 4 * half;
      auto jof = [&](float p) -> int {
        const uint32_t q = __float_as_uint(p) & qmask;
        return (int)((q >> 1) * kTileN + (q & 1u) * 32u) + r32;
      };
      // the 32 lanes of this half hold the whole row rl (one register each):
      // wave ballots give its candidate count and every candidate's list slot
      // (lane order) - no LDS atomics; each row's count is written once
      const unsigned long long b1 = __ballot(ms1[i] <= T), b2 = __ballot(ms2[i] <= T);
      const unsigned long long b3 = __ballot(ms3[i] <= T);   // lane may hide more: dense
      const uint32_t b1l = (uint32_t)b1, b1h = (uint32_t)(b1 >> 32);
      const uint32_t b2l = (uint32_t)b2, b2h = (uint32_t)(b2 >> 32);
      const int c1 = __popc(half ? b1h : b1l), c2 = __popc(half ? b2h : b2l);
      const bool d3 = (half ? (uint32_t)(b3 >> 32) : (uint32_t)b3) != 0u;
      const int s1 = (int)__builtin_amdgcn_mbcnt_hi(b1h, __builtin_amdgcn_mbcnt_lo(b1l, 0u)) -
                     (half ? __popc(b1l) : 0);
      const int s2 = c1 + (int)__builtin_amdgcn_mbcnt_hi(b2h, __builtin_amdgcn_mbcnt_lo(b2l, 0u)) -
                     (half ? __popc(b2l) : 0);
      *((ms1[i] <= T && s1 < kMaxCand) ? cand + rl * kMaxCand + s1 : sink) = jof(ms1[i]);
      *((ms2[i] <= T && s2 < kMaxCand) ? cand + rl * kMaxCand + s2 : sink) = jof(ms2[i]);
      *(r32 == 0 ? cnt + rl : sink) = c1 + c2 + (d3 ? kMaxCand + 1 : 0);
    }
    // Hamerly bounds of this row (distances, not squared): ub >= |x - c_min|,
    // lb <= distance to every NON-candidate centroid (the smallest filter
    // value above T minus the bound; for a one-candidate row the 2nd
    // smallest), from D = |x|^2 + D'/alpha^2 with an fp32 margin.  A
    // multi-candidate row whose non-candidates stay beyond the band under
    // the next centroid shifts keeps its candidate set (bounds_filter).
#if SQ_X64_STAMP
    const unsigned long long sc2 = SQ_STAMP_NOW();
    st_cl += sc2 - sc1;
#endif
    float ub_own = 0.f, lb_own = 0.f;
    if (ub) {
      const float ncmin = row_min(nc);
      const float ia2 = 1.0f / (alpha * alpha);
      const float d1 = (__uint_as_float(__float_as_uint(rmin) & keep) + E) * ia2;
      const float d2 = (__uint_as_float(__float_as_uint(ncmin) & keep) - E) * ia2;
      const float marg = 0x1p-20f * (xn_own + fabsf(d1) + fabsf(d2));
      ub_own = sqrtf(fmaxf(xn_own + d1 + marg, 0.f)) * (1.0f + 0x1p-20f);
      lb_own = sqrtf(fmaxf(xn_own + d2 - marg, 0.f)) * (1.0f - 0x1p-20f);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
#if SQ_X64_STAMP
    st_cand += SQ_STAMP_NOW() - sc0;
    st_ub += SQ_STAMP_NOW() - sc2;
#endif

    // ---- classify the wave's 32 rows (lane r32 < 32 owns row r32)
    const bool valid = row0 + r32 < ne;
    const long long g = row_at(row0 + r32);
    // bounds of row r32 live on lane 2 * rl_inv(r32) of its half
    if (ub) {
      const int src = ((r32 & 3) + 4 * ((r32 >> 3) & 3)) * 2 + 32 * ((r32 >> 2) & 1);
      const float u = __shfl(ub_own, src, 64), l = __shfl(lb_own, src, 64);
      if (valid && half == 0) {
        ub[g] = u;   // multi rows: replaced by the re-check (label distance)
        lb[g] = cnt[r32] <= kMaxCand ? l : 0.0f;   // dense: always re-evaluate
      }
    }
    const int c_r = cnt[r32];
    const bool dense = c_r > kMaxCand;
    const bool multi = valid && !dense && c_r >= 2;
    if (mflag && valid && half == 0 && !multi) mflag[g] = 0;
    if (valid && half == 0) {
      if (dense) {
        const int s = atomicAdd(dense_count, 1);
        if (s < dense_cap) dense_rows[s] = g;
        labels[g] = -1;
      } else if (c_r == 1) {
        labels[g] = cand[r32 * kMaxCand];
        mind[g] = -1.0f;   // filled by the M-step's segmented reduce
      }
    }
    // multi-candidate rows -> global list; their fp64 re-check runs in
    // recheck_rows_kernel (latency-bound global loads kept out of this
    // MFMA-bound sweep); a full list routes rows to the dense path
    const bool mrow = multi && half == 0;
    const unsigned long long mm = __ballot(mrow);
    const int nm = __popcll(mm);
    int mbase = 0;
    if (lane == 0 && nm) mbase = atomicAdd(multi_count, nm);
    mbase = __shfl(mbase, 0, 64);
    if (mrow) {
      const long long slot = (long long)mbase + __popcll(mm & ((1ull << lane) - 1ull));
      if (mflag) mflag[g] = slot < n ? 1 : 0;
      if (slot < n) {
        mrows[slot] = g;
        int* mc = mcand + g * (kMaxCand + 1);   // per row: kept across iterations
        mc[0] = c_r;
        for (int c = 0; c < c_r; ++c) mc[1 + c] = cand[r32 * kMaxCand + c];
      } else {
        const int s2 = atomicAdd(dense_count, 1);
        if (s2 < dense_cap) dense_rows[s2] = g;
        labels[g] = -1;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    }   // row sets
#pragma unroll
    for (int st = 0; st < RS; ++st) xn_cur[st] = xn_nxt[st];
#if SQ_X64_STAMP
    st_post += SQ_STAMP_NOW() - sp0;
#endif
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#if SQ_X64_STAMP
  const int sidx = blockIdx.x * NW + wave;
  if (lane == 0 && sidx < kStampWaves) {
    unsigned long long* o = g_x64_stamps + (size_t)sidx * kStampN;
    o[0] = SQ_STAMP_NOW() - st_t0; o[1] = st_sweep; o[2] = st_sync; o[3] = st_sync0;
    o[4] = st_post; o[5] = st_blocks; o[6] = st_stage; o[7] = st_cand; o[8] = st_aload;
    o[9] = st_rmin; o[10] = st_cl; o[11] = st_ub;
  }
#endif
}

// ---------------------------------------------------------------------------
// Hamerly pruning of the certified E-step (exact).  After a centroid update
// with per-centroid shifts s_j = |c_j' - c_j| (fp64): ub_i += s_{label_i},
// lb_i -= max_j s_j.  ub bounds the distance to the label, lb the distance to
// every centroid outside the row's candidate set S (S = {label} for a
// one-candidate row).  When lb_i > 0 and lb_i^2 - ub_i^2 > delta, every
// centroid outside S is more than delta beyond the label's squared distance
// under the new centroids, so the argmin and the whole delta-band lie in S:
//   * |S| = 1 (mflag = 0): the label stands, the row is skipped;
//   * |S| >= 2: the row skips the filter sweep and goes straight to the fp64
//     re-check over S (its candidate list is copied from the previous
//     iteration's multi list; its candidates stay in the per-row mcand).
// The rest go to rlist for the x64 kernel.  No host sync: both counts stay
// on the device (one atomic per 4K-row chunk and list).
// A few centroids move far more than the rest (the contested ones: median
// shift ~0.006 vs max ~1 on the bench), so max_j s_j would collapse every
// row's lb: the nf fastest centroids F are taken out of the max (sm = the
// largest shift outside F) and bounded one by one: max(lb - s_f, cc[l][f] -
// ub) with Elkan's cc[l][f] = |c_l' - c_f'| (rounded down; +inf for f = l)
// from fast_centroids - never weaker than lb - max_j s_j.
// Rows per workgroup = 256 PER: 4096 on large shards (one list atomic per
// chunk), 1024 below ~4M rows so a small shard (8-GPU strong scaling: 1.25M
// rows per rank) still spreads over >= 1024 workgroups instead of 305.
template <int PER>
__global__ void __launch_bounds__(256) bounds_filter_kernel(
    const int* __restrict__ labels, float* __restrict__ ub, float* __restrict__ lb,
    const double* __restrict__ shift, const double* __restrict__ smax, long long n, double delta,
    long long* __restrict__ rlist, int* __restrict__ rcount, const int* __restrict__ mflag,
    long long* __restrict__ mrows, int* __restrict__ multi_count, const float* __restrict__ cc,
    const int* __restrict__ fidx, int nf, int k, int rec_on, int it_now, int it_lo,
    long long* __restrict__ mrows_b, int* __restrict__ count_b, float* __restrict__ corr,
    int* __restrict__ rec_count) {
  constexpr int kBoundsChunk = PER * 256;   // PER rows per thread (bit masks)
  // A multi row whose bounds hold keeps its candidate set; when its gap
  // record is current (mflag = 2 + the record's base iteration b, it_lo <= b
  // < it_now; the sweep stores 1 for a multi row without one) the row goes to
  // list B, where the record is moved by the centroid shifts since b (the
  // fp16 row, 512 B), else to the multi list (fp32 screen of the fp32 row)
  __shared__ int wsum[4], wsum_b[4];
  __shared__ int base_a, base_m, base_b;
  __shared__ double sf_s[65];               // shifts of the fast centroids, [nf] = max
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (tid < nf) sf_s[tid] = shift[fidx[tid]];
  __syncthreads();
  if (tid == 0) {
    double m = 0.0;
    for (int f = 0; f < nf; ++f) m = fmax(m, sf_s[f]);
    sf_s[nf] = m;
  }
  __syncthreads();
  const double sm = *smax;
  const long long c0 = (long long)blockIdx.x * kBoundsChunk;
  unsigned long long act = 0, rec = 0, recb = 0;   // bit p: row c0 + p * 256 + tid
  // rows in batches of 4: every load of a batch (the row's label / bounds /
  // flag, then the label's shift and Elkan minimum) is issued before any of
  // the batch's math - a thread's PER rows are 3 dependent-load latencies
  // per batch, not per row
  constexpr int B = PER % 4 == 0 ? 4 : 1;
  for (int p0 = 0; p0 < PER; p0 += B) {
    int lv[B], mfv[B];
    float ubv[B], lbv[B];
    bool inb[B];
#pragma unroll
    for (int q = 0; q < B; ++q) {
      const long long i = c0 + (long long)(p0 + q) * 256 + tid;
      inb[q] = i < n;
      const long long ii = inb[q] ? i : 0;
      lv[q] = inb[q] ? labels[ii] : -1;
      // the E-step's per-row corrections start at 0 (this pass visits every
      // row: the separate memset of the list-mode E-step is not needed)
      if (corr && inb[q]) corr[ii] = 0.0f;
      ubv[q] = ub[ii];
      lbv[q] = lb[ii];
      mfv[q] = mflag[ii];
    }
    double shv[B];
    float cmv[B];
#pragma unroll
    for (int q = 0; q < B; ++q) {
      const int l = lv[q];
      shv[q] = l >= 0 ? shift[l] : 1e300;
      cmv[q] = (l >= 0 && nf > 0) ? cc[(size_t)k * nf + l] : 0.0f;
    }
#pragma unroll
    for (int q = 0; q < B; ++q) {
      if (!inb[q]) continue;
      const int p = p0 + q;
      const long long i = c0 + (long long)p * 256 + tid;
      const int l = lv[q];
      const double u = (double)ubv[q] + shv[q];
      // the moved lower bound lb0 -> w (every centroid except the label)
      auto wbound = [&](double lb0) -> double {
        double w = lb0 - sm;
        // the nf fastest centroids (excluded from sm): the better of Elkan's
        // bound through the label, |x - c_f'| >= |c_l' - c_f'| - |x - c_l'| >=
        // cc[l][f] - u, and the moved lower bound lb - s_f
        if (l >= 0 && nf > 0 && w > 0.0) {   // (w <= 0: active anyway)
          // cheap form first: every fast centroid is at least cmin[l] from the
          // label and moved at most s_F = max_f s_f
          const double wc = fmin(w, fmax((double)cmv[q] - u, lb0 - sf_s[nf]));
          if (wc > 0.0 && wc * wc - u * u > delta * (1.0 + 1e-9) + 1e-30) {
            w = wc;
          } else {   // per fast centroid (tighter)
            const float* cl = cc + (size_t)l * nf;
            if ((nf & 3) == 0) {
              for (int f = 0; f < nf; f += 4) {
                const float4 c4 = *reinterpret_cast<const float4*>(cl + f);
                w = fmin(w, fmax((double)c4.x - u, lb0 - sf_s[f]));
                w = fmin(w, fmax((double)c4.y - u, lb0 - sf_s[f + 1]));
                w = fmin(w, fmax((double)c4.z - u, lb0 - sf_s[f + 2]));
                w = fmin(w, fmax((double)c4.w - u, lb0 - sf_s[f + 3]));
              }
            } else {
              for (int f = 0; f < nf; ++f) w = fmin(w, fmax((double)cl[f] - u, lb0 - sf_s[f]));
            }
          }
        }
        return w;
      };
      const double w = wbound((double)lbv[q]);
      const bool holds = l >= 0 && w > 0.0 && w * w - u * u > delta * (1.0 + 1e-9) + 1e-30;
      if (!holds) {
        act |= 1ull << p;
      } else {
        ub[i] = (float)u * (1.0f + 0x1p-22f);
        lb[i] = (float)w * (1.0f - 0x1p-22f);
        if (mfv[q]) {
          if (rec_on && mfv[q] >= it_lo + 2 && mfv[q] <= it_now + 1) recb |= 1ull << p;
          else rec |= 1ull << p;
        }
      }
    }
  }
  // block-wide exclusive scan of both per-thread counts (packed 16 | 16 bits:
  // a chunk holds 2^14 rows), ONE atomic per list and chunk
  const int mine = __popcll(act) | (__popcll(rec) << 16);
  const int mine_b = __popcll(recb);
  int incl = mine, incl_b = mine_b;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int v = __shfl_up(incl, o, 64);
    const int vb = __shfl_up(incl_b, o, 64);
    if (lane >= o) {
      incl += v;
      incl_b += vb;
    }
  }
  if (lane == 63) {
    wsum[wv] = incl;
    wsum_b[wv] = incl_b;
  }
  __syncthreads();
  int before = 0, total = 0, before_b = 0, total_b = 0;
#pragma unroll
  for (int w2 = 0; w2 < 4; ++w2) {
    before += w2 < wv ? wsum[w2] : 0;
    total += wsum[w2];
    before_b += w2 < wv ? wsum_b[w2] : 0;
    total_b += wsum_b[w2];
  }
  if (tid == 0) {
    base_a = (total & 0xffff) ? atomicAdd(rcount, total & 0xffff) : 0;
    base_m = (total >> 16) ? atomicAdd(multi_count, total >> 16) : 0;
    // the multi list's head (this pass's rows, before the sweep appends):
    // the incremental M-step's second row list
    if (rec_count && (total >> 16)) atomicAdd(rec_count, total >> 16);
    base_b = total_b ? atomicAdd(count_b, total_b) : 0;
  }
  __syncthreads();
  const int ex = before + incl - mine;
  int pos = base_a + (ex & 0xffff);
  for (int p = 0; p < PER && act; ++p) {
    if (act & (1ull << p)) {
      rlist[pos++] = c0 + (long long)p * 256 + tid;
      act &= ~(1ull << p);
    }
  }
  int mpos = base_m + (ex >> 16);
  for (int p = 0; p < PER && rec; ++p) {
    if (rec & (1ull << p)) {
      mrows[mpos++] = c0 + (long long)p * 256 + tid;
      rec &= ~(1ull << p);
    }
  }
  int bpos = base_b + before_b + incl_b - mine_b;
  for (int p = 0; p < PER && recb; ++p) {
    if (recb & (1ull << p)) {
      mrows_b[bpos++] = c0 + (long long)p * 256 + tid;
      recb &= ~(1ull << p);
    }
  }
}

// the gap records of the calling thread's next filter / screen launches (null
// rec: off) - set by the engine before each certified E-step
struct MultiRec {
  GapRec* rec = nullptr;
  int* mflag = nullptr;            // the per-row multi flag (2 + record base)
  int it_now = 0, it_lo = 0;       // records with base in [it_lo, it_now - 1] are current
  int ring = 0;                    // shift operands per base iteration b (slot b % ring)
  const _Float16* dsh = nullptr;   // [ring][k][d_pad] fp16 c(now) - c(b)
  const float* dq = nullptr;       // [ring][k][8] their per-centroid terms
  long long dsh_stride = 0;        // halves per ring slot
  long long* mrows_b = nullptr;    // list B (rows with a current record)
  int* count_b = nullptr;
  int* n_done = nullptr;           // list-B rows the gap screen resolved
};
static thread_local MultiRec g_mrec;
// second overflow list of the dense-row 3-pass kernel (null: off) - the
// calling thread's next certified E-steps
struct Ovf2 {
  void* rows = nullptr;   // int64 [cap]
  int* count = nullptr;   // int32 [1], zeroed with the E-step's counters
};
static thread_local Ovf2 g_ovf2;
extern "C" int sq_set_overflow2(void* rows, void* count) {
  g_ovf2.rows = rows;
  g_ovf2.count = (int*)count;
  return (rows != nullptr) != (count != nullptr) ? (int)hipErrorInvalidValue : 0;
}
extern "C" int sq_multi_records(void* rec, void* mflag, int it_now, int it_lo, int ring,
                                const void* dsh, const void* dq, long long dsh_stride,
                                void* mrows_b, void* count_b, void* n_done) {
  g_mrec.rec = (GapRec*)rec;
  g_mrec.mflag = (int*)mflag;
  g_mrec.it_now = it_now;
  g_mrec.it_lo = it_lo;
  g_mrec.ring = ring;
  g_mrec.dsh = (const _Float16*)dsh;
  g_mrec.dq = (const float*)dq;
  g_mrec.dsh_stride = dsh_stride;
  g_mrec.mrows_b = (long long*)mrows_b;
  g_mrec.count_b = (int*)count_b;
  g_mrec.n_done = (int*)n_done;
  return (rec && (it_now < 1 || it_lo < 1 || it_lo > it_now || ring < 2 || ring > 16 || !mflag ||
                  !dsh || !dq || !mrows_b || !count_b))
             ? (int)hipErrorInvalidValue
             : 0;
}

// rcount and multi_count must be zero on entry (the caller clears them with
// the E-step's other counters in one fill).
extern "C" int sq_bounds_filter(const void* labels, void* ub, void* lb, const void* shift,
                                const void* smax, long long n, double delta, void* rlist,
                                void* rcount, const void* mflag, void* mrows, void* multi_count,
                                const void* cc, const void* fidx, int nf, int k, void* stream,
                                void* corr, void* rec_count) {
  if (n <= 0) return 0;
  if (!mflag || !mrows || !multi_count) return (int)hipErrorInvalidValue;
  if (nf < 0 || nf > 64 || (nf > 0 && (!cc || !fidx || k <= nf))) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  // rows per thread: the smallest PER whose grid fits ONE resident round
  // (workgroups per CU from the occupancy query x CUs): a second, mostly
  // empty round doubled the kernel at 10M rows (2442 blocks of 4096)
  static long long resident = 0;
  if (resident == 0) {
    int dev = 0, cus = 0, per_cu = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)bounds_filter_kernel<32>,
                                                 256, 0);
    resident = (long long)(cus > 0 ? cus : 256) * (per_cu > 0 ? per_cu : 4);
  }
  auto pick = [&](int per) { return (n + per * 256LL - 1) / (per * 256LL) <= resident; };
  static const int per_env = [] {   // SQ_BF_PER: a fixed PER (measurements)
    const char* e = getenv("SQ_BF_PER");
    return e ? atoi(e) : 0;
  }();
  // (at least 8: the per-workgroup setup and list atomics dominate 4 rows
  // per thread - measured 38.8 vs 28.4 us on a 1.25M-row shard)
  int per = pick(8) ? 8 : pick(16) ? 16 : pick(20) ? 20 : pick(32) ? 32 : 64;
  if (per_env == 4 || per_env == 8 || per_env == 16 || per_env == 20 || per_env == 32 ||
      per_env == 64)
    per = per_env;
  const long long blocks = (n + per * 256LL - 1) / (per * 256LL);
  auto kern = per == 4 ? bounds_filter_kernel<4> : per == 8 ? bounds_filter_kernel<8>
            : per == 16 ? bounds_filter_kernel<16> : per == 20 ? bounds_filter_kernel<20>
            : per == 32 ? bounds_filter_kernel<32> : bounds_filter_kernel<64>;
  hipLaunchKernelGGL(kern, dim3((unsigned)blocks),
                     dim3(256), 0, st, (const int*)labels, (float*)ub, (float*)lb,
                     (const double*)shift, (const double*)smax, n, delta, (long long*)rlist,
                     (int*)rcount, (const int*)mflag, (long long*)mrows, (int*)multi_count,
                     (const float*)cc, (const int*)fidx, nf, k,
                     g_mrec.rec ? 1 : 0, g_mrec.it_now, g_mrec.it_lo, g_mrec.mrows_b,
                     g_mrec.count_b, (float*)corr, (int*)rec_count);
  return (int)hipGetLastError();
}

// The nf fastest centroids of an update: F = top-nf of the shifts by rank
// (rank of c = #{j : s_j > s_c, or s_j = s_c and j < c}: unique, ties to the
// lower index).  One WAVE per centroid c: each lane counts its k / 64 strided
// shifts (coalesced, L2-resident), one wave sum - k / 4 workgroups instead of
// one thread walking all k shifts (29.6 -> ~4 us at k = 1024).
// With shift_sq != null the shifts are first made from the squared
// per-centroid shifts of the finalize, s = sqrt(s^2) (1 + 1e-12) rounded up
// (the Hamerly update's margin), and written to shift (the fused form of the
// former sqrt / scale launches); every lane recomputes the same values.
// idx[rank] = c for rank < nf, smax_rest = the shift of rank nf.
__global__ void __launch_bounds__(256) fast_select_kernel(double* __restrict__ shift,
                                                          const double* __restrict__ shift_sq,
                                                          int k, int nf, int* __restrict__ idx,
                                                          double* __restrict__ smax_rest) {
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= k) return;
  auto sv = [&](int j) -> double {
    return shift_sq ? sqrt(shift_sq[j]) * (1.0 + 1e-12) : shift[j];
  };
  const double v = sv(c);
  int rank = 0;
  for (int j = lane; j < k; j += 64) {
    const double u = sv(j);
    rank += (u > v || (u == v && j < c)) ? 1 : 0;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) rank += __shfl_xor(rank, o, 64);
  if (lane == 0) {
    if (shift_sq) shift[c] = v;
    if (rank < nf) idx[rank] = c;
    if (rank == nf) *smax_rest = v > 0.0 ? v : 0.0;
  }
}

// cc[j][f] = |c_j - c_idx[f]| (fp64 from the fp32 centroids, rounded down to
// fp32), +inf for j = idx[f]; cc[k nf + j] = min_f cc[j][f].  One workgroup
// per centroid j, wave w takes f = w, w + 4, ...
__global__ void __launch_bounds__(256) fast_cc_kernel(const float* __restrict__ C, int k, int d,
                                                      const int* __restrict__ idx, int nf,
                                                      float* __restrict__ cc) {
  __shared__ float wmin[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int j = blockIdx.x;
  float m = __builtin_inff();
  for (int f = w; f < nf; f += 4) {
    const int jf = idx[f];
    double s = 0.0;
    for (int c = lane; c < d; c += 64) {
      const double e = (double)C[(size_t)j * d + c] - (double)C[(size_t)jf * d + c];
      s = fma(e, e, s);
    }
    s = wave_sum(s);
    const float v = j == jf ? __builtin_inff() : (float)sqrt(s) * (1.0f - 0x1p-20f) - 1e-30f;
    if (lane == 0) cc[(size_t)j * nf + f] = v;
    m = fminf(m, v);
  }
  if (lane == 0) wmin[w] = m;
  __syncthreads();
  if (threadIdx.x == 0)
    cc[(size_t)k * nf + j] = fminf(fminf(wmin[0], wmin[1]), fminf(wmin[2], wmin[3]));
}

extern "C" int sq_fast_centroids(void* shift, const void* shift_sq, const void* C, int k, int d,
                                 int nf, void* idx, void* smax_rest, void* cc, void* stream) {
  if (k <= 0) return 0;
  if (nf < 0 || nf > 64 || nf >= k) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(fast_select_kernel, dim3((unsigned)((k + 3) / 4)), dim3(256), 0, st,
                     (double*)shift, (const double*)shift_sq, k, nf, (int*)idx,
                     (double*)smax_rest);
  if (nf > 0)
    hipLaunchKernelGGL(fast_cc_kernel, dim3((unsigned)k), dim3(256), 0, st, (const float*)C, k, d,
                       (const int*)idx, nf, (float*)cc);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// fp64 re-check of the multi-candidate rows listed by estep_x64_kernel: the
// candidates' distances sum_f (x_f - c_f)^2 in fp64 (scipy cdist's formula,
// the reference's ``_dmeans.py:736-737``), then the delta-band rule exactly
// as band.h: min, members {d <= min + delta}, the member of kappa rank
// r = band_rank(u, |band|), kappa(j) = (j mod 32, j div 32).  A wave takes 4
// list rows (16 lanes each, 16 features per lane at d = 256) and keeps its
// row in registers across that row's candidates (two at a time); lane t of a
// row's group then holds candidate t, so min, band and kappa ranks are
// group-wide shuffles rather than per-lane O(16^2) loops.
template <int DX>
__global__ void __launch_bounds__(256) recheck_rows_kernel(
    const float* __restrict__ X, const float* __restrict__ Cm, const long long* __restrict__ mrows,
    const int* __restrict__ mcand, const int* __restrict__ multi_count, int* __restrict__ labels,
    float* __restrict__ mind, long long cap, double delta, RngKey key, long long row_offset,
    float* __restrict__ corr, float* __restrict__ ub, const unsigned char* __restrict__ xflag) {
  constexpr int LPR = 16;                  // lanes per row
  constexpr int FPL = DX / LPR;            // features per lane (DX >= 64) or fewer
  constexpr int F4 = FPL >= 4 ? FPL / 4 : 1;
  const int lane = threadIdx.x & 63;
  const int sub = lane & (LPR - 1);
  const int gbase = lane & ~(LPR - 1);
  const unsigned long long gmask = 0xffffull << gbase;
  const long long cnt = min((long long)*multi_count, cap);
  const long long gw = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const long long nw = ((long long)gridDim.x * blockDim.x) >> 6;
  auto cdist = [&](const float4 (&xv)[F4], int j) -> double {
    const float* cr = Cm + (size_t)j * DX;
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < F4; ++q) {
      if (4 * (q * LPR + sub) < DX) {   // group-contiguous float4s: coalesced
        const float4 cv = *reinterpret_cast<const float4*>(cr + 4 * (q * LPR + sub));
        const double e0 = (double)xv[q].x - (double)cv.x, e1 = (double)xv[q].y - (double)cv.y;
        const double e2 = (double)xv[q].z - (double)cv.z, e3 = (double)xv[q].w - (double)cv.w;
        s = fma(e0, e0, fma(e1, e1, fma(e2, e2, fma(e3, e3, s))));
      }
    }
    return s;
  };
  auto process = [&](long long e, bool live) {
    const long long g = live ? mrows[e] : 0;
    const int* mc = mcand + g * (kMaxCand + 1);
    const int c_r = live ? mc[0] : 0;
    // lane sub of the row's group holds candidate sub (index, distance)
    const bool mine = sub < c_r;
    const int myj = mine ? mc[1 + sub] : 0;
    float4 xv[F4];
    const float* xr = X + (size_t)g * DX;
#pragma unroll
    for (int q = 0; q < F4; ++q)
      xv[q] = (4 * (q * LPR + sub) < DX)
                  ? *reinterpret_cast<const float4*>(xr + 4 * (q * LPR + sub))
                  : make_float4(0.f, 0.f, 0.f, 0.f);
    int cmax = c_r;
#pragma unroll
    for (int o = 16; o < 64; o <<= 1) cmax = max(cmax, __shfl_xor(cmax, o, 64));
    double dme = __builtin_inf();
    // candidates in pairs: both centroid fragments in flight at once
    for (int c = 0; c < cmax; c += 2) {            // wave-uniform trip count
      const int j0 = __shfl(myj, gbase + c, 64);
      const int j1 = __shfl(myj, gbase + min(c + 1, LPR - 1), 64);
      double s0 = cdist(xv, c < c_r ? j0 : 0);
      double s1 = cdist(xv, c + 1 < c_r ? j1 : 0);
#pragma unroll
      for (int o = 1; o < LPR; o <<= 1) {
        s0 += __shfl_xor(s0, o, 64);
        s1 += __shfl_xor(s1, o, 64);
      }
      if (sub == c) dme = s0;
      if (sub == c + 1) dme = s1;
    }
    // delta-band over the group's lanes (band.h's rule): min, members
    // {d <= min + delta}, the member of kappa rank r = band_rank(u, |band|)
    double dmin = mine ? dme : __builtin_inf();
#pragma unroll
    for (int o = 1; o < LPR; o <<= 1) dmin = fmin(dmin, __shfl_xor(dmin, o, 64));
    const bool inb = mine && dme <= dmin + delta;
    const unsigned long long bm = __ballot(inb) & gmask;
    const int b = __popcll(bm);
    const int kme = inb ? (((myj & 31) << 20) | (myj >> 5)) : 0x7fffffff;
    int rank = 0;
#pragma unroll
    for (int t = 0; t < LPR; ++t) rank += __shfl(kme, gbase + t, 64) < kme ? 1 : 0;
    const int r = b > 0 ? band_rank(band_u(key, row_offset + g), b) : 0;
    const unsigned long long pm = __ballot(inb && rank == r) & gmask;
    const int plane = pm ? __ffsll((long long)pm) - 1 : gbase;
    const int pick = __shfl(myj, plane, 64);
    const double dpick = __shfl(dme, plane, 64);
    if (live && sub == 0) {
      labels[g] = pick;
      mind[g] = (float)dmin;
      if (corr) corr[g] = (float)(dmin - dpick);
      // Hamerly upper bound of a multi row: the distance to its LABEL (the
      // filter moves it by the label's shift)
      if (ub) ub[g] = (float)sqrt(dpick) * (1.0f + 0x1p-20f);
    }
  };
  if (!xflag) {   // contiguous slice per wave (page locality, see the screen)
    const long long per = ((cnt + nw - 1) / nw + 3) / 4 * 4;
    const long long e_end = min(cnt, (gw + 1) * per);
    for (long long base = gw * per; base < e_end; base += 4) {
      const long long e = base + (lane >> 4);
      process(e, e < e_end);
    }
    return;
  }
  // flagged entries only (the fp32 screen's leftovers): a wave scans 64
  // list entries, its 4 row groups take the flagged ones 4 at a time
  const int q = lane >> 4;
  for (long long base = gw * 64; base < cnt; base += nw * 64) {
    const long long el = base + lane;
    unsigned long long m = __ballot(el < cnt && xflag[el] != 0);
    while (m) {   // wave-uniform
      unsigned long long mm = m;
      for (int t = 0; t < q; ++t) mm &= mm - 1ull;
      const bool live = mm != 0ull;
      process(live ? base + (__ffsll((long long)mm) - 1) : 0, live);
      for (int t = 0; t < 4; ++t) m &= m - 1ull;
    }
  }
}

// fp32 screen of the multi-candidate rows (Lloyd steps with the incremental
// M-step, where only labels, the label-vs-min corrections and the Hamerly
// upper bounds are consumed): the candidates' distances in fp32 (the same
// sum of squared differences; 20 roundings -> |D32 - D| <= 2^-18 D32), then
// each candidate's band membership is CERTAIN when
//   in : D32_c + B_c <= min_j (D32_j - B_j) + delta,
//   out: D32_c - B_c >  min_j (D32_j + B_j) + delta.
// A row whose every candidate is certainly in or out of the band is done
// here: band {argmin} -> label = argmin, corr = 0 (the memset value); a wider
// band -> the member of kappa rank band_rank(u, |band|) (the fp64 pass's rule
// and Philox word: the same label) with corr = min - label distance from the
// fp32 distances; ub from D32 + B (mind is not needed by the incremental
// steps that run the screen).  Rows with an uncertain member are flagged for
// recheck_rows_kernel (fp64).
// The kernel is bound by memory transactions per row (the list entry, the
// per-row candidate record, the row, the scattered label / bound stores),
// not by arithmetic: loads are software-pipelined across steps.
#ifndef SQ_SCREEN_LPR
#define SQ_SCREEN_LPR 16
#endif
template <int DX, int LPR, bool UB>
__global__ void __launch_bounds__(256) recheck_fast_kernel(
    const float* __restrict__ X, const float* __restrict__ Cm, const long long* __restrict__ mrows,
    const int* __restrict__ mcand, const int* __restrict__ multi_count, int* __restrict__ labels,
    float* __restrict__ mind, long long cap, double delta, float* __restrict__ ub,
    unsigned char* __restrict__ xflag, int il, GapRec* __restrict__ rec, int* __restrict__ rec_it,
    int it_now, RngKey key, long long row_offset, float* __restrict__ corr) {
  constexpr int RPW = 64 / LPR;   // rows per wave step
  constexpr int FPL = DX / LPR;
  constexpr int F4 = FPL >= 4 ? FPL / 4 : 1;
  const int lane = threadIdx.x & 63;
  const int sub = lane & (LPR - 1);
  const int gbase = lane & ~(LPR - 1);
  const long long cnt = min((long long)*multi_count, cap);
  const long long gw = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const long long nw = ((long long)gridDim.x * blockDim.x) >> 6;
  // group-contiguous float4 slices of a row: coalesced
  auto ldrow = [&](const float* r, float4 (&v)[F4]) {
#pragma unroll
    for (int q = 0; q < F4; ++q)
      v[q] = (4 * (q * LPR + sub) < DX) ? *reinterpret_cast<const float4*>(r + 4 * (q * LPR + sub))
                                        : make_float4(0.f, 0.f, 0.f, 0.f);
  };
  auto sqd = [&](const float4 (&xv)[F4], const float4 (&cv)[F4]) -> float {
    float s = 0.0f;
#pragma unroll
    for (int q = 0; q < F4; ++q) {
      const float e0 = xv[q].x - cv[q].x, e1 = xv[q].y - cv[q].y;
      const float e2 = xv[q].z - cv[q].z, e3 = xv[q].w - cv[q].w;
      s = fmaf(e0, e0, fmaf(e1, e1, fmaf(e2, e2, fmaf(e3, e3, s))));
    }
    return s;
  };
  // each wave walks a CONTIGUOUS slice of the list (rows in ascending
  // order within a 4K-row chunk): few pages of X live per CU at a time.
  // Three-stage software pipeline over the wave's steps (RPW rows each) -
  // the list entry of step s + 2, the candidate list and the row of step
  // s + 1 and the first two candidate centroids of step s + 1 are in flight
  // while step s computes (the chain list -> candidates -> centroid rows was
  // three dependent memory latencies per step)
  // step s of a wave covers RPW list entries: a contiguous slice per wave
  // (il = 0), or interleaved - step s of every wave inside one window of
  // nw * RPW entries (il = 1: the rows in flight chip-wide stay within a few
  // MB of X and of the candidate records, TLB locality)
  const long long per = ((cnt + nw - 1) / nw + RPW - 1) / RPW * RPW;
  const long long e_beg = gw * per;
  const long long lim = il ? cnt : min(cnt, (gw + 1) * per);
  const long long nsteps = il ? (gw * RPW < cnt ? (cnt - gw * RPW + nw * RPW - 1) / (nw * RPW) : 0)
                              : (e_beg < lim ? (lim - e_beg + RPW - 1) / RPW : 0);
  if (nsteps <= 0) return;
  auto entry = [&](long long st) -> long long {
    const long long e = (il ? (st * nw + gw) * RPW : e_beg + st * RPW) + lane / LPR;
    return e < lim ? e : lim - 1;
  };
  // every load below is unconditional (clamped to a valid entry / record;
  // the values are masked afterwards): a load under a data-dependent branch
  // makes the compiler drain vmcnt(0) - the whole pipeline - before it
  // entries past the wave's slice mirror its last entry: the same inputs give
  // the same results, so the stores below can be unconditional (identical
  // values to identical addresses) - no exec-masked store, exact vmcnt counts
  auto load_g = [&](long long st) -> long long { return mrows[entry(st)]; };
  struct Rw {
    long long g;
    int c_r, myj, j0, j1;   // raw record words: masked by c_r at use
  };
  auto load_c = [&](long long g) -> Rw {
    Rw r;
    r.g = g;
    const int* mc = mcand + (g >= 0 ? g : 0) * (kMaxCand + 1);
    r.c_r = mc[0];
    r.myj = mc[1 + sub];
    r.j0 = mc[1];
    r.j1 = mc[2];
    return r;
  };
  auto fix = [&](Rw& r) {   // once the record has landed
    r.c_r = r.g >= 0 ? min(max(r.c_r, 0), kMaxCand) : 0;
    r.myj = sub < r.c_r ? r.myj : 0;
    r.j0 = r.c_r > 0 ? r.j0 : 0;
    r.j1 = r.c_r > 1 ? r.j1 : r.j0;
  };
  // two register sets (A: the step being computed, B: the next step's loads)
  // swap roles every step; the loop is unrolled by two so no register copy
  // (a copy of a loaded register waits for its load) sits between steps
  float4 xA[F4], c0A[F4], c1A[F4], xB[F4], c0B[F4], c1B[F4];
  // list entries run two steps ahead of the candidate records: the entry a
  // step's record load needs was issued a whole step of unconditional loads
  // earlier, so its vmcnt wait does not cover the previous step's
  // (conditional) stores
  long long g2 = load_g(1), g3 = load_g(2);
  Rw rA = load_c(load_g(0)), rB;
  fix(rA);
  ldrow(X + (size_t)(rA.g >= 0 ? rA.g : 0) * DX, xA);
  ldrow(Cm + (size_t)rA.j0 * DX, c0A);
  ldrow(Cm + (size_t)rA.j1 * DX, c1A);
  auto step = [&](long long st, Rw& cur, const float4 (&xv)[F4], const float4 (&c0)[F4],
                  const float4 (&c1)[F4], Rw& nxt, float4 (&xn_)[F4], float4 (&c0n)[F4],
                  float4 (&c1n)[F4]) {
    // stage 1 / 2 for the next steps
    const long long g4 = load_g(st + 3);
    nxt = load_c(g2);
    ldrow(X + (size_t)(nxt.g >= 0 ? nxt.g : 0) * DX, xn_);
    // ---- step base: the candidates' fp32 squared distances
    const long long e = entry(st);
    const bool live = true;
    const long long g = cur.g;
    const int c_r = cur.c_r;
    const bool fits = c_r <= LPR;   // one candidate per lane of the group
    const bool mine = sub < c_r;
    int cmax = c_r;
#pragma unroll
    for (int o = LPR; o < 64; o <<= 1) cmax = max(cmax, __shfl_xor(cmax, o, 64));
    cmax = min(cmax, LPR);
    float s0 = sqd(xv, c0), s1 = sqd(xv, c1);
#pragma unroll
    for (int o = 1; o < LPR; o <<= 1) {
      s0 += __shfl_xor(s0, o, 64);
      s1 += __shfl_xor(s1, o, 64);
    }
    float dme = sub == 0 ? s0 : (sub == 1 ? s1 : __builtin_inff());
    for (int c = 2; c < cmax; c += 2) {   // rows with more than two candidates (rare)
      const int ja = __shfl(cur.myj, gbase + c, 64);
      const int jb = __shfl(cur.myj, gbase + min(c + 1, LPR - 1), 64);
      float4 ca[F4], cb[F4];
      ldrow(Cm + (size_t)(c < c_r ? ja : 0) * DX, ca);
      ldrow(Cm + (size_t)(c + 1 < c_r ? jb : 0) * DX, cb);
      float sa = sqd(xv, ca), sb = sqd(xv, cb);
#pragma unroll
      for (int o = 1; o < LPR; o <<= 1) {
        sa += __shfl_xor(sa, o, 64);
        sb += __shfl_xor(sb, o, 64);
      }
      if (sub == c) dme = sa;
      if (sub == c + 1) dme = sb;
    }
    // fp32 interval [lo, hi] around the exact D: the distance bound is
    // 2^-18 D; 2^-16 D + 2^-20 delta also absorbs the fp32 roundings of these
    // products and of the (min + delta) sums below (each <= 2^-24 of a
    // magnitude <= D + delta)
    const float dlt = (float)delta;
    const float slack = dme * 0x1p-16f + dlt * 0x1p-20f + 1e-30f;
    const float lo = mine ? dme - slack : __builtin_inff();
    const float hi = mine ? dme + slack : __builtin_inff();
    float minlo = lo, minhi = hi;
#pragma unroll
    for (int o = 1; o < LPR; o <<= 1) {
      minlo = fminf(minlo, __shfl_xor(minlo, o, 64));
      minhi = fminf(minhi, __shfl_xor(minhi, o, 64));
    }
    const bool cin = mine && hi <= minlo + dlt;
    const bool cout = mine && lo > minhi + dlt;
    const unsigned long long gmask = ((1ull << LPR) - 1ull) << gbase;
    const unsigned long long inm = __ballot(cin) & gmask;
    const bool unsure = !fits || (__ballot(mine && !cin && !cout) & gmask) != 0;
    // every candidate certainly in or out: the band is known, and so is the
    // label - the member of kappa rank band_rank(u, |band|) (recheck_rows'
    // rule, the same Philox word); a wider band also needs its correction
    // min - label distance (fp32 distances here, fp64 in recheck_rows)
    const int bsz = __popcll(inm);
    const bool done_any = live && !unsure && bsz >= 1;
    const bool done = done_any && bsz == 1;   // band {argmin}
    int plane = inm ? __ffsll((long long)inm) - 1 : gbase;
    const bool wide = done_any && bsz >= 2;
    float dmin_w = 0.0f;
    if (__ballot(wide)) {   // wave-uniform
      const int kme = cin ? (((cur.myj & 31) << 20) | (cur.myj >> 5)) : 0x7fffffff;
      int rank = 0;
#pragma unroll
      for (int t = 0; t < LPR; ++t) rank += __shfl(kme, gbase + t, 64) < kme ? 1 : 0;
      const int r = band_rank(band_u(key, row_offset + g), bsz > 0 ? bsz : 1);
      const unsigned long long pm = __ballot(cin && rank == r) & gmask;
      if (wide && pm) plane = __ffsll((long long)pm) - 1;
      dmin_w = mine ? dme : __builtin_inff();
#pragma unroll
      for (int o = 1; o < LPR; o <<= 1) dmin_w = fminf(dmin_w, __shfl_xor(dmin_w, o, 64));
    }
    const int pick = __shfl(cur.myj, plane, 64);
    const float hpick = __shfl(hi, plane, 64);
    const float dpick = __shfl(dme, plane, 64);
    // the smallest lower bound of the OTHER candidates (the row's record)
    float lo_o = (mine && lane != plane) ? lo : __builtin_inff();
#pragma unroll
    for (int o = 1; o < LPR; o <<= 1) lo_o = fminf(lo_o, __shfl_xor(lo_o, o, 64));
    fix(nxt);
    // stage 3 for the next step (its first two candidate centroids) BEFORE
    // this step's stores: vmcnt retires in issue order, so a load issued
    // after the scattered stores would make the next step wait for them
    ldrow(Cm + (size_t)nxt.j0 * DX, c0n);
    ldrow(Cm + (size_t)nxt.j1 * DX, c1n);
    __builtin_amdgcn_sched_barrier(0);
    // every lane of the group stores its row's values unconditionally: a row
    // that is not done gets placeholder values that recheck_rows_kernel
    // overwrites (it rewrites labels / mind / ub of every flagged row).  No
    // mind store: the screen runs only in incremental steps, whose inertia
    // comes from the cluster statistics and the corrections (each scattered
    // 4-B store is one more memory transaction per row - the kernel's bound)
    labels[g] = pick;
    if constexpr (UB) ub[g] = sqrtf(hpick) * (1.0f + 0x1p-20f);
    if (wide && sub == 0 && corr) corr[g] = dmin_w - dpick;
    // the rest -> flagged for the fp64 pass (a per-entry byte: no atomics)
    xflag[e] = done_any ? 0 : 1;
    // a row whose band is certainly {argmin}: its record (distance bounds to
    // the argmin and to the nearest other candidate, sqrt domain) lets later
    // iterations certify the same band from the centroid shifts alone
    // (bounds_filter_kernel) without reading the row
    if (rec) {
      // the row's gap record (lanes 0..7 of the group: one word each; the
      // upper half of the group repeats them - identical stores): gaps from
      // the fp32 distances, each within slack_c + slack_pick (+ the rounding
      // of the difference)
      const float dpl = __shfl(dme, plane, 64), spl = __shfl(slack, plane, 64);
      const float gc = mine ? dme - dpl : 0.0f;
      float ge = mine ? slack + spl + fabsf(gc) * 0x1p-23f : 0.0f;
#pragma unroll
      for (int o = 1; o < LPR; o <<= 1) ge = fmaxf(ge, __shfl_xor(ge, o, 64));
      const int w = sub & 7;
      const float gw = __shfl(gc, gbase + min(max(w - 2, 0), LPR - 1), 64);
      const float v = w == 0 ? dpl : (w == 1 ? ge : gw);
      // candidate ids (slots past c_r repeat candidate 0)
      const unsigned i0 = (unsigned)__shfl(cur.myj, gbase, 64) & 0x3FFFu;
      const unsigned i1 = (unsigned)__shfl(cur.myj, gbase + 1, 64) & 0x3FFFu;
      const unsigned i2 = (unsigned)__shfl(cur.myj, gbase + 2, 64) & 0x3FFFu;
      const unsigned i3 = (unsigned)__shfl(cur.myj, gbase + 3, 64) & 0x3FFFu;
      const unsigned cm1 = (unsigned)min(max(c_r, 1), kGapCand) - 1u;
      const unsigned id0 = i0 | ((unsigned)(plane - gbase) & 3u) << 14 |
                           (c_r > 1 ? i1 : i0) << 16 | cm1 << 30;
      const unsigned id1 = (c_r > 2 ? i2 : i0) | (c_r > 3 ? i3 : i0) << 16;
      float* rw = reinterpret_cast<float*>(rec + g) + w;
      if (w < 6) *rw = v;
      else *reinterpret_cast<unsigned*>(rw) = w == 6 ? id0 : id1;
      if (sub == 0) rec_it[g] = (done && c_r <= kGapCand) ? it_now + 2 : 1;
    }
    __builtin_amdgcn_sched_barrier(0);
    g2 = g3;
    g3 = g4;
  };
  for (long long st = 0; st < nsteps; st += 2) {
    step(st, rA, xA, c0A, c1A, rB, xB, c0B, c1B);
    if (st + 1 >= nsteps) break;
    step(st + 1, rB, xB, c0B, c1B, rA, xA, c0A, c1A);
  }
}

// ---------------------------------------------------------------------------
// Gap screen (list B: multi rows whose candidate set is unchanged and whose
// gap record is from the previous iteration).  Between two iterations the
// squared distance to centroid j moves by
//   D_j(t) - D_j(t-1) = -2 x.S_j + q_j,   S_j = c_j(t) - c_j(t-1),
//   q_j = |c_j(t)|^2 - |c_j(t-1)|^2,
// so the record's gaps move by 2 (x.S_a - x.S_c) + q_c - q_a and da by
// -2 x.S_a + q_a.  x.S_j needs the row, but only to the accuracy of a SHIFT:
// the fp16 row (the filter's operand, 512 B at d = 256) against the fp16
// shift operand (shift_operand_kernel) is exact to
//   E_j = ex |S_j| + |x~| (e_j + gam (|S_j| + e_j)),
// ex = |x - x~| <= 2^-11 |x| + sqrt(d) 2^-25 / alpha, e_j = |S_j - S~_j| (exact,
// per centroid), gam the fp32 accumulation of the fp16 products.  The record's
// err grows by 2 (E_a + max_c E_c) + rounding per iteration; a row whose band
// is still certainly {argmin} (every other candidate's gap > delta + 2 err) is
// resolved - label, Hamerly upper bound and a new record - without reading its
// fp32 row or any centroid row.  The rest are appended to the multi list for
// the fp32 screen (which re-records them exactly).
// Layout: a wave takes TWO rows per step (32 lanes each).  The vector
// memory path is the screen's bound, so every load carries distinct data: the
// per-row values (the 8-word record, |x|^2, the candidates' 8-word
// per-centroid terms) come as ONE dword per lane (lane w of a row loads word
// w) and are broadcast with lane shuffles, the list entries of 32 steps come
// in one load; the records are read from the previous iteration's buffer and
// written to the other one.  Three-stage pipeline: a step issues the next
// step's record / |x|^2 words, computes, then issues the next step's fp16 row,
// shift rows and per-centroid words (its record has landed meanwhile).
typedef _Float16 gs_h2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float gs_dot(const uint4 a, const uint4 b, float acc) {
  acc = __builtin_amdgcn_fdot2(__builtin_bit_cast(gs_h2, a.x), __builtin_bit_cast(gs_h2, b.x), acc,
                               false);
  acc = __builtin_amdgcn_fdot2(__builtin_bit_cast(gs_h2, a.y), __builtin_bit_cast(gs_h2, b.y), acc,
                               false);
  acc = __builtin_amdgcn_fdot2(__builtin_bit_cast(gs_h2, a.z), __builtin_bit_cast(gs_h2, b.z), acc,
                               false);
  acc = __builtin_amdgcn_fdot2(__builtin_bit_cast(gs_h2, a.w), __builtin_bit_cast(gs_h2, b.w), acc,
                               false);
  return acc;
}
__device__ __forceinline__ float gs_dot(const uint2 a, const uint2 b, float acc) {
  acc = __builtin_amdgcn_fdot2(__builtin_bit_cast(gs_h2, a.x), __builtin_bit_cast(gs_h2, b.x), acc,
                               false);
  acc = __builtin_amdgcn_fdot2(__builtin_bit_cast(gs_h2, a.y), __builtin_bit_cast(gs_h2, b.y), acc,
                               false);
  return acc;
}
__device__ __forceinline__ uint4 gs_zero(uint4) { return make_uint4(0u, 0u, 0u, 0u); }
template <int CTRL>
__device__ __forceinline__ float gs_dpp_add(float v) {
  return v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF,
                                                         false));
}
__device__ __forceinline__ uint2 gs_zero(uint2) { return make_uint2(0u, 0u); }

template <int DX>
__global__ void __launch_bounds__(256) gap_screen_kernel(
    const _Float16* __restrict__ Xh, const float* __restrict__ xn,
    const long long* __restrict__ mrows_b, const int* __restrict__ count_b,
    const _Float16* __restrict__ dsh, long long dsh_stride, const float* __restrict__ dq,
    long long dq_stride, float inv_alpha, float delta, int* __restrict__ labels,
    GapRec* __restrict__ rec, int* __restrict__ mflag, int it_now, int ring, int rebase_age,
    long long* __restrict__ mrows, int* __restrict__ multi_count, long long cap,
    int* __restrict__ n_done) {
  constexpr int LPR = 32;
  using VT = typename std::conditional<DX % 256 == 0, uint4, uint2>::type;
  constexpr int HV = (int)sizeof(VT) / 2;   // halves per vector
  constexpr int V = DX / (LPR * HV);        // vectors per lane per row
  static_assert(DX % 128 == 0 && V >= 1, "gap screen: d_pad multiple of 128");
  const int lane = threadIdx.x & 63;
  const int sub = lane & (LPR - 1);
  const bool hi = lane >= LPR;
  const long long cnt = min((long long)*count_b, cap);
  const long long gw = (long long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const long long nw = (long long)gridDim.x * (blockDim.x >> 6);
  // a wave owns blocks of 64 list entries (lane r: entry r of the block)
  const long long nblk = (cnt + 63) / 64;
  const float sub_err = sqrtf((float)DX) * 0x1p-25f * inv_alpha;
  constexpr float gam = (float)(DX + 16) * 0x1p-24f;
  uint32_t done_cnt = 0;
  auto rl = [](int v, int l) -> int { return __builtin_amdgcn_readlane(v, l); };
  auto rlf = [](float v, int l) -> float {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
  };
  for (long long blk = gw; blk < nblk; blk += nw) {
    // ---- the lane's own row: entry, record, |x|^2, its candidates' terms
    const long long e = blk * 64 + lane;
    const bool live = e < cnt;
    const long long g = mrows_b[live ? e : cnt - 1];
    const int base_it = mflag[g] - 2;   // the record's base iteration (filter: current)
    const int rslot = base_it % ring, age = it_now - base_it;
    const float4* rp = reinterpret_cast<const float4*>(rec + g);
    const float4 r0 = rp[0], r1 = rp[1];
    const float xq = xn[g];
    const unsigned id0 = __float_as_uint(r1.z), id1 = __float_as_uint(r1.w);
    const int c_r = (int)(id0 >> 30) + 1, slot = (int)((id0 >> 14) & 3u);
    int jc[kGapCand];
    jc[0] = (int)(id0 & 0x3FFFu);
    jc[1] = (int)((id0 >> 16) & 0x3FFFu);
    jc[2] = (int)(id1 & 0x3FFFu);
    jc[3] = (int)((id1 >> 16) & 0x3FFFu);
    const float* dqs = dq + (size_t)rslot * dq_stride;
    float4 d0[kGapCand];
    float inv[kGapCand];
#pragma unroll
    for (int c = 0; c < kGapCand; ++c) {
      d0[c] = reinterpret_cast<const float4*>(dqs)[2 * jc[c]];
      inv[c] = dqs[8 * jc[c] + 4];
    }
    // ---- x.S for every row of the block: 32 passes of two rows (32 lanes
    // per row), the fp16 row and its candidates' shift rows double-buffered;
    // each pass's sums land in the owning lanes (v_writelane)
    float y[kGapCand] = {0.0f, 0.0f, 0.0f, 0.0f};
    constexpr int NB = 4;   // passes in flight
    VT xv[NB][V], sv[NB][kGapCand][V];
    int pcm[NB];   // the pass's widest row (candidate loads past it skipped)
    auto issue = [&](int p, int b) {
      const int ra = 2 * p, rb = 2 * p + 1;
      const long long ga = ((long long)rl((int)(g >> 32), ra) << 32) | (unsigned)rl((int)g, ra);
      const long long gb = ((long long)rl((int)(g >> 32), rb) << 32) | (unsigned)rl((int)g, rb);
      const long long gm = hi ? gb : ga;
      const VT* xr = reinterpret_cast<const VT*>(Xh + (size_t)gm * DX);
#pragma unroll
      for (int q = 0; q < V; ++q) xv[b][q] = xr[q * LPR + sub];
      const int sa = rl(rslot, ra), sb = rl(rslot, rb);
      const _Float16* ds = dsh + (size_t)(hi ? sb : sa) * dsh_stride;
      pcm[b] = max(rl(c_r, ra), rl(c_r, rb));
#pragma unroll
      for (int c = 0; c < kGapCand; ++c) {
        if (c < 2 || c < pcm[b]) {   // wave-uniform
          const int j = hi ? rl(jc[c], rb) : rl(jc[c], ra);
          const VT* sr = reinterpret_cast<const VT*>(ds + (size_t)j * DX);
#pragma unroll
          for (int q = 0; q < V; ++q) sv[b][c][q] = sr[q * LPR + sub];
        } else {
#pragma unroll
          for (int q = 0; q < V; ++q) sv[b][c][q] = gs_zero(VT{});
        }
      }
    };
    auto consume = [&](int p, int b) {
#pragma unroll
      for (int c = 0; c < kGapCand; ++c) {
        if (c < 2 || c < pcm[b]) {
          float acc = 0.0f;
#pragma unroll
          for (int q = 0; q < V; ++q) acc = gs_dot(xv[b][q], sv[b][c][q], acc);
          acc = gs_dpp_add<0xB1>(acc);    // quad_perm [1,0,3,2]
          acc = gs_dpp_add<0x4E>(acc);    // quad_perm [2,3,0,1]
          acc = gs_dpp_add<0x141>(acc);   // row_half_mirror
          acc = gs_dpp_add<0x140>(acc);   // row_mirror
          const float a = rlf(acc, 0) + rlf(acc, 16), bb = rlf(acc, 32) + rlf(acc, 48);
          y[c] = lane == 2 * p ? a : (lane == 2 * p + 1 ? bb : y[c]);
        }
      }
    };
#pragma unroll
    for (int b = 0; b < NB - 1; ++b) issue(b, b);
#pragma unroll 1
    for (int p = 0; p < 32; p += NB) {
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        if (p + b + NB - 1 < 32) issue(p + b + NB - 1, (b + NB - 1) % NB);
        consume(p + b, b);
      }
    }
    // ---- the lane's own row: move the record, decide
    const float nx = sqrtf(xq) * (1.0f + 0x1p-16f);
    const float ex = 0x1p-11f * nx + sub_err, nxh = nx + ex;
    float yr[kGapCand], E[kGapCand], qv[kGapCand];
#pragma unroll
    for (int c = 0; c < kGapCand; ++c) {
      // dq[j] = {q_j, err(q_j), |S_j| (up), e_j (up)}, inv = 1 / (alpha beta_j)
      yr[c] = y[c] * inv[c];
      E[c] = ex * d0[c].z + nxh * (d0[c].w + gam * (d0[c].z + d0[c].w)) + d0[c].y;
      qv[c] = d0[c].x;
    }
    float ya = 0.0f, Ea = 0.0f, qa = 0.0f;
#pragma unroll
    for (int c = 0; c < kGapCand; ++c)
      if (c == slot) {
        ya = yr[c];
        Ea = E[c];
        qa = qv[c];
      }
    const float gold[kGapCand] = {r0.z, r0.w, r1.x, r1.y};
    float gn[kGapCand], gmax = 0.0f, Emax = 0.0f, ymax = fabsf(ya), qmax = fabsf(qa);
#pragma unroll
    for (int c = 0; c < kGapCand; ++c) {
      const bool in = c < c_r;
      gn[c] = in ? (c == slot ? 0.0f : gold[c] + 2.0f * (ya - yr[c]) + (qv[c] - qa))
                 : __builtin_inff();
      if (in) {
        gmax = fmaxf(gmax, fabsf(gold[c]));
        Emax = fmaxf(Emax, E[c]);
        ymax = fmaxf(ymax, fabsf(yr[c]));
        qmax = fmaxf(qmax, fabsf(qv[c]));
      }
    }
    const float da = r0.x - 2.0f * ya + qa;
    // propagated error: the record's bound, the x.S estimates (+ the q terms'
    // bounds) of the argmin and the worst other candidate, and <= 3 fp32
    // roundings of sums bounded by |g| + 4 max|y| + 2 max|q| (or |da| + ...)
    float err = r0.y + 2.0f * (Ea + Emax) +
                0x1p-22f * (fmaxf(gmax, fabsf(r0.x)) + 4.0f * ymax + 2.0f * qmax);
    err *= 1.0f + 0x1p-20f;
    int m = 0;
    float gm = gn[0];
#pragma unroll
    for (int c = 1; c < kGapCand; ++c)
      if (gn[c] < gm) {
        gm = gn[c];
        m = c;
      }
    // certain: every other candidate more than delta + 2 err above the argmin
    bool done = live && c_r >= 2 && slot < c_r && err < 0.25f * delta + 1.0f;
    float gmx = 0.0f;
#pragma unroll
    for (int c = 0; c < kGapCand; ++c)
      if (c < c_r && c != m) {
        done = done && (gn[c] - gm > delta + 2.0f * err);
        gmx = fmaxf(gmx, gn[c]);
      }
    // a resolved row stores nothing while its label (= the record's argmin
    // slot) stands and its record is young: the record keeps its base and the
    // next iteration moves it by the shifts since then.  A label change or an
    // old base rebases the record on this iteration (err_n covers the moved
    // values; m != slot: both gaps carry err).
    if (done && (m != slot || age >= rebase_age)) {
      const float da_n = da + gm;
      float err_n =
          (m == slot ? err : 2.0f * err) + 0x1p-22f * (gmx + fabsf(da_n) + fabsf(gm));
      err_n *= 1.0f + 0x1p-20f;
      float gr[kGapCand];
#pragma unroll
      for (int c = 0; c < kGapCand; ++c) gr[c] = c < c_r ? gn[c] - gm : 0.0f;
      float4* wp = reinterpret_cast<float4*>(rec + g);
      wp[0] = make_float4(da_n, err_n, gr[0], gr[1]);
      wp[1] = make_float4(gr[2], gr[3],
                          __uint_as_float((id0 & ~(3u << 14)) | (unsigned)m << 14),
                          __uint_as_float(id1));
      if (m != slot) labels[g] = jc[0] * (m == 0) + jc[1] * (m == 1) + jc[2] * (m == 2) +
                                 jc[3] * (m == 3);
      mflag[g] = it_now + 2;
    }
    // the rest -> the multi list (fp32 screen): one atomic per block
    const bool fwd = live && !done;
    const unsigned long long fm = __ballot(fwd);
    if (fm) {   // wave-uniform
      int fb = 0;
      if (lane == 0) fb = atomicAdd(multi_count, __popcll(fm));
      fb = __shfl(fb, 0, 64);
      const long long se = (long long)fb + __popcll(fm & ((1ull << lane) - 1ull));
      if (fwd && se < cap) mrows[se] = g;
    }
    done_cnt += __popcll(__ballot(done));
  }
  if (n_done && lane == 0 && done_cnt) atomicAdd(n_done, (int)done_cnt);
}

// The gap screen's shift operands after the update c(t) -> c(t+1): for every
// ring slot s whose base iteration b (s = b % ring) can still be current at
// the next E-step (bit s of `valid`), per centroid j (one wave) the
// accumulated shift S_j = c_j(t+1) - c_j(b) in fp64 (exact: fp32 inputs),
// fp16 S~_j = rn(beta_j S_j) with beta_j a power of two putting max|S_j| near
// 2^14, and dq[s][j] = {q_j = |c_j(t+1)|^2 - |c_j(b)|^2 (fp32), its error
// bound, |S_j| (rounded up), e_j = |S_j - S~_j / beta_j| (rounded up),
// 1 / (alpha beta_j), 0, 0, 0}.  c(b) comes from the snapshot ring; slot
// `snew` (b = t) takes c(t) itself, which the kernel also snapshots.  Padded
// columns d..d_pad are zero.
__global__ void __launch_bounds__(256) shift_operand_kernel(
    const float* __restrict__ Cprev, const float* __restrict__ Cnew, int ldc, int d, int d_pad,
    int k, double alpha, float* __restrict__ snap, _Float16* __restrict__ dsh,
    float* __restrict__ dq, int snew, unsigned valid) {
  const int lane = threadIdx.x & 63;
  const int j = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int sl = blockIdx.y;
  if (j >= k || !((valid >> sl) & 1u)) return;
  const size_t rs = (size_t)sl * k + j;
  const float* cn = Cnew + (size_t)j * ldc;
  float* sn = snap + rs * d_pad;
  const bool fresh = sl == snew;
  const float* co = fresh ? Cprev + (size_t)j * ldc : sn;
  double amax = 0.0;
  for (int f = lane; f < d; f += 64) amax = fmax(amax, fabs((double)cn[f] - (double)co[f]));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) amax = fmax(amax, __shfl_xor(amax, o, 64));
  int ex2 = 0;
  if (amax > 0.0) frexp(amax, &ex2);   // amax in [2^(ex2-1), 2^ex2)
  const double beta = amax > 0.0 ? ldexp(1.0, 14 - ex2) : 1.0;
  double q = 0.0, nrm = 0.0, nd = 0.0, e2 = 0.0;
  for (int f = lane; f < d_pad; f += 64) {
    const float a32 = f < d ? co[f] : 0.0f;
    const double a = (double)a32, b = f < d ? (double)cn[f] : 0.0;
    const double sft = b - a;
    const _Float16 h = (_Float16)(float)(beta * sft);
    dsh[rs * d_pad + f] = h;
    if (fresh) sn[f] = a32;
    const double r = sft - (double)h / beta;
    q += sft * (b + a);
    nrm += b * b + a * a;
    nd += sft * sft;
    e2 += r * r;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    q += __shfl_xor(q, o, 64);
    nrm += __shfl_xor(nrm, o, 64);
    nd += __shfl_xor(nd, o, 64);
    e2 += __shfl_xor(e2, o, 64);
  }
  if (lane < 8) {
    const float qf = (float)q;
    float v = 0.0f;
    if (lane == 0) v = qf;
    // fp64 sums (<= 2d roundings of terms <= |c|^2 each) + the fp32 rounding
    if (lane == 1) v = (float)(fabs(q - (double)qf) + 1e-13 * nrm + 1e-30) * (1.0f + 0x1p-20f);
    if (lane == 2) v = (float)sqrt(nd) * (1.0f + 0x1p-20f);
    if (lane == 3) v = (float)(sqrt(e2) * (1.0 + 1e-12)) * (1.0f + 0x1p-20f) + 1e-30f;
    if (lane == 4) v = (float)(1.0 / (alpha * beta));
    dq[rs * 8 + lane] = v;
  }
}

extern "C" int sq_shift_operand(const void* Cprev, const void* Cnew, int ldc, int d, int d_pad,
                                int k, double alpha, void* snap, void* dsh, void* dq, int ring,
                                int snew, unsigned valid, void* stream) {
  if (k <= 0 || !valid) return 0;
  if (d > d_pad || d > ldc || ring < 1 || ring > 16 || snew < 0 || snew >= ring)
    return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(shift_operand_kernel, dim3((unsigned)((k + 3) / 4), (unsigned)ring),
                     dim3(256), 0, (hipStream_t)stream, (const float*)Cprev, (const float*)Cnew,
                     ldc, d, d_pad, k, alpha, (float*)snap, (_Float16*)dsh, (float*)dq, snew,
                     valid);
  return (int)hipGetLastError();
}

// Rows resolved by the 3-pass kernel (dense list): corr = mind - exact fp64
// |x - c_label|^2 (the per-cluster inertia of the incremental M-step counts
// every row at its label's distance; corr brings it back to the min).
__global__ void __launch_bounds__(256) dense_corr_kernel(
    const float* __restrict__ X, const float* __restrict__ Cm, const long long* __restrict__ rows,
    const int* __restrict__ count, const int* __restrict__ labels, const float* __restrict__ mind,
    float* __restrict__ corr, long long cap, int d) {
  // 16 lanes per row, 4 rows per wave in flight (the row -> label -> row
  // data chain is three dependent loads: one row per wave left the grid
  // latency-bound on a 200K-row dense list)
  const int lane = threadIdx.x & 63, sub = lane & 15, grp = lane >> 4;
  const long long cnt = min((long long)*count, cap);
  const long long wv = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const long long nwv = (long long)gridDim.x * 4;
  for (long long e0 = wv * 4; e0 < cnt; e0 += nwv * 4) {
    const long long e = e0 + grp;
    const bool live = e < cnt;
    const long long r = rows[live ? e : e0];
    const int l = labels[r];
    const bool ok = live && l >= 0;
    const float* xr = X + (size_t)r * d;
    const float* cr = Cm + (size_t)(l >= 0 ? l : 0) * d;
    double s = 0.0;
    for (int f = 4 * sub; f < d; f += 64) {
      const float4 xv = *reinterpret_cast<const float4*>(xr + f);
      const float4 cv = *reinterpret_cast<const float4*>(cr + f);
      const double d0 = (double)xv.x - (double)cv.x, d1 = (double)xv.y - (double)cv.y;
      const double d2 = (double)xv.z - (double)cv.z, d3 = (double)xv.w - (double)cv.w;
      s = fma(d0, d0, fma(d1, d1, fma(d2, d2, fma(d3, d3, s))));
    }
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) s += __shfl_xor(s, o, 64);
    if (ok && sub == 0) corr[r] = (float)((double)mind[r] - s);
  }
}

// ---------------------------------------------------------------------------
// mind of the rows the filter resolved with a single candidate (marker < 0):
// exact fp64 |x - c_label|^2, one wave per row.  The Lloyd step does this
// inside the segmented reduce (it streams the rows anyway); this standalone
// pass serves estep() calls outside a step (final E-step, predict/score).
__global__ void __launch_bounds__(256) fill_mind_kernel(const float* __restrict__ X, int ldx,
                                                        const float* __restrict__ Cm, int d,
                                                        const int* __restrict__ labels,
                                                        float* __restrict__ mind, long long n) {
  const int lane = threadIdx.x & 63;
  for (long long r = (long long)blockIdx.x * 4 + (threadIdx.x >> 6); r < n;
       r += (long long)gridDim.x * 4) {
    if (!(mind[r] < 0.0f)) continue;   // wave-uniform
    const int l = labels[r];
    if (l < 0) continue;
    double s = 0.0;
    for (int f = lane; f < d; f += 64) {
      const double df = (double)X[(size_t)r * ldx + f] - (double)Cm[(size_t)l * d + f];
      s = fma(df, df, s);
    }
    s = wave_sum(s);
    if (lane == 0) mind[r] = (float)s;
  }
}

// deterministic sum of n floats: every block sums a fixed contiguous chunk in
// a fixed thread order and tree; the launcher reduces the block partials with
// the one-block sum_partials kernel (kmeans.hip) - bit-reproducible.
__global__ void __launch_bounds__(256) sum_f32_blocks_kernel(const float* __restrict__ v,
                                                             long long n, double* __restrict__ part) {
  __shared__ double red[256];
  // block ranges in whole 1024-float pieces (16-B aligned float4 loads; v is
  // a 256-B aligned allocation), 4 independent float4 loads in flight per
  // thread; fixed association (deterministic)
  const long long per = (n + (long long)gridDim.x * 1024 - 1) / ((long long)gridDim.x * 1024) * 1024;
  const long long b = (long long)blockIdx.x * per, e = min(n, b + per);
  double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
  const long long e4 = b < e ? b + (e - b) / 4 * 4 : b;
  const float4* v4 = reinterpret_cast<const float4*>(v);
  long long i = b / 4 + threadIdx.x;
  for (; i + 768 < e4 / 4; i += 1024) {
    const float4 a = v4[i], c = v4[i + 256], f = v4[i + 512], g = v4[i + 768];
    s0 += ((double)a.x + (double)a.y) + ((double)a.z + (double)a.w);
    s1 += ((double)c.x + (double)c.y) + ((double)c.z + (double)c.w);
    s2 += ((double)f.x + (double)f.y) + ((double)f.z + (double)f.w);
    s3 += ((double)g.x + (double)g.y) + ((double)g.z + (double)g.w);
  }
  for (; i < e4 / 4; i += 256) {
    const float4 a = v4[i];
    s0 += ((double)a.x + (double)a.y) + ((double)a.z + (double)a.w);
  }
  for (long long t = e4 + threadIdx.x; t < e; t += 256) s1 += (double)v[t];
  red[threadIdx.x] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

// ---------------------------------------------------------------------------
// fp16-split centroid operand from fp32 centroids (initial centres; the
// per-iteration operand is written by centroid_finalize in kmeans.hip):
// one workgroup per padded centroid row.
SQ_DEV void write_f16_operand_row(_Float16* op, int j, int k, const float* c, int d, int d_pad,
                                  float alpha, int tid, double* red) {
  const int dch = d_pad / 8;
  const int cpr = 2 * dch + 2;
  _Float16* base = op + (size_t)(j >> 6) * cpr * 512 + (size_t)(j & 63) * 8;
  auto hi_at = [&](int f) -> _Float16& { return base[(size_t)(f >> 3) * 512 + (f & 7)]; };
  auto lo_at = [&](int f) -> _Float16& { return base[(size_t)(dch + 2 + (f >> 3)) * 512 + (f & 7)]; };
  double nn = 0.0;
  for (int f = tid; f < d_pad; f += 256) {
    _Float16 h = (_Float16)0.0f, l = (_Float16)0.0f;
    if (j < k && f < d) {
      const float v = c[f];
      const double a = (double)v * (double)alpha;
      nn += a * a;
      const float s = -2.0f * alpha * v;             // exact scaling
      h = (_Float16)s;
      l = (_Float16)(s - (float)h);
    }
    hi_at(f) = h;
    lo_at(f) = l;
  }
  for (int f = d_pad + 3 + tid; f < d_pad + 16; f += 256) hi_at(f) = (_Float16)0.0f;
  nn = wave_sum(nn);
  if ((tid & 63) == 0) red[tid >> 6] = nn;
  __syncthreads();
  if (tid == 0) {
    if (j >= k) {
      // padding centroids: a norm above every real scaled distance
      hi_at(d_pad) = hi_at(d_pad + 1) = hi_at(d_pad + 2) = (_Float16)65504.0f;
    } else {
      const float t = (float)(red[0] + red[1] + red[2] + red[3]);
      const _Float16 hi = (_Float16)t;
      const float r1 = t - (float)hi;
      const _Float16 mid = (_Float16)r1;
      const _Float16 lo = (_Float16)(r1 - (float)mid);
      hi_at(d_pad) = hi;
      hi_at(d_pad + 1) = mid;
      hi_at(d_pad + 2) = lo;
    }
  }
}

__global__ void __launch_bounds__(256) centers_f16_operand_kernel(const float* __restrict__ Cm,
                                                                  _Float16* __restrict__ op,
                                                                  int k, int d, int d_pad,
                                                                  float alpha) {
  __shared__ double red[4];
  const int j = blockIdx.x;
  write_f16_operand_row(op, j, k, Cm + (size_t)(j < k ? j : 0) * d, d, d_pad, alpha, threadIdx.x,
                        red);
}

}  // namespace sq

using namespace sq;

extern "C" int sq_sum_partials(const void* part, int n, void* out, void* stream);
extern "C" int sq_rows_f64(const void* X, long long ldx, const void* C, long long ldc, int d, int k,
                           const void* rows, const void* count, long long n_direct, long long cap,
                           void* labels, void* mind, void* corr, void* ub, double delta,
                           unsigned k0, unsigned k1, unsigned s0, unsigned s1,
                           long long row_offset, int grid, void* stream);

template <int KSD, int TOP = 2>
static int launch_estep_f32(const void* X, const void* C, const void* xn, void* labels, void* mind,
                            void* ovf_rows, void* ovf_count, void* part, int part_cap,
                            void* inertia, long long n, int k_pad, float alpha, float inv_a2,
                            float delta_s, RngKey key, long long row_offset, int ovf_cap,
                            hipStream_t st, const void* rlist = nullptr,
                            const void* rcount = nullptr, const void* cmax2 = nullptr,
                            void* mrows = nullptr, void* mcand = nullptr,
                            void* multi_count = nullptr, void* xflag = nullptr,
                            long long mcap = 0) {
  constexpr int NW = 4;
  const size_t lds = 2 * (size_t)((2 * KSD + 1) * 2048);
  auto kern = estep_f32_kernel<KSD, TOP>;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  static int resident = 0;
  if (resident == 0) {
    int dev = 0, cus = 0, per_cu = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)kern, NW * 64, lds);
    resident = (cus > 0 ? cus : 256) * (per_cu > 0 ? per_cu : 1);
  }
  const long long nblk = (n + NW * 32 - 1) / (NW * 32);
  // list mode: the row count is on the device - every resident slot launches
  unsigned grid = (unsigned)(nblk < resident && !rlist ? nblk : resident);
  if ((long long)grid * NW > part_cap) grid = (unsigned)(part_cap / NW);
  if (grid == 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(kern, dim3(grid), dim3(NW * 64), lds, st, (const float*)X,
                     (const _Float16*)C, (const float*)xn, (int*)labels, (float*)mind,
                     (long long*)ovf_rows, (int*)ovf_count, (double*)part, n, k_pad, alpha, inv_a2,
                     delta_s, key, row_offset, ovf_cap, (const long long*)rlist,
                     (const int*)rcount, (const float*)cmax2, (long long*)mrows, (int*)mcand,
                     (int*)multi_count, (unsigned char*)xflag, mcap);
  // per-wave inertia partials summed in a fixed order (bit-reproducible)
  if (!inertia) return (int)hipGetLastError();
  return sq_sum_partials(part, (int)grid * NW, inertia, st);
}

template <int KSD>
static int launch_estep_x64(const void* Xh, const void* X, const void* C, const void* Cm,
                            const void* xn, const void* cmax2, void* labels, void* mind,
                            void* dense_rows, void* dense_count, void* mrows, void* mcand,
                            void* multi_count, void* corr, long long n, int k_pad, float alpha,
                            float delta_s, double delta, RngKey key, long long row_offset,
                            int dense_cap, hipStream_t st, const void* rlist, const void* rcount,
                            void* ub, void* lb, void* mflag, void* xflag, int list_rs,
                            bool defer_rows = false) {
  // list mode (the rows the bounds could not prune): one row set per wave -
  // half the rows per workgroup, so a short list (the per-GPU share of a
  // strong-scaled run) finishes in one half-length sweep; a full sweep keeps
  // the two row sets that halve the centroid staging per row
  int qbits = 1;
  while ((1 << qbits) < 2 * (k_pad / kTileN)) ++qbits;
  auto go = [&](auto RS_) {
    constexpr int RS = decltype(RS_)::value;
    constexpr int NW = kX64Waves;
    const size_t lds =
        kX64Ring * (size_t)X64Geom<KSD>::SLOT + (size_t)NW * RS * 32 * (kMaxCand + 1) * 4 +
        (size_t)NW * 64 * 4;   // + per-lane dump slots
    auto kern = estep_x64_kernel<KSD, RS>;
    static bool attr = false;
    if (!attr) {
      hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                          160 * 1024);
      attr = true;
    }
    static int resident = 0;
    if (resident == 0) {
      int dev = 0, cus = 0, per_cu = 0;
      hipGetDevice(&dev);
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)kern, NW * 64, lds);
      resident = (cus > 0 ? cus : 256) * (per_cu > 0 ? per_cu : 1);
    }
    const long long nblk = (n + NW * 32 * RS - 1) / (NW * 32 * RS);
    // list mode: the row count is on the device - every resident slot launches
    const unsigned grid = (unsigned)(nblk < resident && !rlist ? nblk : resident);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(NW * 64), lds, st, (const _Float16*)Xh,
                       (const float*)X, (const _Float16*)C, (const float*)Cm, (const float*)xn,
                       (const float*)cmax2, (int*)labels, (float*)mind, (long long*)dense_rows,
                       (int*)dense_count, (long long*)mrows, (int*)mcand, (int*)multi_count, n,
                       k_pad, alpha, delta_s, key, row_offset, dense_cap, qbits,
                       (const long long*)rlist, (const int*)rcount, (float*)ub, (float*)lb,
                       (int*)mflag);
  };
  static const bool list_rs1 = [] {
    const char* e = getenv("SQ_X64_LIST_RS1");
    return !(e && e[0] == '0');
  }();
  // list_rs (host hint): 1 / 2 row sets in list mode, 0 = the default (1)
  if (rlist && (list_rs == 1 || (list_rs == 0 && list_rs1)))
    go(std::integral_constant<int, 1>{});
  else
    go(std::integral_constant<int, X64RowSets<KSD>::value>{});
  int rc = (int)hipGetLastError();
  if (rc) return rc;
  // the re-check: one pass over the multi list (count read on the device);
  // with xrows the fp32 screen first, the fp64 pass over what it left
  const long long rblocks = (n / 16 + 63) / 64;
  const unsigned rgrid = (unsigned)(rblocks < 4096 ? (rblocks > 0 ? rblocks : 1) : 4096);
  if (xflag && g_mrec.rec && ub) {
    if constexpr (KSD * 16 % 128 == 0) {
      // list B first: its uncertain rows join the multi list
      // one resident round of long-lived waves (each takes blocks of 64 rows)
      static long long gres = 0;
      if (gres == 0) {
        int dev = 0, cus = 0, per_cu = 0;
        hipGetDevice(&dev);
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &per_cu, (const void*)gap_screen_kernel<KSD * 16>, 256, 0);
        gres = (long long)(cus > 0 ? cus : 256) * (per_cu > 0 ? per_cu : 2);
      }
      const unsigned bgrid = (unsigned)min(max(rblocks, 1LL), gres);
      hipLaunchKernelGGL(gap_screen_kernel<KSD * 16>, dim3(bgrid), dim3(256), 0, st,
                         (const _Float16*)Xh, (const float*)xn, g_mrec.mrows_b, g_mrec.count_b,
                         g_mrec.dsh, g_mrec.dsh_stride, g_mrec.dq,
                         g_mrec.dsh_stride / (KSD * 16) * 8, 1.0f / alpha, (float)delta,
                         (int*)labels, g_mrec.rec, g_mrec.mflag, g_mrec.it_now, g_mrec.ring,
                         max(1, g_mrec.ring / 2), (long long*)mrows, (int*)multi_count, n,
                         g_mrec.n_done);
    }
  }
  if (xflag) {
    // one resident round of long-lived waves (each walks its slice with the
    // load pipeline warm) instead of several rounds of short ones
    static int sgrid = 0, sil = 0;
    if (sgrid == 0) {
      const char* ei = getenv("SQ_SCREEN_IL");
      sil = ei ? atoi(ei) : 0;
      const char* e = getenv("SQ_SCREEN_GRID");
      sgrid = e ? atoi(e) : 1024;
      if (sgrid <= 0) sgrid = 4096;
    }
    const unsigned fgrid2 = (unsigned)(rblocks < sgrid ? (rblocks > 0 ? rblocks : 1) : sgrid);
    auto fk = ub ? recheck_fast_kernel<KSD * 16, SQ_SCREEN_LPR, true>
                 : recheck_fast_kernel<KSD * 16, SQ_SCREEN_LPR, false>;
    hipLaunchKernelGGL(fk, dim3(fgrid2), dim3(256), 0, st, (const float*)X, (const float*)Cm,
                       (const long long*)mrows, (const int*)mcand, (const int*)multi_count,
                       (int*)labels, (float*)mind, n, delta, (float*)ub, (unsigned char*)xflag,
                       sil, g_mrec.rec, g_mrec.mflag, g_mrec.it_now, key, row_offset,
                       (float*)corr);
  }
  // (defer_rows: the caller launches it after the dense-row passes, which
  // append their near-edge rows to the multi list)
  if (!defer_rows)
    hipLaunchKernelGGL(recheck_rows_kernel<KSD * 16>, dim3(rgrid), dim3(256), 0, st,
                       (const float*)X, (const float*)Cm, (const long long*)mrows,
                       (const int*)mcand, (const int*)multi_count, (int*)labels, (float*)mind, n,
                       delta, key, row_offset, (float*)corr, (float*)ub,
                       (const unsigned char*)xflag);
  return (int)hipGetLastError();
}

extern "C" {

// X: fp32 [n][d_pad] (zero-padded), C: fp16-split operand (see
// centers_f16_operand_kernel), alpha: power of two, delta in data units.
int sq_estep_f32(const void* X, const void* C, const void* xn, void* labels, void* mind,
                 void* ovf_rows, void* ovf_count, void* part, int part_cap, void* inertia,
                 long long n, int d_pad, int k_pad, double alpha, double delta, unsigned k0,
                 unsigned k1, unsigned s0, unsigned s1, long long row_offset, int ovf_cap,
                 void* stream) {
  if (n <= 0) return 0;
  if (k_pad % kTileN != 0 || k_pad <= 0 || k_pad > 32768 || part_cap < 4)
    return (int)hipErrorInvalidValue;
  const double a2 = alpha * alpha;
  int aexp = 0;
  if (!(alpha > 0.0) || frexp(alpha, &aexp) != 0.5) return (int)hipErrorInvalidValue;  // 2^e
  RngKey key{k0, k1, s0, s1};
  hipStream_t st = (hipStream_t)stream;
  const float fa = (float)alpha, ia2 = (float)(1.0 / a2), ds = (float)(delta * a2);
  int rc;
  switch (d_pad) {
#define CASE(KSD)                                                                                \
  case KSD * 16:                                                                                 \
    rc = launch_estep_f32<KSD>(X, C, xn, labels, mind, ovf_rows, ovf_count, part, part_cap,      \
                               inertia, n, k_pad, fa, ia2, ds, key, row_offset, ovf_cap, st);    \
    break;
    CASE(1) CASE(2) CASE(4) CASE(8) CASE(16)
#undef CASE
    default:
      return (int)hipErrorInvalidValue;
  }
  return rc;
}

// Certified E-step (the default): filter + fp64 re-check (estep_x64_kernel),
// dense rows through the 3-pass fp32-faithful kernel in list mode, its
// overflow rows through the exact fp64 rows kernel (rows_f64.hip; at d_pad >
// 256 the dense rows go there directly), the multi-candidate rows through
// recheck_rows_kernel.  counts[0] = 3-pass overflow rows, counts[1] = dense
// rows, counts[2] = multi rows; all zero on entry.  xflag [n] (uint8, per
// multi-list entry): with it the fp32 screen runs first and the fp64
// re-check takes only the entries it flags (null: every multi row).  mrows [n] (int64) is the
// multi list, mcand [n][kMaxCand + 1] (int32) the candidate lists BY ROW.  mind holds -1 for rows
// whose distance the M-step (or fill_mind) computes; no inertia here.
// Xh: fp16(alpha x) [n][d_pad]; X: fp32 [n][d_pad]; Cm: fp32 centroids
// [k][d_pad] (zero-padded like X); C: the fp16-split operand.
int sq_estep_x64(const void* Xh, const void* X, const void* C, const void* Cm, const void* xn,
                 const void* cmax2, void* labels, void* mind, void* dense_rows, void* ovf_rows,
                 void* mrows, void* mcand, void* corr, void* rlist, void* rcount, void* ub,
                 void* lb, void* mflag, void* xflag, void* counts, void* part, int part_cap, long long n, int d, int d_pad,
                 int k,
                 int k_pad, double alpha, double delta, unsigned k0, unsigned k1, unsigned s0,
                 unsigned s1, long long row_offset, int list_rs, void* stream) {
  if (n <= 0) return 0;
  if (k_pad % kTileN != 0 || k_pad <= 0 || k_pad > 32768 || k > k_pad || d > d_pad)
    return (int)hipErrorInvalidValue;
  if ((ub != nullptr) != (lb != nullptr) || (ub != nullptr) != (mflag != nullptr))
    return (int)hipErrorInvalidValue;   // bounds need the multi-row slot map
  int aexp = 0;
  if (!(alpha > 0.0) || frexp(alpha, &aexp) != 0.5) return (int)hipErrorInvalidValue;
  RngKey key{k0, k1, s0, s1};
  hipStream_t st = (hipStream_t)stream;
  const double a2 = alpha * alpha;
  const float fa = (float)alpha, ia2 = (float)(1.0 / a2), ds = (float)(delta * a2);
  int* cnt = (int*)counts;
  // list mode follows the bounds filter, which zeroed the corrections
  if (corr && !rlist) hipMemsetAsync(corr, 0, (size_t)n * sizeof(float), st);
  const int cap = (int)min(n, 2147483647LL);
  const unsigned fgrid = (unsigned)min((n + 15) / 16, 512LL);   // exact fp64 rows kernel
  const long long rblocks = (n / 16 + 63) / 64;                  // fp64 re-check (as in launch_estep_x64)
  const unsigned rgrid = (unsigned)(rblocks < 4096 ? (rblocks > 0 ? rblocks : 1) : 4096);
  int rc;
  switch (d_pad) {
    // d_pad <= 256: dense rows through the fp32-faithful 3-pass kernel (list
    // mode), its overflow rows through the exact fp64 rows kernel
#define CASE(KSD)                                                                                \
  case KSD * 16:                                                                                 \
    rc = launch_estep_x64<KSD>(Xh, X, C, Cm, xn, cmax2, labels, mind, dense_rows, cnt + 1,       \
                               mrows, mcand, cnt + 2, corr, n, k_pad, fa, ds, delta, key,        \
                               row_offset, cap, st, rlist, rcount, ub, lb, mflag, xflag,         \
                               list_rs, true);                                                   \
    if (rc) return rc;                                                                           \
    rc = launch_estep_f32<KSD>(X, C, xn, labels, mind, ovf_rows, cnt, part, part_cap, nullptr,   \
                               n, k_pad, fa, ia2, ds, key, row_offset, cap, st, dense_rows,       \
                               cnt + 1, cmax2, mrows, mcand, cnt + 2, xflag, n);                 \
    if (rc) return rc;                                                                           \
    if (g_ovf2.rows) {                                                                           \
      /* the overflow rows once more with 3 members per lane; what still */                      \
      /* overflows goes to the fp64 rows kernel */                                               \
      rc = launch_estep_f32<KSD, 3>(X, C, xn, labels, mind, g_ovf2.rows, g_ovf2.count, part,     \
                                    part_cap, nullptr, n, k_pad, fa, ia2, ds, key, row_offset,   \
                                    cap, st, ovf_rows, cnt, cmax2, mrows, mcand, cnt + 2, xflag, \
                                    n);                                                          \
      if (rc) return rc;                                                                         \
    }                                                                                            \
    if (corr)                                                                                    \
      hipLaunchKernelGGL(dense_corr_kernel, dim3(1024), dim3(256), 0, st, (const float*)X,       \
                         (const float*)Cm, (const long long*)dense_rows, (const int*)(cnt + 1),   \
                         (const int*)labels, (const float*)mind, (float*)corr, n, d_pad);        \
    /* the fp64 re-check of the multi list, incl. the near-edge dense rows */                    \
    hipLaunchKernelGGL(recheck_rows_kernel<KSD * 16>, dim3(rgrid), dim3(256), 0, st,            \
                       (const float*)X, (const float*)Cm, (const long long*)mrows,               \
                       (const int*)mcand, (const int*)(cnt + 2), (int*)labels, (float*)mind, n,  \
                       delta, key, row_offset, (float*)corr, (float*)ub,                         \
                       (const unsigned char*)xflag);                                             \
    rc = sq_rows_f64(X, d_pad, Cm, d_pad, d_pad, k, g_ovf2.rows ? g_ovf2.rows : ovf_rows,        \
                     g_ovf2.rows ? g_ovf2.count : cnt, 0, n, labels, mind, corr,                  \
                     ub, delta, k0, k1, s0, s1, row_offset, (int)fgrid, stream);                 \
    break;
    CASE(1) CASE(2) CASE(4) CASE(8) CASE(16)
#undef CASE
    // d_pad > 256: the dense rows straight to the exact fp64 rows kernel
#define CASE(KSD)                                                                                \
  case KSD * 16:                                                                                 \
    rc = launch_estep_x64<KSD>(Xh, X, C, Cm, xn, cmax2, labels, mind, dense_rows, cnt + 1,       \
                               mrows, mcand, cnt + 2, corr, n, k_pad, fa, ds, delta, key,        \
                               row_offset, cap, st, rlist, rcount, ub, lb, mflag, xflag,         \
                               list_rs);                                                         \
    if (rc) return rc;                                                                           \
    rc = sq_rows_f64(X, d_pad, Cm, d_pad, d_pad, k, dense_rows, cnt + 1, 0, n, labels, mind,      \
                     corr, ub, delta, k0, k1, s0, s1, row_offset, (int)fgrid, stream);           \
    break;
    CASE(24) CASE(32) CASE(40) CASE(48) CASE(56) CASE(64)
#undef CASE
    default:
      return (int)hipErrorInvalidValue;
  }
  if (rc) return rc;
  return (int)hipGetLastError();
}

#if SQ_X64_STAMP
// diagnostic builds: copy the per-wave phase sums (see g_x64_stamps) to host
int sq_x64_stamps(void* host, int n_waves) {
  const int m = n_waves < kStampWaves ? n_waves : kStampWaves;
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_x64_stamps),
                                  (size_t)m * kStampN * sizeof(unsigned long long), 0,
                                  hipMemcpyDeviceToHost);
}
int sq_x64_stamps_clear() {
  static unsigned long long zeros[kStampWaves * kStampN];
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_x64_stamps), zeros, sizeof(zeros), 0,
                                hipMemcpyHostToDevice);
}
#endif

int sq_fill_mind(const void* X, int ldx, const void* Cm, int d, const void* labels, void* mind,
                 long long n, void* stream) {
  if (n <= 0) return 0;
  const unsigned grid = (unsigned)((n + 3) / 4 < 8192 ? (n + 3) / 4 : 8192);
  hipLaunchKernelGGL(fill_mind_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                     (const float*)X, ldx, (const float*)Cm, d, (const int*)labels, (float*)mind, n);
  return (int)hipGetLastError();
}

// inertia[0] = sum of mind[0:n) in a fixed order (part: >= 512 doubles)
// out = sum(v[:n]) + sum(part[512 : 512 + extra]) in a fixed order (the
// extra partials - e.g. the per-cluster inertia parts - are written there by
// an earlier launch: one final reduce for both)
int sq_sum_f32(const void* v, long long n, void* part, int extra, void* out, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const int blocks = 512;
  if (extra < 0 || ((uintptr_t)v & 15u) != 0) return (int)hipErrorInvalidValue;   // float4 loads
  hipLaunchKernelGGL(sum_f32_blocks_kernel, dim3(blocks), dim3(256), 0, st, (const float*)v, n,
                     (double*)part);
  return sq_sum_partials(part, blocks + extra, out, st);
}

int sq_centers_f16_operand(const void* Cm, void* op, int k, int d, int d_pad, int k_pad,
                           double alpha, void* stream) {
  if (k_pad % kTileN != 0 || d_pad % 16 != 0 || d > d_pad) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(centers_f16_operand_kernel, dim3((unsigned)k_pad), dim3(256), 0,
                     (hipStream_t)stream, (const float*)Cm, (_Float16*)op, k, d, d_pad,
                     (float)alpha);
  return (int)hipGetLastError();
}

}  // extern "C"
