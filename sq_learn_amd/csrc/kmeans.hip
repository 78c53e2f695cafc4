// q-means / k-means hot loop on gfx950.
//
// estep_bf16 : fused distance GEMM (MFMA v_mfma_f32_32x32x16_bf16, fp32
//              accumulation) + per-row top-2 / delta-band selection + inertia.
//   * one workgroup = NW waves x 32 rows; each wave keeps its 32 rows of X as
//     A fragments in VGPRs for the whole centroid sweep (X read from HBM once)
//   * centroid tiles of 64 x d_pad bf16 stream through a 2-deep LDS ring filled
//     by global_load_lds (LDS-DMA), XOR-swizzled (chunk ^ row&15) so the
//     ds_read_b128 B-fragment reads are bank-conflict-free
//   * epilogue per accumulator element: d' = ||c||^2 - 2 x.c, the centroid
//     index packed into the low mantissa bits, then m1 = min, m2 = med3 (4 VALU)
//   * after the sweep the 32 lanes sharing a row merge; the delta-band
//     {j : D_ij <= min_i + delta} is resolved exactly from each lane's top-2
//     (a lane whose 2nd-best is inside the band could hide a 3rd candidate ->
//     the row is appended to an overflow list and re-done by band_select)
//   * uniform choice among band members = smallest Philox key
//     hash(seed, stream, global_row, j): shard-invariant and identical to
//     band_select and to the torch CPU path.
// band_select: exact selection over fp32 distance rows (fallback / generic d).
// centroid_accumulate: label-segmented row sums (LDS counting sort per chunk,
//              one 256-B f32 atomic row-add per (chunk, label) segment).
// centroid_finalize: mean, empty-cluster policy, fused truncated-normal
//              tomography noise (Utility.py:88-104), centre shift, bf16 copy
//              and ||c||^2 for the next E-step.
// ipe_estep : distance estimates through robust inner-product estimation
//              (Utility.py:697-737) - median-of-Q Fejer AE per (row, centroid).
#include "common.h"
#include "fejer.h"
#include "band.h"

namespace sq {

typedef __attribute__((ext_vector_type(8))) short bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;

constexpr int kBN = 64;                  // centroids per LDS tile
constexpr float kBig = 3.0e38f;

SQ_DEV float packf(float v, uint32_t keepmask, uint32_t j) {
  return __uint_as_float((__float_as_uint(v) & keepmask) | j);
}
SQ_DEV float valf(float p, uint32_t keepmask) { return __uint_as_float(__float_as_uint(p) & keepmask); }

// single-instruction min / med3: no canonicalising v_max on bit-packed inputs
SQ_DEV float min_raw(float a, float b) {
  float r;
  asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
SQ_DEV float med3_raw(float a, float b, float c) {
  float r;
  asm("v_med3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// delta-band rule helpers (band_key, band_u, band_pick_wave, ...): band.h

// Centroid operand layout (written by centroid_finalize / centers_to_bf16):
// per 64-centroid tile, CPR = (d_pad + 16) / 8 chunks of 16 B, chunk-major:
//   elem(j, f) at ((tile * CPR + f / 8) * 64 + j % 64) * 8 + f % 8
// holding C' = -2 c for f < d_pad and, in the augmented chunk f = d_pad ..
// d_pad + 7, [hi, mid, lo, 0 ...] (3-way bf16 split of ||c||^2).  With the
// constant A fragment [1, 1, 1, 0 ...] for that chunk the MFMA accumulates
// D' = ||c||^2 - 2 x.c directly.  The tile is one contiguous 16-B-per-lane
// LDS-DMA copy and every B-fragment read is base + constant offset: lanes of
// a ds_read_b128 group hit 16 consecutive 16-B slots (conflict-free).
//
// Persistent: the grid is sized to the resident workgroups and each one walks
// row blocks blk = blockIdx.x, + gridDim.x, ...  The centroid-tile ring runs
// continuously across blocks (tile 0 of the next block is staged while the
// last tiles of the current one are multiplied), and the next block's X rows
// are loaded into the A registers as soon as the last MFMA of the current
// block has consumed them, so their latency hides behind the epilogue and
// the merge instead of stalling a fresh workgroup's first MFMA.
#ifndef SQ_ESTEP_PF
#define SQ_ESTEP_PF 1
#endif
#ifndef SQ_ESTEP_PAIR
#define SQ_ESTEP_PAIR 0
#endif
// compile-time ablations (timing experiments only; results invalid):
// bit 1 = no centroid staging after tile 1, bit 2 = no top-2 epilogue.
// Compile-time so that no runtime branch splits the pipelined basic block.
#ifndef SQ_ESTEP_ABLATE
#define SQ_ESTEP_ABLATE 0
#endif
template <int KSD, int NW>
__global__ void __launch_bounds__(NW * 64, 2) estep_kernel(
    const uint16_t* __restrict__ X, const uint16_t* __restrict__ C, float* __restrict__ ovf_thr,
    const float* __restrict__ xn, int* __restrict__ labels, float* __restrict__ mind,
    long long* __restrict__ ovf_rows, int* __restrict__ ovf_count, double* __restrict__ inertia,
    long long n, int k, int k_pad, float delta, RngKey key, long long row_offset, int ovf_cap,
    int idx_bits, int dbg) {
  (void)dbg;
  (void)k;
  constexpr int KS = KSD + 1;            // data k-steps + augmented norm step
  constexpr int DX = KSD * 16;           // X row length (padded features)
  constexpr int CPR = KS * 2;            // 16-B chunks per centroid (incl. norms)
  constexpr int TILE_BYTES = kBN * CPR * 16;
  constexpr int PIECES = TILE_BYTES / 1024;  // 1 KiB LDS-DMA pieces per tile
  constexpr int ROWS = NW * 32;          // rows per block
  constexpr int PF = SQ_ESTEP_PF;        // B-fragment prefetch distance (k-steps)
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  // ring of RING tile slots; PAIR mode stages two tiles per DMA round and
  // synchronises the workgroup once per two tiles (half the barriers)
  constexpr int RING = SQ_ESTEP_PAIR ? 4 : 2;
  auto buf = [&](int g) -> unsigned char* { return smem + (g & (RING - 1)) * TILE_BYTES; };

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r32 = lane & 31;
  const int half = lane >> 5;
  const uint32_t keep = ~((1u << idx_bits) - 1u);
  const int n_tiles = k_pad / kBN;
  const long long nblk = (n + ROWS - 1) / ROWS;
  long long blk = blockIdx.x;
  if (blk >= nblk) return;

  // ---- LDS-DMA of centroid tile (G mod n_tiles) into ring slot G & 1: a
  // contiguous 16-B-per-lane copy
  auto stage = [&](int G) {
    const int t = (int)(G % n_tiles);
    const unsigned char* tile = reinterpret_cast<const unsigned char*>(C) + (size_t)t * TILE_BYTES;
    unsigned char* dst = buf(G);
    if ((SQ_ESTEP_ABLATE & 2) && G > 1) return;   // ablation: no centroid staging
    for (int p = wave; p < PIECES; p += NW) {
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(tile + p * 1024 + lane * 16),
          (__attribute__((address_space(3))) void*)(dst + p * 1024), 16, 0, 0);
    }
  };

  // ---- A fragments: this wave's 32 rows, all of K, kept in VGPRs; the
  // augmented step is the constant [1, 1, 1, 0, ...] (k = 0..2 of the step)
  bf16x8 a[KS];
  auto load_a = [&](long long b) {
    long long r = b * ROWS + wave * 32 + r32;
    const uint16_t* xr = X + (size_t)(r < n ? r : n - 1) * DX + half * 8;
#pragma unroll
    for (int ks = 0; ks < KSD; ++ks) a[ks] = *reinterpret_cast<const bf16x8*>(xr + ks * 16);
  };
  {
    bf16x8 aug = (bf16x8)0;
    if (half == 0) { aug[0] = aug[1] = aug[2] = (short)0x3f80; }   // hi + mid + lo
    a[KSD] = aug;
  }

  float m1[16], m2[16];

  // chunk-major tile: B fragment of (k-step ks, 32-col block nb) for this
  // lane = base + ks * 2048 + nb * 512 (immediate offsets, no VALU math)
  const int lane_off = (half * 64 + r32) * 16;
  auto ldb = [&](const unsigned char* cur, int nb, int ks) -> bf16x8 {
    return *reinterpret_cast<const bf16x8*>(cur + lane_off + ks * 2048 + nb * 512);
  };
  // Cross-tile software pipeline: while the MFMAs of tile t+1 run, the VALU
  // epilogue (index packing, top-2) of tile t executes in the MFMA shadow.
  // Two accumulator sets (pA, pB) alternate with static names.
  auto tile_step = [&](const unsigned char* cur, f32x16& n0, f32x16& n1, bool do_mfma,
                       const f32x16& o0, const f32x16& o1acc, int t_prev, bool do_epi) {
    const uint32_t j0 = (uint32_t)(t_prev * kBN + r32);
    const uint32_t j1 = j0 + 32;
    const bool epi = do_epi && !(SQ_ESTEP_ABLATE & 4);
    // top-2 update of row i of the previous tile (3 VALU per value)
    auto epi_row = [&](int i) {
      float p0 = packf(o0[i], keep, j0);
      float p1 = packf(o1acc[i], keep, j1);
      float q1 = m1[i];
      float q2 = m2[i];
      q2 = med3_raw(q1, p0, q2);
      q1 = min_raw(q1, p0);
      q2 = med3_raw(q1, p1, q2);
      q1 = min_raw(q1, p1);
      m1[i] = q1;
      m2[i] = q2;
    };
    if (do_mfma) {
      // explicit software pipeline: the source order IS the schedule
      // (sched_barrier after every k-step): B reads PF k-steps ahead, the two
      // MFMAs of the k-step, then the slice of the previous tile's epilogue
      // that runs in their shadow
      f32x16 acc0 = {0}, acc1 = {0};
      bf16x8 b0[PF + 1], b1[PF + 1];
#pragma unroll
      for (int q = 0; q < PF && q < KS; ++q) { b0[q] = ldb(cur, 0, q); b1[q] = ldb(cur, 1, q); }
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        if (ks + PF < KS) {
          b0[(ks + PF) % (PF + 1)] = ldb(cur, 0, ks + PF);
          b1[(ks + PF) % (PF + 1)] = ldb(cur, 1, ks + PF);
        }
        acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[ks], b0[ks % (PF + 1)], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[ks], b1[ks % (PF + 1)], acc1, 0, 0, 0);
        if (epi) {
#pragma unroll
          for (int i = (ks * 16) / KS; i < ((ks + 1) * 16) / KS; ++i) epi_row(i);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      n0 = acc0;
      n1 = acc1;
    } else if (epi) {
#pragma unroll
      for (int i = 0; i < 16; ++i) epi_row(i);
    }
  };
  auto sync_tile = [&]() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  };
  auto merge2 = [](float& a1, float& a2, float b1, float b2) {
    float lo2 = min_raw(a2, b2);
    a2 = med3_raw(a1, b1, lo2);   // 2nd smallest of two sorted pairs
    a1 = min_raw(a1, b1);
  };

  // hooks around the MFMA of tile Gc: issue the next DMA, then synchronise
  auto pre_tile = [&](int Gc) {
    if (SQ_ESTEP_PAIR) {
      if ((Gc & 1) == 0) { stage(Gc + 2); stage(Gc + 3); }
    } else {
      stage(Gc + 1);
    }
  };
  auto post_tile = [&](int Gc) {
    if (!SQ_ESTEP_PAIR || (Gc & 1)) sync_tile();
  };

  int G = 0;   // global tile sequence number: tile G lives in buf(G)
  stage(0);
  if (SQ_ESTEP_PAIR) stage(1);
  load_a(blk);
  sync_tile();
  double my_inertia = 0.0;

  for (; blk < nblk; blk += gridDim.x) {
    const long long row0 = blk * ROWS + wave * 32;
#pragma unroll
    for (int i = 0; i < 16; ++i) { m1[i] = __builtin_inff(); m2[i] = __builtin_inff(); }
    f32x16 pA0, pA1, pB0, pB1;
    // block prologue: tile G (landed) -> pA while tile G+1 streams in
    pre_tile(G);
    tile_step(buf(G), pA0, pA1, true, pA0, pA1, 0, false);
    post_tile(G);
    // steady state: every combined step is ONE basic block (unconditional MFMA
    // + epilogue) so the scheduler can interleave them; static pA/pB names by
    // unrolling two steps; the block's last epilogue runs alone, after the
    // next block's X loads were issued.
    int t = 0;
    while (true) {
      if (t + 1 >= n_tiles) {
        load_a(blk + gridDim.x);   // unconditional (clamped rows): no phi on a[]
        tile_step(smem, pB0, pB1, false, pA0, pA1, t, true);
        break;
      }
      pre_tile(G + 1);
      tile_step(buf(G + 1), pB0, pB1, true, pA0, pA1, t, true);
      post_tile(G + 1);
      ++t;
      ++G;
      if (t + 1 >= n_tiles) {
        load_a(blk + gridDim.x);   // unconditional (clamped rows): no phi on a[]
        tile_step(smem, pA0, pA1, false, pB0, pB1, t, true);
        break;
      }
      pre_tile(G + 1);
      tile_step(buf(G + 1), pA0, pA1, true, pB0, pB1, t, true);
      post_tile(G + 1);
      ++t;
      ++G;
    }
    ++G;   // the block's last tile is consumed; tile G (next block) has landed

    // ---- merge the 32 lanes of each half: transposed top-2 reduce-scatter.
    // Each stage halves the rows a lane carries (xor 16, 8, 4, 2), so a lane
    // ends with the global top-2 of row i = r32 >> 1 after 15 (not 80)
    // shuffle-merges; xor 1 pairs the two lanes that share a row.
    float R1[16], R2[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) { R1[i] = m1[i]; R2[i] = m2[i]; }
#pragma unroll
    for (int o = 16, c = 8; o >= 2; o >>= 1, c >>= 1) {
      const bool hi = (r32 & o) != 0;   // keep the upper half of the rows
#pragma unroll
      for (int j = 0; j < c; ++j) {
        float s1 = hi ? R1[j] : R1[c + j], s2 = hi ? R2[j] : R2[c + j];
        float k1 = hi ? R1[c + j] : R1[j], k2 = hi ? R2[c + j] : R2[j];
        float t1 = __shfl_xor(s1, o, 64), t2 = __shfl_xor(s2, o, 64);
        merge2(k1, k2, t1, t2);
        R1[j] = k1;
        R2[j] = k2;
      }
    }
    float q1 = R1[0], q2 = R2[0];
    merge2(q1, q2, __shfl_xor(R1[0], 1, 64), __shfl_xor(R2[0], 1, 64));

    const int irow = r32 >> 1;
    const int rloc = (irow & 3) + 8 * (irow >> 2) + 4 * half;
    const long long grow_local = row0 + rloc;
    const bool owner = ((r32 & 1) == 0) && grow_local < n;
    const float mval = valf(q1, keep);
    const float thr = mval + delta;
    const bool band2 = valf(q2, keep) <= thr;
    if (owner) {
      const float dist = fmaxf(xn[grow_local] + mval, 0.0f);
      mind[grow_local] = dist;
      if (!band2) labels[grow_local] = (int)(__float_as_uint(q1) & ~keep);
      my_inertia += (double)dist;
    }
    // rows with >= 2 band members: rank rule over the per-lane top-2 lists
    // (lane r32 holds the candidates j = r32 mod 32, so lane order is kappa
    // order); a lane holding two members -> exact fallback (overflow list)
    const unsigned long long slow = __ballot(owner && band2);
    if (slow && !SQ_ESTEP_ABLATE) {   // (ablation runs skip band resolution)
      const float urow = band_u(key, row_offset + grow_local);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const unsigned long long sel = slow & ((1ull << (2 * i)) | (1ull << (32 + 2 * i)));
        if (!sel) continue;
        const int src = 32 * half + 2 * i;
        const bool mine = (slow >> src) & 1ull;
        const float thr_i = __shfl(thr, src, 64);
        const float u_i = __shfl(urow, src, 64);
        const bool v1 = mine && valf(m1[i], keep) <= thr_i;
        const bool v2 = mine && valf(m2[i], keep) <= thr_i;
        const uint32_t hb1 = (uint32_t)(__ballot(v1) >> (32 * half));
        const uint32_t hb2 = (uint32_t)(__ballot(v2) >> (32 * half));
        const int c = __popc(hb1);
        const int pick = hb2 == 0u && c > 0 ? nth_set_bit(hb1, band_rank(u_i, c)) : 0;
        const uint32_t jsel = (uint32_t)__shfl((int)(__float_as_uint(m1[i]) & ~keep),
                                               32 * half + pick, 64);
        if (mine && r32 == 2 * i) {
          const long long g = row0 + (i & 3) + 8 * (i >> 2) + 4 * half;
          if (hb2 != 0u) {
            int slot = atomicAdd(ovf_count, 1);
            if (slot < ovf_cap) { ovf_rows[slot] = g; ovf_thr[slot] = thr_i; }
            labels[g] = -1;
          } else {
            labels[g] = (int)jsel;
          }
        }
      }
    }
  }
  // per-wave partial (no float atomics: the launcher sums the partials in a
  // fixed order, so the inertia is bit-reproducible)
  my_inertia = wave_sum(my_inertia);
  if (lane == 0) inertia[(size_t)blockIdx.x * NW + wave] = my_inertia;
  // drain the ring's surplus prefetch before the LDS is released
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ---------------------------------------------------------------------------
// estep64: the same E-step with 64 rows per wave (two 32-row MFMA blocks
// sharing every B fragment) at one wave per SIMD (up to 512 registers):
// half the LDS traffic per MFMA, room for a 3-deep B ring and for both
// accumulator sets of the cross-tile pipeline, so the top-2 epilogue of tile
// t can actually be interleaved with the MFMAs of tile t+1 (the 32-row
// kernel runs at the 256-register limit of two waves per SIMD and the
// compiler serialises both).  4 waves per workgroup, 256 rows per block.
struct Acc4 {
  f32x16 v[2][2];   // [row block][column block]
};

template <int KSD>
__global__ void __launch_bounds__(256, 1) estep64_kernel(
    const uint16_t* __restrict__ X, const uint16_t* __restrict__ C, float* __restrict__ ovf_thr,
    const float* __restrict__ xn, int* __restrict__ labels, float* __restrict__ mind,
    long long* __restrict__ ovf_rows, int* __restrict__ ovf_count, double* __restrict__ inertia,
    long long n, int k, int k_pad, float delta, RngKey key, long long row_offset, int ovf_cap,
    int idx_bits, int dbg) {
  (void)k;
  constexpr int NW = 4;
  constexpr int KS = KSD + 1;
  constexpr int DX = KSD * 16;
  constexpr int CPR = KS * 2;
  constexpr int TILE_BYTES = kBN * CPR * 16;
  constexpr int PIECES = TILE_BYTES / 1024;
  constexpr int ROWS = NW * 64;
  constexpr int PF = SQ_ESTEP_PF + 1;    // B prefetch distance (k-steps)
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  auto buf = [&](int g) -> unsigned char* { return smem + (g & 1) * TILE_BYTES; };

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r32 = lane & 31;
  const int half = lane >> 5;
  const uint32_t keep = ~((1u << idx_bits) - 1u);
  const int n_tiles = k_pad / kBN;
  const long long nblk = (n + ROWS - 1) / ROWS;
  long long blk = blockIdx.x;
  if (blk >= nblk) return;
  (void)dbg;

  auto stage = [&](int G) {
    const int t = (int)(G % n_tiles);
    const unsigned char* tile = reinterpret_cast<const unsigned char*>(C) + (size_t)t * TILE_BYTES;
    unsigned char* dst = buf(G);
    if ((SQ_ESTEP_ABLATE & 2) && G > 1) return;
    for (int p = wave; p < PIECES; p += NW) {
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(tile + p * 1024 + lane * 16),
          (__attribute__((address_space(3))) void*)(dst + p * 1024), 16, 0, 0);
    }
  };

  bf16x8 a0[KSD], a1[KSD];
  auto load_a = [&](long long b) {
    const long long r = b * ROWS + wave * 64 + r32;
    const uint16_t* x0 = X + (size_t)(r < n ? r : n - 1) * DX + half * 8;
    const uint16_t* x1 = X + (size_t)(r + 32 < n ? r + 32 : n - 1) * DX + half * 8;
#pragma unroll
    for (int ks = 0; ks < KSD; ++ks) {
      a0[ks] = *reinterpret_cast<const bf16x8*>(x0 + ks * 16);
      a1[ks] = *reinterpret_cast<const bf16x8*>(x1 + ks * 16);
    }
  };
  bf16x8 aug = (bf16x8)0;
  if (half == 0) { aug[0] = aug[1] = aug[2] = (short)0x3f80; }

  float m1[2][16], m2[2][16];
  const int lane_off = (half * 64 + r32) * 16;
  auto ldb = [&](const unsigned char* cur, int nb, int ks) -> bf16x8 {
    return *reinterpret_cast<const bf16x8*>(cur + lane_off + ks * 2048 + nb * 512);
  };
  auto tile_step = [&](const unsigned char* cur, Acc4& nacc, bool do_mfma, const Acc4& oacc,
                       int t_prev, bool do_epi) {
    const uint32_t j0 = (uint32_t)(t_prev * kBN + r32);
    const uint32_t j1 = j0 + 32;
    const bool epi = do_epi && !(SQ_ESTEP_ABLATE & 4);
    auto epi_row = [&](int q) {   // q = rb * 16 + i
      const int rb = q >> 4, i = q & 15;
      float p0 = packf(oacc.v[rb][0][i], keep, j0);
      float p1 = packf(oacc.v[rb][1][i], keep, j1);
      float q1 = m1[rb][i];
      float q2 = m2[rb][i];
      q2 = med3_raw(q1, p0, q2);
      q1 = min_raw(q1, p0);
      q2 = med3_raw(q1, p1, q2);
      q1 = min_raw(q1, p1);
      m1[rb][i] = q1;
      m2[rb][i] = q2;
    };
    if (do_mfma) {
#pragma unroll
      for (int rb = 0; rb < 2; ++rb)
#pragma unroll
        for (int nb = 0; nb < 2; ++nb) nacc.v[rb][nb] = (f32x16){0};
      bf16x8 b0[PF + 1], b1[PF + 1];
#pragma unroll
      for (int q = 0; q < PF && q < KS; ++q) { b0[q] = ldb(cur, 0, q); b1[q] = ldb(cur, 1, q); }
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        if (ks + PF < KS) {
          b0[(ks + PF) % (PF + 1)] = ldb(cur, 0, ks + PF);
          b1[(ks + PF) % (PF + 1)] = ldb(cur, 1, ks + PF);
        }
        const bf16x8 A0 = ks < KSD ? a0[ks] : aug;
        const bf16x8 A1 = ks < KSD ? a1[ks] : aug;
        const bf16x8 B0 = b0[ks % (PF + 1)], B1 = b1[ks % (PF + 1)];
        nacc.v[0][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A0, B0, nacc.v[0][0], 0, 0, 0);
        nacc.v[1][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A1, B0, nacc.v[1][0], 0, 0, 0);
        nacc.v[0][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A0, B1, nacc.v[0][1], 0, 0, 0);
        nacc.v[1][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A1, B1, nacc.v[1][1], 0, 0, 0);
        if (epi) {
#pragma unroll
          for (int q = (ks * 32) / KS; q < ((ks + 1) * 32) / KS; ++q) epi_row(q);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    } else if (epi) {
#pragma unroll
      for (int q = 0; q < 32; ++q) epi_row(q);
    }
  };
  auto sync_tile = [&]() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  };
  auto merge2 = [](float& x1, float& x2, float y1, float y2) {
    float lo2 = min_raw(x2, y2);
    x2 = med3_raw(x1, y1, lo2);
    x1 = min_raw(x1, y1);
  };

  int G = 0;
  stage(0);
  load_a(blk);
  sync_tile();
  double my_inertia = 0.0;

  for (; blk < nblk; blk += gridDim.x) {
    const long long row0 = blk * ROWS + wave * 64;
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int i = 0; i < 16; ++i) { m1[rb][i] = __builtin_inff(); m2[rb][i] = __builtin_inff(); }
    Acc4 pA, pB;
    stage(G + 1);
    tile_step(buf(G), pA, true, pA, 0, false);
    sync_tile();
    int t = 0;
    while (true) {
      if (t + 1 >= n_tiles) {
        load_a(blk + gridDim.x);
        tile_step(smem, pB, false, pA, t, true);
        break;
      }
      stage(G + 2);
      tile_step(buf(G + 1), pB, true, pA, t, true);
      sync_tile();
      ++t;
      ++G;
      if (t + 1 >= n_tiles) {
        load_a(blk + gridDim.x);
        tile_step(smem, pA, false, pB, t, true);
        break;
      }
      stage(G + 2);
      tile_step(buf(G + 1), pA, true, pB, t, true);
      sync_tile();
      ++t;
      ++G;
    }
    ++G;

#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
      const long long rowb = row0 + rb * 32;
      float R1[16], R2[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) { R1[i] = m1[rb][i]; R2[i] = m2[rb][i]; }
#pragma unroll
      for (int o = 16, c = 8; o >= 2; o >>= 1, c >>= 1) {
        const bool hi = (r32 & o) != 0;
#pragma unroll
        for (int j = 0; j < c; ++j) {
          float s1 = hi ? R1[j] : R1[c + j], s2 = hi ? R2[j] : R2[c + j];
          float k1 = hi ? R1[c + j] : R1[j], k2 = hi ? R2[c + j] : R2[j];
          float t1 = __shfl_xor(s1, o, 64), t2 = __shfl_xor(s2, o, 64);
          merge2(k1, k2, t1, t2);
          R1[j] = k1;
          R2[j] = k2;
        }
      }
      float q1 = R1[0], q2 = R2[0];
      merge2(q1, q2, __shfl_xor(R1[0], 1, 64), __shfl_xor(R2[0], 1, 64));
      const int irow = r32 >> 1;
      const int rloc = (irow & 3) + 8 * (irow >> 2) + 4 * half;
      const long long grow_local = rowb + rloc;
      const bool owner = ((r32 & 1) == 0) && grow_local < n;
      const float mval = valf(q1, keep);
      const float thr = mval + delta;
      const bool band2 = valf(q2, keep) <= thr;
      if (owner) {
        const float dist = fmaxf(xn[grow_local] + mval, 0.0f);
        mind[grow_local] = dist;
        if (!band2) labels[grow_local] = (int)(__float_as_uint(q1) & ~keep);
        my_inertia += (double)dist;
      }
      const unsigned long long slow = __ballot(owner && band2);
      if (slow && !SQ_ESTEP_ABLATE) {
        const float urow = band_u(key, row_offset + grow_local);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const unsigned long long sel = slow & ((1ull << (2 * i)) | (1ull << (32 + 2 * i)));
          if (!sel) continue;
          const int src = 32 * half + 2 * i;
          const bool mine = (slow >> src) & 1ull;
          const float thr_i = __shfl(thr, src, 64);
          const float u_i = __shfl(urow, src, 64);
          const bool v1 = mine && valf(m1[rb][i], keep) <= thr_i;
          const bool v2 = mine && valf(m2[rb][i], keep) <= thr_i;
          const uint32_t hb1 = (uint32_t)(__ballot(v1) >> (32 * half));
          const uint32_t hb2 = (uint32_t)(__ballot(v2) >> (32 * half));
          const int c = __popc(hb1);
          const int pick = hb2 == 0u && c > 0 ? nth_set_bit(hb1, band_rank(u_i, c)) : 0;
          const uint32_t jsel = (uint32_t)__shfl((int)(__float_as_uint(m1[rb][i]) & ~keep),
                                                 32 * half + pick, 64);
          if (mine && r32 == 2 * i) {
            const long long g = rowb + (i & 3) + 8 * (i >> 2) + 4 * half;
            if (hb2 != 0u) {
              int slot = atomicAdd(ovf_count, 1);
              if (slot < ovf_cap) { ovf_rows[slot] = g; ovf_thr[slot] = thr_i; }
              labels[g] = -1;
            } else {
              labels[g] = (int)jsel;
            }
          }
        }
      }
    }
  }
  my_inertia = wave_sum(my_inertia);
  if (lane == 0) inertia[(size_t)blockIdx.x * NW + wave] = my_inertia;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ---------------------------------------------------------------------------
// band_select: rows of full fp32 distances D[m][ldD] (first k valid).  One wave
// per row.  Exact: min, band {D <= min + delta}, member of rank floor(u c)
// in kappa order (band_pick_wave).
// If xn != nullptr the D rows hold ||c||^2 - 2x.c and xn is added.
__global__ void __launch_bounds__(256) band_select_kernel(
    const float* __restrict__ D, const long long* __restrict__ rows, const float* __restrict__ xn,
    int* __restrict__ labels, float* __restrict__ mind, long long m, int k, long long ldD,
    float delta, RngKey key, long long row_offset, int idx_bits) {
  const int lane = threadIdx.x & 63;
  const long long r = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= m) return;
  const float* d = D + r * ldD;
  float mn = __builtin_inff();
  for (int j = lane; j < k; j += 64) mn = fminf(mn, d[j]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mn = fminf(mn, __shfl_xor(mn, o, 64));
  const long long grow = rows ? rows[r] : r;
  const float thr = mn + delta;
  (void)idx_bits;
  auto dist = [&](int j) -> float { return d[j]; };
  const uint32_t win =
      (uint32_t)band_pick_wave(dist, k, thr, band_u(key, row_offset + grow), lane);
  if (lane == 0) {
    labels[grow] = (int)win;
    float base = xn ? xn[grow] : 0.0f;
    mind[grow] = fmaxf(base + mn, 0.0f);
  }
}


// ---------------------------------------------------------------------------
// band_select_rows: fallback for rows the fused kernel flagged (a lane held
// two band members).  Driven by the device-side count, so no host sync: the
// grid covers min(list capacity, 2048) workgroups and surplus ones exit.
// One 256-thread workgroup per row: every thread computes k/256 distances
// from the bf16 operands (x broadcast from LDS, centroid chunks coalesced
// across threads, 4 independent accumulators per distance), the k distances
// are staged in LDS, and wave 0 runs the exact band pick on them.  Distances
// are computed once, so the count and pick passes see the same values.
constexpr int kRowsMaxK = 4096;
__global__ void __launch_bounds__(256) band_select_rows_kernel(
    const uint16_t* __restrict__ X, const uint16_t* __restrict__ C,
    const float* __restrict__ thr_list, const long long* __restrict__ rows,
    const int* __restrict__ count, int* __restrict__ labels, long long cap, int d_pad, int k,
    float delta, RngKey key, long long row_offset) {
  __shared__ float xs[256];
  __shared__ float ds[kRowsMaxK];
  const int tid = threadIdx.x, lane = tid & 63;
  const long long cnt = min((long long)*count, cap);
  const int nch = d_pad / 8;
  const int cpr = nch + 2;   // chunk-major operand (see estep_kernel)
  for (long long slot = blockIdx.x; slot < cnt; slot += gridDim.x) {
    const long long r = rows[slot];
    __syncthreads();
    if (tid < d_pad) xs[tid] = bf16_to_f32(X[(size_t)r * d_pad + tid]);
    __syncthreads();
    // D'(j) = ||c_j||^2 - 2 x.c_j
    for (int j = tid; j < k; j += 256) {
      const uint16_t* base = C + ((size_t)(j >> 6) * cpr * 64 + (j & 63)) * 8;
      float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
#pragma unroll 4
      for (int ch = 0; ch < nch; ++ch) {
        const uint4 v = *reinterpret_cast<const uint4*>(base + (size_t)ch * 512);
        const float* xv = &xs[ch * 8];
        a0 = fmaf(xv[0], __uint_as_float(v.x << 16), a0);
        a1 = fmaf(xv[1], __uint_as_float(v.x & 0xFFFF0000u), a1);
        a2 = fmaf(xv[2], __uint_as_float(v.y << 16), a2);
        a3 = fmaf(xv[3], __uint_as_float(v.y & 0xFFFF0000u), a3);
        a0 = fmaf(xv[4], __uint_as_float(v.z << 16), a0);
        a1 = fmaf(xv[5], __uint_as_float(v.z & 0xFFFF0000u), a1);
        a2 = fmaf(xv[6], __uint_as_float(v.w << 16), a2);
        a3 = fmaf(xv[7], __uint_as_float(v.w & 0xFFFF0000u), a3);
      }
      const uint32_t nv = *reinterpret_cast<const uint32_t*>(base + (size_t)nch * 512);
      ds[j] = ((a0 + a1) + (a2 + a3)) + (__uint_as_float(nv << 16) +
                                         __uint_as_float(nv & 0xFFFF0000u));
    }
    __syncthreads();
    if (tid < 64) {
      auto dist = [&](int j) -> float { return ds[j]; };
      // threshold from the fused kernel (its MFMA min + delta); if rounding of
      // this recomputation leaves the band empty, use our own min
      float thr = thr_list[slot];
      const float u = band_u(key, row_offset + r);
      int win = band_pick_wave(dist, k, thr, u, lane);
      if (win < 0) {
        float mn = __builtin_inff();
        for (int j = lane; j < k; j += 64) mn = fminf(mn, ds[j]);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) mn = fminf(mn, __shfl_xor(mn, o, 64));
        thr = mn + delta;
        win = band_pick_wave(dist, k, thr, u, lane);
      }
      if (lane == 0) labels[r] = win;
    }
  }
}

// ---------------------------------------------------------------------------
// centroid_accumulate: chunk of CH rows per workgroup (256 threads).
template <typename T>
SQ_DEV float4 load4(const T* p);
template <>
SQ_DEV float4 load4<float>(const float* p) { return *reinterpret_cast<const float4*>(p); }
template <>
SQ_DEV float4 load4<uint16_t>(const uint16_t* p) {
  uint2 v = *reinterpret_cast<const uint2*>(p);
  return make_float4(__uint_as_float(v.x << 16), __uint_as_float(v.x & 0xFFFF0000u),
                     __uint_as_float(v.y << 16), __uint_as_float(v.y & 0xFFFF0000u));
}

template <typename T>
__global__ void __launch_bounds__(256) centroid_accumulate_kernel(
    const T* __restrict__ X, const int* __restrict__ labels, const float* __restrict__ w,
    float* __restrict__ sums, double* __restrict__ counts, long long n, int d, int k, int CH) {
  extern __shared__ __attribute__((aligned(16))) int sm[];
  int* hist = sm;            // k
  int* cursor = sm + k;      // k
  int* perm = sm + 2 * k;    // CH
  const int tid = threadIdx.x;
  const long long r0 = (long long)blockIdx.x * CH;
  const int rows = (int)min((long long)CH, n - r0);
  for (int j = tid; j < k; j += 256) hist[j] = 0;
  __syncthreads();
  for (int i = tid; i < rows; i += 256) {
    int l = labels[r0 + i];
    if (l >= 0 && l < k) atomicAdd(&hist[l], 1);
  }
  __syncthreads();
  // exclusive scan of hist -> cursor (single wave, k/64 per lane)
  if (tid < 64) {
    int per = (k + 63) / 64;
    int b = tid * per, e = min(b + per, k);
    int s = 0;
    for (int j = b; j < e; ++j) s += hist[j];
    int incl = s;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      int v = __shfl_up(incl, o, 64);
      if (tid >= o) incl += v;
    }
    int run = incl - s;
    for (int j = b; j < e; ++j) { cursor[j] = run; run += hist[j]; }
  }
  __syncthreads();
  for (int i = tid; i < rows; i += 256) {
    int l = labels[r0 + i];
    if (l >= 0 && l < k) {
      int pos = atomicAdd(&cursor[l], 1);
      perm[pos] = i;
    }
  }
  __syncthreads();
  // cursor[l] now = end of segment l; start = end - hist[l]
  const int wave = tid >> 6, lane = tid & 63;
  for (int l = wave; l < k; l += 4) {
    int cnt = hist[l];
    if (cnt == 0) continue;
    int end = cursor[l], beg = end - cnt;
    for (int c0 = lane * 4; c0 < d; c0 += 256) {
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int p = beg; p < end; ++p) {
        long long r = r0 + perm[p];
        float4 v = load4<T>(X + (size_t)r * d + c0);
        float ww = w ? w[r] : 1.0f;
        acc.x += ww * v.x; acc.y += ww * v.y; acc.z += ww * v.z; acc.w += ww * v.w;
      }
      float* dst = sums + (size_t)l * d + c0;
      atomicAdd(dst + 0, acc.x);
      if (c0 + 1 < d) atomicAdd(dst + 1, acc.y);
      if (c0 + 2 < d) atomicAdd(dst + 2, acc.z);
      if (c0 + 3 < d) atomicAdd(dst + 3, acc.w);
    }
    if (lane == 0) {
      double wsum = 0.0;
      if (w) { for (int p = beg; p < end; ++p) wsum += (double)w[r0 + perm[p]]; }
      else wsum = (double)cnt;
      atomicAdd(&counts[l], wsum);
    }
  }
}


// ---------------------------------------------------------------------------
// centroid reduction by global counting sort (replaces per-chunk LDS sorting):
//   label_hist   : LDS histogram per chunk -> one global int atomic per label
//   label_scan   : exclusive scan (one workgroup)
//   label_scatter: per-chunk LDS ranks + one global cursor atomic per label
//   segment_sum  : each workgroup owns a contiguous range of the label-sorted
//                  permutation; each wave sums its rows (4 row loads in flight)
//                  and flushes one 256-B f32 atomic row-add per label run.
constexpr int kHistChunk = 8192;

// Also zeroes the reduce outputs (sums: nz1 doubles, counts: nz2) grid-stride,
// so the segmented sums that follow need no separate memset launches.
__global__ void __launch_bounds__(256) label_hist_kernel(const int* __restrict__ labels, long long n,
                                                         int k, int* __restrict__ hist,
                                                         double* __restrict__ z1, long long nz1,
                                                         double* __restrict__ z2, int nz2) {
  extern __shared__ __attribute__((aligned(16))) int lh[];
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < nz1;
       i += (long long)gridDim.x * 256)
    z1[i] = 0.0;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < nz2;
       i += (long long)gridDim.x * 256)
    z2[i] = 0.0;
  for (int j = threadIdx.x; j < k; j += 256) lh[j] = 0;
  __syncthreads();
  const long long r0 = (long long)blockIdx.x * kHistChunk;
  const long long r1 = min(n, r0 + kHistChunk);
  for (long long r = r0 + threadIdx.x; r < r1; r += 256) {
    int l = labels[r];
    if (l >= 0 && l < k) atomicAdd(&lh[l], 1);
  }
  __syncthreads();
  for (int j = threadIdx.x; j < k; j += 256)
    if (lh[j]) atomicAdd(&hist[j], lh[j]);
}

// Exclusive scan of the histogram into the scatter cursors; the histogram is
// zeroed after use (it is only consumed here), ready for the next reduce.
__global__ void __launch_bounds__(1024) label_scan_kernel(int* __restrict__ hist, int k,
                                                          int* __restrict__ cursor) {
  __shared__ int part[1024];
  const int t = threadIdx.x;
  const int per = (k + 1023) / 1024;
  const int b = t * per, e = min(b + per, k);
  int s = 0;
  for (int j = b; j < e; ++j) s += hist[j];
  part[t] = s;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    int v = t >= o ? part[t - o] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  int run = part[t] - s;
  for (int j = b; j < e; ++j) { cursor[j] = run; run += hist[j]; hist[j] = 0; }
}

__global__ void __launch_bounds__(256) label_scatter_kernel(const int* __restrict__ labels,
                                                            long long n, int k,
                                                            int* __restrict__ cursor,
                                                            int* __restrict__ perm) {
  extern __shared__ __attribute__((aligned(16))) int sm2[];
  int* lh = sm2;        // k: local counts, then local cursors
  int* base = sm2 + k;  // k
  for (int j = threadIdx.x; j < k; j += 256) lh[j] = 0;
  __syncthreads();
  const long long r0 = (long long)blockIdx.x * kHistChunk;
  const long long r1 = min(n, r0 + kHistChunk);
  for (long long r = r0 + threadIdx.x; r < r1; r += 256) {
    int l = labels[r];
    if (l >= 0 && l < k) atomicAdd(&lh[l], 1);
  }
  __syncthreads();
  for (int j = threadIdx.x; j < k; j += 256) {
    int c = lh[j];
    base[j] = c ? atomicAdd(&cursor[j], c) : 0;
    lh[j] = 0;
  }
  __syncthreads();
  for (long long r = r0 + threadIdx.x; r < r1; r += 256) {
    int l = labels[r];
    if (l >= 0 && l < k) {
      int pos = base[l] + atomicAdd(&lh[l], 1);
      perm[pos] = (int)r;
    }
  }
}

#ifndef SQ_SEG_U
#define SQ_SEG_U 4   // rows in flight per wave (perm -> label/row gathers)
#endif
// ---------------------------------------------------------------------------
// Incremental M-step (the rows are the same every Lloyd iteration, only the
// labels move): the fixed-point cluster statistics
//   S_c = sum q(x_i),  n_c = |{i}|,  Q_c = sum q2(|x_i|^2)     (i: label c)
// are exact integers in fp64 (see the quantisation note above), so
//   S(t+1) = S(t) + sum_{i moved into c} q(x_i) - sum_{i moved out} q(x_i)
// is bit-identical to summing the new members from scratch, in any order.
// Only the moved rows are read: a signed entry list (row << 1 | out) is
// counting-sorted by the label it updates (new label for "in", previous for
// "out") and summed with the same run-length flushes as segment_sum_rows.
// prev < 0 marks "no previous label" (first iteration / after a reset:
// every row enters).  Q feeds the per-cluster inertia (cluster_inertia).
__global__ void __launch_bounds__(256) delta_hist_kernel(const int* __restrict__ labels,
                                                         const int* __restrict__ prev,
                                                         long long n, int k,
                                                         int* __restrict__ hist) {
  extern __shared__ __attribute__((aligned(16))) int dh[];
  for (int j = threadIdx.x; j < k; j += 256) dh[j] = 0;
  __syncthreads();
  const long long r0 = (long long)blockIdx.x * kHistChunk;
  const long long r1 = min(n, r0 + kHistChunk);
  auto one = [&](int l, int p) {
    if (l == p) return;
    if (l >= 0 && l < k) atomicAdd(&dh[l], 1);
    if (p >= 0 && p < k) atomicAdd(&dh[p], 1);
  };
  // 4 rows per load (chunk starts are multiples of 4: int4-aligned)
  for (long long r = r0 + 4 * threadIdx.x; r < r1; r += 1024) {
    if (r + 4 <= r1) {
      const int4 l4 = *reinterpret_cast<const int4*>(labels + r);
      const int4 p4 = *reinterpret_cast<const int4*>(prev + r);
      one(l4.x, p4.x); one(l4.y, p4.y); one(l4.z, p4.z); one(l4.w, p4.w);
    } else {
      for (long long q = r; q < r1; ++q) one(labels[q], prev[q]);
    }
  }
  __syncthreads();
  for (int j = threadIdx.x; j < k; j += 256)
    if (dh[j]) atomicAdd(&hist[j], dh[j]);
}

// Entries carry their label (int2: row, label | out << 30), so the segment
// pass never gathers labels / prev; the place pass also moves prev to the
// new labels (only this thread reads these rows' prev, and only before), so
// no separate prev <- labels copy follows the M-step.
__global__ void __launch_bounds__(256) delta_scatter_kernel(const int* __restrict__ labels,
                                                            int* __restrict__ prev,
                                                            long long n, int k,
                                                            int* __restrict__ cursor,
                                                            int2* __restrict__ perm) {
  extern __shared__ __attribute__((aligned(16))) int ds2[];
  int* lh = ds2;
  int* base = ds2 + k;
  for (int j = threadIdx.x; j < k; j += 256) lh[j] = 0;
  __syncthreads();
  const long long r0 = (long long)blockIdx.x * kHistChunk;
  const long long r1 = min(n, r0 + kHistChunk);
  auto count = [&](int l, int p) {
    if (l == p) return;
    if (l >= 0 && l < k) atomicAdd(&lh[l], 1);
    if (p >= 0 && p < k) atomicAdd(&lh[p], 1);
  };
  auto place = [&](long long r, int l, int p) {
    if (l == p) return;
    if (l >= 0 && l < k) perm[base[l] + atomicAdd(&lh[l], 1)] = make_int2((int)r, l);
    if (p >= 0 && p < k) perm[base[p] + atomicAdd(&lh[p], 1)] = make_int2((int)r, p | (1 << 30));
  };
  for (long long r = r0 + 4 * threadIdx.x; r < r1; r += 1024) {
    if (r + 4 <= r1) {
      const int4 l4 = *reinterpret_cast<const int4*>(labels + r);
      const int4 p4 = *reinterpret_cast<const int4*>(prev + r);
      count(l4.x, p4.x); count(l4.y, p4.y); count(l4.z, p4.z); count(l4.w, p4.w);
    } else {
      for (long long q = r; q < r1; ++q) count(labels[q], prev[q]);
    }
  }
  __syncthreads();
  for (int j = threadIdx.x; j < k; j += 256) {
    const int c = lh[j];
    base[j] = c ? atomicAdd(&cursor[j], c) : 0;
    lh[j] = 0;
  }
  __syncthreads();
  for (long long r = r0 + 4 * threadIdx.x; r < r1; r += 1024) {
    if (r + 4 <= r1) {
      const int4 l4 = *reinterpret_cast<const int4*>(labels + r);
      const int4 p4 = *reinterpret_cast<const int4*>(prev + r);
      place(r, l4.x, p4.x); place(r + 1, l4.y, p4.y);
      place(r + 2, l4.z, p4.z); place(r + 3, l4.w, p4.w);
      if (l4.x != p4.x || l4.y != p4.y || l4.z != p4.z || l4.w != p4.w)
        *reinterpret_cast<int4*>(prev + r) = l4;
    } else {
      for (long long q = r; q < r1; ++q) {
        const int l = labels[q], p = prev[q];
        place(q, l, p);
        if (l != p) prev[q] = l;
      }
    }
  }
}

// List form of delta_hist / delta_scatter: after a FILTERED E-step only the
// rows on its three disjoint row lists can carry a new label (the rows the
// Hamerly bounds could not prune, the pruned multi-candidate rows re-checked
// without a record, the rows of list B); every other row kept its label and
// prev == labels there.  The two passes walk just those rows (the
// concatenation of the lists, lengths on the device) instead of all n - the
// same entries, so the same statistics (exact integer arithmetic: any
// order).  Grid-stride, kDL entries in flight per thread (row -> label /
// prev are dependent gathers).
struct RowLists {
  const long long* L[3];
  const int* c[3];
};
constexpr int kDL = 8;
struct RowListWalk {
  long long c0, c01, total;
  const RowLists& R;
  SQ_DEV RowListWalk(const RowLists& r, long long n) : R(r) {
    const long long a = R.L[0] ? min((long long)*R.c[0], n) : 0;
    const long long b = R.L[1] ? min((long long)*R.c[1], n) : 0;
    const long long c = R.L[2] ? min((long long)*R.c[2], n) : 0;
    c0 = a;
    c01 = a + b;
    total = a + b + c;
  }
  SQ_DEV long long row(long long e) const {
    return e < c0 ? R.L[0][e] : (e < c01 ? R.L[1][e - c0] : R.L[2][e - c01]);
  }
};

__global__ void __launch_bounds__(256) delta_hist_list_kernel(const int* __restrict__ labels,
                                                              const int* __restrict__ prev,
                                                              RowLists R, long long n, int k,
                                                              int* __restrict__ hist) {
  extern __shared__ __attribute__((aligned(16))) int dl[];
  for (int j = threadIdx.x; j < k; j += 256) dl[j] = 0;
  __syncthreads();
  const RowListWalk W(R, n);
  const long long stride = (long long)gridDim.x * 256;
  for (long long e0 = (long long)blockIdx.x * 256 + threadIdx.x; e0 < W.total; e0 += kDL * stride) {
    long long r[kDL];
    int l[kDL], p[kDL];
#pragma unroll
    for (int u = 0; u < kDL; ++u) {
      const long long e = e0 + u * stride;
      r[u] = e < W.total ? W.row(e) : -1;
    }
#pragma unroll
    for (int u = 0; u < kDL; ++u) {
      l[u] = r[u] >= 0 ? labels[r[u]] : 0;
      p[u] = r[u] >= 0 ? prev[r[u]] : 0;
    }
#pragma unroll
    for (int u = 0; u < kDL; ++u) {
      if (r[u] < 0 || l[u] == p[u]) continue;
      if (l[u] >= 0 && l[u] < k) atomicAdd(&dl[l[u]], 1);
      if (p[u] >= 0 && p[u] < k) atomicAdd(&dl[p[u]], 1);
    }
  }
  __syncthreads();
  for (int j = threadIdx.x; j < k; j += 256)
    if (dl[j]) atomicAdd(&hist[j], dl[j]);
}

__global__ void __launch_bounds__(256) delta_scatter_list_kernel(const int* __restrict__ labels,
                                                                 int* __restrict__ prev,
                                                                 RowLists R, long long n, int k,
                                                                 int* __restrict__ cursor,
                                                                 int2* __restrict__ perm) {
  extern __shared__ __attribute__((aligned(16))) int dls[];
  int* lh = dls;
  int* base = dls + k;
  for (int j = threadIdx.x; j < k; j += 256) lh[j] = 0;
  __syncthreads();
  const RowListWalk W(R, n);
  const long long stride = (long long)gridDim.x * 256;
  // pass 1 counts this block's entries per label, pass 2 places them (the
  // same entries: the lists do not change in between)
  for (int pass = 0; pass < 2; ++pass) {
    for (long long e0 = (long long)blockIdx.x * 256 + threadIdx.x; e0 < W.total;
         e0 += kDL * stride) {
      long long r[kDL];
      int l[kDL], p[kDL];
#pragma unroll
      for (int u = 0; u < kDL; ++u) {
        const long long e = e0 + u * stride;
        r[u] = e < W.total ? W.row(e) : -1;
      }
#pragma unroll
      for (int u = 0; u < kDL; ++u) {
        l[u] = r[u] >= 0 ? labels[r[u]] : 0;
        p[u] = r[u] >= 0 ? prev[r[u]] : 0;
      }
#pragma unroll
      for (int u = 0; u < kDL; ++u) {
        if (r[u] < 0 || l[u] == p[u]) continue;
        const bool li = l[u] >= 0 && l[u] < k, pi = p[u] >= 0 && p[u] < k;
        if (pass == 0) {
          if (li) atomicAdd(&lh[l[u]], 1);
          if (pi) atomicAdd(&lh[p[u]], 1);
        } else {
          if (li) perm[base[l[u]] + atomicAdd(&lh[l[u]], 1)] = make_int2((int)r[u], l[u]);
          if (pi)
            perm[base[p[u]] + atomicAdd(&lh[p[u]], 1)] = make_int2((int)r[u], p[u] | (1 << 30));
          prev[r[u]] = l[u];
        }
      }
    }
    __syncthreads();
    if (pass == 0) {
      for (int j = threadIdx.x; j < k; j += 256) {
        const int c = lh[j];
        base[j] = c ? atomicAdd(&cursor[j], c) : 0;
        lh[j] = 0;
      }
      __syncthreads();
    }
  }
}

// one wave per entry (4 fp32 values per lane per 256-column chunk), U entries in
// flight per wave; the entry count is the scanned total (cursor[k-1]).
// Each wave takes a run of max(SQ_DSEG_RUN, total / SQ_DSEG_WAVES) entries:
// long runs keep the fp64 flush atomics few (many moved rows), short ones
// keep the serial gather chain (perm -> label / row) of a few-moved-rows step
// short (measured: 64-entry minimum 78 us/step on a 1.25M-row shard, 16 ->
// 52 us; a fixed 16 costs 27 us at 10M rows through the extra flushes).
#ifndef SQ_DSEG_U
#define SQ_DSEG_U 8
#endif
#ifndef SQ_DSEG_RUN
#define SQ_DSEG_RUN 16
#endif
#ifndef SQ_DSEG_WAVES
#define SQ_DSEG_WAVES 2048
#endif
// M = ceil(d / 256) column chunks of 256 features per lane pass (d <= 1024):
// lane covers features 4 lane + 256 m, m < M, of every entry it streams.
template <int M>
__global__ void __launch_bounds__(512) delta_segment_kernel(
    const float* __restrict__ X, const int2* __restrict__ perm, int d, int range, float xscale,
    double qscale, double* __restrict__ sums, double* __restrict__ counts,
    double* __restrict__ qsum, const int* __restrict__ valid_end) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  // range <= 0: the entry count (on the device) is split evenly over the
  // grid - a few moved rows still keep every block busy
  const long long total = *valid_end;
  constexpr int U = M == 1 ? SQ_DSEG_U : (M == 2 ? 4 : 2);
  // range > 0: a block takes `range` entries, its 8 waves interleaved;
  // range <= 0: each wave takes a CONTIGUOUS run of >= 64 entries (runs of
  // one label stay in one wave: few flushes, few fp64 atomics)
  long long p0, p1, pstep, ustep;
  if (range > 0) {
    p0 = (long long)blockIdx.x * range + wave;
    p1 = min(total, (long long)blockIdx.x * range + range);
    pstep = 8LL * U;
    ustep = 8;
  } else {
    // 2048 waves at most while the runs are short (few moved rows: few
    // flushes); a long list (a first iteration: every row enters) spreads
    // over the whole grid in runs of >= 512 entries - 2048 waves alone leave
    // two waves per SIMD on a serial perm -> row gather chain (3.8 ms for
    // the 10M-row first iteration)
    const long long waves = min((long long)gridDim.x * 8,
                                max((long long)SQ_DSEG_WAVES, total / 512));
    const long long rw = max((long long)SQ_DSEG_RUN, (total + waves - 1) / waves);
    p0 = ((long long)blockIdx.x * 8 + wave) * rw;
    p1 = min(total, p0 + rw);
    pstep = U;
    ustep = 1;
  }
  double a[M][4], aq = 0.0, cnt = 0.0;
#pragma unroll
  for (int m = 0; m < M; ++m) a[m][0] = a[m][1] = a[m][2] = a[m][3] = 0.0;
  int cur = -1;
  auto flush = [&]() {
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const int c0 = lane * 4 + 256 * m;
      double* dst = sums + (size_t)cur * d + c0;
      if (c0 < d) {
        if (a[m][0] != 0.0) atomicAdd(dst + 0, a[m][0]);
        if (a[m][1] != 0.0 && c0 + 1 < d) atomicAdd(dst + 1, a[m][1]);
        if (a[m][2] != 0.0 && c0 + 2 < d) atomicAdd(dst + 2, a[m][2]);
        if (a[m][3] != 0.0 && c0 + 3 < d) atomicAdd(dst + 3, a[m][3]);
      }
    }
    const double q = wave_sum(aq);   // integer-valued: exact in any order
    if (lane == 0) {
      if (cnt != 0.0) atomicAdd(&counts[cur], cnt);
      if (q != 0.0) atomicAdd(&qsum[cur], q);
    }
  };
  // the next batch's entries are loaded while this batch's rows stream in:
  // one memory latency per batch, not the perm -> row chain of two
  int2 en[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long long q = p0 + ustep * u;
    en[u] = q < p1 ? perm[q] : make_int2(0, -1);
  }
  for (long long p = p0; p < p1; p += pstep) {
    int ll[U], out[U];
    float4 v[U][M];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int2 e = en[u];
      const int r = e.x;
      ll[u] = e.y < 0 ? -1 : (e.y & 0x3FFFFFFF);
      out[u] = (e.y >> 30) & 1;
#pragma unroll
      for (int m = 0; m < M; ++m) {
        const int c0 = lane * 4 + 256 * m;
        v[u][m] = (ll[u] >= 0 && c0 < d) ? *reinterpret_cast<const float4*>(X + (size_t)r * d + c0)
                                         : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long q = p + pstep + ustep * u;
      en[u] = q < p1 ? perm[q] : make_int2(0, -1);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (ll[u] < 0) continue;      // wave-uniform (one entry per wave)
      if (ll[u] != cur) {
        if (cur >= 0) flush();
        cur = ll[u];
#pragma unroll
        for (int m = 0; m < M; ++m) a[m][0] = a[m][1] = a[m][2] = a[m][3] = 0.0;
        aq = cnt = 0.0;
      }
      const double sg = out[u] ? -1.0 : 1.0;
#pragma unroll
      for (int m = 0; m < M; ++m) {
        const float4 x = v[u][m];
        a[m][0] += sg * (double)rintf(x.x * xscale);
        a[m][1] += sg * (double)rintf(x.y * xscale);
        a[m][2] += sg * (double)rintf(x.z * xscale);
        a[m][3] += sg * (double)rintf(x.w * xscale);
        const double x0 = x.x, x1 = x.y, x2 = x.z, x3 = x.w;   // squares exact in fp64
        aq += sg * (rint(x0 * x0 * qscale) + rint(x1 * x1 * qscale) + rint(x2 * x2 * qscale) +
                    rint(x3 * x3 * qscale));
      }
      cnt += sg;
    }
  }
  if (cur >= 0) flush();
}

// inertia part of cluster c at the E-step's centroids C (fp32 [k][d]):
//   sum_{i: label c} |x_i - c|^2 = Q_c - 2 c.S_c + n_c |c|^2
// from the fixed-point statistics (fp64; one wave per cluster).
__global__ void __launch_bounds__(256) cluster_inertia_kernel(
    const double* __restrict__ sums, const double* __restrict__ counts,
    const double* __restrict__ qsum, const float* __restrict__ C, int k, int d, double xunit,
    double qunit, double* __restrict__ part) {
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= k) return;
  double cs = 0.0, cc = 0.0;
  for (int f = lane; f < d; f += 64) {
    const double cf = (double)C[(size_t)c * d + f];
    cs = fma(cf, sums[(size_t)c * d + f], cs);
    cc = fma(cf, cf, cc);
  }
  cs = wave_sum(cs);
  cc = wave_sum(cc);
  if (lane == 0) part[c] = qsum[c] * qunit - 2.0 * cs * xunit + counts[c] * cc;
}

// Deterministic segmented sums: every contribution is quantised to an
// integer multiple of 2^qexp (x * 2^-qexp rounded in fp32: exact scaling by a
// power of two, then v_rndne) and accumulated in fp64.  The host picks qexp
// so that max|x| * n * 2^-qexp <= 2^52: every partial and total sum is then
// an integer below 2^53, exactly representable, so fp64 addition is exact
// and therefore associative - the result is independent of the (atomic,
// arbitrary) order of the permutation and the flushes.  A fit is thus
// bit-reproducible run to run and across checkpoint/resume, at a rounding
// of at most 2^qexp / 2 per element (~1e-7 absolute for |x| <= 100 at 10M
// rows, below bf16/fp32 input precision).
// Large-d variant (a row spans the whole wave: 4 values per lane, 8-B/16-B
// loads); measured faster than the chunked variant below at d = 256 bf16
// (1.55 vs 1.84 ms, 10M rows), slower at small d (1.21 vs 0.85 ms, d = 32).
#ifndef SQ_SEG_U
#define SQ_SEG_U 4   // rows in flight per wave (perm -> label/row gathers)
#endif
// With mind != null (fp32 data, d <= 256: one column pass) the rows whose
// E-step left mind < 0 (the certified filter's single-candidate rows) get
// their exact fp64 |x - c_label|^2 here, against the iteration's centroids
// Cold [k][d], while the row is in registers anyway.
template <typename T>
__global__ void __launch_bounds__(512) segment_sum_rows_kernel(
    const T* __restrict__ X, const int* __restrict__ perm, const int* __restrict__ labels,
    const float* __restrict__ w, long long n_sorted, int d, int range, float xscale,
    float wscale, double* __restrict__ sums, double* __restrict__ counts,
    const int* __restrict__ valid_end, float* __restrict__ mind, const float* __restrict__ Cold) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long long p0 = (long long)blockIdx.x * range;
  const long long p1 = min(min(n_sorted, (long long)*valid_end), p0 + range);
  constexpr int U = SQ_SEG_U;
  for (int c0 = lane * 4; c0 < d; c0 += 256) {
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0, cnt = 0.0;
    int cur = -1;
    float4 cold = make_float4(0.f, 0.f, 0.f, 0.f);
    auto flush = [&]() {
      double* dst = sums + (size_t)cur * d + c0;
      if (a0 != 0.0) atomicAdd(dst + 0, a0);
      if (a1 != 0.0 && c0 + 1 < d) atomicAdd(dst + 1, a1);
      if (a2 != 0.0 && c0 + 2 < d) atomicAdd(dst + 2, a2);
      if (a3 != 0.0 && c0 + 3 < d) atomicAdd(dst + 3, a3);
      if (lane == 0 && c0 == 0) atomicAdd(&counts[cur], cnt);
    };
    for (long long p = p0 + wave; p < p1; p += 8 * U) {
      int rr[U], ll[U];
      float4 v[U];
      float ww[U];
      float mk[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        long long q = p + 8LL * u;
        rr[u] = q < p1 ? perm[q] : -1;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        ll[u] = rr[u] >= 0 ? labels[rr[u]] : -1;
        v[u] = rr[u] >= 0 ? load4<T>(X + (size_t)rr[u] * d + c0) : make_float4(0.f, 0.f, 0.f, 0.f);
        ww[u] = (w && rr[u] >= 0) ? w[rr[u]] : 1.0f;
        mk[u] = (mind && rr[u] >= 0) ? mind[rr[u]] : 0.0f;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (ll[u] < 0) continue;
        if (ll[u] != cur) {
          if (cur >= 0) flush();
          cur = ll[u];
          a0 = a1 = a2 = a3 = cnt = 0.0;
          if (mind) cold = *reinterpret_cast<const float4*>(Cold + (size_t)cur * d + c0);
        }
        if (mk[u] < 0.0f) {   // wave-uniform (one row per wave)
          const double e0 = (double)v[u].x - (double)cold.x, e1 = (double)v[u].y - (double)cold.y;
          const double e2 = (double)v[u].z - (double)cold.z, e3 = (double)v[u].w - (double)cold.w;
          double ds = fma(e0, e0, fma(e1, e1, fma(e2, e2, e3 * e3)));
          ds = wave_sum(ds);
          if (lane == 0) mind[rr[u]] = (float)ds;
        }
        const float s = ww[u] * xscale;   // exact when unweighted (power of 2)
        a0 += (double)rintf(v[u].x * s);
        a1 += (double)rintf(v[u].y * s);
        a2 += (double)rintf(v[u].z * s);
        a3 += (double)rintf(v[u].w * s);
        cnt += w ? (double)rintf(ww[u] * wscale) : 1.0;
      }
    }
    if (cur >= 0) flush();
  }
}

// bf16 half-wave variant: 16-B loads (8 values per lane), a row spans 32
// lanes, so each wave instruction gathers two rows; every half-wave owns a
// contiguous slice of the workgroup's positions (fewer label runs touched,
// hence fewer flushes, than a strided split).
__global__ void __launch_bounds__(512) segment_sum_rows_half_kernel(
    const uint16_t* __restrict__ X, const int* __restrict__ perm, const int* __restrict__ labels,
    const float* __restrict__ w, long long n_sorted, int d, int range, float xscale,
    float wscale, double* __restrict__ sums, double* __restrict__ counts,
    const int* __restrict__ valid_end) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int hw = wave * 2 + (lane >> 5), hl = lane & 31;
  const long long pe = min(n_sorted, (long long)*valid_end);
  const int sub = range / 16;
  const long long s0 = (long long)blockIdx.x * range + (long long)hw * sub;
  const long long s1 = min(pe, s0 + sub);
  constexpr int U = SQ_SEG_U;
  for (int c0 = hl * 8; c0 < d; c0 += 256) {
    double a[8], cnt = 0.0;
#pragma unroll
    for (int e = 0; e < 8; ++e) a[e] = 0.0;
    int cur = -1;
    auto flush = [&]() {
      double* dst = sums + (size_t)cur * d + c0;
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (a[e] != 0.0 && c0 + e < d) atomicAdd(dst + e, a[e]);
      if (hl == 0 && c0 == 0) atomicAdd(&counts[cur], cnt);
    };
    for (long long p = s0; p < s1; p += U) {
      int rr[U], ll[U];
      uint4 v[U];
      float ww[U];
#pragma unroll
      for (int u = 0; u < U; ++u) rr[u] = p + u < s1 ? perm[p + u] : -1;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        ll[u] = rr[u] >= 0 ? labels[rr[u]] : -1;
        v[u] = rr[u] >= 0 && c0 < d ? *reinterpret_cast<const uint4*>(X + (size_t)rr[u] * d + c0)
                                    : make_uint4(0u, 0u, 0u, 0u);
        ww[u] = (w && rr[u] >= 0) ? w[rr[u]] : 1.0f;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (ll[u] < 0) continue;
        if (ll[u] != cur) {
          if (cur >= 0) flush();
          cur = ll[u];
#pragma unroll
          for (int e = 0; e < 8; ++e) a[e] = 0.0;
          cnt = 0.0;
        }
        const float s = ww[u] * xscale;   // exact when unweighted (power of 2)
        const uint32_t q[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          a[2 * e] += (double)rintf(__uint_as_float(q[e] << 16) * s);
          a[2 * e + 1] += (double)rintf(__uint_as_float(q[e] & 0xFFFF0000u) * s);
        }
        cnt += w ? (double)rintf(ww[u] * wscale) : 1.0;
      }
    }
    if (cur >= 0) flush();
  }
}

// 16-byte chunk loads: 8 bf16 or 4 fp32 values
template <typename T> struct Chunk16;
template <> struct Chunk16<uint16_t> {
  static constexpr int V = 8;
  SQ_DEV static void load(const uint16_t* p, float v[8]) {
    uint4 u = *reinterpret_cast<const uint4*>(p);
    uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[2 * e] = __uint_as_float(w[e] << 16);
      v[2 * e + 1] = __uint_as_float(w[e] & 0xFFFF0000u);
    }
  }
};
template <> struct Chunk16<float> {
  static constexpr int V = 4;
  SQ_DEV static void load(const float* p, float v[4]) {
    float4 a = *reinterpret_cast<const float4*>(p);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  }
};

// LPR lanes per row (one 16-B chunk each per step, CPL chunks per lane), so a
// wave is 64/LPR "virtual waves" walking their own label runs: full lanes for
// any d (d = 32 bf16 -> 4 lanes per row, 16 rows per wave), U rows in flight.
template <typename T, int LPR>
__global__ void __launch_bounds__(512) segment_sum_kernel(
    const T* __restrict__ X, const int* __restrict__ perm, const int* __restrict__ labels,
    const float* __restrict__ w, long long n_sorted, int d, int range, float xscale,
    float wscale, double* __restrict__ sums, double* __restrict__ counts,
    const int* __restrict__ valid_end) {
  constexpr int V = Chunk16<T>::V;
  constexpr int VW = 64 / LPR;                 // virtual waves per wave
  constexpr int U = 4;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int vl = lane % LPR;                   // chunk slot within the row
  const int vw = wave * VW + lane / LPR;       // virtual wave id in the WG (0 .. 8 VW - 1)
  const int CH = d / V;                        // 16-B chunks per row
  const long long p0 = (long long)blockIdx.x * range;
  const long long p1 = min(min(n_sorted, (long long)*valid_end), p0 + range);
  for (int c = vl; c < ((CH + LPR - 1) / LPR) * LPR; c += LPR) {
    const bool active = c < CH;
    const int c0 = c * V;
    double acc[V];
    double cnt = 0.0;
#pragma unroll
    for (int e = 0; e < V; ++e) acc[e] = 0.0;
    int cur = -1;
    auto flush = [&]() {
      if (active) {
        double* dst = sums + (size_t)cur * d + c0;
#pragma unroll
        for (int e = 0; e < V; ++e)
          if (acc[e] != 0.0) atomicAdd(dst + e, acc[e]);
      }
      if (c == 0 && vl == 0) atomicAdd(&counts[cur], cnt);
    };
    for (long long p = p0 + vw; p < p1; p += (long long)8 * VW * U) {
      int rr[U], ll[U];
      float ww[U];
      float v[U][V];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long long q = p + (long long)8 * VW * u;
        rr[u] = q < p1 ? perm[q] : -1;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        ll[u] = rr[u] >= 0 ? labels[rr[u]] : -1;
        if (rr[u] >= 0 && active) Chunk16<T>::load(X + (size_t)rr[u] * d + c0, v[u]);
        else {
#pragma unroll
          for (int e = 0; e < V; ++e) v[u][e] = 0.f;
        }
        ww[u] = (w && rr[u] >= 0) ? w[rr[u]] : 1.0f;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (ll[u] < 0) continue;
        if (ll[u] != cur) {
          if (cur >= 0) flush();
          cur = ll[u];
#pragma unroll
          for (int e = 0; e < V; ++e) acc[e] = 0.0;
          cnt = 0.0;
        }
        const float sc = ww[u] * xscale;   // exact when unweighted (power of 2)
#pragma unroll
        for (int e = 0; e < V; ++e) acc[e] += (double)rintf(v[u][e] * sc);
        cnt += w ? (double)rintf(ww[u] * wscale) : 1.0;
      }
    }
    if (cur >= 0) flush();
  }
}

// deterministic sum of n doubles (fixed thread order + fixed tree): one WG
__global__ void __launch_bounds__(256) sum_partials_kernel(const double* __restrict__ part,
                                                           int n, double* __restrict__ out) {
  __shared__ double red[256];
  double s = 0.0;
  for (int i = threadIdx.x; i < n; i += 256) s += part[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = red[0];
}

// Iteration scalars for the host convergence test in one launch:
// scalars = [inertia (packed tail, after the all-reduce), shift (per-centroid
// parts summed in the same fixed order as sum_partials_kernel), overflow
// rows]; the overflow counter is reset for the next E-step.
// With cmax2 != null it also writes max_j cn[j] (the fp16 operand's largest
// alpha^2 ||c||^2: the certified E-step's error bound for the next iteration).
// With kept != null, scalars[3] = the rows the iteration's Hamerly filter
// kept (the host's adaptive-pruning signal, carried by the same read).
__global__ void __launch_bounds__(256) iter_scalars_kernel(const double* __restrict__ part, int n,
                                                           double* __restrict__ shift,
                                                           const double* __restrict__ inertia,
                                                           int* __restrict__ ovf_count,
                                                           double* __restrict__ scalars,
                                                           const float* __restrict__ cn,
                                                           float* __restrict__ cmax2,
                                                           const int* __restrict__ kept) {
  __shared__ double red[256];
  __shared__ float redm[256];
  double s = 0.0;
  float mx = 0.0f;
  for (int i = threadIdx.x; i < n; i += 256) {
    s += part[i];
    if (cmax2) mx = fmaxf(mx, cn[i]);
  }
  redm[threadIdx.x] = mx;
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      red[threadIdx.x] += red[threadIdx.x + o];
      redm[threadIdx.x] = fmaxf(redm[threadIdx.x], redm[threadIdx.x + o]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    if (cmax2) cmax2[0] = redm[0];
    shift[0] = red[0];
    scalars[0] = inertia[0];
    scalars[1] = red[0];
    if (ovf_count) {
      scalars[2] = (double)ovf_count[0];
      ovf_count[0] = 0;
    } else {
      scalars[2] = 0.0;
    }
    if (kept) scalars[3] = (double)kept[0];
  }
}

// packed[0:k*d] = sums (f64), packed[k*d : k*d+k] = counts, packed[k*d+k] = inertia;
// sums/counts arrive as integer multiples of the quanta xq / wq
__global__ void __launch_bounds__(256) pack_stats_kernel(
    const double* __restrict__ sums, const double* __restrict__ counts,
    const double* __restrict__ inertia, double* __restrict__ packed, int k, int d, double xq,
    double wq) {
  long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  long long kd = (long long)k * d;
  if (i < kd) packed[i] = (double)sums[i] * xq;
  else if (i < kd + k) packed[i] = (double)counts[i - kd] * wq;
  else if (i == kd + k) packed[i] = inertia ? inertia[0] : 0.0;
}

// The incremental M-step's statistics in two launches (was four):
// mstep_parts_kernel - blocks [0, nb): fixed-range fp64 partial sums of the
// E-step's min-vs-label corrections corr[0:n] (the sum_f32_blocks
// association); blocks [nb, nb + ceil(k / 4)): the per-cluster inertia parts
// Q_c - 2 c.S_c + n_c |c|^2 (cluster_inertia_kernel);
// pack_sum_kernel - packs sums / counts (pack_stats_kernel) while block 0
// sums the nb + k partials (sum_partials association) into inertia[0] and
// the bucket's tail.
__global__ void __launch_bounds__(256) mstep_parts_kernel(
    const float* __restrict__ corr, long long n, int nb, const double* __restrict__ sums,
    const double* __restrict__ counts, const double* __restrict__ qsum,
    const float* __restrict__ C, int k, int d, double xunit, double qunit,
    double* __restrict__ part) {
  __shared__ double red[256];
  if ((int)blockIdx.x < nb) {
    const long long per = (n + (long long)nb * 1024 - 1) / ((long long)nb * 1024) * 1024;
    const long long b = (long long)blockIdx.x * per, e = min(n, b + per);
    double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
    const long long e4 = b < e ? b + (e - b) / 4 * 4 : b;
    const float4* v4 = reinterpret_cast<const float4*>(corr);
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
    for (long long t = e4 + threadIdx.x; t < e; t += 256) s1 += (double)corr[t];
    red[threadIdx.x] = (s0 + s1) + (s2 + s3);
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
      if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
      __syncthreads();
    }
    if (threadIdx.x == 0) part[blockIdx.x] = red[0];
    return;
  }
  const int lane = threadIdx.x & 63;
  const int c = ((int)blockIdx.x - nb) * 4 + (threadIdx.x >> 6);
  if (c >= k) return;
  double cs = 0.0, cc = 0.0;
  for (int f = lane; f < d; f += 64) {
    const double cf = (double)C[(size_t)c * d + f];
    cs = fma(cf, sums[(size_t)c * d + f], cs);
    cc = fma(cf, cf, cc);
  }
  cs = wave_sum(cs);
  cc = wave_sum(cc);
  if (lane == 0) part[nb + c] = qsum[c] * qunit - 2.0 * cs * xunit + counts[c] * cc;
}

__global__ void __launch_bounds__(256) pack_sum_kernel(
    const double* __restrict__ sums, const double* __restrict__ counts,
    const double* __restrict__ part, int npart, double* __restrict__ inertia,
    double* __restrict__ packed, int k, int d, double xq, double wq) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long kd = (long long)k * d;
  if (i < kd) packed[i] = (double)sums[i] * xq;
  else if (i < kd + k) packed[i] = (double)counts[i - kd] * wq;
  if (blockIdx.x == 0) {
    __shared__ double red[256];
    double s = 0.0;
    for (int t = threadIdx.x; t < npart; t += 256) s += part[t];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
      if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      inertia[0] = red[0];
      packed[kd + k] = red[0];
    }
  }
}

// one workgroup per (padded) centroid row
// C_bf16 (bf16 E-step operand) and/or C_f16 (fp16 hi/lo operand of the
// fp32-faithful E-step, csrc/estep_f32.hip, scale alpha) may be null.
__global__ void __launch_bounds__(256) centroid_finalize_kernel(
    const double* __restrict__ packed, const float* __restrict__ C_old, float* __restrict__ C_new,
    uint16_t* __restrict__ C_bf16, float* __restrict__ cn, double* __restrict__ shift, int k, int d,
    int d_pad, float b, float erf_b, RngKey key, int empty_policy, _Float16* __restrict__ C_f16,
    float alpha) {
  const int j = blockIdx.x;
  const int tid = threadIdx.x;
  __shared__ double red[4];
  __shared__ float redf[4];
  __shared__ double redn[4];
  // fp16 operand: per 64-centroid tile [hi chunks: d_pad/8 + 2][lo chunks: d_pad/8]
  const int dch = d_pad / 8;
  _Float16* Cf = C_f16 ? C_f16 + (size_t)(j >> 6) * (2 * dch + 2) * 512 + (size_t)(j & 63) * 8
                       : nullptr;
  auto hi16 = [&](int c) -> _Float16& { return Cf[(size_t)(c >> 3) * 512 + (c & 7)]; };
  auto lo16 = [&](int c) -> _Float16& { return Cf[(size_t)(dch + 2 + (c >> 3)) * 512 + (c & 7)]; };
  // chunk-major E-step operand (see estep_kernel): -2 c, then [hi, mid, lo]
  // of ||bf16(c)||^2 in the augmented chunk, zeros after
  const int cpr = d_pad / 8 + 2;
  uint16_t* Cb = C_bf16 + (size_t)(j >> 6) * cpr * 512 + (size_t)(j & 63) * 8;
  auto at = [&](int c) -> uint16_t& { return Cb[(size_t)(c >> 3) * 512 + (c & 7)]; };
  if (j >= k) {
    if (C_bf16) for (int c = tid; c < d_pad + 16; c += 256) at(c) = 0;
    if (Cf) {
      for (int c = tid; c < d_pad + 16; c += 256) hi16(c) = (_Float16)0.0f;
      for (int c = tid; c < d_pad; c += 256) lo16(c) = (_Float16)0.0f;
    }
    __syncthreads();
    if (tid == 0) {
      if (C_bf16) at(d_pad) = f32_to_bf16_rne(kBig);
      if (Cf) hi16(d_pad) = hi16(d_pad + 1) = hi16(d_pad + 2) = (_Float16)65504.0f;
      cn[j] = kBig;
    }
    return;
  }
  const double cntv = packed[(size_t)k * d + j];
  double sh = 0.0, nn64 = 0.0;
  float nn = 0.0f;
  for (int c = tid; c < d_pad; c += 256) {
    uint16_t hb = 0;
    _Float16 fh = (_Float16)0.0f, fl = (_Float16)0.0f;
    if (c < d) {
      float old = C_old[(size_t)j * d + c];
      float v;
      if (cntv > 0.0) v = (float)(packed[(size_t)j * d + c] / cntv);
      else v = empty_policy == 0 ? old : 0.0f;
      if (b > 0.0f) v += trunc_normal(key.word((unsigned long long)j * d + c), b, erf_b);
      C_new[(size_t)j * d + c] = v;
      double df = (double)v - (double)old;
      sh += df * df;
      uint16_t h = f32_to_bf16_rne(v);
      float hv = bf16_to_f32(h);
      nn += hv * hv;
      hb = f32_to_bf16_rne(-2.0f * hv);   // exact: scaling by -2
      const double av = (double)v * (double)alpha;
      nn64 += av * av;
      const float sv = -2.0f * alpha * v;  // exact: power-of-two scaling
      fh = (_Float16)sv;
      fl = (_Float16)(sv - (float)fh);
    }
    if (C_bf16) at(c) = hb;
    if (Cf) { hi16(c) = fh; lo16(c) = fl; }
  }
  if (C_bf16) for (int c = d_pad + 3 + tid; c < d_pad + 16; c += 256) at(c) = 0;
  if (Cf) for (int c = d_pad + 3 + tid; c < d_pad + 16; c += 256) hi16(c) = (_Float16)0.0f;
  sh = wave_sum(sh);
  nn = wave_sum(nn);
  nn64 = wave_sum(nn64);
  if ((tid & 63) == 0) { red[tid >> 6] = sh; redf[tid >> 6] = nn; redn[tid >> 6] = nn64; }
  __syncthreads();
  if (tid == 0) {
    shift[j] = red[0] + red[1] + red[2] + red[3];   // per-centroid part (fixed-order sum)
    float t = redf[0] + redf[1] + redf[2] + redf[3];
    cn[j] = C_f16 ? (float)(redn[0] + redn[1] + redn[2] + redn[3]) : t;
    if (C_bf16) {
      uint16_t hi = f32_to_bf16_rne(t);
      float r1 = t - bf16_to_f32(hi);
      uint16_t mid = f32_to_bf16_rne(r1);
      uint16_t lo = f32_to_bf16_rne(r1 - bf16_to_f32(mid));
      at(d_pad) = hi;
      at(d_pad + 1) = mid;
      at(d_pad + 2) = lo;
    }
    if (Cf) {
      // 3-way fp16 split of alpha^2 ||c||^2 (same as centers_f16_operand)
      const float tn = (float)(redn[0] + redn[1] + redn[2] + redn[3]);
      const _Float16 hi = (_Float16)tn;
      const float r1 = tn - (float)hi;
      const _Float16 mid = (_Float16)r1;
      hi16(d_pad) = hi;
      hi16(d_pad + 1) = mid;
      hi16(d_pad + 2) = (_Float16)(r1 - (float)mid);
    }
  }
}

// ---------------------------------------------------------------------------
// IPE distances: G[m][ldG] = x_i . c_j (fp32).  One workgroup (256) per row.
// D~_ij = |x|^2 + |c|^2 - 2 IPE(x, c); label = argmin with random tie-break.
__global__ void __launch_bounds__(256) ipe_estep_kernel(
    const float* __restrict__ G, const float* __restrict__ xn, const float* __restrict__ cn,
    int* __restrict__ labels, float* __restrict__ mind, long long m, int k, long long ldG,
    double eps, int Q, RngKey key, long long row_offset, int idx_bits) {
  const long long r = blockIdx.x;
  const int tid = threadIdx.x;
  const long long grow = row_offset + r;
  const double nx2 = (double)xn[r];
  float best = __builtin_inff();
  uint32_t bestk = 0xFFFFFFFFu;
  const uint32_t keep = ~((1u << idx_bits) - 1u);
  __shared__ float sbest[4];
  __shared__ uint32_t skey[4];
  double est[31];
  for (int j = tid; j < k; j += 256) {
    double ip = (double)G[r * ldG + j];
    double ny2 = (double)cn[j];
    double S = nx2 + ny2;
    double dtil;
    if (S <= 0.0) {
      dtil = 0.0;
    } else {
      double a = (S - 2.0 * ip) / (2.0 * S);
      if (fabs(a) <= 1e-15) a = 0.0;
      double eps_a = eps * fmax(1.0, fabs(ip)) / S;
      long long M = ae_bins(eps_a);
      if (M > (1LL << 40)) M = 1LL << 40;
      unsigned long long sid = ((unsigned long long)grow * (unsigned long long)k + j) * Q;
      for (int q = 0; q < Q; ++q) {
        WordStream ws(key, sid + q);
        est[q] = ae_sample(a, M, ws);
      }
      double at = Q == 1 ? est[0] : median_of<31>(est, Q);
      double s = S * (1.0 - 2.0 * at) / 2.0;
      dtil = nx2 + ny2 - 2.0 * s;
    }
    float df = (float)dtil;
    uint32_t rk = (band_key(key, grow, (uint32_t)j) & keep) | (uint32_t)j;
    if (df < best || (df == best && rk < bestk)) { best = df; bestk = rk; }
  }
  // block argmin over (value, key)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    float ob = __shfl_xor(best, o, 64);
    uint32_t ok = (uint32_t)__shfl_xor((int)bestk, o, 64);
    if (ob < best || (ob == best && ok < bestk)) { best = ob; bestk = ok; }
  }
  if ((tid & 63) == 0) { sbest[tid >> 6] = best; skey[tid >> 6] = bestk; }
  __syncthreads();
  if (tid == 0) {
    for (int w = 1; w < 4; ++w)
      if (sbest[w] < best || (sbest[w] == best && skey[w] < bestk)) { best = sbest[w]; bestk = skey[w]; }
    labels[grow - row_offset] = (int)(bestk & ~keep);
    mind[grow - row_offset] = best;
  }
}

}  // namespace sq

using namespace sq;

static int idx_bits_for(int k_pad) {
  int b = 1;
  while ((1 << b) < k_pad) ++b;
  return b;
}

static int estep_dbg() {
  static int v = -1;
  if (v < 0) { const char* e = getenv("SQ_ESTEP_DBG"); v = e ? atoi(e) : 0; }
  return v;
}

template <int KS, int NW>
static int launch_estep(const void* X, const void* C, const void* cn, const void* xn, void* labels,
                        void* mind, void* ovf_rows, void* ovf_count, void* inertia,
                        void* part, int part_cap, long long n, int k, int k_pad, float delta,
                        RngKey key, long long row_offset, int ovf_cap, hipStream_t st) {
  size_t lds = (SQ_ESTEP_PAIR ? 4 : 2) * (size_t)kBN * (KS + 1) * 16 * 2;   // tile ring
  auto kern = estep_kernel<KS, NW>;
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  // persistent grid: every resident workgroup slot once (blocks are strided)
  static int resident = 0;
  if (resident == 0) {
    int dev = 0, cus = 0, per_cu = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)kern, NW * 64, lds);
    resident = (cus > 0 ? cus : 256) * (per_cu > 0 ? per_cu : 1);
  }
  long long rows_per_wg = NW * 32;
  long long nblk = (n + rows_per_wg - 1) / rows_per_wg;
  static int persist = -1;
  if (persist < 0) { const char* e = getenv("SQ_ESTEP_PERSIST"); persist = e ? atoi(e) : 1; }
  unsigned grid = (unsigned)(nblk < resident || !persist ? nblk : resident);
  if ((long long)grid * NW > part_cap) grid = (unsigned)(part_cap / NW);   // still persistent
  if (grid == 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(kern, dim3(grid), dim3(NW * 64), lds, st, (const uint16_t*)X,
                     (const uint16_t*)C, (float*)cn, (const float*)xn, (int*)labels,
                     (float*)mind, (long long*)ovf_rows, (int*)ovf_count, (double*)part, n, k,
                     k_pad, delta, key, row_offset, ovf_cap, idx_bits_for(k_pad), estep_dbg());
  hipLaunchKernelGGL(sum_partials_kernel, dim3(1), dim3(256), 0, st, (const double*)part,
                     (int)grid * NW, (double*)inertia);
  return (int)hipGetLastError();
}

template <int KS>
static int launch_estep64(const void* X, const void* C, const void* cn, const void* xn,
                          void* labels, void* mind, void* ovf_rows, void* ovf_count, void* inertia,
                          void* part, int part_cap, long long n, int k, int k_pad, float delta,
                          RngKey key, long long row_offset, int ovf_cap, hipStream_t st) {
  constexpr int NW = 4;
  size_t lds = 2 * (size_t)kBN * (KS + 1) * 16 * 2;
  auto kern = estep64_kernel<KS>;
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  static int resident = 0;
  if (resident == 0) {
    int dev = 0, cus = 0, per_cu = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)kern, NW * 64, lds);
    resident = (cus > 0 ? cus : 256) * (per_cu > 0 ? per_cu : 1);
  }
  long long rows_per_wg = NW * 64;
  long long nblk = (n + rows_per_wg - 1) / rows_per_wg;
  unsigned grid = (unsigned)(nblk < resident ? nblk : resident);
  if ((long long)grid * NW > part_cap) grid = (unsigned)(part_cap / NW);
  if (grid == 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(kern, dim3(grid), dim3(NW * 64), lds, st, (const uint16_t*)X,
                     (const uint16_t*)C, (float*)cn, (const float*)xn, (int*)labels,
                     (float*)mind, (long long*)ovf_rows, (int*)ovf_count, (double*)part, n, k,
                     k_pad, delta, key, row_offset, ovf_cap, idx_bits_for(k_pad), estep_dbg());
  hipLaunchKernelGGL(sum_partials_kernel, dim3(1), dim3(256), 0, st, (const double*)part,
                     (int)grid * NW, (double*)inertia);
  return (int)hipGetLastError();
}

extern "C" {

int sq_estep_bf16(const void* X, const void* C, void* part, const void* cn, const void* xn,
                  void* labels, void* mind, void* ovf_rows, void* ovf_count, void* inertia,
                  long long n, int d, int k, int k_pad, double delta, int part_cap, unsigned k0,
                  unsigned k1, unsigned s0, unsigned s1, long long row_offset, int ovf_cap,
                  void* stream) {
  if (n <= 0) return 0;
  if (part_cap < 8) return (int)hipErrorInvalidValue;
  if (k_pad % kBN != 0 || k_pad > 32768 || k > k_pad) return (int)hipErrorInvalidValue;
  if ((SQ_ESTEP_PAIR ? 4 : 2) * (size_t)kBN * (d + 16) * 2 > 160 * 1024) return (int)hipErrorInvalidValue;
  RngKey key{k0, k1, s0, s1};
  hipStream_t st = (hipStream_t)stream;
  float dl = (float)delta;
  // 8 waves (2 per SIMD) share each staged centroid tile: half the LDS-DMA
  // issue per row of the 4-wave layout (measured 5.70 vs 6.18 ms, 10M x 256,
  // k = 1024); SQ_ESTEP_NW=4 selects the 4-wave layout.
  int nw = 8;
  const char* env = getenv("SQ_ESTEP_NW");
  if (env && env[0] == '4') nw = 4;
  static int rows64 = -1;
  if (rows64 < 0) { const char* e = getenv("SQ_ESTEP_ROWS"); rows64 = (e && atoi(e) == 64) ? 1 : 0; }
  if (rows64) nw = 64;   // estep64_kernel
#define ESTEP_CASE(KS)                                                                           \
  case KS * 16:                                                                                  \
    if (nw == 64)                                                                              \
      return launch_estep64<KS>(X, C, cn, xn, labels, mind, ovf_rows, ovf_count, inertia, part, \
                                part_cap, n, k, k_pad, dl, key, row_offset, ovf_cap, st);        \
    return nw == 8 ? launch_estep<KS, 8>(X, C, cn, xn, labels, mind, ovf_rows, ovf_count,        \
                                         inertia, part, part_cap, n, k, k_pad, dl, key,         \
                                         row_offset, ovf_cap, st)                               \
                   : launch_estep<KS, 4>(X, C, cn, xn, labels, mind, ovf_rows, ovf_count,        \
                                         inertia, part, part_cap, n, k, k_pad, dl, key,         \
                                         row_offset, ovf_cap, st);
  switch (d) {
    ESTEP_CASE(1)
    ESTEP_CASE(2)
    ESTEP_CASE(4)
    ESTEP_CASE(8)
    ESTEP_CASE(16)
    default:
      return (int)hipErrorInvalidValue;
  }
#undef ESTEP_CASE
}

int sq_band_select(const void* D, const void* rows, const void* xn, void* labels, void* mind,
                   long long m, int k, long long ldD, double delta, unsigned k0, unsigned k1,
                   unsigned s0, unsigned s1, long long row_offset, void* stream) {
  if (m <= 0) return 0;
  RngKey key{k0, k1, s0, s1};
  int kp = ((k + 63) / 64) * 64;
  hipLaunchKernelGGL(band_select_kernel, dim3((unsigned)((m + 3) / 4)), dim3(256), 0,
                     (hipStream_t)stream, (const float*)D, (const long long*)rows,
                     (const float*)xn, (int*)labels, (float*)mind, m, k, ldD, (float)delta, key,
                     row_offset, idx_bits_for(kp));
  return (int)hipGetLastError();
}

int sq_band_select_rows(const void* X, const void* C, const void* cn, const void* xn,
                        const void* rows, const void* count, void* labels, long long cap,
                        int d_pad, int k, int k_pad, double delta, unsigned k0, unsigned k1,
                        unsigned s0, unsigned s1, long long row_offset, void* stream) {
  if (cap <= 0) return 0;
  if (d_pad > 256) return (int)hipErrorInvalidValue;
  if (k > kRowsMaxK) return (int)hipErrorInvalidValue;
  (void)xn;
  (void)k_pad;
  RngKey key{k0, k1, s0, s1};
  hipLaunchKernelGGL(band_select_rows_kernel, dim3((unsigned)(cap < 2048 ? cap : 2048)),
                     dim3(256), 0, (hipStream_t)stream, (const uint16_t*)X, (const uint16_t*)C,
                     (const float*)cn /* per-slot thresholds */, (const long long*)rows,
                     (const int*)count, (int*)labels, cap, d_pad, k, (float)delta, key,
                     row_offset);
  return (int)hipGetLastError();
}

int sq_centroid_accumulate(const void* X, int xdtype, const void* labels, const void* weights,
                           void* sums, void* counts, long long n, int d, int k, int chunk,
                           void* stream) {
  if (n <= 0) return 0;
  if (d % 4 != 0) return (int)hipErrorInvalidValue;
  size_t lds = (size_t)(2 * k + chunk) * 4;
  if (lds > 160 * 1024) return (int)hipErrorInvalidValue;
  unsigned grid = (unsigned)((n + chunk - 1) / chunk);
  hipStream_t st = (hipStream_t)stream;
  if (xdtype == 0) {
    hipFuncSetAttribute((const void*)centroid_accumulate_kernel<float>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipLaunchKernelGGL(centroid_accumulate_kernel<float>, dim3(grid), dim3(256), lds, st,
                       (const float*)X, (const int*)labels, (const float*)weights, (float*)sums,
                       (double*)counts, n, d, k, chunk);
  } else if (xdtype == 2) {
    hipFuncSetAttribute((const void*)centroid_accumulate_kernel<uint16_t>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipLaunchKernelGGL(centroid_accumulate_kernel<uint16_t>, dim3(grid), dim3(256), lds, st,
                       (const uint16_t*)X, (const int*)labels, (const float*)weights, (float*)sums,
                       (double*)counts, n, d, k, chunk);
  } else {
    return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

// A/B knobs (read once): SQ_SEG_HALF=0/1 bf16 half-wave rows, SQ_SEG_RANGE
// positions per workgroup of the large-d segmented sum (multiple of 16)
static int seg_half() {
  static int v = [] { const char* e = getenv("SQ_SEG_HALF"); return e ? atoi(e) : 0; }();
  return v;
}
static int seg_range() {
  static int v = [] {
    const char* e = getenv("SQ_SEG_RANGE");
    int r = e ? atoi(e) : 2048;
    return r < 64 ? 64 : (r / 16) * 16;
  }();
  return v;
}

int sq_centroid_reduce(const void* X, int xdtype, const void* labels, const void* weights,
                       void* sums, void* counts, long long n, int d, int k, int xexp, int wexp,
                       void* ws_hist, void* ws_cursor, void* ws_perm, void* mind,
                       const void* Cold, void* stream) {
  if (mind && (xdtype != 0 || d > 256 || d % 4 != 0 || !Cold)) return (int)hipErrorInvalidValue;
  if (n <= 0) return 0;
  if (d % 4 != 0 || k > 16384 || n > 2147483647LL) return (int)hipErrorInvalidValue;
  if (xexp < -120 || xexp > 120 || wexp < -120 || wexp > 120) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  unsigned chunks = (unsigned)((n + kHistChunk - 1) / kHistChunk);
  // ws_hist is all-zero on entry (zeroed at allocation, re-zeroed by the scan)
  hipLaunchKernelGGL(label_hist_kernel, dim3(chunks), dim3(256), (size_t)k * 4, st,
                     (const int*)labels, n, k, (int*)ws_hist, (double*)sums, (long long)k * d,
                     (double*)counts, k);
  hipLaunchKernelGGL(label_scan_kernel, dim3(1), dim3(1024), 0, st, (int*)ws_hist, k,
                     (int*)ws_cursor);
  hipLaunchKernelGGL(label_scatter_kernel, dim3(chunks), dim3(256), (size_t)k * 8, st,
                     (const int*)labels, n, k, (int*)ws_cursor, (int*)ws_perm);
  // rows with label < 0 are not in the permutation: sum over the first n_valid
  // positions; n_valid <= n and unused tail positions hold stale data, so the
  // kernel bounds itself with the scanned total (cursor[k-1] after scatter)
  const float xs = ldexpf(1.0f, -xexp), wsc = ldexpf(1.0f, -wexp);
  const int V = xdtype == 2 ? 8 : 4;
  if (d / V >= 32 || d % V != 0 || mind) {
    // whole-wave rows (large d, or d not a multiple of the 16-B chunk)
    const int range = seg_range();
    unsigned grid = (unsigned)((n + range - 1) / range);
    if (xdtype == 0)
      hipLaunchKernelGGL(segment_sum_rows_kernel<float>, dim3(grid), dim3(512), 0, st,
                         (const float*)X, (const int*)ws_perm, (const int*)labels,
                         (const float*)weights, n, d, range, xs, wsc, (double*)sums,
                         (double*)counts, (const int*)ws_cursor + (k - 1), (float*)mind,
                         (const float*)Cold);
    else if (xdtype == 2 && d % 8 == 0 && seg_half())
      hipLaunchKernelGGL(segment_sum_rows_half_kernel, dim3(grid), dim3(512), 0, st,
                         (const uint16_t*)X, (const int*)ws_perm, (const int*)labels,
                         (const float*)weights, n, d, range, xs, wsc, (double*)sums,
                         (double*)counts, (const int*)ws_cursor + (k - 1));
    else if (xdtype == 2)
      hipLaunchKernelGGL(segment_sum_rows_kernel<uint16_t>, dim3(grid), dim3(512), 0, st,
                         (const uint16_t*)X, (const int*)ws_perm, (const int*)labels,
                         (const float*)weights, n, d, range, xs, wsc, (double*)sums,
                         (double*)counts, (const int*)ws_cursor + (k - 1), (float*)nullptr,
                         (const float*)nullptr);
    else
      return (int)hipErrorInvalidValue;
    return (int)hipGetLastError();
  }
  int lpr = 1;
  while (lpr < d / V && lpr < 64) lpr <<= 1;
  // every virtual wave flushes once per label run it touches: scale the
  // positions per WG with the virtual-wave count (atomics per row ~ d / 256)
  const int range = 2048 * (64 / lpr);
  unsigned grid = (unsigned)((n + range - 1) / range);
#define SEG_CASE(TT, L)                                                                         \
  case L:                                                                                       \
    hipLaunchKernelGGL((segment_sum_kernel<TT, L>), dim3(grid), dim3(512), 0, st,               \
                       (const TT*)X, (const int*)ws_perm, (const int*)labels,                   \
                       (const float*)weights, n, d, range, xs, wsc, (double*)sums,              \
                       (double*)counts, (const int*)ws_cursor + (k - 1));                       \
    break;
  if (xdtype == 0) {
    switch (lpr) { SEG_CASE(float, 1) SEG_CASE(float, 2) SEG_CASE(float, 4) SEG_CASE(float, 8)
                   SEG_CASE(float, 16) SEG_CASE(float, 32) SEG_CASE(float, 64)
                   default: return (int)hipErrorInvalidValue; }
  } else if (xdtype == 2) {
    switch (lpr) { SEG_CASE(uint16_t, 1) SEG_CASE(uint16_t, 2) SEG_CASE(uint16_t, 4)
                   SEG_CASE(uint16_t, 8) SEG_CASE(uint16_t, 16) SEG_CASE(uint16_t, 32)
                   SEG_CASE(uint16_t, 64) default: return (int)hipErrorInvalidValue; }
  } else {
    return (int)hipErrorInvalidValue;
  }
#undef SEG_CASE
  return (int)hipGetLastError();
}

// Incremental fixed-point cluster statistics (see delta_segment_kernel):
// sums / counts / qsum are UPDATED (not overwritten) by the rows whose label
// differs from prev, and prev becomes labels; qexp is the quantum of the
// squared norms; ws_perm holds 2n int2 entries.
// lists (nullable): the row lists of the filtered E-step that produced
// labels - only those rows are walked (delta_hist_list_kernel); null: all n.
static int centroid_delta_impl(const void* X, const void* labels, const void* prev, void* sums,
                               void* counts, void* qsum, long long n, int d, int k, int xexp,
                               int qexp, void* ws_hist, void* ws_cursor, void* ws_perm,
                               const RowLists* lists, void* stream) {
  if (n <= 0) return 0;
  if (d % 4 != 0 || d > 1024 || k > 16384 || 2 * n > 2147483647LL) return (int)hipErrorInvalidValue;
  if (xexp < -120 || xexp > 120 || qexp < -200 || qexp > 200) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  if (lists) {
    const long long lb = (n + 1023) / 1024;
    const unsigned lgrid = (unsigned)(lb < 256 ? lb : 256);
    hipLaunchKernelGGL(delta_hist_list_kernel, dim3(lgrid), dim3(256), (size_t)k * 4, st,
                       (const int*)labels, (const int*)prev, *lists, n, k, (int*)ws_hist);
    hipLaunchKernelGGL(label_scan_kernel, dim3(1), dim3(1024), 0, st, (int*)ws_hist, k,
                       (int*)ws_cursor);
    hipLaunchKernelGGL(delta_scatter_list_kernel, dim3(lgrid), dim3(256), (size_t)k * 8, st,
                       (const int*)labels, (int*)prev, *lists, n, k, (int*)ws_cursor,
                       (int2*)ws_perm);
  } else {
    const unsigned chunks = (unsigned)((n + kHistChunk - 1) / kHistChunk);
    hipLaunchKernelGGL(delta_hist_kernel, dim3(chunks), dim3(256), (size_t)k * 4, st,
                       (const int*)labels, (const int*)prev, n, k, (int*)ws_hist);
    hipLaunchKernelGGL(label_scan_kernel, dim3(1), dim3(1024), 0, st, (int*)ws_hist, k,
                       (int*)ws_cursor);
    hipLaunchKernelGGL(delta_scatter_kernel, dim3(chunks), dim3(256), (size_t)k * 8, st,
                       (const int*)labels, (int*)prev, n, k, (int*)ws_cursor, (int2*)ws_perm);
  }
  // entries <= 2n, usually far fewer: a fixed grid shares the scanned total
  const long long cap_blocks = (2 * n + 63) / 64;
  const unsigned grid = (unsigned)(cap_blocks < 2048 ? cap_blocks : 2048);
  auto seg = d <= 256 ? delta_segment_kernel<1>
             : d <= 512 ? delta_segment_kernel<2>
             : d <= 768 ? delta_segment_kernel<3> : delta_segment_kernel<4>;
  hipLaunchKernelGGL(seg, dim3(grid), dim3(512), 0, st, (const float*)X,
                     (const int2*)ws_perm, d, 0, ldexpf(1.0f, -xexp), ldexp(1.0, -qexp),
                     (double*)sums, (double*)counts, (double*)qsum,
                     (const int*)ws_cursor + (k - 1));
  return (int)hipGetLastError();
}

int sq_centroid_delta(const void* X, const void* labels, const void* prev, void* sums,
                      void* counts, void* qsum, long long n, int d, int k, int xexp, int qexp,
                      void* ws_hist, void* ws_cursor, void* ws_perm, void* stream) {
  return centroid_delta_impl(X, labels, prev, sums, counts, qsum, n, d, k, xexp, qexp, ws_hist,
                             ws_cursor, ws_perm, nullptr, stream);
}

// rows: three int64 row lists and their int32 device lengths (a null list
// is empty); together they must hold every row whose label can differ from
// prev, each once
int sq_centroid_delta_lists(const void* X, const void* labels, const void* prev, void* sums,
                            void* counts, void* qsum, long long n, int d, int k, int xexp,
                            int qexp, void* ws_hist, void* ws_cursor, void* ws_perm,
                            const void* L0, const void* c0, const void* L1, const void* c1,
                            const void* L2, const void* c2, void* stream) {
  RowLists R{{(const long long*)L0, (const long long*)L1, (const long long*)L2},
             {(const int*)c0, (const int*)c1, (const int*)c2}};
  for (int i = 0; i < 3; ++i)
    if ((R.L[i] != nullptr) != (R.c[i] != nullptr)) return (int)hipErrorInvalidValue;
  return centroid_delta_impl(X, labels, prev, sums, counts, qsum, n, d, k, xexp, qexp, ws_hist,
                             ws_cursor, ws_perm, &R, stream);
}

// part[c] = Q_c - 2 c.S_c + n_c |c|^2 (fp64) for the centroids C the labels
// were assigned with; sums / qsum in their fixed-point units 2^xexp / 2^qexp.
int sq_cluster_inertia(const void* sums, const void* counts, const void* qsum, const void* C,
                       int k, int d, int xexp, int qexp, void* part, void* stream) {
  if (k <= 0) return 0;
  hipLaunchKernelGGL(cluster_inertia_kernel, dim3((unsigned)((k + 3) / 4)), dim3(256), 0,
                     (hipStream_t)stream, (const double*)sums, (const double*)counts,
                     (const double*)qsum, (const float*)C, k, d, ldexp(1.0, xexp),
                     ldexp(1.0, qexp), (double*)part);
  return (int)hipGetLastError();
}

int sq_pack_stats(const void* sums, const void* counts, const void* inertia, void* packed, int k,
                  int d, int xexp, int wexp, void* stream) {
  long long tot = (long long)k * d + k + 1;
  hipLaunchKernelGGL(pack_stats_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, (const double*)sums, (const double*)counts,
                     (const double*)inertia, (double*)packed, k, d, ldexp(1.0, xexp),
                     ldexp(1.0, wexp));
  return (int)hipGetLastError();
}

// corr fp32 [n] (16-B aligned), part fp64 [512 + k]: the incremental
// M-step's inertia (sum of cluster parts + corrections) and packed bucket
int sq_mstep_stats(const void* sums, const void* counts, const void* qsum, const void* C, int k,
                   int d, int xexp, int qexp, const void* corr, long long n, void* part,
                   void* inertia, void* packed, void* stream) {
  if (k <= 0 || ((uintptr_t)corr & 15u) != 0) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  const int nb = 512;
  hipLaunchKernelGGL(mstep_parts_kernel, dim3((unsigned)(nb + (k + 3) / 4)), dim3(256), 0, st,
                     (const float*)corr, n, nb, (const double*)sums, (const double*)counts,
                     (const double*)qsum, (const float*)C, k, d, ldexp(1.0, xexp),
                     ldexp(1.0, qexp), (double*)part);
  const long long tot = (long long)k * d + k;
  hipLaunchKernelGGL(pack_sum_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st,
                     (const double*)sums, (const double*)counts, (const double*)part, nb + k,
                     (double*)inertia, (double*)packed, k, d, ldexp(1.0, xexp), 1.0);
  return (int)hipGetLastError();
}

int sq_sum_partials(const void* part, int n, void* out, void* stream) {
  hipLaunchKernelGGL(sum_partials_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream,
                     (const double*)part, n, (double*)out);
  return (int)hipGetLastError();
}

int sq_centroid_finalize(const void* packed, const void* C_old, void* C_new, void* C_bf16,
                         void* shift_part, void* cn, void* shift, int k, int d, int k_pad,
                         double noise_b, unsigned k0, unsigned k1, unsigned s0, unsigned s1,
                         int empty_policy, void* scalars, void* ovf_count, void* C_f16,
                         double alpha, void* cmax2, const void* kept, void* stream) {
  if (!shift_part) return (int)hipErrorInvalidValue;
  RngKey key{k0, k1, s0, s1};
  float b = (float)noise_b;
  float eb = erff(b * 0.70710678118654752f);
  int d_pad = d <= 16 ? 16 : (d <= 32 ? 32 : (d <= 64 ? 64 : (d <= 128 ? 128 : (d <= 256 ? 256 : ((d + 15) / 16) * 16))));
  hipLaunchKernelGGL(centroid_finalize_kernel, dim3((unsigned)k_pad), dim3(256), 0,
                     (hipStream_t)stream, (const double*)packed, (const float*)C_old,
                     (float*)C_new, (uint16_t*)C_bf16, (float*)cn, (double*)shift_part, k, d,
                     d_pad, b, eb, key, empty_policy, (_Float16*)C_f16, (float)alpha);
  if (scalars)
    hipLaunchKernelGGL(iter_scalars_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream,
                       (const double*)shift_part, k, (double*)shift,
                       (const double*)packed + (long long)k * d + k, (int*)ovf_count,
                       (double*)scalars, (const float*)cn, (float*)cmax2, (const int*)kept);
  else
    hipLaunchKernelGGL(sum_partials_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream,
                       (const double*)shift_part, k, (double*)shift);
  return (int)hipGetLastError();
}

int sq_ipe_estep(const void* G, const void* xn, const void* cn, void* labels, void* mind,
                 long long m, int k, long long ldG, double eps, int Q, unsigned k0, unsigned k1,
                 unsigned s0, unsigned s1, long long row_offset, void* stream) {
  if (m <= 0) return 0;
  if (Q < 1 || Q > 31) return (int)hipErrorInvalidValue;
  RngKey key{k0, k1, s0, s1};
  int kp = ((k + 63) / 64) * 64;
  hipLaunchKernelGGL(ipe_estep_kernel, dim3((unsigned)m), dim3(256), 0, (hipStream_t)stream,
                     (const float*)G, (const float*)xn, (const float*)cn, (int*)labels,
                     (float*)mind, m, k, ldG, eps, Q, key, row_offset, idx_bits_for(kp));
  return (int)hipGetLastError();
}

}  // extern "C"
