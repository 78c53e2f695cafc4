// Fused IPE E-step of q-means: "l2-sampled distance estimation", the
// reference DEFAULT (``true_distance_estimate=True``, sklearn/cluster/
// _dmeans.py:753-772 -> QuantumUtility/Utility.py:697-737).
//
// For every (row x, centroid c):  ip = x.c (exact fp32 MFMA),
//   S = |x|^2 + |c|^2,  a = (S - 2 ip) / (2 S),  eps_a = eps max(1,|ip|) / S,
//   M = ceil(pi / (2 eps_a) (1 + sqrt(1 + 4 eps_a))),  omega = M asin(sqrt a) / pi,
//   a~ = median of Q amplitude-estimation draws sin^2(pi j / M), j ~ Fejer(omega, M)
//   D~ = S - 2 S (1 - 2 a~) / 2 = 2 S a~,      label = argmin_j D~ (random ties)
// and the inner-product matrix G is never materialised.
//
// Sampling, per pair (one lane per pair, in the MFMA epilogue):
//  * odd Q and M <= kIpeWalkM: the median-of-Q is drawn EXACTLY from its own
//    law with ONE uniform: the AE values sin^2(pi j/M) are ordered by the
//    circular bin distance t = min(j, M - j), the class masses
//    p(t) + p(M - t) accumulate into F(t); the median of Q iid draws is
//    F^-1(U_(h)) with U_(h) ~ Beta(h, h), drawn once per pair by inverting
//    G(x) = P(Binomial(Q, x) >= h), then one inverse-CDF walk over t in fp64
//    (angle-addition recurrence, no transcendental or binomial per step);
//  * otherwise Q Fejer draws (fejer.h, exact O(1) sampler) from one Philox
//    stream per pair, the median taken over the circular distances t_q
//    (sin^2 is monotone in t) by a register sorting network - no per-thread
//    double[31] array.
// Layout: a workgroup owns 16 rows, their fp32 A fragments (16x16x4 f32
// MFMA: lane l holds x[l & 15][4s + (l >> 4)]) staged once in LDS and shared
// by its 4 waves, which split the centroid tiles (d_pad * 64 B of LDS: 64 KiB
// at d_pad = 1024); centroid tiles of 16 are read as pre-arranged B fragments
// (ops/kmeans.py: ipe_center_fragments, one coalesced 256-B load per k-step,
// L2-resident).  Accumulator register i of lane l is pair (row 4(l>>4) + i,
// centroid l & 15): 4 pairs per lane per tile keep the per-lane state small
// (the sampling epilogue, not the MFMA, is the cost).  After the sweep the
// 16 lanes of a row merge their (D~, tie key, j) minima, then the 4 waves.

#include "ipe_law.h"

namespace sq {

// One 16 x 16 tile of inner products (fp32 MFMA, D4 k-steps): the B
// fragments (L2-resident centroid tile) and A fragments (LDS) of 8 k-steps
// are loaded before their 8 MFMAs and the next 8 are in flight while those
// run - one wait per MFMA on a load issued 8 MFMAs earlier, instead of a
// full L2 round trip before every MFMA.
template <int D4>
SQ_DEV f32x4 ipe_tile_ip(const float* __restrict__ As, const float* __restrict__ bf, int lane) {
  constexpr int B = 8;
  static_assert(D4 % B == 0, "k-steps in batches of 8");
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  float a0[B], b0[B], a1[B], b1[B];
  // (sched_barrier: the scheduler, squeezed by the kernel's register budget,
  // would otherwise sink each load next to its MFMA)
#pragma unroll
  for (int u = 0; u < B; ++u) {
    b0[u] = bf[u * 64];
    a0[u] = As[u * 64 + lane];
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int s0 = 0; s0 < D4; s0 += 2 * B) {
    if (s0 + B < D4) {
#pragma unroll
      for (int u = 0; u < B; ++u) {
        b1[u] = bf[(s0 + B + u) * 64];
        a1[u] = As[(s0 + B + u) * 64 + lane];
      }
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < B; ++u) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[u], b0[u], acc, 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
    if (s0 + B < D4) {
      if (s0 + 2 * B < D4) {
#pragma unroll
        for (int u = 0; u < B; ++u) {
          b0[u] = bf[(s0 + 2 * B + u) * 64];
          a0[u] = As[(s0 + 2 * B + u) * 64 + lane];
        }
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < B; ++u) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[u], b1[u], acc, 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  return acc;
}

// Layout per lane: register i holds pair (row row0 + 4 q4 + i, centroid
// 16 t + c16) of tile t.  prune = 1 (odd Q): each row's hint pair is sampled
// in full first (hint = hint_labels[row] when valid - the previous
// iteration's label, its inner product by a direct fp32 dot product - else
// the pass-1 exact fp32 distance argmin), its estimate is the row's fixed
// threshold, and every other pair is screened by its hazard.  stats
// (nullable, 5 x u64): screened, full-sampler pairs, fires, fires reaching
// the exact branch, workgroups running pass 1.
template <int D4, bool STATS>
__global__ void __launch_bounds__(256, 2) ipe_fused_kernel(
    const float* __restrict__ X, long long ldx, const float* __restrict__ Cf,
    const float* __restrict__ C, const int* __restrict__ hint_labels,
    const float* __restrict__ xn, const float* __restrict__ cn, int* __restrict__ labels,
    float* __restrict__ mind, long long n, int d, int k, int n_tiles, double eps, int Q,
    RngKey key, RngKey tie_key, RngKey skip_key, IpeScreen sc, long long row_offset, int prune,
    unsigned long long* __restrict__ stats) {
  extern __shared__ __attribute__((aligned(16))) float As[];   // [D4][64] A fragments
  __shared__ float mb[4][16];
  __shared__ uint32_t mk[4][16];
  __shared__ int mj[4][16];
  __shared__ float hip_[4][16];
  __shared__ float hv[16];
  __shared__ int hj[16];
  __shared__ int lh[16];
  __shared__ float lip[16];
  // per-lane queues of the pairs that need the full sampler or fired
  // ([slot][thread]; entry = row slot (2 bits) | fired (1 bit) | centroid)
  // a tile step pushes up to 4 entries per lane and the queue is drained
  // whenever fewer than 4 slots are free: QCAP >= 4 (at d_pad = 1024 the
  // 64 KiB of A fragments + 4 slots leave one workgroup per CU)
  constexpr int QCAP = D4 <= 128 ? 8 : 4;
  static_assert(QCAP >= 4, "a tile step pushes up to 4 queue entries per lane");
  __shared__ uint32_t qj[QCAP * 256];
  __shared__ float qip[QCAP * 256];
  // the lane's running (best D~, label) of its 4 row slots ([slot][thread]):
  // touched only by the drains and the final merge, so they live in LDS
  __shared__ float bestv[4 * 256];
  __shared__ int bestj[4 * 256];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int c16 = lane & 15, q4 = lane >> 4;
  const long long row0 = (long long)blockIdx.x * 16;
  const float INF = __builtin_inff();
  uint32_t st_scr = 0, st_full = 0, st_fire = 0, st_exact = 0;
  // A fragments (16x16x4 f32) of the workgroup's 16 rows, shared by the 4
  // waves: As[s][l] = x[row0 + (l & 15)][4 s + (l >> 4)]; rows past n clamped
  for (int e = threadIdx.x; e < D4 * 64; e += 256) {
    const int s = e >> 6, l = e & 63;
    const long long r = row0 + (l & 15) < n ? row0 + (l & 15) : n - 1;
    const int f = 4 * s + (l >> 4);
    As[e] = f < d ? X[(size_t)r * ldx + f] : 0.0f;
  }
  __syncthreads();
  // register i of this lane = pair (row row0 + 4 q4 + i, centroid 16 t + c16)
  f32x4 nx2;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const long long r = row0 + 4 * q4 + i;
    nx2[i] = xn[r < n ? r : n - 1];
    bestv[i * 256 + threadIdx.x] = INF;
    bestj[i * 256 + threadIdx.x] = -1;
  }
  // label hints: lanes (q4, c16) of wave w take row 4 q4 + w (the row their
  // lane (q4, 0) samples in step -1), 16 lanes per fp32 dot product
  bool need_p1 = prune != 0;
  if (prune && hint_labels) {
    const int rr = 4 * q4 + wave;
    const long long r = row0 + rr;
    const int l = r < n ? hint_labels[r] : 0;
    const bool ok = r >= n || (l >= 0 && l < k);
    float s = 0.0f;
    if (r < n && ok)
      for (int f = c16; f < d; f += 16)
        s = fmaf(As[(f >> 2) * 64 + ((f & 3) << 4) + rr], C[(size_t)l * d + f], s);
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) s += __shfl_xor(s, o, 64);
    if (c16 == 0) {
      lh[rr] = r < n ? (ok ? l : -2) : -1;
      lip[rr] = s;
    }
    need_p1 = __syncthreads_or(!ok) != 0;
  }
  if (need_p1) {
    // ---- pass 1: exact fp32 distance argmin (hint), with its inner product
    f32x4 bd = {INF, INF, INF, INF}, bip = {0.f, 0.f, 0.f, 0.f};
    int bjj[4] = {0x7fffffff, 0x7fffffff, 0x7fffffff, 0x7fffffff};
    for (int t = wave; t < n_tiles; t += 4) {
      const f32x4 acc = ipe_tile_ip<D4>(As, Cf + (size_t)t * D4 * 64 + lane, lane);
      const int j = t * 16 + c16;
      if (j < k) {
        const float ny2 = cn[j];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float Dd = nx2[i] + ny2 - 2.0f * acc[i];
          if (Dd < bd[i]) { bd[i] = Dd; bjj[i] = j; bip[i] = acc[i]; }
        }
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float b = bd[i], p = bip[i];
      int jj = bjj[i];
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        const float ob = __shfl_xor(b, o, 64), op = __shfl_xor(p, o, 64);
        const int oj = __shfl_xor(jj, o, 64);
        if (ob < b || (ob == b && oj < jj)) { b = ob; p = op; jj = oj; }
      }
      if (c16 == 0) {
        mb[wave][4 * q4 + i] = b;
        mj[wave][4 * q4 + i] = jj;
        hip_[wave][4 * q4 + i] = p;
      }
    }
    __syncthreads();
  }
  // hazard budgets of this lane's 4 streams (row g, class wave, column c16)
  // (vector registers written through selects only: never addressable)
  u32x4 bud = {0u, 0u, 0u, 0u};
  f32x4 sthr = {INF, INF, INF, INF};   // the thresholds themselves stay in hv
  auto stream_id = [&](int i) -> unsigned long long {
    const long long g = row_offset + row0 + 4 * q4 + i;
    return (unsigned long long)g * 64ull + (unsigned long long)(wave * 16 + c16);
  };
  if (prune) {
    const long long gb[1] = {row_offset + row0 + 4 * q4};
    u32x4 b1[1];
    ipe_initial_budgets<1>(skip_key, gb, wave * 16 + c16, sc, b1);
    bud = b1[0];
  }
  int qn = 0;
  auto consider = [&](int i, int j, float dt) {
    // row slot i takes (dt, j) if better
    const int e = i * 256 + threadIdx.x;
    const float b = bestv[e];
    const int bjj = bestj[e];
    bool take = dt < b;
    if (!take && dt == b && dt < INF) {   // tie: the random keys decide (rare)
      const long long g = row_offset + row0 + 4 * q4 + i;
      const uint32_t tk = band_key(tie_key, g, (uint32_t)j);
      const uint32_t bk = band_key(tie_key, g, (uint32_t)bjj);
      take = tk < bk || (tk == bk && j < bjj);
    }
    if (take) {
      bestv[e] = dt;
      bestj[e] = j;
    }
  };
  // Pairs that need the full sampler (and fired pairs) go to this lane's LDS
  // queue and are resolved by a wave-wide drain (one inlined copy of the
  // samplers): the expensive paths run max(queue length) times per wave.
  auto drain = [&](int stp) {
    while (__ballot(qn > 0) != 0ull) {   // wave-uniform
      if (qn > 0) {
        --qn;
        const uint32_t pj = qj[qn * 256 + threadIdx.x];
        const float ip = qip[qn * 256 + threadIdx.x];
        const int i = (int)(pj >> 30), j = (int)(pj & 0x1fffffffu);
        const bool fired = (pj >> 29) & 1u;
        float nxi = nx2[0], si = sthr[0];
#pragma unroll
        for (int ii = 1; ii < 4; ++ii) {
          nxi = i == ii ? nx2[ii] : nxi;
          si = i == ii ? sthr[ii] : si;
        }
        const long long g = row_offset + row0 + 4 * q4 + i;
        float dt;
        if (!fired) {
          if (STATS) ++st_full;
          dt = ipe_distance(ip, (double)nxi, (double)cn[j], eps, Q, key,
                            (unsigned long long)g * (unsigned long long)k + (unsigned long long)j);
        } else {
          // the same hazard as at the screen (same inputs, same code)
          uint32_t hq = 0;
          float pbar = 1.0f;
          ipe_hazard(ip, nxi, cn[j], si, sc, hq, pbar);
          WordStream ws(skip_key, stream_id(i));
          ws.b = (uint32_t)(2 * stp + 1);
          const uint32_t w0 = ws.next(), w1 = ws.next(), w2 = ws.next(), w3 = ws.next();
          const uint32_t nb = ipe_budget(w0, w1);   // the stream's next budget
          bud.x = i == 0 ? nb : bud.x;
          bud.y = i == 1 ? nb : bud.y;
          bud.z = i == 2 ? nb : bud.z;
          bud.w = i == 3 ? nb : bud.w;
          const double beff = -expm1(-(double)hq * (1.0 / 4294967296.0));
          const double u = u53(w2, w3) * beff;
          const int h = (Q + 1) / 2;
          const double pib = binom_upper_tail((double)pbar, Q, h) * (1.0 + 1e-12);
          dt = INF;
          if (u < pib) {
            if (STATS) ++st_exact;
            dt = ipe_pruned_exact((double)ip, (double)nxi + (double)cn[j], eps, Q, hv[4 * q4 + i],
                                  u, ws);
          }
        }
        consider(i, j, dt);
      }
    }
  };
  // the 4 slots' hint centroids, 16 bits each (k_pad <= 16384; 0xFFFF: none)
  uint32_t hint01 = 0xFFFFFFFFu, hint23 = 0xFFFFFFFFu;
  // ---- step -1 (prune): the 16 hint pairs (row 4 q4 + w taken by lane
  // (q4, c16 = 0) of wave w) sampled in full; their estimates become the
  // rows' thresholds.  Steps >= 0: the tiles of this wave.
  const int ntl = wave < n_tiles ? (n_tiles - wave + 3) / 4 : 0;   // this wave's tiles
  bool queued = false;
  int jh = -1;
  for (int stp = prune ? -1 : 0; stp < ntl; ++stp) {
    bool fired = false;
    if (stp < 0) {
      if (c16 == 0) {
        const int rr = 4 * q4 + wave;
        int jj = -1;
        float p = 0.0f;
        const int lab = hint_labels ? lh[rr] : -2;
        if (lab >= 0) {
          jj = lab;
          p = lip[rr];
        } else if (lab == -2) {
          float b = mb[0][rr];
          p = hip_[0][rr];
          jj = mj[0][rr];
          for (int w = 1; w < 4; ++w)
            if (mb[w][rr] < b || (mb[w][rr] == b && mj[w][rr] < jj)) {
              b = mb[w][rr]; p = hip_[w][rr]; jj = mj[w][rr];
            }
        }
        if (row0 + rr < n && jj >= 0 && jj < k) {
          qj[threadIdx.x] = ((uint32_t)wave << 30) | (uint32_t)jj;
          qip[threadIdx.x] = p;
          qn = 1;
          queued = true;
          jh = jj;
        }
      }
    } else {
      const int t = wave + 4 * stp;
      const f32x4 acc = ipe_tile_ip<D4>(As, Cf + (size_t)t * D4 * 64 + lane, lane);
      const int j = t * 16 + c16;
      if (j < k) {   // padded centroid columns do nothing
        const float ny2 = cn[j];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const long long r = row0 + 4 * q4 + i;
          const uint32_t hnt = ((i < 2 ? hint01 : hint23) >> (16 * (i & 1))) & 0xFFFFu;
          if (r < n && (uint32_t)j != hnt) {
            bool full = true;
            if (prune) {
              uint32_t hq;
              float pbar;
              if (ipe_hazard(acc[i], nx2[i], ny2, sthr[i], sc, hq, pbar)) {
                full = false;
                if (hq > bud[i]) {   // the stream's budget runs out here: the pair fired
                  qj[qn * 256 + threadIdx.x] = ((uint32_t)i << 30) | (1u << 29) | (uint32_t)j;
                  qip[qn * 256 + threadIdx.x] = acc[i];
                  ++qn;
                  if (STATS) ++st_fire;
                  fired = true;
                } else {
                  bud[i] -= hq;
                  if (STATS) ++st_scr;
                }
              }
            }
            if (full) {
              qj[qn * 256 + threadIdx.x] = ((uint32_t)i << 30) | (uint32_t)j;
              qip[qn * 256 + threadIdx.x] = acc[i];
              ++qn;
            }
          }
        }
      }
    }
    // drain: after the hint step, after a fire (the stream's next budget is
    // drawn there, before its next pair), when a lane could overflow on the
    // next tile (room for 4 more), after the last tile
    const bool flush = stp < 0 || stp == ntl - 1 || qn > QCAP - 4 || fired;
    if (__ballot(flush && qn > 0) != 0ull) drain(stp);
    if (stp < 0) {
      if (c16 == 0) {
        hv[4 * q4 + wave] = queued ? bestv[wave * 256 + threadIdx.x] : INF;
        hj[4 * q4 + wave] = queued ? jh : -1;
      }
      __syncthreads();
      hint01 = hint23 = 0u;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int hi = hj[4 * q4 + i];
        const float b = hi >= 0 ? hv[4 * q4 + i] : INF;
        bestv[i * 256 + threadIdx.x] = b;
        bestj[i * 256 + threadIdx.x] = hi;
        sthr[i] = ipe_sthr(b);
        const uint32_t h16 = hi >= 0 ? (uint32_t)hi : 0xFFFFu;
        if (i < 2) hint01 |= h16 << (16 * i);
        else hint23 |= h16 << (16 * (i - 2));
      }
    }
  }
  // merge the 16 lanes (centroid classes) holding each row, then the 4 waves
  // (the order (D~, tie key, j) is total: any merge order gives the same pick)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float b = bestv[i * 256 + threadIdx.x];
    int jj = bestj[i * 256 + threadIdx.x];
    const long long g = row_offset + row0 + 4 * q4 + i;
    uint32_t kk = jj >= 0 ? band_key(tie_key, g, (uint32_t)jj) : 0xFFFFFFFFu;
    if (jj < 0) jj = 0x7fffffff;
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      const float ob = __shfl_xor(b, o, 64);
      const uint32_t ok = (uint32_t)__shfl_xor((int)kk, o, 64);
      const int oj = __shfl_xor(jj, o, 64);
      if (ipe_better(ob, ok, oj, b, kk, jj)) {
        b = ob;
        kk = ok;
        jj = oj;
      }
    }
    if (c16 == 0) {
      mb[wave][4 * q4 + i] = b;
      mk[wave][4 * q4 + i] = kk;
      mj[wave][4 * q4 + i] = jj;
    }
  }
  __syncthreads();
  if (threadIdx.x < 16) {
    const int rr = threadIdx.x;
    float b = mb[0][rr];
    uint32_t kk = mk[0][rr];
    int jj = mj[0][rr];
    for (int w = 1; w < 4; ++w)
      if (ipe_better(mb[w][rr], mk[w][rr], mj[w][rr], b, kk, jj)) {
        b = mb[w][rr];
        kk = mk[w][rr];
        jj = mj[w][rr];
      }
    const long long r = row0 + rr;
    if (r < n) {
      labels[r] = jj < k ? jj : 0;
      mind[r] = b;
    }
  }
  if (STATS) {
    const uint32_t v[4] = {st_scr, st_full, st_fire, st_exact};
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      uint32_t s = v[c];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) s += (uint32_t)__shfl_xor((int)s, o, 64);
      if (lane == c) atomicAdd(stats + c, (unsigned long long)s);
    }
    if (threadIdx.x == 4 && need_p1) atomicAdd(stats + 4, 1ull);
  }
}


// ------------------------------------------- row-group layout (production)
// R row groups of 16 rows per workgroup: every B fragment (one L2 load per
// k-step) feeds R MFMAs (R independent accumulator chains), so the centroid
// traffic per row drops R-fold; the R A fragments of a k-step are one LDS
// read (As[(s 64 + l) R + g]).
#ifndef SQ_IPE_KB
#define SQ_IPE_KB 16   // k-steps per fragment batch (two batches in flight)
#endif
template <int D4, int R>
SQ_DEV void ipe_tile_ipR(const float* __restrict__ As, const float* __restrict__ bf, int lane,
                         f32x4 (&acc)[R]) {
  constexpr int B = D4 < SQ_IPE_KB ? D4 : SQ_IPE_KB;
  static_assert(D4 % B == 0, "k-steps in whole batches");
  static_assert(R == 1 || R == 2, "one or two row groups");
#pragma unroll
  for (int g = 0; g < R; ++g) acc[g] = f32x4{0.f, 0.f, 0.f, 0.f};
  float a0[B][R], b0[B], a1[B][R], b1[B];
  auto lda = [&](float (&a)[B][R], int s) {
#pragma unroll
    for (int u = 0; u < B; ++u) {
      if constexpr (R == 2) {
        const float2 v = *reinterpret_cast<const float2*>(As + (size_t)((s + u) * 64 + lane) * 2);
        a[u][0] = v.x;
        a[u][1] = v.y;
      } else {
        a[u][0] = As[(s + u) * 64 + lane];
      }
    }
  };
#pragma unroll
  for (int u = 0; u < B; ++u) b0[u] = bf[u * 64];
  lda(a0, 0);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int s0 = 0; s0 < D4; s0 += 2 * B) {
    if (s0 + B < D4) {
#pragma unroll
      for (int u = 0; u < B; ++u) b1[u] = bf[(s0 + B + u) * 64];
      lda(a1, s0 + B);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < B; ++u)
#pragma unroll
      for (int g = 0; g < R; ++g)
        acc[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[u][g], b0[u], acc[g], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
    if (s0 + B < D4) {
      if (s0 + 2 * B < D4) {
#pragma unroll
        for (int u = 0; u < B; ++u) b0[u] = bf[(s0 + 2 * B + u) * 64];
        lda(a0, s0 + 2 * B);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < B; ++u)
#pragma unroll
        for (int g = 0; g < R; ++g)
          acc[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[u][g], b1[u], acc[g], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
}

// The samplers of one list entry (row-group kernel drains), out of line:
// the tile loop's register allocation does not carry the samplers' fp64
// state and their parameters (read from LDS here).
struct IpeDrainArgs {
  RngKey key, skip;
  double eps;
  int Q;
  IpeScreen sc;
};

__device__ __attribute__((noinline)) float ipe_entry_sample(
    float ip, float nxi, float cnj, float sthr, float thr, int j, int fired,
    unsigned long long sid, unsigned long long stream, const IpeDrainArgs* __restrict__ da,
    uint32_t* nb, int* exact) {
  const int Q = da->Q;
  const double eps = da->eps;
  if (!fired) return ipe_distance(ip, (double)nxi, (double)cnj, eps, Q, da->key, sid);
  // the same hazard as at the screen (same inputs, same code)
  uint32_t hq = 0;
  float pbar = 1.0f;
  const IpeScreen sc = da->sc;
  ipe_hazard(ip, nxi, cnj, sthr, sc, hq, pbar);
  WordStream ws(da->skip, stream);
  ws.b = (uint32_t)(2 * (j >> 6) + 1);   // step (t - class) / 4 = j / 64
  const uint32_t w0 = ws.next(), w1 = ws.next(), w2 = ws.next(), w3 = ws.next();
  *nb = ipe_budget(w0, w1);   // the stream's next budget
  const double beff = -expm1(-(double)hq * (1.0 / 4294967296.0));
  const double u = u53(w2, w3) * beff;
  const int h = (Q + 1) / 2;
  const double pib = binom_upper_tail((double)pbar, Q, h) * (1.0 + 1e-12);
  if (!(u < pib)) return __builtin_inff();
  *exact = 1;
  return ipe_pruned_exact((double)ip, (double)nxi + (double)cnj, eps, Q, thr, u, ws);
}

// Row thresholds from label hints, one lane per row (the pre-pass of the
// row-group kernel): the hint pair's inner product by 16 lanes (the fp32
// summation order of ipe_fused_kernel's hint path), then every lane samples
// its row's hint pair in full.  thr = its estimate, hj = the hint centroid;
// hj = -2 marks an invalid hint (the main kernel's first sweep decides).
template <bool STATS>
__global__ void __launch_bounds__(256) ipe_hint_kernel(
    const float* __restrict__ X, long long ldx, const float* __restrict__ C,
    const int* __restrict__ hint_labels, const float* __restrict__ xn,
    const float* __restrict__ cn, float* __restrict__ thr, int* __restrict__ hj, long long n, int d,
    int k, double eps, int Q, RngKey key, long long row_offset,
    unsigned long long* __restrict__ stats) {
  __shared__ float sip[256];
  __shared__ int slab[256];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c16 = lane & 15, q4 = lane >> 4;
  const long long rb = (long long)blockIdx.x * 256 + wave * 64;
  for (int it = 0; it < 16; ++it) {
    const int x = 4 * it + q4;
    const long long r = rb + x;
    const int l = r < n ? hint_labels[r] : -1;
    const bool ok = r < n && l >= 0 && l < k;
    float s = 0.0f;
    if (ok)
      for (int f = c16; f < d; f += 16) s = fmaf(X[(size_t)r * ldx + f], C[(size_t)l * d + f], s);
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) s += __shfl_xor(s, o, 64);
    if (c16 == 0) {
      sip[wave * 64 + x] = s;
      slab[wave * 64 + x] = ok ? l : -2;
    }
  }
  __syncthreads();
  const long long r = rb + lane;
  uint32_t full = 0;
  if (r < n) {
    const int l = slab[threadIdx.x];
    float t = __builtin_inff();
    if (l >= 0) {
      const long long g = row_offset + r;
      t = ipe_distance(sip[threadIdx.x], (double)xn[r], (double)cn[l], eps, Q, key,
                       (unsigned long long)g * (unsigned long long)k + (unsigned long long)l);
      full = 1;
    }
    thr[r] = t;
    hj[r] = l;
  }
  if (STATS) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) full += (uint32_t)__shfl_xor((int)full, o, 64);
    if (lane == 0) atomicAdd(stats + 1, (unsigned long long)full);
  }
}

// The production IPE kernel: 16 R rows per workgroup, the 4 waves split the
// centroid tiles (t = wave mod 4, as the streams' classes), register i of
// row group g of a lane = pair (row 16 g + 4 q4 + i, centroid 16 t + c16).
// Every (row, class, c16) stream, threshold, hazard, budget block and
// sampler stream is the one of ipe_fused_kernel above, so the two layouts
// return the same labels bit for bit.  Pairs that need a sampler are
// appended to a WAVE-wide LDS list (ballot + mbcnt); a drain runs them 64 at
// a time, one per lane.  The rows' thresholds come from ipe_hint_kernel
// (ext_thr / ext_hj) or, for rows without a hint, from a first exact sweep
// whose hint pairs wave 0 samples for the whole workgroup; what is left in
// the 4 lists after the last tile is drained as ONE pooled list (64-entry
// batches dealt to the waves) - the samplers' cost is paid per up-to-64
// pairs of a workgroup, not per up-to-64 pairs of a wave.  Each row's
// running best of a wave is held by lane (row) of that wave (registers);
// drain results reach it through a 64-entry LDS result batch.
template <int D4, int R, bool STATS>
__global__ void __launch_bounds__(256, 2) ipe_fused_rg_kernel(
    const float* __restrict__ X, long long ldx, const float* __restrict__ Cf,
    const float* __restrict__ ext_thr, const int* __restrict__ ext_hj,
    const float* __restrict__ xn, const float* __restrict__ cn, int* __restrict__ labels,
    float* __restrict__ mind, long long n, int d, int k, int n_tiles, double eps, int Q,
    RngKey key, RngKey tie_key, RngKey skip_key, IpeScreen sc, long long row_offset, int prune,
    unsigned long long* __restrict__ stats, const long long* __restrict__ rlist,
    const int* __restrict__ rcount) {
  constexpr int NR = 16 * R;                   // rows per workgroup
  constexpr int CAP = D4 >= 256 ? 256 : 512;   // wave list capacity (>= one unit's 256 pushes)
  extern __shared__ __attribute__((aligned(16))) float As[];   // [D4][64][R]
  __shared__ uint32_t qe[4][CAP];
  __shared__ float qip[4][CAP];
  __shared__ uint32_t re[4][64];
  __shared__ float rdt[4][64];
  __shared__ uint32_t nbud[4][256];            // [slot i][thread]: budgets redrawn by a drain
  __shared__ float r_nx2[NR], r_thr[NR], r_sthr[NR];
  __shared__ int r_hj[NR];
  __shared__ float mb[4][NR], mip[4][NR];
  __shared__ uint32_t mk[4][NR];
  __shared__ int mj[4][NR];
  __shared__ int qc[4];
  // per row: (|x|^2, sthr, hint centroid bits, row < n) - one LDS read per pair
  __shared__ float4 rinfo[NR];
  // the samplers' parameters, read by the drains from LDS (keeps them out of
  // the tile loop's scalar registers)
  __shared__ RngKey s_tie;
  __shared__ IpeDrainArgs s_da;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int c16 = lane & 15, q4 = lane >> 4;
  const long long row0 = (long long)blockIdx.x * NR;
  const float INF = __builtin_inff();
  uint32_t st_scr = 0, st_full = 0, st_fire = 0, st_exact = 0;
  // the workgroup's rows: row0 + rl, or (list mode: the dense rows of the
  // certified fp16 screen, ipe16.hip) rlist[row0 + rl]; -1 past the end
  __shared__ long long rid[NR];
  const long long nrow = rlist ? (long long)*rcount : n;
  if (row0 >= nrow) return;
  for (int rl = threadIdx.x; rl < NR; rl += 256)
    rid[rl] = row0 + rl < nrow ? (rlist ? rlist[row0 + rl] : row0 + rl) : -1;
  __syncthreads();
  if (threadIdx.x == 0) {
    s_tie = tie_key;
    s_da.key = key;
    s_da.skip = skip_key;
    s_da.eps = eps;
    s_da.Q = Q;
    s_da.sc = sc;
  }
  // A fragments: row rl, features 4 s .. 4 s + 3 (one lane: 16 contiguous
  // bytes) -> As[(s 64 + (rl mod 16) + 16 i) R + rl / 16], i = 0..3; the
  // lanes of a store take consecutive rows (2-way bank aliasing at most)
  for (int e = threadIdx.x; e < NR * D4; e += 256) {
    const int rl = e % NR, s4 = e / NR;
    const long long r = rid[rl] >= 0 ? rid[rl] : rid[0];
    const float* xr = X + (size_t)r * ldx;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int f = 4 * s4 + i;
      As[(s4 * 64 + (rl & 15) + 16 * i) * R + (rl >> 4)] = f < d ? xr[f] : 0.0f;
    }
  }
  // the rows' thresholds: given (hint pre-pass), or hj = -2: the first sweep's
  int need = 0;
  for (int rl = threadIdx.x; rl < NR; rl += 256) {
    const long long r = rid[rl];
    r_nx2[rl] = xn[r >= 0 ? r : rid[0]];
    float t = INF;
    int h = -1;
    if (prune && r >= 0) {
      if (ext_hj) {
        t = ext_thr[r];
        h = ext_hj[r];
      } else {
        h = -2;
      }
    }
    r_thr[rl] = t;
    r_hj[rl] = h;
    need |= h == -2 ? 1 : 0;
  }
  const bool need_p1 = __syncthreads_or(need) != 0;
  if (need_p1) {
    // ---- pass 1: exact fp32 distance argmin (hint), with its inner product
    float bd[R][4], bip[R][4], nxr[R][4];
    int bjj[R][4];
#pragma unroll
    for (int g = 0; g < R; ++g)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        bd[g][i] = INF;
        bip[g][i] = 0.0f;
        bjj[g][i] = 0x7fffffff;
        nxr[g][i] = r_nx2[16 * g + 4 * q4 + i];
      }
    for (int t = wave; t < n_tiles; t += 4) {
      f32x4 acc[R];
      ipe_tile_ipR<D4, R>(As, Cf + (size_t)t * D4 * 64 + lane, lane, acc);
      const int j = t * 16 + c16;
      if (j < k) {
        const float ny2 = cn[j];
#pragma unroll
        for (int g = 0; g < R; ++g)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float Dd = nxr[g][i] + ny2 - 2.0f * acc[g][i];
            if (Dd < bd[g][i]) { bd[g][i] = Dd; bjj[g][i] = j; bip[g][i] = acc[g][i]; }
          }
      }
    }
#pragma unroll
    for (int g = 0; g < R; ++g)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float b = bd[g][i], p = bip[g][i];
        int jj = bjj[g][i];
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          const float ob = __shfl_xor(b, o, 64), op = __shfl_xor(p, o, 64);
          const int oj = __shfl_xor(jj, o, 64);
          if (ob < b || (ob == b && oj < jj)) { b = ob; p = op; jj = oj; }
        }
        if (c16 == 0) {
          const int rl = 16 * g + 4 * q4 + i;
          mb[wave][rl] = b;
          mj[wave][rl] = jj;
          mip[wave][rl] = p;
        }
      }
    __syncthreads();
  }
  // hazard budgets of this lane's streams (row 16 g + 4 q4 + i, class wave, c16)
  u32x4 bud[R];
  auto stream_of = [&](int rl, int w, int c) -> unsigned long long {
    const long long g = row_offset + (rid[rl] >= 0 ? rid[rl] : 0);
    return (unsigned long long)g * 64ull + (unsigned long long)(w * 16 + c);
  };
#pragma unroll
  for (int g = 0; g < R; ++g) bud[g] = u32x4{0u, 0u, 0u, 0u};
  if (prune && rlist) {
    long long gr[R][4];
#pragma unroll
    for (int g = 0; g < R; ++g)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const long long r = rid[16 * g + 4 * q4 + i];
        gr[g][i] = row_offset + (r >= 0 ? r : 0);
      }
    ipe_initial_budgets_rows<R>(skip_key, gr, wave * 16 + c16, sc, bud);
  } else if (prune) {
    long long gb[R];
#pragma unroll
    for (int g = 0; g < R; ++g) gb[g] = row_offset + row0 + 16 * g + 4 * q4;
    ipe_initial_budgets<R>(skip_key, gb, wave * 16 + c16, sc, bud);
  }
  // this wave's running best of row `lane` (lanes < NR)
  float bestv = INF;
  int bestj = -1;
  int qcnt = 0;   // wave-uniform list length
  auto push = [&](bool p, uint32_t ent, float ip) {
    const unsigned long long m = __ballot(p);
    if (m != 0ull) {
      if (p) {
        const int pos = qcnt + (int)__builtin_amdgcn_mbcnt_hi(
                                   (uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        qe[wave][pos] = ent;
        qip[wave][pos] = ip;
      }
      qcnt += __popcll(m);
    }
  };
  // entry = j (14 bits) | owner lane << 14 | row << 20 | fired << 26.
  // mode 0: this wave's list, results to the row owners; 1: the hint pairs
  // (results are the rows' thresholds); 2: the 4 lists pooled, their 64-entry
  // batches dealt round-robin to the 4 waves.
  auto drain = [&](int mode) {
    const int tot = mode == 2 ? qc[0] + qc[1] + qc[2] + qc[3] : qcnt;
    const int bstep = mode == 2 ? 256 : 64;
    for (int b0 = mode == 2 ? 64 * wave : 0; b0 < tot; b0 += bstep) {
      int e = b0 + lane;
      if (e < tot) {
        int w = wave;
        if (mode == 2) {
          w = 0;
          while (e >= qc[w]) e -= qc[w++];
        }
        const uint32_t ent = qe[w][e];
        const float ip = qip[w][e];
        const int j = (int)(ent & 0x3fffu), ol = (int)((ent >> 14) & 63u);
        const int rl = (int)((ent >> 20) & 63u);
        const bool fired = (ent >> 26) & 1u;
        const long long g = row_offset + rid[rl];
        uint32_t nb = 0;
        int ex = 0;
        const float dt = ipe_entry_sample(
            ip, r_nx2[rl], cn[j], r_sthr[rl], r_thr[rl], j, fired ? 1 : 0,
            (unsigned long long)g * (unsigned long long)k + (unsigned long long)j,
            stream_of(rl, w, ol & 15), &s_da, &nb, &ex);
        if (fired) nbud[rl & 3][w * 64 + ol] = nb;
        if (STATS) {
          st_full += fired ? 0u : 1u;
          st_exact += (uint32_t)ex;
        }
        if (mode == 1) {
          r_thr[rl] = dt;
          r_hj[rl] = j;
        } else {
          re[wave][lane] = ent;
          rdt[wave][lane] = dt;
        }
      }
      if (mode != 1) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const int m = tot - b0 < 64 ? tot - b0 : 64;
        for (int x = 0; x < m; ++x) {
          const uint32_t ent = re[wave][x];
          const float dt = rdt[wave][x];
          if (lane == (int)((ent >> 20) & 63u)) {
            const int j = (int)(ent & 0x3fffu);
            bool take = dt < bestv;
            if (!take && dt == bestv && dt < INF) {   // tie: the random keys decide (rare)
              const long long g = row_offset + rid[lane];
              const RngKey tk_ = s_tie;
              const uint32_t tk = band_key(tk_, g, (uint32_t)j);
              const uint32_t bk = band_key(tk_, g, (uint32_t)bestj);
              take = tk < bk || (tk == bk && j < bestj);
            }
            if (take) {
              bestv = dt;
              bestj = j;
            }
          }
        }
        __builtin_amdgcn_wave_barrier();
      }
    }
    qcnt = 0;
  };
  // unit -1: the hint pairs of the rows without a threshold (wave 0, lane
  // = row); units 0 .. nun-1: (tile step, row group) of this wave; unit nun:
  // the pooled drain (every wave: qcnt = the pooled length)
  const int ntl = wave < n_tiles ? (n_tiles - wave + 3) / 4 : 0;
  const int nun = ntl * R;
  f32x4 accs[R];
  float ny2 = 0.0f;   // |c_j|^2 of this lane's centroid of the current tile
  for (int u = -1; u <= nun; ++u) {
    bool any_fired = false;
    int g = 0;
    uint32_t fmask = 0;
    int mode = 0;
    if (u < 0) {
      mode = 1;
      if (need_p1 && wave == 0) {
        const int rl = lane;
        bool p = false;
        uint32_t ent = 0;
        float ip = 0.0f;
        if (lane < NR && r_hj[rl] == -2) {
          float b = mb[0][rl];
          ip = mip[0][rl];
          int jj = mj[0][rl];
          for (int w = 1; w < 4; ++w)
            if (mb[w][rl] < b || (mb[w][rl] == b && mj[w][rl] < jj)) {
              b = mb[w][rl]; ip = mip[w][rl]; jj = mj[w][rl];
            }
          p = jj >= 0 && jj < k;
          if (!p) r_hj[rl] = -1;
          ent = (uint32_t)jj | ((uint32_t)rl << 20);
        }
        push(p, ent, ip);
      }
    } else if (u == nun) {
      mode = 2;
      qc[wave] = qcnt;
      __syncthreads();
      qcnt = qc[0] + qc[1] + qc[2] + qc[3];
    } else {
      const int stp = R == 2 ? u >> 1 : u;
      g = u - stp * R;
      const int t = wave + 4 * stp;
      const int j = t * 16 + c16;
      const bool jv = j < k;   // padded centroid columns do nothing
      if (g == 0) {
        ny2 = cn[jv ? j : 0];   // issued before the tile's MFMAs: no exposed L2 latency
        ipe_tile_ipR<D4, R>(As, Cf + (size_t)t * D4 * 64 + lane, lane, accs);
      }
      f32x4 acc = accs[0];
      u32x4 bd = bud[0];
      if constexpr (R == 2) {
        if (g) {
          acc = accs[1];
          bd = bud[1];
        }
      }
      // straight-line screen of the 4 pairs; one ballot decides whether any
      // lane appends (full-sampler pairs and fired pairs are rare)
      bool pp[4];
      if (prune) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float4 ri = rinfo[16 * g + 4 * q4 + i];
          const bool valid = jv & !(ri.w < 0.0f) & (j != __float_as_int(ri.z));
          uint32_t hq;
          float pbar;
          const bool ok = ipe_hazard(acc[i], ri.x, ny2, ri.y, ri.w, sc, hq, pbar) & valid;
          const bool fired = ok & (hq > bd[i]);   // the stream's budget runs out here
          const bool scr = ok & !fired;
          bd[i] = scr ? bd[i] - hq : bd[i];
          pp[i] = valid & !scr;
          fmask |= fired ? 1u << i : 0u;
          if (STATS) {
            st_fire += fired ? 1u : 0u;
            st_scr += scr ? 1u : 0u;
          }
        }
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float4 ri = rinfo[16 * g + 4 * q4 + i];
          pp[i] = jv & !(ri.w < 0.0f) & (j != __float_as_int(ri.z));
        }
      }
      if (__ballot(pp[0] || pp[1] || pp[2] || pp[3]) != 0ull) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int rl = 16 * g + 4 * q4 + i;
          push(pp[i],
               (uint32_t)j | ((uint32_t)lane << 14) | ((uint32_t)rl << 20) |
                   ((fmask >> i) & 1u) << 26,
               acc[i]);
        }
      }
      bud[0] = g == 0 ? bd : bud[0];
      if constexpr (R == 2) bud[1] = g ? bd : bud[1];
      any_fired = __ballot(fmask != 0u) != 0ull;
    }
    // drain: the hint pairs, after a fire (the stream's next budget is drawn
    // before its next pair, one tile step later), when the next unit could
    // overflow the list, the pooled rest
    if (qcnt > 0 && (u < 0 || u == nun || qcnt > CAP - 256 || any_fired)) {
      drain(mode);
      if (fmask) {
        u32x4 bd = bud[0];
        if constexpr (R == 2) bd = g ? bud[1] : bud[0];
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (fmask & (1u << i)) bd[i] = nbud[i][threadIdx.x];
        bud[0] = g == 0 ? bd : bud[0];
        if constexpr (R == 2) bud[1] = g ? bd : bud[1];
      }
    }
    if (u < 0) {
      __syncthreads();
      for (int rl = threadIdx.x; rl < NR; rl += 256) {
        const float st = ipe_sthr(r_thr[rl]);
        r_sthr[rl] = st;
        // .w: the row's hazard factor kt (>= 0 or NaN), -1 past the last row
        rinfo[rl] = make_float4(r_nx2[rl], st, __int_as_float(r_hj[rl]),
                                rid[rl] >= 0 ? ipe_kt(st) : -1.0f);
      }
      __syncthreads();
      if (lane < NR) {
        bestv = r_hj[lane] >= 0 ? r_thr[lane] : INF;
        bestj = r_hj[lane] >= 0 ? r_hj[lane] : -1;
      }
    }
  }
  // merge the 4 waves (the order (D~, tie key, j) is total)
  if (lane < NR) {
    const long long g = row_offset + (rid[lane] >= 0 ? rid[lane] : 0);
    mb[wave][lane] = bestv;
    mk[wave][lane] = bestj >= 0 ? band_key(s_tie, g, (uint32_t)bestj) : 0xFFFFFFFFu;
    mj[wave][lane] = bestj >= 0 ? bestj : 0x7fffffff;
  }
  __syncthreads();
  if (threadIdx.x < NR) {
    const int rr = threadIdx.x;
    float b = mb[0][rr];
    uint32_t kk = mk[0][rr];
    int jj = mj[0][rr];
    for (int w = 1; w < 4; ++w)
      if (ipe_better(mb[w][rr], mk[w][rr], mj[w][rr], b, kk, jj)) {
        b = mb[w][rr];
        kk = mk[w][rr];
        jj = mj[w][rr];
      }
    const long long r = rid[rr];
    if (r >= 0) {
      labels[r] = jj < k ? jj : 0;
      mind[r] = b;
    }
  }
  if (STATS) {
    const uint32_t v[4] = {st_scr, st_full, st_fire, st_exact};
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      uint32_t s = v[c];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) s += (uint32_t)__shfl_xor((int)s, o, 64);
      if (lane == c) atomicAdd(stats + c, (unsigned long long)s);
    }
    if (threadIdx.x == 4 && need_p1) atomicAdd(stats + 4, 1ull);
  }
}

}  // namespace sq

using namespace sq;

extern "C" int sq_ipe_fused(const void* X, long long ldx, const void* Cf, const void* C,
                            const void* hint_labels, const void* xn, const void* cn, void* labels,
                            void* mind, long long n, int d, int d_pad, int k, int k_pad, double eps,
                            int Q, unsigned k0, unsigned k1, unsigned s0, unsigned s1, unsigned t0,
                            unsigned t1, unsigned ts0, unsigned ts1, unsigned q0, unsigned q1,
                            unsigned qs0, unsigned qs1, long long row_offset, int prune,
                            void* stats, void* scratch, void* stream, const void* rlist,
                            const void* rcount, long long list_n, const void* ext_thr_in,
                            const void* ext_hj_in) {
  if (n <= 0) return 0;
  // list mode (rlist, rcount on the device, list_n >= *rcount rows on the
  // host for the grid): the row-group kernel over the listed rows, with the
  // thresholds / hints given (ext_thr_in / ext_hj_in, e.g. ipe16's prep)
  const long long* rl_p = (const long long*)rlist;
  const int* rc_p = (const int*)rcount;
  if (rl_p && (!rc_p || !ext_thr_in || !ext_hj_in || !(prune & 1) || !(Q & 1) || list_n <= 0))
    return rl_p && list_n == 0 ? 0 : (int)hipErrorInvalidValue;
  if (Q < 1 || Q > kIpeMaxQ || k < 1 || k_pad % 16 != 0 || k_pad < k || k_pad > 16384 || d < 1 ||
      d > d_pad || ldx < d || !(eps > 0.0) || (hint_labels && !C))
    return (int)hipErrorInvalidValue;
  RngKey key{k0, k1, s0, s1};
  RngKey tie{t0, t1, ts0, ts1};
  RngKey skip{q0, q1, qs0, qs1};
  IpeScreen sc;
  const int h = (Q + 1) / 2;
  double cq = 1.0;
  for (int i = 0; i < h; ++i) cq = cq * (double)(Q - i) / (double)(i + 1);
  sc.hf = (float)h;
  sc.cqh = (float)(cq * (1.0002 * (1.0 + 1e-6)));
  sc.kq = (float)((1.0 - 3e-6) * (1.0 - 1e-6) / (1.4142135623730951 * eps));
  sc.smax = (float)(6.0e10 * eps * (1.0 - 1e-6));
  sc.cap = (uint32_t)(((k + 63) / 64) * (1u << 23));   // <= 2^31 (k <= 16384)
  sc.ucap = exp(-(double)sc.cap * 0x1p-32);
  const int nt = k_pad / 16;
  const int pr = (prune & 1) && (Q & 1) ? 1 : 0;
  // layout (prune bits 1-2): 0 auto, 1 / 2 row groups, 3 the per-lane-queue kernel
  const int layout = (prune >> 1) & 3;
  hipStream_t hs = (hipStream_t)stream;
  unsigned long long* stp = (unsigned long long*)stats;
  // row-group layouts: label hints become thresholds in a pre-pass
  // (scratch: float thr[n] then int hj[n])
  float* ext_thr = nullptr;
  int* ext_hj = nullptr;
  if (rl_p) {
    ext_thr = (float*)ext_thr_in;
    ext_hj = (int*)ext_hj_in;
  } else if (layout != 3 && pr && hint_labels) {
    if (!scratch) return (int)hipErrorInvalidValue;
    ext_thr = (float*)scratch;
    ext_hj = (int*)((float*)scratch + n);
    const dim3 hg((unsigned)((n + 255) / 256));
    if (stats)
      ipe_hint_kernel<true><<<hg, 256, 0, hs>>>(
          (const float*)X, ldx, (const float*)C, (const int*)hint_labels, (const float*)xn,
          (const float*)cn, ext_thr, ext_hj, n, d, k, eps, Q, key, row_offset, stp);
    else
      ipe_hint_kernel<false><<<hg, 256, 0, hs>>>(
          (const float*)X, ldx, (const float*)C, (const int*)hint_labels, (const float*)xn,
          (const float*)cn, ext_thr, ext_hj, n, d, k, eps, Q, key, row_offset, nullptr);
  }
#define ARGS                                                                                    \
  (const float*)X, ldx, (const float*)Cf, (const float*)C, (const int*)hint_labels,             \
      (const float*)xn, (const float*)cn, (int*)labels, (float*)mind, n, d, k, nt, eps, Q, key, \
      tie, skip, sc, row_offset, pr
#define RARGS                                                                                   \
  (const float*)X, ldx, (const float*)Cf, ext_thr, ext_hj, (const float*)xn, (const float*)cn,  \
      (int*)labels, (float*)mind, n, d, k, nt, eps, Q, key, tie, skip, sc, row_offset, pr
#define OLD(DP)                                                                                 \
  {                                                                                             \
    const dim3 grid((unsigned)((n + 15) / 16));                                                 \
    if (stats)                                                                                  \
      ipe_fused_kernel<DP / 4, true><<<grid, 256, (size_t)DP * 64, hs>>>(ARGS, stp);            \
    else                                                                                        \
      ipe_fused_kernel<DP / 4, false><<<grid, 256, (size_t)DP * 64, hs>>>(ARGS, nullptr);       \
  }
#define RG(DP, RR)                                                                              \
  {                                                                                             \
    const long long nr_ = rl_p ? list_n : n;                                                    \
    const dim3 grid((unsigned)((nr_ + 16 * RR - 1) / (16 * RR)));                               \
    const size_t shm = (size_t)DP * 64 * RR;                                                    \
    if (shm > 64 * 1024) {   /* d_pad 2048: 128 KiB of A fragments, one workgroup per CU */     \
      static bool attr_ = false;                                                                \
      if (!attr_) {                                                                             \
        hipFuncSetAttribute((const void*)ipe_fused_rg_kernel<DP / 4, RR, true>,                  \
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);              \
        hipFuncSetAttribute((const void*)ipe_fused_rg_kernel<DP / 4, RR, false>,                 \
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);              \
        attr_ = true;                                                                           \
      }                                                                                         \
    }                                                                                           \
    if (stats)                                                                                  \
      ipe_fused_rg_kernel<DP / 4, RR, true><<<grid, 256, shm, hs>>>(RARGS, stp, rl_p, rc_p);    \
    else                                                                                        \
      ipe_fused_rg_kernel<DP / 4, RR, false><<<grid, 256, shm, hs>>>(RARGS, nullptr, rl_p, rc_p); \
  }
#define CASE(DP)                                                                                \
  case DP:                                                                                      \
    if (layout == 3 && !rl_p) OLD(DP)                                                           \
    else if (layout == 1 || DP > 256) RG(DP, 1)                                                 \
    else RG(DP, 2)                                                                              \
    break;
  switch (d_pad) {
    CASE(32)
    CASE(64)
    CASE(128)
    CASE(256)
    CASE(512)
    CASE(1024)
    case 2048:   // the row-group layout only (128 KiB of A fragments)
      RG(2048, 1)
      break;
    default:
      return (int)hipErrorInvalidValue;
  }
#undef CASE
#undef RG
#undef OLD
#undef ARGS
#undef RARGS
  return (int)hipGetLastError();
}
