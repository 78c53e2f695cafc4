// delta-band selection rule shared by every E-step kernel (csrc/kmeans.hip,
// csrc/estep_f32.hip) and the torch twin (ops/kmeans.py band_select_torch).
//
// members M = {j : D_j <= min + delta}, c = |M|, ordered by
// kappa(j) = (j mod 32, j div 32); the label is the member of rank
// r = floor(u * c), u = u01(word g of key) - ONE Philox word per row (not per
// member), so the band resolution costs a few wave ops.  A uniform choice
// among the qualifying indices, like the reference's ``random.choice``
// (``sklearn/cluster/_dmeans.py:742-751``).
#pragma once
#include "common.h"

namespace sq {

SQ_DEV uint32_t band_key(const RngKey& key, long long grow, uint32_t j) {
  unsigned long long idx = ((unsigned long long)grow << 16) | (unsigned long long)j;
  return key.block(idx).x;
}

SQ_DEV float band_u(const RngKey& key, long long grow) {
  return u01(key.word((unsigned long long)grow));
}
SQ_DEV int band_rank(float u, int c) {
  int r = (int)(u * (float)c);
  return r < c ? r : c - 1;
}
// position of the (r+1)-th set bit of m (r < popcount(m))
SQ_DEV int nth_set_bit(unsigned long long m, int r) {
  int pos = 0;
#pragma unroll
  for (int w = 32; w > 0; w >>= 1) {
    const unsigned long long lo = m & ((1ull << w) - 1ull);
    const int c = __popcll(lo);
    if (r >= c) { r -= c; m >>= w; pos += w; } else { m = lo; }
  }
  return pos;
}
// One wave picks the band member of rank r for one row; lanes scan
// j = lane + 64 t.  dist(j) must be a pure function (called in two passes);
// T is the distance type (float rows of the fused kernels, double rows of
// the fp64 re-check).
template <typename T, typename DistF>
SQ_DEV int band_pick_wave(DistF dist, int k, T thr, float u, int lane) {
  int c = 0;
  for (int j = lane; j < k; j += 64) c += dist(j) <= thr ? 1 : 0;
  const int cr = c + __shfl_xor(c, 32, 64);          // count of class rho = lane & 31
  int incl = cr;
#pragma unroll
  for (int o = 1; o < 32; o <<= 1) {
    const int v = __shfl_up(incl, o, 32);
    if ((lane & 31) >= o) incl += v;
  }
  const int total = __shfl(incl, 31, 64);
  if (total == 0) return -1;
  const int r = band_rank(u, total);
  const unsigned long long hit = __ballot(lane < 32 && incl > r);
  const int rho = __ffsll((long long)hit) - 1;
  int rr = r - __shfl(incl - cr, rho, 64);
  for (int base = 0;; base += 64) {                  // members of class rho in j order
    const int j = rho + 32 * (base + lane);
    const bool mem = j < k && dist(j) <= thr;
    const unsigned long long b = __ballot(mem);
    const int cnt = __popcll(b);
    if (rr < cnt) return rho + 32 * (base + nth_set_bit(b, rr));
    rr -= cnt;
    if (rho + 32 * base >= k) return -1;             // unreachable for a consistent dist
  }
}

}  // namespace sq
