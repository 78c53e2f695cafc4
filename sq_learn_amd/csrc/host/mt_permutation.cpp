// Head of numpy RandomState.permutation(n) (legacy MT19937 stream), native.
//
// The reference's 'random' initialisation is ``random_state.permutation(n)
// [:k]`` (sklearn/cluster/_kmeans.py _init_centroids); reproducing its draws
// needs the whole Fisher-Yates pass over arange(n) (every draw moves the
// stream and any position can end up in the head).  numpy runs it over an
// int64 array; here the same pass runs over int32 (n < 2^31) with an inlined
// MT19937 and the legacy bounded-integer rejection (random_interval: mask to
// the next power of two minus one, redraw while above the bound; 32-bit draws
// for bounds < 2^32).  The generator state is read from and written back to
// the caller's (key[624], pos), so the Python RandomState continues exactly
// where numpy's own permutation would have left it.
#include <cstdint>
#include <vector>

#include "host.h"

namespace {

struct MT19937 {
  uint32_t* key;
  int pos;
  void twist() {
    constexpr uint32_t kUpper = 0x80000000u, kLower = 0x7fffffffu, kMatrix = 0x9908b0dfu;
    int i = 0;
    for (; i < 624 - 397; ++i) {
      const uint32_t y = (key[i] & kUpper) | (key[i + 1] & kLower);
      key[i] = key[i + 397] ^ (y >> 1) ^ ((y & 1u) ? kMatrix : 0u);
    }
    for (; i < 623; ++i) {
      const uint32_t y = (key[i] & kUpper) | (key[i + 1] & kLower);
      key[i] = key[i + 397 - 624] ^ (y >> 1) ^ ((y & 1u) ? kMatrix : 0u);
    }
    const uint32_t y = (key[623] & kUpper) | (key[0] & kLower);
    key[623] = key[396] ^ (y >> 1) ^ ((y & 1u) ? kMatrix : 0u);
    pos = 0;
  }
  inline uint32_t next32() {
    if (pos >= 624) twist();
    uint32_t y = key[pos++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
  }
  inline uint64_t next64() {
    const uint64_t hi = next32();
    return (hi << 32) | next32();
  }
  inline uint64_t interval(uint64_t mx) {
    if (mx == 0) return 0;
    uint64_t mask = mx;
    mask |= mask >> 1;
    mask |= mask >> 2;
    mask |= mask >> 4;
    mask |= mask >> 8;
    mask |= mask >> 16;
    mask |= mask >> 32;
    uint64_t v;
    if (mx <= 0xffffffffull) {
      while ((v = (next32() & mask)) > mx) {
      }
    } else {
      while ((v = (next64() & mask)) > mx) {
      }
    }
    return v;
  }
};

}  // namespace

extern "C" int sqh_mt_permutation_head(uint32_t* key, int* pos, long long n, long long k,
                                                long long* out) {
  if (n < 0 || k < 0 || k > n || n >= (1LL << 31) || *pos < 0 || *pos > 624) return 1;
  MT19937 g{key, *pos};
  std::vector<int32_t> a((size_t)n);
  for (long long i = 0; i < n; ++i) a[(size_t)i] = (int32_t)i;
  // the draws of the next B steps first (the stream is sequential, the
  // swap targets are not): their cache lines are prefetched, then the swaps
  // run in the original order - the random a[j] reads were the cost
  constexpr int B = 64;
  long long js[B];
  for (long long i0 = n - 1; i0 >= 1; i0 -= B) {
    const int m = (int)(i0 >= B ? B : i0);
    for (int t = 0; t < m; ++t) {
      js[t] = (long long)g.interval((uint64_t)(i0 - t));
      __builtin_prefetch(&a[(size_t)js[t]], 1, 0);
    }
    for (int t = 0; t < m; ++t) {
      const long long i = i0 - t, j = js[t];
      const int32_t v = a[(size_t)i];
      a[(size_t)i] = a[(size_t)j];
      a[(size_t)j] = v;
    }
  }
  for (long long i = 0; i < k; ++i) out[i] = a[(size_t)i];
  *pos = g.pos;
  return 0;
}
