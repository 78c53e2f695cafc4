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
#include <sys/mman.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstdint>
#include <thread>
#include <vector>

#include "host.h"

namespace {

struct MT19937 {
  uint32_t* key;
  int pos;
  uint32_t tmp[624];   // the tempered outputs of the current block (one pass per twist)
  void temper_all() {
    for (int q = 0; q < 624; ++q) {
      uint32_t y = key[q];
      y ^= y >> 11;
      y ^= (y << 7) & 0x9d2c5680u;
      y ^= (y << 15) & 0xefc60000u;
      y ^= y >> 18;
      tmp[q] = y;
    }
  }
  void twist() {
    constexpr uint32_t kUpper = 0x80000000u, kLower = 0x7fffffffu, kMatrix = 0x9908b0dfu;
    int i = 0;
    for (; i < 624 - 397; ++i) {
      const uint32_t y = (key[i] & kUpper) | (key[i + 1] & kLower);
      key[i] = key[i + 397] ^ (y >> 1) ^ ((0u - (y & 1u)) & kMatrix);
    }
    for (; i < 623; ++i) {
      const uint32_t y = (key[i] & kUpper) | (key[i + 1] & kLower);
      key[i] = key[i + 397 - 624] ^ (y >> 1) ^ ((0u - (y & 1u)) & kMatrix);
    }
    const uint32_t y = (key[623] & kUpper) | (key[0] & kLower);
    key[623] = key[396] ^ (y >> 1) ^ ((0u - (y & 1u)) & kMatrix);
    temper_all();
    pos = 0;
  }
  inline uint32_t next32() {
    if (pos >= 624) twist();
    return tmp[pos++];
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
  // the array on 2 MiB pages (transparent huge pages on request): the random
  // a[j] accesses otherwise miss the TLB nearly every time.  Allocated before
  // the generator starts, so a failed allocation leaves (key, pos) untouched.
  const size_t huge = (size_t)2 << 20;
  const size_t bytes = ((size_t)n * sizeof(int32_t) + huge - 1) & ~(huge - 1);
  int32_t* a = static_cast<int32_t*>(std::aligned_alloc(huge, bytes > 0 ? bytes : huge));
  if (!a) return 2;
  madvise(a, bytes, MADV_HUGEPAGE);
  MT19937 g;
  g.key = key;
  g.pos = *pos;
  g.temper_all();
  const long long steps = n > 1 ? n - 1 : 0;   // i = n - 1 .. 1
  // Two threads: the generator stream is sequential and so are the swaps,
  // but they only meet through the swap targets - a producer draws the
  // targets of chunk c (MT19937 + the rejection loop) while the main thread
  // initialises the array and then applies chunk c - 1's swaps (random
  // a[j] accesses, prefetched a batch ahead inside the known chunk).
  constexpr long long CH = 1 << 15;   // steps per chunk
  constexpr int NCH = 8;              // chunks in flight
  const long long nchunks = (steps + CH - 1) / CH;
  std::vector<int32_t> ring((size_t)NCH * CH);
  std::atomic<long long> produced{0}, consumed{0};
  std::thread producer([&] {
    for (long long c = 0; c < nchunks; ++c) {
      while (c - consumed.load(std::memory_order_acquire) >= NCH) std::this_thread::yield();
      int32_t* dst = ring.data() + (size_t)(c % NCH) * CH;
      const long long i0 = n - 1 - c * CH;
      const long long m = std::min(CH, steps - c * CH);
      for (long long t = 0; t < m; ++t) dst[t] = (int32_t)g.interval((uint64_t)(i0 - t));
      produced.store(c + 1, std::memory_order_release);
    }
  });
  for (long long i = 0; i < n; ++i) a[(size_t)i] = (int32_t)i;
  constexpr int PF = 48;   // prefetch distance (swaps)
  for (long long c = 0; c < nchunks; ++c) {
    while (produced.load(std::memory_order_acquire) <= c) std::this_thread::yield();
    const int32_t* js = ring.data() + (size_t)(c % NCH) * CH;
    const long long i0 = n - 1 - c * CH;
    const long long m = std::min(CH, steps - c * CH);
    for (long long t = 0; t < std::min<long long>(PF, m); ++t) __builtin_prefetch(&a[(size_t)js[t]], 1, 0);
    for (long long t = 0; t < m; ++t) {
      if (t + PF < m) __builtin_prefetch(&a[(size_t)js[t + PF]], 1, 0);
      const long long i = i0 - t, j = js[t];
      const int32_t v = a[(size_t)i];
      a[(size_t)i] = a[(size_t)j];
      a[(size_t)j] = v;
    }
    consumed.store(c + 1, std::memory_order_release);
  }
  producer.join();
  for (long long i = 0; i < k; ++i) out[i] = a[(size_t)i];
  std::free(a);
  *pos = g.pos;
  return 0;
}
