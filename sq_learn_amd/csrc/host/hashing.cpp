// MurmurHash3_x86_32 and the feature-hashing transform.
//
// Reference behaviour: ``utils/murmurhash.pyx`` (murmurhash3_int_u32 /
// murmurhash3_bytes_s32 ..., seed, positive flag) over the public-domain
// MurmurHash3_x86_32 (``utils/src/MurmurHash3.cpp:105``), and
// ``feature_extraction/_hashing_fast.pyx`` (index = |h| mod n_features, value
// sign from h < 0 when alternate_sign).  Written from the algorithm's
// specification: 4-byte little-endian blocks, c1/c2 multipliers, rotl 15/13,
// tail bytes, fmix32 finaliser.
#include <cstdint>
#include <cstring>

#include "host.h"

namespace sqh {

static inline uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

static inline uint32_t fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h;
}

uint32_t murmur3_32(const void* key, int len, uint32_t seed) {
  const uint8_t* data = static_cast<const uint8_t*>(key);
  const int nblocks = len / 4;
  uint32_t h1 = seed;
  const uint32_t c1 = 0xcc9e2d51u, c2 = 0x1b873593u;
  for (int i = 0; i < nblocks; ++i) {
    uint32_t k1;
    std::memcpy(&k1, data + 4 * i, 4);   // little-endian host (x86-64)
    k1 *= c1;
    k1 = rotl32(k1, 15);
    k1 *= c2;
    h1 ^= k1;
    h1 = rotl32(h1, 13);
    h1 = h1 * 5 + 0xe6546b64u;
  }
  const uint8_t* tail = data + 4 * nblocks;
  uint32_t k1 = 0;
  switch (len & 3) {
    case 3: k1 ^= uint32_t(tail[2]) << 16; [[fallthrough]];
    case 2: k1 ^= uint32_t(tail[1]) << 8; [[fallthrough]];
    case 1:
      k1 ^= tail[0];
      k1 *= c1;
      k1 = rotl32(k1, 15);
      k1 *= c2;
      h1 ^= k1;
  }
  h1 ^= uint32_t(len);
  return fmix32(h1);
}

}  // namespace sqh

extern "C" {

// int32 keys (hashed as their 4 little-endian bytes); out: uint32 bit pattern
void sqh_murmur_i32(const int32_t* keys, long long n, uint32_t seed, uint32_t* out) {
  for (long long i = 0; i < n; ++i) out[i] = sqh::murmur3_32(&keys[i], 4, seed);
}

// byte strings packed back to back; offsets has n + 1 entries
void sqh_murmur_bytes(const uint8_t* buf, const long long* offsets, long long n, uint32_t seed,
                      uint32_t* out) {
  for (long long i = 0; i < n; ++i)
    out[i] = sqh::murmur3_32(buf + offsets[i], (int)(offsets[i + 1] - offsets[i]), seed);
}

// Feature hashing of (string feature, value) pairs: column = |h_s32| mod
// n_features (h = INT_MIN maps to (INT_MAX - (n_features - 1)) mod n_features,
// as the reference does); value *= -1 when alternate_sign and h_s32 < 0.
void sqh_hash_features(const uint8_t* buf, const long long* offsets, const double* values,
                       long long n, long long n_features, int alternate_sign, uint32_t seed,
                       int32_t* cols, double* vals) {
  for (long long i = 0; i < n; ++i) {
    const int32_t h = (int32_t)sqh::murmur3_32(buf + offsets[i],
                                               (int)(offsets[i + 1] - offsets[i]), seed);
    if (h == INT32_MIN)
      cols[i] = (int32_t)((2147483647LL - (n_features - 1)) % n_features);
    else
      cols[i] = (int32_t)((h < 0 ? -(long long)h : (long long)h) % n_features);
    double v = values[i];
    if (alternate_sign && h < 0) v = -v;
    vals[i] = v;
  }
}

}  // extern "C"
