// sq_learn_amd native layer - shared device helpers for gfx950 (CDNA4).
//
// * Philox4x32-10 counter RNG, bit-identical to sq_learn_amd/runtime/rng.py
//   (counter = (idx_lo, idx_hi, stream_lo, stream_hi), key = seed).
// * uniform / normal / truncated-normal transforms shared by every kernel.
// * wave64 reductions (CDNA wavefront = 64 lanes, never 32).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#define SQ_DEV __device__ __forceinline__

namespace sq {

// ---------------------------------------------------------------- Philox
struct u4 { uint32_t x, y, z, w; };

SQ_DEV void mulhilo32(uint32_t a, uint32_t b, uint32_t& hi, uint32_t& lo) {
  uint64_t p = (uint64_t)a * (uint64_t)b;
  hi = (uint32_t)(p >> 32);
  lo = (uint32_t)p;
}

SQ_DEV u4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                        uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
    uint32_t hi0, lo0, hi1, lo1;
    mulhilo32(0xD2511F53u, c0, hi0, lo0);
    mulhilo32(0xCD9E8D57u, c2, hi1, lo1);
    uint32_t n0 = hi1 ^ c1 ^ k0;
    uint32_t n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
  }
  return u4{c0, c1, c2, c3};
}

struct RngKey {
  uint32_t k0, k1, s0, s1;
  SQ_DEV u4 block(uint64_t idx) const {
    return philox4x32_10((uint32_t)idx, (uint32_t)(idx >> 32), s0, s1, k0, k1);
  }
  // uniform word for flat element e: word (e & 3) of block (e >> 2)
  SQ_DEV uint32_t word(uint64_t e) const {
    u4 b = block(e >> 2);
    uint32_t m = (uint32_t)(e & 3);
    return m == 0 ? b.x : (m == 1 ? b.y : (m == 2 ? b.z : b.w));
  }
};

// (0,1) open uniform from 24 high bits - identical to rng.uniform_from_u32
SQ_DEV float u01(uint32_t x) { return ((float)(x >> 8) + 0.5f) * (1.0f / 16777216.0f); }
SQ_DEV double u01d(uint32_t x) { return ((double)(x >> 8) + 0.5) * (1.0 / 16777216.0); }

// standard normal truncated to [-b, b] from one uniform word
SQ_DEV float trunc_normal(uint32_t w, float b, float erf_b) {
  float v = 2.0f * u01(w) - 1.0f;
  float z = 1.41421356237f * erfinvf(v * erf_b);
  return fminf(fmaxf(z, -b), b);
}

// ---------------------------------------------------------------- waves
SQ_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
SQ_DEV double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
SQ_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// positive-float atomic max through the int bit pattern (values >= 0)
SQ_DEV void atomic_max_pos(float* addr, float v) {
  atomicMax(reinterpret_cast<int*>(addr), __float_as_int(v));
}

SQ_DEV float bf16_to_f32(uint16_t h) { return __uint_as_float(((uint32_t)h) << 16); }
SQ_DEV uint16_t f32_to_bf16_rne(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7F800000u) == 0x7F800000u) return (uint16_t)((u >> 16) | ((u & 0xFFFF) ? 0x40 : 0));
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

}  // namespace sq
