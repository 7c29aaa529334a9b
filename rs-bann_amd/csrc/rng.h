// rng.h — counter-based Philox4x32-10 for device-side sampling (synthetic
// cohorts, momenta).  Stateless: every draw is a pure function of
// (seed, stream, counter), so results do not depend on the launch geometry.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

struct u32x4 {
  uint32_t x, y, z, w;
};

__host__ __device__ inline uint32_t mulhi32(uint32_t a, uint32_t b) {
  return (uint32_t)(((uint64_t)a * (uint64_t)b) >> 32);
}

__host__ __device__ inline u32x4 philox4x32(u32x4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0 = mulhi32(0xD2511F53u, c.x), lo0 = 0xD2511F53u * c.x;
    uint32_t hi1 = mulhi32(0xCD9E8D57u, c.z), lo1 = 0xCD9E8D57u * c.z;
    c = u32x4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// 4 uniform draws in [0, 1) (24-bit resolution) for counter (stream, idx).
__host__ __device__ inline u32x4 philox_bits(uint64_t seed, uint64_t stream, uint64_t idx) {
  u32x4 c{(uint32_t)idx, (uint32_t)(idx >> 32), (uint32_t)stream, (uint32_t)(stream >> 32)};
  return philox4x32(c, (uint32_t)seed, (uint32_t)(seed >> 32));
}

__host__ __device__ inline float u01(uint32_t x) { return (float)(x >> 8) * (1.0f / 16777216.0f); }
// strictly inside (0, 1)
__host__ __device__ inline float u01_open(uint32_t x) { return ((float)(x >> 8) + 0.5f) * (1.0f / 16777216.0f); }
