// Philox4x32-10 on the device, bit-identical to har/ops/rng.py:
// counter = (idx_lo, idx_hi, stream, "HAR!"), key = (seed_lo, seed_hi).
#pragma once
#include <stdint.h>

__device__ __forceinline__ void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
    const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
    const uint32_t n1 = (uint32_t)p1;
    const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
    const uint32_t n3 = (uint32_t)p0;
    c[0] = n0; c[1] = n1; c[2] = n2; c[3] = n3;
  }
}

__device__ __forceinline__ uint32_t philox_u32(uint64_t seed, uint32_t stream, uint64_t idx) {
  uint32_t c[4] = {(uint32_t)idx, (uint32_t)(idx >> 32), stream, 0x48415221u};
  philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  return c[0];
}
