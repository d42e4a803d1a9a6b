// Shared helpers for the gfx950 (CDNA4) kernels of the har framework.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
typedef uint16_t bf16_t;  // raw bf16 storage

#define HAR_WAVE 64

__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }

__device__ __forceinline__ bf16_t f2bf(float f) {
  // round-to-nearest-even in hardware: the cast lowers to v_cvt_pk_bf16_f32 on gfx950 (two
  // adjacent conversions share one instruction) instead of a 5-op integer rounding sequence
  return __builtin_bit_cast(bf16_t, (__bf16)f);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Bijective XCD-aware remap of a linear workgroup id (guide §5.5 T1): blocks that
// the dispatcher places on the same XCD (id % 8) get a contiguous range of tiles.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  if (nwg <= 8) return orig;
  int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

#define HAR_CHECK_LAUNCH() \
  do { hipError_t e__ = hipGetLastError(); if (e__ != hipSuccess) return (int)e__; } while (0)
