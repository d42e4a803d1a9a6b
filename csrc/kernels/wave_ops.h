// Cross-lane wave64 primitives on the VALU (DPP row ops, row broadcasts, v_permlane16/32_swap,
// v_readlane) instead of the LDS crossbar: __shfl / __shfl_up / __shfl_xor lower to ds_bpermute_b32,
// a full LDS round trip per step (a 13-step softmax chain measured ~1.4k cycles that way).
// Shared by the MLP kernels (mlp_frag.h) and the tree split search (tree.hip).
#pragma once
#include "common.h"

namespace wops {

// DPP controls (GFX9 encoding, gfx950): row_shr:n 0x110 + n, row_ror:n 0x120 + n (16-lane rows),
// row_bcast:15 / :31 (lane 15 of each row -> the next row / lane 31 -> rows 2 and 3)
constexpr int DPP_SHR1 = 0x111, DPP_SHR2 = 0x112, DPP_SHR4 = 0x114, DPP_SHR8 = 0x118;
constexpr int DPP_ROR8 = 0x128, DPP_ROR4 = 0x124, DPP_ROR2 = 0x122, DPP_ROR1 = 0x121;
constexpr int DPP_BCAST15 = 0x142, DPP_BCAST31 = 0x143;
constexpr int DPP_QUAD_XOR1 = 0xb1;  // quad_perm [1,0,3,2]

// lanes whose source is outside the row (or whose row is masked off) read 0
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ int dpp_i(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, ROW_MASK, 0xf, false);
}
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ float dpp_f(float v) {
  return __builtin_bit_cast(float, dpp_i<CTRL, ROW_MASK>(__builtin_bit_cast(int, v)));
}
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = (uint32_t)dpp_i<CTRL>((int)(uint32_t)u), hi = (uint32_t)dpp_i<CTRL>((int)(uint32_t)(u >> 32));
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

// max as one v_max_f32: fmaxf of a DPP-moved value makes hipcc quiet both operands first (IEEE mode),
// two extra VALU per step on a dependent chain
__device__ __forceinline__ float vmaxf(float a, float b) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
// all-reduce over the 16 lanes of each DPP row (lanes 16r .. 16r + 15).  The max steps are single
// v_max_f32_dpp instructions (a DPP move + v_max_f32 is two): inline asm, with the s_nop 1 a DPP read
// of a VGPR written by the previous VALU instruction needs (the compiler does not see inside the asm)
__device__ __forceinline__ float row16_max(float v) {
  asm("s_nop 1\n\tv_max_f32_dpp %0, %0, %0 row_ror:8 row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1\n\tv_max_f32_dpp %0, %0, %0 row_ror:4 row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1\n\tv_max_f32_dpp %0, %0, %0 row_ror:2 row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1\n\tv_max_f32_dpp %0, %0, %0 row_ror:1 row_mask:0xf bank_mask:0xf"
      : "+v"(v));
  return v;
}
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp_f<DPP_ROR8>(v);
  v += dpp_f<DPP_ROR4>(v);
  v += dpp_f<DPP_ROR2>(v);
  return v + dpp_f<DPP_ROR1>(v);
}
__device__ __forceinline__ int row16_min(int v) {
  v = min(v, dpp_i<DPP_ROR8>(v));
  v = min(v, dpp_i<DPP_ROR4>(v));
  v = min(v, dpp_i<DPP_ROR2>(v));
  return min(v, dpp_i<DPP_ROR1>(v));
}

// The value lane ^ 16 / lane ^ 32 holds, by the gfx950 row / half swaps (VALU).  `self` of the swap of
// the lane's own id fixes which of the two outputs carries the partner, independent of the operand
// order convention.
struct LaneSwap {
  bool hi16, hi32;
  __device__ __forceinline__ explicit LaneSwap(int lane) {
    const auto a = __builtin_amdgcn_permlane16_swap((uint32_t)lane, (uint32_t)lane, false, false);
    const auto b = __builtin_amdgcn_permlane32_swap((uint32_t)lane, (uint32_t)lane, false, false);
    hi16 = a[0] == (uint32_t)(lane ^ 16);
    hi32 = b[0] == (uint32_t)(lane ^ 32);
  }
  __device__ __forceinline__ uint32_t x16(uint32_t v) const {
    const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return hi16 ? r[0] : r[1];
  }
  __device__ __forceinline__ uint32_t x32(uint32_t v) const {
    const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return hi32 ? r[0] : r[1];
  }
  __device__ __forceinline__ float x16f(float v) const { return __builtin_bit_cast(float, x16(__builtin_bit_cast(uint32_t, v))); }
  __device__ __forceinline__ float x32f(float v) const { return __builtin_bit_cast(float, x32(__builtin_bit_cast(uint32_t, v))); }
  __device__ __forceinline__ double x16d(double v) const {
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    return __builtin_bit_cast(double, ((uint64_t)x16((uint32_t)(u >> 32)) << 32) | x16((uint32_t)u));
  }
  __device__ __forceinline__ double x32d(double v) const {
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    return __builtin_bit_cast(double, ((uint64_t)x32((uint32_t)(u >> 32)) << 32) | x32((uint32_t)u));
  }
};

// inclusive prefix sum over each 32-lane half (lanes 0..31, 32..63): the 16-lane row scans, then
// lane 15's row total added to rows 1 and 3
__device__ __forceinline__ float scan32_add(float v) {
  v += dpp_f<DPP_SHR1>(v);
  v += dpp_f<DPP_SHR2>(v);
  v += dpp_f<DPP_SHR4>(v);
  v += dpp_f<DPP_SHR8>(v);
  return v + dpp_f<DPP_BCAST15, 0xa>(v);
}
// inclusive prefix sum over the wave
__device__ __forceinline__ float scan64_add(float v) {
  v = scan32_add(v);
  return v + dpp_f<DPP_BCAST31, 0xc>(v);
}
__device__ __forceinline__ int scan64_add(int v) {
  v += dpp_i<DPP_SHR1>(v);
  v += dpp_i<DPP_SHR2>(v);
  v += dpp_i<DPP_SHR4>(v);
  v += dpp_i<DPP_SHR8>(v);
  v += dpp_i<DPP_BCAST15, 0xa>(v);
  return v + dpp_i<DPP_BCAST31, 0xc>(v);
}

// all-reduce sum over the wave (every lane gets the total)
__device__ __forceinline__ float wave_sum_dpp(float v, const LaneSwap& sw) {
  v = row16_sum(v);
  v += sw.x16f(v);
  return v + sw.x32f(v);
}

// all-reduce sums over the wave on the VALU (the __shfl_xor butterfly of common.h's wave_sum / wave_sum_d
// is an LDS round trip per step, two per step for a double): row sums by DPP rotations, then the row and
// half swaps.  A swap of v with itself leaves {own, partner} in its two outputs, so the sum takes both
// outputs directly (no select; a + b == b + a, every lane ends with the same bits)
__device__ __forceinline__ float wave_sum_f_dpp(float v) {
  v = row16_sum(v);
  const uint32_t u = __builtin_bit_cast(uint32_t, v);
  const auto a = __builtin_amdgcn_permlane16_swap(u, u, false, false);
  v = __builtin_bit_cast(float, (uint32_t)a[0]) + __builtin_bit_cast(float, (uint32_t)a[1]);
  const uint32_t w = __builtin_bit_cast(uint32_t, v);
  const auto b = __builtin_amdgcn_permlane32_swap(w, w, false, false);
  return __builtin_bit_cast(float, (uint32_t)b[0]) + __builtin_bit_cast(float, (uint32_t)b[1]);
}
__device__ __forceinline__ double wave_sum_d_dpp(double v) {
  v += dpp_d<DPP_ROR8>(v);
  v += dpp_d<DPP_ROR4>(v);
  v += dpp_d<DPP_ROR2>(v);
  v += dpp_d<DPP_ROR1>(v);
  auto swap_add = [](double x, bool half) {
    const uint64_t u = __builtin_bit_cast(uint64_t, x);
    const uint32_t lo = (uint32_t)u, hi = (uint32_t)(u >> 32);
    const auto l = half ? __builtin_amdgcn_permlane32_swap(lo, lo, false, false)
                        : __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto h = half ? __builtin_amdgcn_permlane32_swap(hi, hi, false, false)
                        : __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    const double x0 = __builtin_bit_cast(double, ((uint64_t)(uint32_t)h[0] << 32) | (uint32_t)l[0]);
    const double x1 = __builtin_bit_cast(double, ((uint64_t)(uint32_t)h[1] << 32) | (uint32_t)l[1]);
    return x0 + x1;
  };
  v = swap_add(v, false);
  return swap_add(v, true);
}

// wave argmax of (gain, index): the largest gain, the lowest index among equal gains — an
// associative, commutative combine, so the butterfly order (half swap, row swap, row rotations)
// does not change the winner; every lane ends with it
__device__ __forceinline__ void argmax_combine(double& g, int& idx, double og, int oi) {
  if (og > g || (og == g && oi < idx)) {
    g = og;
    idx = oi;
  }
}
__device__ __forceinline__ void wave_argmax(double& g, int& idx, const LaneSwap& sw) {
  argmax_combine(g, idx, sw.x32d(g), (int)sw.x32((uint32_t)idx));
  argmax_combine(g, idx, sw.x16d(g), (int)sw.x16((uint32_t)idx));
  argmax_combine(g, idx, dpp_d<DPP_ROR8>(g), dpp_i<DPP_ROR8>(idx));
  argmax_combine(g, idx, dpp_d<DPP_ROR4>(g), dpp_i<DPP_ROR4>(idx));
  argmax_combine(g, idx, dpp_d<DPP_ROR2>(g), dpp_i<DPP_ROR2>(idx));
  argmax_combine(g, idx, dpp_d<DPP_ROR1>(g), dpp_i<DPP_ROR1>(idx));
}

// value of lane `l` (wave-uniform l) as a scalar read (v_readlane_b32)
__device__ __forceinline__ float lane_f(float v, int l) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}

}  // namespace wops
