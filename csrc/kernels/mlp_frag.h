// MFMA fragment helpers shared by the fused MLP kernels (mlp_fused.hip, mlp_step.hip).
//
// gfx950 16x16x32 bf16 MFMA (v_mfma_f32_16x16x32_bf16): lane l holds A[row l & 15][k = 8 (l >> 4) + i]
// and B[k = 8 (l >> 4) + i][col l & 15] (i < 8); C/D: col = l & 15, row = 4 (l >> 4) + reg.  The
// 16x16x16 form (_1k) takes 4 k per lane: k = 4 (l >> 4) + i.
#pragma once
#include "common.h"
#include "wave_ops.h"

namespace mlpf {

typedef __attribute__((ext_vector_type(4))) short s16x4_t;
typedef __attribute__((ext_vector_type(8))) short s16x8_t;
typedef __attribute__((address_space(3))) s16x4_t lds_s16x4_t;
typedef __attribute__((ext_vector_type(4))) uint32_t u32x4_t;
typedef __attribute__((ext_vector_type(2))) uint32_t u32x2_t;
typedef __attribute__((ext_vector_type(2))) short s16x2_t;
typedef __attribute__((ext_vector_type(2))) unsigned short u16x2_t;

typedef __attribute__((ext_vector_type(2))) float f32x2_t;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;

// two fp32 -> one packed bf16 pair: a single v_cvt_pk_bf16_f32 (round to nearest even).  Packing two
// scalar conversions instead makes hipcc pair the wrong operands and re-assemble the halves with
// shifts / ORs (~6 extra VALU per pair).
__device__ __forceinline__ uint32_t pack2(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2_t{a, b}, bf16x2_t));
}

// element offset of lane l's 16 bytes (row l & 15, k 8 (l >> 4) .. + 7) inside a 1 KB fragment block
// of the fragment-ordered weight copies (mlp.hip frag_pos: lane order)
__device__ __forceinline__ int frag_lane_off(int lane) { return lane * 8; }

__device__ __forceinline__ f32x4_t mma32(bf16x8_t a, bf16x8_t b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4_t mma16(s16x4_t a, s16x4_t b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ bf16x8_t cat8(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  return __builtin_bit_cast(bf16x8_t, u32x4_t{a, b, c, d});
}

// relu of two packed bf16 (sign bit set = negative, -0 -> +0): one v_pk_max_i16
__device__ __forceinline__ uint32_t relu2(uint32_t p) {
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(s16x2_t, p), s16x2_t{0, 0}));
}

// Non-temporal 16-byte store (one global_store_dwordx4 ... nt; the consumer is the next kernel)
__device__ __forceinline__ void nt_store16(void* p, u32x4_t v) {
  __builtin_nontemporal_store(v, reinterpret_cast<u32x4_t*>(p));
}

// Write-through (sc1) stores through a raw buffer descriptor of `base` (wave-uniform): the line is not
// left dirty in the XCD's L2, so the dependent launch's boundary does not wait for its write-back
// (MI355X_MICROARCH boundary row: + bytes / 6 TB/s of dirty L2 at a kernel's end).  byte_off < 2^31.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wt_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ void wt_store16(__amdgpu_buffer_rsrc_t r, uint32_t byte_off, u32x4_t v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, byte_off, 0, 16);
}
__device__ __forceinline__ void wt_store4(__amdgpu_buffer_rsrc_t r, uint32_t byte_off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, byte_off, 0, 16);
}

// MFMA operand fragment (8 consecutive k of column lane & 15, natural k order) of a [k][cols] bf16
// LDS image: two transposing 4 x 16 reads per lane
__device__ __forceinline__ bf16x8_t frag_tr(const bf16_t* img, int pitch, int col0, int lane) {
  const int li = lane & 15, g = lane >> 4;
  const bf16_t* p0 = img + (8 * g + (li >> 2)) * pitch + col0 + 4 * (li & 3);
  const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)p0);
  const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(p0 + 4 * pitch));
  const s16x8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, v);
}

// Same with the permuted k order of a 32-row step: lane group g supplies rows 4g..4g+3 and
// 16+4g..16+4g+3 (both operands of a product must use it).  With a row pitch of an odd multiple
// of 8 dwords the 32 lanes of an LDS bank group read 8 consecutive rows: conflict-free.
__device__ __forceinline__ bf16x8_t frag_rows(const bf16_t* img, int pitch, int col0, int lane) {
  const int li = lane & 15, g = lane >> 4;
  const bf16_t* p0 = img + (4 * g + (li >> 2)) * pitch + col0 + 4 * (li & 3);
  const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)p0);
  const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(p0 + 16 * pitch));
  const s16x8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, v);
}

// frag_rows of an image whose rows with bit 2 set have their 16-byte column chunks swapped in pairs
// (column ^ 8; col0 a multiple of 16): the lane's rows 4g + (li >> 2) (+ 16) all have bit 2 = g & 1
__device__ __forceinline__ bf16x8_t frag_rows_sw(const bf16_t* img, int pitch, int col0, int lane) {
  const int li = lane & 15, g = lane >> 4;
  const bf16_t* p0 = img + (4 * g + (li >> 2)) * pitch + col0 + ((4 * (li & 3)) ^ (8 * (g & 1)));
  const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)p0);
  const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(p0 + 16 * pitch));
  const s16x8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, v);
}

// frag_rows of an image whose 4-column (8-byte) chunks are XOR-swizzled by row within each 16-column
// block: the chunk of columns 4c .. 4c + 3 of row r lives at chunk c ^ ((r >> 2) & 3) (col0 a multiple
// of 16).  The lane's rows 4g + (li >> 2) (+ 16, + 32 ks) all have (r >> 2) & 3 = g.  8-byte stores of
// 16 consecutive rows at one column (bank group of 16 lanes) then hit 32 distinct banks at a pitch of
// 40 dwords (unswizzled: 4-way), and these transposing reads stay conflict-free.
__device__ __forceinline__ bf16x8_t frag_rows_q(const bf16_t* img, int pitch, int col0, int lane) {
  const int li = lane & 15, g = lane >> 4;
  const bf16_t* p0 = img + (4 * g + (li >> 2)) * pitch + col0 + 4 * ((li & 3) ^ g);
  const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)p0);
  const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(p0 + 16 * pitch));
  const s16x8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, v);
}

// frag_rows of an image whose 4-column chunks are XOR-permuted per row: `x` = the chunk XOR of the
// lane's rows 4g + (li >> 2) (+ 16) (the caller's swizzle must give those rows one value)
__device__ __forceinline__ bf16x8_t frag_rows_x(const bf16_t* img, int pitch, int col0, int lane, int x) {
  const int li = lane & 15, g = lane >> 4;
  const bf16_t* p0 = img + (4 * g + (li >> 2)) * pitch + col0 + 4 * ((li & 3) ^ x);
  const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)p0);
  const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(p0 + 16 * pitch));
  const s16x8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, v);
}

// packed bf16 pair `v` times relu'(h) of the packed relu'd bf16 pair `h` (each half in [0, 0x7fff]):
// min(half, 1) is the 0 / 1 derivative, a 16-bit multiply applies it — 2 VALU per pair.  Inline asm:
// written as vector min / multiply, clang turns it into 16-bit compares + selects + repacking
__device__ __forceinline__ uint32_t relu_d_mul(uint32_t v, uint32_t h) {
  uint32_t d, r;
  asm("v_pk_min_u16 %0, %1, 1 op_sel_hi:[1,0]" : "=v"(d) : "v"(h));
  asm("v_pk_mul_lo_u16 %0, %1, %2" : "=v"(r) : "v"(v), "v"(d));
  return r;
}

// cross-lane steps on the VALU (DPP / permlane): wave_ops.h (dpp_i / dpp_f, vmaxf, row16_*, LaneSwap)
using namespace wops;

}  // namespace mlpf
