// Fused training step of the flagship MLP (BASELINE.json config 3: 43-256-256-6, bf16 MFMA; SURVEY.md
// K23), H = 256 hidden units, K0 = 32 / 64 padded inputs, <= 16 classes, batch a multiple of 64.
// Three kernels per step: mlp_fwd3 -> mlp_bwd4 (the wave-specialized backward) -> grad_reduce_adam
// (mlp.hip).
//
// The forward hands the backward dact2 = (dz . Wout) * relu'(h2) ([B][256] bf16, written in the
// backward's LDS tile order with its chunk swizzle); the backward recomputes h1 = relu(W0 x + b0)
// from the X tiles it reads anyway.
//
// mlp_fwd3 (persistent, one 8-wave workgroup per CU, 32-row tiles).  Wave w owns hidden units
// [32w, 32w + 32) of both layers; its slices of W0, W1 and Wout stay in registers.  Per tile:
//   stage 1  h1^T = W0 . X^T (bias as the initial accumulator) -> LDS h1 tile        | B1
//   stage 5  (previous tile) dWout^T += h2^T . dz over its 32 rows (operands from LDS images) and
//            dact2 of the wave's units (16x16x16 MFMAs, relu'(h2) from the h2 image) -> global
//   stage 2  h2^T = W1 . h1^T (h1 from LDS, 16-byte reads, software-pipelined)
//   stage 3  partial logits over the wave's 32 units -> LDS; h2 images for stage 5      | B2
//   softmax  spread over ALL 512 lanes — lane = (row 4w + g, class c16): the 8 partials in a fixed
//            order, max / sum over the 16 class lanes of the row, CE, argmax, dz -> LDS
// Two barriers per tile and no serial section: stage 5 of a tile runs after the next tile's B1, so
// the dz exchange needs no barrier of its own (dz and the h2 images are double-buffered).
//
// mlp_bwd4 (S row slices x 4 h1-unit quadrants of 64 units; 64-row tiles, one barrier per tile;
// producer waves 0-3 / consumer waves 4-7, see the kernel's comment):
//   producers: dact2 tile i+1 (copied, loaded two tiles ahead) -> LDS | X tile i+2 -> LDS | h1 tile
//              i+1 recomputed from X | (c) dW0 += dact1^T . X and db0 of tile i-1
//   consumers: (a) dact1^T = W1^T[u] . dact2^T, relu'(h1) | (b) dW1 += h1^T . dact2 | db1 = sum_rows
//              dact2 (a ones-row MFMA, 64 j per quadrant)
// One deterministic partial per (slice, quadrant), laid out like the flat parameter buffer.
#include <algorithm>
#include <type_traits>
#include <cstdlib>

#include "common.h"
#include "mlp_frag.h"
#include "../har_kernels.h"

using namespace mlpf;

// Diagnostic phase stamps (tools/mlp_phase_probe.py --stamps): a separate STAMP instantiation of the
// step kernels, launched only while a stamp buffer is set, has lane 0 of every wave store s_memtime
// (shader clock) at fixed points into its own 40-slot row of that buffer (slots 38 / 39:
// s_memrealtime at entry / exit, 100 MHz, one clock for the whole chip).  Nothing else reads them.
uint64_t* g_har_mlp_stamps = nullptr;

namespace {

constexpr size_t STAMP_BWD_OFF = (size_t)256 * 8 * 40;  // the backward's rows follow the forward's
#define HAR_STAMP(NW, k)                                                                                   \
  if constexpr (STAMP) {                                                                                   \
    if ((threadIdx.x & 63) == 0)                                                                           \
      stamps[((size_t)blockIdx.x * (NW) + (threadIdx.x >> 6)) * 40 + (k)] = __builtin_amdgcn_s_memtime();  \
  }
#define HAR_STAMP_REAL(NW, k)                                                                                  \
  if constexpr (STAMP) {                                                                                       \
    if ((threadIdx.x & 63) == 0)                                                                               \
      stamps[((size_t)blockIdx.x * (NW) + (threadIdx.x >> 6)) * 40 + (k)] = __builtin_amdgcn_s_memrealtime(); \
  }

constexpr int NCLS = 16;
constexpr int HH = 256;

// ------------------------------------------------------------------------------------------------
// forward
// ------------------------------------------------------------------------------------------------
constexpr int FW = 8;                  // waves (2 per SIMD)
constexpr int FRT = 32;                // rows per tile
// h1 tile: pitch 136 dwords, and the 16-byte column chunks of rows with bit 2 set swapped in pairs
// (column ^ 8): the 16-byte reads of stage 2 are conflict-free (the stage-1 8-byte stores 2-way)
constexpr int FHP = HH + 16;
// [32 rows][16 cols] images (dz, h2) read by stage 5: unpadded rows (8 dwords) with their four 4-column
// chunks XOR-permuted by row — h2 images: chunk c of row r at c ^ fh(r), fh(r) = 2 ((r >> 2) & 1);
// dz: c ^ fz(r), fz(r) = 2 ((r >> 3) & 1).  The 16-byte relu' reads, the dz reads and the transposing
// fragment reads are conflict-free, the stage-3 8-byte stores 2-way (an odd fh making those
// conflict-free too needs a lane-dependent swap of the relu' words: 8 more VALU per tile)
constexpr int FSP = 16;
constexpr int FIMG = FRT * FSP;
// partial logits of one (wave, half): lane group g's 16 lanes x 4 classes at dword 72 g + 4 c16: the
// softmax lanes (row, class) then read 16 distinct banks per row and disjoint banks per row pair
constexpr int ZREG = 4 * 72;
constexpr int FWD_SLAB = NCLS * HH + NCLS;  // per workgroup: dWout rows 0..15 [16][H], dbout [16]
#ifndef HAR_FWD_PD
#define HAR_FWD_PD 2
#endif
#ifndef HAR_FWD_KROT
#define HAR_FWD_KROT 0
#endif
#ifndef HAR_FWD_PIN
#define HAR_FWD_PIN 1
#endif
constexpr int FPD = HAR_FWD_PD;      // stage-2 h1 read prefetch distance (k chunks)
constexpr bool FPIN = HAR_FWD_PIN;   // pin the read / MFMA interleave with scheduling groups
// FILL (template argument, HAR_MLP_FWD_FILL): VALU instructions of the tile's softmax interleaved
// after each stage-2 MFMA (0: the softmax runs on its own, before stage 5)
constexpr size_t FWD_LDS = (size_t)2 * FRT * FHP * 2 + (size_t)2 * FW * 2 * ZREG * 4 + (size_t)2 * FIMG * 2 +
                           (size_t)FW * 4 * FIMG * 2;

template <int K0>
__device__ __forceinline__ bf16x8_t ldx(const bf16_t* __restrict__ X, int row, int kc, int g) {
  return *reinterpret_cast<const bf16x8_t*>(X + (size_t)row * K0 + kc * 32 + g * 8);
}

// INFER: the serving forward of the same pipeline — no labels, no dz / relu' mask / dWout / W1^T copy;
// `slab` receives the logits [B][C] (fp32, bias included) and `block_correct` the argmax [B].
template <int K0, bool STAMP, bool INFER = false, int FFILL = 0>
__global__ __launch_bounds__(512) void mlp_fwd3_kernel(
    const bf16_t* __restrict__ X, bf16_t* __restrict__ Wf, const float* __restrict__ b0,
    const float* __restrict__ b1, const bf16_t* __restrict__ Wo,
    const float* __restrict__ bo, const int32_t* __restrict__ labels, int B, int C, float scale,
    bf16_t* __restrict__ dact2_out, float* __restrict__ slab,
    float* __restrict__ block_loss, int32_t* __restrict__ block_correct, uint64_t* __restrict__ stamps,
    int stagger, int wt) {
  constexpr int K0C = K0 / 32, KC = HH / 32;
  extern __shared__ __attribute__((aligned(16))) bf16_t lds[];
  bf16_t* const h1s = lds;                                                // [2 bufs][32][FHP]
  float* const zs = reinterpret_cast<float*>(h1s + 2 * FRT * FHP);        // [2 bufs][8 waves][2 halves][ZREG]
  bf16_t* const dzs = reinterpret_cast<bf16_t*>(zs + 2 * FW * 2 * ZREG);  // [2 bufs][32 rows][FSP]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int c16 = lane & 15, g = lane >> 4;
  const int u0 = wave * 32;
  bf16_t* const img = dzs + 2 * FIMG + wave * 4 * FIMG;                 // [2 bufs][2 unit tiles][32][FSP]
  HAR_STAMP_REAL(FW, 38)
  HAR_STAMP(FW, 0)

  // softmax lane: tile row sr = 4 wave + g (half sh, row srr of it), class c16
  const int sr = 4 * wave + g, sh = sr >> 4, srr = sr & 15;
  const int hsw = 8 * ((c16 >> 2) & 1);  // h1 tile chunk swap of this lane's rows (16h + c16)
  // stage-5 image chunk XORs of this lane's rows 16 h + c16 (FSP)
  const int fh_row = 2 * ((c16 >> 2) & 1), fz_row = 2 * ((c16 >> 3) & 1);
  f32x4_t acc5[2] = {f32x4_t{0.f, 0.f, 0.f, 0.f}, f32x4_t{0.f, 0.f, 0.f, 0.f}};
  float dbo = 0.f, lsum = 0.f, ncorr = 0.f;
  const int ntiles = B / FRT;
  const int nt = (int)blockIdx.x < ntiles ? (ntiles - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
  // tile k of this workgroup; past the last one clamped to it (staged, computed, never consumed), so
  // every load is unconditional and the compiler's counted waits stay exact on every path
  auto tile_of = [&](int k) __attribute__((always_inline)) { return (int)blockIdx.x + min(k, nt - 1) * (int)gridDim.x; };
  bf16x8_t xb[2][K0C];
  auto load_x = [&](int k) __attribute__((always_inline)) {
    const int r = tile_of(k) * FRT;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int kc = 0; kc < K0C; ++kc)  // (uniform tile base + 32-bit lane offset: SGPR-base loads)
        xb[h][kc] = *reinterpret_cast<const bf16x8_t*>((X + (size_t)r * K0) + ((16 * h + c16) * K0 + kc * 32 + g * 8));
  };

  // ---- this wave's weight slices, in registers for the whole kernel, from the fragment-ordered
  // copies (MlpFragSpec: one 1 KB-contiguous load per fragment).  Issue order: W0, b0, the first X
  // tile and its labels, THEN W1 / Wout / b1 (the bulk: 16 KB per wave), so stage 1 of tile 0 waits
  // only for what it reads ----
  const bf16_t* const W0f = Wf;
  const bf16_t* const W1f = Wf + HH * K0;
  bf16x8_t w0f[2][K0C], w1f[2][KC];
  // k-chunk rotation per workgroup (register kc holds chunk (kc + krot)): the CUs' prologue requests
  // spread over the lines of W1 instead of all asking for the same ones together
  // (off: with a per-workgroup rotation every stage-2 LDS read needs a VALU address add; the rotation
  // did not measurably shorten the prologue)
  const int krot = HAR_FWD_KROT ? (int)blockIdx.x & (KC - 1) : 0;
  float4 b0r[2], b1r[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
#pragma unroll
    for (int kc = 0; kc < K0C; ++kc)
      w0f[t][kc] = *reinterpret_cast<const bf16x8_t*>(W0f + (size_t)((2 * wave + t) * K0C + kc) * 512 + frag_lane_off(lane));
    b0r[t] = *reinterpret_cast<const float4*>(b0 + u0 + 16 * t + 4 * g);
  }
  int ynext = 0;
  if (nt > 0) {
    load_x(0);
    if constexpr (!INFER) ynext = (labels + (size_t)tile_of(0) * FRT)[sr];
  }
  __builtin_amdgcn_sched_barrier(0);
  // b1 first, then W1 k-chunk-major (both unit tiles of chunk kc together): tile 0's stage 2 waits, at
  // chunk kc, only for the loads up to that chunk, so the tail of the W1 stream overlaps its MFMAs
#pragma unroll
  for (int t = 0; t < 2; ++t) b1r[t] = *reinterpret_cast<const float4*>(b1 + u0 + 16 * t + 4 * g);
#pragma unroll
  for (int kc = 0; kc < KC; ++kc)
#pragma unroll
    for (int t = 0; t < 2; ++t)
      w1f[t][kc] = *reinterpret_cast<const bf16x8_t*>(W1f + (size_t)((2 * wave + t) * KC + ((kc + krot) & (KC - 1))) * 512 + frag_lane_off(lane));
  // stage-3 A fragment: Wout[class c16][u0 + 4g + j] (j < 4), [u0 + 16 + 4g + j - 4] (j >= 4): the k
  // order of the h2 register pairs (C layout: unit 4g + r of a 16-unit tile in register r)
  const uint2 wlo = *reinterpret_cast<const uint2*>(Wo + (size_t)c16 * HH + u0 + 4 * g);
  const uint2 whi = *reinterpret_cast<const uint2*>(Wo + (size_t)c16 * HH + u0 + 16 + 4 * g);
  const bf16x8_t wo3 = cat8(wlo.x, wlo.y, whi.x, whi.y);
  // padded class lanes (c16 >= C): bias -inf, so their logit is -inf, exp 0, dz 0 with no per-lane selects
  const float bo_s = c16 < C ? bo[c16] : -INFINITY;
  // dact2 A fragments (16x16x16, K = the 16 classes): row m of block t is unit 8 (m >> 2) + 4 t + (m & 3)
  // of the wave's 32 (C row 4 g + r -> unit 8 g + 4 t + r: blocks t = 0, 1 give each lane the 8
  // CONSECUTIVE units 8 g .. 8 g + 7 of a row, one 16-byte store); A[m][k = class 4 g + i] =
  // Wout[4 g + i][u0 + 8 (c16 >> 2) + 4 t + (c16 & 3)]
  s16x4_t woT[2];
  if constexpr (!INFER) {
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        woT[t][i] = (short)Wo[(size_t)(4 * g + i) * HH + u0 + 8 * (c16 >> 2) + 4 * t + (c16 & 3)];
  }
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (STAMP) __builtin_amdgcn_s_waitcnt(0x0f70);
  HAR_STAMP(FW, 1)
  // ---- stage 1: h1^T = W0 . X^T for this wave's units -> h1 buffer `buf` ----
  // (the backward recomputes h1 from X: writing it here for the backward to copy — write-through,
  // 16-byte granules — cost the forward ~4 us of store traffic and saved the backward nothing,
  // profiles/r6/mlp_h1_copy_ab.md)
  auto stage1 = [&](int buf) __attribute__((always_inline)) {
    bf16_t* hb = h1s + buf * FRT * FHP;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        f32x4_t a = {b0r[t].x, b0r[t].y, b0r[t].z, b0r[t].w};
#pragma unroll
        for (int kc = 0; kc < K0C; ++kc) a = mma32(w0f[t][kc], xb[h][kc], a);
        *reinterpret_cast<uint2*>(hb + (16 * h + c16) * FHP + ((u0 + 16 * t + 4 * g) ^ hsw)) =
            make_uint2(relu2(pack2(a[0], a[1])), relu2(pack2(a[2], a[3])));
      }
  };
  // ---- stages 2 + 3 of tile k from h1 buffer `buf`: h2^T = W1 . h1^T, relu' mask, partial logits
  // -> zs buffer `buf`, h2 images for stage 5 -> image buffer `buf` ----
  auto stage23 = [&](int k, int buf, auto&& fill) __attribute__((always_inline)) {
    const int r0 = tile_of(k) * FRT;
    const bf16_t* hsrc = h1s + buf * FRT * FHP;
    f32x4_t acc[2][2];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int t = 0; t < 2; ++t) acc[h][t] = f32x4_t{b1r[t].x, b1r[t].y, b1r[t].z, b1r[t].w};
    // software-pipelined h1 reads (prefetch distance FPD k chunks, pinned by scheduling groups: the 2
    // reads of chunk kc + FPD, then the 4 MFMAs of chunk kc).  Left to the scheduler each chunk's two
    // reads were issued right before its MFMAs and every chunk waited out an LDS round trip (stage
    // 2 + 3 ~1.9k cycles per wave for 34 MFMAs, profiles/r5)
    bf16x8_t hb[KC][2];
    if constexpr (FPIN) __builtin_amdgcn_sched_barrier(0);  // an isolated region: the groups take only these
    auto ld_hb = [&](int kc) __attribute__((always_inline)) {
#pragma unroll
      for (int h = 0; h < 2; ++h)
        hb[kc][h] = *reinterpret_cast<const bf16x8_t*>(hsrc + (16 * h + c16) * FHP +
                                                        ((8 * g) ^ hsw) + ((kc + krot) & (KC - 1)) * 32);
    };
#pragma unroll
    for (int kc = 0; kc < FPD; ++kc) ld_hb(kc);
    // the previous tile's softmax (a dependent VALU / DPP chain on partial logits read before stage 5):
    // its VALU work goes into the MFMA shadow, FFILL instructions after each MFMA
    fill();
    if constexpr (FPIN) __builtin_amdgcn_sched_group_barrier(0x100, 2 * FPD, 0);  // the FPD chunks ahead
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      if (kc + FPD < KC) {
        ld_hb(kc + FPD);
        if constexpr (FPIN) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
      }
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int t = 0; t < 2; ++t) acc[h][t] = mma32(w1f[t][kc], hb[kc][h], acc[h][t]);
      if constexpr (FPIN) {
        if constexpr (FFILL > 0) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, FFILL, 0);
          }
        } else {
          __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
        }
      }
    }
    if constexpr (FPIN) __builtin_amdgcn_sched_barrier(0);
    uint32_t h2p[2][2][2];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        h2p[h][t][0] = relu2(pack2(acc[h][t][0], acc[h][t][1]));
        h2p[h][t][1] = relu2(pack2(acc[h][t][2], acc[h][t][3]));
      }
    float* zb = zs + buf * FW * 2 * ZREG;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const f32x4_t zp = mma32(wo3, cat8(h2p[h][0][0], h2p[h][0][1], h2p[h][1][0], h2p[h][1][1]),
                               f32x4_t{0.f, 0.f, 0.f, 0.f});
      *reinterpret_cast<f32x4_t*>(zb + (wave * 2 + h) * ZREG + 72 * g + 4 * c16) = zp;
    }
    if constexpr (!INFER) {
      bf16_t* ib = img + buf * 2 * FIMG;
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int t = 0; t < 2; ++t)
          *reinterpret_cast<uint2*>(ib + t * FIMG + (16 * h + c16) * FSP + 4 * (g ^ fh_row)) =
              make_uint2(h2p[h][t][0], h2p[h][t][1]);
    }
  };
  // ---- softmax / CE / argmax / dz of tile k (zs buffer `buf`): lane = (row sr, class c16) ----
  // (split: sm_load issues the 8 partial-logit reads, sm_compute the rest)
  auto sm_load = [&](int buf, float (&zp)[FW]) __attribute__((always_inline)) {
    const float* zb = zs + buf * FW * 2 * ZREG;
#pragma unroll
    for (int w = 0; w < FW; ++w) zp[w] = zb[(w * 2 + sh) * ZREG + 72 * (c16 >> 2) + 4 * srr + (c16 & 3)];
  };
  auto sm_compute = [&](int k, int buf, int yc, const float (&zp)[FW]) __attribute__((always_inline)) {
    const int r0 = tile_of(k) * FRT;
    float z = 0.f;
#pragma unroll
    for (int w = 0; w < FW; ++w) z += zp[w];
    asm volatile("" : "+v"(z));  // computed by every lane: no exec-masked branch splits the loop body
    const float zz = z + bo_s;  // (-inf on the padded class lanes: their partial logits are 0)
    // the 16 class lanes of a row are one DPP row: max, argmax (smallest class at the max), sum
    const float mx = row16_max(zz);
    const int amx = row16_min(zz == mx ? c16 : (1 << 30));  // (mx is finite: C >= 1 real classes)
    if constexpr (INFER) {
      if (c16 < C) slab[(size_t)(r0 + sr) * C + c16] = zz;
      if (c16 == 0) block_correct[r0 + sr] = amx;
      return;
    }
    const float e = __expf(zz - mx);  // exactly 0 on the padded class lanes
    const float se = row16_sum(e);
    // v_rcp_f32 (1 ulp) rather than the IEEE division sequence, which hipcc sinks into an
    // exec-masked branch; dz is rounded to bf16 right after (0 on the padded class lanes: e = 0, yc < C)
    const float dl = (e * __builtin_amdgcn_rcpf(se) - (c16 == yc ? 1.f : 0.f)) * scale;
    const bf16_t db = f2bf(dl);
    // ln se as v_log_f32 * ln 2: se >= 1 (the max term is exp 0), so no denormal range scaling
    lsum += c16 == yc ? (mx + __builtin_amdgcn_logf(se) * 0.693147180559945f) - zz : 0.f;
    ncorr += (c16 == 0 && amx == yc) ? 1.f : 0.f;
    dbo += bf2f(db);
    dzs[buf * FIMG + sr * FSP + (c16 ^ (8 * ((sr >> 3) & 1)))] = db;
  };
  auto softmax = [&](int k, int buf, int yc) __attribute__((always_inline)) {
    float zp[FW];
    sm_load(buf, zp);
    sm_compute(k, buf, yc, zp);
  };
  auto no_fill = [] {};
  // ---- stage 5 of a tile (dz buffer / image buffer `buf`, rows r0 ..): dWout^T += h2^T . dz over its
  // 32 rows, and the backward's layer-2 gradient dact2 = (dz . Wout) * relu'(h2) of the wave's 32
  // units -> dact2_out (bf16 [B][256], the 16-byte chunks of rows with bit 2 set swapped in pairs —
  // the backward's LDS tile image, so its producers copy rows verbatim).  Two 16x16x16 MFMAs per 16
  // rows (K = the 16 classes, unit-permuted A rows: woT) give lane (c16, g) the units 8 g .. 8 g + 7 of
  // row c16: one 16-byte relu' read of the wave's own h2 image, one 16-byte global store ----
  // (a wave-uniform row base + a 32-bit lane offset: the stores take the SGPR-base form, no 64-bit
  // address arithmetic per store)
  const int d2off = c16 * HH + ((u0 + 8 * g) ^ hsw);
  const __amdgpu_buffer_rsrc_t d2rs = wt_rsrc(dact2_out);
  auto stage5 = [&](int buf, int r0) __attribute__((always_inline)) {
    const bf16_t* zb = dzs + buf * FIMG;
    // (the permuted k order of frag_rows on both operands: k runs over the 32 tile rows)
    const bf16x8_t bz = frag_rows_x(zb, FSP, 0, lane, 2 * (g >> 1));
    const bf16_t* ip = img + buf * 2 * FIMG;
#pragma unroll
    for (int t = 0; t < 2; ++t) acc5[t] = mma32(frag_rows_x(ip + t * FIMG, FSP, 0, lane, 2 * (g & 1)), bz, acc5[t]);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const s16x4_t dzb = *reinterpret_cast<const s16x4_t*>(zb + (16 * h + c16) * FSP + 4 * (g ^ fz_row));
      // h2 units 8 g .. 8 g + 7 of row 16 h + c16: image block g >> 1, columns 8 (g & 1) .. — chunks
      // 2 (g & 1), + 1 at the 16-byte pair (g & 1) ^ (fh >> 1)
      const u32x4_t hv = *reinterpret_cast<const u32x4_t*>(ip + (g >> 1) * FIMG + (16 * h + c16) * FSP +
                                                           8 * ((g & 1) ^ (fh_row >> 1)));
      const f32x4_t v0 = mma16(woT[0], dzb, f32x4_t{0.f, 0.f, 0.f, 0.f});
      const f32x4_t v1 = mma16(woT[1], dzb, f32x4_t{0.f, 0.f, 0.f, 0.f});
      // relu'(h2): a relu'd bf16 half is in [0, 0x7fff], so min(half, 1) is the 0 / 1 derivative and
      // a 16-bit multiply applies it (v_pk_min_u16 + v_pk_mul_lo_u16: 2 VALU per dword, was 5)
      // (inline asm: written as vector min / multiply, clang turns them into 16-bit compares + selects +
      // repacking, 7 VALU per dword; and __builtin_bit_cast of a vector-element lvalue, hv[e], read
      // element 0 for every e with this clang — checked on the host)
      const uint32_t ov[4] = {pack2(v0[0], v0[1]), pack2(v0[2], v0[3]), pack2(v1[0], v1[1]), pack2(v1[2], v1[3])};
      u32x4_t o;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const uint32_t he = hv[e];
        o[e] = relu_d_mul(ov[e], he);
      }
      if (wt) {  // (uniform: a kernel argument)
        wt_store16(d2rs, (uint32_t)(((r0 + 16 * h) * HH + d2off) * 2), o);
      } else {
        bf16_t* const rowp = dact2_out + (size_t)(r0 + 16 * h) * HH;
        *reinterpret_cast<u32x4_t*>(rowp + d2off) = o;
      }
    }
  };

  // Software pipeline, ONE barrier per tile.  Iteration k: softmax of tile k | stage 5 of tile k-1 |
  // stages 2 + 3 of tile k+1 | stage 1 of tile k+2 | barrier.  The softmax's dependent chain (LDS
  // reads, cross-lane max / sum, exp / log) and the next tile's MFMAs share one barrier interval, so
  // the scheduler interleaves them; h1, the partial logits, dz and the h2 images are double-buffered.
  if (nt > 0) {
    stage1(0);
    load_x(1);
    __syncthreads();  // h1 of tile 0
    stage23(0, 0, no_fill);
    stage1(1);
    load_x(2);
    __syncthreads();  // partial logits of tile 0, h1 of tile 1
  }
  // iteration k: softmax(k) | stage5(k-1) | stages 2+3 (k+1) | stage1 (k+2).  The first and the last
  // iterations are peeled so the steady-state body is ONE basic block (no k > 0 / k + 1 < nt
  // branches): the scheduler can then interleave the softmax's VALU / DPP chain with the stage-2
  // MFMAs instead of running them back to back.
  // Staggered roles (stagger != 0): the two waves of a SIMD (w and w + 4) run the SAME phases of an
  // iteration in a different ORDER — waves 0..3 softmax(k) first, waves 4..7 last (after stage 5 and
  // the next tile's MFMA stages) — so one wave's VALU / DPP softmax chain issues beside its partner's
  // stage-2 MFMAs instead of both SIMD partners reaching the softmax (MFMA pipe idle) and then the
  // MFMAs (pipe shared) together.  Legal: within an iteration the phases touch disjoint buffers
  // (softmax: zs[k], dzs[k]; stage 5: dzs[k-1], the wave's own img[k-1]; stages 2 + 3: h1[k+1] ->
  // zs[k+1], own img[k+1]; stage 1: h1[k+2]) and the wave's own img[k-1] is read before its img[k+1]
  // (the same buffer) is written in both orders.
  auto iter = [&](int k, bool first, bool last, auto late) __attribute__((always_inline)) {
    if (k < 32) HAR_STAMP(FW, 2 + k)
    const int yc = ynext;
    if constexpr (!INFER) ynext = (labels + (size_t)tile_of(k + 1) * FRT)[sr];
    // softmax(k) inside the stage-2 region of tile k+1 (FFILL > 0; not in the stamped build, whose
    // stamps would split it) or on its own
    constexpr int SMP = decltype(late)::value;  // where the softmax runs: 0 first, 1 after stage 5, 2 last
    constexpr bool fill = FFILL > 0 && !STAMP && SMP == 0;
    float zp[FW];
    if (fill && !last) {
      sm_load(k & 1, zp);
    } else if constexpr (SMP == 0) {
      softmax(k, k & 1, yc);
    }
    if (k == 4) HAR_STAMP(FW, 10)
    if (!INFER && !first) stage5((k - 1) & 1, tile_of(k - 1) * FRT);
    if constexpr (SMP == 1) softmax(k, k & 1, yc);
    if (k == 4) HAR_STAMP(FW, 11)
    if (!last) {
      if (fill)
        stage23(k + 1, (k + 1) & 1, [&] { sm_compute(k, k & 1, yc, zp); });
      else
        stage23(k + 1, (k + 1) & 1, no_fill);
      if (k == 4) HAR_STAMP(FW, 12)
      // stage 1 reads the X tile whose loads were issued just before the last barrier: hoisted to the
      // top of the body (as the scheduler likes, to fill the MFMA pipe beside the softmax) it waits out
      // their whole latency there; here the softmax and stages 2 + 3 cover it.  (Moved ahead of stage
      // 5 so that its X wait no longer also covers stage 5's write-through stores — hipcc's counted
      // wait cannot count a store — measured 0.5 us slower per forward on one box, gpurun_out/abso_es1.)
      __builtin_amdgcn_sched_barrier(0);
      stage1(k & 1);   // tile k+2 (clamped) into the buffer tile k left
      load_x(k + 3);
      if (k == 4) HAR_STAMP(FW, 13)
    }
    if constexpr (SMP == 2) softmax(k, k & 1, yc);
    __syncthreads();
  };
  // (nt == 1 apart, so that every path into the loop issues its loads in the loop body's order: a
  // path with other pending loads makes the counted wait for the label at the loop top conservative)
  auto run = [&](auto late) __attribute__((always_inline)) {
    if (nt == 1) {
      iter(0, true, true, late);
    } else if (nt > 1) {
      iter(0, true, false, late);
      for (int k = 1; k < nt - 1; ++k) iter(k, false, false, late);
      iter(nt - 1, false, true, late);
    }
  };
  // stagger 1: waves 4..7 run their softmax last; 2: right after stage 5 (while waves 0..3, which ran
  // theirs first, are in stage 5: the DPP / transcendental chain of one SIMD partner beside the LDS
  // reads and MFMAs of the other, in both halves)
  if (stagger && __builtin_amdgcn_readfirstlane(wave) >= FW / 2) {
    if (stagger == 2)
      run(std::integral_constant<int, 1>{});
    else
      run(std::integral_constant<int, 2>{});
  } else {
    run(std::integral_constant<int, 0>{});
  }
  HAR_STAMP(FW, 34)
  if constexpr (INFER) return;
  // The W1^T fragment copy the backward of this step reads (Wf + H K0 + H H; the Adam kernel writes
  // only the W0 / W1 copies): fragment f = (unit block ub = f & 15, k chunk jc = f >> 4) holds
  // W1[32 jc .. + 32][16 ub .. + 16], i.e. rows this workgroup's wave jc has in registers (W1 rows
  // 32 jc .. + 32 = its units): transposed through the h1 buffer, free after the last tile.  (Done here,
  // not in the prologue, where wave jc had to wait for its W1 loads before the workgroup's first barrier.)
  for (int f = blockIdx.x; nt > 0 && f < 8 * (HH / 16); f += gridDim.x) {
    const int ub = f & 15, jc = f >> 4;
    if (wave == jc) {
      bf16_t* tt = h1s + wave * 32 * 24;  // this wave's [32 j][16 u] (+ pad)
      const int kcs = ((ub >> 1) - krot) & (KC - 1);
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int kc = 0; kc < KC; ++kc)
          if (kc == kcs && (g >> 1) == (ub & 1))
            *reinterpret_cast<bf16x8_t*>(tt + (16 * t + c16) * 24 + 8 * (g & 1)) = w1f[t][kc];
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the wave's own LDS stores
      __builtin_amdgcn_wave_barrier();
      *reinterpret_cast<bf16x8_t*>(Wf + HH * K0 + HH * HH + (size_t)(ub * KC + jc) * 512 + frag_lane_off(lane)) =
          frag_tr(tt, 24, 0, lane);
      __builtin_amdgcn_wave_barrier();
    }
  }
  if (nt > 0) stage5((nt - 1) & 1, tile_of(nt - 1) * FRT);
  // ---- this workgroup's slab: dWout rows 0..15 x this wave's units, dbout; loss, #correct ----
  float* out = slab + (size_t)blockIdx.x * FWD_SLAB;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    if (wt)
      wt_store16(wt_rsrc(slab), (uint32_t)(((size_t)blockIdx.x * FWD_SLAB + c16 * HH + u0 + 16 * t + 4 * g) * 4),
                 __builtin_bit_cast(u32x4_t, acc5[t]));
    else
      nt_store16(out + (size_t)c16 * HH + u0 + 16 * t + 4 * g, __builtin_bit_cast(u32x4_t, acc5[t]));
  }
  {  // (VALU lane swaps / DPP, not LDS-routed shuffles)
    const LaneSwap sw(lane);
    dbo += sw.x16f(dbo);
    dbo += sw.x32f(dbo);
    lsum = wave_sum_dpp(lsum, sw);
    ncorr = wave_sum_dpp(ncorr, sw);
  }
  float* red = zs;  // free: its last reads (the softmax) precede the barrier above
  if (g == 0) red[wave * NCLS + c16] = dbo;
  if (lane == 0) {
    red[FW * NCLS + wave] = lsum;
    red[FW * NCLS + FW + wave] = ncorr;
  }
  __syncthreads();
  if (tid < NCLS) {
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < FW; ++w) s += red[w * NCLS + tid];
    out[NCLS * HH + tid] = s;
  }
  if (tid == 0) {
    float l = 0.f, c = 0.f;
#pragma unroll
    for (int w = 0; w < FW; ++w) {
      l += red[FW * NCLS + w];
      c += red[FW * NCLS + FW + w];
    }
    block_loss[blockIdx.x] = l;
    block_correct[blockIdx.x] = (int)c;
  }
  if constexpr (STAMP) __builtin_amdgcn_s_waitcnt(0x0f70);
  HAR_STAMP(FW, 35)
  HAR_STAMP_REAL(FW, 39)
}

// ------------------------------------------------------------------------------------------------
// backward
// ------------------------------------------------------------------------------------------------
constexpr int BQ = 4, BQU = HH / BQ;  // 64 h1 units per workgroup
constexpr int BRT = 64;               // rows per pipeline tile
constexpr int BDP = HH + 16;          // dact2 tile pitch: 136 dwords (8 mod 64)
constexpr int BUP = BQU + 16;         // h1 / dact1 quadrant tile pitch: 40 dwords; 8-byte chunks
                                      // swizzled by row (frag_rows_q)

template <int K0> struct Bwd4Lds {
  static constexpr int XP = K0 + 16;
  static constexpr int NXB = 4;  // X tile buffers (staged two tiles ahead; read by h1 / (c) two tiles apart)
  static_assert((NXB & (NXB - 1)) == 0, "buffer indices are taken with & (NXB - 1)");
  static constexpr int DSM = BRT * BDP, HS = BRT * BUP, XS = BRT * XP;
  static constexpr size_t bytes = (size_t)(2 * DSM + 2 * HS + 2 * HS + NXB * XS) * sizeof(bf16_t);
  static_assert((size_t)NCLS * HH + HH * BQU <= (size_t)2 * DSM, "the prologue images fit the dact2 buffers");
};

// ------------------------------------------------------------------------------------------------
// backward, wave-specialized (mlp_bwd4): the 8 waves split by role.  Waves 0..3 PRODUCE the next
// tile's operands (the dact2 tile copied from the forward's dact2 rows, the X tile staging and the h1
// recompute: loads, LDS stores and a few small MFMAs) and take the (c) dW0 / db0 products of the
// previous tile; waves 4..7 CONSUME the current tile (the (a) dact1, (b) dW1, db1 products: MFMA with
// LDS fragment reads).  Each SIMD hosts one
// producer and one consumer, so the producer's load / LDS-store stream issues beside the consumer's
// MFMA stream.  Each role runs its own loop (disjoint register live ranges: max, not sum, of the two
// roles' state) with the same barrier sequence: one workgroup barrier per tile.
//   consumer c: (a) unit blocks 2 (c & 1) .. + 1 x row blocks 2 (c >> 1) .. + 1 (W1^T fragments in
//               registers, dact2 rows from LDS); (b) all 4 unit blocks x j blocks 4c .. 4c + 3
//               (64 dW1 accumulators); db1 of j block 4q + c
//   producer p: dact2 / X staging (8 / 1-2 16-byte pieces per thread, loaded two tiles ahead); h1
//               unit block p x all 4 row blocks; (c) unit block p x every input block, db0 of unit block p
// The forward computes dact2 = (dz . Wout) * relu'(h2) beside its dWout stage (16x16x16 MFMAs on data
// it holds anyway) and writes it in this kernel's LDS tile order: the 4 quadrant workgroups of a row
// slice then copy the same rows (one HBM read, three L2 / MALL hits) instead of each rebuilding them
// from dz and a relu' bit mask (16 MFMAs + table-driven masking per producer wave and tile: the
// producers had become the critical path, profiles/r5).
template <int K0, bool STAMP>
__global__ __launch_bounds__(512) void mlp_bwd4_kernel(
    const bf16_t* __restrict__ dact2, const bf16_t* __restrict__ X,
    const bf16_t* __restrict__ Wf, const float* __restrict__ b0,
    int B, int S, float* __restrict__ gw1, float* __restrict__ gw0,
    float* __restrict__ gb0, float* __restrict__ gb1, int64_t slab_stride, int32_t* __restrict__ tick,
    const float* __restrict__ fslab, int fslab_w, int nfwd, float* __restrict__ gwo, float* __restrict__ gbo,
    uint64_t* __restrict__ stamps, int nt_slab) {
  using L = Bwd4Lds<K0>;
  constexpr int NXB = L::NXB, KC = HH / 32, XP = L::XP, NFW = K0 / 32, NFB = K0 / 16;
  constexpr int XV = BRT * K0 / 8;  // 16-byte vectors of an X tile (512 / 256)
  constexpr int XPT = XV / 256;     // per producer thread (2 / 1)
  constexpr int DV = BRT * HH / 8 / 256;  // 16-byte dact2 pieces per producer thread and tile (8)
  if (tick && blockIdx.x == 0 && threadIdx.x == 0) *tick += 1;
  extern __shared__ __attribute__((aligned(16))) bf16_t lds[];
  bf16_t* const dsm0 = lds;                // [2][64][BDP] dact2 tiles
  bf16_t* const hs0 = dsm0 + 2 * L::DSM;   // [2][64][BUP] h1 quadrant tiles
  bf16_t* const d1s0 = hs0 + 2 * L::HS;    // [2][64][BUP] dact1 quadrant tiles
  bf16_t* const xs0 = d1s0 + 2 * L::HS;    // [NXB][64][XP] X tiles
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // scalar: the role branches are s_cbranch
  const int c16 = lane & 15, g = lane >> 4;
  HAR_STAMP_REAL(8, 38)
  HAR_STAMP(8, 0)
  const int b = xcd_remap(blockIdx.x, gridDim.x);
  const int slice = b / BQ, q = b % BQ, qu0 = q * BQU;
  const bool prod = wave < 4;
  const int pw = wave & 3;
  const int ntiles = B / BRT, per = (ntiles + S - 1) / S;
  const int t0 = slice * per, n = max(0, min(ntiles, t0 + per) - t0);

  // ---- prologue (all waves): W1^T quadrant fragments into LDS, the forward's dWout slabs ----
  const bf16_t* const W0f = Wf;
  const bf16_t* const W1tq = Wf + HH * K0 + HH * HH + (size_t)(4 * q) * KC * 512;
  bf16_t* const w1q = lds + NCLS * HH;
  {
    uint4 st[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) st[i] = *reinterpret_cast<const uint4*>(W1tq + (size_t)(i * 8 + wave) * 512 + lane * 8);
#pragma unroll
    for (int i = 0; i < 4; ++i) *reinterpret_cast<uint4*>(w1q + (i * 8 + wave) * 512 + lane * 8) = st[i];
  }
  __syncthreads();
  // a row of ones (A operand: row 0) / a column of ones (B operand: column 0): the same registers
  const bf16x8_t ones = __builtin_bit_cast(bf16x8_t, c16 == 0 ? s16x8_t{0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80,
                                                                        0x3f80, 0x3f80, 0x3f80}
                                                              : s16x8_t{0, 0, 0, 0, 0, 0, 0, 0});
  const int tlast = ntiles - 1;

  if (prod) {
    // ================================ producer ================================
    const int ptid = tid;  // 0..255
    static_assert(XPT == 1 || XPT == 2, "one or two X vectors per producer thread");
    static_assert(DV == 8, "8 dact2 pieces per producer thread");
    // dact2 piece i of a tile: row (ptid >> 5) + 8 i, 16-byte chunk ptid & 31 (a wave-instruction reads
    // two whole 512-byte rows); LDS rows BDP apart (the forward wrote the chunk swizzle already)
    // (lane offsets 32-bit, tile bases wave-uniform: the loads take the SGPR-base form)
    const uint32_t d2src = (uint32_t)((ptid >> 5) * HH + (ptid & 31) * 8);  // (unsigned: zero-extended offsets)
    const int d2dst = (ptid >> 5) * BDP + (ptid & 31) * 8;
    // (macros, not lambdas: a lambda-captured register array is kept in scratch)
    // two register sets of dact2 pieces: the tile staged at iteration i was loaded at iteration i - 2
    // (one iteration ahead left ~700 cycles of the refill still in flight at its use, profiles/r5)
    uint4 da0, da1, da2, da3, da4, da5, da6, da7, db0_, db1_, db2_, db3_, db4_, db5_, db6_, db7_;
    uint4 xr0, xr1, xq0, xq1;  // xq: X tile t0 + 1, loaded with tile t0
#define HAR_B4_LOAD_D(t, ...) HAR_B4_LOAD_D_I(t, __VA_ARGS__)
#define HAR_B4_LOAD_D_I(t, r0_, r1_, r2_, r3_, r4_, r5_, r6_, r7_)            \
  {                                                                           \
    const int tt_ = min(t, tlast);                                            \
    const bf16_t* dp_ = dact2 + (size_t)tt_ * (BRT * HH);                     \
    r0_ = *reinterpret_cast<const uint4*>(dp_ + (d2src + 0 * 8 * HH));        \
    r1_ = *reinterpret_cast<const uint4*>(dp_ + (d2src + 1 * 8 * HH));        \
    r2_ = *reinterpret_cast<const uint4*>(dp_ + (d2src + 2 * 8 * HH));        \
    r3_ = *reinterpret_cast<const uint4*>(dp_ + (d2src + 3 * 8 * HH));        \
    r4_ = *reinterpret_cast<const uint4*>(dp_ + (d2src + 4 * 8 * HH));        \
    r5_ = *reinterpret_cast<const uint4*>(dp_ + (d2src + 5 * 8 * HH));        \
    r6_ = *reinterpret_cast<const uint4*>(dp_ + (d2src + 6 * 8 * HH));        \
    r7_ = *reinterpret_cast<const uint4*>(dp_ + (d2src + 7 * 8 * HH));        \
  }
#define HAR_B4_STAGE_D(buf, ...) HAR_B4_STAGE_D_I(buf, __VA_ARGS__)
#define HAR_B4_STAGE_D_I(buf, r0_, r1_, r2_, r3_, r4_, r5_, r6_, r7_)         \
  {                                                                           \
    bf16_t* d_ = dsm0 + (buf) * L::DSM + d2dst;                               \
    *reinterpret_cast<uint4*>(d_ + 0 * 8 * BDP) = r0_;                        \
    *reinterpret_cast<uint4*>(d_ + 1 * 8 * BDP) = r1_;                        \
    *reinterpret_cast<uint4*>(d_ + 2 * 8 * BDP) = r2_;                        \
    *reinterpret_cast<uint4*>(d_ + 3 * 8 * BDP) = r3_;                        \
    *reinterpret_cast<uint4*>(d_ + 4 * 8 * BDP) = r4_;                        \
    *reinterpret_cast<uint4*>(d_ + 5 * 8 * BDP) = r5_;                        \
    *reinterpret_cast<uint4*>(d_ + 6 * 8 * BDP) = r6_;                        \
    *reinterpret_cast<uint4*>(d_ + 7 * 8 * BDP) = r7_;                        \
  }
#define HAR_DA da0, da1, da2, da3, da4, da5, da6, da7
#define HAR_DB db0_, db1_, db2_, db3_, db4_, db5_, db6_, db7_
#define HAR_B4_LOAD_XR(t, xa_, xb2_)                                                          \
  {                                                                                           \
    const int tt_ = min(t, tlast);                                                            \
    const bf16_t* xp_ = X + (size_t)tt_ * (XV * 8);                                           \
    xa_ = *reinterpret_cast<const uint4*>(xp_ + (uint32_t)(ptid * 8));                        \
    if constexpr (XPT == 2) xb2_ = *reinterpret_cast<const uint4*>(xp_ + (uint32_t)((ptid + 256) * 8)); \
  }
#define HAR_B4_STAGE_XR(i, xa_, xb2_)                                                                      \
  {                                                                                                        \
    bf16_t* xb_ = xs0 + ((i) & (NXB - 1)) * L::XS;                                                         \
    *reinterpret_cast<uint4*>(xb_ + (ptid / (K0 / 8)) * XP + (ptid % (K0 / 8)) * 8) = xa_;                 \
    if constexpr (XPT == 2)                                                                                \
      *reinterpret_cast<uint4*>(xb_ + ((ptid + 256) / (K0 / 8)) * XP + ((ptid + 256) % (K0 / 8)) * 8) = xb2_; \
  }
#define HAR_B4_LOAD_X(t) HAR_B4_LOAD_XR(t, xr0, xr1)
#define HAR_B4_STAGE_X(i) HAR_B4_STAGE_XR(i, xr0, xr1)
    // the first tiles' loads go out before anything else of the prologue (W0 fragments, the dWout
    // slabs): dact2 tile 0 and X tiles 0 / 1 land in one round trip, staged after the barrier below
    HAR_B4_LOAD_D(t0, HAR_DA)
    HAR_B4_LOAD_X(t0)
    HAR_B4_LOAD_XR(t0 + 1, xq0, xq1)
    bf16x8_t w0q[NFW];
#pragma unroll
    for (int kc = 0; kc < NFW; ++kc)
      w0q[kc] = *reinterpret_cast<const bf16x8_t*>(W0f + (size_t)((4 * q + pw) * NFW + kc) * 512 + frag_lane_off(lane));
    const float4 b0q = *reinterpret_cast<const float4*>(b0 + qu0 + 16 * pw + 4 * g);
    constexpr int WO4 = NCLS * HH / 4, NC4 = WO4 + NCLS / 4;
    f32x4_t px[4];
    auto wo_load = [&](int c4) __attribute__((always_inline)) {
      const float* src = fslab + (c4 < WO4 ? 4 * c4 : NCLS * HH + 4 * (c4 - WO4));
#pragma unroll
      for (int r = 0; r < 4; ++r)
        px[r] = lane + 64 * r < nfwd ? *reinterpret_cast<const f32x4_t*>(src + (size_t)(lane + 64 * r) * fslab_w)
                                     : f32x4_t{0.f, 0.f, 0.f, 0.f};
    };
    if (fslab && 4 * b + pw < NC4) wo_load(4 * b + pw);
    if constexpr (STAMP) __builtin_amdgcn_s_waitcnt(0x0f70);
    HAR_STAMP(8, 1)

    // h1 unit block pw x 4 row blocks of tile i (X buffer i & 3) -> h1 buffer i & 1 (the forward's
    // operands, accumulation order and rounding: bit-identical h1)
    auto tile_h1 = [&](int i) __attribute__((always_inline)) {
      const bf16_t* xs = xs0 + (i & (NXB - 1)) * L::XS;
      bf16_t* hs = hs0 + (i & 1) * L::HS;
      // every X fragment read first (one LDS round trip per tile, not one per row block)
      bf16x8_t xf[4][NFW];
#pragma unroll
      for (int rr = 0; rr < 4; ++rr)
#pragma unroll
        for (int kc = 0; kc < NFW; ++kc)
          xf[rr][kc] = *reinterpret_cast<const bf16x8_t*>(xs + (16 * rr + c16) * XP + kc * 32 + 8 * g);
      __builtin_amdgcn_sched_barrier(0);
      f32x4_t a[4];
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        a[rr] = f32x4_t{b0q.x, b0q.y, b0q.z, b0q.w};
#pragma unroll
        for (int kc = 0; kc < NFW; ++kc) a[rr] = mma32(w0q[kc], xf[rr][kc], a[rr]);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int rr = 0; rr < 4; ++rr)
        *reinterpret_cast<uint2*>(hs + (16 * rr + c16) * BUP + 16 * pw + 4 * (g ^ (c16 >> 2))) =
            make_uint2(relu2(pack2(a[rr][0], a[rr][1])), relu2(pack2(a[rr][2], a[rr][3])));
    };
    // (c) dW0[u][f] += dact1^T . X of tile i (unit block pw, every input block) and db0: on the producer
    // side since the consumers' (a) + (b) MFMA stream had become the longer half of a tile (profiles/r5)
    f32x4_t acc0[NFB], accd0 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int f = 0; f < NFB; ++f) acc0[f] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    auto tile_c = [&](int i) __attribute__((always_inline)) {
      const bf16_t* d1s = d1s0 + (i & 1) * L::HS;
      const bf16_t* xs = xs0 + (i & (NXB - 1)) * L::XS;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const bf16x8_t A = frag_rows_q(d1s + 32 * ks * BUP, BUP, 16 * pw, lane);
#pragma unroll
        for (int f = 0; f < NFB; ++f) acc0[f] = mma32(A, frag_rows(xs + 32 * ks * XP, XP, 16 * f, lane), acc0[f]);
        accd0 = mma32(A, ones, accd0);
      }
    };
    // invariant at the top of iteration i: the dact2 set of i's parity (A even, B odd) holds tile i+1,
    // the other set tile i+2; xr = X tile i+2 (loaded)
    __syncthreads();  // the prologue images are read: the tile buffers may be written
    HAR_B4_STAGE_D(0, HAR_DA)
    HAR_B4_STAGE_X(0)
    HAR_B4_STAGE_XR(1, xq0, xq1)
    HAR_B4_LOAD_D(t0 + 1, HAR_DA)
    HAR_B4_LOAD_D(t0 + 2, HAR_DB)
    HAR_B4_LOAD_X(t0 + 2)
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();  // dact2 tile 0, X tiles 0 and 1 are in LDS
    tile_h1(0);
    __syncthreads();  // h1 tile 0 complete
#define HAR_B4_ITER(i, ...)                                                                             \
  {                                                                                                     \
    if ((i) < 24) HAR_STAMP(8, 2 + (i))                                                                 \
    if constexpr (STAMP) { /* (stamped build only: how long the dact2 refill is still in flight) */    \
      if ((i) == 4) {                                                                                   \
        __builtin_amdgcn_s_waitcnt(0x0f70 | (8 + XPT));                                                 \
        HAR_STAMP(8, 32)                                                                                \
      }                                                                                                 \
    }                                                                                                   \
    HAR_B4_STAGE_D(((i) + 1) & 1, __VA_ARGS__) /* waits for the dact2 loads issued two iterations ago */ \
    if ((i) == 4) HAR_STAMP(8, 26)                                                                      \
    HAR_B4_STAGE_X((i) + 2)                                                                             \
    /* the refills may not be hoisted above the last reads of the registers they overwrite: a hoisted  \
       load gets fresh registers, and the loop-carried copy back then waits out its whole latency */   \
    __builtin_amdgcn_sched_barrier(0);                                                                  \
    HAR_B4_LOAD_D(t0 + (i) + 3, __VA_ARGS__)                                                            \
    HAR_B4_LOAD_X(t0 + (i) + 3)                                                                         \
    __builtin_amdgcn_sched_barrier(0); /* the refills are issued before the h1 recompute */           \
    if ((i) == 4) HAR_STAMP(8, 27)                                                                      \
    tile_h1((i) + 1); /* X tile i+1 has been in LDS since the last barrier */                         \
    if ((i) == 4) HAR_STAMP(8, 28)                                                                      \
    if ((i) > 0) tile_c((i) - 1); /* dact1 i-1 completed at the last barrier; X i-1 is still staged */  \
    if ((i) == 4) HAR_STAMP(8, 33)                                                                      \
    __syncthreads(); /* dact2 i+1 / X i+2 staged, h1 i+1 complete; the consumers finished tile i */    \
  }
    int i = 0;
    for (; i + 1 < n; i += 2) {
      HAR_B4_ITER(i, HAR_DA)
      HAR_B4_ITER(i + 1, HAR_DB)
    }
    if (i < n) HAR_B4_ITER(i, HAR_DA)
#undef HAR_B4_ITER
#undef HAR_B4_STAGE_D
#undef HAR_B4_STAGE_D_I
#undef HAR_DA
#undef HAR_DB
#undef HAR_B4_LOAD_D
#undef HAR_B4_LOAD_D_I
#undef HAR_B4_LOAD_X
#undef HAR_B4_STAGE_X
#undef HAR_B4_LOAD_XR
#undef HAR_B4_STAGE_XR
    HAR_STAMP(8, 34)
    if (n > 0) tile_c(n - 1);
    float* w0o = gw0 + (size_t)slice * slab_stride;
    if (nt_slab == 2) {  // write-through (see the consumers' slab stores)
      const __amdgpu_buffer_rsrc_t rs = wt_rsrc(gw0);
#pragma unroll
      for (int f = 0; f < NFB; ++f)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          wt_store4(rs, (uint32_t)(((size_t)slice * slab_stride + (size_t)(qu0 + 16 * pw + 4 * g + r) * K0 + 16 * f + c16) * 4),
                    acc0[f][r]);
    } else {
#pragma unroll
      for (int f = 0; f < NFB; ++f)
#pragma unroll
        for (int r = 0; r < 4; ++r) w0o[(size_t)(qu0 + 16 * pw + 4 * g + r) * K0 + 16 * f + c16] = acc0[f][r];
    }
    if (c16 == 0) *reinterpret_cast<f32x4_t*>(gb0 + (size_t)slice * slab_stride + qu0 + 16 * pw + 4 * g) = accd0;
    // the forward's dWout / dbout slabs (one per forward workgroup) -> gwo / gbo: 4-column group
    // 4 b + pw per producer wave (b the XCD-remapped index: the 8 groups of a 128-byte line in two
    // workgroups of one XCD), its loads issued in the prologue and summed here, after the last tile.
    // (In the prologue proper the task waves started their tiles ~4k cycles late; loaded here, with
    // neighbouring groups on other XCDs, the gather took ~17k cycles, profiles/r5)
    if (fslab) {
      const LaneSwap lsw(lane);
      for (int c4 = 4 * b + pw; c4 < NC4; c4 += 4 * (int)gridDim.x) {
        if (c4 != 4 * b + pw) wo_load(c4);
        f32x4_t v = (px[0] + px[1]) + (px[2] + px[3]);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = wave_sum_dpp(v[e], lsw);
        if (lane == 0) *reinterpret_cast<f32x4_t*>(c4 < WO4 ? gwo + 4 * c4 : gbo + 4 * (c4 - WO4)) = v;
      }
    }
  } else {
    // ================================ consumer ================================
    const int ua0 = 2 * (pw & 1), ra0 = 2 * (pw >> 1);
    bf16x8_t w1t[2][KC];  // (a) A fragments: A[u][k = j] = W1[32 kc + 8g + i][qu0 + 16 (ua0 + e) + c16]
#pragma unroll
    for (int e = 0; e < 2; ++e)
#pragma unroll
      for (int kc = 0; kc < KC; ++kc)
        w1t[e][kc] = *reinterpret_cast<const bf16x8_t*>(w1q + ((ua0 + e) * KC + kc) * 512 + frag_lane_off(lane));
    if constexpr (STAMP) __builtin_amdgcn_s_waitcnt(0x0f70);
    HAR_STAMP(8, 1)
    // (paired with the producers' "prologue images are read" barrier: the W1^T image is read above,
    // the producers then overwrite it with dact2 tile 0)
    __syncthreads();
    f32x4_t acc1[4][4], accb = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int u = 0; u < 4; ++u) acc1[j][u] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    // (a) dact1^T = W1^T[u] . dact2^T over row blocks ra0, ra0 + 1; relu'(h1); dact1 -> LDS
    // (the same 32 x 32 block as 16 v_mfma_f32_32x32x16 per tile — A fragments gathered from w1q, one 1 KB
    // dact2 read per k step — measured slower on one box: backward 30.3 vs 28.0 us, step 0.0551 vs
    // 0.0525 ms with one accumulator chain, 31.5 vs 28.5 us with two; profiles/r6/mlp_a32_ab.txt)
    // Software-pipelined: the dact2 fragments of k chunk kc + 3 are read while the MFMAs of chunk kc
    // run (pinned by scheduling groups: 2 LDS reads, then 4 MFMAs, per chunk), and the relu'(h1)
    // words are read first; written plainly, each chunk's reads were issued right before their MFMAs
    // and every chunk waited out an LDS round trip
    // (par = the tile's buffer parity, a compile-time constant in the 2-unrolled loop below: every LDS
    // address is a lane base + an immediate offset, no per-tile address arithmetic)
    auto tile_a = [&](int par) __attribute__((always_inline)) {
      const bf16_t* dsm = dsm0 + par * L::DSM;
      const bf16_t* hs = hs0 + par * L::HS;
      bf16_t* d1s = d1s0 + par * L::HS;
      constexpr int PD = 3;  // prefetch distance (k chunks)
      const int swz = 8 * ((c16 >> 2) & 1);
      // (an isolated scheduling region whose first group is the hm reads + the PD chunks ahead: without
      // it the scheduler put each chunk's own reads into the per-chunk read groups, right before their
      // MFMAs — no prefetch at all, profiles/r5)
      __builtin_amdgcn_sched_barrier(0);
      uint2 hm[2][2];
#pragma unroll
      for (int rr = 0; rr < 2; ++rr)
#pragma unroll
        for (int e = 0; e < 2; ++e)
          hm[rr][e] = *reinterpret_cast<const uint2*>(hs + (16 * (ra0 + rr) + c16) * BUP + 16 * (ua0 + e) + 4 * (g ^ (c16 >> 2)));
      bf16x8_t bv[2][KC];
#pragma unroll
      for (int kc = 0; kc < PD; ++kc)
#pragma unroll
        for (int rr = 0; rr < 2; ++rr)
          bv[rr][kc] = *reinterpret_cast<const bf16x8_t*>(dsm + (16 * (ra0 + rr) + c16) * BDP + ((kc * 32 + 8 * g) ^ swz));
      __builtin_amdgcn_sched_group_barrier(0x100, 2 * PD + 4, 0);
      f32x4_t acc[2][2];
#pragma unroll
      for (int rr = 0; rr < 2; ++rr)
#pragma unroll
        for (int e = 0; e < 2; ++e) acc[rr][e] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) {
        if (kc + PD < KC) {
#pragma unroll
          for (int rr = 0; rr < 2; ++rr)
            bv[rr][kc + PD] =
                *reinterpret_cast<const bf16x8_t*>(dsm + (16 * (ra0 + rr) + c16) * BDP + (((kc + PD) * 32 + 8 * g) ^ swz));
          __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);  // the 2 LDS reads of chunk kc + PD
        }
#pragma unroll
        for (int rr = 0; rr < 2; ++rr)
#pragma unroll
          for (int e = 0; e < 2; ++e) acc[rr][e] = mma32(w1t[e][kc], bv[rr][kc], acc[rr][e]);
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);  // then the 4 MFMAs of chunk kc
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int rr = 0; rr < 2; ++rr)
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const f32x4_t& a = acc[rr][e];
          const uint2 m = hm[rr][e];  // relu'd h1 (bf16 pairs): dact1 = dact1_pre * relu'(h1)
          *reinterpret_cast<uint2*>(d1s + (16 * (ra0 + rr) + c16) * BUP + 16 * (ua0 + e) + 4 * (g ^ (c16 >> 2))) =
              make_uint2(relu_d_mul(pack2(a[0], a[1]), m.x), relu_d_mul(pack2(a[2], a[3]), m.y));
        }
    };
    // (b) dW1[j][u] += dact2^T . h1 for j blocks 4 pw .. + 3 x all unit blocks; db1 of j block 4q + pw
    auto tile_b = [&](int par) __attribute__((always_inline)) {
      const bf16_t* dsm = dsm0 + par * L::DSM;
      const bf16_t* hs = hs0 + par * L::HS;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8_t hb[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) hb[u] = frag_rows_q(hs + 32 * ks * BUP, BUP, 16 * u, lane);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const bf16x8_t da = frag_rows_sw(dsm + 32 * ks * BDP, BDP, 16 * (4 * pw + j), lane);
#pragma unroll
          for (int u = 0; u < 4; ++u) acc1[j][u] = mma32(hb[u], da, acc1[j][u]);  // C[u][j]
        }
        accb = mma32(ones, frag_rows_sw(dsm + 32 * ks * BDP, BDP, 16 * (4 * q + pw), lane), accb);
      }
    };
    __builtin_amdgcn_s_setprio(1);  // the consumers' MFMA stream is the critical path of a tile
    __syncthreads();  // (paired with the producers' barrier: dact2 0, X 0 / 1 staged)
    __syncthreads();  // (paired: h1 tile 0 complete)
    auto citer = [&](int i, auto parc) __attribute__((always_inline)) {
      constexpr int par = decltype(parc)::value;
      if (i < 24) HAR_STAMP(8, 2 + i)
      tile_a(par);
      if (i == 4) HAR_STAMP(8, 29)
      tile_b(par);
      if (i == 4) HAR_STAMP(8, 30)
      __syncthreads();  // dact1 i complete; the buffers of tile i may be overwritten
    };
    int i = 0;
    for (; i + 1 < n; i += 2) {
      citer(i, std::integral_constant<int, 0>{});
      citer(i + 1, std::integral_constant<int, 1>{});
    }
    if (i < n) citer(i, std::integral_constant<int, 0>{});
    HAR_STAMP(8, 34)
    __builtin_amdgcn_s_setprio(0);
    // ---- this wave's parts of slab `slice` (flat parameter layout) ----
    // (staging both roles' partials through an LDS image and storing whole rows measured 0.5 us slower
    // per step on one box: 0.0540 / 0.0536 / 0.0535 vs 0.0530 / 0.0532 / 0.0530 ms, gpurun_out/ab_epi)
    float* w1o = gw1 + (size_t)slice * slab_stride;
    // nt_slab: 1 nontemporal, 2 write-through (sc1: the slabs are not left dirty in L2 for the reduction
    // launch's boundary), 0 plain
    const __amdgpu_buffer_rsrc_t w1rs = wt_rsrc(gw1);
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (nt_slab == 2)
          wt_store16(w1rs, (uint32_t)(((size_t)slice * slab_stride + (size_t)(16 * (4 * pw + j) + c16) * HH + qu0 + 16 * u + 4 * g) * 4),
                     __builtin_bit_cast(u32x4_t, acc1[j][u]));
        else if (nt_slab)
          nt_store16(w1o + (size_t)(16 * (4 * pw + j) + c16) * HH + qu0 + 16 * u + 4 * g, __builtin_bit_cast(u32x4_t, acc1[j][u]));
        else
          *reinterpret_cast<f32x4_t*>(w1o + (size_t)(16 * (4 * pw + j) + c16) * HH + qu0 + 16 * u + 4 * g) = acc1[j][u];
    if (g == 0) gb1[(size_t)slice * slab_stride + 16 * (4 * q + pw) + c16] = accb[0];
  }
  if constexpr (STAMP) __builtin_amdgcn_s_waitcnt(0x0f70);
  HAR_STAMP(8, 35)
  HAR_STAMP_REAL(8, 39)
}

// HAR_MLP_FWD_STAGGER=1: waves 4..7 run their softmax after the MFMA stages (off by default)
static int fwd_stagger() {
  static const int v = [] {
    const char* e = getenv("HAR_MLP_FWD_STAGGER");
    return e ? atoi(e) : 0;  // measured slower (fwd 21.9 vs 21.1 us, profiles/r5/mlp_fwd_variants.md)
  }();
  return v;
}

template <int K0>
void launch_fwd3(const bf16_t* X, bf16_t* Wf, const float* b0, const float* b1, const bf16_t* Wo,
                 const float* bo, const int32_t* labels, int B, int C, float scale, bf16_t* dact2,
                 float* slab, float* bl, int32_t* bc, int nwg, hipStream_t s) {
  static const int fill = [] {
    const char* e = getenv("HAR_MLP_FWD_FILL");
    return e ? atoi(e) : 0;
  }();
  auto k = g_har_mlp_stamps ? mlp_fwd3_kernel<K0, true>
           : fill == 1      ? mlp_fwd3_kernel<K0, false, false, 1>
           : fill == 2      ? mlp_fwd3_kernel<K0, false, false, 2>
           : fill >= 3      ? mlp_fwd3_kernel<K0, false, false, 3>
                            : mlp_fwd3_kernel<K0, false>;
  // dact2 / dWout slab stores write-through (sc1; HAR_MLP_WT=0: plain / nontemporal): the 33.5 MB of
  // dact2 are then not dirty in the L2s when the backward launches — forward 22.0 -> 19.3 us, step
  // 0.0571 -> 0.0540 ms (profiles/r6/mlp_write_through_ab.md)
  static const int wt = [] {
    const char* e = getenv("HAR_MLP_WT");
    return e ? atoi(e) : 1;
  }();
  const int wtl = (wt & 1) && (size_t)B * HH * 2 < 0x7fffffffu ? 1 : 0;  // (32-bit buffer offsets)
  k<<<nwg, 512, FWD_LDS, s>>>(X, Wf, b0, b1, Wo, bo, labels, B, C, scale, dact2, slab, bl, bc, g_har_mlp_stamps,
                              fwd_stagger(), wtl);
}

template <int K0>
void launch_fwd3_infer(const bf16_t* X, bf16_t* Wf, const float* b0, const float* b1, const bf16_t* Wo,
                       const float* bo, int B, int C, float* logits, int32_t* pred, int nwg, hipStream_t s) {
  mlp_fwd3_kernel<K0, false, true><<<nwg, 512, FWD_LDS, s>>>(X, Wf, b0, b1, Wo, bo, nullptr, B, C, 1.f, nullptr,
                                                              logits, nullptr, pred, nullptr, fwd_stagger(), 0);
}

template <int K0>
void launch_bwd4(const bf16_t* dact2, const bf16_t* X, const bf16_t* Wf, const float* b0, int B, int S, float* gw1,
                 float* gw0, float* gb0, float* gb1, int64_t stride, int32_t* tick, const float* fslab, int fslab_w,
                 int nfwd, float* gwo, float* gbo, hipStream_t s) {
  // HAR_MLP_BWD_NT=1: the dW1 partial slabs written with nontemporal stores
  static const int nt = [] {
    // the dW1 / dW0 partial slabs: 2 write-through (default: not dirty in L2 at the reduction's launch),
    // 1 nontemporal, 0 plain
    const char* e = getenv("HAR_MLP_BWD_NT");
    return e ? atoi(e) : 2;
  }();
  auto k = g_har_mlp_stamps ? mlp_bwd4_kernel<K0, true> : mlp_bwd4_kernel<K0, false>;
  const int ntl = nt == 2 && (size_t)S * stride * 4 >= 0x7fffffffu ? 0 : nt;  // (32-bit buffer offsets)
  k<<<S * BQ, 512, Bwd4Lds<K0>::bytes, s>>>(dact2, X, Wf, b0, B, S, gw1, gw0, gb0, gb1, stride, tick, fslab, fslab_w,
                                           nfwd, gwo, gbo, g_har_mlp_stamps ? g_har_mlp_stamps + STAMP_BWD_OFF : nullptr,
                                           ntl);
}

}  // namespace

extern "C" int har_mlp_step_grid(int B) { return std::max(1, std::min(256, B / FRT)); }
// Row slices of the backward (x 4 unit quadrants = workgroups; one fp32 gradient slab per slice):
// 4 tiles per slice at large batches (the slab traffic stays 64 slabs), but at least min(16, tiles)
// slices at small ones, so a batch of 256 runs 16 workgroups instead of 4 (every workgroup's
// prologue and slab stores are a fixed cost; their parallelism is what a small step needs).
extern "C" int har_mlp_step_slices(int B) {
  const int tiles = B / BRT;
  return std::max(1, std::min(64, std::max(tiles / 4, std::min(tiles, 16))));
}
extern "C" int har_mlp_step_fwd_slab_width(int H) { return NCLS * H + NCLS; }

// Forward of the step: dact2 [B][256] bf16 (the layer-2 gradient (dz . Wout) * relu'(h2), the 16-byte
// chunks of rows with bit 2 set swapped in pairs: the backward's LDS tile image) and per workgroup
// (har_mlp_step_grid(B) of them) dWout rows 0..15 + dbout (width har_mlp_step_fwd_slab_width), loss
// and #correct.
extern "C" int har_mlp_step_fwd(const uint16_t* X, int K0, uint16_t* Wf, const float* b0, const float* b1,
                                int H, const uint16_t* Wo, const float* bo, const int32_t* labels, int B, int C,
                                float scale, uint16_t* dact2, float* slab, float* block_loss,
                                int32_t* block_correct, hipStream_t s) {
  if (H != HH || (K0 != 32 && K0 != 64) || B <= 0 || B % 64 || C < 1 || C > NCLS) return -2;
  if (((uintptr_t)X | (uintptr_t)Wf | (uintptr_t)Wo | (uintptr_t)b0 | (uintptr_t)b1 | (uintptr_t)slab |
       (uintptr_t)dact2) & 15)
    return -3;
  const int nwg = har_mlp_step_grid(B);
  bf16_t* d2 = reinterpret_cast<bf16_t*>(dact2);
  if (K0 == 64)
    launch_fwd3<64>(X, Wf, b0, b1, Wo, bo, labels, B, C, scale, d2, slab, block_loss, block_correct, nwg, s);
  else
    launch_fwd3<32>(X, Wf, b0, b1, Wo, bo, labels, B, C, scale, d2, slab, block_loss, block_correct, nwg, s);
  HAR_CHECK_LAUNCH();
  return 0;
}

// Serving forward on the step's pipeline (the INFER instantiation of mlp_fwd3): X bf16 [B][K0] padded,
// the W0 / W1 fragment copies in Wf (as the training step keeps them); logits [B][C] fp32 and the argmax
// [B] int32 out.
extern "C" int har_mlp_step_fwd_infer(const uint16_t* X, int K0, const uint16_t* Wf, const float* b0, const float* b1,
                                      int H, const uint16_t* Wo, const float* bo, int B, int C, float* logits,
                                      int32_t* pred, hipStream_t s) {
  if (H != HH || (K0 != 32 && K0 != 64) || B <= 0 || B % 64 || C < 1 || C > NCLS || !logits || !pred) return -2;
  if (((uintptr_t)X | (uintptr_t)Wf | (uintptr_t)Wo | (uintptr_t)b0 | (uintptr_t)b1) & 15) return -3;
  const int nwg = har_mlp_step_grid(B);
  bf16_t* wf = const_cast<bf16_t*>(reinterpret_cast<const bf16_t*>(Wf));  // read only in INFER
  if (K0 == 64)
    launch_fwd3_infer<64>(reinterpret_cast<const bf16_t*>(X), wf, b0, b1, reinterpret_cast<const bf16_t*>(Wo), bo, B, C,
                          logits, pred, nwg, s);
  else
    launch_fwd3_infer<32>(reinterpret_cast<const bf16_t*>(X), wf, b0, b1, reinterpret_cast<const bf16_t*>(Wo), bo, B, C,
                          logits, pred, nwg, s);
  HAR_CHECK_LAUNCH();
  return 0;
}

// Backward of the step (from the forward's dact2 rows and X): per row slice s < har_mlp_step_slices(B)
// the partials of dW1, dW0, db0 (and db1) at gw1 / gw0 / gb0 / gb1 + s * slab_stride.  With fslab (the
// forward's har_mlp_step_grid(B) per-workgroup slabs, row stride fslab_w) it also writes their sums:
// dWout rows 0..15 to gwo and dbout to gbo (fixed summation order).
extern "C" int har_mlp_step_bwd(const uint16_t* dact2, const uint16_t* X, int K0, const uint16_t* Wf, int H,
                                const float* b0, int B, float* gw1, float* gw0, float* gb0, float* gb1,
                                int64_t slab_stride, int32_t* tick, const float* fslab, int fslab_w, float* gwo,
                                float* gbo, hipStream_t s) {
  if (H != HH || B <= 0 || B % BRT || (K0 != 32 && K0 != 64) || slab_stride < (int64_t)H * H) return -2;
  if (((uintptr_t)dact2 | (uintptr_t)X | (uintptr_t)Wf | (uintptr_t)b0 | (uintptr_t)gw1 | (uintptr_t)fslab |
       (uintptr_t)gwo | (uintptr_t)gbo) & 15)
    return -3;
  const int nfwd = har_mlp_step_grid(B);
  if (fslab && (fslab_w < har_mlp_step_fwd_slab_width(H) || fslab_w % 4 || nfwd > 256 || !gwo || !gbo)) return -2;
  const int S = har_mlp_step_slices(B);
  const bf16_t* d2 = reinterpret_cast<const bf16_t*>(dact2);
  const bf16_t* x = reinterpret_cast<const bf16_t*>(X);
  const bf16_t* wf = reinterpret_cast<const bf16_t*>(Wf);
  if (K0 == 64)
    launch_bwd4<64>(d2, x, wf, b0, B, S, gw1, gw0, gb0, gb1, slab_stride, tick, fslab, fslab_w, nfwd, gwo, gbo, s);
  else
    launch_bwd4<32>(d2, x, wf, b0, B, S, gw1, gw0, gb0, gb1, slab_stride, tick, fslab, fslab_w, nfwd, gwo, gbo, s);
  HAR_CHECK_LAUNCH();
  return 0;
}

extern "C" void har_mlp_set_stamps(uint64_t* p) { g_har_mlp_stamps = p; }
