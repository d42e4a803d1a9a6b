// Fused MLP forward + classifier head + head weight gradient: one kernel per step
// for the 2-hidden-layer MLP (input K0 = 32/64 padded features, hidden H = 128/256,
// <= 16 classes).  Replaces four launches of the unfused step (two forward GEMMs,
// head_fused, the dWout GEMM) and their activation round trips through HBM: h2
// and dlogits never leave the CU.
//
// Work split: persistent grid (<= one workgroup per CU, 4 waves); each wave owns
// 16-row batch tiles and runs the whole chain in registers using the TRANSPOSED
// products, so the accumulator of one MFMA is directly the B operand of the next:
//
//   stage 1  h1^T = W0 . X^T            16x16x32 MFMA, A = W0 (L2), B = X rows (16-B loads)
//   stage 2  h2^T = W1 . h1^T           A = W1 (LDS-resident, swizzled), B = h1^T registers
//   stage 3  z^T  = Wout . h2^T         A = Wout (LDS), B = h2^T registers
//            softmax / CE / argmax over the class rows (in-lane + 2 shuffles)
//   stage 4  dact2^T = Wout^T . dz^T    16x16x16 MFMA (K = 16 classes), mask relu'(h2)
//   stage 5  dWout^T += h2^T . dz       16x16x16 MFMA (K = the 16 batch rows of the tile),
//            operands re-laid through a per-wave LDS tile + ds_read_b64_tr_b16
//
// Operand trick (stages 2/3): the C/D layout puts unit 4g+r of a 16-unit tile in
// register r of lane group g; as a B operand a lane must supply 8 k-values.  A
// 32-unit k-chunk is formed from two consecutive 16-unit tiles, k-slot j -> unit
// (j < 4 ? 4g + j : 16 + 4g + j - 4); the A operand (weights) is read from LDS with
// the SAME permutation (two 8-byte reads), so the contraction is unchanged.
//
// Outputs: h1 (bf16, for dW1 / dgrad), dact2 = (dz . Wout) * (h2 > 0) (bf16, for
// dW1 / dgrad), per-workgroup dWout rows 0..15 + dbout slabs (fp32, deterministic
// reduction later), per-workgroup loss / #correct.
#include <cstdlib>

#include "common.h"
#include "../har_kernels.h"

namespace {

typedef __attribute__((ext_vector_type(4))) short s16x4_t;
typedef __attribute__((address_space(3))) s16x4_t lds_s16x4_t;
typedef __attribute__((ext_vector_type(4))) uint32_t u32x4_t;

constexpr int NCLS = 16;
// per-workgroup gradient slab of the forward kernel: dWout rows 0..15 [16][H], dbout [16], db1 [H]
__host__ __device__ constexpr int fwd_slab_width(int H) { return NCLS * H + NCLS + H; }
constexpr int SCR = 3 * 256;  // per-wave scratch: 2 h2 tiles + 1 dz tile, 16x16 bf16 each

// [rows][H + 8] bf16 images (one 16-byte pad per row): the 8-byte A-fragment reads of
// stages 2/3 (row 16t + lane&15, column 32kc + 4g [+16]) hit bank pair 2(2 row + chunk)
// mod 64 -> conflict-free per 32-lane group, and every address is one per-lane base plus
// a compile-time offset (no per-(t, kc) address registers).
template <int H> struct Pitch { static constexpr int v = H + 8; };

__device__ __forceinline__ uint32_t pack2(float a, float b) {
  return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16);
}

__device__ __forceinline__ f32x4_t mma32(bf16x8_t a, bf16x8_t b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4_t mma16(s16x4_t a, s16x4_t b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ bf16x8_t cat8(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  return __builtin_bit_cast(bf16x8_t, u32x4_t{a, b, c, d});
}

__device__ __forceinline__ bool bf_pos(uint32_t h) { return (h & 0x8000u) == 0 && (h & 0xffffu) != 0; }

// An empty asm that consumes N loaded vectors: the compiler must issue all N loads before it
// (one vmcnt wait for the batch) instead of sinking each load next to its LDS store.
template <int N> __device__ __forceinline__ void hold_all(u32x4_t (&b)[N]);
template <> __device__ __forceinline__ void hold_all<8>(u32x4_t (&b)[8]) {
  asm volatile("" ::"v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]), "v"(b[4]), "v"(b[5]), "v"(b[6]), "v"(b[7]));
}
template <> __device__ __forceinline__ void hold_all<16>(u32x4_t (&b)[16]) {
  asm volatile("" ::"v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]), "v"(b[4]), "v"(b[5]), "v"(b[6]), "v"(b[7]),
               "v"(b[8]), "v"(b[9]), "v"(b[10]), "v"(b[11]), "v"(b[12]), "v"(b[13]), "v"(b[14]), "v"(b[15]));
}

// X fragment of one lane: 8 consecutive k of row `row`.  XF = 0: padded bf16 [B][K0];
// XF = 1 (serving): raw fp32 features [B][ldx] with F valid columns, converted in registers —
// no separate cast/pad pass over the input.
template <int K0, int XF>
__device__ __forceinline__ bf16x8_t load_x(const bf16_t* __restrict__ X, int row, int kc, int g, int F, int ldx) {
  if constexpr (XF == 0) {
    return *reinterpret_cast<const bf16x8_t*>(X + (size_t)row * K0 + kc * 32 + g * 8);
  } else {
    const float* xf = reinterpret_cast<const float*>(X) + (size_t)row * ldx;
    const int k0 = kc * 32 + g * 8;
    bf16x8_t r;
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = (__bf16)(k0 + j < F ? xf[k0 + j] : 0.f);
    return r;
  }
}

// INFER = true: the serving variant — stages 1-3 only; writes the logits [B][C] (fp32) and the
// argmax class per row, no label / loss / gradient work and no h1 store.
template <int H, int K0, bool INFER, int XF = 0>
__global__ __launch_bounds__(256) void mlp_fwd_head_kernel(
    const bf16_t* __restrict__ X, const bf16_t* __restrict__ W0, const float* __restrict__ b0,
    const bf16_t* __restrict__ W1, const float* __restrict__ b1, const bf16_t* __restrict__ Wo,
    const float* __restrict__ bo, const int32_t* __restrict__ labels, int B, int C, float scale,
    bf16_t* __restrict__ h1out, bf16_t* __restrict__ dact, float* __restrict__ slab,
    float* __restrict__ block_loss, int32_t* __restrict__ block_correct, float* __restrict__ logits_out,
    int32_t* __restrict__ pred_out, int F, int ldx) {
  constexpr int NT = H / 16, KC = H / 32, K0C = K0 / 32;
  extern __shared__ __attribute__((aligned(16))) bf16_t lds[];
  constexpr int P = Pitch<H>::v;
  bf16_t* W1s = lds;              // [H][P]
  bf16_t* Wos = W1s + H * P;      // [16][P]
  bf16_t* WoT = Wos + NCLS * P;   // [H][16]
  float* bs = reinterpret_cast<float*>(WoT + H * NCLS);  // b0 [H], b1 [H]
  bf16_t* scr = reinterpret_cast<bf16_t*>(bs + 2 * H);   // [4][SCR]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int c16 = lane & 15, g = lane >> 4;

  // ---- prologue: every global load of the weights is issued before the first wait ----
  // W0 A-fragments stay in registers for the whole kernel (no global loads in the loop:
  // vmcnt is in-order on CDNA, so a load behind the previous tile's stores would wait for them)
  bf16x8_t w0f[NT][K0C];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int kc = 0; kc < K0C; ++kc)
      w0f[t][kc] = *reinterpret_cast<const bf16x8_t*>(W0 + (size_t)(16 * t + c16) * K0 + kc * 32 + g * 8);
  {
    constexpr int NV = H * H / 8, NB = NV / 256 < 16 ? NV / 256 : 16;  // W1 16-byte vectors in flight
    static_assert(NV % (NB * 256) == 0, "W1 staging: whole batches");
    constexpr int NO = NCLS * H / 8;        // Wout rows 0..15
    uint4 wo[(NO + 255) / 256];
#pragma unroll
    for (int i = 0; i < (NO + 255) / 256; ++i) {
      const int v = i * 256 + tid;
      wo[i] = v < NO ? *reinterpret_cast<const uint4*>(Wo + (size_t)v * 8) : make_uint4(0, 0, 0, 0);
    }
    const float bv0 = tid < H ? b0[tid] : 0.f, bv1 = tid < H ? b1[tid] : 0.f;
#pragma unroll 1
    for (int v0 = 0; v0 < NV; v0 += NB * 256) {
      u32x4_t buf[NB];
#pragma unroll
      for (int i = 0; i < NB; ++i) buf[i] = *reinterpret_cast<const u32x4_t*>(W1 + (size_t)(v0 + i * 256 + tid) * 8);
      hold_all<NB>(buf);  // every load issued before the first wait (else: load / wait / store x NB)
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const int v = v0 + i * 256 + tid;
        *reinterpret_cast<u32x4_t*>(W1s + (v / (H / 8)) * P + (v % (H / 8)) * 8) = buf[i];
      }
    }
#pragma unroll
    for (int i = 0; i < (NO + 255) / 256; ++i) {
      const int v = i * 256 + tid;
      if (v < NO) *reinterpret_cast<uint4*>(Wos + (v / (H / 8)) * P + (v % (H / 8)) * 8) = wo[i];
    }
    if (tid < H) {
      bs[tid] = bv0;
      bs[H + tid] = bv1;
    }
  }
  __syncthreads();
  for (int e = tid; e < NCLS * H; e += 256) {  // Wout^T image from the LDS copy
    const int cls = e / H, u = e % H;
    WoT[u * NCLS + cls] = Wos[cls * P + u];
  }
  __syncthreads();

  bf16_t* sw = scr + wave * SCR;
  bf16_t* dzs = sw + 2 * 256;
  const int tr_off = (4 * g + (c16 >> 2)) * 16 + (c16 & 3) * 4;  // ds_read_b64_tr_b16 lane address in a tile
  f32x4_t acc5[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc5[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  float dbo[4] = {0.f, 0.f, 0.f, 0.f};
  float lsum = 0.f;
  int ncorr = 0;
  float bo_r[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) bo_r[r] = (4 * g + r < C) ? bo[4 * g + r] : 0.f;

  const int ntiles = B / 16;
  const int stride = gridDim.x * 4;
  int T = blockIdx.x * 4 + wave;
  bf16x8_t xb[K0C];
  int y = 0;
  if (T < ntiles) {
#pragma unroll
    for (int kc = 0; kc < K0C; ++kc)
      xb[kc] = load_x<K0, XF>(X, T * 16 + c16, kc, g, F, ldx);
    if (!INFER) y = labels[T * 16 + c16];
  }
  // drain the first prefetch here: otherwise the loop-header wait the compiler derives from
  // this path (vmcnt(0)) also applies on the back edge, where it would wait for every
  // dact2 store of the previous tile
  __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0)
  for (; T < ntiles; T += stride) {
    const int row = T * 16 + c16;
    // ---- stage 1: h1^T = W0 . X^T ----
    uint32_t h1p[NT][2];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      f32x4_t a = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kc = 0; kc < K0C; ++kc) a = mma32(w0f[t][kc], xb[kc], a);
      const float4 bb = *reinterpret_cast<const float4*>(bs + 16 * t + 4 * g);
      h1p[t][0] = pack2(fmaxf(a[0] + bb.x, 0.f), fmaxf(a[1] + bb.y, 0.f));
      h1p[t][1] = pack2(fmaxf(a[2] + bb.z, 0.f), fmaxf(a[3] + bb.w, 0.f));
      if (!INFER)
        *reinterpret_cast<uint2*>(h1out + (size_t)row * H + 16 * t + 4 * g) = make_uint2(h1p[t][0], h1p[t][1]);
    }
    // prefetch the next tile's X rows and labels (issued before this tile's dact2 stores)
    const int Tn = T + stride;
    const int yc = y;
    if (Tn < ntiles) {
#pragma unroll
      for (int kc = 0; kc < K0C; ++kc)
        xb[kc] = load_x<K0, XF>(X, Tn * 16 + c16, kc, g, F, ldx);
      if (!INFER) y = labels[Tn * 16 + c16];
    }
    __builtin_amdgcn_sched_barrier(0);
    // ---- stage 2: h2^T = W1 . h1^T  (A fragments software-pipelined one tile ahead) ----
    uint32_t h2p[NT][2];
    uint2 fr[2][KC][2];
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      fr[0][kc][0] = *reinterpret_cast<const uint2*>(W1s + c16 * P + 32 * kc + 4 * g);
      fr[0][kc][1] = *reinterpret_cast<const uint2*>(W1s + c16 * P + 32 * kc + 16 + 4 * g);
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int cb = t & 1, nb = cb ^ 1;
      if (t + 1 < NT) {
        const int wr = 16 * (t + 1) + c16;
#pragma unroll
        for (int kc = 0; kc < KC; ++kc) {
          fr[nb][kc][0] = *reinterpret_cast<const uint2*>(W1s + wr * P + 32 * kc + 4 * g);
          fr[nb][kc][1] = *reinterpret_cast<const uint2*>(W1s + wr * P + 32 * kc + 16 + 4 * g);
        }
      }
      f32x4_t a = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kc = 0; kc < KC; ++kc)
        a = mma32(cat8(fr[cb][kc][0].x, fr[cb][kc][0].y, fr[cb][kc][1].x, fr[cb][kc][1].y),
                  cat8(h1p[2 * kc][0], h1p[2 * kc][1], h1p[2 * kc + 1][0], h1p[2 * kc + 1][1]), a);
      const float4 bb = *reinterpret_cast<const float4*>(bs + H + 16 * t + 4 * g);
      h2p[t][0] = pack2(fmaxf(a[0] + bb.x, 0.f), fmaxf(a[1] + bb.y, 0.f));
      h2p[t][1] = pack2(fmaxf(a[2] + bb.z, 0.f), fmaxf(a[3] + bb.w, 0.f));
      __builtin_amdgcn_sched_barrier(0);
    }
    // ---- stage 3: z^T = Wout . h2^T  (lane: classes 4g..4g+3 of batch row c16) ----
    f32x4_t z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      const uint2 lo = *reinterpret_cast<const uint2*>(Wos + c16 * P + 32 * kc + 4 * g);
      const uint2 hi = *reinterpret_cast<const uint2*>(Wos + c16 * P + 32 * kc + 16 + 4 * g);
      z = mma32(cat8(lo.x, lo.y, hi.x, hi.y),
                cat8(h2p[2 * kc][0], h2p[2 * kc][1], h2p[2 * kc + 1][0], h2p[2 * kc + 1][1]), z);
    }
    float zz[4];
    float mx = -INFINITY;
    int amx = 1 << 30;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int cls = 4 * g + r;
      zz[r] = cls < C ? z[r] + bo_r[r] : -INFINITY;
      if (zz[r] > mx) { mx = zz[r]; amx = cls; }
    }
#pragma unroll
    for (int o = 16; o <= 32; o <<= 1) {
      const float om = __shfl_xor(mx, o, 64);
      const int oa = __shfl_xor(amx, o, 64);
      if (om > mx || (om == mx && oa < amx)) { mx = om; amx = oa; }
    }
    if constexpr (INFER) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (4 * g + r < C) logits_out[(size_t)row * C + 4 * g + r] = zz[r];
      if (g == 0) pred_out[row] = amx;
      continue;
    }
    float e[4], se = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      e[r] = (4 * g + r < C) ? __expf(zz[r] - mx) : 0.f;
      se += e[r];
    }
    se += __shfl_xor(se, 16, 64);
    se += __shfl_xor(se, 32, 64);
    const float inv = 1.f / se, lse = mx + __logf(se);
    float dl[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int cls = 4 * g + r;
      dl[r] = cls < C ? (e[r] * inv - (cls == yc ? 1.f : 0.f)) * scale : 0.f;
      if (cls == yc) lsum += lse - zz[r];
    }
    if (g == 0 && amx == yc) ncorr += 1;
    const uint32_t dz01 = pack2(dl[0], dl[1]), dz23 = pack2(dl[2], dl[3]);
    dbo[0] += __uint_as_float(dz01 << 16);
    dbo[1] += __uint_as_float(dz01 & 0xffff0000u);
    dbo[2] += __uint_as_float(dz23 << 16);
    dbo[3] += __uint_as_float(dz23 & 0xffff0000u);
    const s16x4_t dzv = __builtin_bit_cast(s16x4_t, make_uint2(dz01, dz23));
    __builtin_amdgcn_sched_barrier(0);
    // ---- stage 4: dact2^T = Wout^T . dz^T, masked by relu'(h2) ----
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const s16x4_t a = *reinterpret_cast<const s16x4_t*>(WoT + (16 * t + c16) * NCLS + 4 * g);
      const f32x4_t d = mma16(a, dzv, f32x4_t{0.f, 0.f, 0.f, 0.f});
      const uint32_t m0 = h2p[t][0], m1 = h2p[t][1];
      const float d0 = bf_pos(m0) ? d[0] : 0.f, d1 = bf_pos(m0 >> 16) ? d[1] : 0.f;
      const float d2 = bf_pos(m1) ? d[2] : 0.f, d3 = bf_pos(m1 >> 16) ? d[3] : 0.f;
      *reinterpret_cast<uint2*>(dact + (size_t)row * H + 16 * t + 4 * g) = make_uint2(pack2(d0, d1), pack2(d2, d3));
    }
    __builtin_amdgcn_sched_barrier(0);
    // ---- stage 5: dWout^T += h2^T . dz over the tile's 16 rows ----
    *reinterpret_cast<uint2*>(dzs + c16 * 16 + 4 * g) = make_uint2(dz01, dz23);
#pragma unroll
    for (int t0 = 0; t0 < NT; t0 += 2) {
#pragma unroll
      for (int tt = 0; tt < 2; ++tt)
        *reinterpret_cast<uint2*>(sw + tt * 256 + c16 * 16 + 4 * g) = make_uint2(h2p[t0 + tt][0], h2p[t0 + tt][1]);
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's tiles are in LDS
      __builtin_amdgcn_wave_barrier();
      const s16x4_t bz = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(dzs + tr_off));
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) {
        const s16x4_t ah = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(sw + tt * 256 + tr_off));
        acc5[t0 + tt] = mma16(ah, bz, acc5[t0 + tt]);
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);  // reads done before the tiles are overwritten
      __builtin_amdgcn_wave_barrier();
    }
    __builtin_amdgcn_sched_barrier(0);
  }

  if constexpr (INFER) return;
  // ---- per-workgroup reduction (fixed order) into this workgroup's slab ----
  __syncthreads();  // W1 image no longer needed: reuse it
  float* red = reinterpret_cast<float*>(lds);  // [4][16 classes][H]
#pragma unroll
  for (int t = 0; t < NT; ++t)
    *reinterpret_cast<f32x4_t*>(red + (size_t)(wave * NCLS + c16) * H + 16 * t + 4 * g) = acc5[t];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) dbo[r] += __shfl_xor(dbo[r], o, 64);
  float* redb = red + 4 * NCLS * H;  // [4][16]
  float* redl = redb + 4 * NCLS;     // [4] loss, [4] correct
  if (c16 == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) redb[wave * NCLS + 4 * g + r] = dbo[r];
  }
  lsum = wave_sum(lsum);
  const float nc = wave_sum((float)ncorr);
  if (lane == 0) { redl[wave] = lsum; redl[4 + wave] = nc; }
  __syncthreads();
  float* out = slab + (size_t)blockIdx.x * fwd_slab_width(H);  // v1 leaves db1 to the unfused backward
  for (int i = tid; i < NCLS * H; i += 256)
    out[i] = ((red[i] + red[NCLS * H + i]) + (red[2 * NCLS * H + i] + red[3 * NCLS * H + i]));
  if (tid < NCLS) out[NCLS * H + tid] = (redb[tid] + redb[NCLS + tid]) + (redb[2 * NCLS + tid] + redb[3 * NCLS + tid]);
  if (tid == 0) {
    block_loss[blockIdx.x] = (redl[0] + redl[1]) + (redl[2] + redl[3]);
    block_correct[blockIdx.x] = (int)((redl[4] + redl[5]) + (redl[6] + redl[7]));
  }
}

template <int H, int K0, bool INFER = false, int XF = 0>
int launch(const bf16_t* X, const bf16_t* W0, const float* b0, const bf16_t* W1, const float* b1,
           const bf16_t* Wo, const float* bo, const int32_t* labels, int B, int C, float scale, bf16_t* h1,
           bf16_t* dact, float* slab, float* block_loss, int32_t* block_correct, int nwg, hipStream_t s,
           float* logits = nullptr, int32_t* pred = nullptr, int F = K0, int ldx = K0) {
  const size_t lds = ((size_t)(H + NCLS) * Pitch<H>::v + NCLS * H + 4 * SCR) * sizeof(bf16_t) + 2 * H * sizeof(float);
  mlp_fwd_head_kernel<H, K0, INFER, XF><<<nwg, 256, lds, s>>>(X, W0, b0, W1, b1, Wo, bo, labels, B, C, scale, h1,
                                                              dact, slab, block_loss, block_correct, logits, pred, F,
                                                              ldx);
  HAR_CHECK_LAUNCH();
  return 0;
}


}  // namespace

extern "C" int har_mlp_fwd_head_grid(int B) {
  // persistent: at most one workgroup per CU; a workgroup-tile is 32 rows (v2: two 16-row halves,
  // v1: two waves' 16-row tiles)
  return std::max(1, std::min(256, (B / 16 + 1) / 2));
}

extern "C" int har_mlp_fwd_head(const uint16_t* X, int K0, const uint16_t* W0, const float* b0, const uint16_t* W1,
                                const float* b1, int H, const uint16_t* Wo, const float* bo, const int32_t* labels,
                                int B, int C, float scale, uint16_t* h1, uint16_t* dact, float* slab,
                                float* block_loss, int32_t* block_correct, hipStream_t s) {
  if (B <= 0 || B % 16 || C < 1 || C > NCLS) return -2;
  if (((uintptr_t)X | (uintptr_t)W0 | (uintptr_t)W1 | (uintptr_t)Wo | (uintptr_t)h1 | (uintptr_t)dact |
       (uintptr_t)b0 | (uintptr_t)b1 | (uintptr_t)slab) & 15)
    return -3;
  const int nwg = har_mlp_fwd_head_grid(B);
  if (H == 256 && K0 == 64) return launch<256, 64>(X, W0, b0, W1, b1, Wo, bo, labels, B, C, scale, h1, dact, slab, block_loss, block_correct, nwg, s);
  if (H == 256 && K0 == 32) return launch<256, 32>(X, W0, b0, W1, b1, Wo, bo, labels, B, C, scale, h1, dact, slab, block_loss, block_correct, nwg, s);
  if (H == 128 && K0 == 64) return launch<128, 64>(X, W0, b0, W1, b1, Wo, bo, labels, B, C, scale, h1, dact, slab, block_loss, block_correct, nwg, s);
  if (H == 128 && K0 == 32) return launch<128, 32>(X, W0, b0, W1, b1, Wo, bo, labels, B, C, scale, h1, dact, slab, block_loss, block_correct, nwg, s);
  return -4;
}

extern "C" int har_mlp_fwd_infer(const uint16_t* X, int K0, const uint16_t* W0, const float* b0, const uint16_t* W1,
                                 const float* b1, int H, const uint16_t* Wo, const float* bo, int B, int C,
                                 float* logits, int32_t* pred, hipStream_t s) {
  if (B <= 0 || B % 16 || C < 1 || C > NCLS) return -2;
  if (((uintptr_t)X | (uintptr_t)W0 | (uintptr_t)W1 | (uintptr_t)Wo | (uintptr_t)b0 | (uintptr_t)b1) & 15) return -3;
  const int nwg = har_mlp_fwd_head_grid(B);
  const bf16_t* x = X;
  if (H == 256 && K0 == 64) return launch<256, 64, true>(x, W0, b0, W1, b1, Wo, bo, nullptr, B, C, 1.f, nullptr, nullptr, nullptr, nullptr, nullptr, nwg, s, logits, pred);
  if (H == 256 && K0 == 32) return launch<256, 32, true>(x, W0, b0, W1, b1, Wo, bo, nullptr, B, C, 1.f, nullptr, nullptr, nullptr, nullptr, nullptr, nwg, s, logits, pred);
  if (H == 128 && K0 == 64) return launch<128, 64, true>(x, W0, b0, W1, b1, Wo, bo, nullptr, B, C, 1.f, nullptr, nullptr, nullptr, nullptr, nullptr, nwg, s, logits, pred);
  if (H == 128 && K0 == 32) return launch<128, 32, true>(x, W0, b0, W1, b1, Wo, bo, nullptr, B, C, 1.f, nullptr, nullptr, nullptr, nullptr, nullptr, nwg, s, logits, pred);
  return -4;
}

// Serving from raw fp32 features X [B][ldx] (F <= K0 valid columns): the bf16 cast / zero pad
// happens in the kernel's X loads.
extern "C" int har_mlp_fwd_infer_f32(const float* X, int ldx, int F, int K0, const uint16_t* W0, const float* b0,
                                     const uint16_t* W1, const float* b1, int H, const uint16_t* Wo, const float* bo,
                                     int B, int C, float* logits, int32_t* pred, hipStream_t s) {
  if (B <= 0 || B % 16 || C < 1 || C > NCLS || F < 1 || F > K0 || ldx < F) return -2;
  if (((uintptr_t)W0 | (uintptr_t)W1 | (uintptr_t)Wo | (uintptr_t)b0 | (uintptr_t)b1) & 15) return -3;
  const int nwg = har_mlp_fwd_head_grid(B);
  const bf16_t* x = reinterpret_cast<const bf16_t*>(X);
#define HAR_INFER_F32(HH, KK)                                                                                     \
  if (H == HH && K0 == KK)                                                                                        \
    return launch<HH, KK, true, 1>(x, W0, b0, W1, b1, Wo, bo, nullptr, B, C, 1.f, nullptr, nullptr, nullptr,       \
                                   nullptr, nullptr, nwg, s, logits, pred, F, ldx);
  HAR_INFER_F32(256, 64) HAR_INFER_F32(256, 32) HAR_INFER_F32(128, 64) HAR_INFER_F32(128, 32)
#undef HAR_INFER_F32
  return -4;
}
