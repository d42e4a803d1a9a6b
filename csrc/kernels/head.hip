// Fused classifier head + first backward layer of the MLP step, and the grouped
// (two-level, deterministic) split-K slab reduction.
//
// head_fused: one wave per 16-row tile (64 rows per workgroup):
//   logits = H . Wout^T + b           (v_mfma_f32_16x16x32_bf16, K = hidden dim)
//   softmax, cross-entropy, argmax    (16-lane shuffles; per-workgroup partial loss / #correct)
//   dz     = (p - onehot(y)) * scale  -> dlogits [B][32] bf16 (input of the dWout GEMM)
//   dH     = (dz . Wout) * (H > 0)    (K = 32: one MFMA per 16 output columns; Wout
//                                      staged once per workgroup as a [class][hidden]
//                                      LDS image read with ds_read_b64_tr_b16)
// so the separate data-gradient GEMM of the last hidden layer and its re-read of
// dlogits disappear; dH leaves through LDS as 16-byte row vectors with the ReLU
// mask applied from 16-byte reads of H (L2-hot: this workgroup just streamed it).
#include "common.h"
#include "../har_kernels.h"

namespace {

typedef __attribute__((ext_vector_type(4))) short s16x4_t;
typedef __attribute__((ext_vector_type(8))) short s16x8_t;
typedef __attribute__((address_space(3))) s16x4_t lds_s16x4_t;

constexpr int ROWS = 64;  // 4 waves x 16 rows
constexpr int DZP = 40;   // dz LDS pitch (32 classes + 16-byte pad)

// DT = compile-time hidden width (0 = runtime D): a static trip count lets hipcc issue every
// H-row load of the logits loop up front.
template <int DT>
__global__ __launch_bounds__(256) void head_fused_kernel(
    const bf16_t* __restrict__ H, const bf16_t* __restrict__ W, const float* __restrict__ bias,
    const int32_t* __restrict__ labels, int B, int Drt, int C, float scale, bf16_t* __restrict__ dlogits,
    bf16_t* __restrict__ dH, float* __restrict__ block_loss, int32_t* __restrict__ block_correct) {
  const int D = DT ? DT : Drt;
  extern __shared__ __attribute__((aligned(16))) bf16_t lds[];
  const int WP = D + 8;                       // Wout image pitch
  bf16_t* Ws = lds;                           // [32][D+8]
  bf16_t* dzs = Ws + 32 * WP;                 // [4][16][DZP]
  bf16_t* hs = dzs + 4 * 16 * DZP;            // [4][16][D+8] staging of dH
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r16 = lane & 15, q = lane >> 4;

  // stage Wout [32][D] (row-major = [k = class][n = hidden]) into LDS, 16-byte vectors
  for (int v = tid; v < 32 * D / 8; v += 256) {
    const int r = v / (D / 8), c = (v % (D / 8)) * 8;
    *reinterpret_cast<uint4*>(Ws + r * WP + c) = *reinterpret_cast<const uint4*>(W + (size_t)r * D + c);
  }

  __syncthreads();  // Wout image ready
  const int row0 = blockIdx.x * ROWS + wave * 16;
  const int arow = min(row0 + r16, B - 1);
  const int c0 = r16, c1 = r16 + 16;
  const bool v0 = c0 < C, v1 = c1 < C;
  f32x4_t acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  {
    const bf16_t* hrow = H + (size_t)arow * D + q * 8;
    const bf16_t* w0 = Ws + r16 * WP + q * 8;         // class rows straight from the LDS image
    const bf16_t* w1 = Ws + (r16 + 16) * WP + q * 8;
#pragma unroll
    for (int k = 0; k < D; k += 32) {
      bf16x8_t a = *reinterpret_cast<const bf16x8_t*>(hrow + k);
      acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, *reinterpret_cast<const bf16x8_t*>(w0 + k), acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, *reinterpret_cast<const bf16x8_t*>(w1 + k), acc1, 0, 0, 0);
    }
  }
  const float b0 = v0 ? bias[c0] : 0.f, b1 = v1 ? bias[c1] : 0.f;
  float lsum = 0.f;
  int ncorrect = 0;
  bf16_t* dzw = dzs + wave * 16 * DZP;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int rl = q * 4 + r, row = row0 + rl;
    const bool rok = row < B;
    const float z0 = v0 ? acc0[r] + b0 : -INFINITY;
    const float z1 = v1 ? acc1[r] + b1 : -INFINITY;
    float mx = fmaxf(z0, z1);
    int amx = (z1 > z0) ? c1 : c0;
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      const float om = __shfl_xor(mx, o, 64);
      const int oa = __shfl_xor(amx, o, 64);
      if (om > mx || (om == mx && oa < amx)) { mx = om; amx = oa; }
    }
    const float e0 = v0 ? __expf(z0 - mx) : 0.f, e1 = v1 ? __expf(z1 - mx) : 0.f;
    float se = e0 + e1;
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) se += __shfl_xor(se, o, 64);
    const int y = rok ? labels[row] : -1;
    const float inv = 1.f / se;
    const float g0 = (v0 && rok) ? (e0 * inv - (c0 == y ? 1.f : 0.f)) * scale : 0.f;
    const float g1 = (v1 && rok) ? (e1 * inv - (c1 == y ? 1.f : 0.f)) * scale : 0.f;
    const bf16_t gb0 = f2bf(g0), gb1 = f2bf(g1);
    dzw[rl * DZP + c0] = gb0;
    dzw[rl * DZP + c1] = gb1;
    if (rok) {
      dlogits[(size_t)row * 32 + c0] = gb0;
      dlogits[(size_t)row * 32 + c1] = gb1;
      const float lse = mx + __logf(se);
      if (c0 == y) lsum += lse - z0;
      if (c1 == y) lsum += lse - z1;
      if (r16 == 0 && amx == y) ncorrect += 1;
    }
  }
  __builtin_amdgcn_s_waitcnt(0);  // this wave's dz tile is in LDS (only this wave reads it)
  __builtin_amdgcn_wave_barrier();

  // ---- dH = dz . Wout  (K = 32 classes: one MFMA per 16 hidden columns) ----
  const bf16x8_t a = *reinterpret_cast<const bf16x8_t*>(dzw + r16 * DZP + q * 8);
  bf16_t* hw = hs + wave * 16 * WP;
  for (int j = 0; j < D / 16; ++j) {
    // B[k][n] from the [class][hidden] image: transposing reads, lane group q -> k = 8q .. 8q+7
    const int li = r16;
    const bf16_t* p0 = Ws + (8 * q + (li >> 2)) * WP + j * 16 + 4 * (li & 3);
    const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)p0);
    const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(p0 + 4 * WP));
    const s16x8_t bv = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    f32x4_t d = {0.f, 0.f, 0.f, 0.f};
    d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, __builtin_bit_cast(bf16x8_t, bv), d, 0, 0, 0);
#pragma unroll
    for (int r = 0; r < 4; ++r) hw[(q * 4 + r) * WP + j * 16 + r16] = f2bf(d[r]);
  }
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_wave_barrier();
  // copy-out with the ReLU mask: 16 rows x D columns, 8 bf16 per lane-vector
  const int vpr = D / 8;
  for (int v = lane; v < 16 * vpr; v += 64) {
    const int rl = v / vpr, c = (v % vpr) * 8;
    const int row = row0 + rl;
    if (row >= B) continue;
    union { uint4 u; bf16_t e[8]; } val, mk;
    val.u = *reinterpret_cast<const uint4*>(hw + rl * WP + c);
    mk.u = *reinterpret_cast<const uint4*>(H + (size_t)row * D + c);
#pragma unroll
    for (int e = 0; e < 8; ++e)
      if (!((mk.e[e] & 0x8000u) == 0 && mk.e[e] != 0)) val.e[e] = 0;
    *reinterpret_cast<uint4*>(dH + (size_t)row * D + c) = val.u;
  }

  // ---- per-workgroup partial loss / correct ----
  __shared__ float sl[4];
  __shared__ int sc[4];
  lsum = wave_sum(lsum);
  const float nc = wave_sum((float)ncorrect);
  if (lane == 0) { sl[wave] = lsum; sc[wave] = (int)nc; }
  __syncthreads();
  if (tid == 0) {
    block_loss[blockIdx.x] = sl[0] + sl[1] + sl[2] + sl[3];
    block_correct[blockIdx.x] = sc[0] + sc[1] + sc[2] + sc[3];
  }
}

// dst[g][i] = sum over slabs s in group g of slabs[s][i]  (G groups of ceil(S/G) slabs)
__global__ __launch_bounds__(256) void reduce_slabs_grouped_kernel(const float* __restrict__ slabs, int S, int64_t n,
                                                                   int64_t lds, float* __restrict__ dst, int G,
                                                                   int64_t ldd, int32_t* __restrict__ tick) {
  const int g = blockIdx.y;
  // optional optimizer-step tick (saves a one-thread launch; the Adam kernel runs after this one)
  if (tick && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) *tick += 1;
  const int per = (S + G - 1) / G;
  const int s0 = g * per, s1 = min(S, s0 + per);
  const int64_t n4 = n / 4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    int s = s0;
    for (; s + 4 <= s1; s += 4) {  // 4 independent loads in flight
      const float4 x0 = reinterpret_cast<const float4*>(slabs + (size_t)s * lds)[i];
      const float4 x1 = reinterpret_cast<const float4*>(slabs + (size_t)(s + 1) * lds)[i];
      const float4 x2 = reinterpret_cast<const float4*>(slabs + (size_t)(s + 2) * lds)[i];
      const float4 x3 = reinterpret_cast<const float4*>(slabs + (size_t)(s + 3) * lds)[i];
      acc.x += (x0.x + x1.x) + (x2.x + x3.x);
      acc.y += (x0.y + x1.y) + (x2.y + x3.y);
      acc.z += (x0.z + x1.z) + (x2.z + x3.z);
      acc.w += (x0.w + x1.w) + (x2.w + x3.w);
    }
    for (; s < s1; ++s) {
      const float4 x = reinterpret_cast<const float4*>(slabs + (size_t)s * lds)[i];
      acc.x += x.x; acc.y += x.y; acc.z += x.z; acc.w += x.w;
    }
    reinterpret_cast<float4*>(dst + (size_t)g * ldd)[i] = acc;
  }
}

// Several independent grouped reductions in ONE launch (blockIdx.z = segment): the per-step
// first reduction level of the MLP gradient (split-K slabs of W0..b1 + the fused kernel's
// per-workgroup dWout / dbout slabs) costs one launch instead of three.
struct ReduceSegs {
  const float* slabs[6];
  float* dst[6];
  int64_t n[6], lds[6], ldd[6];
  int S[6];
};

__global__ __launch_bounds__(256) void reduce_slabs_multi_kernel(ReduceSegs sg, int G, int32_t* __restrict__ tick) {
  const int z = blockIdx.z, g = blockIdx.y;
  if (tick && blockIdx.x == 0 && g == 0 && z == 0 && threadIdx.x == 0) *tick += 1;
  const float* __restrict__ slabs = sg.slabs[z];
  const int S = sg.S[z];
  const int64_t lds = sg.lds[z];
  const int per = (S + G - 1) / G;
  const int s0 = g * per, s1 = min(S, s0 + per);
  const int64_t n4 = sg.n[z] / 4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    int s = s0;
    for (; s + 4 <= s1; s += 4) {
      const float4 x0 = reinterpret_cast<const float4*>(slabs + (size_t)s * lds)[i];
      const float4 x1 = reinterpret_cast<const float4*>(slabs + (size_t)(s + 1) * lds)[i];
      const float4 x2 = reinterpret_cast<const float4*>(slabs + (size_t)(s + 2) * lds)[i];
      const float4 x3 = reinterpret_cast<const float4*>(slabs + (size_t)(s + 3) * lds)[i];
      acc.x += (x0.x + x1.x) + (x2.x + x3.x);
      acc.y += (x0.y + x1.y) + (x2.y + x3.y);
      acc.z += (x0.z + x1.z) + (x2.z + x3.z);
      acc.w += (x0.w + x1.w) + (x2.w + x3.w);
    }
    for (; s < s1; ++s) {
      const float4 x = reinterpret_cast<const float4*>(slabs + (size_t)s * lds)[i];
      acc.x += x.x; acc.y += x.y; acc.z += x.z; acc.w += x.w;
    }
    reinterpret_cast<float4*>(sg.dst[z] + (size_t)g * sg.ldd[z])[i] = acc;
  }
}

}  // namespace

extern "C" int har_reduce_slabs_multi(int nseg, const float* const* slabs, const int* S, const int64_t* n,
                                      const int64_t* lds, float* const* dst, const int64_t* ldd, int G, int32_t* tick,
                                      hipStream_t s) {
  if (nseg <= 0 || nseg > 6 || G <= 0) return -2;
  ReduceSegs sg{};
  int64_t n4max = 1;
  for (int z = 0; z < nseg; ++z) {
    if (n[z] % 4 || lds[z] % 4 || ldd[z] % 4 || lds[z] < n[z] || (G > 1 && ldd[z] < n[z]) || S[z] <= 0) return -2;
    if ((reinterpret_cast<uintptr_t>(slabs[z]) | reinterpret_cast<uintptr_t>(dst[z])) & 15) return -3;
    sg.slabs[z] = slabs[z]; sg.dst[z] = dst[z]; sg.n[z] = n[z]; sg.lds[z] = lds[z]; sg.ldd[z] = ldd[z];
    sg.S[z] = S[z];
    n4max = std::max<int64_t>(n4max, n[z] / 4);
  }
  const int bx = (int)std::max<int64_t>(1, std::min<int64_t>(1024, (n4max + 255) / 256));
  reduce_slabs_multi_kernel<<<dim3(bx, G, nseg), 256, 0, s>>>(sg, G, tick);
  HAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int har_head_fused_blocks(int B) { return (int)(((int64_t)B + ROWS - 1) / ROWS); }

extern "C" int har_head_fused(const uint16_t* H, const uint16_t* W, const float* bias, const int32_t* labels, int B,
                              int D, int C, float scale, uint16_t* dlogits, uint16_t* dH, float* block_loss,
                              int32_t* block_correct, hipStream_t s) {
  if (C > 32 || D % 32 || D > 1024) return -2;
  const int blocks = har_head_fused_blocks(B);
  if (blocks == 0) return 0;
  const size_t lds = (size_t)(32 * (D + 8) + 4 * 16 * DZP + 4 * 16 * (D + 8)) * sizeof(uint16_t);
  if (lds > 160 * 1024) return -3;
#define HEAD_LAUNCH(DT)                                                                                 \
  head_fused_kernel<DT><<<blocks, 256, lds, s>>>(H, W, bias, labels, B, D, C, scale, dlogits, dH, block_loss, \
                                                 block_correct)
  switch (D) {
    case 128: HEAD_LAUNCH(128); break;
    case 256: HEAD_LAUNCH(256); break;
    case 512: HEAD_LAUNCH(512); break;
    default: HEAD_LAUNCH(0);
  }
#undef HEAD_LAUNCH
  HAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int har_reduce_slabs_grouped(const float* slabs, int S, int64_t n, int64_t lds, float* dst, int G,
                                        int64_t ldd, int32_t* tick, hipStream_t s) {
  if (n % 4 || lds % 4 || ldd % 4 || lds < n || (G > 1 && ldd < n) || G <= 0 || S <= 0) return -2;
  if ((reinterpret_cast<uintptr_t>(slabs) | reinterpret_cast<uintptr_t>(dst)) & 15) return -3;
  const int64_t n4 = n / 4;
  const int bx = (int)std::max<int64_t>(1, std::min<int64_t>(1024, (n4 + 255) / 256));
  reduce_slabs_grouped_kernel<<<dim3(bx, G), 256, 0, s>>>(slabs, S, n, lds, dst, G, ldd, tick);
  HAR_CHECK_LAUNCH();
  return 0;
}
