// MLP step kernels: fused softmax-cross-entropy classifier head, fused Adam,
// padded bf16 casts.  The GEMMs of the step live in gemm.hip.
#include "common.h"
#include "../har_kernels.h"

namespace {

// One wave = 16 rows x 32 classes (two 16x16 MFMA accumulators), K = hidden dim.
// Operand fragments are loaded straight from global memory (W is tiny and
// L2-resident; H rows are streamed once): the GEMV-like regime where an LDS
// round trip is pure overhead (guide §5, 'GEMV / M <= 16' row).
__global__ __launch_bounds__(256) void softmax_ce_head_kernel(
    const bf16_t* __restrict__ H, const bf16_t* __restrict__ W, const float* __restrict__ bias,
    const int32_t* __restrict__ labels, int B, int D, int C, float scale, bf16_t* __restrict__ dlogits,
    float* __restrict__ dbias, float* __restrict__ loss_sum, int32_t* __restrict__ correct,
    float* __restrict__ logits_out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r16 = lane & 15, q = lane >> 4;
  const int row0 = (blockIdx.x * 4 + wave) * 16;
  if (row0 >= B) return;  // wave-uniform
  const int arow = min(row0 + r16, B - 1);

  f32x4_t acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  const bf16_t* hrow = H + (size_t)arow * D + q * 8;
  const bf16_t* w0 = W + (size_t)r16 * D + q * 8;
  const bf16_t* w1 = W + (size_t)(r16 + 16) * D + q * 8;
  for (int k = 0; k < D; k += 32) {
    bf16x8_t a = *reinterpret_cast<const bf16x8_t*>(hrow + k);
    bf16x8_t b0 = *reinterpret_cast<const bf16x8_t*>(w0 + k);
    bf16x8_t b1 = *reinterpret_cast<const bf16x8_t*>(w1 + k);
    acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b0, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b1, acc1, 0, 0, 0);
  }
  // lane holds rows row0 + 4q + r (r<4), columns c0 = r16 and c1 = r16 + 16
  const int c0 = r16, c1 = r16 + 16;
  const bool v0 = c0 < C, v1 = c1 < C;
  const float b0 = v0 ? bias[c0] : 0.f, b1 = v1 ? bias[c1] : 0.f;
  float lsum = 0.f, g0sum = 0.f, g1sum = 0.f;
  int ncorrect = 0;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = row0 + q * 4 + r;
    const bool rok = row < B;
    float z0 = v0 ? acc0[r] + b0 : -INFINITY;
    float z1 = v1 ? acc1[r] + b1 : -INFINITY;
    // row max / argmax over the 16-lane group (xor 1..8 stays inside the group)
    float mx = fmaxf(z0, z1);
    int amx = (z1 > z0) ? c1 : c0;
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      float om = __shfl_xor(mx, o, 64);
      int oa = __shfl_xor(amx, o, 64);
      if (om > mx || (om == mx && oa < amx)) { mx = om; amx = oa; }
    }
    float e0 = v0 ? __expf(z0 - mx) : 0.f, e1 = v1 ? __expf(z1 - mx) : 0.f;
    float se = e0 + e1;
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) se += __shfl_xor(se, o, 64);
    const float inv = 1.f / se;
    if (logits_out && rok) {
      if (v0) logits_out[(size_t)row * C + c0] = z0;
      if (v1) logits_out[(size_t)row * C + c1] = z1;
    }
    if (labels && rok) {
      const int y = labels[row];
      float p0 = e0 * inv, p1 = e1 * inv;
      float g0 = v0 ? (p0 - (c0 == y ? 1.f : 0.f)) * scale : 0.f;
      float g1 = v1 ? (p1 - (c1 == y ? 1.f : 0.f)) * scale : 0.f;
      bf16_t gb0 = f2bf(g0), gb1 = f2bf(g1);
      dlogits[(size_t)row * 32 + c0] = gb0;
      dlogits[(size_t)row * 32 + c1] = gb1;
      g0sum += bf2f(gb0);
      g1sum += bf2f(gb1);
      if (c0 == y) lsum += (mx + __logf(se)) - z0;
      if (c1 == y) lsum += (mx + __logf(se)) - z1;
      if (r16 == 0 && amx == y) ncorrect += 1;
    }
  }
  if (!labels) return;
  // bias gradient: reduce the 4 lanes sharing a column (q = 0..3)
  g0sum += __shfl_xor(g0sum, 16, 64);
  g0sum += __shfl_xor(g0sum, 32, 64);
  g1sum += __shfl_xor(g1sum, 16, 64);
  g1sum += __shfl_xor(g1sum, 32, 64);
  if (q == 0) {
    if (v0) atomicAdd(dbias + c0, g0sum);
    if (v1) atomicAdd(dbias + c1, g1sum);
  }
  lsum = wave_sum(lsum);
  float nc = wave_sum((float)ncorrect);
  if (lane == 0) {
    atomicAdd(loss_sum, lsum);
    atomicAdd(correct, (int)nc);
  }
}

// Step counter lives on the device so a captured hipGraph replays correct bias corrections.
__global__ void adam_tick_kernel(int32_t* step) { *step += 1; }

__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ param, const float* __restrict__ grad,
                                                   float* __restrict__ m, float* __restrict__ v,
                                                   bf16_t* __restrict__ pb, int64_t n, float lr, float b1,
                                                   float b2, float eps, float wd, float gs,
                                                   const int32_t* __restrict__ step) {
  const float t = (float)(*step);
  const float bc1 = 1.f - powf(b1, t), bc2 = 1.f - powf(b2, t);
  // 4 elements per thread per iteration (16-byte accesses), grid-stride
  const int64_t n4 = n / 4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 p = reinterpret_cast<float4*>(param)[i];
    float4 g = reinterpret_cast<const float4*>(grad)[i];
    float4 mm = reinterpret_cast<float4*>(m)[i];
    float4 vv = reinterpret_cast<float4*>(v)[i];
    float* pp = &p.x; float* gg = &g.x; float* mp = &mm.x; float* vp = &vv.x;
    ushort4 ob;
    unsigned short* op = &ob.x;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float gj = gg[j] * gs;
      mp[j] = b1 * mp[j] + (1.f - b1) * gj;
      vp[j] = b2 * vp[j] + (1.f - b2) * gj * gj;
      float upd = (mp[j] / bc1) / (sqrtf(vp[j] / bc2) + eps);
      pp[j] = pp[j] - lr * (upd + wd * pp[j]);
      op[j] = f2bf(pp[j]);
    }
    reinterpret_cast<float4*>(param)[i] = p;
    reinterpret_cast<float4*>(m)[i] = mm;
    reinterpret_cast<float4*>(v)[i] = vv;
    reinterpret_cast<ushort4*>(pb)[i] = ob;
  }
  // tail
  for (int64_t i = n4 * 4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float gj = grad[i] * gs;
    m[i] = b1 * m[i] + (1.f - b1) * gj;
    v[i] = b2 * v[i] + (1.f - b2) * gj * gj;
    float upd = (m[i] / bc1) / (sqrtf(v[i] / bc2) + eps);
    param[i] = param[i] - lr * (upd + wd * param[i]);
    pb[i] = f2bf(param[i]);
  }
}

__global__ void cast_pad_kernel(const float* __restrict__ in, int rows, int cin, int ldin,
                                bf16_t* __restrict__ out, int cout) {
  int64_t total = (int64_t)rows * cout;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    int r = (int)(i / cout), c = (int)(i % cout);
    out[i] = c < cin ? f2bf(in[(size_t)r * ldin + c]) : (bf16_t)0;
  }
}

}  // namespace

extern "C" int har_softmax_ce_head(const uint16_t* H, const uint16_t* W, const float* bias, const int32_t* labels,
                                   int B, int D, int C, float scale, uint16_t* dlogits, float* dbias,
                                   float* loss_sum, int32_t* correct, float* logits_out, hipStream_t s) {
  if (C > 32 || D % 32) return -2;
  int blocks = (B + 63) / 64;
  if (blocks == 0) return 0;
  softmax_ce_head_kernel<<<blocks, 256, 0, s>>>(H, W, bias, labels, B, D, C, scale, dlogits, dbias, loss_sum,
                                                correct, logits_out);
  HAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int har_adam_step(float* param, const float* grad, float* m, float* v, uint16_t* pb, int64_t n,
                             float lr, float b1, float b2, float eps, float wd, float gs, int32_t* step,
                             hipStream_t s) {
  int64_t blocks = std::min<int64_t>(2048, (n / 4 + 255) / 256 + 1);
  adam_tick_kernel<<<1, 1, 0, s>>>(step);
  adam_kernel<<<(int)blocks, 256, 0, s>>>(param, grad, m, v, pb, n, lr, b1, b2, eps, wd, gs, step);
  HAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int har_cast_pad_bf16(const float* in, int rows, int cin, int ldin, uint16_t* out, int cout,
                                 hipStream_t s) {
  int64_t total = (int64_t)rows * cout;
  int blocks = (int)std::min<int64_t>(4096, (total + 255) / 256);
  if (blocks == 0) return 0;
  cast_pad_kernel<<<blocks, 256, 0, s>>>(in, rows, cin, ldin, out, cout);
  HAR_CHECK_LAUNCH();
  return 0;
}
