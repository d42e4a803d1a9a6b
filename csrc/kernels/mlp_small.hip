// Small-batch training step of the 2-hidden-layer MLP (H = 128 / 256, 16 padded classes): the WHOLE
// forward + backward of a 32-row tile in ONE workgroup, then the existing slab reduction + Adam kernel
// (mlp.hip grad_reduce_adam) — two launches per step instead of the three-kernel step's persistent
// forward, per-quadrant backward and reduction, whose prologues and slab epilogues are a fixed cost that
// a batch of 256 rows (8 forward workgroups, 16 backward workgroups) cannot amortize
// (profiles/r4/mlp_phase_probe.txt: 31.6 us per step at B = 256).
//
// One workgroup = 32 rows, 8 waves; every product is a 16x16 bf16 MFMA block with fp32 accumulation,
// activations as row-major [32][H] bf16 LDS images, weights from the fragment-ordered copies (W0, W1,
// W1^T: one 1 KB-contiguous load per fragment) and Wout staged in LDS:
//   h1^T = relu(W0 . X^T + b0)      h2^T = relu(W1 . h1^T + b1)      z^T = Wout . h2^T + bo (waves 0, 1)
//   softmax / CE / argmax per row -> dz (bf16, x 1 / global batch)
//   dWout = dz^T . h2, dbout         dact2^T = (Wout^T . dz^T) * relu'(h2)   (16x16x16, K = classes)
//   dW1 = dact2^T . h1, db1          dact1^T = (W1^T . dact2^T) * relu'(h1)
//   dW0 = dact1^T . X, db0
// The row-sum products (bias gradients, dW = act^T . act over the tile's 32 rows) take their operands
// with the transposing LDS reads (frag_tr: K = the 32 rows, one MFMA per 16x16 output block).  The
// workgroup's partial gradient goes to slab blockIdx.x in the flat parameter layout; the reduction sums
// the B / 32 slabs in a fixed order (bitwise reproducible) and runs Adam, refreshing Pb and all three
// fragment copies (W1^T included: no step kernel of this path writes it).
//
// Reference: none (the reference has no MLP); BASELINE.json config 3 ("test accuracy on WISDM": the
// batch-256 fit of the bench's WISDM accuracy run and main.py's MLP preset).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "../har_kernels.h"
#include "common.h"
#include "mlp_frag.h"

namespace {

using namespace mlpf;

constexpr int SR = 32;   // rows per workgroup
constexpr int NC16 = 16; // padded classes

template <int K0, int H>
struct SmallLds {
  static constexpr int HP = H + 16;      // [32][H] image pitch (bf16)
  static constexpr int XP = K0 + 16;     // X tile pitch
  static constexpr int ZP = NC16 + 8;    // dz pitch
  static constexpr int xs = 0;
  static constexpr int h1 = xs + SR * XP;
  static constexpr int h2 = h1 + SR * HP;
  static constexpr int d2 = h2 + SR * HP;
  static constexpr int d1 = d2 + SR * HP;
  static constexpr int dz = d1 + SR * HP;
  static constexpr int wo = dz + SR * ZP;
  static constexpr int end = wo + NC16 * HP;               // bf16 elements
  static constexpr size_t bytes = (size_t)end * 2 + 4 * sizeof(float) * 2;  // + loss / correct partials
};

template <int K0, int H>
__global__ __launch_bounds__(512) void mlp_small_step_kernel(MlpSmallStepArgs a) {
  using L = SmallLds<K0, H>;
  constexpr int UB = H / 16, KC = H / 32, K0C = K0 / 32, UPW = UB / 8;
  constexpr int HP = L::HP, XP = L::XP, ZP = L::ZP;
  extern __shared__ __attribute__((aligned(16))) bf16_t lds[];
  bf16_t* const xs = lds + L::xs;
  bf16_t* const h1s = lds + L::h1;
  bf16_t* const h2s = lds + L::h2;
  bf16_t* const d2s = lds + L::d2;
  bf16_t* const d1s = lds + L::d1;
  bf16_t* const dzs = lds + L::dz;
  bf16_t* const wos = lds + L::wo;
  float* const red = reinterpret_cast<float*>(lds + L::end);  // [2 waves] loss, [2] correct

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 15, g = lane >> 4;
  const int r0 = blockIdx.x * SR;
  if (a.tick && blockIdx.x == 0 && tid == 0) *a.tick += 1;  // Adam's step counter (graph-replay safe)
  const bf16_t* const W0f = a.Wf;
  const bf16_t* const W1f = a.Wf + H * K0;
  const bf16_t* const W1tf = a.Wf + H * K0 + H * H;
  float* const slab = a.slab + (size_t)blockIdx.x * a.total;

  // ---- stage X [32][K0] and Wout [16][H] (16-byte vectors) ----
  for (int v = tid; v < SR * K0 / 8; v += 512) {
    const int r = v / (K0 / 8), c = v % (K0 / 8);
    *reinterpret_cast<bf16x8_t*>(xs + r * XP + 8 * c) =
        *reinterpret_cast<const bf16x8_t*>(a.X + (size_t)(r0 + r) * K0 + 8 * c);
  }
  for (int v = tid; v < NC16 * H / 8; v += 512) {
    const int r = v / (H / 8), c = v % (H / 8);
    *reinterpret_cast<bf16x8_t*>(wos + r * HP + 8 * c) = *reinterpret_cast<const bf16x8_t*>(a.Wo + (size_t)r * H + 8 * c);
  }
  __syncthreads();

  // ---- h1^T = relu(W0 . X^T + b0): unit blocks wave * UPW .. + UPW - 1, both row blocks ----
#pragma unroll
  for (int t = 0; t < UPW; ++t) {
    const int ub = wave * UPW + t;
    bf16x8_t wf[K0C];
#pragma unroll
    for (int kc = 0; kc < K0C; ++kc)
      wf[kc] = *reinterpret_cast<const bf16x8_t*>(W0f + (size_t)(ub * K0C + kc) * 512 + frag_lane_off(lane));
    const float4 bb = *reinterpret_cast<const float4*>(a.b0 + 16 * ub + 4 * g);
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
      f32x4_t acc = {bb.x, bb.y, bb.z, bb.w};
#pragma unroll
      for (int kc = 0; kc < K0C; ++kc)
        acc = mma32(wf[kc], *reinterpret_cast<const bf16x8_t*>(xs + (16 * rb + li) * XP + 32 * kc + 8 * g), acc);
      *reinterpret_cast<uint2*>(h1s + (16 * rb + li) * HP + 16 * ub + 4 * g) =
          make_uint2(relu2(pack2(acc[0], acc[1])), relu2(pack2(acc[2], acc[3])));
    }
  }
  __syncthreads();

  // ---- h2^T = relu(W1 . h1^T + b1) ----
#pragma unroll
  for (int t = 0; t < UPW; ++t) {
    const int ub = wave * UPW + t;
    const float4 bb = *reinterpret_cast<const float4*>(a.b1 + 16 * ub + 4 * g);
    f32x4_t acc[2] = {f32x4_t{bb.x, bb.y, bb.z, bb.w}, f32x4_t{bb.x, bb.y, bb.z, bb.w}};
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      const bf16x8_t wf = *reinterpret_cast<const bf16x8_t*>(W1f + (size_t)(ub * KC + kc) * 512 + frag_lane_off(lane));
#pragma unroll
      for (int rb = 0; rb < 2; ++rb)
        acc[rb] = mma32(wf, *reinterpret_cast<const bf16x8_t*>(h1s + (16 * rb + li) * HP + 32 * kc + 8 * g), acc[rb]);
    }
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
      *reinterpret_cast<uint2*>(h2s + (16 * rb + li) * HP + 16 * ub + 4 * g) =
          make_uint2(relu2(pack2(acc[rb][0], acc[rb][1])), relu2(pack2(acc[rb][2], acc[rb][3])));
  }
  __syncthreads();

  // ---- logits z^T = Wout . h2^T + bo, softmax / CE / argmax, dz (waves 0 and 1: row block = wave) ----
  if (wave < 2) {
    const int rb = wave, row = 16 * rb + li;
    f32x4_t z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kc = 0; kc < KC; ++kc)
      z = mma32(*reinterpret_cast<const bf16x8_t*>(wos + li * HP + 32 * kc + 8 * g),
                *reinterpret_cast<const bf16x8_t*>(h2s + row * HP + 32 * kc + 8 * g), z);
    // lane: row `row`, classes 4 g + r
    const int y = a.labels[r0 + row];
    float zc[4], mx = -INFINITY;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int c = 4 * g + r;
      zc[r] = c < a.C ? z[r] + a.bo[c] : -INFINITY;
      mx = fmaxf(mx, zc[r]);
    }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    float e[4], se = 0.f;
    int amx = 1 << 30;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int c = 4 * g + r;
      e[r] = c < a.C ? __expf(zc[r] - mx) : 0.f;
      se += e[r];
      amx = (c < a.C && zc[r] == mx) ? min(amx, c) : amx;
    }
    se += __shfl_xor(se, 16, 64);
    se += __shfl_xor(se, 32, 64);
    amx = min(amx, __shfl_xor(amx, 16, 64));
    amx = min(amx, __shfl_xor(amx, 32, 64));
    const float inv = __builtin_amdgcn_rcpf(se);
    float lrow = 0.f;
    uint32_t pk[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      float d[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int r = 2 * q + h, c = 4 * g + r;
        d[h] = c < a.C ? (e[r] * inv - (c == y ? 1.f : 0.f)) * a.scale : 0.f;
        lrow += c == y ? (mx + __logf(se)) - zc[r] : 0.f;
      }
      pk[q] = pack2(d[0], d[1]);
    }
    *reinterpret_cast<uint2*>(dzs + row * ZP + 4 * g) = make_uint2(pk[0], pk[1]);
    float ncorr = (g == 0 && amx == y) ? 1.f : 0.f;
    lrow = wave_sum(lrow);
    ncorr = wave_sum(ncorr);
    if (lane == 0) {
      red[wave] = lrow;
      red[2 + wave] = ncorr;
    }
  }
  __syncthreads();
  if (tid == 0) {
    a.block_loss[blockIdx.x] = red[0] + red[1];
    a.block_correct[blockIdx.x] = (int32_t)(red[2] + red[3]);
  }

  // a row of ones (A operand, row 0): row 0 of ones . M = the column sums of M over the tile's rows
  const bf16x8_t ones = __builtin_bit_cast(bf16x8_t, li == 0 ? s16x8_t{0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80,
                                                                       0x3f80, 0x3f80, 0x3f80}
                                                             : s16x8_t{0, 0, 0, 0, 0, 0, 0, 0});
  const bf16x8_t dzT = frag_tr(dzs, ZP, 0, lane);  // A = dz^T [class li][rows 8g ..]

  // ---- dWout = dz^T . h2, dbout; dact2^T = (Wout^T . dz^T) * relu'(h2) ----
  const s16x4_t dzB[2] = {*reinterpret_cast<const s16x4_t*>(dzs + li * ZP + 4 * g),
                          *reinterpret_cast<const s16x4_t*>(dzs + (16 + li) * ZP + 4 * g)};  // B = dz^T [4g ..][row]
#pragma unroll
  for (int t = 0; t < UPW; ++t) {
    const int ub = wave * UPW + t;
    const f32x4_t dwo = mma32(dzT, frag_tr(h2s, HP, 16 * ub, lane), f32x4_t{0.f, 0.f, 0.f, 0.f});
#pragma unroll
    for (int r = 0; r < 4; ++r) slab[a.off_wo + (size_t)(4 * g + r) * H + 16 * ub + li] = dwo[r];
    // A = Wout^T [unit 16 ub + li][classes 4g .. 4g + 3]: one transposing 4 x 16 read of the Wout image
    const s16x4_t woT = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_s16x4_t*)(wos + (4 * g + (li >> 2)) * HP + 16 * ub + 4 * (li & 3)));
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
      const f32x4_t v = mma16(woT, dzB[rb], f32x4_t{0.f, 0.f, 0.f, 0.f});  // [unit 16ub + 4g + r][row 16rb + li]
      const int row = 16 * rb + li;
      const uint2 hm = *reinterpret_cast<const uint2*>(h2s + row * HP + 16 * ub + 4 * g);
      const float d0 = (hm.x & 0xffffu) ? v[0] : 0.f, d1 = (hm.x >> 16) ? v[1] : 0.f;
      const float d2 = (hm.y & 0xffffu) ? v[2] : 0.f, d3 = (hm.y >> 16) ? v[3] : 0.f;
      *reinterpret_cast<uint2*>(d2s + row * HP + 16 * ub + 4 * g) = make_uint2(pack2(d0, d1), pack2(d2, d3));
    }
  }
  if (wave == 0) {
    const f32x4_t db = mma32(ones, dzT, f32x4_t{0.f, 0.f, 0.f, 0.f});  // row 0: class sums (dzT read as B)
    if (g == 0) slab[a.off_bo + li] = db[0];
  }
  __syncthreads();

  // ---- dW1 = dact2^T . h1 (j blocks of this wave x every unit block), db1; dact1^T = (W1^T . dact2^T) * relu'(h1) ----
#pragma unroll
  for (int t = 0; t < UPW; ++t) {
    const int jb = wave * UPW + t;
    const bf16x8_t aT = frag_tr(d2s, HP, 16 * jb, lane);  // A = dact2^T [j 16 jb + li][rows]
#pragma unroll 4
    for (int ub = 0; ub < UB; ++ub) {
      const f32x4_t w = mma32(aT, frag_tr(h1s, HP, 16 * ub, lane), f32x4_t{0.f, 0.f, 0.f, 0.f});
#pragma unroll
      for (int r = 0; r < 4; ++r) slab[a.off_w1 + (size_t)(16 * jb + 4 * g + r) * H + 16 * ub + li] = w[r];
    }
    const f32x4_t db = mma32(ones, aT, f32x4_t{0.f, 0.f, 0.f, 0.f});  // (aT read as B: dact2 [rows][16 jb ..])
    if (g == 0) slab[a.off_b1 + 16 * jb + li] = db[0];
  }
#pragma unroll
  for (int t = 0; t < UPW; ++t) {
    const int ub = wave * UPW + t;
    f32x4_t acc[2] = {f32x4_t{0.f, 0.f, 0.f, 0.f}, f32x4_t{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      const bf16x8_t wf = *reinterpret_cast<const bf16x8_t*>(W1tf + (size_t)(ub * KC + kc) * 512 + frag_lane_off(lane));
#pragma unroll
      for (int rb = 0; rb < 2; ++rb)
        acc[rb] = mma32(wf, *reinterpret_cast<const bf16x8_t*>(d2s + (16 * rb + li) * HP + 32 * kc + 8 * g), acc[rb]);
    }
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
      const int row = 16 * rb + li;
      const uint2 hm = *reinterpret_cast<const uint2*>(h1s + row * HP + 16 * ub + 4 * g);
      const f32x4_t& v = acc[rb];
      const float d0 = (hm.x & 0xffffu) ? v[0] : 0.f, d1 = (hm.x >> 16) ? v[1] : 0.f;
      const float d2 = (hm.y & 0xffffu) ? v[2] : 0.f, d3 = (hm.y >> 16) ? v[3] : 0.f;
      *reinterpret_cast<uint2*>(d1s + row * HP + 16 * ub + 4 * g) = make_uint2(pack2(d0, d1), pack2(d2, d3));
    }
  }
  __syncthreads();

  // ---- dW0 = dact1^T . X, db0 ----
#pragma unroll
  for (int t = 0; t < UPW; ++t) {
    const int ub = wave * UPW + t;
    const bf16x8_t aT = frag_tr(d1s, HP, 16 * ub, lane);
#pragma unroll
    for (int fb = 0; fb < K0 / 16; ++fb) {
      const f32x4_t w = mma32(aT, frag_tr(xs, XP, 16 * fb, lane), f32x4_t{0.f, 0.f, 0.f, 0.f});
#pragma unroll
      for (int r = 0; r < 4; ++r) slab[a.off_w0 + (size_t)(16 * ub + 4 * g + r) * K0 + 16 * fb + li] = w[r];
    }
    const f32x4_t db = mma32(ones, aT, f32x4_t{0.f, 0.f, 0.f, 0.f});  // (aT is also dact1 [rows][16 ub ..] as B)
    if (g == 0) slab[a.off_b0 + 16 * ub + li] = db[0];
  }
}

template <int K0, int H>
int launch_small(const MlpSmallStepArgs& a, hipStream_t s) {
  using L = SmallLds<K0, H>;
  static_assert(L::bytes <= 160 * 1024, "the small-step images fit the LDS");
  static bool attr = [] {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&mlp_small_step_kernel<K0, H>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)L::bytes) == hipSuccess;
  }();
  if (!attr) return -4;
  mlp_small_step_kernel<K0, H><<<a.B / SR, 512, L::bytes, s>>>(a);
  HAR_CHECK_LAUNCH();
  return 0;
}

}  // namespace

extern "C" int har_mlp_small_step_max_batch() { return 512; }

extern "C" int har_mlp_small_step(const MlpSmallStepArgs* args, int K0, int H, hipStream_t s) {
  const MlpSmallStepArgs& a = *args;
  if (!a.X || !a.Wf || !a.Wo || !a.labels || !a.slab || !a.block_loss || !a.block_correct || a.B <= 0 || a.B % SR ||
      a.B > har_mlp_small_step_max_batch() || a.C < 1 || a.C > NC16 || a.total <= 0 ||
      a.off_w0 + (int64_t)H * K0 > a.total || a.off_w1 + (int64_t)H * H > a.total ||
      a.off_wo + (int64_t)NC16 * H > a.total || a.off_bo + NC16 > a.total || a.off_b0 + H > a.total ||
      a.off_b1 + H > a.total)
    return -2;
  if (((uintptr_t)a.X | (uintptr_t)a.Wf | (uintptr_t)a.Wo | (uintptr_t)a.b0 | (uintptr_t)a.b1) & 15) return -3;
  if (K0 == 64 && H == 256) return launch_small<64, 256>(a, s);
  if (K0 == 32 && H == 256) return launch_small<32, 256>(a, s);
  if (K0 == 64 && H == 128) return launch_small<64, 128>(a, s);
  if (K0 == 32 && H == 128) return launch_small<32, 128>(a, s);
  return -2;
}
