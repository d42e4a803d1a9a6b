// MLP step kernels: fused softmax-cross-entropy classifier head, fused Adam
// (with the split-K gradient-slab reduction folded in), slab reduction, padded
// bf16 casts.  The GEMMs of the step live in gemm.hip.
//
// No same-address atomics anywhere on the step's critical path: per-workgroup
// partials are stored and reduced later (guide §6 G12: same-address float atomics
// serialize at L2; slab reductions are also bitwise reproducible).
#include "common.h"
#include "../har_kernels.h"

namespace {

constexpr int HEAD_ROWS_PER_BLOCK = 256;  // 4 waves x 4 row-tiles of 16

// One wave = 16 rows x 32 classes per row tile (two 16x16 MFMA accumulators), K = hidden dim.
// Operand fragments are loaded straight from global memory (W is tiny and
// L2-resident; H rows are streamed once): the GEMV-like regime where an LDS
// round trip is pure overhead (guide §5, 'GEMV / M <= 16' row).
__global__ __launch_bounds__(256) void softmax_ce_head_kernel(
    const bf16_t* __restrict__ H, const bf16_t* __restrict__ W, const float* __restrict__ bias,
    const int32_t* __restrict__ labels, int B, int D, int C, float scale, bf16_t* __restrict__ dlogits,
    float* __restrict__ block_loss, int32_t* __restrict__ block_correct, float* __restrict__ logits_out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r16 = lane & 15, q = lane >> 4;
  const int c0 = r16, c1 = r16 + 16;
  const bool v0 = c0 < C, v1 = c1 < C;
  const float b0 = v0 ? bias[c0] : 0.f, b1 = v1 ? bias[c1] : 0.f;
  float lsum = 0.f;
  int ncorrect = 0;

  for (int t = 0; t < HEAD_ROWS_PER_BLOCK / 64; ++t) {
    const int row0 = blockIdx.x * HEAD_ROWS_PER_BLOCK + (t * 4 + wave) * 16;
    if (row0 >= B) break;  // wave-uniform
    const int arow = min(row0 + r16, B - 1);
    f32x4_t acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
    const bf16_t* hrow = H + (size_t)arow * D + q * 8;
    const bf16_t* w0 = W + (size_t)r16 * D + q * 8;
    const bf16_t* w1 = W + (size_t)(r16 + 16) * D + q * 8;
    for (int k = 0; k < D; k += 32) {
      bf16x8_t a = *reinterpret_cast<const bf16x8_t*>(hrow + k);
      bf16x8_t bb0 = *reinterpret_cast<const bf16x8_t*>(w0 + k);
      bf16x8_t bb1 = *reinterpret_cast<const bf16x8_t*>(w1 + k);
      acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bb0, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bb1, acc1, 0, 0, 0);
    }
    // lane holds rows row0 + 4q + r (r<4), columns c0 and c1
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
      if (logits_out && rok) {
        if (v0) logits_out[(size_t)row * C + c0] = z0;
        if (v1) logits_out[(size_t)row * C + c1] = z1;
      }
      if (labels && rok) {
        const int y = labels[row];
        const float inv = 1.f / se;
        float g0 = v0 ? (e0 * inv - (c0 == y ? 1.f : 0.f)) * scale : 0.f;
        float g1 = v1 ? (e1 * inv - (c1 == y ? 1.f : 0.f)) * scale : 0.f;
        dlogits[(size_t)row * 32 + c0] = f2bf(g0);
        dlogits[(size_t)row * 32 + c1] = f2bf(g1);
        const float lse = mx + __logf(se);
        if (c0 == y) lsum += lse - z0;
        if (c1 == y) lsum += lse - z1;
        if (r16 == 0 && amx == y) ncorrect += 1;
      }
    }
  }
  if (!labels) return;
  __shared__ float sl[4];
  __shared__ int sc[4];
  lsum = wave_sum(lsum);
  float nc = wave_sum((float)ncorrect);
  if (lane == 0) { sl[wave] = lsum; sc[wave] = (int)nc; }
  __syncthreads();
  if (threadIdx.x == 0) {
    block_loss[blockIdx.x] = sl[0] + sl[1] + sl[2] + sl[3];
    block_correct[blockIdx.x] = sc[0] + sc[1] + sc[2] + sc[3];
  }
}

struct GradRegions {
  const float* src[8];
  int64_t start[8], len[8], lds[8];
  int S[8];
  int nreg;
};

// ---- MFMA-fragment-ordered bf16 copies of W0 / W1 for the step kernels (mlp_step.hip) ----
// A 16x16x32 A-operand fragment (16 rows x 32 k, lane l: row l & 15, k 8 (l >> 4) .. + 7) of a [R][C]
// matrix is stored as ONE contiguous KB in LANE order (lane l's 16 bytes at 16 l): element (r, c) at
// frag_pos(r, c, C).  A wave loads a fragment with one instruction whose 64 lanes read consecutive
// 16-byte pieces (frag_lane_off(l) = 8 l, mlp_frag.h): every quarter-wave touches 2 cache lines.  The
// row-major order inside the block (r4) put the 16 lanes of a quarter-wave on 16 lines 64 bytes apart
// and the forward's weight prologue stayed at ~8.7k cycles (profiles/r4/mlp_stamps_bwd4.txt) against
// 2.7k for a lane-sequential load (profiles/r4/prologue_probe.txt); the price is the optimizer's
// fragment stores (8-byte pieces, ~160 KB per step).  Layout of MlpFragSpec::dst: W0 [H][K0], W1 [H][H]
// (forward A: rows = layer-2 units), W1^T (backward A: rows = layer-1 units).
__device__ __forceinline__ int64_t frag_pos(int r, int c, int C) {
  return ((((int64_t)(r >> 4) * (C >> 5) + (c >> 5)) * 64 + ((c & 31) >> 3) * 16 + (r & 15)) << 3) + (c & 7);
}

// element e .. e + 3 of the flat parameter buffer (bf16 values ob) into the fragment copies; the
// W1^T copy too when `transposed` (2-byte scatter: the Adam kernel writes it from an LDS tile instead)
template <bool transposed>
__device__ __forceinline__ void frag_store4(const MlpFragSpec& f, int64_t e, ushort4 ob) {
  const int H = f.H, K0 = f.K0;
  const int64_t a0 = e - f.w0_off, a1 = e - f.w1_off;
  if (a0 >= 0 && a0 < (int64_t)H * K0) {
    const int u = (int)(a0 / K0), k = (int)(a0 % K0);
    *reinterpret_cast<ushort4*>(f.dst + frag_pos(u, k, K0)) = ob;
  } else if (a1 >= 0 && a1 < (int64_t)H * H) {
    const int j = (int)(a1 / H), u = (int)(a1 % H);
    bf16_t* w1 = f.dst + (int64_t)H * K0;
    *reinterpret_cast<ushort4*>(w1 + frag_pos(j, u, H)) = ob;
    if constexpr (transposed) {
      bf16_t* w1t = w1 + (int64_t)H * H;
      w1t[frag_pos(u, j, H)] = ob.x;
      w1t[frag_pos(u + 1, j, H)] = ob.y;
      w1t[frag_pos(u + 2, j, H)] = ob.z;
      w1t[frag_pos(u + 3, j, H)] = ob.w;
    }
  }
}

// refresh of the fragment copies from the flat bf16 copy (engine init / checkpoint load)
__global__ void mlp_pack_frag_kernel(const bf16_t* __restrict__ pb, MlpFragSpec f) {
  const int64_t n0 = (int64_t)f.H * f.K0 / 4, n1 = (int64_t)f.H * f.H / 4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n0 + n1; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = i < n0 ? f.w0_off + 4 * i : f.w1_off + 4 * (i - n0);
    frag_store4<true>(f, e, *reinterpret_cast<const ushort4*>(pb + e));
  }
}

// Step counter lives on the device so a captured hipGraph replays correct bias corrections.
__global__ void adam_tick_kernel(int32_t* step) { *step += 1; }

__device__ __forceinline__ float4 load_grad4(const float* __restrict__ grad, const float* __restrict__ slabs,
                                             int nslabs, int64_t n, int64_t i4) {
  if (!slabs) return reinterpret_cast<const float4*>(grad)[i4];
  float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int s = 0; s < nslabs; ++s) {
    float4 x = reinterpret_cast<const float4*>(slabs + (size_t)s * n)[i4];
    g.x += x.x; g.y += x.y; g.z += x.z; g.w += x.w;
  }
  return g;
}

__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ param, const float* __restrict__ grad,
                                                   const float* __restrict__ slabs, int nslabs,
                                                   float* __restrict__ m, float* __restrict__ v,
                                                   bf16_t* __restrict__ pb, int64_t n, float lr, float b1,
                                                   float b2, float eps, float wd, float gs,
                                                   const int32_t* __restrict__ step) {
  const float t = (float)(*step);
  const float bc1 = 1.f - powf(b1, t), bc2 = 1.f - powf(b2, t);
  // n is a multiple of 4 (flat buffers are 64-element padded): 16-byte accesses, grid-stride
  const int64_t n4 = n / 4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 p = reinterpret_cast<float4*>(param)[i];
    float4 g = load_grad4(grad, slabs, nslabs, n, i);
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
}

__global__ __launch_bounds__(256) void reduce_slabs_kernel(const float* __restrict__ slabs, int nslabs, int64_t n,
                                                           float* __restrict__ dst) {
  const int64_t n4 = n / 4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x)
    reinterpret_cast<float4*>(dst)[i] = load_grad4(nullptr, slabs, nslabs, n, i);
}

// 8 outputs per thread (one 16-byte store): thread t = (row t / (cout / 8), chunk t % (cout / 8)), so
// consecutive threads read consecutive 32-byte runs of a row and write consecutive 16-byte runs (the
// element-per-thread form below did an integer division per element)
__global__ __launch_bounds__(256) void cast_pad8_kernel(const float* __restrict__ in, int rows, int cin, int ldin,
                                                        bf16_t* __restrict__ out, int cout) {
  const int cpr = cout / 8;
  const int64_t n = (int64_t)rows * cpr;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += (int64_t)gridDim.x * blockDim.x) {
    const int r = (int)(t / cpr), c0 = (int)(t - (int64_t)r * cpr) * 8;
    const float* p = in + (size_t)r * ldin;
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = c0 + 2 * i;
      const float a = c < cin ? p[c] : 0.f, b = c + 1 < cin ? p[c + 1] : 0.f;
      w[i] = (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16);
    }
    *reinterpret_cast<uint4*>(out + (size_t)r * cout + c0) = make_uint4(w[0], w[1], w[2], w[3]);
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

// ---- gradient reduction + Adam (one kernel, shared by every world size) ----
// Sources of the flat gradient: up to 8 disjoint, 4-aligned regions [start, start + len), each
// the sum of S slabs (slab s at src + s * lds).  Modes (bit set):
//   GR_REDUCE  g = sum of the region's slabs (fixed order)    else g = G[i] (already reduced)
//   GR_STORE   G[i] = g                                         (DP: before the all-reduce)
//   GR_ADAM    Adam update of param / m / v / bf16 copy with t = *step (ticked earlier in the step
//              by the fused backward kernel or adam_tick_kernel: no kernel both ticks and reads it)
//   GR_REFRESH (alone) the bf16 copy and the fragment copies from param, no update: the sharded DP
//              step after its all-gather of the fp32 parameters (one launch instead of a torch cast +
//              the pack kernel)
// A workgroup = GR_W (4 by default; 8 / 16 by HAR_GR_W) waves x 64 float4 columns: wave q sums slabs
// q, q + GR_W, q + 2 GR_W, ... (eight loads in flight per step), the GR_W partials are added in a
// fixed tree order -> bitwise reproducible, and N = 1 (GR_REDUCE |
// GR_ADAM) and N > 1 (GR_REDUCE | GR_STORE, all-reduce, GR_ADAM) apply the same summation and the
// same Adam arithmetic.  With fragment copies (MlpFragSpec) the new bf16 values also go to the W0 and
// W1 fragment copies (8-byte runs); the W1^T copy is written by the step's forward kernel, which
// holds W1 in registers anyway (a tiled transposing variant of this kernel measured 1.5 us slower).
// Prefetch workgroups (PrefetchSpec: blocks main_blocks .. of the launch): the NEXT step's input rows read
// once per 64-byte line while the reduction runs, so the next forward stages them from the memory-side
// cache instead of HBM — an epoch over more rows than that cache holds (the 1.3 GB of rows of the
// 1B-sample pass) lost ~5 us per step in the forward; with the prefetch ~2 (profiles/r6/mlp_cold_x_probe.txt;
// a separate prefetch kernel on a side stream beside the backward cost ~6 us per step instead).  Reads
// only: the loaded words are folded into one value stored to a scratch word under a data-dependent test,
// so every thread's loads stay.
struct PrefetchSpec {
  const uint32_t* p;   // region 0 (the rows) ...
  int64_t lines;       // ... in lines of `dw` dwords (64 bytes; HAR_PF_LINE)
  int dw;
  const uint32_t* p1;  // region 1 (the labels), its lines follow region 0's
  int64_t lines1;
  uint32_t* sink;
  int main_blocks;
};

constexpr int GR_REDUCE = 1, GR_STORE = 2, GR_ADAM = 4, GR_REFRESH = 8;
template <int GR_W>  // waves per workgroup
__global__ __launch_bounds__(64 * GR_W) void grad_reduce_adam_kernel(GradRegions rg, int64_t n, float* __restrict__ G,
                                                                float* __restrict__ param, float* __restrict__ m,
                                                                float* __restrict__ v, bf16_t* __restrict__ pb,
                                                                float lr, float b1, float b2, float eps, float wd,
                                                                const int32_t* __restrict__ step, int mode,
                                                                MlpFragSpec frag, int wide, PrefetchSpec pf) {
  if ((int)blockIdx.x >= pf.main_blocks) {  // a prefetch workgroup (uniform per block)
    const int64_t nt = (int64_t)(gridDim.x - pf.main_blocks) * blockDim.x;
    const int64_t t0 = (int64_t)(blockIdx.x - pf.main_blocks) * blockDim.x + threadIdx.x;
    uint32_t acc = 0;
    const int64_t all = pf.lines + pf.lines1;
    for (int64_t l = t0; l < all; l += 8 * nt) {
      uint32_t x[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {  // 8 loads in flight
        const int64_t q = min(l + j * nt, all - 1);
        x[j] = q < pf.lines ? pf.p[q * pf.dw] : pf.p1[(q - pf.lines) * pf.dw];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) acc += x[j];
    }
    if (t0 == 0 || acc == 0x9e3779b9u) *pf.sink = acc;
    return;
  }
  __shared__ float4 part[GR_W][64];
  const int q = threadIdx.x >> 6, k = threadIdx.x & 63;
  const int64_t i4 = (int64_t)blockIdx.x * 64 + k, e = i4 * 4;
  if (mode == GR_REFRESH) {
    if (q == 0 && e < n) {
      const float4 pp = reinterpret_cast<const float4*>(param)[i4];
      const ushort4 ob = make_ushort4(f2bf(pp.x), f2bf(pp.y), f2bf(pp.z), f2bf(pp.w));
      reinterpret_cast<ushort4*>(pb)[i4] = ob;
      if (frag.dst) {
        if (frag.w1t) frag_store4<true>(frag, e, ob);
        else frag_store4<false>(frag, e, ob);
      }
    }
    return;
  }
  // the Adam operands do not depend on the reduction: wave 0 issues their loads first, so their
  // latency overlaps the slab loads instead of following them
  const bool do_adam = q == 0 && e < n && (mode & GR_ADAM);
  float4 pp = make_float4(0.f, 0.f, 0.f, 0.f), mm = pp, vv = pp;
  int32_t t_int = 0;
  if (do_adam) {
    pp = reinterpret_cast<const float4*>(param)[i4];
    mm = reinterpret_cast<const float4*>(m)[i4];
    vv = reinterpret_cast<const float4*>(v)[i4];
    t_int = *step;
  }
  if (mode & GR_REDUCE) {
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    if (e < n) {
      for (int r = 0; r < rg.nreg; ++r) {
        if (e < rg.start[r] || e >= rg.start[r] + rg.len[r]) continue;
        const float* p = rg.src[r] + (e - rg.start[r]);
        const int S = rg.S[r];
        const int64_t ld = rg.lds[r];
        int s = q;
        if (wide) {  // 16 loads in flight per step (HAR_GR_NL=16)
          for (; s + 15 * GR_W < S; s += 16 * GR_W) {
            float4 x[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) x[j] = *reinterpret_cast<const float4*>(p + (size_t)(s + j * GR_W) * ld);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              x[j].x += x[j + 8].x; x[j].y += x[j + 8].y; x[j].z += x[j + 8].z; x[j].w += x[j + 8].w;
            }
            acc.x += ((x[0].x + x[1].x) + (x[2].x + x[3].x)) + ((x[4].x + x[5].x) + (x[6].x + x[7].x));
            acc.y += ((x[0].y + x[1].y) + (x[2].y + x[3].y)) + ((x[4].y + x[5].y) + (x[6].y + x[7].y));
            acc.z += ((x[0].z + x[1].z) + (x[2].z + x[3].z)) + ((x[4].z + x[5].z) + (x[6].z + x[7].z));
            acc.w += ((x[0].w + x[1].w) + (x[2].w + x[3].w)) + ((x[4].w + x[5].w) + (x[6].w + x[7].w));
          }
        }
        for (; s + 7 * GR_W < S; s += 8 * GR_W) {
          float4 x[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) x[j] = *reinterpret_cast<const float4*>(p + (size_t)(s + j * GR_W) * ld);
          acc.x += ((x[0].x + x[1].x) + (x[2].x + x[3].x)) + ((x[4].x + x[5].x) + (x[6].x + x[7].x));
          acc.y += ((x[0].y + x[1].y) + (x[2].y + x[3].y)) + ((x[4].y + x[5].y) + (x[6].y + x[7].y));
          acc.z += ((x[0].z + x[1].z) + (x[2].z + x[3].z)) + ((x[4].z + x[5].z) + (x[6].z + x[7].z));
          acc.w += ((x[0].w + x[1].w) + (x[2].w + x[3].w)) + ((x[4].w + x[5].w) + (x[6].w + x[7].w));
        }
        for (; s + 3 * GR_W < S; s += 4 * GR_W) {
          float4 x[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) x[j] = *reinterpret_cast<const float4*>(p + (size_t)(s + j * GR_W) * ld);
          acc.x += (x[0].x + x[1].x) + (x[2].x + x[3].x);
          acc.y += (x[0].y + x[1].y) + (x[2].y + x[3].y);
          acc.z += (x[0].z + x[1].z) + (x[2].z + x[3].z);
          acc.w += (x[0].w + x[1].w) + (x[2].w + x[3].w);
        }
        for (; s < S; s += GR_W) {
          const float4 x = *reinterpret_cast<const float4*>(p + (size_t)s * ld);
          acc.x += x.x; acc.y += x.y; acc.z += x.z; acc.w += x.w;
        }
      }
    }
    part[q][k] = acc;
    __syncthreads();
    if (GR_W == 16 && q < 4) {  // 16 -> 4 partials (fixed pairs)
      const float4 a = part[q][k], b = part[q + 4][k], c = part[q + 8][k], d = part[q + 12][k];
      part[q][k] = make_float4((a.x + b.x) + (c.x + d.x), (a.y + b.y) + (c.y + d.y), (a.z + b.z) + (c.z + d.z),
                               (a.w + b.w) + (c.w + d.w));
    }
    if (GR_W == 8 && q < 4) {
      const float4 a = part[q][k], b = part[q + 4][k];
      part[q][k] = make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
    }
    if (GR_W > 4) __syncthreads();
  }
  if (q == 0 && e < n) {
    float4 g;
    if (mode & GR_REDUCE) {
      const float4 a = part[0][k], b = part[1][k], c = part[2][k], d = part[3][k];
      g = make_float4((a.x + b.x) + (c.x + d.x), (a.y + b.y) + (c.y + d.y), (a.z + b.z) + (c.z + d.z),
                      (a.w + b.w) + (c.w + d.w));
    } else {
      g = reinterpret_cast<const float4*>(G)[i4];
    }
    if (mode & GR_STORE) reinterpret_cast<float4*>(G)[i4] = g;
    if (do_adam) {
      const float t = (float)t_int;
      const float bc1 = 1.f - powf(b1, t), bc2 = 1.f - powf(b2, t);
      float* pa = &pp.x; float* ma = &mm.x; float* va = &vv.x; const float* ga = &g.x;
      ushort4 ob;
      unsigned short* oa = &ob.x;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        ma[j] = b1 * ma[j] + (1.f - b1) * ga[j];
        va[j] = b2 * va[j] + (1.f - b2) * ga[j] * ga[j];
        const float upd = (ma[j] / bc1) / (sqrtf(va[j] / bc2) + eps);
        pa[j] = pa[j] - lr * (upd + wd * pa[j]);
        oa[j] = f2bf(pa[j]);
      }
      reinterpret_cast<float4*>(param)[i4] = pp;
      reinterpret_cast<float4*>(m)[i4] = mm;
      reinterpret_cast<float4*>(v)[i4] = vv;
      reinterpret_cast<ushort4*>(pb)[i4] = ob;
      if (frag.dst) {
        if (frag.w1t) frag_store4<true>(frag, e, ob);
        else frag_store4<false>(frag, e, ob);
      }
    }
  }
}

int grid_for(int64_t n4) { return (int)std::max<int64_t>(1, std::min<int64_t>(2048, (n4 + 255) / 256)); }

}  // namespace

extern "C" int har_softmax_ce_head_blocks(int B) {
  return (int)(((int64_t)B + HEAD_ROWS_PER_BLOCK - 1) / HEAD_ROWS_PER_BLOCK);
}

extern "C" int har_softmax_ce_head(const uint16_t* H, const uint16_t* W, const float* bias, const int32_t* labels,
                                   int B, int D, int C, float scale, uint16_t* dlogits, float* block_loss,
                                   int32_t* block_correct, float* logits_out, hipStream_t s) {
  if (C > 32 || D % 32) return -2;
  int blocks = har_softmax_ce_head_blocks(B);
  if (blocks == 0) return 0;
  softmax_ce_head_kernel<<<blocks, 256, 0, s>>>(H, W, bias, labels, B, D, C, scale, dlogits, block_loss,
                                                block_correct, logits_out);
  HAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int har_adam_step(float* param, const float* grad, const float* slabs, int nslabs, float* m, float* v,
                             uint16_t* pb, int64_t n, float lr, float b1, float b2, float eps, float wd, float gs,
                             int32_t* step, int tick, hipStream_t s) {
  if (n % 4) return -2;
  if (tick) adam_tick_kernel<<<1, 1, 0, s>>>(step);
  adam_kernel<<<grid_for(n / 4), 256, 0, s>>>(param, grad, slabs, nslabs, m, v, pb, n, lr, b1, b2, eps, wd, gs,
                                              step);
  HAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int har_reduce_slabs(const float* slabs, int nslabs, int64_t n, float* dst, hipStream_t s) {
  if (n % 4) return -2;
  reduce_slabs_kernel<<<grid_for(n / 4), 256, 0, s>>>(slabs, nslabs, n, dst);
  HAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int har_cast_pad_bf16(const float* in, int rows, int cin, int ldin, uint16_t* out, int cout,
                                 hipStream_t s) {
  int64_t total = (int64_t)rows * cout;
  if (cout % 8 == 0 && (reinterpret_cast<uintptr_t>(out) & 15) == 0) {
    const int64_t n8 = total / 8;
    const int blocks = (int)std::min<int64_t>(8192, (n8 + 255) / 256);
    if (blocks == 0) return 0;
    cast_pad8_kernel<<<blocks, 256, 0, s>>>(in, rows, cin, ldin, reinterpret_cast<bf16_t*>(out), cout);
    HAR_CHECK_LAUNCH();
    return 0;
  }
  int blocks = (int)std::min<int64_t>(4096, (total + 255) / 256);
  if (blocks == 0) return 0;
  cast_pad_kernel<<<blocks, 256, 0, s>>>(in, rows, cin, ldin, out, cout);
  HAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int har_grad_reduce_adam(int nreg, const float* const* src, const int64_t* start, const int64_t* len,
                                    const int64_t* lds, const int* S, int64_t n, float* G, float* param, float* m,
                                    float* v, uint16_t* pb, float lr, float b1, float b2, float eps, float wd,
                                    int32_t* step, int tick, int mode, const MlpFragSpec* frag_spec,
                                    hipStream_t s, const void* pf, int64_t pf_bytes, uint32_t* pf_sink,
                                    const void* pf1, int64_t pf1_bytes) {
  if (n % 4 || nreg < 0 || nreg > 8 || ((mode & GR_REDUCE) && nreg == 0)) return -2;
  if (pf && (!pf_sink || pf_bytes < 0 || (reinterpret_cast<uintptr_t>(pf) & 3))) return -2;
  if (pf1 && (!pf || pf1_bytes < 0 || (reinterpret_cast<uintptr_t>(pf1) & 3))) return -2;
  if ((mode & GR_REFRESH) && mode != GR_REFRESH) return -2;  // the refresh runs alone
  MlpFragSpec frag{};
  if (frag_spec && frag_spec->dst) {
    frag = *frag_spec;
    if (frag.H % 32 || frag.K0 % 32 || frag.w0_off % 4 || frag.w1_off % 4 || (reinterpret_cast<uintptr_t>(frag.dst) & 7) ||
        frag.w0_off + (int64_t)frag.H * frag.K0 > n || frag.w1_off + (int64_t)frag.H * frag.H > n)
      return -2;
  }
  GradRegions rg{};
  rg.nreg = nreg;
  for (int r = 0; r < nreg; ++r) {
    if (start[r] % 4 || len[r] % 4 || lds[r] % 4 || S[r] <= 0 || start[r] < 0 || start[r] + len[r] > n) return -2;
    if (reinterpret_cast<uintptr_t>(src[r]) & 15) return -3;
    if (r > 0 && start[r] < start[r - 1] + len[r - 1]) return -2;  // sorted, disjoint
    rg.src[r] = src[r]; rg.start[r] = start[r]; rg.len[r] = len[r]; rg.lds[r] = lds[r]; rg.S[r] = S[r];
  }
  const int64_t blocks = (n / 4 + 63) / 64;
  if (blocks == 0) return 0;
  if (tick) adam_tick_kernel<<<1, 1, 0, s>>>(step);
  // prefetch workgroups: one per 2048 lines (8 loads per thread), at most 256
  static const int pf_line = [] {  // bytes per touched line (tuning: HAR_PF_LINE = 64 / 128 / 256)
    const char* e = getenv("HAR_PF_LINE");
    const int v = e ? atoi(e) : 64;
    return v == 128 || v == 256 ? v : 64;
  }();
  PrefetchSpec ps{reinterpret_cast<const uint32_t*>(pf), pf ? pf_bytes / pf_line : 0, pf_line / 4,
                  reinterpret_cast<const uint32_t*>(pf1), pf && pf1 ? pf1_bytes / pf_line : 0, pf_sink, (int)blocks};
  const int64_t pfl = ps.lines + ps.lines1;
  const int64_t pfb = pf && pfl > 0 ? std::min<int64_t>(256, (pfl + 2047) / 2048) : 0;
  const int64_t grid = blocks + pfb;
  // waves per workgroup: 4 (tools/gpu_qnwg_ab.sh a: flagship reduction + Adam 6.6 -> 4.9 us with 64 slabs,
  // the small-batch step 21.7 -> 20.8 us with 8; 8 waves 5.4 / 20.9; 16 was the round-3 choice)
  static const int w = [] {
    const char* e = getenv("HAR_GR_W");
    return e ? atoi(e) : 4;
  }();
  static const int wide = [] {
    const char* e = getenv("HAR_GR_NL");
    return e && atoi(e) == 16 ? 1 : 0;
  }();
  if (w == 4)
    grad_reduce_adam_kernel<4><<<(int)grid, 256, 0, s>>>(rg, n, G, param, m, v, pb, lr, b1, b2, eps, wd, step, mode,
                                                         frag, wide, ps);
  else if (w == 8)
    grad_reduce_adam_kernel<8><<<(int)grid, 512, 0, s>>>(rg, n, G, param, m, v, pb, lr, b1, b2, eps, wd, step, mode,
                                                         frag, wide, ps);
  else
    grad_reduce_adam_kernel<16><<<(int)grid, 1024, 0, s>>>(rg, n, G, param, m, v, pb, lr, b1, b2, eps, wd, step,
                                                           mode, frag, wide, ps);
  HAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int har_mlp_pack_frag(const uint16_t* pb, const MlpFragSpec* f, hipStream_t s) {
  if (!f || !f->dst || f->H % 32 || f->K0 % 32 || f->w0_off % 4 || f->w1_off % 4 ||
      (reinterpret_cast<uintptr_t>(f->dst) & 7) || (reinterpret_cast<uintptr_t>(pb) & 7))
    return -2;
  const int64_t n4 = ((int64_t)f->H * f->K0 + (int64_t)f->H * f->H) / 4;
  mlp_pack_frag_kernel<<<(int)std::min<int64_t>(1024, (n4 + 255) / 256), 256, 0, s>>>(pb, *f);
  HAR_CHECK_LAUNCH();
  return 0;
}
