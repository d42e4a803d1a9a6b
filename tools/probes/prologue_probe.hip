// Weight-prologue probe: how fast can 256 workgroups (one per CU, 512 threads) each pull the SAME
// ~168 KB of bf16 weights (the MLP step forward's W0 + W1 + Wout) on chip?  Variants:
//   0  fragment-shaped register loads (the mlp_fwd3 prologue: per lane 16-byte pieces of 16 rows)
//   1  row-contiguous register loads (each wave-instruction reads 1 KB contiguous)
//   2  LDS-DMA (global_load_lds_dwordx4) of the whole W1 into LDS, 1 KB per wave-instruction
//   3  variant 0 with a "dirtying" writer kernel before every launch (the Adam kernel rewrites Pb)
// Per wave: s_memtime at entry and after the data has arrived; median / max over waves, plus the
// event time per launch.  Build: hipcc --offload-arch=gfx950 -O3 -o prologue_probe prologue_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;
constexpr int H = 256, K0 = 64, NW = 8;
constexpr size_t W0_E = (size_t)H * K0, W1_E = (size_t)H * H, WO_E = (size_t)16 * H;
constexpr size_t TOT_E = W0_E + W1_E + WO_E;

__global__ void dirty_kernel(uint16_t* w, size_t n, int salt) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    w[i] = (uint16_t)(i * 2654435761u + salt);
}

template <int V>
__global__ __launch_bounds__(512) void probe_kernel(const uint16_t* __restrict__ W, uint32_t* __restrict__ out,
                                                    uint64_t* __restrict__ stamps) {
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, c16 = lane & 15, g = lane >> 4;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  const uint16_t* W0 = W;
  const uint16_t* W1 = W + W0_E;
  const uint16_t* Wo = W1 + W1_E;
  uint32_t acc = 0;
  if constexpr (V == 0 || V == 3) {
    const int u0 = wave * 32;
    u32x4 w0f[2][2], w1f[2][8];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int kc = 0; kc < 2; ++kc)
        w0f[t][kc] = *reinterpret_cast<const u32x4*>(W0 + (size_t)(u0 + 16 * t + c16) * K0 + kc * 32 + g * 8);
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int kc = 0; kc < 8; ++kc)
        w1f[t][kc] = *reinterpret_cast<const u32x4*>(W1 + (size_t)(u0 + 16 * t + c16) * H + kc * 32 + g * 8);
    const uint2 wlo = *reinterpret_cast<const uint2*>(Wo + (size_t)c16 * H + u0 + 4 * g);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
      for (int kc = 0; kc < 2; ++kc) acc ^= w0f[t][kc].x ^ w0f[t][kc].w;
#pragma unroll
      for (int kc = 0; kc < 8; ++kc) acc ^= w1f[t][kc].x ^ w1f[t][kc].w;
    }
    acc ^= wlo.x;
  } else if constexpr (V == 1) {
    // the same bytes per wave, but each wave-instruction reads 1 KB contiguous: wave w reads rows
    // [32w, 32w + 32) of W1 (16 KB) as 16 instructions of 64 lanes x 16 B
    u32x4 r[16];
#pragma unroll
    for (int i = 0; i < 16; ++i)
      r[i] = *reinterpret_cast<const u32x4*>(W1 + (size_t)wave * 32 * H + (size_t)i * 512 + lane * 8);
    u32x4 q[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) q[i] = *reinterpret_cast<const u32x4*>(W0 + (size_t)wave * 32 * K0 + (size_t)i * 512 + lane * 8);
    const u32x4 o = *reinterpret_cast<const u32x4*>(Wo + (size_t)wave * 512 + lane * 8);
#pragma unroll
    for (int i = 0; i < 16; ++i) acc ^= r[i].x ^ r[i].w;
#pragma unroll
    for (int i = 0; i < 4; ++i) acc ^= q[i].x ^ q[i].w;
    acc ^= o.x;
  } else {
    // LDS-DMA of the whole 168 KB? LDS holds 160 KB: W1 (128 KB) + W0 (32 KB); Wout to registers
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const size_t e = ((size_t)(i * NW + wave) * 64 + lane) * 8;  // wave-instruction = 1 KB
      __builtin_amdgcn_global_load_lds(W1 + e, lds + (size_t)(i * NW + wave) * 512, 16, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const size_t e = ((size_t)(i * NW + wave) * 64 + lane) * 8;
      __builtin_amdgcn_global_load_lds(W0 + e, lds + W1_E + (size_t)(i * NW + wave) * 512, 16, 0, 0);
    }
    const uint2 wlo = *reinterpret_cast<const uint2*>(Wo + (size_t)c16 * H + wave * 32 + 4 * g);
    __builtin_amdgcn_s_waitcnt(0x0f70);
    __syncthreads();
    acc ^= *reinterpret_cast<const uint32_t*>(lds + (size_t)tid * 8) ^ wlo.x;
  }
  __builtin_amdgcn_s_waitcnt(0x0f70);
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) {
    stamps[((size_t)blockIdx.x * NW + wave) * 2] = t0;
    stamps[((size_t)blockIdx.x * NW + wave) * 2 + 1] = t1;
  }
  if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

template <int V>
void run(const char* name, uint16_t* W, uint32_t* out, uint64_t* st, int nwg, bool dirty) {
  const size_t lds = V == 2 ? (W1_E + W0_E) * 2 : 0;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  std::vector<double> cyc;
  float ms_sum = 0.f;
  const int reps = 50;
  for (int r = 0; r < reps + 5; ++r) {
    if (dirty) dirty_kernel<<<1024, 256>>>(W, TOT_E, r);
    CK(hipEventRecord(a));
    probe_kernel<V><<<nwg, 512, lds>>>(W, out, st);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    if (r >= 5) {
      ms_sum += ms;
      std::vector<uint64_t> h((size_t)nwg * NW * 2);
      CK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
      for (size_t i = 0; i < (size_t)nwg * NW; ++i) cyc.push_back((double)(h[2 * i + 1] - h[2 * i]));
    }
  }
  std::sort(cyc.begin(), cyc.end());
  printf("%-34s nwg %4d dirty %d: wave cycles median %7.0f p90 %7.0f max %7.0f | event %.2f us\n", name, nwg,
         (int)dirty, cyc[cyc.size() / 2], cyc[cyc.size() * 9 / 10], cyc.back(), 1e3 * ms_sum / reps);
}

int main() {
  uint16_t* W;
  uint32_t* out;
  uint64_t* st;
  CK(hipMalloc(&W, TOT_E * 2));
  CK(hipMalloc(&out, 4096 * 4));
  CK(hipMalloc(&st, 4096 * NW * 2 * 8));
  dirty_kernel<<<1024, 256>>>(W, TOT_E, 7);
  CK(hipFuncSetAttribute((const void*)probe_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  CK(hipDeviceSynchronize());
  for (int dirty = 0; dirty < 2; ++dirty) {
    for (int nwg : {256, 128, 32}) {
      run<0>("frag-shaped regs (mlp_fwd3)", W, out, st, nwg, dirty);
      run<1>("row-contiguous regs", W, out, st, nwg, dirty);
      run<2>("LDS-DMA W1+W0 -> LDS", W, out, st, nwg, dirty);
    }
  }
  CK(hipDeviceSynchronize());
  printf("done\n");
  return 0;
}
