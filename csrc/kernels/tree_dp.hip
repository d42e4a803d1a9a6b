// Data-parallel forest level: the wire format of the per-node histogram store.
//
// A DP level sums every rank's per-node histograms [A][m][bins][K] (fp32, integer-valued: bootstrap x
// fold weights) before the split search.  Every rank already knows each candidate node's GLOBAL class
// counts (the previous level's winners carry them; the roots' are all-reduced), so the store travels
// as packed integers:
//   * only the classes PRESENT in the node (a class with zero weight in the node has an all-zero
//     histogram on every rank): a deep node of a 12-class forest holds two or three classes;
//   * each count in the narrowest field its node's total weight w allows, several fields per 32-bit
//     word: 8 bits when w < 2^8, 16 bits when w < 2^16, else 32.  The integer SUM of packed words over
//     the ranks is then exact field by field — every field's sum is <= w, so no carry crosses a field.
// The host assigns nodes to owner ranks by contiguous word-balanced ranges; rank r's nodes fill row r
// of a [P][Wmax] int32 buffer (reduce-scattered), and the owner unpacks its summed row back into an
// fp32 [n][m][bins][K] store (absent classes zero) for the unchanged split kernel.
//
// Reference: Main/main.py:478-481 (RandomForestClassifier.fit: Spark ships per-node aggregates of the
// node group in reduceByKey); SURVEY.md M9 / §7.5.3 (narrow counts).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../har_kernels.h"
#include "common.h"

namespace {

// one workgroup per node: word w of node a packs counts i = w * per .. + per - 1 of the node's
// sequence (fb, j) -> store[a][fb][cls[a][j]], fb = feature x bin, j = present class
__global__ __launch_bounds__(256) void dp_pack_kernel(const float* __restrict__ store, int64_t slot, int mb, int K,
                                                      const int32_t* __restrict__ cls, const int32_t* __restrict__ kp,
                                                      const int32_t* __restrict__ bw, const int64_t* __restrict__ woff,
                                                      int32_t* __restrict__ out) {
  const int a = blockIdx.x;
  const int kpa = kp[a], b = bw[a], per = 4 / b, sh = 8 * b;
  const int64_t n = (int64_t)mb * kpa, nw = (n + per - 1) / per;
  const float* src = store + (int64_t)a * slot;
  const int32_t* ca = cls + (int64_t)a * K;
  int32_t* dst = out + woff[a];
  for (int64_t w = threadIdx.x; w < nw; w += blockDim.x) {
    uint32_t word = 0;
    for (int e = 0; e < per; ++e) {
      const int64_t i = w * per + e;
      if (i < n) {
        const int64_t fb = i / kpa;
        const int j = (int)(i - fb * kpa);
        const uint32_t v = (uint32_t)__float2uint_rn(src[fb * K + ca[j]]);
        word |= b == 4 ? v : (v << (sh * e));
      }
    }
    dst[w] = (int32_t)word;
  }
}

// one workgroup per owned node a0 + blockIdx.x: the summed words -> fp32 [mb][K] (absent classes 0)
__global__ __launch_bounds__(256) void dp_unpack_kernel(const int32_t* __restrict__ in, int a0, int64_t slot, int mb,
                                                        int K, const int32_t* __restrict__ cls,
                                                        const int32_t* __restrict__ kp, const int32_t* __restrict__ bw,
                                                        const int64_t* __restrict__ woff, int64_t base,
                                                        float* __restrict__ local) {
  const int a = a0 + blockIdx.x;
  const int kpa = kp[a], b = bw[a], per = 4 / b, sh = 8 * b;
  const uint32_t fmask = b == 4 ? 0xffffffffu : ((1u << sh) - 1u);
  const int32_t* src = in + (woff[a] - base);
  const int32_t* ca = cls + (int64_t)a * K;
  float* dst = local + (int64_t)blockIdx.x * slot;
  for (int64_t e = threadIdx.x; e < slot; e += blockDim.x) {  // the absent classes' slots
    const int k = (int)(e % K);
    bool present = false;
    for (int j = 0; j < kpa; ++j) present |= ca[j] == k;
    if (!present) dst[e] = 0.f;
  }
  const int64_t n = (int64_t)mb * kpa;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
    const uint32_t word = (uint32_t)src[i / per];
    const uint32_t v = b == 4 ? word : ((word >> (sh * (int)(i % per))) & fmask);
    const int64_t fb = i / kpa;
    dst[fb * K + ca[i - fb * kpa]] = (float)v;
  }
}

}  // namespace

extern "C" int har_tree_dp_pack(const float* store, int A, int64_t slot, int mb, int K, const int32_t* cls,
                                const int32_t* kp, const int32_t* bw, const int64_t* woff, int32_t* out,
                                hipStream_t s) {
  if (A < 0 || K < 1 || mb < 1 || slot != (int64_t)mb * K || A > 0x7fffffff) return -2;
  if (A == 0) return 0;
  dp_pack_kernel<<<A, 256, 0, s>>>(store, slot, mb, K, cls, kp, bw, woff, out);
  HAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int har_tree_dp_unpack(const int32_t* in, int a0, int n, int64_t slot, int mb, int K, const int32_t* cls,
                                  const int32_t* kp, const int32_t* bw, const int64_t* woff, int64_t base,
                                  float* local, hipStream_t s) {
  if (n < 0 || a0 < 0 || K < 1 || mb < 1 || slot != (int64_t)mb * K) return -2;
  if (n == 0) return 0;
  dp_unpack_kernel<<<n, 256, 0, s>>>(in, a0, slot, mb, K, cls, kp, bw, woff, base, local);
  HAR_CHECK_LAUNCH();
  return 0;
}
