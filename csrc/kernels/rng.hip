// Philox bucket assignment (train/test split, k-fold ids) keyed by global row id
// (SURVEY.md K7): out[r] = #{b : thr[b] <= u32(seed, stream, row0 + r)}.
#include "common.h"
#include "philox.h"
#include "../har_kernels.h"

namespace {

__global__ __launch_bounds__(256) void philox_buckets_kernel(uint64_t seed, uint32_t stream, int64_t row0, int64_t n,
                                                             const uint32_t* __restrict__ thr, int nthr,
                                                             int32_t* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t u = philox_u32(seed, stream, (uint64_t)(row0 + i));
    int b = 0;
    while (b < nthr && thr[b] <= u) ++b;
    out[i] = b;
  }
}

}  // namespace

extern "C" int har_philox_buckets(uint64_t seed, uint32_t stream, int64_t row0, int64_t n, const uint32_t* thr,
                                  int nthr, int32_t* out, hipStream_t s) {
  if (n < 0 || nthr < 0) return -2;
  if (n == 0) return 0;
  int blocks = (int)std::min<int64_t>(4096, (n + 255) / 256);
  philox_buckets_kernel<<<blocks, 256, 0, s>>>(seed, stream, row0, n, thr, nthr, out);
  HAR_CHECK_LAUNCH();
  return 0;
}
