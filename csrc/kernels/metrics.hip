// Evaluation reductions: confusion matrix and regression
// moments; value_counts (K3/K5): counts of dictionary codes — StringIndexer's countByValue
// and groupBy().count() (Main/main.py:35-38, 55-61) on the device.  LDS-privatized counters per workgroup, one global atomic per
// counter per workgroup; fp64 accumulation for the moments.
#include "common.h"
#include "../har_kernels.h"

namespace {

constexpr int MAXK2 = 64 * 64;

__global__ __launch_bounds__(256) void confusion_kernel(const int32_t* __restrict__ label,
                                                        const int32_t* __restrict__ pred, int64_t n, int K,
                                                        unsigned long long* __restrict__ cm) {
  __shared__ unsigned int h[MAXK2];
  const int KK = K * K;
  for (int i = threadIdx.x; i < KK; i += blockDim.x) h[i] = 0;
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    atomicAdd(&h[label[i] * K + pred[i]], 1u);
  __syncthreads();
  for (int i = threadIdx.x; i < KK; i += blockDim.x)
    if (h[i]) atomicAdd(cm + i, (unsigned long long)h[i]);
}

// codes in [0, V) (others ignored: -1 = null); LDS-privatized 32-bit counters, one 64-bit global
// atomic per non-zero counter per workgroup (integer adds: order-independent, exact)
// B models at once (CrossValidator scoring): cm[b] over the rows with mask[b][i] != 0; grid (row
// chunks, B).  Out-of-range labels / predictions are skipped (the host checks the ranges).
__global__ __launch_bounds__(256) void confusion_batched_kernel(const int32_t* __restrict__ label,
                                                                const int32_t* __restrict__ pred,
                                                                const uint8_t* __restrict__ mask, int64_t n, int K,
                                                                unsigned long long* __restrict__ cm) {
  __shared__ unsigned int h[MAXK2];
  const int KK = K * K, b = blockIdx.y;
  const int32_t* pb = pred + (size_t)b * n;
  const uint8_t* mb = mask + (size_t)b * n;
  for (int i = threadIdx.x; i < KK; i += blockDim.x) h[i] = 0;
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int l = label[i], p = pb[i];
    if (mb[i] && (unsigned)l < (unsigned)K && (unsigned)p < (unsigned)K) atomicAdd(&h[l * K + p], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < KK; i += blockDim.x)
    if (h[i]) atomicAdd(cm + (size_t)b * KK + i, (unsigned long long)h[i]);
}

__global__ __launch_bounds__(256) void value_counts_kernel(const int64_t* __restrict__ codes, int64_t n, int V,
                                                           unsigned long long* __restrict__ out) {
  extern __shared__ unsigned int hv[];
  for (int i = threadIdx.x; i < V; i += blockDim.x) hv[i] = 0;
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t c = codes[i];
    if (c >= 0 && c < V) atomicAdd(&hv[c], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < V; i += blockDim.x)
    if (hv[i]) atomicAdd(out + i, (unsigned long long)hv[i]);
}

__global__ __launch_bounds__(256) void moments_kernel(const float* __restrict__ y, const float* __restrict__ yh,
                                                      int64_t n, double* __restrict__ out) {
  double c = 0, se = 0, ae = 0, sy = 0, syy = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    double a = y[i], d = a - (double)yh[i];
    c += 1; se += d * d; ae += fabs(d); sy += a; syy += a * a;
  }
  __shared__ double red[5][4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  double v[5] = {c, se, ae, sy, syy};
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    double s = wave_sum_d(v[k]);
    if (lane == 0) red[k][w] = s;
  }
  __syncthreads();
  if (threadIdx.x < 5) {
    double s = 0;
    for (int j = 0; j < (int)(blockDim.x >> 6); ++j) s += red[threadIdx.x][j];
    atomicAdd(out + threadIdx.x, s);
  }
}

}  // namespace

extern "C" int har_confusion_matrix(const int32_t* label, const int32_t* pred, int64_t n, int K, int64_t* cm,
                                    hipStream_t s) {
  if (K <= 0 || (int64_t)K * K > MAXK2 || n < 0) return -2;
  if (n == 0) return 0;
  int blocks = (int)std::min<int64_t>(1024, (n + 255) / 256);
  confusion_kernel<<<blocks, 256, 0, s>>>(label, pred, n, K, reinterpret_cast<unsigned long long*>(cm));
  HAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int har_confusion_matrix_batched(const int32_t* label, const int32_t* pred, const uint8_t* mask, int64_t n,
                                            int B, int K, int64_t* cm, hipStream_t s) {
  if (K <= 0 || (int64_t)K * K > MAXK2 || n < 0 || B <= 0 || B > 65535) return -2;
  if (const hipError_t e = hipMemsetAsync(cm, 0, sizeof(int64_t) * (size_t)B * K * K, s); e != hipSuccess) return (int)e;
  if (n == 0) return 0;
  const int chunks = (int)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, std::max(1, 1024 / B)));
  confusion_batched_kernel<<<dim3(chunks, B), 256, 0, s>>>(label, pred, mask, n, K,
                                                             reinterpret_cast<unsigned long long*>(cm));
  HAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int har_regression_moments(const float* y, const float* yhat, int64_t n, double* out6, hipStream_t s) {
  if (n < 0) return -2;
  if (n == 0) return 0;
  int blocks = (int)std::min<int64_t>(1024, (n + 255) / 256);
  moments_kernel<<<blocks, 256, 0, s>>>(y, yhat, n, out6);
  HAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int har_value_counts(const int64_t* codes, int64_t n, int V, int64_t* out, hipStream_t s) {
  if (V <= 0 || V > 32768 || n < 0) return -2;  // LDS counters: <= 128 KB
  if (const hipError_t e = hipMemsetAsync(out, 0, sizeof(int64_t) * (size_t)V, s); e != hipSuccess) return (int)e;
  if (n == 0) return 0;
  const int blocks = (int)std::min<int64_t>(256, (n + 255) / 256);
  value_counts_kernel<<<blocks, 256, sizeof(unsigned int) * (size_t)V, s>>>(codes, n, V,
                                                                        reinterpret_cast<unsigned long long*>(out));
  HAR_CHECK_LAUNCH();
  return 0;
}
