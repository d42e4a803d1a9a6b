// Fused softmax + cross-entropy + residual for B logistic-regression models
// sharing one margin matrix Z [N][ld] (columns b*K .. b*K+K-1 belong to model b).
//
//   R[i][b*K+c] = rw[b][i] * inv_wsum[b] * (softmax(Z_ib)[c] - [c == y_i])
//   loss[b]    += rw[b][i] * inv_wsum[b] * (logsumexp(Z_ib) - Z_ib[y_i])
//
// One lane per row, a wave walks all B models of its 64 rows; per-model losses
// are wave-reduced before one double atomic per wave and model.  Columns
// >= B*K of R are written as zeros (so the following split-K GEMM can run over
// the padded width).  Memory-bound: Z is read once, R written once.
#include "common.h"
#include "../har_kernels.h"

namespace {

constexpr int MAXK = 64;

__global__ __launch_bounds__(256) void logreg_softmax_grad_kernel(const float* __restrict__ Z, int64_t n, int B,
                                                                  int K, int ld, const int32_t* __restrict__ y,
                                                                  const float* __restrict__ rw,
                                                                  const float* __restrict__ inv_wsum,
                                                                  float* __restrict__ R, double* __restrict__ loss) {
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool ok = i < n;
  const int yi = ok ? y[i] : 0;
  const float* zrow = Z + (ok ? i : 0) * (int64_t)ld;
  float* rrow = R + (ok ? i : 0) * (int64_t)ld;
  for (int b = 0; b < B; ++b) {
    float l = 0.f;
    if (ok) {
      const float w = rw[(int64_t)b * n + i] * inv_wsum[b];
      const float* z = zrow + b * K;
      float mx = -INFINITY;
      for (int c = 0; c < K; ++c) mx = fmaxf(mx, z[c]);
      float se = 0.f;
      for (int c = 0; c < K; ++c) se += __expf(z[c] - mx);
      const float inv = 1.f / se;
      for (int c = 0; c < K; ++c) {
        float pc = __expf(z[c] - mx) * inv;
        rrow[b * K + c] = w * (pc - (c == yi ? 1.f : 0.f));
      }
      l = (w != 0.f) ? w * ((mx + __logf(se)) - z[yi]) : 0.f;
    }
    double lw = wave_sum_d((double)l);
    if (lane == 0) atomicAdd(loss + b, lw);
  }
  if (ok)
    for (int c = B * K; c < ld; ++c) rrow[c] = 0.f;
}

}  // namespace

extern "C" int har_logreg_softmax_grad(const float* Z, int64_t n, int nmodels, int K, int ld, const int32_t* y,
                                       const float* rw, const float* inv_wsum, float* R, double* loss,
                                       hipStream_t s) {
  if (K > MAXK || nmodels * K > ld) return -2;
  if (n == 0) return 0;
  int blocks = (int)((n + 255) / 256);
  logreg_softmax_grad_kernel<<<blocks, 256, 0, s>>>(Z, n, nmodels, K, ld, y, rw, inv_wsum, R, loss);
  HAR_CHECK_LAUNCH();
  return 0;
}
