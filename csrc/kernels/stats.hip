// Column statistics and tree binning.
//
// column_stats: count / sum / sum of squares / min / max of every column of a
//   row-major [n][ld] fp32 matrix with optional row weights, fp64 accumulation.
//   Lanes walk columns (coalesced row segments), workgroups own row ranges, and
//   per-workgroup partials land in a [blocks][5][ncols] buffer that one final
//   pass reduces (no same-address atomics) — Spark's describe() / summarizer.
// bin_features: uint8 bin id of every (feature, row) = number of thresholds
//   strictly below x (x <= thr[b] goes left at split b); output feature-major
//   [F][n] so a tree node's rows read one feature contiguously.
#include "common.h"
#include "../har_kernels.h"

namespace {

constexpr int ROWS_PER_BLOCK = 256;

// T = float (fp32 feature matrices) or double (the fp64 columns of the device CSV, for Spark's
// describe() digits).  center (optional, [ncols]): q accumulates (x - center)^2 — the second pass
// of a two-pass variance.
template <typename T>
__global__ __launch_bounds__(256) void column_stats_partial(const T* __restrict__ X, int64_t n, int ncols, int ld,
                                                            const float* __restrict__ w,
                                                            const double* __restrict__ center,
                                                            double* __restrict__ part) {
  const int64_t r0 = (int64_t)blockIdx.y * ROWS_PER_BLOCK;
  const int64_t r1 = min(n, r0 + ROWS_PER_BLOCK);
  for (int c = blockIdx.x * 256 + threadIdx.x; c < ncols; c += gridDim.x * 256) {
    double cnt = 0, s = 0, q = 0, mn = INFINITY, mx = -INFINITY;
    const double ctr = center ? center[c] : 0.0;
    for (int64_t r = r0; r < r1; ++r) {
      const double x = (double)X[r * ld + c];
      const double wr = w ? (double)w[r] : 1.0;
      if (wr != 0.0 && x == x) {
        const double d = x - ctr;
        cnt += wr; s += wr * x; q += wr * d * d;
        mn = fmin(mn, x); mx = fmax(mx, x);
      }
    }
    double* p = part + (size_t)blockIdx.y * 5 * ncols;
    p[c] = cnt; p[ncols + c] = s; p[2 * ncols + c] = q; p[3 * ncols + c] = mn; p[4 * ncols + c] = mx;
  }
}

__global__ __launch_bounds__(256) void column_stats_final(const double* __restrict__ part, int nblocks, int ncols,
                                                          double* __restrict__ stats) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= ncols) return;
  double cnt = 0, s = 0, q = 0, mn = INFINITY, mx = -INFINITY;
  for (int b = 0; b < nblocks; ++b) {
    const double* p = part + (size_t)b * 5 * ncols;
    cnt += p[c]; s += p[ncols + c]; q += p[2 * ncols + c];
    mn = fmin(mn, p[3 * ncols + c]); mx = fmax(mx, p[4 * ncols + c]);
  }
  stats[c] = cnt; stats[ncols + c] = s; stats[2 * ncols + c] = q; stats[3 * ncols + c] = mn; stats[4 * ncols + c] = mx;
}

// column-major fp64 planes [ncols][n]: workgroup (c, b) reduces rows [b*256, b*256+256) of column
// c (coalesced) with a fixed-order wave + LDS reduction
__global__ __launch_bounds__(256) void column_stats_planes(const double* __restrict__ X, int64_t n,
                                                           const double* __restrict__ center,
                                                           double* __restrict__ part, int ncols) {
  __shared__ double red[5][4];
  const int c = blockIdx.x;
  const int64_t r = (int64_t)blockIdx.y * ROWS_PER_BLOCK + threadIdx.x;
  const double x = r < n ? X[(int64_t)c * n + r] : NAN;
  const bool ok = x == x;
  const double d = ok ? x - (center ? center[c] : 0.0) : 0.0;
  double v[5] = {ok ? 1.0 : 0.0, ok ? x : 0.0, d * d, ok ? x : INFINITY, ok ? x : -INFINITY};
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    v[0] += __shfl_xor(v[0], o, 64);
    v[1] += __shfl_xor(v[1], o, 64);
    v[2] += __shfl_xor(v[2], o, 64);
    v[3] = fmin(v[3], __shfl_xor(v[3], o, 64));
    v[4] = fmax(v[4], __shfl_xor(v[4], o, 64));
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0)
    for (int q = 0; q < 5; ++q) red[q][w] = v[q];
  __syncthreads();
  if (threadIdx.x == 0) {
    double* p = part + (size_t)blockIdx.y * 5 * ncols;
    p[c] = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
    p[ncols + c] = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
    p[2 * ncols + c] = (red[2][0] + red[2][1]) + (red[2][2] + red[2][3]);
    p[3 * ncols + c] = fmin(fmin(red[3][0], red[3][1]), fmin(red[3][2], red[3][3]));
    p[4 * ncols + c] = fmax(fmax(red[4][0], red[4][1]), fmax(red[4][2], red[4][3]));
  }
}

__global__ __launch_bounds__(256) void bin_features_kernel(const float* __restrict__ X, int64_t n, int F, int ld,
                                                           const float* __restrict__ thr, int maxb,
                                                           const int32_t* __restrict__ nthr,
                                                           uint8_t* __restrict__ bins) {
  const int f = blockIdx.y;
  const int nt = nthr[f];
  const float* t = thr + (size_t)f * maxb;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float x = X[i * ld + f];
    int lo = 0, hi = nt;  // first index with t[idx] >= x  (== #thresholds < x)
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (t[mid] < x) lo = mid + 1; else hi = mid;
    }
    bins[(size_t)f * n + i] = (uint8_t)(x == x ? lo : nt);  // NaN -> last bin (numpy searchsorted order)
  }
}

}  // namespace

extern "C" int har_column_stats(const float* X, int64_t n, int ncols, int ld, const float* w, double* stats,
                                double* workspace, hipStream_t s) {
  if (n < 0 || ncols < 0 || ld < ncols) return -2;
  if (n == 0 || ncols == 0) return 0;
  const int nb = (int)((n + ROWS_PER_BLOCK - 1) / ROWS_PER_BLOCK);
  dim3 grid((ncols + 255) / 256, nb);
  column_stats_partial<float><<<grid, 256, 0, s>>>(X, n, ncols, ld, w, nullptr, workspace);
  column_stats_final<<<(ncols + 255) / 256, 256, 0, s>>>(workspace, nb, ncols, stats);
  HAR_CHECK_LAUNCH();
  return 0;
}

// fp64 input, column-major [ncols][n] (one device-CSV value plane per column); center as above
extern "C" int har_column_stats_f64(const double* X, int64_t n, int ncols, const double* center, double* stats,
                                    double* workspace, hipStream_t s) {
  if (n < 0 || ncols < 0) return -2;
  if (n == 0 || ncols == 0) return 0;
  const int nb = (int)((n + ROWS_PER_BLOCK - 1) / ROWS_PER_BLOCK);
  // column-major planes: one workgroup column per input column, lanes walk rows
  dim3 grid(ncols, nb);
  column_stats_planes<<<grid, 256, 0, s>>>(X, n, center, workspace, ncols);
  column_stats_final<<<(ncols + 255) / 256, 256, 0, s>>>(workspace, nb, ncols, stats);
  HAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int64_t har_column_stats_workspace(int64_t n, int ncols) {
  return ((n + ROWS_PER_BLOCK - 1) / ROWS_PER_BLOCK) * 5 * (int64_t)ncols;
}

extern "C" int har_bin_features(const float* X, int64_t n, int F, int ld, const float* thr, int maxb,
                                const int32_t* nthr, uint8_t* bins, hipStream_t s) {
  if (n < 0 || F < 0 || F > 65535 || ld < F) return -2;
  if (n == 0 || F == 0) return 0;
  dim3 grid((unsigned)std::min<int64_t>(1024, (n + 255) / 256), F);
  bin_features_kernel<<<grid, 256, 0, s>>>(X, n, F, ld, thr, maxb, nthr, bins);
  HAR_CHECK_LAUNCH();
  return 0;
}
