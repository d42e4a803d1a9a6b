// Windowed feature extraction over raw IMU streams.
//
// Input: stream [S][A] fp32 (sample-major, axes interleaved), windows of W
// samples every `stride` samples.  One wave64 per window: the window's W*A
// contiguous floats are staged into LDS with coalesced loads, then every lane
// owns samples lane, lane+64, ... and the statistics are wave-reduced in two
// passes (pass 1: sum / min / max / sum of squares; pass 2: deviations, 10-bin
// distribution, cross-axis covariance, resultant, peaks).
//
// Output row (F = 17*A + 4*(A/3) floats), WISDM-43 first for A = 3:
//   [bins: A x 10][avg: A][peak ms: A][absdev: A][std: A][resultant: A/3]
//   [min: A][max: A][energy: A][corr: 3 per axis triad (xy, xz, yz)]
// WISDM definitions (Kwapisz et al. 2010): bins = fraction of samples in 10
// equal-width bins spanning [min, max] of the window; absdev = mean |x - mean|;
// std = population standard deviation; resultant = mean sqrt(x^2+y^2+z^2);
// peak = mean time (ms) between local maxima above mean + 0.5 (max - mean)
// (NaN — the '?' of the WISDM table — when fewer than two peaks).
#include "common.h"
#include "../har_kernels.h"

namespace {

constexpr int MAXA = 9;
constexpr int NB = 10;
constexpr int WAVES = 4;

// A is a template parameter so every per-axis register array is statically indexed
// (runtime-indexed register arrays spill to scratch — guide §5.4 rule 20).
template <int A>
__global__ __launch_bounds__(WAVES * 64) void window_features_kernel(const float* __restrict__ stream,
                                                                     int64_t n_samples, int W, int stride,
                                                                     int64_t n_windows, float ms_per_sample,
                                                                     float* __restrict__ out, int ld_out) {
  extern __shared__ float lds[];  // [WAVES][W*A]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t win = (int64_t)blockIdx.x * WAVES + wave;
  if (win >= n_windows) return;  // wave-uniform; no block barrier below
  float* buf = lds + (size_t)wave * W * A;
  const float* src = stream + win * (int64_t)stride * A;
  const int n = W * A;
  for (int i = lane; i < n; i += 64) buf[i] = src[i];
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_wave_barrier();

  const float invW = 1.f / (float)W;
  float mean[A], mn[A], mx[A], en[A];
  // ---- pass 1 ----
#pragma unroll
  for (int a = 0; a < A; ++a) {
    float s = 0.f, q = 0.f, lo = INFINITY, hi = -INFINITY;
    for (int t = lane; t < W; t += 64) {
      float v = buf[t * A + a];
      s += v; q += v * v; lo = fminf(lo, v); hi = fmaxf(hi, v);
    }
    s = wave_sum(s);
    q = wave_sum(q);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      lo = fminf(lo, __shfl_xor(lo, o, 64));
      hi = fmaxf(hi, __shfl_xor(hi, o, 64));
    }
    mean[a] = s * invW; en[a] = q * invW; mn[a] = lo; mx[a] = hi;
  }
  constexpr int T3 = A / 3;
  float* o = out + win * (int64_t)ld_out;
  const int off_avg = A * NB, off_peak = off_avg + A, off_abs = off_peak + A, off_std = off_abs + A;
  const int off_res = off_std + A, off_min = off_res + T3, off_max = off_min + A, off_en = off_max + A;
  const int off_corr = off_en + A;
  // ---- pass 2: per axis ----
  float var[A];
#pragma unroll
  for (int a = 0; a < A; ++a) {
    const float m = mean[a], lo = mn[a], range = mx[a] - mn[a];
    const float thr = m + 0.5f * (mx[a] - m);
    float ad = 0.f, v2 = 0.f;
    int cnt[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) cnt[b] = 0;
    int first = 0x7fffffff, last = -1, npk = 0;
    for (int t = lane; t < W; t += 64) {
      const float v = buf[t * A + a];
      const float d = v - m;
      ad += fabsf(d);
      v2 += d * d;
      int b = range > 0.f ? (int)((v - lo) / range * NB) : 0;
      b = b < 0 ? 0 : (b >= NB ? NB - 1 : b);
#pragma unroll
      for (int k = 0; k < NB; ++k) cnt[k] += (k == b);
      if (t > 0 && t < W - 1) {
        const float pv = buf[(t - 1) * A + a], nv = buf[(t + 1) * A + a];
        if (v > pv && v >= nv && v > thr) {
          first = min(first, t); last = max(last, t); ++npk;
        }
      }
    }
    ad = wave_sum(ad);
    v2 = wave_sum(v2);
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      int c = cnt[k];
#pragma unroll
      for (int s = 32; s > 0; s >>= 1) c += __shfl_xor(c, s, 64);
      cnt[k] = c;
    }
#pragma unroll
    for (int s = 32; s > 0; s >>= 1) {
      first = min(first, __shfl_xor(first, s, 64));
      last = max(last, __shfl_xor(last, s, 64));
      npk += __shfl_xor(npk, s, 64);
    }
    var[a] = v2 * invW;
    // every lane holds the reduced counts; lane k writes bin k (static register indices only)
    float mine = 0.f;
#pragma unroll
    for (int k = 0; k < NB; ++k) mine = (lane == k) ? (float)cnt[k] : mine;
    if (lane < NB) o[a * NB + lane] = mine * invW;
    if (lane == 0) {
      o[off_avg + a] = m;
      o[off_peak + a] = npk >= 2 ? (float)(last - first) / (float)(npk - 1) * ms_per_sample : NAN;
      o[off_abs + a] = ad * invW;
      o[off_std + a] = sqrtf(var[a]);
      o[off_min + a] = mn[a];
      o[off_max + a] = mx[a];
      o[off_en + a] = en[a];
    }
  }
  // ---- per triad: resultant + correlations ----
#pragma unroll
  for (int g = 0; g < T3; ++g) {
    const int ax = 3 * g;
    float res = 0.f, cxy = 0.f, cxz = 0.f, cyz = 0.f;
    for (int t = lane; t < W; t += 64) {
      const float x = buf[t * A + ax], y = buf[t * A + ax + 1], z = buf[t * A + ax + 2];
      res += sqrtf(x * x + y * y + z * z);
      const float dx = x - mean[ax], dy = y - mean[ax + 1], dz = z - mean[ax + 2];
      cxy += dx * dy; cxz += dx * dz; cyz += dy * dz;
    }
    res = wave_sum(res); cxy = wave_sum(cxy); cxz = wave_sum(cxz); cyz = wave_sum(cyz);
    if (lane == 0) {
      o[off_res + g] = res * invW;
      const float sx = sqrtf(var[ax]), sy = sqrtf(var[ax + 1]), sz = sqrtf(var[ax + 2]);
      o[off_corr + 3 * g + 0] = (sx > 0.f && sy > 0.f) ? cxy * invW / (sx * sy) : 0.f;
      o[off_corr + 3 * g + 1] = (sx > 0.f && sz > 0.f) ? cxz * invW / (sx * sz) : 0.f;
      o[off_corr + 3 * g + 2] = (sy > 0.f && sz > 0.f) ? cyz * invW / (sy * sz) : 0.f;
    }
  }
}

}  // namespace

extern "C" int har_window_features(const float* stream, int64_t n_samples, int axes, int window, int stride,
                                   int64_t n_windows, float hz, int nbins, float* out, int ld_out, hipStream_t s) {
  if (axes > MAXA || axes % 3 || nbins != NB || window < 3 || stride <= 0) return -2;
  if ((n_windows - 1) * (int64_t)stride + window > n_samples) return -3;  // every window must be in bounds
  if (ld_out < 17 * axes + 4 * (axes / 3)) return -4;
  const size_t lds = (size_t)WAVES * window * axes * sizeof(float);
  if (lds > 160 * 1024) return -5;
  if (n_windows == 0) return 0;
  const int64_t blocks = (n_windows + WAVES - 1) / WAVES;
  const float ms = 1000.f / hz;
  switch (axes) {
    case 3: window_features_kernel<3><<<(unsigned)blocks, WAVES * 64, lds, s>>>(stream, n_samples, window, stride,
                                                                                 n_windows, ms, out, ld_out); break;
    case 6: window_features_kernel<6><<<(unsigned)blocks, WAVES * 64, lds, s>>>(stream, n_samples, window, stride,
                                                                                 n_windows, ms, out, ld_out); break;
    default: window_features_kernel<9><<<(unsigned)blocks, WAVES * 64, lds, s>>>(stream, n_samples, window, stride,
                                                                                  n_windows, ms, out, ld_out);
  }
  HAR_CHECK_LAUNCH();
  return 0;
}
