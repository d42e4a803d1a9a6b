// Windowed feature extraction over raw IMU streams.
//
// Input: stream [S][A] fp32 (sample-major, axes interleaved), windows of W
// samples every `stride` samples.  A group of LPW lanes per window — 16 (four
// windows per wave) when the block's window images fit 64 KB of LDS, else the
// whole wave: the windows' W*A floats are staged into LDS (one contiguous 16-byte
// load stream per wave for non-overlapping windows), every lane owns samples
// sub, sub+LPW, ... and the statistics are group-reduced with xor shuffles in
// two passes (pass 1: sum / min / max / sum of squares; pass 2: deviations,
// 10-bin distribution — two 16-bit counters per register — cross-axis
// covariance, resultant, peaks).
//
// Output row (F = 17*A + 4*(A/3) floats), WISDM-43 first for A = 3:
//   [bins: A x 10][avg: A][peak ms: A][absdev: A][std: A][resultant: A/3]
//   [min: A][max: A][energy: A][corr: 3 per axis triad (xy, xz, yz)]
// WISDM definitions (Kwapisz et al. 2010): bins = fraction of samples in 10
// equal-width bins spanning [min, max] of the window; absdev = mean |x - mean|;
// std = population standard deviation; resultant = mean sqrt(x^2+y^2+z^2);
// peak = mean time (ms) between local maxima above mean + 0.5 (max - mean)
// (NaN — the '?' of the WISDM table — when fewer than two peaks).
#include <type_traits>

#include "common.h"
#include "../har_kernels.h"

namespace {

constexpr int MAXA = 9;
constexpr int NB = 10;
constexpr int WAVES = 4;

// Reductions over the LPW lanes of one window group; every lane ends with the group's result.
// VALU data-parallel-primitive moves instead of ds_bpermute shuffles (LDS round trips): inside a
// 16-lane row a butterfly of quad_perm xor-1, quad_perm xor-2, row_half_mirror and row_mirror
// (after the quad steps every lane of a quad holds the quad's value, so the mirrors pair whole
// quads, then whole half-rows); across rows (LPW = 64) the gfx950 permlane16 / permlane32 swaps.
template <int CTRL> __device__ __forceinline__ int dpp_i(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
}
template <int CTRL> __device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(dpp_i<CTRL>(__float_as_int(v)));
}
__device__ __forceinline__ int swap16_i(int v) {  // value of lane ^ 16
  const auto r = __builtin_amdgcn_permlane16_swap((uint32_t)v, (uint32_t)v, false, false);
  const auto me = __builtin_amdgcn_permlane16_swap((uint32_t)__lane_id(), (uint32_t)__lane_id(), false, false);
  return (int)(me[0] == (uint32_t)(__lane_id() ^ 16) ? r[0] : r[1]);
}
__device__ __forceinline__ int swap32_i(int v) {  // value of lane ^ 32
  const auto r = __builtin_amdgcn_permlane32_swap((uint32_t)v, (uint32_t)v, false, false);
  const auto me = __builtin_amdgcn_permlane32_swap((uint32_t)__lane_id(), (uint32_t)__lane_id(), false, false);
  return (int)(me[0] == (uint32_t)(__lane_id() ^ 32) ? r[0] : r[1]);
}

template <int LPW, typename T, typename Op> __device__ __forceinline__ T greduce(T v, Op op) {
  static_assert(LPW == 16 || LPW == 64, "window groups of 16 or 64 lanes");
  auto mv = [](T x, auto ctrl) {
    constexpr int C = decltype(ctrl)::value;
    if constexpr (sizeof(T) == 4 && (T)0.5f != 0) return dpp_f<C>(x);
    else return (T)dpp_i<C>((int)x);
  };
  v = op(v, mv(v, std::integral_constant<int, 0xB1>{}));   // xor 1
  v = op(v, mv(v, std::integral_constant<int, 0x4E>{}));   // xor 2
  v = op(v, mv(v, std::integral_constant<int, 0x141>{}));  // row_half_mirror: quad <-> quad
  v = op(v, mv(v, std::integral_constant<int, 0x140>{}));  // row_mirror: half-row <-> half-row
  if constexpr (LPW == 64) {
    if constexpr ((T)0.5f != 0) {
      v = op(v, __int_as_float(swap16_i(__float_as_int(v))));
      v = op(v, __int_as_float(swap32_i(__float_as_int(v))));
    } else {
      v = op(v, (T)swap16_i((int)v));
      v = op(v, (T)swap32_i((int)v));
    }
  }
  return v;
}
template <int LPW> __device__ __forceinline__ float gsum(float v) {
  return greduce<LPW, float>(v, [](float a, float b) { return a + b; });
}
template <int LPW> __device__ __forceinline__ int gsumi(int v) {
  return greduce<LPW, int>(v, [](int a, int b) { return a + b; });
}
template <int LPW> __device__ __forceinline__ float gmin(float v) {
  return greduce<LPW, float>(v, [](float a, float b) { return fminf(a, b); });
}
template <int LPW> __device__ __forceinline__ float gmax(float v) {
  return greduce<LPW, float>(v, [](float a, float b) { return fmaxf(a, b); });
}
template <int LPW> __device__ __forceinline__ int gmini(int v) {
  return greduce<LPW, int>(v, [](int a, int b) { return min(a, b); });
}
template <int LPW> __device__ __forceinline__ int gmaxi(int v) {
  return greduce<LPW, int>(v, [](int a, int b) { return max(a, b); });
}

// A is a template parameter so every per-axis register array is statically indexed
// (runtime-indexed register arrays spill to scratch — guide §5.4 rule 20).
// LPW lanes per window: 16 (four windows per wave — every shuffle-reduction instruction
// serves four windows, and a 200-sample window keeps 12-13 samples per lane busy) or 64
// (one window per wave, for windows whose LDS image is large).
// MLP = true: the training-input variant — every feature is written as bf16
// ((isnan(v) ? nan_value : v) - mean[f]) * inv_std[f] into a zero-padded [n_windows][ld_out] row,
// so featurize -> NaN fill -> standardize -> cast -> pad is ONE pass.
struct MlpOut {
  const float* mean;
  const float* inv_std;
  float nan_value;
  uint16_t* out;
};

// The statistics of one window group's windows from their LDS image (`buf`: this group's window,
// W samples x A axes, sample-major).  Shared by the one-shot and the persistent kernels.
template <int A, int LPW, bool MLP>
__device__ __forceinline__ void window_compute(const float* buf, int W, bool valid, int64_t win, int sub,
                                               float ms_per_sample, float* __restrict__ out, int ld_out,
                                               const MlpOut& mo) {
  const float invW = 1.f / (float)W;
  float mean[A], mn[A], mx[A], en[A];
  // ---- pass 1: one sweep over the samples for all axes ----
  {
    float s[A], q[A], lo[A], hi[A];
#pragma unroll
    for (int a = 0; a < A; ++a) { s[a] = 0.f; q[a] = 0.f; lo[a] = INFINITY; hi[a] = -INFINITY; }
    if (valid)
      for (int t = sub; t < W; t += LPW) {
#pragma unroll
        for (int a = 0; a < A; ++a) {
          const float v = buf[t * A + a];
          s[a] += v; q[a] += v * v; lo[a] = fminf(lo[a], v); hi[a] = fmaxf(hi[a], v);
        }
      }
#pragma unroll
    for (int a = 0; a < A; ++a) {
      mean[a] = gsum<LPW>(s[a]) * invW; en[a] = gsum<LPW>(q[a]) * invW;
      mn[a] = gmin<LPW>(lo[a]); mx[a] = gmax<LPW>(hi[a]);
    }
  }
  constexpr int T3 = A / 3;
  float* o = MLP ? nullptr : out + (valid ? win : 0) * (int64_t)ld_out;
  uint16_t* ob = MLP ? mo.out + (valid ? win : 0) * (int64_t)ld_out : nullptr;
  auto emit = [&](int f, float v) {
    if constexpr (MLP) {
      const float x = v != v ? mo.nan_value : v;
      ob[f] = f2bf((x - mo.mean[f]) * mo.inv_std[f]);
    } else {
      o[f] = v;
    }
  };
  if constexpr (MLP) {  // zero the pad columns of the row
    constexpr int F = 17 * A + 4 * (A / 3);
    for (int f = F + sub; f < ld_out; f += LPW)
      if (valid) ob[f] = 0;
  }
  const int off_avg = A * NB, off_peak = off_avg + A, off_abs = off_peak + A, off_std = off_abs + A;
  const int off_res = off_std + A, off_min = off_res + T3, off_max = off_min + A, off_en = off_max + A;
  const int off_corr = off_en + A;
  // ---- pass 2: per axis ----
  float var[A];
#pragma unroll
  for (int a = 0; a < A; ++a) {
    const float m = mean[a], lo = mn[a], range = mx[a] - mn[a];
    const float bscale = range > 0.f ? (float)NB / range : 0.f;  // one reciprocal per axis, not per sample
    const float thr = m + 0.5f * (mx[a] - m);
    float ad = 0.f, v2 = 0.f;
    int cnt[NB / 2];  // two 16-bit bin counters per register (W < 65536): 5 reductions, not 10
#pragma unroll
    for (int b = 0; b < NB / 2; ++b) cnt[b] = 0;
    int first = 0x7fffffff, last = -1, npk = 0;
    if (valid)
      for (int t = sub; t < W; t += LPW) {
        const float v = buf[t * A + a];
        const float d = v - m;
        ad += fabsf(d);
        v2 += d * d;
        int b = (int)((v - lo) * bscale);
        b = b < 0 ? 0 : (b >= NB ? NB - 1 : b);
        const int inc = (b & 1) ? 0x10000 : 1;
#pragma unroll
        for (int k = 0; k < NB / 2; ++k) cnt[k] += ((b >> 1) == k) ? inc : 0;
        if (t > 0 && t < W - 1) {
          const float pv = buf[(t - 1) * A + a], nv = buf[(t + 1) * A + a];
          if (v > pv && v >= nv && v > thr) {
            first = min(first, t); last = max(last, t); ++npk;
          }
        }
      }
    ad = gsum<LPW>(ad);
    v2 = gsum<LPW>(v2);
#pragma unroll
    for (int k = 0; k < NB / 2; ++k) cnt[k] = gsumi<LPW>(cnt[k]);
    first = gmini<LPW>(first);
    last = gmaxi<LPW>(last);
    npk = gsumi<LPW>(npk);
    var[a] = v2 * invW;
    // every lane of the group holds the reduced counts; lane k % LPW of the group writes bin k
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      const int c = (k & 1) ? (cnt[k >> 1] >> 16) : (cnt[k >> 1] & 0xffff);
      if (valid && sub == k % LPW) emit(a * NB + k, (float)c * invW);
    }
    if (valid && sub == 0) {
      emit(off_avg + a, m);
      emit(off_peak + a, npk >= 2 ? (float)(last - first) / (float)(npk - 1) * ms_per_sample : NAN);
      emit(off_abs + a, ad * invW);
      emit(off_std + a, sqrtf(var[a]));
      emit(off_min + a, mn[a]);
      emit(off_max + a, mx[a]);
      emit(off_en + a, en[a]);
    }
  }
  // ---- per triad: resultant + correlations ----
#pragma unroll
  for (int g = 0; g < T3; ++g) {
    const int ax = 3 * g;
    float res = 0.f, cxy = 0.f, cxz = 0.f, cyz = 0.f;
    if (valid)
      for (int t = sub; t < W; t += LPW) {
        const float x = buf[t * A + ax], y = buf[t * A + ax + 1], z = buf[t * A + ax + 2];
        res += sqrtf(x * x + y * y + z * z);
        const float dx = x - mean[ax], dy = y - mean[ax + 1], dz = z - mean[ax + 2];
        cxy += dx * dy; cxz += dx * dz; cyz += dy * dz;
      }
    res = gsum<LPW>(res); cxy = gsum<LPW>(cxy); cxz = gsum<LPW>(cxz); cyz = gsum<LPW>(cyz);
    if (valid && sub == 0) {
      emit(off_res + g, res * invW);
      const float sx = sqrtf(var[ax]), sy = sqrtf(var[ax + 1]), sz = sqrtf(var[ax + 2]);
      emit(off_corr + 3 * g + 0, (sx > 0.f && sy > 0.f) ? cxy * invW / (sx * sy) : 0.f);
      emit(off_corr + 3 * g + 1, (sx > 0.f && sz > 0.f) ? cxz * invW / (sx * sz) : 0.f);
      emit(off_corr + 3 * g + 2, (sy > 0.f && sz > 0.f) ? cyz * invW / (sy * sz) : 0.f);
    }
  }
}

template <int A, int LPW, bool MLP>
__global__ __launch_bounds__(WAVES * 64) void window_features_kernel(const float* __restrict__ stream,
                                                                     int64_t n_samples, int W, int stride,
                                                                     int64_t n_windows, float ms_per_sample,
                                                                     float* __restrict__ out, int ld_out,
                                                                     MlpOut mo) {
  constexpr int G = 64 / LPW;  // windows per wave
  extern __shared__ __attribute__((aligned(16))) float lds[];  // [WAVES * G][W*A]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int sub = lane % LPW, grp = lane / LPW;
  const int64_t win0 = ((int64_t)blockIdx.x * WAVES + wave) * G;
  if (win0 >= n_windows) return;  // wave-uniform; no block barrier below
  const int64_t win = win0 + grp;
  const bool valid = win < n_windows;
  const int n = W * A;
  float* wbuf = lds + (size_t)wave * G * n;
  float* buf = wbuf + (size_t)grp * n;
  // ---- stage the wave's windows in LDS ----
  const int nw = (int)min<int64_t>(G, n_windows - win0);
  if (stride == W && G > 1) {
    // non-overlapping windows: the wave's windows are one contiguous run; 16-byte loads when aligned
    const float* src = stream + win0 * (int64_t)W * A;
    const int tot = nw * n;
    if (((reinterpret_cast<uintptr_t>(src) & 15) == 0) && (tot % 4 == 0) && (n % 4 == 0)) {
      const float4* s4 = reinterpret_cast<const float4*>(src);
      float4* d4 = reinterpret_cast<float4*>(wbuf);
      for (int i = lane; i < tot / 4; i += 64) d4[i] = s4[i];
    } else {
      for (int i = lane; i < tot; i += 64) wbuf[i] = src[i];
    }
  } else if (valid) {
    const float* src = stream + win * (int64_t)stride * A;
    for (int i = sub; i < n; i += LPW) buf[i] = src[i];
  }
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_wave_barrier();

  window_compute<A, LPW, MLP>(buf, W, valid, win, sub, ms_per_sample, out, ld_out, mo);
}

// Persistent variant: each wave walks window groups g, g + waves_in_grid, ...; the contiguous
// sample span of the NEXT group (G windows, (G - 1) stride + W samples) is loaded into PV 16-byte
// registers per lane while the current group is computed from LDS, so HBM latency hides behind
// the statistics instead of being paid once per group.  Loads are unconditional (indices clamped
// into the stream: the duplicates are never read) so the waits stay counted.  Needs the span to
// fit 64 * PV float4 and 16-byte alignment of every group start (host checks).
template <int A, int LPW, bool MLP, int PV>
__global__ __launch_bounds__(WAVES * 64) __attribute__((amdgpu_waves_per_eu(2, 3)))
void window_features_persistent_kernel(
    const float* __restrict__ stream, int64_t n_samples, int W, int stride, int64_t n_windows, float ms_per_sample,
    float* __restrict__ out, int ld_out, MlpOut mo) {
  constexpr int G = 64 / LPW;
  extern __shared__ __attribute__((aligned(16))) float lds[];  // [WAVES][PV * 64 float4]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int sub = lane % LPW, grp = lane / LPW;
  // native clang vectors, not HIP's float4 struct: struct copies of an array element defeat the
  // alloca-to-register promotion and put `pre` in scratch
  typedef float v4f __attribute__((ext_vector_type(4)));
  v4f* img = reinterpret_cast<v4f*>(lds) + (size_t)wave * PV * 64;
  const int64_t ngroups = (n_windows + G - 1) / G;
  const int64_t step = (int64_t)gridDim.x * WAVES;
  const int64_t total4 = n_samples * A / 4;  // whole float4s of the stream
  const v4f* s4 = reinterpret_cast<const v4f*>(stream);
  v4f pre[PV];
  int64_t g = (int64_t)blockIdx.x * WAVES + wave;
  if (g >= ngroups) return;  // wave-uniform; no block barrier below
  {
    const int64_t base = g * G * (int64_t)stride * A / 4;
#pragma unroll
    for (int j = 0; j < PV; ++j) {
      const int64_t i = base + lane + 64 * j;
      pre[j] = s4[i < total4 ? i : total4 - 1];
    }
  }
  for (; g < ngroups; g += step) {
    __builtin_amdgcn_wave_barrier();  // this wave's reads of the previous image are issued first
#pragma unroll
    for (int j = 0; j < PV; ++j) img[lane + 64 * j] = pre[j];
    {
      const int64_t gn = g + step < ngroups ? g + step : ngroups - 1;
      const int64_t base = gn * G * (int64_t)stride * A / 4;
#pragma unroll
      for (int j = 0; j < PV; ++j) {
        const int64_t i = base + lane + 64 * j;
        pre[j] = s4[i < total4 ? i : total4 - 1];
      }
    }
    __builtin_amdgcn_sched_barrier(0);  // the prefetch goes out before the compute
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the image is written
    __builtin_amdgcn_wave_barrier();
    const int64_t win = g * G + grp;
    const bool valid = win < n_windows;
    window_compute<A, LPW, MLP>(reinterpret_cast<const float*>(img) + (size_t)grp * stride * A, W, valid, win, sub,
                                ms_per_sample, out, ld_out, mo);
  }
}

constexpr int PV16 = 12, PV64 = 20;  // prefetch registers (float4 per lane) of the persistent kernels

int cu_count() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                 hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

template <int A, bool MLP>
int launch_axes(const float* stream, int64_t n_samples, int window, int stride, int64_t n_windows, float ms,
                float* out, int ld_out, MlpOut mo, hipStream_t s) {
  // persistent + register-prefetched when a group's contiguous span fits the prefetch registers
  // and every group starts 16-byte aligned (the common non-overlapping / half-overlapping cases)
  const bool aligned = (reinterpret_cast<uintptr_t>(stream) & 15) == 0 && (n_samples * A) % 4 == 0;
  const int64_t span16 = (int64_t)(3 * stride + window) * A, span64 = (int64_t)window * A;
  if (false && aligned && stride <= window && span16 <= PV16 * 256 && window <= 16 * 15) {  // measured slower (105 vs 97 us)
    const int64_t groups = (n_windows + 3) / 4;
    const int64_t blocks = std::min<int64_t>((groups + WAVES - 1) / WAVES, (int64_t)cu_count() * 3);
    window_features_persistent_kernel<A, 16, MLP, PV16><<<(unsigned)blocks, WAVES * 64, WAVES * PV16 * 64 * 16, s>>>(
        stream, n_samples, window, stride, n_windows, ms, out, ld_out, mo);
    HAR_CHECK_LAUNCH();
    return 0;
  }
  if (aligned && stride <= window && ((int64_t)stride * A) % 4 == 0 && span64 <= PV64 * 256) {
    const int64_t blocks = std::min<int64_t>((n_windows + WAVES - 1) / WAVES, (int64_t)cu_count() * 2);
    window_features_persistent_kernel<A, 64, MLP, PV64><<<(unsigned)blocks, WAVES * 64, WAVES * PV64 * 64 * 16, s>>>(
        stream, n_samples, window, stride, n_windows, ms, out, ld_out, mo);
    HAR_CHECK_LAUNCH();
    return 0;
  }
  // four windows per wave while the block's 16 window images fit 64 KB of LDS, else one
  const size_t img = (size_t)window * A * sizeof(float);
  // (measured on MI355X, 200-sample 3-axis windows: 16 lanes 0.255 ms/stream step, 8 lanes 0.308,
  //  a register-resident chunk layout 0.271)
  if ((size_t)WAVES * 4 * img <= 64 * 1024) {
    const int64_t blocks = (n_windows + WAVES * 4 - 1) / (WAVES * 4);
    window_features_kernel<A, 16, MLP><<<(unsigned)blocks, WAVES * 64, WAVES * 4 * img, s>>>(
        stream, n_samples, window, stride, n_windows, ms, out, ld_out, mo);
  } else {
    if ((size_t)WAVES * img > 160 * 1024) return -5;
    const int64_t blocks = (n_windows + WAVES - 1) / WAVES;
    window_features_kernel<A, 64, MLP><<<(unsigned)blocks, WAVES * 64, WAVES * img, s>>>(
        stream, n_samples, window, stride, n_windows, ms, out, ld_out, mo);
  }
  HAR_CHECK_LAUNCH();
  return 0;
}

}  // namespace

extern "C" int har_window_features(const float* stream, int64_t n_samples, int axes, int window, int stride,
                                   int64_t n_windows, float hz, int nbins, float* out, int ld_out, hipStream_t s) {
  if (axes > MAXA || axes % 3 || nbins != NB || window < 3 || window >= 65536 || stride <= 0) return -2;
  if ((n_windows - 1) * (int64_t)stride + window > n_samples) return -3;  // every window must be in bounds
  if (ld_out < 17 * axes + 4 * (axes / 3)) return -4;
  if (n_windows == 0) return 0;
  const float ms = 1000.f / hz;
  const MlpOut none{nullptr, nullptr, 0.f, nullptr};
  switch (axes) {
    case 3: return launch_axes<3, false>(stream, n_samples, window, stride, n_windows, ms, out, ld_out, none, s);
    case 6: return launch_axes<6, false>(stream, n_samples, window, stride, n_windows, ms, out, ld_out, none, s);
    default: return launch_axes<9, false>(stream, n_samples, window, stride, n_windows, ms, out, ld_out, none, s);
  }
}

extern "C" int har_window_features_mlp(const float* stream, int64_t n_samples, int axes, int window, int stride,
                                       int64_t n_windows, float hz, const float* mean, const float* inv_std,
                                       float nan_value, uint16_t* out, int ld_out, hipStream_t s) {
  if (axes > MAXA || axes % 3 || window < 3 || window >= 65536 || stride <= 0) return -2;
  if ((n_windows - 1) * (int64_t)stride + window > n_samples) return -3;
  if (ld_out < 17 * axes + 4 * (axes / 3) || !mean || !inv_std || !out) return -4;
  if (n_windows == 0) return 0;
  const float ms = 1000.f / hz;
  const MlpOut mo{mean, inv_std, nan_value, out};
  switch (axes) {
    case 3: return launch_axes<3, true>(stream, n_samples, window, stride, n_windows, ms, nullptr, ld_out, mo, s);
    case 6: return launch_axes<6, true>(stream, n_samples, window, stride, n_windows, ms, nullptr, ld_out, mo, s);
    default: return launch_axes<9, true>(stream, n_samples, window, stride, n_windows, ms, nullptr, ld_out, mo, s);
  }
}
