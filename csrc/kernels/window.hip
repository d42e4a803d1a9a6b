// Windowed feature extraction over raw IMU streams (the columns of
// the reference's pre-windowed table, Main/wisdm_main_ver_0.0/data/wisdm_data.csv:1, read at
// Main/main.py:16-20).
//
// Input: stream [S][A] fp32 (sample-major, axes interleaved), windows of W samples every
// `stride` samples.  Every feature is per axis or per axis triad (x, y, z), so the unit of work
// is a GROUP = (window, triad): 16 lanes (one 16-lane row of a wave, four groups per wave) own
// one group, lane `sub` taking samples t = sub, sub + 16, sub + 32, ...
//
//   * a block stages the contiguous sample span of its windows (overlapping windows share the
//     span) HBM -> LDS with 16-byte loads, eight in flight per thread;
//   * pass 1 (sum, sum of squares, min, max) and pass 2 (|x - mean|, (x - mean)^2, the 10-bin
//     distribution, peaks, resultant, triad covariances) read the group's samples from LDS —
//     consecutive lanes read consecutive samples, A (odd) floats apart: conflict-free banks —
//     and accumulate per lane with no per-sample masking except in the first and the last
//     iterations (t = 0, t >= W - 1);
//   * the distribution counts are packed 6 bits per bin in one 64-bit register per axis
//     (one v_lshl_add_u64 per sample) and the local maxima as one bit per iteration,
//     both flushed every 32 iterations; npk / first / last come from popcount / ctz / clz;
//   * the 16-lane reductions are DPP butterflies (quad_perm, row_half_mirror, row_mirror):
//     VALU moves, no LDS round trips.
//
// Output row (F = 17*A + 4*(A/3) floats), WISDM-43 first for A = 3:
//   [bins: A x 10][avg: A][peak ms: A][absdev: A][std: A][resultant: A/3]
//   [min: A][max: A][energy: A][corr: 3 per axis triad (xy, xz, yz)]
// WISDM definitions (Kwapisz et al. 2010): bins = fraction of samples in 10 equal-width bins
// spanning [min, max] of the window; absdev = mean |x - mean|; std = population standard
// deviation; resultant = mean sqrt(x^2+y^2+z^2); peak = mean time (ms) between local maxima
// above mean + 0.5 (max - mean) (NaN — the '?' of the WISDM table — when fewer than two peaks).
#include "common.h"
#include "../har_kernels.h"

namespace {

constexpr int MAXA = 9;
constexpr int NB = 10;
constexpr int PAD = 12;    // floats of LDS before the staged span: the t = -1 neighbour read stays inside
constexpr int SLACK = 16;  // floats after it: the t = W neighbour read of the last window stays inside

typedef float v4f __attribute__((ext_vector_type(4)));

// Reductions over one 16-lane row; every lane ends with the row's result.  quad_perm xor-1,
// quad_perm xor-2, then row_half_mirror and row_mirror (after the quad steps every lane of a
// quad holds the quad's value, so the mirrors pair whole quads, then whole half-rows).
template <int CTRL> __device__ __forceinline__ int dpp_i(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
}
template <typename T, typename Op> __device__ __forceinline__ T rreduce(T v, Op op) {
  auto mv = [](T x, auto ctrl) {
    constexpr int C = decltype(ctrl)::value;
    if constexpr (sizeof(T) == 4 && (T)0.5f != 0) return __int_as_float(dpp_i<C>(__float_as_int(x)));
    else return (T)dpp_i<C>((int)x);
  };
  v = op(v, mv(v, std::integral_constant<int, 0xB1>{}));   // xor 1
  v = op(v, mv(v, std::integral_constant<int, 0x4E>{}));   // xor 2
  v = op(v, mv(v, std::integral_constant<int, 0x141>{}));  // row_half_mirror: quad <-> quad
  v = op(v, mv(v, std::integral_constant<int, 0x140>{}));  // row_mirror: half-row <-> half-row
  return v;
}
__device__ __forceinline__ float rsum(float v) { return rreduce<float>(v, [](float a, float b) { return a + b; }); }
__device__ __forceinline__ uint32_t rsumu(uint32_t v) {
  return rreduce<uint32_t>(v, [](uint32_t a, uint32_t b) { return a + b; });
}
__device__ __forceinline__ float rmin(float v) { return rreduce<float>(v, [](float a, float b) { return fminf(a, b); }); }
__device__ __forceinline__ float rmax(float v) { return rreduce<float>(v, [](float a, float b) { return fmaxf(a, b); }); }
__device__ __forceinline__ int rmini(int v) { return rreduce<int>(v, [](int a, int b) { return min(a, b); }); }
__device__ __forceinline__ int rmaxi(int v) { return rreduce<int>(v, [](int a, int b) { return max(a, b); }); }

// MLP = true: the training-input variant — every feature is written as bf16
// ((isnan(v) ? nan_value : v) - mean[f]) * inv_std[f] into a zero-padded [n_windows][ld_out] row,
// so featurize -> NaN fill -> standardize -> cast -> pad is ONE pass.
struct MlpOut {
  const float* mean;
  const float* inv_std;
  float nan_value;
  uint16_t* out;
};

// per-axis constants of pass 2 (from the pass-1 reductions)
struct Pass2K {
  float m[3], lo[3], bsc[3], thr[3];
};
// per-lane pass-2 accumulators of one triad
struct Pass2Acc {
  float ad[3], v2[3], res, cxy, cxz, cyz;
  uint64_t h[3];    // 10 bins x 6 bits (at most 32 samples per lane between flushes)
  uint32_t pk[3];   // bit j: the sample of iteration kbase + j is a peak
  uint32_t hw[3][5];  // flushed counts, two 16-bit bins per word
  int npk[3], first[3], last[3];
};

// One iteration of pass 2 at sample t.  EDGE iterations (the first, and those reaching t >= W - 1)
// mask samples past the window and exclude t = 0 / t = W - 1 from the peaks.
template <int A, bool EDGE>
__device__ __forceinline__ void pass2_step(const float* img, int t, int W, const Pass2K& K, Pass2Acc& a,
                                           uint32_t bit) {
  bool ok = true, pkok = true;
  int tt = t;
  if constexpr (EDGE) {
    ok = t < W;
    pkok = t > 0 && t < W - 1;
    tt = ok ? t : W - 1;
  }
  const float* p = img + tt * A;
  float v[3], d[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float pv = p[c - A], x = p[c], nv = p[c + A];
    v[c] = x;
    float dc = x - K.m[c];
    if constexpr (EDGE) dc = ok ? dc : 0.f;
    d[c] = dc;
    a.ad[c] += fabsf(dc);
    a.v2[c] = fmaf(dc, dc, a.v2[c]);
    uint32_t b = __float2uint_rz((x - K.lo[c]) * K.bsc[c]);  // x >= lo: non-negative
    b = b < NB - 1 ? b : NB - 1;
    const uint64_t inc = (EDGE && !ok) ? 0ull : 1ull;
    a.h[c] += inc << (6 * b);
    const bool peak = x > pv && x >= nv && x > K.thr[c] && pkok;
    a.pk[c] |= peak ? bit : 0u;
  }
  const float r = __builtin_sqrtf(fmaf(v[0], v[0], fmaf(v[1], v[1], v[2] * v[2])));
  a.res += (EDGE && !ok) ? 0.f : r;
  a.cxy = fmaf(d[0], d[1], a.cxy);
  a.cxz = fmaf(d[0], d[2], a.cxz);
  a.cyz = fmaf(d[1], d[2], a.cyz);
}

// fold the packed counts and peak bits of the 32-iteration chunk starting at kbase
__device__ __forceinline__ void pass2_flush(Pass2Acc& a, int sub, int kbase) {
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const uint64_t h = a.h[c];
#pragma unroll
    for (int j = 0; j < 5; ++j)
      a.hw[c][j] += (uint32_t)((h >> (12 * j)) & 63) | ((uint32_t)((h >> (12 * j + 6)) & 63) << 16);
    a.h[c] = 0;
    const uint32_t pk = a.pk[c];
    a.npk[c] += __builtin_popcount(pk);
    const int f = sub + 16 * (kbase + __builtin_ctz(pk | 0x80000000u));
    const int l = sub + 16 * (kbase + 31 - __builtin_clz(pk | 1u));
    a.first[c] = pk ? min(a.first[c], f) : a.first[c];
    a.last[c] = pk ? max(a.last[c], l) : a.last[c];
    a.pk[c] = 0;
  }
}

// One block = `waves` waves = 4 * waves groups = 4 * waves / (A / 3) whole windows (host picks
// `waves` so that divides).  One-shot: stage, compute, write.
template <int A, bool MLP>
__global__ __launch_bounds__(256) void window_features_kernel(const float* __restrict__ stream, int64_t n_samples,
                                                              int W, int stride, int64_t n_windows,
                                                              float ms_per_sample, float* __restrict__ out,
                                                              int ld_out, MlpOut mo) {
  constexpr int T3 = A / 3;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int nt = (int)blockDim.x, tid = (int)threadIdx.x;
  const int wpb = (nt >> 6) * 4 / T3;
  const int64_t w0 = (int64_t)blockIdx.x * wpb;
  const int nwin = (int)min<int64_t>(wpb, n_windows - w0);
  const bool contiguous = stride <= W;
  const int istride = (contiguous ? stride : W) * A;  // floats between window images in LDS
  float* img0;
  // ---- stage the block's windows in LDS ----
  if (contiguous) {
    const int64_t s0 = w0 * stride * A;
    const int64_t len = ((int64_t)(nwin - 1) * stride + W) * A;
    const int lead = (int)(s0 & 3);
    float* dst = lds + PAD;  // 16-byte aligned; holds the span from the float4 containing s0
    img0 = dst + lead;
    if ((reinterpret_cast<uintptr_t>(stream) & 15) == 0) {
      const int64_t t4 = n_samples * A >> 2;  // whole float4s of the stream
      const int64_t a4 = (s0 - lead) >> 2;
      const int n4 = (int)((lead + len + 3) >> 2);
      const v4f* s4 = reinterpret_cast<const v4f*>(stream);
      v4f* d4 = reinterpret_cast<v4f*>(dst);
      for (int i0 = tid; i0 < n4; i0 += 8 * nt) {
        v4f r[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {  // unconditional (clamped) loads: eight in flight
          const int64_t gi = a4 + i0 + j * nt;
          r[j] = s4[gi < t4 ? gi : t4 - 1];
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int i = i0 + j * nt;
          if (i < n4 && a4 + i < t4) d4[i] = r[j];
        }
      }
      // floats past the stream's last whole float4 (n_samples * A % 4 != 0)
      for (int64_t e = max(t4 * 4, s0) + tid; e < s0 + len; e += nt) img0[e - s0] = stream[e];
    } else {
      for (int64_t e = tid; e < len; e += nt) img0[e] = stream[s0 + e];
    }
  } else {  // windows with gaps between them: one image each
    img0 = lds + PAD;
    const int n = W * A;
    for (int i = 0; i < nwin; ++i) {
      const float* src = stream + (w0 + i) * stride * A;
      for (int e = tid; e < n; e += nt) img0[i * n + e] = src[e];
    }
  }
  __syncthreads();

  const int lane = tid & 63, sub = lane & 15;
  const int gl = (tid >> 6) * 4 + (lane >> 4);  // this row's group
  const int wi = gl / T3, g = gl % T3;
  const bool valid = wi < nwin;
  const int64_t win = w0 + (valid ? wi : 0);
  const float* img = img0 + (valid ? wi : 0) * istride + 3 * g;  // the group's triad: A floats per sample
  const int C = (W + 15) >> 4;       // iterations (samples per lane, the last partial)
  const int kfull = (W - 1) >> 4;    // k < kfull: every t = sub + 16k lies in [0, W - 2]
  const float invW = 1.f / (float)W;

  // ---- pass 1: sum, sum of squares, min, max ----
  float mean[3], mn[3], mx[3], en[3];
  {
    float s[3], q[3], lo[3], hi[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) { s[c] = 0.f; q[c] = 0.f; lo[c] = INFINITY; hi[c] = -INFINITY; }
    const float* p = img + sub * A;
    int k = 0;
#pragma unroll 2
    for (; k < kfull; ++k, p += 16 * A) {
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const float v = p[c];
        s[c] += v; q[c] = fmaf(v, v, q[c]); lo[c] = fminf(lo[c], v); hi[c] = fmaxf(hi[c], v);
      }
    }
    for (; k < C; ++k) {
      const int t = sub + 16 * k;
      const bool ok = t < W;
      const float* pp = img + (ok ? t : W - 1) * A;  // a duplicate of a window sample: min / max unchanged
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const float v = pp[c], vm = ok ? v : 0.f;
        s[c] += vm; q[c] = fmaf(vm, vm, q[c]); lo[c] = fminf(lo[c], v); hi[c] = fmaxf(hi[c], v);
      }
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      mean[c] = rsum(s[c]) * invW; en[c] = rsum(q[c]) * invW;
      mn[c] = rmin(lo[c]); mx[c] = rmax(hi[c]);
    }
  }

  // ---- pass 2 ----
  Pass2K K;
  Pass2Acc a;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float range = mx[c] - mn[c];
    K.m[c] = mean[c]; K.lo[c] = mn[c];
    K.bsc[c] = range > 0.f ? (float)NB / range : 0.f;  // one reciprocal per axis, not per sample
    K.thr[c] = mean[c] + 0.5f * (mx[c] - mean[c]);
    a.ad[c] = 0.f; a.v2[c] = 0.f; a.h[c] = 0; a.pk[c] = 0;
    a.npk[c] = 0; a.first[c] = 0x7fffffff; a.last[c] = -1;
#pragma unroll
    for (int j = 0; j < 5; ++j) a.hw[c][j] = 0;
  }
  a.res = 0.f; a.cxy = 0.f; a.cxz = 0.f; a.cyz = 0.f;
  pass2_step<A, true>(img, sub, W, K, a, 1u);  // k = 0 holds t = 0
  int k = 1;
#pragma unroll 2
  for (; k < kfull; ++k) {
    pass2_step<A, false>(img, sub + 16 * k, W, K, a, 1u << (k & 31));
    if ((k & 31) == 31) pass2_flush(a, sub, k - 31);
  }
  for (; k < C; ++k) {
    pass2_step<A, true>(img, sub + 16 * k, W, K, a, 1u << (k & 31));
    if ((k & 31) == 31) pass2_flush(a, sub, k - 31);
  }
  if (C & 31) pass2_flush(a, sub, (C - 1) & ~31);

  // ---- reduce + write ----
  float* o = MLP ? nullptr : out + win * (int64_t)ld_out;
  uint16_t* ob = MLP ? mo.out + win * (int64_t)ld_out : nullptr;
  auto emit = [&](bool on, int f, float v) {
    if (!(on && valid)) return;
    if constexpr (MLP) {
      const float x = v != v ? mo.nan_value : v;
      ob[f] = f2bf((x - mo.mean[f]) * mo.inv_std[f]);
    } else {
      o[f] = v;
    }
  };
  constexpr int F = 17 * A + 4 * T3;
  if constexpr (MLP) {  // zero the pad columns of the row (triad 0's group)
    if (g == 0)
      for (int f = F + sub; f < ld_out; f += 16)
        if (valid) ob[f] = 0;
  }
  const int off_avg = A * NB, off_peak = off_avg + A, off_abs = off_peak + A, off_std = off_abs + A;
  const int off_res = off_std + A, off_min = off_res + T3, off_max = off_min + A, off_en = off_max + A;
  const int off_corr = off_en + A;
  float sd[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const int ax = 3 * g + c;
    const float ad = rsum(a.ad[c]) * invW;
    const float var = rsum(a.v2[c]) * invW;
    sd[c] = sqrtf(var);
    const int npk = (int)rsumu((uint32_t)a.npk[c]);
    const int first = rmini(a.first[c]), last = rmaxi(a.last[c]);
    // bins: lane `sub` < 10 writes bin `sub` (its word picked by a select chain, not an indexed array)
    uint32_t word = 0;
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      const uint32_t wj = rsumu(a.hw[c][j]);
      word = (sub >> 1) == j ? wj : word;
    }
    const uint32_t cnt = (sub & 1) ? word >> 16 : word & 0xffffu;
    emit(sub < NB, ax * NB + sub, (float)cnt * invW);
    // scalars: lanes 0..6
    const float peak = npk >= 2 ? (float)(last - first) / (float)(npk - 1) * ms_per_sample : NAN;
    float v = mean[c];
    int f = off_avg + ax;
    v = sub == 1 ? peak : v;       f = sub == 1 ? off_peak + ax : f;
    v = sub == 2 ? ad : v;         f = sub == 2 ? off_abs + ax : f;
    v = sub == 3 ? sd[c] : v;      f = sub == 3 ? off_std + ax : f;
    v = sub == 4 ? mn[c] : v;      f = sub == 4 ? off_min + ax : f;
    v = sub == 5 ? mx[c] : v;      f = sub == 5 ? off_max + ax : f;
    v = sub == 6 ? en[c] : v;      f = sub == 6 ? off_en + ax : f;
    emit(sub < 7, f, v);
  }
  // triad: resultant (lane 0) and the three correlations (lanes 1..3)
  {
    const float res = rsum(a.res) * invW;
    const float cxy = rsum(a.cxy) * invW, cxz = rsum(a.cxz) * invW, cyz = rsum(a.cyz) * invW;
    const float rxy = (sd[0] > 0.f && sd[1] > 0.f) ? cxy / (sd[0] * sd[1]) : 0.f;
    const float rxz = (sd[0] > 0.f && sd[2] > 0.f) ? cxz / (sd[0] * sd[2]) : 0.f;
    const float ryz = (sd[1] > 0.f && sd[2] > 0.f) ? cyz / (sd[1] * sd[2]) : 0.f;
    float v = res;
    int f = off_res + g;
    v = sub == 1 ? rxy : v;  f = sub == 1 ? off_corr + 3 * g : f;
    v = sub == 2 ? rxz : v;  f = sub == 2 ? off_corr + 3 * g + 1 : f;
    v = sub == 3 ? ryz : v;  f = sub == 3 ? off_corr + 3 * g + 2 : f;
    emit(sub < 4, f, v);
  }
}

template <int A, bool MLP>
int launch_axes(const float* stream, int64_t n_samples, int window, int stride, int64_t n_windows, float ms,
                float* out, int ld_out, MlpOut mo, hipStream_t s) {
  constexpr int T3 = A / 3;
  const bool contiguous = stride <= window;
  auto lds_bytes = [&](int wpb) -> int64_t {
    const int64_t span = contiguous ? ((int64_t)(wpb - 1) * stride + window) * A : (int64_t)wpb * window * A;
    return (PAD + 4 + span + SLACK) * (int64_t)sizeof(float);
  };
  // waves per block: 4 * waves groups must be whole windows (T3 = 3: three waves = four windows);
  // otherwise the most waves whose span stays within 64 KB (three or more blocks per CU)
  int waves = 0;
  if constexpr (T3 == 3) {
    if (lds_bytes(4) <= 160 * 1024) waves = 3;
  } else {
    for (int w = 4; w >= 1 && !waves; w >>= 1)
      if (lds_bytes(4 * w / T3) <= 64 * 1024 || (w == 1 && lds_bytes(4 / T3) <= 160 * 1024)) waves = w;
  }
  if (!waves) return -5;  // one block's windows do not fit the LDS
  const int wpb = 4 * waves / T3;
  const int64_t blocks = (n_windows + wpb - 1) / wpb;
  window_features_kernel<A, MLP><<<(unsigned)blocks, 64 * waves, (size_t)lds_bytes(wpb), s>>>(
      stream, n_samples, window, stride, n_windows, ms, out, ld_out, mo);
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
