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
//     (one v_lshl_add_u64 per sample) and the local maxima as a shift register of flags,
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
#include <algorithm>
#include <type_traits>

#include "common.h"
#include "mlp_frag.h"
#include "../har_kernels.h"

// A/B switch for probes: the pre-v3 kernels only (window_features_kernel / _persistent_kernel)
bool g_window_legacy = false;

namespace {

constexpr int MAXA = 9;
constexpr int NB = 10;
constexpr int PAD = 12;    // floats of LDS before the staged span: the t = -1 neighbour read stays inside
constexpr int SLACK = 16;  // floats after it: the t = W neighbour read of the last window stays inside
// floats of the register kernel's MLP-mode normalization image (F means + F inverse std devs, 16-byte rounded)
__host__ __device__ constexpr int reg_nrm_floats(int A) { return (2 * (17 * A + 4 * (A / 3)) + 3) & ~3; }

typedef float v4f __attribute__((ext_vector_type(4)));

// Reductions over one group of LPW = 8 or 16 lanes; every lane ends with the group's result.
// quad_perm xor-1, quad_perm xor-2, then row_half_mirror (and row_mirror for 16 lanes): after
// the quad steps every lane of a quad holds the quad's value, so the mirrors pair whole quads,
// then whole half-rows.
template <int CTRL> __device__ __forceinline__ int dpp_i(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
}
template <int LPW, typename T, typename Op> __device__ __forceinline__ T rreduce(T v, Op op) {
  static_assert(LPW == 8 || LPW == 16, "window groups of 8 or 16 lanes");
  auto mv = [](T x, auto ctrl) {
    constexpr int C = decltype(ctrl)::value;
    if constexpr (sizeof(T) == 4 && (T)0.5f != 0) return __int_as_float(dpp_i<C>(__float_as_int(x)));
    else return (T)dpp_i<C>((int)x);
  };
  v = op(v, mv(v, std::integral_constant<int, 0xB1>{}));   // xor 1
  v = op(v, mv(v, std::integral_constant<int, 0x4E>{}));   // xor 2
  v = op(v, mv(v, std::integral_constant<int, 0x141>{}));  // row_half_mirror: quad <-> quad
  if constexpr (LPW == 16) v = op(v, mv(v, std::integral_constant<int, 0x140>{}));  // row_mirror: half-row <-> half-row
  return v;
}
template <int LPW> __device__ __forceinline__ float rsum(float v) {
  return rreduce<LPW, float>(v, [](float a, float b) { return a + b; });
}
template <int LPW> __device__ __forceinline__ uint32_t rsumu(uint32_t v) {
  return rreduce<LPW, uint32_t>(v, [](uint32_t a, uint32_t b) { return a + b; });
}
template <int LPW> __device__ __forceinline__ float rmin(float v) {
  return rreduce<LPW, float>(v, [](float a, float b) { return fminf(a, b); });
}
template <int LPW> __device__ __forceinline__ float rmax(float v) {
  return rreduce<LPW, float>(v, [](float a, float b) { return fmaxf(a, b); });
}
template <int LPW> __device__ __forceinline__ int rmini(int v) {
  return rreduce<LPW, int>(v, [](int a, int b) { return min(a, b); });
}
template <int LPW> __device__ __forceinline__ int rmaxi(int v) {
  return rreduce<LPW, int>(v, [](int a, int b) { return max(a, b); });
}

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
  uint32_t pk[3];   // shift register of peak flags: bit j <-> iteration kbase + n - 1 - j of an n-iteration chunk
  uint32_t hw[3][5];  // flushed counts, two 16-bit bins per word
  int npk[3], first[3], last[3];
};

// One iteration of pass 2 at sample t.  EDGE iterations (the first, and those reaching t >= W - 1)
// mask samples past the window and exclude t = 0 / t = W - 1 from the peaks.
template <int A, bool EDGE>
__device__ __forceinline__ void pass2_step(const float* img, int t, int W, const Pass2K& K, Pass2Acc& a) {
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
    a.pk[c] = (a.pk[c] << 1) + (peak ? 1u : 0u);  // one v_addc (pk + pk + carry)
  }
  const float r = __builtin_amdgcn_sqrtf(fmaf(v[0], v[0], fmaf(v[1], v[1], v[2] * v[2])));  // v_sqrt_f32, no denormal scaling
  a.res += (EDGE && !ok) ? 0.f : r;
  a.cxy = fmaf(d[0], d[1], a.cxy);
  a.cxz = fmaf(d[0], d[2], a.cxz);
  a.cyz = fmaf(d[1], d[2], a.cyz);
}

// fold the packed counts and peak bits of the n-iteration chunk starting at kbase
template <int LPW> __device__ __forceinline__ void pass2_flush(Pass2Acc& a, int sub, int kbase, int n) {
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const uint64_t h = a.h[c];
#pragma unroll
    for (int j = 0; j < 5; ++j)
      a.hw[c][j] += (uint32_t)((h >> (12 * j)) & 63) | ((uint32_t)((h >> (12 * j + 6)) & 63) << 16);
    a.h[c] = 0;
    const uint32_t pk = a.pk[c];
    a.npk[c] += __builtin_popcount(pk);
    const int f = sub + LPW * (kbase + n - 1 - (31 - __builtin_clz(pk | 1u)));  // oldest flag: highest bit
    const int l = sub + LPW * (kbase + n - 1 - __builtin_ctz(pk | 0x80000000u));  // newest: lowest bit
    a.first[c] = pk ? min(a.first[c], f) : a.first[c];
    a.last[c] = pk ? max(a.last[c], l) : a.last[c];
    a.pk[c] = 0;
  }
}

// The statistics of every (window, triad) group of one staged batch: `img0` holds windows
// w0 .. w0 + nwin - 1, `pitch` floats apart.
template <int A, int LPW, bool MLP>
__device__ __forceinline__ void window_groups(const float* img0, int64_t w0, int nwin, int W, int pitch,
                                              float ms_per_sample, float* __restrict__ out, int ld_out,
                                              const MlpOut& mo) {
  constexpr int T3 = A / 3, GPW = 64 / LPW;
  const int tid = (int)threadIdx.x;
  const int lane = tid & 63, sub = lane % LPW;
  const int wave = tid >> 6, g = wave % T3;
  const int wi = GPW * (wave / T3) + lane / LPW;
  const bool valid = wi < nwin;
  const int64_t win = w0 + (valid ? wi : 0);
  const float* img = img0 + (valid ? wi : 0) * pitch + 3 * g;  // the group's triad: A floats per sample
  const int C = (W + LPW - 1) / LPW;  // iterations (samples per lane, the last partial)
  const int kfull = (W - 1) / LPW;    // k < kfull: every t = sub + LPW k lies in [0, W - 2]
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
    for (; k < kfull; ++k, p += LPW * A) {
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const float v = p[c];
        s[c] += v; q[c] = fmaf(v, v, q[c]); lo[c] = fminf(lo[c], v); hi[c] = fmaxf(hi[c], v);
      }
    }
    for (; k < C; ++k) {
      const int t = sub + LPW * k;
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
      mean[c] = rsum<LPW>(s[c]) * invW; en[c] = rsum<LPW>(q[c]) * invW;
      mn[c] = rmin<LPW>(lo[c]); mx[c] = rmax<LPW>(hi[c]);
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
  pass2_step<A, true>(img, sub, W, K, a);  // k = 0 holds t = 0
  int k = 1;
#pragma unroll 2
  for (; k < kfull; ++k) {
    pass2_step<A, false>(img, sub + LPW * k, W, K, a);
    if ((k & 31) == 31) pass2_flush<LPW>(a, sub, k - 31, 32);
  }
  for (; k < C; ++k) {
    pass2_step<A, true>(img, sub + LPW * k, W, K, a);
    if ((k & 31) == 31) pass2_flush<LPW>(a, sub, k - 31, 32);
  }
  if (C & 31) pass2_flush<LPW>(a, sub, C & ~31, C & 31);

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
      for (int f = F + sub; f < ld_out; f += LPW)
        if (valid) ob[f] = 0;
  }
  const int off_avg = A * NB, off_peak = off_avg + A, off_abs = off_peak + A, off_std = off_abs + A;
  const int off_res = off_std + A, off_min = off_res + T3, off_max = off_min + A, off_en = off_max + A;
  const int off_corr = off_en + A;
  float sd[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const int ax = 3 * g + c;
    // a constant axis (max == min) has exactly zero spread: its fp32 mean need not equal the sample, so
    // the deviation sums need not cancel (a clipped, saturated sensor gave correlations of +-1 for 0)
    const bool flat = !(mx[c] > mn[c]);
    const float ad = flat ? 0.f : rsum<LPW>(a.ad[c]) * invW;
    const float var = rsum<LPW>(a.v2[c]) * invW;
    sd[c] = flat ? 0.f : __builtin_amdgcn_sqrtf(var);
    const int npk = (int)rsumu<LPW>((uint32_t)a.npk[c]);
    const int first = rmini<LPW>(a.first[c]), last = rmaxi<LPW>(a.last[c]);
    // bins: lane `sub` writes bin `sub` (and lanes 0, 1 of 8-lane groups bins 8, 9); the word is
    // picked by a select chain, not an indexed register array
    uint32_t hw[5];
#pragma unroll
    for (int j = 0; j < 5; ++j) hw[j] = rsumu<LPW>(a.hw[c][j]);
    {
      uint32_t word = hw[0];
#pragma unroll
      for (int j = 1; j < 5; ++j) word = (sub >> 1) == j ? hw[j] : word;
      const uint32_t cnt = (sub & 1) ? word >> 16 : word & 0xffffu;
      emit(sub < NB, ax * NB + sub, (float)cnt * invW);
    }
    if constexpr (LPW < NB) {
      const uint32_t cnt = (sub & 1) ? hw[4] >> 16 : hw[4] & 0xffffu;
      emit(sub < NB - LPW, ax * NB + LPW + sub, (float)cnt * invW);
    }
    // scalars: lanes 0..6
    const float peak =
        npk >= 2 ? (float)(last - first) * __builtin_amdgcn_rcpf((float)(npk - 1)) * ms_per_sample : NAN;
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
    const float res = rsum<LPW>(a.res) * invW;
    const float cxy = rsum<LPW>(a.cxy) * invW, cxz = rsum<LPW>(a.cxz) * invW, cyz = rsum<LPW>(a.cyz) * invW;
    const float rxy = (sd[0] > 0.f && sd[1] > 0.f) ? cxy * __builtin_amdgcn_rcpf(sd[0] * sd[1]) : 0.f;
    const float rxz = (sd[0] > 0.f && sd[2] > 0.f) ? cxz * __builtin_amdgcn_rcpf(sd[0] * sd[2]) : 0.f;
    const float ryz = (sd[1] > 0.f && sd[2] > 0.f) ? cyz * __builtin_amdgcn_rcpf(sd[1] * sd[2]) : 0.f;
    float v = res;
    int f = off_res + g;
    v = sub == 1 ? rxy : v;  f = sub == 1 ? off_corr + 3 * g : f;
    v = sub == 2 ? rxz : v;  f = sub == 2 ? off_corr + 3 * g + 1 : f;
    v = sub == 3 ? ryz : v;  f = sub == 3 ? off_corr + 3 * g + 2 : f;
    emit(sub < 4, f, v);
  }
}

// One block = `waves` waves = 4 * waves groups = 4 * waves / (A / 3) whole windows (host picks
// `waves` as a multiple of A / 3).  Wave v takes triad v % (A / 3) of the four windows
// 4 (v / (A / 3)) .. + 3, one per row.  Every window gets its own LDS image, `pitch` floats apart:
// with pitch = 16 A (mod 64) dwords the four rows of a wave (same triad, consecutive images)
// read disjoint bank sets — lane banks A * sub + r * pitch are distinct over the 64 lanes for odd A
// (the host picks the pitch).  One-shot: stage, compute, write.
template <int A, int LPW, bool MLP>
__global__ __launch_bounds__(256) void window_features_kernel(const float* __restrict__ stream, int64_t n_samples,
                                                              int W, int stride, int64_t n_windows,
                                                              float ms_per_sample, float* __restrict__ out,
                                                              int ld_out, MlpOut mo, int pitch) {
  constexpr int T3 = A / 3, GPW = 64 / LPW;  // groups per wave
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int nt = (int)blockDim.x, tid = (int)threadIdx.x;
  const int wpb = (nt >> 6) * GPW / T3;
  const int64_t w0 = (int64_t)blockIdx.x * wpb;
  const int nwin = (int)min<int64_t>(wpb, n_windows - w0);
  float* img0 = lds + PAD;
  // ---- stage the block's windows in LDS ----
  const int n = W * A;
  if ((reinterpret_cast<uintptr_t>(stream) & 15) == 0 && ((int64_t)stride * A) % 4 == 0 &&
      (int64_t)stride * A * nwin < 0x7fffffff) {
    // every window starts on a float4: 16-byte loads, eight in flight per thread
    const int64_t t4 = n_samples * A >> 2;  // whole float4s of the stream
    const int n4 = (n + 3) >> 2;            // float4s per window (the last may run past it: pitch >= that)
    const int tot = nwin * n4;
    const v4f* s4 = reinterpret_cast<const v4f*>(stream);
    const int64_t g40 = w0 * stride * A >> 2;
    const int gs4 = stride * A >> 2;
    const int p4 = pitch >> 2;
    v4f* d4 = reinterpret_cast<v4f*>(img0);
    // flat float4 index f -> (window i, float4 j): i = umulhi(f, magic) is exact for f * n4 < 2^32
    const uint32_t magic = 0xffffffffu / (uint32_t)n4 + 1u;
    const int64_t lim = t4 - g40;  // relative float4 indices at or past this are outside the stream
    const int rlim = (int)min<int64_t>(lim, 0x7fffffff);
    const v4f* sb = s4 + g40;
    for (int f0 = tid; f0 < tot; f0 += 8 * nt) {
      v4f r[8];
      int rel[8], di[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int f = f0 + u * nt;
        const int i = (int)__umulhi((uint32_t)f, magic), j = f - i * n4;
        rel[u] = i * gs4 + j;
        di[u] = i * p4 + j;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) r[u] = sb[rel[u] < rlim ? rel[u] : rlim - 1];  // unconditional (clamped) loads
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (f0 + u * nt < tot && rel[u] < rlim) d4[di[u]] = r[u];
    }
    // floats past the stream's last whole float4 (n_samples * A % 4 != 0): the last window only
    const int64_t last0 = (w0 + nwin - 1) * stride * A;
    for (int64_t e = max(t4 * 4, last0) + tid; e < last0 + n; e += nt) img0[(nwin - 1) * pitch + (e - last0)] = stream[e];
  } else {
    for (int i = 0; i < nwin; ++i) {
      const float* src = stream + (w0 + i) * stride * A;
      for (int e = tid; e < n; e += nt) img0[i * pitch + e] = src[e];
    }
  }
  __syncthreads();

  window_groups<A, LPW, MLP>(img0, w0, nwin, W, pitch, ms_per_sample, out, ld_out, mo);
}

// Persistent variant (16-byte aligned window starts): each block walks batches b, b + grid, ...
// of `wpb` windows.  The NEXT batch is loaded into NR float4 registers per thread while the
// current one is computed from LDS, so the HBM latency of a batch hides behind the statistics of
// the previous one instead of being paid by every block up front (one-shot blocks: stage, then
// compute, with only four or two blocks per CU).  Loads are unconditional (clamped into the
// stream) so their waits stay counted; the host picks NR >= float4s per batch / threads.
template <int A, int LPW, bool MLP, int NR>
__global__ __launch_bounds__(256) void window_features_persistent_kernel(
    const float* __restrict__ stream, int64_t n_samples, int W, int stride, int64_t n_windows, float ms_per_sample,
    float* __restrict__ out, int ld_out, MlpOut mo, int pitch) {
  constexpr int T3 = A / 3, GPW = 64 / LPW;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int nt = (int)blockDim.x, tid = (int)threadIdx.x;
  const int wpb = (nt >> 6) * GPW / T3;
  const int64_t nbatch = (n_windows + wpb - 1) / wpb;
  float* img0 = lds + PAD;
  v4f* d4 = reinterpret_cast<v4f*>(img0);
  const int n = W * A, n4 = (n + 3) >> 2, p4 = pitch >> 2, gs4 = stride * A >> 2;
  // non-overlapping windows with unpadded images: float4 f of a batch is float4 f of its image
  // span in the stream AND in LDS — no (window, offset) split per float4
  const bool flat = stride == W && pitch == n;
  const int64_t t4 = n_samples * A >> 2;  // whole float4s of the stream
  const v4f* s4 = reinterpret_cast<const v4f*>(stream);
  const uint32_t magic = 0xffffffffu / (uint32_t)n4 + 1u;  // f / n4 = umulhi(f, magic) for f * n4 < 2^32
  const int totmax = wpb * n4;
  int64_t b = blockIdx.x;
  if (b >= nbatch) return;  // block-uniform; no barrier reached
  // (stream, LDS) float4 offsets of this thread's u-th float4 of a batch; slots past the batch
  // re-load slot 0 (cache hits).  Recomputed per use behind an opaque copy of tid: held, they
  // would cost two VGPRs per float4.
  int tid_ = tid;
  auto offs = [&](int u, int& rel, int& di) {
    const int f0 = tid_ + u * nt, f = f0 < totmax ? f0 : tid_;
    if (flat) {
      rel = f; di = f;
    } else {
      const int i = (int)__umulhi((uint32_t)f, magic), j = f - i * n4;
      rel = i * gs4 + j; di = i * p4 + j;
    }
  };
  auto base = [&](int64_t batch, int& rlim) {
    const int64_t g40 = batch * wpb * (int64_t)stride * A >> 2;
    rlim = (int)min<int64_t>(t4 - g40, 0x7fffffff);
    return s4 + g40;
  };
  v4f r[NR];
  {
    asm volatile("" : "+v"(tid_));
    int rlim;
    const v4f* sb = base(b, rlim);
#pragma unroll
    for (int u = 0; u < NR; ++u) {
      int rel, di;
      offs(u, rel, di);
      r[u] = sb[rel < rlim ? rel : rlim - 1];  // unconditional (clamped) loads: counted waits
    }
  }
  for (; b < nbatch; b += gridDim.x) {
    const int64_t w0 = b * wpb;
    const int nwin = (int)min<int64_t>(wpb, n_windows - w0);
    const int tot = nwin * n4;
    const bool more = b + gridDim.x < nbatch;
    {
      asm volatile("" : "+v"(tid_));
      int rlim, rlim_n;
      base(b, rlim);
      const v4f* sbn = base(more ? b + gridDim.x : b, rlim_n);
      // store this batch's float4 u, then reuse its registers for the next batch's float4 u (the
      // last batch re-loads itself: cache hits)
#pragma unroll
      for (int u = 0; u < NR; ++u) {
        int rel, di;
        offs(u, rel, di);
        if (tid + u * nt < tot && rel < rlim) d4[di] = r[u];
        r[u] = sbn[rel < rlim_n ? rel : rlim_n - 1];  // unconditional: a conditional load would drain vmcnt
      }
      // floats past the stream's last whole float4 (n_samples * A % 4 != 0): the last window only
      const int64_t last0 = (w0 + nwin - 1) * stride * A;
      for (int64_t e = max(t4 * 4, last0) + tid; e < last0 + n; e += nt)
        img0[(nwin - 1) * pitch + (e - last0)] = stream[e];
    }
    __syncthreads();
    window_groups<A, LPW, MLP>(img0, w0, nwin, W, pitch, ms_per_sample, out, ld_out, mo);
    __syncthreads();  // every wave is done with the images before they are overwritten
  }
}

// ------------------------------------------------------------------------------------------------
// Register-resident variant: a group of LPW = 16 / 32 / 64 lanes per (window, triad), lane `sub`
// owning the CONTIGUOUS run of C samples t = sub*C .. sub*C + C - 1 (C odd, LPW*C >= W), read once
// from LDS into registers.  Both passes then run on registers: the neighbours of the peak test are
// the lane's own x[k-1] / x[k+1] (only the run's first prev comes from LDS, and the run's last
// "rising" bit from the next lane), so a sample costs one LDS read per axis instead of four, and no
// pass carries a per-sample mask: the run positions past the window hold copies of sample W - 1,
// whose contributions are subtracted once per window (D = LPW*C - W of them), and the peak bits
// of t = 0 / t >= W - 1 are cleared with one per-lane mask.  The block stages the CONTIGUOUS
// sample span of its windows (overlapping windows share it), so a batch of stride < W windows
// reads every sample once.  One-shot blocks, several per CU: the loads of one block overlap the
// arithmetic of the others.
// ------------------------------------------------------------------------------------------------
constexpr int RCMAX_LONG = 31;  // samples per lane held in registers (C <= 31: the flag words hold C bits);
                                // runs of C <= 17 use a 17-register instantiation (fewer VGPRs)

// reduction over a group of LPW = 8 / 16 / 32 / 64 lanes: 8- / 16-lane DPP butterflies, then the
// gfx950 row (lane ^ 16) and half (lane ^ 32) swaps on the VALU.  A swap of v with itself leaves
// {own, partner} in its two outputs (which is which depends on the lane's row / half), so the
// commutative op takes both outputs directly: no select of the partner
template <int LPW, typename T, typename Op>
__device__ __forceinline__ T greduce(T v, Op op, const mlpf::LaneSwap&) {
  v = rreduce<(LPW < 16 ? LPW : 16), T>(v, op);
  if constexpr (LPW >= 32) {
    const uint32_t u = __builtin_bit_cast(uint32_t, v);
    const auto r = __builtin_amdgcn_permlane16_swap(u, u, false, false);
    v = op(__builtin_bit_cast(T, (uint32_t)r[0]), __builtin_bit_cast(T, (uint32_t)r[1]));
  }
  if constexpr (LPW >= 64) {
    const uint32_t u = __builtin_bit_cast(uint32_t, v);
    const auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
    v = op(__builtin_bit_cast(T, (uint32_t)r[0]), __builtin_bit_cast(T, (uint32_t)r[1]));
  }
  return v;
}

// min / max as one v_min_f32 / v_max_f32: fminf / fmaxf make hipcc quiet BOTH operands first in
// IEEE mode (a v_max_f32 x, x each, also on the running accumulator across the guarded k-steps:
// 6 VALU per sample and axis for min + max instead of 2; fmed3 with an infinity folds back to that);
// the samples are finite sensor data
__device__ __forceinline__ float vmin(float a, float b) {
  float r;
  asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ float vmax(float a, float b) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
// three-operand forms: pass 1 folds two run samples into the running min / max per instruction
__device__ __forceinline__ float vmin3(float a, float b, float c) {
  float r;
  asm("v_min3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ float vmax3(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// One sample's peak flags into the two shift registers: R = 2R + (x > prev), PT = 2PT + (x > prev &&
// x > thr), as two compares into SGPR masks and two v_addc (R + R + carry); written by hipcc it is a
// v_cndmask + v_lshl_or per flag
__device__ __forceinline__ void flag_step(uint32_t& R, uint32_t& PT, float x, float prev, float thr) {
  uint64_t m1, m2, cc;
  asm("v_cmp_gt_f32_e64 %[m1], %[x], %[p]\n\t"
      "v_cmp_gt_f32_e64 %[m2], %[x], %[t]\n\t"
      "s_and_b64 %[m2], %[m1], %[m2]\n\t"
      "v_addc_co_u32_e64 %[R], %[cc], %[R], %[R], %[m1]\n\t"
      "v_addc_co_u32_e64 %[PT], %[cc], %[PT], %[PT], %[m2]"
      : [R] "+v"(R), [PT] "+v"(PT), [m1] "=&s"(m1), [m2] "=&s"(m2), [cc] "=&s"(cc)
      : [x] "v"(x), [p] "v"(prev), [t] "v"(thr)
      : "scc");
}

// bin of a sample: (x - lo) * (10 / range) in fp32, the legacy kernel's arithmetic (x >= lo, so the
// conversion never sees a negative), clamped to bin 9.  (The one-fma form x sc + (-lo sc), one VALU less
// per sample and axis, moved boundary samples of quantized sensor data — WISDM's 2-decimal readings sit
// exactly on bin edges — off the float64 definition's bins: tests/test_raw.py; rejected)
__device__ __forceinline__ uint32_t bin_raw(float x, float sc, float lo) { return (uint32_t)((x - lo) * sc); }
__device__ __forceinline__ uint32_t bin_of(float x, float sc, float lo) {
  const uint32_t b = (uint32_t)((x - lo) * sc);
  return b < (uint32_t)(NB - 1) ? b : (uint32_t)(NB - 1);
}

// P32: non-overlapping windows (stride == W) with 32-sample runs (C = 32, even): every window gets its
// own LDS image with a 4-float pad after each 32 samples (sample t at t A + 4 (t >> 5)), so the lanes of a
// group, 32 A + 4 floats apart, still read distinct banks (an unpadded 32 A stride would put 16 lanes on
// 2 - 4 banks).  The pads keep every float4 of the copy 16-byte aligned (32 A is a multiple of 4).  It
// lets a 500-sample 9-axis window run on 16-lane groups (16 x 32 >= 500) instead of 32 x 17.
__host__ __device__ constexpr int p32_pos(int t, int A) { return t * A + 4 * (t >> 5); }
__host__ __device__ inline int p32_pitch(int W, int A) { return (p32_pos(W, A) + 4 + 3) & ~3; }

// The statistics of one staged batch (windows w0 .. w0 + nwin - 1, their samples at `span`, `ip` floats
// per window image): each lane reads its run into registers, then both passes, the reductions and the
// row write.
template <int A, int LPW, bool MLP, int RCMAX, bool P32, bool FIXC>
__device__ __forceinline__ void reg_window_batch(const float* span, int64_t w0, int nwin, int W, int ip, int C,
                                                 float ms_per_sample, float* __restrict__ out, int ld_out,
                                                 const MlpOut& mo, const float* nrm) {
  constexpr int T3 = A / 3, GPW = 64 / LPW;
  const int tid = (int)threadIdx.x;
  auto pos = [&](int t) { return P32 ? p32_pos(t, A) : t * A; };
  const int lane = tid & 63;
  const int wave = tid >> 6, sub = lane % LPW;
  const int g = wave % T3;
  const int wi = GPW * (wave / T3) + lane / LPW;
  const bool valid = wi < nwin;
  const int64_t win = w0 + (valid ? wi : 0);
  const float* img = span + (valid ? wi : 0) * ip + 3 * g;  // the group's triad
  const mlpf::LaneSwap sw(lane);
  const int tb = sub * C;
  const float invW = 1.f / (float)W;
  const float D = (float)(LPW * C - W);  // copies of sample W - 1 in the runs

  // Runtime C <= RCMAX: every k-step is guarded by the uniform k < C, which also keeps the
  // scheduler from hoisting all 3*RCMAX loads and their consumers at once (register pressure)
  float x[3][RCMAX];
  // FIXC: the run read unclamped from one base address (immediate LDS offsets — the clamped form cost a
  // 24-bit multiply, a min and a 64-bit address multiply-add per sample); run positions past W - 1 read
  // the span's next samples or its slack (sized by the launcher) and get the copies of sample W - 1 below
  constexpr bool FLAT = FIXC && !P32;
#pragma unroll
  for (int k = 0; k < RCMAX; ++k)
    if (k < C) {
      const float* p = FLAT ? img + (tb + k) * A : img + pos(min(tb + k, W - 1));
#pragma unroll
      for (int c = 0; c < 3; ++c) x[c][k] = p[c];
    }
  float xl[3], pv0[3];
  {
    const float* pl = img + pos(W - 1);
    // sample before the run (t = -1: the PAD / previous window; P32: sample 0 — lane 0's t = 0 peak
    // bit is masked either way)
    const float* pp = img + (P32 ? pos(max(min(tb, W) - 1, 0)) : (min(tb, W) - 1) * A);
#pragma unroll
    for (int c = 0; c < 3; ++c) { xl[c] = pl[c]; pv0[c] = pp[c]; }
  }
  if constexpr (FLAT) {
    if (LPW * RCMAX != W) {  // (uniform: runs that overhang the window; none at W = LPW C)
#pragma unroll
      for (int k = 0; k < RCMAX; ++k) {
        const bool over = tb + k > W - 1;
#pragma unroll
        for (int c = 0; c < 3; ++c) x[c][k] = over ? xl[c] : x[c][k];
      }
    }
  }

  // ---- pass 1 ----
  float mean[3], mn[3], mx[3], en[3];
  {
    float s[3], q[3], lo[3], hi[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) { s[c] = 0.f; q[c] = 0.f; lo[c] = x[c][0]; hi[c] = x[c][0]; }
#pragma unroll
    for (int k = 0; k < RCMAX; ++k)
      if (k < C) {
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const float v = x[c][k];
          s[c] += v; q[c] = fmaf(v, v, q[c]);
        }
      }
    // min / max: samples 1, 2 | 3, 4 | ... in one v_min3 / v_max3 each (sample 0 is the seed)
#pragma unroll
    for (int k = 1; k < RCMAX; k += 2) {
      if (k + 1 < RCMAX && k + 1 < C) {
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          lo[c] = vmin3(lo[c], x[c][k], x[c][k + 1]);
          hi[c] = vmax3(hi[c], x[c][k], x[c][k + 1]);
        }
      } else if (k < C) {
#pragma unroll
        for (int c = 0; c < 3; ++c) { lo[c] = vmin(lo[c], x[c][k]); hi[c] = vmax(hi[c], x[c][k]); }
      }
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float S = greduce<LPW, float>(s[c], [](float a, float b) { return a + b; }, sw) - D * xl[c];
      const float Q = greduce<LPW, float>(q[c], [](float a, float b) { return a + b; }, sw) - D * xl[c] * xl[c];
      mean[c] = S * invW; en[c] = Q * invW;
      mn[c] = greduce<LPW, float>(lo[c], [](float a, float b) { return vmin(a, b); }, sw);
      mx[c] = greduce<LPW, float>(hi[c], [](float a, float b) { return vmax(a, b); }, sw);
    }
  }

  // ---- pass 2 ----
  float sc[3], off[3], thr[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float range = mx[c] - mn[c];
    sc[c] = range > 0.f ? (float)NB / range : 0.f;
    off[c] = mn[c];  // bin_of's lo
    thr[c] = mean[c] + 0.5f * (mx[c] - mean[c]);
  }
  float ad[3] = {0.f, 0.f, 0.f}, v2[3] = {0.f, 0.f, 0.f}, res = 0.f, cxy = 0.f, cxz = 0.f, cyz = 0.f;
  // per-lane bin counts packed SB bits per slot: runs of C <= 31 samples fit 5 bits, so the 11 slots of
  // an unclamped bin (0..10: (x - lo) * sc reaches 10 only at x == max) fit 55 bits and the clamp to
  // bin 9 happens once per window (slot 10 folded into bin 9) instead of once per sample
  constexpr int SB = RCMAX <= 31 ? 5 : 6;
  const auto slot = [](uint64_t hh, int j) { return (uint32_t)(hh >> (SB * j)) & ((1u << SB) - 1u); };
  uint64_t h[3] = {0, 0, 0};
  uint32_t R[3] = {0, 0, 0}, PT[3] = {0, 0, 0};  // bit j <-> run sample k = C - 1 - j
#pragma unroll
  for (int k = 0; k < RCMAX; ++k)
    if (k < C) {
      float d[3];
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const float xv = x[c][k], pv = k ? x[c][k - 1] : pv0[c];
        const float dc = xv - mean[c];
        d[c] = dc;
        ad[c] += fabsf(dc);
        v2[c] = fmaf(dc, dc, v2[c]);
        // v_mul_u32_u24, not the quarter-rate mul_lo; 5-bit slots take the unclamped bin (slot 10: x == max)
        h[c] += 1ull << __umul24(SB == 5 ? bin_raw(xv, sc[c], off[c]) : bin_of(xv, sc[c], off[c]), (uint32_t)SB);
        flag_step(R[c], PT[c], xv, pv, thr[c]);
      }
      res += __builtin_amdgcn_sqrtf(fmaf(x[0][k], x[0][k], fmaf(x[1][k], x[1][k], x[2][k] * x[2][k])));
      cxy = fmaf(d[0], d[1], cxy);
      cxz = fmaf(d[0], d[2], cxz);
      cyz = fmaf(d[1], d[2], cyz);
      // (fixed-length runs: pin the resultant sum to its k-step — left free, LLVM sinks every square root
      // past the reductions and keeps all 75 run samples alive there: 65 spilled VGPRs)
      if constexpr (FIXC) asm volatile("" : "+v"(res));
    }

  // a constant axis (max == min: its bin scale sc is 0) has exactly zero spread, but its fp32 mean need
  // not equal the sample, so the deviation sums need not cancel (a clipped, saturated sensor gave
  // correlations of +-1 for 0): its per-lane deviation sums are zeroed before the reductions
  {
    const bool f0 = sc[0] == 0.f, f1 = sc[1] == 0.f, f2 = sc[2] == 0.f;
    ad[0] = f0 ? 0.f : ad[0]; v2[0] = f0 ? 0.f : v2[0];
    ad[1] = f1 ? 0.f : ad[1]; v2[1] = f1 ? 0.f : v2[1];
    ad[2] = f2 ? 0.f : ad[2]; v2[2] = f2 ? 0.f : v2[2];
    cxy = (f0 || f1) ? 0.f : cxy; cxz = (f0 || f2) ? 0.f : cxz; cyz = (f1 || f2) ? 0.f : cyz;
  }

  // peak positions: 0 < t < W - 1 (t = tb + k), i.e. bits j in [C - 1 - kh, C - 1 - kl]
  const int kl = sub == 0 ? 1 : 0, kh = min(C - 1, W - 2 - tb);
  const uint32_t pmask =
      kh >= kl ? (uint32_t)(((1ull << (C - kl)) - 1ull) & ~((1ull << (C - 1 - kh)) - 1ull)) : 0u;  // (C <= 32)

  // ---- reduce + write ----
  float* o = MLP ? nullptr : out + win * (int64_t)ld_out;
  uint16_t* ob = MLP ? mo.out + win * (int64_t)ld_out : nullptr;
  auto emit = [&](bool on, int f, float v) {
    if (!(on && valid)) return;
    if constexpr (MLP) {
      const float xv = v != v ? mo.nan_value : v;
      ob[f] = f2bf((xv - nrm[f]) * nrm[17 * A + 4 * T3 + f]);  // (the staged means / inverse std devs)
    } else {
      o[f] = v;
    }
  };
  constexpr int F = 17 * A + 4 * T3;
  if constexpr (MLP) {  // zero the pad columns of the row (triad 0's group)
    if (g == 0 && valid)
      for (int f = F + sub; f < ld_out; f += LPW) ob[f] = 0;
  }
  const int off_avg = A * NB, off_peak = off_avg + A, off_abs = off_peak + A, off_std = off_abs + A;
  const int off_res = off_std + A, off_min = off_res + T3, off_max = off_min + A, off_en = off_max + A;
  const int off_corr = off_en + A;
  const auto fsum = [](float a, float b) { return a + b; };
  const auto usum = [](uint32_t a, uint32_t b) { return a + b; };
  float sd[3], dl[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const int ax = 3 * g + c;
    dl[c] = sc[c] == 0.f ? 0.f : xl[c] - mean[c];  // (a constant axis: no deviation, see above)
    const float adv = (greduce<LPW, float>(ad[c], fsum, sw) - D * fabsf(dl[c])) * invW;
    const float var = fmaxf(greduce<LPW, float>(v2[c], fsum, sw) - D * dl[c] * dl[c], 0.f) * invW;
    sd[c] = __builtin_amdgcn_sqrtf(var);
    // the next lane's first rising bit closes this lane's run (the group's last lane: masked)
    const uint32_t rC = (uint32_t)__shfl((int)(R[c] >> (C - 1)) & 1, (lane + 1) & 63, 64);
    const uint32_t P = PT[c] & ~((R[c] << 1) | rC) & pmask;
    const int npk = (int)greduce<LPW, uint32_t>((uint32_t)__builtin_popcount(P), usum, sw);
    const int first = greduce<LPW, int>(P ? tb + C - 1 - (31 - __builtin_clz(P)) : 0x7fffffff,
                                         [](int a, int b) { return min(a, b); }, sw);
    const int last = greduce<LPW, int>(P ? tb + C - 1 - __builtin_ctz(P) : -1, [](int a, int b) { return max(a, b); }, sw);
    // bins: packed 6-bit counts -> five words of two 16-bit bins; lane `sub` < NB writes bin `sub`
    uint32_t hw[5];
#pragma unroll
    for (int j = 0; j < 5; ++j)
      hw[j] = greduce<LPW, uint32_t>(slot(h[c], 2 * j) | (slot(h[c], 2 * j + 1) + (j == 4 && SB == 5 ? slot(h[c], 10) : 0u)) << 16,
                                     usum, sw);
    // lane `sub` writes bin `sub` (and bin sub + 8 for 8-lane groups)
#pragma unroll
    for (int b0 = 0; b0 < NB; b0 += LPW) {
      const int bn = b0 + sub;
      uint32_t word = hw[0];
#pragma unroll
      for (int j = 1; j < 5; ++j) word = (bn >> 1) == j ? hw[j] : word;
      uint32_t cnt = (bn & 1) ? word >> 16 : word & 0xffffu;
      cnt -= (uint32_t)bn == bin_of(xl[c], sc[c], off[c]) ? (uint32_t)(LPW * C - W) : 0u;
      emit(bn < NB, ax * NB + bn, (float)cnt * invW);
    }
    const float peak =
        npk >= 2 ? (float)(last - first) * __builtin_amdgcn_rcpf((float)(npk - 1)) * ms_per_sample : NAN;
    float v = mean[c];
    int f = off_avg + ax;
    v = sub == 1 ? peak : v;       f = sub == 1 ? off_peak + ax : f;
    v = sub == 2 ? adv : v;        f = sub == 2 ? off_abs + ax : f;
    v = sub == 3 ? sd[c] : v;      f = sub == 3 ? off_std + ax : f;
    v = sub == 4 ? mn[c] : v;      f = sub == 4 ? off_min + ax : f;
    v = sub == 5 ? mx[c] : v;      f = sub == 5 ? off_max + ax : f;
    v = sub == 6 ? en[c] : v;      f = sub == 6 ? off_en + ax : f;
    emit(sub < 7, f, v);
  }
  // triad: resultant (lane 0) and the three correlations (lanes 1..3)
  {
    const float rl = __builtin_amdgcn_sqrtf(fmaf(xl[0], xl[0], fmaf(xl[1], xl[1], xl[2] * xl[2])));
    const float rs = (greduce<LPW, float>(res, fsum, sw) - D * rl) * invW;
    const float sxy = (greduce<LPW, float>(cxy, fsum, sw) - D * dl[0] * dl[1]) * invW;
    const float sxz = (greduce<LPW, float>(cxz, fsum, sw) - D * dl[0] * dl[2]) * invW;
    const float syz = (greduce<LPW, float>(cyz, fsum, sw) - D * dl[1] * dl[2]) * invW;
    const float rxy = (sd[0] > 0.f && sd[1] > 0.f) ? sxy * __builtin_amdgcn_rcpf(sd[0] * sd[1]) : 0.f;
    const float rxz = (sd[0] > 0.f && sd[2] > 0.f) ? sxz * __builtin_amdgcn_rcpf(sd[0] * sd[2]) : 0.f;
    const float ryz = (sd[1] > 0.f && sd[2] > 0.f) ? syz * __builtin_amdgcn_rcpf(sd[1] * sd[2]) : 0.f;
    float v = rs;
    int f = off_res + g;
    v = sub == 1 ? rxy : v;  f = sub == 1 ? off_corr + 3 * g : f;
    v = sub == 2 ? rxz : v;  f = sub == 2 ? off_corr + 3 * g + 1 : f;
    v = sub == 3 ? ryz : v;  f = sub == 3 ? off_corr + 3 * g + 2 : f;
    emit(sub < 4, f, v);
  }
}

// (Rejected, same-box A/B in profiles/r6/window_global_reads_rejected.txt: the 8 x 25 runs read straight from
// global memory with no LDS staging — fp32 rows 2% faster, MLP rows, the 1B pass's mode, 2.5% slower.)
// (Rejected, same-box A/B in profiles/r6/window_rows_flags_rejected.txt: MLP rows assembled in the freed
// span and stored as 16-byte chunks — stride 100 unchanged, stride 200 +2 us (100 VGPRs: 4 waves per SIMD
// instead of 5); the peak bits as R & T with no per-sample s_and_b64 — no gain.)
// FIXC: the run length is RCMAX itself (a compile-time constant): no per-k-step `k < C` guards, whose
// compare + branch cost ~6 instructions per step and sample pass, and only the registers the runs use.
// (A persistent variant — the next batch's span copied HBM -> LDS by global_load_lds while the current one
// is computed from registers — measured slower on the stride-100 shape: 83 us with 4-wave and 103 us with
// 1-wave blocks vs 63 us one-shot at 131k windows, and 1.3x slower at 1.3M; and a register-prefetch
// persistent variant — the next span's 10 float4 per thread loaded right after the runs are read, stored to
// LDS after pass 2, 168 VGPRs at 3 waves per SIMD, no spills — 73 vs 62 us: one-shot blocks it is.)
template <int A, int LPW, bool MLP, int RCMAX, bool P32 = false, int WPE = 1, bool FIXC = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void window_features_reg_kernel(const float* __restrict__ stream, int W,
                                                                  int stride, int64_t n_windows, float ms_per_sample,
                                                                  float* __restrict__ out, int ld_out, MlpOut mo,
                                                                  int Carg, int wpb, int ipw) {
  const int C = FIXC ? RCMAX : Carg;
  static_assert(LPW == 8 || LPW == 16 || LPW == 32 || LPW == 64, "groups of 8, 16, 32 or 64 lanes");
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int nt = (int)blockDim.x, tid = (int)threadIdx.x;
  // MLP rows: the F means and inverse std devs staged in LDS ahead of the span (reg_nrm_floats), so the
  // row write reads them there instead of ~20 scattered global loads per lane at the kernel's end
  constexpr int NR = MLP ? reg_nrm_floats(A) : 0;
  float* const span = lds + NR + PAD;
  if constexpr (MLP) {
    constexpr int F = 17 * A + 4 * (A / 3);
    for (int f = tid; f < 2 * F; f += nt) lds[f] = f < F ? mo.mean[f] : mo.inv_std[f - F];
  }
  // image pitch (floats) between consecutive windows: P32 images, padded images (ipw > 0, non-overlapping
  // windows: a pitch of 16 mod 32 floats puts the two 16-lane windows of a 32-lane LDS bank group on
  // disjoint banks — the contiguous 600-float pitch of W = 200 x 3 axes had 32% bank-conflict cycles,
  // profiles/r5/window_pmc.md), or the shared span (stride A floats per window)
  const int ip = P32 ? p32_pitch(W, A) : ipw > 0 ? ipw : stride * A;

  const int64_t w0 = (int64_t)blockIdx.x * wpb;
  const int nwin = (int)min<int64_t>(wpb, n_windows - w0);
  // float4 loads in flight per thread while staging: 12 — a 4-wave block's ~2,470-float4 span (the
  // 200-sample shapes) is then ONE round of loads instead of two dependent ones
  constexpr int SU = 12;
  if (P32 || ipw > 0) {  // ---- stage the windows, one padded image each (float4 granules) ----
    const v4f* s4 = reinterpret_cast<const v4f*>(stream + w0 * (int64_t)W * A);
    const int n4w = W * A / 4, n4 = nwin * n4w;
    const uint32_t magic = 0xffffffffu / (uint32_t)n4w + 1u;  // f / n4w = umulhi(f, magic) for f * n4w < 2^32
    for (int f0 = tid; f0 < n4; f0 += SU * nt) {
      v4f r[SU];
#pragma unroll
      for (int u = 0; u < SU; ++u) r[u] = s4[min(f0 + u * nt, n4 - 1)];
#pragma unroll
      for (int u = 0; u < SU; ++u) {
        const int f = min(f0 + u * nt, n4 - 1), wl = (int)__umulhi((uint32_t)f, magic), e = 4 * (f - wl * n4w);
        *reinterpret_cast<v4f*>(span + wl * ip + e + (P32 ? 4 * (e / (32 * A)) : 0)) = r[u];
      }
    }
  } else {
  // ---- stage the span: samples [w0 * stride, (w0 + nwin - 1) * stride + W), A floats each ----
  {
    const float* src = stream + w0 * stride * A;
    const int nspan = ((nwin - 1) * stride + W) * A;
    int done = 0;
    if ((reinterpret_cast<uintptr_t>(src) & 15) == 0) {
      const int n4 = nspan >> 2;
      const v4f* s4 = reinterpret_cast<const v4f*>(src);
      v4f* d4 = reinterpret_cast<v4f*>(span);
      // unconditional (clamped) loads and stores: no exec-masked branches between them, so all SU
      // loads are in flight before the first store waits (a clamped slot rewrites the last float4)
      for (int f0 = tid; f0 < n4; f0 += SU * nt) {
        v4f r[SU];
#pragma unroll
        for (int u = 0; u < SU; ++u) r[u] = s4[min(f0 + u * nt, n4 - 1)];
#pragma unroll
        for (int u = 0; u < SU; ++u) d4[min(f0 + u * nt, n4 - 1)] = r[u];
      }
      done = n4 * 4;
    }
    for (int e = done + tid; e < nspan; e += nt) span[e] = src[e];
  }
  }
  __syncthreads();
  reg_window_batch<A, LPW, MLP, RCMAX, P32, FIXC>(span, w0, nwin, W, ip, C, ms_per_sample, out, ld_out, mo,
                                                 MLP ? lds : nullptr);
}

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
  constexpr int T3 = A / 3;
  // image pitch: 16 A (mod 64) dwords for odd A (conflict-free rows, see the kernel); 32 (mod 64)
  // for A = 6 (even A only ever reaches even banks: rows one image apart stay disjoint)
  const int n = window * A;
  // do the 64 lanes of a wave (rows one image apart, lanes A floats apart) hit 64 distinct banks?
  auto conflict_free = [&](int lpw, int pitch) {
    uint64_t seen = 0;
    for (int l = 0; l < 64; ++l) {
      const uint64_t bit = 1ull << (((l / lpw) * pitch + (l % lpw) * A) & 63);
      if (seen & bit) return false;
      seen |= bit;
    }
    return true;
  };
  auto pitch_for = [&](int lpw) {
    // contiguous images (flat staging, see the persistent kernel) unless that costs bank conflicts
    if (stride == window && n % 4 == 0 && (conflict_free(lpw, n) || A % 2 == 0)) return n;
    const int want = (A % 2) ? (lpw * A) % 64 : 32;
    return n + (((want - n) % 64) + 64) % 64;
  };
  auto lds_bytes = [&](int wpb, int pitch) -> int64_t {
    return (PAD + (int64_t)wpb * pitch + SLACK) * (int64_t)sizeof(float);
  };
  const bool vec = (reinterpret_cast<uintptr_t>(stream) & 15) == 0 && ((int64_t)stride * A) % 4 == 0;
  // one block's launch: persistent + register-prefetched when the window starts are 16-byte
  // aligned and a batch fits 24 float4 registers per thread (two waves per SIMD), else one-shot
  auto launch = [&](auto lpw_c, int waves, int pitch) -> int {
    constexpr int LPW = decltype(lpw_c)::value;
    const int wpb = waves * (64 / LPW) / T3, nt = 64 * waves;
    const int64_t bytes = lds_bytes(wpb, pitch);
    const int64_t nbatch = (n_windows + wpb - 1) / wpb;
    const int per = (int)((wpb * (int64_t)((n + 3) / 4) + nt - 1) / nt);  // float4s per thread per batch
    if (vec && per <= 24 && (int64_t)stride * A * wpb < 0x7fffffff) {
      const int64_t resident = std::max<int64_t>(1, std::min<int64_t>(8, (160 * 1024) / bytes));
      const unsigned grid = (unsigned)std::min<int64_t>(nbatch, resident * cu_count());
#define HAR_WIN_P(NR)                                                                              \
  window_features_persistent_kernel<A, LPW, MLP, NR><<<grid, nt, (size_t)bytes, s>>>(              \
      stream, n_samples, window, stride, n_windows, ms, out, ld_out, mo, pitch)
      if (per <= 8) HAR_WIN_P(8);
      else if (per <= 16) HAR_WIN_P(16);
      else HAR_WIN_P(24);
#undef HAR_WIN_P
    } else {
      window_features_kernel<A, LPW, MLP><<<(unsigned)nbatch, nt, (size_t)bytes, s>>>(
          stream, n_samples, window, stride, n_windows, ms, out, ld_out, mo, pitch);
    }
    HAR_CHECK_LAUNCH();
    return 0;
  };
  // register-resident kernel: the smallest group (8 / 16 / 32 / 64 lanes) whose runs of C <= RCMAX
  // samples (C odd: lanes C*A floats apart hit distinct LDS banks for odd A) cover the window
  if (!g_window_legacy) {
    // the smallest group (8 / 16 / 32 / 64 lanes), then the shortest odd run C <= 31 (lanes C*A
    // floats apart hit distinct LDS banks for odd A) with LPW * C >= W (W <= 1984): the fewer lanes
    // per window, the fewer cross-lane reductions per sample (~a third of the VALU at 32 lanes)
    // (8-lane groups only for overlapping windows: their span is shared, so the LDS per window — which
    // bounds the waves per CU — stays small; measured: W = 200 stride 100 69 vs 77 us, stride 200 54
    // vs 47 us with 8- vs 16-lane groups; round 6 with fixed-length runs, stride 100: 64 vs 77.5 us)
    int lpw = 0, C = 0;
    for (int l = stride < window ? 8 : 16; l <= 64 && !lpw; l *= 2)
      for (int c = 5; c <= RCMAX_LONG; c += 2)
        if (l * c >= window) { lpw = l; C = c; break; }
    // non-overlapping windows of (16 x 31, 16 x 32] samples: 16-lane groups of 32-sample runs on padded
    // per-window images (P32) instead of 32-lane groups (fewer cross-lane reductions per window).  Opt-in
    // (HAR_WINDOW_P32=1): measured 364 vs 328 us on the 9-axis 500-sample shape — four windows' images per
    // 3-wave block (73 KB) halve the resident waves, which costs more than the saved reductions
    static const bool p32_on = [] {
      const char* e = std::getenv("HAR_WINDOW_P32");
      return e && std::atoi(e) != 0;
    }();
    const bool p32 = p32_on && stride == window && (window * A) % 4 == 0 &&
                     (reinterpret_cast<uintptr_t>(stream) & 15) == 0 && lpw > 16 && window <= 16 * 32;
    if (p32) { lpw = 16; C = 32; }
    if (lpw) {
      const int gpw = 64 / lpw;
      // non-overlapping 16-lane windows: padded images, pitch = 16 (mod 32) floats (see the kernel)
      const bool pimg = !p32 && lpw == 16 && A % 2 == 1 && stride == window && (window * A) % 4 == 0 &&
                        (reinterpret_cast<uintptr_t>(stream) & 15) == 0 && (window * A) % 32 != 16 &&
                        !std::getenv("HAR_WINDOW_NOPAD");
      const int ipw = pimg ? window * A + (((16 - window * A) % 32) + 32) % 32 : 0;
      // (the fixed-length runs read D = lpw C - window samples past the last window unclamped)
      const bool fixc = !p32 && ((lpw == 8 && C == 25) || (lpw == 16 && C == 13));
      const int slack = fixc ? std::max(SLACK, (lpw * C - window) * A + 4) : SLACK;
      constexpr int NR = MLP ? reg_nrm_floats(A) : 0;
      auto span_bytes = [&](int wpb) -> int64_t {
        if (p32) return (NR + PAD + (int64_t)wpb * p32_pitch(window, A) + slack) * (int64_t)sizeof(float);
        if (ipw) return (NR + PAD + (int64_t)wpb * ipw + slack) * (int64_t)sizeof(float);
        return (NR + PAD + ((int64_t)(wpb - 1) * stride + window) * A + slack) * (int64_t)sizeof(float);
      };
      // waves per block: a multiple of T3, at most 4; the most whose span fits 48 KB (>= 3 blocks per CU)
      int m = 0;
      // (measured on the stride-100 shape: 2- and 1-wave blocks 70 / 68 us vs 64 us with 4 — the staged span is
      // shared by fewer windows and more blocks start on a stage)
      for (int mm = 4 / T3; mm >= 1; --mm)
        if (span_bytes(mm * gpw) <= 48 * 1024) { m = mm; break; }
      if (!m && span_bytes(gpw) <= 160 * 1024) m = 1;
      if (m) {
        const int wpb = m * gpw, nt = 64 * T3 * m;
        const int64_t nblk = (n_windows + wpb - 1) / wpb;
        const size_t bytes = (size_t)span_bytes(wpb);
        const unsigned grid = (unsigned)nblk;  // one-shot blocks (a persistent DMA-prefetch variant measured slower)
#define HAR_WIN_R(L)                                                                                          \
  if (C <= 17)                                                                                             \
    window_features_reg_kernel<A, L, MLP, 17><<<grid, nt, bytes, s>>>(stream, window, stride, n_windows, ms, out, \
                                                                      ld_out, mo, C, wpb, ipw);            \
  else                                                                                                     \
    window_features_reg_kernel<A, L, MLP, RCMAX_LONG><<<grid, nt, bytes, s>>>(stream, window, stride, n_windows, \
                                                                              ms, out, ld_out, mo, C, wpb, ipw)
        if (p32)
          window_features_reg_kernel<A, 16, MLP, 32, true><<<grid, nt, bytes, s>>>(stream, window, stride, n_windows,
                                                                                   ms, out, ld_out, mo, C, wpb, ipw);
        else if (lpw == 8 && C == 25) {  // (the stride-100 200-sample shape: 8 x 25, held to 128 VGPRs: 4 waves
                                          // per SIMD, not 3; fixed-length runs)
          window_features_reg_kernel<A, 8, MLP, 25, false, 4, true><<<grid, nt, bytes, s>>>(
              stream, window, stride, n_windows, ms, out, ld_out, mo, C, wpb, ipw);
        }
        else if (lpw == 16 && C == 13)  // (the 200-sample non-overlapping shape: 16 x 13, fixed-length runs)
          window_features_reg_kernel<A, 16, MLP, 13, false, 1, true><<<grid, nt, bytes, s>>>(
              stream, window, stride, n_windows, ms, out, ld_out, mo, C, wpb, ipw);
        else if (lpw == 8) { HAR_WIN_R(8); }
        else if (lpw == 16) { HAR_WIN_R(16); }
        else if (lpw == 32) { HAR_WIN_R(32); }
        else { HAR_WIN_R(64); }
#undef HAR_WIN_R
        HAR_CHECK_LAUNCH();
        return 0;
      }
    }
  }
  // 8-lane groups (half the reduction and write-out work per window) when two waves' sixteen
  // 3-axis windows fit 64 KB — the short-window WISDM case; else 16-lane groups
  if constexpr (A == 3) {
    if (lds_bytes(16, pitch_for(8)) <= 64 * 1024) return launch(std::integral_constant<int, 8>{}, 2, pitch_for(8));
  }
  const int pitch = pitch_for(16);
  // waves per block: a multiple of T3 (whole windows); the most whose images fit 64 KB (three or
  // more blocks per CU), else the fewest if they fit the 160 KB LDS
  int waves = 0;
  for (int w = 4; w >= 1; --w) {
    if (w % T3) continue;
    if (lds_bytes(4 * w / T3, pitch) <= 64 * 1024) { waves = w; break; }
  }
  if (!waves && lds_bytes(4, pitch) <= 160 * 1024) waves = T3;
  if (!waves) return -5;  // one block's windows do not fit the LDS
  return launch(std::integral_constant<int, 16>{}, waves, pitch);
}


}  // namespace

extern "C" void har_window_set_legacy(int on) { g_window_legacy = on != 0; }

extern "C" int har_window_features(const float* stream, int64_t n_samples, int axes, int window, int stride,
                                   int64_t n_windows, float hz, int nbins, float* out, int ld_out, hipStream_t s) {
  if (axes > MAXA || axes % 3 || nbins != NB || window < 3 || window >= 65536 || stride <= 0 || n_windows < 0)
    return -2;
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
  if (axes > MAXA || axes % 3 || window < 3 || window >= 65536 || stride <= 0 || n_windows < 0) return -2;
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
