// Decision-tree / random-forest kernels.
//
// tree_hist_split: one workgroup per (active node, feature chunk).  The node's
//   rows (grouped contiguously by the caller) are streamed once per chunk; every
//   (row, feature) pair adds its bootstrap weight to an LDS-privatized histogram
//   [chunk features][bins][classes].  Then one wave per feature runs an inclusive
//   prefix scan over the bins (one lane per bin, <= 64 bins), evaluates the
//   impurity gain of every threshold in fp64, and the workgroup reduces the best
//   (gain, feature, bin) — the histogram never leaves LDS.  Ties break to the
//   lowest (feature slot, bin), matching the CPU oracle.
// forest_predict: one lane per row walks every tree (SoA node arrays, L2
//   resident) and accumulates the (normalized) leaf class statistics.
// poisson_bootstrap: Philox4x32-10 keyed by (seed, tree, global row id) ->
//   Poisson(1) counts, identical to har/ops/rng.py.
#include "common.h"
#include "philox.h"
#include "../har_kernels.h"

namespace {

constexpr int KMAX = 32;
#ifndef HIST_UNROLL
#define HIST_UNROLL 4
#endif

__global__ __launch_bounds__(256) void tree_hist_split_kernel(
    const uint8_t* __restrict__ bins, int64_t fstride, int64_t rstride, const int32_t* __restrict__ nbins_feat,
    const int32_t* __restrict__ rows, const float* __restrict__ row_w, const int32_t* __restrict__ node_start,
    const int32_t* __restrict__ node_count, const int32_t* __restrict__ feats, int m, int fc,
    const int32_t* __restrict__ label, int K, int maxbins, float min_inst, float min_gain, int impurity,
    float* __restrict__ out_gain, int32_t* __restrict__ out_feat, int32_t* __restrict__ out_bin,
    float* __restrict__ out_left, float* __restrict__ out_total, int mode, float* __restrict__ ghist) {
  // mode 0: fused histogram + split; 1: histogram only -> ghist [A][m][maxbins][K] (data parallel:
  // summed across ranks by RCCL); 2: split search from a (reduced) ghist
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int a = blockIdx.y, c = blockIdx.x, chunks = gridDim.x;
  const int f_lo = c * fc;
  const int f_n = min(fc, m - f_lo);
  float* hist = smem;                                          // [fc][maxbins][K]
  int* fid = reinterpret_cast<int*>(smem + (size_t)fc * maxbins * K);  // [fc]
  __shared__ double red_gain[4];
  __shared__ int red_idx[4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // grid.z > 1 (histogram-only mode): the node's rows are split over gridDim.z workgroups
  const int cnt_all = node_count[a];
  const int per_z = (cnt_all + gridDim.z - 1) / gridDim.z;
  const int zb = min(cnt_all, (int)blockIdx.z * per_z);
  const int start = node_start[a] + zb, cnt = min(cnt_all, zb + per_z) - zb;

  float* gh = ghist ? ghist + ((size_t)a * m + f_lo) * maxbins * K : nullptr;
  for (int i = tid; i < f_n * maxbins * K; i += blockDim.x) hist[i] = (mode == 2) ? gh[i] : 0.f;
  for (int i = tid; i < f_n; i += blockDim.x) fid[i] = feats[(size_t)a * m + f_lo + i];
  __syncthreads();

  // ---- histogram ----
  const int rpi = f_n <= 64 ? (int)blockDim.x / f_n : 0;
  if (mode != 2 && rpi > 0) {
    // (row, feature slot) pairs with the feature slot fastest: the lanes of one instruction
    // add into f_n different feature histograms (a row-at-a-time mapping sends most lanes of a
    // nearly pure node to the same (bin, class) word — same-address LDS atomics serialize), and
    // the lanes sharing a row read its id / weight / label as one broadcast and its row-major
    // bins from one line.  Slot and row phase come from tid once; no division in the loop.
    const int fs = tid % f_n, rs = tid / f_n;
    if (rs < rpi) {
      const int64_t fo = (int64_t)fid[fs] * fstride;
      float* hb = hist + fs * maxbins * K;
      // HU rows in flight per lane: the row id -> (bins, label) loads are a dependent chain of
      // two L2 / MALL round trips, so issue HU chains before the first atomic needs its data
      constexpr int HU = HIST_UNROLL;
      int ri = rs;
      for (; ri + (HU - 1) * rpi < cnt; ri += HU * rpi) {
        int r[HU], b[HU], l[HU];
        float w[HU];
#pragma unroll
        for (int u = 0; u < HU; ++u) {
          r[u] = rows[start + ri + u * rpi];
          w[u] = row_w[start + ri + u * rpi];
        }
#pragma unroll
        for (int u = 0; u < HU; ++u) {
          b[u] = bins[fo + (int64_t)r[u] * rstride];
          l[u] = label[r[u]];
        }
#pragma unroll
        for (int u = 0; u < HU; ++u) atomicAdd(hb + b[u] * K + l[u], w[u]);
      }
      for (; ri < cnt; ri += rpi) {
        const int r = rows[start + ri];
        const float w = row_w[start + ri];
        const int b = bins[fo + (int64_t)r * rstride];
        atomicAdd(hb + b * K + label[r], w);
      }
    }
  } else if (mode != 2 && cnt >= (int)blockDim.x) {
    // large node: one row per lane, its (row id, weight, label) loaded once for all f_n features
    for (int ri = tid; ri < cnt; ri += blockDim.x) {
      const int r = rows[start + ri];
      const float w = row_w[start + ri];
      float* hl = hist + label[r];
      for (int fs = 0; fs < f_n; ++fs) {
        const int b = bins[fid[fs] * fstride + r * rstride];
        atomicAdd(hl + (fs * maxbins + b) * K, w);
      }
    }
  } else if (mode != 2) {
    // small node: (feature slot, row) pairs, rows fastest, so every lane has work
    // j -> (fs, ri) by a float reciprocal + one correction step instead of an integer division
    // (~40 VALU ops per pair; j < 2^24 is exact in fp32, so the estimate is off by at most one)
    const int pairs = cnt * f_n;
    const float inv_cnt = 1.f / (float)cnt;
    for (int j = tid; j < pairs; j += blockDim.x) {
      int fs = (int)((float)j * inv_cnt);
      int ri = j - fs * cnt;
      if (ri < 0) { --fs; ri += cnt; } else if (ri >= cnt) { ++fs; ri -= cnt; }
      const int r = rows[start + ri];
      const float w = row_w[start + ri];
      const int b = bins[fid[fs] * fstride + r * rstride];
      atomicAdd(&hist[(fs * maxbins + b) * K + label[r]], w);
    }
  }
  __syncthreads();
  if (mode == 1) {
    if (gridDim.z == 1) {
      for (int i = tid; i < f_n * maxbins * K; i += blockDim.x) gh[i] = hist[i];
    } else {  // row-split node: merge into the zeroed global histogram (integer-valued sums: exact)
      for (int i = tid; i < f_n * maxbins * K; i += blockDim.x)
        if (hist[i] != 0.f) atomicAdd(gh + i, hist[i]);
    }
    return;
  }

  // ---- split search: one wave per feature slot, one lane per bin ----
  // Per lane (= threshold bin) the class loop keeps only running sums — no per-class arrays
  // (which lived in scratch): gini needs sum c^2 of left / right / parent, entropy needs
  // sum c log2 c (imp = log2 w - sum c log2 c / w), plus the weights.
  double best_g = -INFINITY;
  int best_i = 0x7fffffff;
  for (int fs = wave; fs < f_n; fs += (int)(blockDim.x >> 6)) {
    const int nb = nbins_feat[fid[fs]];
    double wl = 0.0, wt = 0.0, ql = 0.0, qr = 0.0, qt = 0.0;
    for (int k = 0; k < K; ++k) {
      // the bin scan runs in fp32 (one ds_bpermute per step instead of two): the sums are exact
      // for integer-valued weights below 2^24 (bootstrap counts, fold masks) and are what the
      // CPU oracle's float32 cumsum computes anyway; the gains below are fp64
      float vf = (lane < nb && lane < maxbins) ? hist[(fs * maxbins + lane) * K + k] : 0.f;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const float u = __shfl_up(vf, o, 64);
        if (lane >= o) vf += u;
      }
      const double v = (double)vf;
      const double t = (double)__shfl(vf, max(nb - 1, 0), 64);
      const double r = t - v;
      wl += v;
      wt += t;
      if (impurity == 0) {
        ql += v * v; qr += r * r; qt += t * t;
      } else {
        ql += v > 0 ? v * log2(v) : 0.0;
        qr += r > 0 ? r * log2(r) : 0.0;
        qt += t > 0 ? t * log2(t) : 0.0;
      }
    }
    const double wr = wt - wl;
    double g = -INFINITY;
    if (lane < nb - 1 && wl >= min_inst && wr >= min_inst && wt > 0) {
      double ip, il, ir;
      if (impurity == 0) {
        ip = 1.0 - qt / (wt * wt); il = 1.0 - ql / (wl * wl); ir = 1.0 - qr / (wr * wr);
      } else {
        ip = log2(wt) - qt / wt; il = log2(wl) - ql / wl; ir = log2(wr) - qr / wr;
      }
      g = ip - (wl / wt) * il - (wr / wt) * ir;
    }
    int idx = fs * maxbins + lane;
    // wave argmax, lowest index on ties
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      double og = __shfl_xor(g, o, 64);
      int oi = __shfl_xor(idx, o, 64);
      if (og > g || (og == g && oi < idx)) { g = og; idx = oi; }
    }
    if (g > best_g || (g == best_g && idx < best_i)) { best_g = g; best_i = idx; }
  }
  if (lane == 0) { red_gain[wave] = best_g; red_idx[wave] = best_i; }
  __syncthreads();
  if (tid == 0) {
    double g = red_gain[0];
    int idx = red_idx[0];
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w)
      if (red_gain[w] > g || (red_gain[w] == g && red_idx[w] < idx)) { g = red_gain[w]; idx = red_idx[w]; }
    const size_t o = (size_t)a * chunks + c;
    const bool ok = isfinite(g) && g >= (double)min_gain;
    out_gain[o] = ok ? (float)g : -INFINITY;
    const int fs = ok ? idx / maxbins : 0, b = ok ? idx % maxbins : 0;
    out_feat[o] = fid[fs];
    out_bin[o] = b;
    for (int k = 0; k < K; ++k) {
      float s = 0.f;
      for (int bb = 0; bb <= b; ++bb) s += hist[(fs * maxbins + bb) * K + k];
      out_left[o * K + k] = ok ? s : 0.f;
    }
    if (c == 0) {
      for (int k = 0; k < K; ++k) {
        float s = 0.f;
        for (int bb = 0; bb < maxbins; ++bb) s += hist[bb * K + k];
        out_total[(size_t)a * K + k] = s;
      }
    }
  }
}

// Leaf statistics of tree t for input row x (normalized to a distribution when asked), added
// into acc[0..K).  KC >= K is a compile-time bound so acc stays in registers.
template <int KC>
__device__ __forceinline__ void add_tree(const float* __restrict__ x, size_t base, const int32_t* __restrict__ feature,
                                         const float* __restrict__ thr, const int32_t* __restrict__ left,
                                         const int32_t* __restrict__ right, const float* __restrict__ leaf, int K,
                                         int max_depth, int normalize, float (&acc)[KC]) {
  int node = 0;
  for (int d = 0; d <= max_depth; ++d) {
    const int f = feature[base + node];
    if (f < 0) break;
    node = (x[f] <= thr[base + node]) ? left[base + node] : right[base + node];
  }
  const float* st = leaf + (base + node) * K;
  float v[KC];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < KC; ++k) {
    v[k] = k < K ? st[k] : 0.f;
    s += v[k];
  }
  const float sc = normalize ? (s > 0.f ? 1.f / s : 0.f) : 1.f;
#pragma unroll
  for (int k = 0; k < KC; ++k) acc[k] += v[k] * sc;
}

// Many rows: one lane per row walks every tree.
template <int KC>
__global__ __launch_bounds__(256) void forest_predict_kernel(
    const float* __restrict__ X, int64_t n, int ld, const int32_t* __restrict__ feature,
    const float* __restrict__ thr, const int32_t* __restrict__ left, const int32_t* __restrict__ right,
    const float* __restrict__ leaf, int T, int maxn, int K, int max_depth, int normalize, float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float acc[KC];
#pragma unroll
  for (int k = 0; k < KC; ++k) acc[k] = 0.f;
  const float* x = X + i * (int64_t)ld;
  for (int t = 0; t < T; ++t)
    add_tree<KC>(x, (size_t)t * maxn, feature, thr, left, right, leaf, K, max_depth, normalize, acc);
#pragma unroll
  for (int k = 0; k < KC; ++k)
    if (k < K) out[i * K + k] = acc[k];
}

// Few rows (serving batches, evaluation sets): one wave per row, lanes split the trees, one
// wave reduction per class — 64x the parallelism of the lane-per-row form.
template <int KC>
__global__ __launch_bounds__(256) void forest_predict_wave_kernel(
    const float* __restrict__ X, int64_t n, int ld, const int32_t* __restrict__ feature,
    const float* __restrict__ thr, const int32_t* __restrict__ left, const int32_t* __restrict__ right,
    const float* __restrict__ leaf, int T, int maxn, int K, int max_depth, int normalize, float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (i >= n) return;  // wave-uniform
  float acc[KC];
#pragma unroll
  for (int k = 0; k < KC; ++k) acc[k] = 0.f;
  const float* x = X + i * (int64_t)ld;
  for (int t = lane; t < T; t += 64)
    add_tree<KC>(x, (size_t)t * maxn, feature, thr, left, right, leaf, K, max_depth, normalize, acc);
#pragma unroll
  for (int k = 0; k < KC; ++k) {
    float v = acc[k];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == k && k < K) out[i * K + k] = v;
  }
}

template <int KC>
void launch_predict(const float* X, int64_t n, int ld, const int32_t* feat, const float* thr, const int32_t* left,
                    const int32_t* right, const float* leaf, int ntrees, int maxn, int K, int max_depth,
                    int normalize, float* raw_out, hipStream_t s) {
  if (ntrees >= 16) {  // 1M rows x 100 trees on MI355X: 11.5 ms here vs 16.8 ms lane-per-row
    forest_predict_wave_kernel<KC><<<(int)((n + 3) / 4), 256, 0, s>>>(X, n, ld, feat, thr, left, right, leaf, ntrees,
                                                                       maxn, K, max_depth, normalize, raw_out);
  } else {
    forest_predict_kernel<KC><<<(int)((n + 255) / 256), 256, 0, s>>>(X, n, ld, feat, thr, left, right, leaf, ntrees,
                                                                     maxn, K, max_depth, normalize, raw_out);
  }
}

__global__ __launch_bounds__(256) void poisson_bootstrap_kernel(uint64_t seed, int tree0, int ntrees, int64_t row0,
                                                                int64_t n, uint8_t* __restrict__ out) {
  // uint32 CDF thresholds of Poisson(1) (same table as har/ops/rng.py)
  const uint32_t thr[15] = {1580030168u, 3160060337u, 3950075421u, 4213413783u, 4279248373u, 4292415291u,
                            4294609777u, 4294923276u, 4294962463u, 4294966817u, 4294967252u, 4294967292u,
                            4294967295u, 4294967295u, 4294967295u};
  const int64_t total = (int64_t)ntrees * n;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < total; j += (int64_t)gridDim.x * blockDim.x) {
    const int t = (int)(j / n);
    const int64_t r = j - (int64_t)t * n;
    const uint32_t u = philox_u32(seed, 0x1000u + (uint32_t)(tree0 + t), (uint64_t)(row0 + r));
    int k = 0;
    while (k < 15 && u >= thr[k]) ++k;
    out[j] = (uint8_t)k;
  }
}

// One pass per fit over the (tree, row) slots: bootstrap weight (Poisson(1) from Philox keyed by
// (seed, global tree, global row), or 1) times an optional row weight -> W [T][N] fp32; node
// ids [T][N] (0, or -1 where the weight is 0); root class counts written straight into
// stats[t][0][K] (stats zeroed by the caller).  Labels outside [0, K) set *bad.  The counts are
// sums of integer-valued weights (< 2^24), so the LDS partials and the one global atomic per
// (workgroup, class) are exact in any order: the result is deterministic.
constexpr int INIT_ROWS = 2048;
__global__ __launch_bounds__(256) void tree_init_kernel(uint64_t seed, int tree0, int64_t row0, int64_t n,
                                                        int bootstrap, const float* __restrict__ rw,
                                                        const int32_t* __restrict__ y, int K,
                                                        float* __restrict__ W, int32_t* __restrict__ node_of,
                                                        float* __restrict__ stats, int64_t stats_tree_stride,
                                                        int32_t* __restrict__ bad) {
  const uint32_t thr[15] = {1580030168u, 3160060337u, 3950075421u, 4213413783u, 4279248373u, 4292415291u,
                            4294609777u, 4294923276u, 4294962463u, 4294966817u, 4294967252u, 4294967292u,
                            4294967295u, 4294967295u, 4294967295u};
  __shared__ float cnt[KMAX];
  const int t = blockIdx.y;
  if (threadIdx.x < KMAX) cnt[threadIdx.x] = 0.f;
  __syncthreads();
  const int64_t r0 = (int64_t)blockIdx.x * INIT_ROWS, r1 = min(n, r0 + INIT_ROWS);
  int badl = 0;
  for (int64_t r = r0 + threadIdx.x; r < r1; r += 256) {
    float w = 1.f;
    if (bootstrap) {
      const uint32_t u = philox_u32(seed, 0x1000u + (uint32_t)(tree0 + t), (uint64_t)(row0 + r));
      int k = 0;
      while (k < 15 && u >= thr[k]) ++k;
      w = (float)k;
    }
    if (rw) w *= rw[(int64_t)t * n + r];
    W[(int64_t)t * n + r] = w;
    node_of[(int64_t)t * n + r] = w == 0.f ? -1 : 0;
    const int c = y[r];
    if (c < 0 || c >= K) badl = 1;
    else if (w != 0.f) atomicAdd(&cnt[c], w);
  }
  if (badl) *bad = 1;
  __syncthreads();
  if (threadIdx.x < K && cnt[threadIdx.x] != 0.f) atomicAdd(stats + t * stats_tree_stride + threadIdx.x, cnt[threadIdx.x]);
}

// findSplits after the sort (ops/tree.py find_thresholds_device): one workgroup per feature of
// the [F][n] sorted sample (NaN last).  A block-wide scan over the distinct-value starts gives
// every sorted position its distinct rank (LDS) and compacts the distinct values; then the
// ns = maxBins - 1 candidate cut points — every midpoint when there are few distinct values,
// else the fp64 quantile targets t = nvalid (k + 1) / (ns + 1) mapped to the distinct rank of
// sorted position ceil(t) - 1 — are deduplicated and written in order.  out [F][ns + 1]: the
// thresholds, then their count (as float): the ONE device -> host copy of findSplits.
constexpr int FS_MAXN = 16384;
__global__ __launch_bounds__(256) void find_splits_post_sort_kernel(const float* __restrict__ sorted, int n, int ns,
                                                                    float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) int fs_smem[];
  int* drank = fs_smem;                                     // [n]
  float* U = reinterpret_cast<float*>(fs_smem + n);         // [n] distinct values
  __shared__ int wsum[4], s_nvalid, s_base;
  __shared__ int Jk[64];
  const int f = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float* s = sorted + (size_t)f * n;
  if (tid == 0) { s_nvalid = n; s_base = 0; }
  __syncthreads();
  for (int i = tid; i < n; i += 256)
    if (isnan(s[i]) && (i == 0 || !isnan(s[i - 1]))) s_nvalid = i;  // the single NaN start
  __syncthreads();
  const int nvalid = s_nvalid;
  for (int c0 = 0; c0 < n; c0 += 256) {
    const int i = c0 + tid;
    const bool nd = i < nvalid && (i == 0 || s[i] != s[i - 1]);
    const uint64_t mask = __ballot(nd);
    const int before = __popcll(mask & ((1ull << lane) - 1));
    if (lane == 0) wsum[wave] = __popcll(mask);
    __syncthreads();
    int off = s_base;
    for (int w = 0; w < wave; ++w) off += wsum[w];
    const int rank = off + before + (nd ? 1 : 0) - 1;  // distinct index of this sorted position
    if (i < n) {
      drank[i] = rank;
      if (nd) U[rank] = s[i];
    }
    __syncthreads();
    if (tid == 0) s_base += wsum[0] + wsum[1] + wsum[2] + wsum[3];
    __syncthreads();
  }
  const int ndist = s_base;
  const bool few = ndist - 1 <= ns;
  if (tid < ns) {
    int j;
    if (few) {
      j = tid;
    } else {
      const double tq = (double)nvalid * (double)(tid + 1) / (double)(ns + 1);
      int64_t q = (int64_t)ceil(tq) - 1;
      q = q < 0 ? 0 : (q > n - 1 ? n - 1 : q);
      j = drank[q];
      j = min(j, max(ndist - 2, 0));
      j = max(j, 0);
    }
    Jk[tid] = j;
  }
  __syncthreads();
  if (wave == 0) {
    bool keep = lane < ns && ndist > 1;
    if (keep) keep = few ? lane < ndist - 1 : (lane == 0 || Jk[lane] != Jk[lane - 1]);
    const uint64_t mask = __ballot(keep);
    const int pos = __popcll(mask & ((1ull << lane) - 1));
    float* o = out + (size_t)f * (ns + 1);
    if (keep) o[pos] = (U[Jk[lane]] + U[Jk[lane] + 1]) / 2.0f;
    if (lane == 0) o[ns] = (float)__popcll(mask);
  }
}

}  // namespace

// bins: feature-major [F][N] (row_major = 0) or row-major [N][F] (row_major = 1: the bytes of one
// row's sampled features share one or two cache lines — the deep levels gather far less).
extern "C" int har_tree_hist_split(const uint8_t* bins, int64_t N, int F, int row_major, const int32_t* nbins_feat,
                                   const int32_t* rows, const float* row_w, const int32_t* node_start,
                                   const int32_t* node_count, int A, const int32_t* feats, int m, int fc,
                                   const int32_t* label, int K, int maxbins, float min_inst, float min_gain,
                                   int impurity, float* out_gain, int32_t* out_feat, int32_t* out_bin,
                                   float* out_left, float* out_total, int mode, float* ghist, int row_chunks,
                                   hipStream_t s) {
  if (K > KMAX || maxbins > 64 || fc <= 0 || m <= 0) return -2;
  if (mode != 0 && !ghist) return -4;
  if (A == 0) return 0;
  const int chunks = (m + fc - 1) / fc;
  const size_t lds = (size_t)fc * maxbins * K * sizeof(float) + (size_t)fc * sizeof(int);
  if (lds > 150 * 1024) return -3;
  if (row_chunks > 1 && mode != 1) return -5;
  dim3 grid(chunks, A, row_chunks > 1 ? row_chunks : 1);
  const int64_t fstride = row_major ? 1 : N, rstride = row_major ? F : 1;
  tree_hist_split_kernel<<<grid, 256, lds, s>>>(bins, fstride, rstride, nbins_feat, rows, row_w, node_start, node_count, feats, m,
                                                fc, label, K, maxbins, min_inst, min_gain, impurity, out_gain,
                                                out_feat, out_bin, out_left, out_total, mode, ghist);
  HAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int har_forest_predict(const float* X, int64_t n, int F, int ld, const int32_t* feat, const float* thr,
                                  const int32_t* left, const int32_t* right, const float* leaf, int ntrees,
                                  int maxn, int K, int max_depth, int normalize, float* raw_out, hipStream_t s) {
  if (K > KMAX) return -2;
  if (n == 0) return 0;
  if (K <= 8) launch_predict<8>(X, n, ld, feat, thr, left, right, leaf, ntrees, maxn, K, max_depth, normalize, raw_out, s);
  else if (K <= 16) launch_predict<16>(X, n, ld, feat, thr, left, right, leaf, ntrees, maxn, K, max_depth, normalize,
                                       raw_out, s);
  else launch_predict<32>(X, n, ld, feat, thr, left, right, leaf, ntrees, maxn, K, max_depth, normalize, raw_out, s);
  HAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int har_poisson_bootstrap(uint64_t seed, int tree0, int ntrees, int64_t row0, int64_t n, uint8_t* out,
                                     hipStream_t s) {
  int64_t total = (int64_t)ntrees * n;
  if (total == 0) return 0;
  int blocks = (int)std::min<int64_t>(4096, (total + 255) / 256);
  poisson_bootstrap_kernel<<<blocks, 256, 0, s>>>(seed, tree0, ntrees, row0, n, out);
  HAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int har_tree_init(uint64_t seed, int tree0, int ntrees, int64_t row0, int64_t n, int bootstrap,
                             const float* rw, const int32_t* y, int K, float* W, int32_t* node_of, float* stats,
                             int64_t stats_tree_stride, int32_t* bad, hipStream_t s) {
  if (K <= 0 || K > KMAX) return -2;
  if (n == 0 || ntrees == 0) return 0;
  dim3 grid((unsigned)((n + INIT_ROWS - 1) / INIT_ROWS), (unsigned)ntrees);
  tree_init_kernel<<<grid, 256, 0, s>>>(seed, tree0, row0, n, bootstrap, rw, y, K, W, node_of, stats,
                                        stats_tree_stride, bad);
  HAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int har_find_splits_post_sort(const float* sorted, int F, int n, int ns, float* out, hipStream_t s) {
  if (n <= 0 || n > FS_MAXN || ns <= 0 || ns > 63) return -2;
  if (F == 0) return 0;
  find_splits_post_sort_kernel<<<F, 256, (size_t)2 * n * sizeof(int), s>>>(sorted, n, ns, out);
  HAR_CHECK_LAUNCH();
  return 0;
}
