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
#include "wave_ops.h"
#include "../har_kernels.h"

namespace {

constexpr int KMAX = 32;
#ifndef HIST_UNROLL
#define HIST_UNROLL 4
#endif

// Split search of TWO feature slots per wave (maxBins <= 32): lanes 0..31 hold the bins of slot
// 2p, lanes 32..63 those of slot 2p + 1.  KC class prefix sums at a time advance together through
// ONE 5-step scan over the 32-lane halves (independent shuffles pipeline), instead of a dependent
// 6-step 64-lane scan per class and slot.  The per-lane gain arithmetic (fp64, classes summed in
// order) and the lowest-index tie rule are those of the one-slot-per-wave search, so the winner
// is bit for bit the same.
// smap (optional): the slots to search, smap[0 .. f_n) (the numeric slots of a SPARSE chunk); the winner
// index is still slot * maxbins + bin
template <int KC>
__device__ __forceinline__ void split_search_pairs(const float* hist, const int* fid, const int32_t* nbins_feat,
                                                   int f_n, int maxbins, int K, float min_inst, int impurity,
                                                   int wave, int nwaves, int lane, double& best_g, int& best_i,
                                                   const short* smap = nullptr) {
  const int half = lane >> 5, bl = lane & 31;
  const wops::LaneSwap sw(lane);
  for (int fp = wave; 2 * fp < f_n; fp += nwaves) {
    const int fi = 2 * fp + half;
    const bool fv = fi < f_n;
    const int fs = smap ? (fv ? (int)smap[fi] : 0) : fi;
    const int nb = fv ? nbins_feat[fid[fs]] : 0;
    // each half's last bin (uniform per half): the totals are two scalar lane reads, not a permute
    const int last0 = max(__builtin_amdgcn_readlane(nb, 0) - 1, 0);
    const int last1 = 32 + max(__builtin_amdgcn_readlane(nb, 32) - 1, 0);
    double wl = 0.0, wt = 0.0, ql = 0.0, qr = 0.0, qt = 0.0;
    // classes in groups of KC (registers), accumulated in class order
    for (int k0 = 0; k0 < K; k0 += KC) {
      float c[KC];
#pragma unroll
      for (int k = 0; k < KC; ++k)
        c[k] = (k0 + k < K && bl < nb && bl < maxbins) ? hist[(fs * maxbins + bl) * K + k0 + k] : 0.f;
      // inclusive bin scans of the KC classes over each 32-lane half (DPP row shifts + row broadcast:
      // VALU, independent chains pipeline)
#pragma unroll
      for (int k = 0; k < KC; ++k) c[k] = wops::scan32_add(c[k]);
#pragma unroll
      for (int k = 0; k < KC; ++k) {
        const float tf = half ? wops::lane_f(c[k], last1) : wops::lane_f(c[k], last0);
        if (k0 + k < K) {
          const double v = (double)c[k], t = (double)tf, r = t - v;
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
      }
    }
    const double wr = wt - wl;
    double g = -INFINITY;
    if (fv && bl < nb - 1 && wl >= min_inst && wr >= min_inst && wt > 0) {
      double ip, il, ir;
      if (impurity == 0) {
        ip = 1.0 - qt / (wt * wt); il = 1.0 - ql / (wl * wl); ir = 1.0 - qr / (wr * wr);
      } else {
        ip = log2(wt) - qt / wt; il = log2(wl) - ql / wl; ir = log2(wr) - qr / wr;
      }
      g = ip - (wl / wt) * il - (wr / wt) * ir;
    }
    int idx = fs * maxbins + bl;
    wops::wave_argmax(g, idx, sw);
    if (g > best_g || (g == best_g && idx < best_i)) { best_g = g; best_i = idx; }
  }
}

// Histogram add.  INTW: the weights are non-negative integers (bootstrap / subsample counts x 0/1
// fold masks — every weight the forest builder produces), so the LDS histogram accumulates them as
// uint32 (ds_add_u32) and is converted to fp32 once before the split search: the same sums (exact
// below 2^24) without the float LDS atomic.
template <bool INTW>
__device__ __forceinline__ void hist_add(float* p, float w) {
  if constexpr (INTW) atomicAdd(reinterpret_cast<unsigned int*>(p), (unsigned int)w);
  else atomicAdd(p, w);
}

// One-hot-aware histograms (SPARSE; ops/tree.py, the reference encoding's 3,090 binary one-hot
// columns beside 10 numeric ones, Main/main.py:51-66).  Per row the one-hot blocks hold at most one 1
// each (sp.cat [N][ncat]: the global column of the row's 1, -1 = none), so a node's histogram of a
// one-hot column with the split 0 | 1 (the column's one threshold, 0.5) is: bin 1 = the weight of the
// node's rows whose entry is that column, added over the ncat entries of every row — O(rows x ncat)
// instead of O(rows x features) — and bin 0 = the node's class totals minus bin 1 (integer weights:
// exact).  The numeric columns of the chunk are histogrammed from the bins as in the dense path.  The
// split search, the stores and every mode are the dense kernel's: the forest is the same node for node.
constexpr int SP_NCAT = 4;  // one-hot blocks per row handled in registers (more: the dense path)

template <bool INTW, bool SPARSE>
__global__ __launch_bounds__(256) void tree_hist_split_kernel(
    const uint8_t* __restrict__ bins, int64_t fstride, int64_t rstride, const int32_t* __restrict__ nbins_feat,
    const int32_t* __restrict__ rows, const float* __restrict__ row_w, const int32_t* __restrict__ node_start,
    const int32_t* __restrict__ node_count, const int32_t* __restrict__ feats, int m, int fc,
    const int32_t* __restrict__ label, int K, int maxbins, float min_inst, float min_gain, int impurity,
    float* __restrict__ out_gain, int32_t* __restrict__ out_feat, int32_t* __restrict__ out_bin,
    float* __restrict__ out_left, float* __restrict__ out_total, int mode, float* __restrict__ ghist,
    const int32_t* __restrict__ plan, int prows, int by_node, const float* __restrict__ hprev,
    const int32_t* __restrict__ derive_from, const int32_t* __restrict__ parent_of, TreeSparse sp) {
  // mode 0: fused histogram + split; 1: histogram only -> ghist [A][m][maxbins][K] (data parallel:
  // summed across ranks by RCCL); 2: split search from a (reduced) ghist.
  // Planned (load-balanced) level, plan = tree_plan_kernel's output (see there):
  // mode 3: work item blockIdx.y: a node of <= prows rows -> fused histogram + split (as mode 0);
  //         one prows-row chunk of a larger node -> its histogram added into that node's ghist slot
  // mode 4: blockIdx.y = big-node slot: split search from its merged ghist (as mode 2)
  // Sibling subtraction (by_node = 1: ghist is the level's per-node histogram store [A][m][bins][K],
  // every node's histogram is kept there for the next level):
  //   mode 3 skips the nodes marked derive_from[a] >= 0 (their rows were not grouped), writes each
  //   fused node's LDS histogram to its store slot, and merges big-node chunks into slot a;
  //   mode 5: blockIdx.y = node a with derive_from[a] = sibling s: hist = hprev[parent_of[a]] -
  //   store[s] (integer-valued weights: exact), kept in store[a], then the split search (mode 2).
  // Data parallel (by_node = 1): mode 6 = the work items of mode 3, histogram only: a node of one
  // item stores its slot outright (zero rows on this rank: zeros), the chunks of a big node add into
  // its slot (zeroed by tree_plan), so the store needs no zero fill; it is then summed across ranks
  // (all-reduce, or reduce-scatter by node owner); mode 7 = split search from the rank's slice of it.
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int c = blockIdx.x, chunks = gridDim.x;
  int a = blockIdx.y, gslot = blockIdx.y;
  const int f_lo = c * fc;
  const int f_n = min(fc, m - f_lo);
  float* hist = smem;                                          // [fc][maxbins][K]
  int* fid = reinterpret_cast<int*>(smem + (size_t)fc * maxbins * K);  // [fc]
  // SPARSE: class totals [K] (uint32), global column -> chunk slot [F] (-1: not in the chunk), the
  // chunk's numeric slots, per-slot kind (0 numeric, 1 one-hot with its 0 | 1 split, 2 one-hot
  // without a threshold: every row in bin 0)
  unsigned int* ktot = reinterpret_cast<unsigned int*>(fid + fc);
  short* slot_of = reinterpret_cast<short*>(ktot + K);
  short* dlist = slot_of + (SPARSE ? sp.F : 0);
  uint8_t* sflag = reinterpret_cast<uint8_t*>(dlist + fc);
  __shared__ int nd_s;
  __shared__ double red_gain[4];
  __shared__ int red_idx[4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int start, cnt;
  bool direct = false;  // mode 6, a node of one work item: its slot is stored, not added into
  if (mode == 7) {
    // data parallel: split search from the rank's slice of the reduced store (ghist, feats, outputs
    // all start at global node prows = a0); nodes at or past the level's device count exit
    if (prows + (int)blockIdx.y >= plan[2]) return;
    mode = 2;
    start = 0;
    cnt = 0;
  } else if (mode == 3 || mode == 4 || mode == 6) {
    const int A = plan[2];
    const int32_t* item_start = plan + 4;            // [A + 1]
    const int32_t* big_rank = item_start + A + 1;    // [A]  (-1: not big)
    const int32_t* big_list = big_rank + A;          // [A]
    const int32_t* item_node = big_list + A;         // [items]
    if (mode != 4) {
      if ((int)blockIdx.y >= plan[0]) return;        // beyond this level's work items
      a = item_node[blockIdx.y];
      if (derive_from && derive_from[a] >= 0) return;  // histogram = parent - sibling (mode 5)
      gslot = big_rank[a];
      const int z = blockIdx.y - item_start[a];
      const int cnt_all = node_count[a];
      start = node_start[a] + z * prows;
      cnt = gslot < 0 ? cnt_all : min(prows, cnt_all - z * prows);
      // mode 6 (data parallel): every item only adds its histogram into the node's zeroed store
      // slot; the split search follows the cross-rank reduction (mode 7)
      direct = mode == 6 && gslot < 0;
      if (gslot >= 0 || mode == 6) mode = 1;         // a chunk of a big node: histogram only
      else mode = 0;
      if (by_node) gslot = a;
    } else {
      if ((int)blockIdx.y >= plan[1]) return;        // beyond this level's big nodes
      a = big_list[blockIdx.y];
      gslot = by_node ? a : blockIdx.y;
      mode = 2;
      start = 0;
      cnt = 0;
    }
  } else if (mode == 5) {
    if (a >= plan[2] || derive_from[a] < 0) return;
    start = 0;
    cnt = 0;
  } else {
    // grid.z > 1 (histogram-only mode): the node's rows are split over gridDim.z workgroups
    const int cnt_all = node_count[a];
    const int per_z = (cnt_all + gridDim.z - 1) / gridDim.z;
    const int zb = min(cnt_all, (int)blockIdx.z * per_z);
    start = node_start[a] + zb;
    cnt = min(cnt_all, zb + per_z) - zb;
  }
  const bool merge = (gridDim.z > 1) || (plan != nullptr);  // mode 1 adds into a zeroed ghist

  float* gh = ghist ? ghist + ((size_t)gslot * m + f_lo) * maxbins * K : nullptr;
  if (mode == 5) {
    const size_t slot = (size_t)m * maxbins * K, off = (size_t)f_lo * maxbins * K;
    const float* hp = hprev + (size_t)parent_of[a] * slot + off;
    const float* hs = ghist + (size_t)derive_from[a] * slot + off;
    for (int i = tid; i < f_n * maxbins * K; i += blockDim.x) {
      const float v = hp[i] - hs[i];
      hist[i] = v;
      gh[i] = v;
    }
    mode = 2;
  } else {
    for (int i = tid; i < f_n * maxbins * K; i += blockDim.x) hist[i] = (mode == 2) ? gh[i] : 0.f;
  }
  for (int i = tid; i < f_n; i += blockDim.x) fid[i] = feats[(size_t)a * m + f_lo + i];
  if constexpr (SPARSE) {
    // (every mode: the split search takes the one-hot and the numeric slots apart)
    if (mode != 2)
      for (int i = tid; i < sp.F; i += blockDim.x) slot_of[i] = -1;
    for (int k = tid; k < K; k += blockDim.x) ktot[k] = 0u;
    if (tid == 0) nd_s = 0;
    __syncthreads();
    for (int i = tid; i < f_n; i += blockDim.x) {
      const int f = feats[(size_t)a * m + f_lo + i];
      const bool oh = sp.onehot[f] != 0;
      if (mode != 2) slot_of[f] = (short)i;
      sflag[i] = oh ? (nbins_feat[f] >= 2 ? 1 : 2) : 0;
      if (!oh) dlist[atomicAdd(&nd_s, 1)] = (short)i;  // (order free: integer sums, index-ordered ties)
    }
  }
  __syncthreads();

  // ---- histogram ----
  const int rpi = f_n <= 64 ? (int)blockDim.x / f_n : 0;
  if constexpr (SPARSE) {
    if (mode != 2) {
      // one thread per row, U rows in flight (the row id -> label / one-hot entries loads are a
      // dependent chain); class totals in registers (K <= 8) or LDS atomics
      unsigned int* hu = reinterpret_cast<unsigned int*>(hist);
      const int nd = nd_s, nc = sp.ncat;
      unsigned int acc[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
      auto row_add = [&](int r, unsigned int wu, int l, const int (&fr)[SP_NCAT]) __attribute__((always_inline)) {
#pragma unroll
        for (int c = 0; c < SP_NCAT; ++c) {
          if (fr[c] >= 0) {
            const int sl = slot_of[fr[c]];
            if (sl >= 0 && sflag[sl] == 1) atomicAdd(hu + (sl * maxbins + 1) * K + l, wu);
          }
        }
        for (int d = 0; d < nd; ++d) {
          const int sl = dlist[d];
          const int b = bins[(int64_t)fid[sl] * fstride + (int64_t)r * rstride];
          atomicAdd(hu + (sl * maxbins + b) * K + l, wu);
        }
        if (K <= 8) {
#pragma unroll
          for (int k = 0; k < 8; ++k) acc[k] += l == k ? wu : 0u;
        } else {
          atomicAdd(ktot + l, wu);
        }
      };
      constexpr int U = 4;
      int ri = tid;
      for (; ri + (U - 1) * (int)blockDim.x < cnt; ri += U * (int)blockDim.x) {
        int r[U], l[U], fr[U][SP_NCAT];
        unsigned int wu[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          r[u] = rows[start + ri + u * (int)blockDim.x];
          wu[u] = (unsigned int)row_w[start + ri + u * (int)blockDim.x];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          l[u] = label[r[u]];
#pragma unroll
          for (int c = 0; c < SP_NCAT; ++c) fr[u][c] = c < nc ? sp.cat[(int64_t)r[u] * nc + c] : -1;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) row_add(r[u], wu[u], l[u], fr[u]);
      }
      for (; ri < cnt; ri += blockDim.x) {
        const int r = rows[start + ri];
        const unsigned int wu = (unsigned int)row_w[start + ri];
        int fr[SP_NCAT];
#pragma unroll
        for (int c = 0; c < SP_NCAT; ++c) fr[c] = c < nc ? sp.cat[(int64_t)r * nc + c] : -1;
        row_add(r, wu, label[r], fr);
      }
      if (K <= 8) {
        const wops::LaneSwap sw(lane);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          // (integer-valued sums below 2^24: exact in fp32)
          const float v = wops::wave_sum_dpp((float)acc[k], sw);
          if (k < K && lane == 0 && v != 0.f) atomicAdd(ktot + k, (unsigned int)v);
        }
      }
      __syncthreads();
      // bin 0 of every one-hot slot = class totals - bin 1
      for (int i = tid; i < f_n * K; i += blockDim.x) {
        const int sl = i / K, k = i - sl * K;
        if (sflag[sl]) hu[sl * maxbins * K + k] = ktot[k] - hu[(sl * maxbins + 1) * K + k];
      }
    }
  } else if (mode != 2 && rpi > 0) {
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
        for (int u = 0; u < HU; ++u) hist_add<INTW>(hb + b[u] * K + l[u], w[u]);
      }
      for (; ri < cnt; ri += rpi) {
        const int r = rows[start + ri];
        const float w = row_w[start + ri];
        const int b = bins[fo + (int64_t)r * rstride];
        hist_add<INTW>(hb + b * K + label[r], w);
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
        hist_add<INTW>(hl + (fs * maxbins + b) * K, w);
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
      hist_add<INTW>(&hist[(fs * maxbins + b) * K + label[r]], w);
    }
  }
  __syncthreads();
  if (INTW && mode != 2) {  // uint32 counts -> fp32 (exact below 2^24)
    const unsigned int* hu = reinterpret_cast<const unsigned int*>(hist);
    for (int i = tid; i < f_n * maxbins * K; i += blockDim.x) hist[i] = (float)hu[i];
    __syncthreads();
  }
  if (mode == 0 && by_node)  // keep the fused node's histogram for its children's subtraction
    for (int i = tid; i < f_n * maxbins * K; i += blockDim.x) gh[i] = hist[i];
  if (mode == 1) {
    if (!merge || direct) {
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
  const int nwaves = (int)(blockDim.x >> 6);
  const bool pairs = maxbins <= 32;
  if constexpr (SPARSE) {
    // one-hot slots: one LANE per slot — their only candidate is bin 0 (the 0 | 1 split); the per-lane
    // arithmetic is the pair search's at bin 0 (v = bin 0, t = bin 0 + bin 1 in fp32, classes in order),
    // so the gains, and with the (gain, lowest index) rule the winner, are bit for bit the same
    const wops::LaneSwap sws(lane);
    for (int base = wave * 64; base < f_n; base += nwaves * 64) {
      const int fs = base + lane;
      double g = -INFINITY;
      if (fs < f_n && sflag[fs] == 1) {
        double wl = 0.0, wt = 0.0, ql = 0.0, qr = 0.0, qt = 0.0;
        for (int k = 0; k < K; ++k) {
          const float c0 = hist[fs * maxbins * K + k], c1 = hist[(fs * maxbins + 1) * K + k];
          const float tf = c0 + c1;
          const double v = (double)c0, t = (double)tf, r = t - v;
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
        if (wl >= min_inst && wr >= min_inst && wt > 0) {
          double ip, il, ir;
          if (impurity == 0) {
            ip = 1.0 - qt / (wt * wt); il = 1.0 - ql / (wl * wl); ir = 1.0 - qr / (wr * wr);
          } else {
            ip = log2(wt) - qt / wt; il = log2(wl) - ql / wl; ir = log2(wr) - qr / wr;
          }
          g = ip - (wl / wt) * il - (wr / wt) * ir;
        }
      }
      int idx = fs * maxbins;
      wops::wave_argmax(g, idx, sws);
      if (g > best_g || (g == best_g && idx < best_i)) { best_g = g; best_i = idx; }
    }
    // numeric slots: the pair search over their list
    split_search_pairs<8>(hist, fid, nbins_feat, nd_s, maxbins, K, min_inst, impurity, wave, nwaves, lane, best_g,
                          best_i, dlist);
  } else if (pairs)
    split_search_pairs<8>(hist, fid, nbins_feat, f_n, maxbins, K, min_inst, impurity, wave, nwaves, lane, best_g,
                          best_i);
  const wops::LaneSwap swl(lane);
  for (int fs = wave; !pairs && fs < f_n; fs += nwaves) {
    const int nb = __builtin_amdgcn_readfirstlane(nbins_feat[fid[fs]]);
    double wl = 0.0, wt = 0.0, ql = 0.0, qr = 0.0, qt = 0.0;
    for (int k = 0; k < K; ++k) {
      // the bin scan runs in fp32 on the VALU (DPP): the sums are exact for integer-valued weights
      // below 2^24 (bootstrap counts, fold masks), as the CPU oracle's float32 cumsum; the gains
      // below are fp64
      float vf = (lane < nb && lane < maxbins) ? hist[(fs * maxbins + lane) * K + k] : 0.f;
      vf = wops::scan64_add(vf);
      const double v = (double)vf;
      const double t = (double)wops::lane_f(vf, max(nb - 1, 0));
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
    wops::wave_argmax(g, idx, swl);  // lowest index on ties
    if (g > best_g || (g == best_g && idx < best_i)) { best_g = g; best_i = idx; }
  }
  if (lane == 0) { red_gain[wave] = best_g; red_idx[wave] = best_i; }
  __syncthreads();
  if (wave == 0) {
    // every lane reads the four wave winners (LDS broadcast); lanes = bins for the class sums:
    // the left child's counts (bins <= b of the winning feature) and the node totals are wave
    // reductions instead of one thread's 2 x K x maxbins serial LDS reads (integer-valued
    // weights: the sums are exact in any order)
    double g = red_gain[0];
    int idx = red_idx[0];
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w)
      if (red_gain[w] > g || (red_gain[w] == g && red_idx[w] < idx)) { g = red_gain[w]; idx = red_idx[w]; }
    const size_t o = (size_t)a * chunks + c;
    const bool ok = isfinite(g) && g >= (double)min_gain;
    const int fs = ok ? idx / maxbins : 0, b = ok ? idx % maxbins : 0;
    if (lane == 0) {
      out_gain[o] = ok ? (float)g : -INFINITY;
      out_feat[o] = fid[fs];
      out_bin[o] = b;
    }
    for (int k = 0; k < K; ++k) {
      float vl = (ok && lane <= b) ? hist[(fs * maxbins + lane) * K + k] : 0.f;
      float vt = (c == 0 && lane < maxbins) ? hist[lane * K + k] : 0.f;
      vl = wops::wave_sum_dpp(vl, swl);
      vt = wops::wave_sum_dpp(vt, swl);
      if (lane == 0) {
        out_left[o * K + k] = vl;
        if (c == 0) out_total[(size_t)a * K + k] = vt;
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
  const wops::LaneSwap sw(lane);
#pragma unroll
  for (int k = 0; k < KC; ++k) {
    const float v = wops::wave_sum_dpp(acc[k], sw);
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
struct CdfTable {
  uint32_t thr[16];
  int n;  // 0: every weight 1 (no sampling)
};

__global__ __launch_bounds__(256) void tree_init_kernel(uint64_t seed, int tree0, int64_t row0, int64_t n,
                                                        CdfTable cdf, const float* __restrict__ rw,
                                                        const int32_t* __restrict__ y, int K,
                                                        float* __restrict__ W, int32_t* __restrict__ node_of,
                                                        float* __restrict__ stats, int64_t stats_tree_stride,
                                                        int32_t* __restrict__ bad) {
  __shared__ float cnt[KMAX];
  const int t = blockIdx.y;
  if (threadIdx.x < KMAX) cnt[threadIdx.x] = 0.f;
  __syncthreads();
  const int64_t r0 = (int64_t)blockIdx.x * INIT_ROWS, r1 = min(n, r0 + INIT_ROWS);
  int badl = 0;
  for (int64_t r = r0 + threadIdx.x; r < r1; r += 256) {
    float w = 1.f;
    if (cdf.n > 0) {  // bootstrap draw: #{k : u >= thr[k]} (Poisson(rate) or Bernoulli(rate) table)
      const uint32_t u = philox_u32(seed, 0x1000u + (uint32_t)(tree0 + t), (uint64_t)(row0 + r));
      int k = 0;
      while (k < cdf.n && u >= cdf.thr[k]) ++k;
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

// findSplits sample sort: column f of the row-major sample X [n][ld] -> ascending out[f][0..n) with
// NaN last (torch.sort's order), one workgroup per feature: order-preserving uint32 keys (NaN ->
// 0xFFFFFFFF, also the padding up to the power of two N2 <= FS_MAXN) bitonic-sorted in LDS.
__device__ __forceinline__ uint32_t sort_key(float x) {
  const uint32_t u = __float_as_uint(x);
  return isnan(x) ? 0xFFFFFFFFu : ((u >> 31) ? ~u : (u | 0x80000000u));
}
__device__ __forceinline__ float sort_val(uint32_t k) {
  return k == 0xFFFFFFFFu ? __uint_as_float(0x7FC00000u) : __uint_as_float((k >> 31) ? (k & 0x7FFFFFFFu) : ~k);
}
__global__ __launch_bounds__(1024) void sort_columns_kernel(const float* __restrict__ X, int n, int ld, int N2,
                                                            float* __restrict__ out) {
  extern __shared__ uint32_t skey[];
  const int f = blockIdx.x, tid = threadIdx.x;
  for (int i = tid; i < N2; i += 1024) skey[i] = i < n ? sort_key(X[(size_t)i * ld + f]) : 0xFFFFFFFFu;
  __syncthreads();
  for (int k = 2; k <= N2; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < (N2 >> 1); i += 1024) {
        const int a = ((i & ~(j - 1)) << 1) | (i & (j - 1)), b = a + j;
        const uint32_t ka = skey[a], kb = skey[b];
        if ((ka > kb) == ((a & k) == 0)) {
          skey[a] = kb;
          skey[b] = ka;
        }
      }
      __syncthreads();
    }
  }
  float* o = out + (size_t)f * n;
  for (int i = tid; i < n; i += 1024) o[i] = sort_val(skey[i]);
}
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

// Load-balanced level plan (one workgroup): node a is one work item when it has <= prows rows,
// else ceil(count / prows) chunk items and a slot in the merged-histogram buffer.  plan layout
// (int32): [0] items, [1] big nodes, [2] A, [3] unused, item_start [A + 1], big_rank [A] (-1 = not
// big), big_list [A], item_node [items].  Thread t owns the contiguous nodes [t * per, (t+1) * per):
// one pass sums its items / big nodes, ONE block scan gives its offsets, a second pass writes —
// two barriers per level instead of three per 1024 nodes.
__global__ __launch_bounds__(1024) void tree_plan_kernel(const int32_t* __restrict__ counts, int A, int prows,
                                                         int32_t* __restrict__ plan, const int32_t* __restrict__ a_dev) {
  __shared__ int wsum_i[16], wsum_b[16];
  if (a_dev) A = *a_dev;  // the level's candidate count (the host's A is then only a bound)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int32_t* item_start = plan + 4;
  int32_t* big_rank = item_start + A + 1;
  int32_t* big_list = big_rank + A;
  int32_t* item_node = big_list + A;
  const int per = (A + 1023) >> 10;
  const int b = min(A, tid * per), e = min(A, b + per);
  int ti = 0, tb = 0;
  for (int a = b; a < e; ++a) {
    const int cnt = counts[a];
    const bool big = cnt > prows;
    ti += big ? (cnt + prows - 1) / prows : 1;
    tb += big;
  }
  // exclusive block scan of (items, big nodes): wave shuffles, then the 16 wave totals
  const int si = wops::scan64_add(ti), sb = wops::scan64_add(tb);
  if (lane == 63) { wsum_i[wave] = si; wsum_b[wave] = sb; }
  __syncthreads();
  int oi = si - ti, ob = sb - tb, all_i = 0, all_b = 0;
#pragma unroll
  for (int w = 0; w < 16; ++w) {
    oi += w < wave ? wsum_i[w] : 0;
    ob += w < wave ? wsum_b[w] : 0;
    all_i += wsum_i[w];
    all_b += wsum_b[w];
  }
  for (int a = b; a < e; ++a) {
    const int cnt = counts[a];
    const bool big = cnt > prows;
    const int zc = big ? (cnt + prows - 1) / prows : 1;
    item_start[a] = oi;
    big_rank[a] = big ? ob : -1;
    if (big) big_list[ob++] = a;
    for (int z = 0; z < zc; ++z) item_node[oi + z] = a;
    oi += zc;
  }
  if (tid == 0) {
    item_start[A] = all_i;
    plan[0] = all_i;
    plan[1] = all_b;
    plan[2] = A;
    plan[3] = 0;
  }
}

// Zero the merged-histogram slots of this level's big nodes only (grid = an upper bound; the
// real count is read from the plan).
__global__ __launch_bounds__(256) void tree_plan_zero_kernel(const int32_t* __restrict__ plan, int64_t slot_elems,
                                                             float* __restrict__ ghist, int by_node) {
  const int64_t n = (int64_t)plan[1] * slot_elems;
  const int32_t* big_list = plan + 4 + (plan[2] + 1) + plan[2];
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    // by_node: the big nodes' own slots of the per-node store (else slots 0..big nodes - 1)
    const int64_t j = i / slot_elems;
    ghist[by_node ? (int64_t)big_list[j] * slot_elems + (i - j * slot_elems) : i] = 0.f;
  }
}

// Bins of a hybrid (one-hot index + numeric) matrix straight from its parts, feature-major [F][n]
// like bin_features of the dense matrix (zeroed by the launcher): a numeric column's bin = #thresholds
// strictly below x (NaN -> last), a one-hot column with its threshold (0.5) gets bin 1 in the rows
// whose entry it is.  One thread per row; no dense [n][F] matrix is read.
__global__ __launch_bounds__(256) void tree_bins_hybrid_kernel(const float* __restrict__ dense, int64_t n, int Fd,
                                                               const int32_t* __restrict__ dense_cols,
                                                               const int32_t* __restrict__ cat, int ncat,
                                                               const float* __restrict__ thr, int maxb,
                                                               const int32_t* __restrict__ nbins,
                                                               uint8_t* __restrict__ bins) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  for (int j = 0; j < Fd; ++j) {
    const int f = dense_cols[j];
    const int nt = nbins[f] - 1;
    const float* t = thr + (size_t)f * maxb;
    const float x = dense[i * Fd + j];
    int lo = 0, hi = nt;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (t[mid] < x) lo = mid + 1; else hi = mid;
    }
    bins[(size_t)f * n + i] = (uint8_t)(x == x ? lo : nt);
  }
  for (int c = 0; c < ncat; ++c) {
    const int f = cat[i * ncat + c];
    if (f >= 0 && nbins[f] >= 2) bins[(size_t)f * n + i] = 1;
  }
}

// findSplits of a hybrid matrix on the device (ops/tree.py thresholds_hybrid_device): the ones of every
// one-hot column over the (sampled) rows, then per column its thresholds row of the padded matrix
// [F][maxb] (+inf after the count) and its bin count: a one-hot column gets the 0 | 1 split (0.5) when
// the rows hold both values, a numeric column the sorted-sample thresholds of find_splits_post_sort
// (dthr [Fd][ns + 1], the count last).  No host round trip.
__global__ __launch_bounds__(256) void tree_onehot_counts_kernel(const int32_t* __restrict__ cat, int64_t n, int ncat,
                                                                 int32_t* __restrict__ ones) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * ncat) return;
  const int f = cat[i];
  if (f >= 0) atomicAdd(ones + f, 1);
}

__global__ __launch_bounds__(256) void tree_thresholds_hybrid_kernel(int F, const int32_t* __restrict__ colmap,
                                                                     const int32_t* __restrict__ ones, int n,
                                                                     const float* __restrict__ dthr, int ns, int maxb,
                                                                     float* __restrict__ thr_mat,
                                                                     int32_t* __restrict__ nbins) {
  const int f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= F) return;
  float* row = thr_mat + (size_t)f * maxb;
  const int j = colmap[f];  // numeric column index, < 0: one-hot
  int cnt;
  if (j >= 0) {
    const float* d = dthr + (size_t)j * (ns + 1);
    cnt = (int)d[ns];
    for (int k = 0; k < maxb; ++k) row[k] = k < cnt ? d[k] : INFINITY;
  } else {
    const int o = ones[f];
    cnt = (o > 0 && o < n) ? 1 : 0;
    for (int k = 0; k < maxb; ++k) row[k] = (k == 0 && cnt) ? 0.5f : INFINITY;
  }
  nbins[f] = cnt + 1;
}

}  // namespace

extern "C" int har_tree_thresholds_hybrid(const int32_t* cat, int64_t n, int ncat, int F, const int32_t* colmap,
                                          const float* dthr, int ns, int maxb, int32_t* ones, float* thr_mat,
                                          int32_t* nbins, hipStream_t s) {
  if (n <= 0 || ncat < 0 || F <= 0 || ns <= 0 || maxb < ns || n > 0x7fffffff) return -2;
  if (hipMemsetAsync(ones, 0, (size_t)F * sizeof(int32_t), s) != hipSuccess) return -1;
  if (ncat > 0)
    tree_onehot_counts_kernel<<<(unsigned)((n * ncat + 255) / 256), 256, 0, s>>>(cat, n, ncat, ones);
  tree_thresholds_hybrid_kernel<<<(F + 255) / 256, 256, 0, s>>>(F, colmap, ones, (int)n, dthr, ns, maxb, thr_mat, nbins);
  HAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int har_tree_bins_hybrid(const float* dense, int64_t n, int Fd, const int32_t* dense_cols,
                                    const int32_t* cat, int ncat, int F, const float* thr, int maxb,
                                    const int32_t* nbins, uint8_t* bins, hipStream_t s) {
  if (n < 0 || Fd < 0 || ncat < 0 || F <= 0 || maxb <= 0) return -2;
  if (n == 0) return 0;
  if (hipMemsetAsync(bins, 0, (size_t)F * n, s) != hipSuccess) return -1;
  tree_bins_hybrid_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(dense, n, Fd, dense_cols, cat, ncat, thr, maxb,
                                                                     nbins, bins);
  HAR_CHECK_LAUNCH();
  return 0;
}

// bins: feature-major [F][N] (row_major = 0) or row-major [N][F] (row_major = 1: the bytes of one
// row's sampled features share one or two cache lines — the deep levels gather far less).
extern "C" int har_tree_hist_split(const uint8_t* bins, int64_t N, int F, int row_major, const int32_t* nbins_feat,
                                   const int32_t* rows, const float* row_w, const int32_t* node_start,
                                   const int32_t* node_count, int A, const int32_t* feats, int m, int fc,
                                   const int32_t* label, int K, int maxbins, float min_inst, float min_gain,
                                   int impurity, float* out_gain, int32_t* out_feat, int32_t* out_bin,
                                   float* out_left, float* out_total, int mode, float* ghist, int row_chunks,
                                   const TreeSparse* sparse, hipStream_t s) {
  return har_tree_hist_split_planned(bins, N, F, row_major, nbins_feat, rows, row_w, node_start, node_count, A, feats,
                                     m, fc, label, K, maxbins, min_inst, min_gain, impurity, out_gain, out_feat,
                                     out_bin, out_left, out_total, mode, ghist, row_chunks, nullptr, 0, 0, 0,
                                     nullptr, nullptr, nullptr, sparse, s);
}

// planned modes (plan != nullptr): grid.y = `bound` (work items for modes 3 / 6, big-node slots for
// mode 4, nodes for mode 5, the rank's node slice for mode 7, whose first global node is `prows`)
extern "C" int har_tree_hist_split_planned(const uint8_t* bins, int64_t N, int F, int row_major,
                                           const int32_t* nbins_feat, const int32_t* rows, const float* row_w,
                                           const int32_t* node_start, const int32_t* node_count, int A,
                                           const int32_t* feats, int m, int fc, const int32_t* label, int K,
                                           int maxbins, float min_inst, float min_gain, int impurity,
                                           float* out_gain, int32_t* out_feat, int32_t* out_bin, float* out_left,
                                           float* out_total, int mode, float* ghist, int row_chunks,
                                           const int32_t* plan, int prows, int bound, int by_node,
                                           const float* hprev, const int32_t* derive_from,
                                           const int32_t* parent_of, const TreeSparse* sparse, hipStream_t s) {
  if (K > KMAX || maxbins > 64 || fc <= 0 || m <= 0) return -2;
  // one-hot-aware histograms: integer weights, <= SP_NCAT one-hot entries per row, the maps in LDS
  const bool sp_on = sparse && sparse->cat && sparse->onehot && sparse->ncat > 0;
  if (sp_on && (sparse->ncat > SP_NCAT || sparse->F != F || maxbins < 2 || maxbins > 32 || F > 32767)) return -8;
  if (mode != 0 && !ghist) return -4;
  const bool planned = mode >= 3 && mode <= 7;
  if (planned && (!plan || (mode != 7 && prows <= 0) || prows < 0)) return -6;
  if (mode == 5 && (!by_node || !hprev || !derive_from || !parent_of)) return -7;
  if ((mode == 6 || mode == 7) && (!by_node || derive_from)) return -7;
  if (by_node && !planned) return -7;
  if (A == 0) return 0;
  const int chunks = (m + fc - 1) / fc;
  const size_t lds = (size_t)fc * maxbins * K * sizeof(float) + (size_t)fc * sizeof(int) +
                     (sp_on ? (size_t)K * 4 + (size_t)F * 2 + (size_t)fc * 3 : 0);
  if (lds > 150 * 1024) return -3;
  if (row_chunks > 1 && mode != 1) return -5;
  if (planned && bound <= 0) return 0;
  dim3 grid(chunks, planned ? bound : A, row_chunks > 1 ? row_chunks : 1);
  const int64_t fstride = row_major ? 1 : N, rstride = row_major ? F : 1;
  // integer-weight accumulation unless HAR_HIST_FLOAT_ATOMICS=1 (A/B switch; same results)
  static const bool float_atomics = [] {
    const char* e = getenv("HAR_HIST_FLOAT_ATOMICS");
    return e && e[0] == '1';
  }();
  if (sp_on && float_atomics) return -8;  // (bin 0 = totals - bin 1 is exact for the integer counts only)
  const TreeSparse spv = sp_on ? *sparse : TreeSparse{};
  auto kern = sp_on ? tree_hist_split_kernel<true, true>
              : float_atomics ? tree_hist_split_kernel<false, false> : tree_hist_split_kernel<true, false>;
  kern<<<grid, 256, lds, s>>>(bins, fstride, rstride, nbins_feat, rows, row_w, node_start, node_count, feats, m, fc,
                              label, K, maxbins, min_inst, min_gain, impurity, out_gain, out_feat, out_bin, out_left,
                              out_total, mode, ghist, planned ? plan : nullptr, prows, by_node, hprev, derive_from,
                              parent_of, spv);
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
  if (ntrees < 0 || n < 0) return -2;
  int64_t total = (int64_t)ntrees * n;
  if (total == 0) return 0;
  int blocks = (int)std::min<int64_t>(4096, (total + 255) / 256);
  poisson_bootstrap_kernel<<<blocks, 256, 0, s>>>(seed, tree0, ntrees, row0, n, out);
  HAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int har_tree_init(uint64_t seed, int tree0, int ntrees, int64_t row0, int64_t n, const uint32_t* cdf,
                             int ncdf, const float* rw, const int32_t* y, int K, float* W, int32_t* node_of,
                             float* stats, int64_t stats_tree_stride, int32_t* bad, hipStream_t s) {
  if (K <= 0 || K > KMAX || ncdf < 0 || ncdf > 16) return -2;
  if (n == 0 || ntrees == 0) return 0;
  CdfTable tab{};
  tab.n = ncdf;
  for (int i = 0; i < ncdf; ++i) tab.thr[i] = cdf[i];  // host array (kernel argument)
  dim3 grid((unsigned)((n + INIT_ROWS - 1) / INIT_ROWS), (unsigned)ntrees);
  tree_init_kernel<<<grid, 256, 0, s>>>(seed, tree0, row0, n, tab, rw, y, K, W, node_of, stats, stats_tree_stride,
                                        bad);
  HAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int har_sort_columns(const float* X, int n, int F, int ld, float* out, hipStream_t s) {
  if (n <= 0 || n > FS_MAXN || F < 0 || ld < F) return -2;
  if (F == 0) return 0;
  int N2 = 2;
  while (N2 < n) N2 <<= 1;
  sort_columns_kernel<<<F, 1024, (size_t)N2 * sizeof(uint32_t), s>>>(X, n, ld, N2, out);
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

extern "C" int har_tree_plan(const int32_t* counts, int A, int prows, int32_t* plan, int64_t slot_elems,
                             float* ghist, int max_big, int by_node, const int32_t* a_dev, hipStream_t s) {
  if (A <= 0 || prows <= 0) return -2;
  tree_plan_kernel<<<1, 1024, 0, s>>>(counts, A, prows, plan, a_dev);
  HAR_CHECK_LAUNCH();
  if (ghist && max_big > 0) {
    const int64_t n = (int64_t)max_big * slot_elems;
    const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>(4096, (n + 255) / 256));
    tree_plan_zero_kernel<<<blocks, 256, 0, s>>>(plan, slot_elems, ghist, by_node);
    HAR_CHECK_LAUNCH();
  }
  return 0;
}
