// Per-level bookkeeping of the level-synchronous forest builder (SURVEY.md K13/K16,
// N8 BaggedPoint / node assignment), so a level runs on the device without the
// host or chains of int64 tensor ops over all (tree, row) pairs:
//
//   tree_feature_subsets : per (tree, node) pair, Floyd sampling of m distinct features
//                          out of F with Philox4x32-10 — bit-identical to
//                          har/ops/rng.py feature_subsets (counter t<<32 | n<<8 | i,
//                          stream 0x7F000000), sorted ascending (featureSubsetStrategy).
//   tree_level_keys      : key[t][r] = candidate index of the node row r of tree t sits in
//                          (-1: out of bag, finished, or node not split this level).
//   tree_level_group     : the level's (tree, row) -> candidate grouping WITHOUT a sort:
//                          per-chunk counts, a column prefix over chunks, one scan over
//                          candidates, then a stable wave-ordered scatter of row ids and
//                          bootstrap weights — the same order as a stable sort of the
//                          keys, but only the active rows are written and no key array
//                          ever reaches HBM.
//   tree_partition       : after the level's splits, move every row of a split node to
//                          its child (bin <= threshold bin -> left) and retire the rows
//                          of nodes that became leaves — one pass over [T][N] int32.
#include "common.h"
#include "philox.h"
#include "../har_kernels.h"

namespace {

constexpr uint32_t STREAM_FEATURE_SUBSET = 0x7F000000u;
constexpr int MAX_SUBSET = 128;

// One wave per (tree, node): lane L draws Floyd step i = L (and L + 64) — the Philox values
// do not depend on earlier steps — then the m sequential membership tests are wave ballots over
// the lanes' chosen values (no per-thread scratch arrays), and the ascending order is each
// value's rank among the m distinct choices.
__global__ __launch_bounds__(256) void tree_feature_subsets_kernel(uint64_t seed, const int32_t* __restrict__ trees,
                                                                   const int32_t* __restrict__ nodes, int64_t P,
                                                                   int F, int m, int32_t* __restrict__ out,
                                                                   const int32_t* __restrict__ p_dev) {
  const int lane = threadIdx.x & 63;
  const int64_t p = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (p >= (p_dev ? (int64_t)*p_dev : P)) return;  // wave-uniform (P = grid bound when p_dev is given)
  const uint64_t base = ((uint64_t)(uint32_t)trees[p] << 32) | ((uint64_t)(uint32_t)nodes[p] << 8);
  int t0 = 0, t1 = 0;  // the draw of step lane / lane + 64 (t in [0, j], j = F - m + i)
  if (lane < m) t0 = (int)(philox_u32(seed, STREAM_FEATURE_SUBSET, base + (uint64_t)lane) % (uint32_t)(F - m + lane + 1));
  if (lane + 64 < m)
    t1 = (int)(philox_u32(seed, STREAM_FEATURE_SUBSET, base + (uint64_t)(lane + 64)) % (uint32_t)(F - m + lane + 65));
  int c0 = -1, c1 = -1;  // chosen[lane], chosen[lane + 64]
  for (int i = 0; i < m; ++i) {
    const int t = i < 64 ? __shfl(t0, i, 64) : __shfl(t1, i - 64, 64);
    const bool dup = __any((c0 == t) || (c1 == t));
    const int v = dup ? F - m + i : t;
    if (i < 64) { if (lane == i) c0 = v; } else if (lane == i - 64) c1 = v;
  }
  int r0 = 0, r1 = 0;  // ranks among the distinct choices
  for (int q = 0; q < m; ++q) {
    const int v = q < 64 ? __shfl(c0, q, 64) : __shfl(c1, q - 64, 64);
    r0 += v < c0;
    r1 += v < c1;
  }
  int32_t* o = out + p * m;
  if (lane < m) o[r0] = c0;
  if (lane + 64 < m) o[r1] = c1;
}

__global__ __launch_bounds__(256) void tree_level_keys_kernel(const int32_t* __restrict__ node_of,
                                                              const int32_t* __restrict__ cand_idx, int T, int64_t N,
                                                              int maxn, int32_t* __restrict__ key) {
  const int64_t total = (int64_t)T * N;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < total; j += (int64_t)gridDim.x * blockDim.x) {
    const int n = node_of[j];
    const int t = (int)(j / N);
    key[j] = n >= 0 ? cand_idx[(int64_t)t * maxn + n] : -1;
  }
}

__global__ __launch_bounds__(256) void tree_partition_kernel(int32_t* __restrict__ node_of,
                                                             const int32_t* __restrict__ lvl_feat,
                                                             const int32_t* __restrict__ lvl_bin,
                                                             const int32_t* __restrict__ lvl_left,
                                                             const uint8_t* __restrict__ bins, int T, int64_t N,
                                                             int maxn) {
  const int64_t total = (int64_t)T * N;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < total; j += (int64_t)gridDim.x * blockDim.x) {
    const int n = node_of[j];
    if (n < 0) continue;
    const int t = (int)(j / N);
    const int64_t r = j - (int64_t)t * N;
    const int64_t o = (int64_t)t * maxn + n;
    const int f = lvl_feat[o];
    if (f < 0) { node_of[j] = -1; continue; }  // leaf (or not split this level): the row is done
    const int b = bins[(int64_t)f * N + r];
    node_of[j] = lvl_left[o] + (b <= lvl_bin[o] ? 0 : 1);
  }
}


// ---- level grouping (replaces sort + gather + binary search of the level keys) ----------
// Chunks of GROUP_CH rows of one tree, one wave each (4 per workgroup); the candidates of a
// tree are the contiguous range [tree_lo[t], tree_lo[t+1]) (the frontier is tree-ordered), so a
// wave keeps per-candidate counters for its tree in a private LDS slice of nt_max ints.
constexpr int GROUP_CH = 1024;
constexpr int GROUP_WAVES = 4;
constexpr int GROUP_MAX_NT = 4096;  // 4 waves x 4096 x 4 B = 64 KB of LDS

__device__ __forceinline__ int group_key(const int32_t* __restrict__ no, const int32_t* __restrict__ ci, int64_t r,
                                         int64_t r1, int lo) {
  if (r >= r1) return -1;
  const int n = no[r];
  if (n < 0) return -1;
  const int a = ci[n];
  return a >= 0 ? a - lo : -1;
}

__global__ __launch_bounds__(256) void tree_group_count_kernel(const int32_t* __restrict__ node_of,
                                                               const int32_t* __restrict__ cand_idx,
                                                               const int32_t* __restrict__ tree_lo, int64_t N,
                                                               int maxn, int nch, int A, int nt_max,
                                                               int32_t* __restrict__ cnt) {
  extern __shared__ int32_t glds[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int t = blockIdx.y, c = blockIdx.x * GROUP_WAVES + wave;
  const int lo = tree_lo[t], nt = tree_lo[t + 1] - lo;
  if (nt == 0) return;  // block-uniform: no candidate of tree t at this level, nothing to count
  const bool live = c < nch;
  int32_t* h = glds + wave * nt_max;
  for (int i = lane; i < nt; i += 64) h[i] = 0;
  __syncthreads();
  const int32_t* no = node_of + (int64_t)t * N;
  const int32_t* ci = cand_idx + (int64_t)t * maxn;
  const int64_t r0 = (int64_t)c * GROUP_CH, r1 = live ? (r0 + GROUP_CH < N ? r0 + GROUP_CH : N) : r0;
  for (int64_t r = r0 + lane; r < r1; r += 64) {
    const int k = group_key(no, ci, r, r1, lo);
    if (k >= 0) atomicAdd(&h[k], 1);
  }
  __syncthreads();
  if (live)
    for (int i = lane; i < nt; i += 64) cnt[(int64_t)c * A + lo + i] = h[i];
}

// cnt[c][a] -> exclusive prefix over chunks c; total[a] = sum.  Coalesced over a.
// A is the row stride of cnt; a_dev (if given) the level's candidate count (<= A).
__global__ __launch_bounds__(256) void tree_group_colscan_kernel(int32_t* __restrict__ cnt, int nch, int A,
                                                                 int32_t* __restrict__ total,
                                                                 const int32_t* __restrict__ a_dev) {
  const int a = blockIdx.x * 256 + threadIdx.x;
  if (a >= (a_dev ? *a_dev : A)) return;
  // 8 chunk counts loaded before any prefix is stored: the loads of a group are independent
  // (one latency per 8 chunks instead of one per chunk)
  constexpr int U = 8;
  int run = 0, c = 0;
  for (; c + U <= nch; c += U) {
    int v[U];
#pragma unroll
    for (int j = 0; j < U; ++j) v[j] = cnt[(int64_t)(c + j) * A + a];
#pragma unroll
    for (int j = 0; j < U; ++j) {
      cnt[(int64_t)(c + j) * A + a] = run;
      run += v[j];
    }
  }
  for (; c < nch; ++c) {
    const int v = cnt[(int64_t)c * A + a];
    cnt[(int64_t)c * A + a] = run;
    run += v;
  }
  total[a] = run;
}

// One workgroup: exclusive scan of total[0..A) -> starts (A is the level's candidate count).
__global__ __launch_bounds__(1024) void tree_group_scan_kernel(const int32_t* __restrict__ total, int A,
                                                               int32_t* __restrict__ starts,
                                                               const int32_t* __restrict__ a_dev) {
  __shared__ int32_t wsum[16];
  if (a_dev) A = *a_dev;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int per = (A + 1023) / 1024;
  const int b = tid * per, e = b + per < A ? b + per : A;
  int s = 0;
  for (int i = b; i < e; ++i) s += total[i];
  int x = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  int run = x - s;
  for (int i = 0; i < w; ++i) run += wsum[i];
  for (int i = b; i < e; ++i) {
    starts[i] = run;
    run += total[i];
  }
}

// Stable scatter: a wave walks its chunk 64 rows at a time; lanes with the same candidate
// find each other with one ballot per key bit, the lowest such lane advances the LDS cursor,
// and each lane's slot is the cursor plus the number of same-key lanes below it — exactly
// the position a stable sort of (key, tree * N + row) would give.
__global__ __launch_bounds__(256) void tree_group_scatter_kernel(const int32_t* __restrict__ node_of,
                                                                 const int32_t* __restrict__ cand_idx,
                                                                 const int32_t* __restrict__ tree_lo,
                                                                 const float* __restrict__ W, int64_t N, int maxn,
                                                                 int nch, int A, int nt_max,
                                                                 const int32_t* __restrict__ cnt,
                                                                 const int32_t* __restrict__ starts,
                                                                 int32_t* __restrict__ rows,
                                                                 float* __restrict__ row_w) {
  extern __shared__ int32_t glds[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int t = blockIdx.y, c = blockIdx.x * GROUP_WAVES + wave;
  const int lo = tree_lo[t], nt = tree_lo[t + 1] - lo;
  if (nt == 0) return;  // block-uniform
  const bool live = c < nch;
  int32_t* h = glds + wave * nt_max;
  if (live)
    for (int i = lane; i < nt; i += 64) h[i] = cnt[(int64_t)c * A + lo + i] + starts[lo + i];
  __syncthreads();
  const int nbits = nt > 1 ? 32 - __clz(nt - 1) : 0;
  const int32_t* no = node_of + (int64_t)t * N;
  const int32_t* ci = cand_idx + (int64_t)t * maxn;
  const float* wt = W + (int64_t)t * N;
  const uint64_t below = (1ull << lane) - 1ull;
  const int64_t r0 = (int64_t)c * GROUP_CH, r1 = live ? (r0 + GROUP_CH < N ? r0 + GROUP_CH : N) : r0;
  for (int64_t rb = r0; rb < r1; rb += 64) {  // wave-uniform trip count: every ballot has all lanes
    const int64_t r = rb + lane;
    const int k = group_key(no, ci, r, r1, lo);
    uint64_t peers = __ballot(k >= 0);
    for (int bit = 0; bit < nbits; ++bit) {
      const int on = (k >> bit) & 1;
      const uint64_t m = __ballot(on);
      peers &= on ? m : ~m;
    }
    const int base = k >= 0 ? h[k] : 0;
    __builtin_amdgcn_wave_barrier();
    if (k >= 0) {
      if ((peers & below) == 0) h[k] = base + (int)__popcll(peers);
      const int pos = base + (int)__popcll(peers & below);
      rows[pos] = (int32_t)r;
      row_w[pos] = wt[r];
    }
    __builtin_amdgcn_wave_barrier();
  }
}

// One thread per node split this level: write the node's split (feature, bin, threshold,
// children, gain) and both children's class statistics — the level's ~15 index_put / gather
// launches as one.  Indices come from the host (int64, one pinned upload).
__global__ __launch_bounds__(256) void tree_commit_level_kernel(
    int S, const int64_t* __restrict__ ti, const int64_t* __restrict__ ni, const int64_t* __restrict__ cl,
    const int64_t* __restrict__ dsi, const int32_t* __restrict__ rfeat, const int32_t* __restrict__ rbin,
    const float* __restrict__ rgain, const float* __restrict__ rleft, const float* __restrict__ rtotal, int K,
    const float* __restrict__ thr_mat, int ldthr, int maxn, int32_t* __restrict__ feature,
    int32_t* __restrict__ split_bin, float* __restrict__ thresh, int32_t* __restrict__ left,
    int32_t* __restrict__ right, float* __restrict__ gains, float* __restrict__ stats,
    const int32_t* __restrict__ s_dev) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (s_dev ? *s_dev : S)) return;
  const int64_t j = dsi[i];
  const int64_t o = ti[i] * maxn + ni[i];
  const int c = (int)cl[i];
  const int f = rfeat[j], b = rbin[j];
  feature[o] = f;
  split_bin[o] = b;
  thresh[o] = thr_mat[(int64_t)f * ldthr + b];
  left[o] = c;
  right[o] = c + 1;
  const float* L = rleft + j * K;
  const float* Tt = rtotal + j * K;
  float* sl = stats + (ti[i] * maxn + c) * K;
  float tw = 0.f;
  for (int k = 0; k < K; ++k) {
    const float l = L[k], t = Tt[k];
    sl[k] = l;
    sl[K + k] = t - l;
    tw += t;
  }
  gains[o] = rgain[j] * tw;
}

// Row -> child move reading the committed split arrays directly (feature < 0: the node is a
// leaf or was not split this level, the row is done).
__global__ __launch_bounds__(256) void tree_partition_split_kernel(int32_t* __restrict__ node_of,
                                                                   const int32_t* __restrict__ feature,
                                                                   const int32_t* __restrict__ split_bin,
                                                                   const int32_t* __restrict__ left,
                                                                   const uint8_t* __restrict__ bins, int T,
                                                                   int64_t N, int maxn) {
  const int64_t total = (int64_t)T * N;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < total; j += (int64_t)gridDim.x * blockDim.x) {
    const int n = node_of[j];
    if (n < 0) continue;
    const int t = (int)(j / N);
    const int64_t r = j - (int64_t)t * N;
    const int64_t o = (int64_t)t * maxn + n;
    const int f = feature[o];
    if (f < 0) { node_of[j] = -1; continue; }
    const int b = bins[(int64_t)f * N + r];
    node_of[j] = left[o] + (b <= split_bin[o] ? 0 : 1);
  }
}

// Per candidate after the split search: split or not, and whether each child is itself a
// candidate of the next level (impurity > 1e-12 in fp64 and weight >= 2 * min_instances) —
// out rows: [do_split, left ok, right ok, left weight, right weight], one D2H copy per level.
__global__ __launch_bounds__(256) void tree_level_decide_kernel(int A, const float* __restrict__ gain,
                                                                const float* __restrict__ left,
                                                                const float* __restrict__ total, int K,
                                                                int impurity, float min2, float* __restrict__ out,
                                                                const int32_t* __restrict__ a_dev) {
  // A: row stride of out; a_dev (if given): the level's candidate count
  const int a = blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= (a_dev ? *a_dev : A)) return;
  const float g = gain[a];
  const float* L = left + (int64_t)a * K;
  const float* Tt = total + (int64_t)a * K;
  float wl = 0.f, wr = 0.f;
  for (int k = 0; k < K; ++k) {
    wl += L[k];
    wr += Tt[k] - L[k];
  }
  const double dl = fmax((double)wl, 1e-30), dr = fmax((double)wr, 1e-30);
  double il = 0.0, ir = 0.0;
  for (int k = 0; k < K; ++k) {
    const double pl = (double)L[k] / dl, pr = (double)(Tt[k] - L[k]) / dr;
    if (impurity == 0) {
      il += pl * pl;
      ir += pr * pr;
    } else {
      il -= pl > 0 ? pl * log2(fmax(pl, 1e-30)) : 0.0;
      ir -= pr > 0 ? pr * log2(fmax(pr, 1e-30)) : 0.0;
    }
  }
  if (impurity == 0) {
    il = 1.0 - il;
    ir = 1.0 - ir;
  }
  out[a] = (g > 0.f && isfinite(g)) ? 1.f : 0.f;
  out[A + a] = (il > 1e-12 && wl >= min2) ? 1.f : 0.f;
  out[2 * A + a] = (ir > 1e-12 && wr >= min2) ? 1.f : 0.f;
  out[3 * A + a] = wl;
  out[4 * A + a] = wr;
}

// ---- device-resident frontier: the level's split bookkeeping without host numpy ------------
// Exclusive scan of (flags > 0) over n entries (n = n_mul * *n_dev when n_dev is given) in
// one workgroup; out[n] = total.  Tiles of 1024 x 8 entries: each thread reads its 8
// consecutive flags as two 16-byte loads (scalar loads only in the ragged last tile, so no
// load passes n), a wave shuffle scan + 16 wave sums give the exclusive prefix, and the
// tile total carries into the next tile.
__global__ __launch_bounds__(1024) void frontier_scan_kernel(const float* __restrict__ flags, int n_static,
                                                             const int32_t* __restrict__ n_dev, int n_mul,
                                                             int32_t* __restrict__ out) {
  constexpr int PT = 8, TILE = 1024 * PT;
  __shared__ int32_t wsum[16];
  const int n = n_dev ? n_mul * (*n_dev) : n_static;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  int carry = 0;
  for (int base = 0; base < n; base += TILE) {
    const int i0 = base + tid * PT;
    int v[PT];
    if (i0 + PT <= n) {
      const float4 f0 = *reinterpret_cast<const float4*>(flags + i0);
      const float4 f1 = *reinterpret_cast<const float4*>(flags + i0 + 4);
      v[0] = f0.x > 0.f; v[1] = f0.y > 0.f; v[2] = f0.z > 0.f; v[3] = f0.w > 0.f;
      v[4] = f1.x > 0.f; v[5] = f1.y > 0.f; v[6] = f1.z > 0.f; v[7] = f1.w > 0.f;
    } else {
#pragma unroll
      for (int j = 0; j < PT; ++j) v[j] = (i0 + j < n) ? (flags[i0 + j] > 0.f) : 0;
    }
    int s = 0;
#pragma unroll
    for (int j = 0; j < PT; ++j) s += v[j];
    int x = s;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    int run = carry + x - s, tot = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int ws = wsum[k];
      run += k < w ? ws : 0;
      tot += ws;
    }
    __syncthreads();  // wsum is rewritten by the next tile
    int r[PT];
#pragma unroll
    for (int j = 0; j < PT; ++j) {
      r[j] = run;
      run += v[j];
    }
    if (i0 + PT <= n) {
      *reinterpret_cast<int4*>(out + i0) = make_int4(r[0], r[1], r[2], r[3]);
      *reinterpret_cast<int4*>(out + i0 + 4) = make_int4(r[4], r[5], r[6], r[7]);
    } else {
#pragma unroll
      for (int j = 0; j < PT; ++j)
        if (i0 + j < n) out[i0 + j] = r[j];
    }
    carry += tot;
  }
  if (tid == 0) out[n] = carry;
}

// Per candidate a that splits (slot p = pos[a]): its commit record (tree, node, left child id,
// candidate index) and its two children's "candidate next level" flags at front[2p], [2p+1];
// per tree t: the node counter advances by 2 x its splits (into n_nodes_next).
__global__ __launch_bounds__(256) void frontier_children_kernel(int A, int Tn, const int32_t* __restrict__ ct,
                                                                const int32_t* __restrict__ cn,
                                                                const int32_t* __restrict__ tlo,
                                                                const float* __restrict__ dec,
                                                                const int32_t* __restrict__ pos,
                                                                const int32_t* __restrict__ n_nodes,
                                                                int32_t* __restrict__ n_nodes_next,
                                                                int64_t* __restrict__ ti, int64_t* __restrict__ ni,
                                                                int64_t* __restrict__ cl, int64_t* __restrict__ dsi,
                                                                float* __restrict__ front,
                                                                const int32_t* __restrict__ a_dev,
                                                                int32_t* __restrict__ scal) {
  // A: row stride of dec; An: the level's candidate count; scal[0] = splits (the next scan's n)
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int An = a_dev ? *a_dev : A;
  if (i == 0) scal[0] = pos[An];
  if (i < Tn) n_nodes_next[i] = n_nodes[i] + 2 * (pos[tlo[i + 1]] - pos[tlo[i]]);
  if (i >= An || !(dec[i] > 0.f)) return;
  const int p = pos[i], t = ct[i];
  const int c = n_nodes[t] + 2 * (p - pos[tlo[t]]);
  ti[p] = t;
  ni[p] = cn[i];
  cl[p] = c;
  dsi[p] = i;
  front[2 * p] = dec[A + i];
  front[2 * p + 1] = dec[2 * A + i];
}

// Front entry e (child e & 1 of split e >> 1) that is a candidate becomes next-level candidate
// q[e]: its (tree, node), weight and cand_idx entry; tree starts of the next level; scalars
// [splits, next candidates, max candidates per tree, max candidate weight (float bits)].
__global__ __launch_bounds__(256) void frontier_next_kernel(int A, int Tn, int maxn, const int32_t* __restrict__ tlo,
                                                            const float* __restrict__ dec,
                                                            const int32_t* __restrict__ pos,
                                                            const int64_t* __restrict__ ti,
                                                            const int64_t* __restrict__ cl,
                                                            const int64_t* __restrict__ dsi,
                                                            const float* __restrict__ front,
                                                            const int32_t* __restrict__ q,
                                                            int32_t* __restrict__ ct_next,
                                                            int32_t* __restrict__ cn_next,
                                                            int32_t* __restrict__ tlo_next,
                                                            int32_t* __restrict__ cand_idx,
                                                            int32_t* __restrict__ scal,
                                                            const int32_t* __restrict__ a_dev,
                                                            int32_t* __restrict__ parent_of,
                                                            int32_t* __restrict__ derive_from) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  const int S = pos[a_dev ? *a_dev : A];
  if (e <= Tn) {
    const int lo = q[2 * pos[tlo[e]]];
    tlo_next[e] = lo;
    if (e < Tn) atomicMax(&scal[2], q[2 * pos[tlo[e + 1]]] - lo);
  }
  if (e == 0) {
    scal[0] = S;
    scal[1] = q[2 * S];
  }
  if (e >= 2 * S || !(front[e] > 0.f)) return;
  const int p = e >> 1, i = q[e];
  const int t = (int)ti[p], n = (int)cl[p] + (e & 1);
  const float wgt = dec[(3 + (e & 1)) * A + dsi[p]];
  // sibling subtraction (parent_of given): of two candidate siblings the heavier (the right one
  // on a tie) takes its histogram as parent - sibling, and its rows are not grouped (cand_idx -1)
  bool derived = false;
  if (parent_of) {
    const float wsib = dec[(3 + ((e & 1) ^ 1)) * A + dsi[p]];
    derived = front[e ^ 1] > 0.f && (wgt > wsib || (wgt == wsib && (e & 1)));
    parent_of[i] = (int)dsi[p];
    derive_from[i] = derived ? q[e ^ 1] : -1;
  }
  ct_next[i] = t;
  cn_next[i] = n;
  cand_idx[(int64_t)t * maxn + n] = derived ? -1 : i;
  atomicMax(&scal[3], __float_as_int(wgt));  // weights >= 0: float order == int order
}

// Root frontier on the device (one workgroup): tree t's root is a candidate when its impurity is
// > 1e-12 (fp64) and its weight >= 2 minInstances — the rule of tree_level_decide_kernel.
// Candidates are compacted in tree order: ct (tree ids), cn = 0, tlo[t] = first candidate of tree t,
// cand_idx[t][0]; scal = [0, candidates, 1 (max per tree), max candidate weight (float bits)].
// Thread i owns the contiguous trees [i * per, (i + 1) * per); one block scan.
__global__ __launch_bounds__(1024) void tree_root_frontier_kernel(const float* __restrict__ stats, int Tn, int K,
                                                                  int64_t tree_stride, int impurity, float min2,
                                                                  int maxn, int32_t* __restrict__ ct,
                                                                  int32_t* __restrict__ cn, int32_t* __restrict__ tlo,
                                                                  int32_t* __restrict__ cand_idx,
                                                                  int32_t* __restrict__ scal) {
  __shared__ int wsum[16];
  __shared__ int wmax[16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int per = (Tn + 1023) >> 10;
  const int b = min(Tn, tid * per), e = min(Tn, b + per);
  auto cand = [&](int t, float& w_out) {
    const float* st = stats + (int64_t)t * tree_stride;
    float w = 0.f;
    for (int k = 0; k < K; ++k) w += st[k];
    const double dw = fmax((double)w, 1e-30);
    double q = 0.0;
    for (int k = 0; k < K; ++k) {
      const double p = (double)st[k] / dw;
      if (impurity == 0) q += p * p;
      else q -= p > 0 ? p * log2(fmax(p, 1e-30)) : 0.0;
    }
    const double imp = impurity == 0 ? 1.0 - q : q;
    w_out = w;
    return imp > 1e-12 && w >= min2;
  };
  int cnt = 0, mx = 0;
  for (int t = b; t < e; ++t) {
    float w;
    if (cand(t, w)) { ++cnt; mx = max(mx, __float_as_int(w)); }  // weights >= 0: int order = float order
  }
  int x = cnt, m = mx;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
    m = max(m, __shfl_xor(m, o, 64));
  }
  if (lane == 63) wsum[wave] = x;
  if (lane == 0) wmax[wave] = m;
  __syncthreads();
  int run = x - cnt, tot = 0, gmax = 0;
#pragma unroll
  for (int w = 0; w < 16; ++w) {
    run += w < wave ? wsum[w] : 0;
    tot += wsum[w];
    gmax = max(gmax, wmax[w]);
  }
  for (int t = b; t < e; ++t) {
    float w;
    const bool c = cand(t, w);
    tlo[t] = run;
    if (c) {
      ct[run] = t;
      cn[run] = 0;
      cand_idx[(int64_t)t * maxn] = run;
      ++run;
    }
  }
  if (tid == 0) {
    tlo[Tn] = tot;
    scal[0] = 0;
    scal[1] = tot;
    scal[2] = 1;
    scal[3] = gmax;
  }
}

int grid_for(int64_t total) { return (int)std::max<int64_t>(1, std::min<int64_t>(8192, (total + 255) / 256)); }

}  // namespace

extern "C" int har_tree_feature_subsets(uint64_t seed, const int32_t* trees, const int32_t* nodes, int64_t P, int F,
                                        int m, int32_t* out, const int32_t* p_dev, hipStream_t s) {
  if (m <= 0 || m > MAX_SUBSET || m > F) return -2;
  if (P == 0) return 0;
  tree_feature_subsets_kernel<<<(unsigned)((P + 3) / 4), 256, 0, s>>>(seed, trees, nodes, P, F, m, out, p_dev);
  HAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int har_tree_level_keys(const int32_t* node_of, const int32_t* cand_idx, int T, int64_t N, int maxn,
                                   int32_t* key, hipStream_t s) {
  if ((int64_t)T * N == 0) return 0;
  tree_level_keys_kernel<<<grid_for((int64_t)T * N), 256, 0, s>>>(node_of, cand_idx, T, N, maxn, key);
  HAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int har_tree_partition(int32_t* node_of, const int32_t* lvl_feat, const int32_t* lvl_bin,
                                  const int32_t* lvl_left, const uint8_t* bins, int T, int64_t N, int maxn,
                                  hipStream_t s) {
  if ((int64_t)T * N == 0) return 0;
  tree_partition_kernel<<<grid_for((int64_t)T * N), 256, 0, s>>>(node_of, lvl_feat, lvl_bin, lvl_left, bins, T, N,
                                                                 maxn);
  HAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int har_tree_level_group(const int32_t* node_of, const int32_t* cand_idx, const int32_t* tree_lo,
                                    const float* W, int T, int64_t N, int maxn, int A, int nt_max, int32_t* cnt_ws,
                                    int32_t* counts, int32_t* starts, int32_t* rows, float* row_w,
                                    const int32_t* a_dev, hipStream_t s) {
  if (nt_max > GROUP_MAX_NT || nt_max < 1) return -4;
  if (A == 0 || T == 0 || N == 0) return 0;
  const int nch = (int)((N + GROUP_CH - 1) / GROUP_CH);
  const dim3 grid((nch + GROUP_WAVES - 1) / GROUP_WAVES, T);
  const size_t lds = (size_t)GROUP_WAVES * nt_max * sizeof(int32_t);
  tree_group_count_kernel<<<grid, 64 * GROUP_WAVES, lds, s>>>(node_of, cand_idx, tree_lo, N, maxn, nch, A, nt_max,
                                                              cnt_ws);
  HAR_CHECK_LAUNCH();
  tree_group_colscan_kernel<<<(A + 255) / 256, 256, 0, s>>>(cnt_ws, nch, A, counts, a_dev);
  HAR_CHECK_LAUNCH();
  tree_group_scan_kernel<<<1, 1024, 0, s>>>(counts, A, starts, a_dev);
  HAR_CHECK_LAUNCH();
  tree_group_scatter_kernel<<<grid, 64 * GROUP_WAVES, lds, s>>>(node_of, cand_idx, tree_lo, W, N, maxn, nch, A,
                                                                nt_max, cnt_ws, starts, rows, row_w);
  HAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int har_tree_level_group_chunks(int64_t N) { return (int)((N + GROUP_CH - 1) / GROUP_CH); }

extern "C" int har_tree_commit_level(int S, const int64_t* ti, const int64_t* ni, const int64_t* cl, const int64_t* dsi,
                                     const int32_t* rfeat, const int32_t* rbin, const float* rgain, const float* rleft,
                                     const float* rtotal, int K, const float* thr_mat, int ldthr, int maxn,
                                     int32_t* feature, int32_t* split_bin, float* thresh, int32_t* left,
                                     int32_t* right, float* gains, float* stats, const int32_t* s_dev,
                                     hipStream_t s) {
  if (S <= 0) return 0;
  tree_commit_level_kernel<<<(S + 255) / 256, 256, 0, s>>>(S, ti, ni, cl, dsi, rfeat, rbin, rgain, rleft, rtotal, K,
                                                           thr_mat, ldthr, maxn, feature, split_bin, thresh, left,
                                                           right, gains, stats, s_dev);
  HAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int har_tree_partition_split(int32_t* node_of, const int32_t* feature, const int32_t* split_bin,
                                        const int32_t* left, const uint8_t* bins, int T, int64_t N, int maxn,
                                        hipStream_t s) {
  if ((int64_t)T * N == 0) return 0;
  tree_partition_split_kernel<<<grid_for((int64_t)T * N), 256, 0, s>>>(node_of, feature, split_bin, left, bins, T, N,
                                                                       maxn);
  HAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int har_tree_level_decide(int A, const float* gain, const float* left, const float* total, int K,
                                     int impurity, float min2, float* out, const int32_t* a_dev, hipStream_t s) {
  if (A <= 0) return 0;
  tree_level_decide_kernel<<<(A + 255) / 256, 256, 0, s>>>(A, gain, left, total, K, impurity, min2, out, a_dev);
  HAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int har_tree_frontier(int A, int Tn, int maxn, const int32_t* ct, const int32_t* cn, const int32_t* tlo,
                                 const float* dec, const int32_t* n_nodes, int32_t* n_nodes_next, int32_t* pos_ws,
                                 int64_t* ti, int64_t* ni, int64_t* cl, int64_t* dsi, float* front, int32_t* q_ws,
                                 int32_t* ct_next, int32_t* cn_next, int32_t* tlo_next, int32_t* cand_idx,
                                 int32_t* scal, const int32_t* a_dev, int32_t* parent_of, int32_t* derive_from,
                                 hipStream_t s) {
  if (A <= 0) return -2;
  // frontier_scan_kernel reads / writes 16-byte vectors from these bases
  if (((uintptr_t)dec | (uintptr_t)front | (uintptr_t)pos_ws | (uintptr_t)q_ws) & 15) return -3;
  hipError_t err = hipMemsetAsync(scal, 0, 4 * sizeof(int32_t), s);
  if (err != hipSuccess) return (int)err;
  frontier_scan_kernel<<<1, 1024, 0, s>>>(dec, A, a_dev, 1, pos_ws);
  HAR_CHECK_LAUNCH();
  const int g1 = (std::max(A, Tn + 1) + 255) / 256;
  frontier_children_kernel<<<g1, 256, 0, s>>>(A, Tn, ct, cn, tlo, dec, pos_ws, n_nodes, n_nodes_next, ti, ni, cl, dsi,
                                              front, a_dev, scal);
  HAR_CHECK_LAUNCH();
  frontier_scan_kernel<<<1, 1024, 0, s>>>(front, 0, scal, 2, q_ws);  // n = 2 x splits (scal[0])
  HAR_CHECK_LAUNCH();
  const int g2 = (std::max(2 * A, Tn + 1) + 255) / 256;
  frontier_next_kernel<<<g2, 256, 0, s>>>(A, Tn, maxn, tlo, dec, pos_ws, ti, cl, dsi, front, q_ws, ct_next, cn_next,
                                          tlo_next, cand_idx, scal, a_dev, parent_of, derive_from);
  HAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int har_tree_root_frontier(const float* stats, int Tn, int K, int64_t tree_stride, int impurity, float min2,
                                      int maxn, int32_t* ct, int32_t* cn, int32_t* tlo, int32_t* cand_idx,
                                      int32_t* scal, hipStream_t s) {
  if (Tn <= 0 || K <= 0) return -2;
  tree_root_frontier_kernel<<<1, 1024, 0, s>>>(stats, Tn, K, tree_stride, impurity, min2, maxn, ct, cn, tlo, cand_idx,
                                               scal);
  HAR_CHECK_LAUNCH();
  return 0;
}
