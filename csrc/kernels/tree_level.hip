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
//   tree_partition       : after the level's splits, move every row of a split node to
//                          its child (bin <= threshold bin -> left) and retire the rows
//                          of nodes that became leaves — one pass over [T][N] int32.
#include "common.h"
#include "philox.h"
#include "../har_kernels.h"

namespace {

constexpr uint32_t STREAM_FEATURE_SUBSET = 0x7F000000u;
constexpr int MAX_SUBSET = 128;

__global__ __launch_bounds__(256) void tree_feature_subsets_kernel(uint64_t seed, const int32_t* __restrict__ trees,
                                                                   const int32_t* __restrict__ nodes, int64_t P,
                                                                   int F, int m, int32_t* __restrict__ out) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P) return;
  const uint64_t base = ((uint64_t)(uint32_t)trees[p] << 32) | ((uint64_t)(uint32_t)nodes[p] << 8);
  int chosen[MAX_SUBSET];
  for (int i = 0; i < m; ++i) {
    const int j = F - m + i;
    const uint32_t d = philox_u32(seed, STREAM_FEATURE_SUBSET, base + (uint64_t)i);
    const int t = (int)(d % (uint32_t)(j + 1));
    bool dup = false;
    for (int q = 0; q < i; ++q) dup |= chosen[q] == t;
    chosen[i] = dup ? j : t;
  }
  for (int i = 1; i < m; ++i) {  // insertion sort (m <= 128, mostly ~sqrt(F))
    const int v = chosen[i];
    int q = i - 1;
    while (q >= 0 && chosen[q] > v) { chosen[q + 1] = chosen[q]; --q; }
    chosen[q + 1] = v;
  }
  int32_t* o = out + p * m;
  for (int i = 0; i < m; ++i) o[i] = chosen[i];
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

int grid_for(int64_t total) { return (int)std::max<int64_t>(1, std::min<int64_t>(8192, (total + 255) / 256)); }

}  // namespace

extern "C" int har_tree_feature_subsets(uint64_t seed, const int32_t* trees, const int32_t* nodes, int64_t P, int F,
                                        int m, int32_t* out, hipStream_t s) {
  if (m <= 0 || m > MAX_SUBSET || m > F) return -2;
  if (P == 0) return 0;
  tree_feature_subsets_kernel<<<(unsigned)((P + 255) / 256), 256, 0, s>>>(seed, trees, nodes, P, F, m, out);
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
