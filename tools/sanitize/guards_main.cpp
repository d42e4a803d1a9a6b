// Host AddressSanitizer + UBSan driver for the launch contracts of the HIP kernels
// (csrc/har_kernels.h).  Every launcher validates shapes, alignment and pointers on the
// host before it enqueues anything: a kernel started with operands its grid does not expect
// faults the GPU, so these guards are what keeps a bad call an error code.  This driver calls
// the launchers with contract-violating arguments and checks that each one returns its
// documented negative code without touching the device (no GPU is needed: a guard that let a
// call through would reach the HIP runtime and fail the run), and sweeps the host-side
// sizing helpers over edge sizes so UBSan sees any integer overflow in them.
// Built by tools/sanitize/guards.sh: every kernel source compiled with -Xarch_host
// -fsanitize=address,undefined (device code is built normally; GPU ASan is not available).
#include <climits>
#include <cstdint>
#include <cstdio>
#include <vector>

#include "../../csrc/har_kernels.h"

static int g_fail = 0, g_checks = 0;

#define EXPECT(call, code)                                                                  \
  do {                                                                                      \
    ++g_checks;                                                                             \
    const int rc__ = (call);                                                                \
    if (rc__ != (code)) {                                                                   \
      std::fprintf(stderr, "FAIL %s:%d  %s -> %d, expected %d\n", __FILE__, __LINE__, #call, \
                   rc__, (code));                                                           \
      ++g_fail;                                                                             \
    }                                                                                       \
  } while (0)

#define EXPECT_TRUE(cond)                                                          \
  do {                                                                             \
    ++g_checks;                                                                    \
    if (!(cond)) {                                                                 \
      std::fprintf(stderr, "FAIL %s:%d  %s\n", __FILE__, __LINE__, #cond);         \
      ++g_fail;                                                                    \
    }                                                                              \
  } while (0)

// Host buffers stand in for device pointers: rejected calls never dereference them, and
// they give the alignment checks real 16-byte-aligned (and deliberately misaligned) addresses.
alignas(64) static float fbuf[1024];
alignas(64) static uint16_t hbuf[1024];
alignas(64) static int32_t ibuf[1024];

static void mlp_contracts() {
  const float* src[9] = {fbuf, fbuf, fbuf, fbuf, fbuf, fbuf, fbuf, fbuf, fbuf};
  int64_t start[9] = {0, 4, 8, 12, 16, 20, 24, 28, 32}, len[9] = {4, 4, 4, 4, 4, 4, 4, 4, 4};
  int64_t lds[9] = {36, 36, 36, 36, 36, 36, 36, 36, 36};
  int S[9] = {2, 2, 2, 2, 2, 2, 2, 2, 2};
  // n % 4, too many regions, REDUCE without regions, S <= 0, region past n, unsorted, misaligned
  EXPECT(har_grad_reduce_adam(1, src, start, len, lds, S, 6, fbuf, fbuf, fbuf, fbuf, hbuf, 0, 0, 0, 0, 0, ibuf, 0, 1, nullptr, 0), -2);
  EXPECT(har_grad_reduce_adam(9, src, start, len, lds, S, 36, fbuf, fbuf, fbuf, fbuf, hbuf, 0, 0, 0, 0, 0, ibuf, 0, 1, nullptr, 0), -2);
  EXPECT(har_grad_reduce_adam(0, src, start, len, lds, S, 36, fbuf, fbuf, fbuf, fbuf, hbuf, 0, 0, 0, 0, 0, ibuf, 0, 1, nullptr, 0), -2);
  int S0[1] = {0};
  EXPECT(har_grad_reduce_adam(1, src, start, len, lds, S0, 36, fbuf, fbuf, fbuf, fbuf, hbuf, 0, 0, 0, 0, 0, ibuf, 0, 1, nullptr, 0), -2);
  int64_t far[1] = {36};
  EXPECT(har_grad_reduce_adam(1, src, far, len, lds, S, 36, fbuf, fbuf, fbuf, fbuf, hbuf, 0, 0, 0, 0, 0, ibuf, 0, 1, nullptr, 0), -2);
  int64_t unsorted[2] = {8, 0};
  EXPECT(har_grad_reduce_adam(2, src, unsorted, len, lds, S, 36, fbuf, fbuf, fbuf, fbuf, hbuf, 0, 0, 0, 0, 0, ibuf, 0, 1, nullptr, 0), -2);
  const float* mis[1] = {fbuf + 1};
  EXPECT(har_grad_reduce_adam(1, mis, start, len, lds, S, 36, fbuf, fbuf, fbuf, fbuf, hbuf, 0, 0, 0, 0, 0, ibuf, 0, 1, nullptr, 0), -3);

  EXPECT(har_adam_step(fbuf, fbuf, nullptr, 0, fbuf, fbuf, hbuf, 6, 0, 0, 0, 0, 0, 1, ibuf, 0, 0), -2);
  EXPECT(har_reduce_slabs(fbuf, 2, 6, fbuf, 0), -2);
  EXPECT(har_softmax_ce_head(hbuf, hbuf, fbuf, ibuf, 64, 256, 33, 1.f, hbuf, fbuf, ibuf, nullptr, 0), -2);
  EXPECT(har_softmax_ce_head(hbuf, hbuf, fbuf, ibuf, 64, 250, 6, 1.f, hbuf, fbuf, ibuf, nullptr, 0), -2);

  // fused forward: B % 16, B <= 0, C outside [1, 16], misaligned operands
  EXPECT(har_mlp_fwd_head(hbuf, 64, hbuf, fbuf, hbuf, fbuf, 256, hbuf, fbuf, ibuf, 40, 6, 1.f, hbuf, hbuf, fbuf, fbuf, ibuf, 0), -2);
  EXPECT(har_mlp_fwd_head(hbuf, 64, hbuf, fbuf, hbuf, fbuf, 256, hbuf, fbuf, ibuf, 0, 6, 1.f, hbuf, hbuf, fbuf, fbuf, ibuf, 0), -2);
  EXPECT(har_mlp_fwd_head(hbuf, 64, hbuf, fbuf, hbuf, fbuf, 256, hbuf, fbuf, ibuf, 64, 17, 1.f, hbuf, hbuf, fbuf, fbuf, ibuf, 0), -2);
  EXPECT(har_mlp_fwd_head(hbuf, 64, hbuf, fbuf, hbuf, fbuf, 256, hbuf, fbuf, ibuf, 64, 0, 1.f, hbuf, hbuf, fbuf, fbuf, ibuf, 0), -2);
  EXPECT(har_mlp_fwd_head(hbuf + 1, 64, hbuf, fbuf, hbuf, fbuf, 256, hbuf, fbuf, ibuf, 64, 6, 1.f, hbuf, hbuf, fbuf, fbuf, ibuf, 0), -3);
  EXPECT(har_mlp_fwd_infer(hbuf, 64, hbuf, fbuf, hbuf + 1, fbuf, 256, hbuf, fbuf, 64, 6, fbuf, ibuf, 0), -3);
  EXPECT(har_mlp_fwd_infer(hbuf, 64, hbuf, fbuf, hbuf, fbuf, 256, hbuf, fbuf, 48 + 1, 6, fbuf, ibuf, 0), -2);
  // serving from fp32 features: F > K0, ldx < F
  EXPECT(har_mlp_fwd_infer_f32(fbuf, 43, 65, 64, hbuf, fbuf, hbuf, fbuf, 256, hbuf, fbuf, 64, 6, fbuf, ibuf, 0), -2);
  EXPECT(har_mlp_fwd_infer_f32(fbuf, 40, 43, 64, hbuf, fbuf, hbuf, fbuf, 256, hbuf, fbuf, 64, 6, fbuf, ibuf, 0), -2);
  // unsupported hidden width -> no kernel instance
  EXPECT(har_mlp_fwd_infer(hbuf, 64, hbuf, fbuf, hbuf, fbuf, 192, hbuf, fbuf, 64, 6, fbuf, ibuf, 0), -4);

  // three-kernel step: H != 256, K0 not 32 / 64, B % 64, C outside [1, 16], short slab stride, misaligned
  float* g = fbuf;
  EXPECT(har_mlp_step_fwd(hbuf, 64, hbuf, fbuf, fbuf, 128, hbuf, fbuf, ibuf, 64, 6, 1.f, hbuf, g, g, ibuf, 0), -2);
  EXPECT(har_mlp_step_fwd(hbuf, 48, hbuf, fbuf, fbuf, 256, hbuf, fbuf, ibuf, 64, 6, 1.f, hbuf, g, g, ibuf, 0), -2);
  EXPECT(har_mlp_step_fwd(hbuf, 64, hbuf, fbuf, fbuf, 256, hbuf, fbuf, ibuf, 96, 6, 1.f, hbuf, g, g, ibuf, 0), -2);
  EXPECT(har_mlp_step_fwd(hbuf, 64, hbuf, fbuf, fbuf, 256, hbuf, fbuf, ibuf, 64, 17, 1.f, hbuf, g, g, ibuf, 0), -2);
  EXPECT(har_mlp_step_fwd(hbuf + 4, 64, hbuf, fbuf, fbuf, 256, hbuf, fbuf, ibuf, 64, 6, 1.f, hbuf, g, g, ibuf, 0), -3);
  EXPECT(har_mlp_step_bwd(hbuf, hbuf, 64, hbuf, 128, fbuf, 64, g, g, g, g, 1 << 20, ibuf, nullptr, 0, g, g, 0), -2);
  EXPECT(har_mlp_step_bwd(hbuf, hbuf, 64, hbuf, 256, fbuf, 96, g, g, g, g, 1 << 20, ibuf, nullptr, 0, g, g, 0), -2);
  EXPECT(har_mlp_step_bwd(hbuf, hbuf, 48, hbuf, 256, fbuf, 64, g, g, g, g, 1 << 20, ibuf, nullptr, 0, g, g, 0), -2);
  EXPECT(har_mlp_step_bwd(hbuf, hbuf, 64, hbuf, 256, fbuf, 64, g, g, g, g, 256 * 255, ibuf, nullptr, 0, g, g, 0), -2);
  EXPECT(har_mlp_step_bwd(hbuf + 1, hbuf, 64, hbuf, 256, fbuf, 64, g, g, g, g, 1 << 20, ibuf, nullptr, 0, g, g, 0), -3);
  EXPECT(har_mlp_step_bwd(hbuf, hbuf, 64, hbuf, 256, fbuf, 64, g, g, g, g, 1 << 20, ibuf, g, 100, g, g, 0), -2);
}

static void window_contracts() {
  // axes not a multiple of 3, too few samples per window, bad stride, wrong bin count,
  // windows past the stream end, short output rows, negative window counts
  EXPECT(har_window_features(fbuf, 1000, 4, 200, 100, 5, 20.f, 10, fbuf, 64, 0), -2);
  EXPECT(har_window_features(fbuf, 1000, 3, 2, 100, 5, 20.f, 10, fbuf, 64, 0), -2);
  EXPECT(har_window_features(fbuf, 1000, 3, 200, 0, 5, 20.f, 10, fbuf, 64, 0), -2);
  EXPECT(har_window_features(fbuf, 1000, 3, 200, 100, 5, 20.f, 12, fbuf, 64, 0), -2);
  EXPECT(har_window_features(fbuf, 1000, 3, 200, 100, 10, 20.f, 10, fbuf, 64, 0), -3);
  EXPECT(har_window_features(fbuf, 1000, 3, 200, 100, 5, 20.f, 10, fbuf, 54, 0), -4);
  EXPECT(har_window_features(fbuf, 1000, 3, 200, 100, -1, 20.f, 10, fbuf, 64, 0), -2);
  EXPECT(har_window_features(fbuf, 1000, 3, 200, 100, 0, 20.f, 10, fbuf, 64, 0), 0);  // nothing to do
  EXPECT(har_window_features_mlp(fbuf, 1000, 3, 200, 100, 5, 20.f, nullptr, fbuf, 0.f, hbuf, 64, 0), -4);
  EXPECT(har_window_features_mlp(fbuf, 1000, 3, 200, 100, 10, 20.f, fbuf, fbuf, 0.f, hbuf, 64, 0), -3);
  EXPECT(har_window_features_mlp(fbuf, 1000, 3, 200, 100, -3, 20.f, fbuf, fbuf, 0.f, hbuf, 64, 0), -2);
  // a window longer than the int32 sample counter range of the kernel
  EXPECT(har_window_features(fbuf, int64_t(1) << 40, 3, 70000, 100, 5, 20.f, 10, fbuf, 64, 0), -2);
}

static void tree_contracts() {
  // findSplits: sample too large for the LDS sort, too many cut points
  EXPECT(har_find_splits_post_sort(fbuf, 4, 16385, 31, fbuf, 0), -2);
  EXPECT(har_find_splits_post_sort(fbuf, 4, 100, 64, fbuf, 0), -2);
  EXPECT(har_find_splits_post_sort(fbuf, 4, 0, 31, fbuf, 0), -2);
  EXPECT(har_sort_columns(fbuf, 16385, 4, 4, fbuf, 0), -2);
  EXPECT(har_sort_columns(fbuf, 100, 4, 3, fbuf, 0), -2);
  EXPECT(har_sort_columns(fbuf, 100, 0, 0, fbuf, 0), 0);  // no columns: nothing enqueued
  // bootstrap init: too many classes, CDF table too long
  uint32_t cdf[17] = {};
  EXPECT(har_tree_init(1, 0, 2, 0, 10, cdf, 17, nullptr, ibuf, 6, fbuf, ibuf, fbuf, 8, ibuf, 0), -2);
  EXPECT(har_tree_init(1, 0, 2, 0, 10, cdf, 4, nullptr, ibuf, 0, fbuf, ibuf, fbuf, 8, ibuf, 0), -2);
  EXPECT(har_tree_init(1, 0, 2, 0, 10, cdf, 4, nullptr, ibuf, 1 << 20, fbuf, ibuf, fbuf, 8, ibuf, 0), -2);
}

static void data_contracts() {
  // negative sizes / class counts / ld < columns are rejected before any launch
  int64_t cm[64];
  double d6[6], st[5];
  uint8_t bins[16];
  int64_t codes[4];
  EXPECT(har_confusion_matrix(ibuf, ibuf, 10, -3, cm, 0), -2);
  EXPECT(har_confusion_matrix(ibuf, ibuf, 10, 1 << 20, cm, 0), -2);
  EXPECT(har_confusion_matrix(ibuf, ibuf, -5, 6, cm, 0), -2);
  EXPECT(har_regression_moments(fbuf, fbuf, -1, d6, 0), -2);
  EXPECT(har_value_counts(codes, 4, 0, cm, 0), -2);
  EXPECT(har_value_counts(codes, 4, 40000, cm, 0), -2);
  EXPECT(har_value_counts(codes, -4, 8, cm, 0), -2);
  EXPECT(har_philox_buckets(1, 0, 0, -7, nullptr, 0, ibuf, 0), -2);
  EXPECT(har_column_stats(fbuf, -2, 4, 4, nullptr, st, d6, 0), -2);
  EXPECT(har_column_stats(fbuf, 10, 4, 3, nullptr, st, d6, 0), -2);
  EXPECT(har_column_stats_f64(nullptr, 10, -1, nullptr, st, d6, 0), -2);
  EXPECT(har_bin_features(fbuf, 10, 70000, 70000, fbuf, 32, ibuf, bins, 0), -2);
  EXPECT(har_bin_features(fbuf, 10, 8, 4, fbuf, 32, ibuf, bins, 0), -2);
  EXPECT(har_bin_features(fbuf, -10, 8, 8, fbuf, 32, ibuf, bins, 0), -2);
  EXPECT(har_poisson_bootstrap(1, 0, -2, 0, 100, bins, 0), -2);
  EXPECT(har_roc_pr_sums(fbuf, fbuf, -1, d6, 0), -2);
  EXPECT(har_roc_pr_sums(fbuf, fbuf, int64_t(1) << 30, d6, 0), -2);
  EXPECT(har_csv_count_newlines(bins, -1, ibuf, 0), -2);
  EXPECT(har_csv_count_newlines(bins, 0, ibuf, 0), 0);  // empty buffer: nothing enqueued
}

static void sizing_helpers() {
  const int Bs[] = {1, 15, 16, 31, 32, 63, 64, 65, 256, 4096, 65536, 1 << 20, INT_MAX / 2, INT_MAX};
  for (int B : Bs) {
    const int grid = har_mlp_fwd_head_grid(B), sl = har_mlp_step_slices(B);
    EXPECT_TRUE(har_mlp_step_grid(B) >= 1 && har_mlp_step_grid(B) <= 256);
    EXPECT_TRUE(grid >= 1 && grid <= 256);
    EXPECT_TRUE(sl >= 1 && sl <= 64);
    EXPECT_TRUE(har_softmax_ce_head_blocks(B) >= 1);
    EXPECT_TRUE(har_head_fused_blocks(B) >= 1);
  }
  const int64_t ns[] = {0, 1, 1000, 1 << 20, int64_t(1) << 31};
  for (int64_t n : ns) {
    EXPECT_TRUE(har_column_stats_workspace(n, 3100) >= 0);
    EXPECT_TRUE(har_logreg_eval_tiles(n) >= 0);
    EXPECT_TRUE(har_qn_chunks(n, 1) >= 1 && har_qn_chunks(n, 45) >= 1 && har_qn_chunks(n, 0) >= 1);
    EXPECT_TRUE(har_tree_level_group_chunks(n) >= 0);
  }
}

int main() {
  mlp_contracts();
  window_contracts();
  tree_contracts();
  data_contracts();
  sizing_helpers();
  if (g_fail) {
    std::fprintf(stderr, "guard sanitizer run: %d of %d checks FAILED\n", g_fail, g_checks);
    return 1;
  }
  std::printf("guard sanitizer run: OK (%d checks)\n", g_checks);
  return 0;
}
