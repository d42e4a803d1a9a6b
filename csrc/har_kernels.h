// C ABI of the har HIP kernels (gfx950).  Every launcher takes raw device
// pointers plus the HIP stream to enqueue on, never allocates or synchronizes
// (so every launch can be captured into a hipGraph), and returns 0 or a
// hipError_t / negative contract-violation code.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct GemmParams {
  const void* A;
  const void* B;
  void* C;
  const float* bias;      // EPI_BIAS*, may be null
  const void* mask;       // EPI_RELU_GRAD: bf16 activations of the forward pass
  float* rowsum;          // optional fused sum_k A(m,k) (bias gradient of a weight-grad product)
  int M, N, K;
  int lda, ldb, ldc, ldmask;
  int k_split;            // EPI_F32_ATOMIC / EPI_F32_SLAB: K range per grid.z slice (multiple of 32)
  int tile;               // -1 = automatic tile choice, else tile id (gemm.hip)
  int64_t slab_stride;    // EPI_F32_SLAB: elements between the C slabs of consecutive splits
  int64_t slab_stride_rowsum;  // elements between rowsum slabs
  float alpha;
} GemmParams;

int har_gemm_bf16(const GemmParams* p, int layout, int epi, hipStream_t s);
int har_gemm_f32(const GemmParams* p, int layout, int epi, hipStream_t s);

// Fused classifier head: logits = H . W^T + b (C <= 32 classes, W padded to 32 rows),
// softmax, cross-entropy, dlogits = (p - onehot) * scale (bf16, 32 columns).
// Per-workgroup partial CE sums / correct counts go to block_loss[blockIdx] /
// block_correct[blockIdx] (no same-address atomics; the host sums them lazily).
// Returns the number of workgroups through *nblocks_out if non-null.
int har_softmax_ce_head(const uint16_t* H, const uint16_t* W, const float* bias, const int32_t* labels,
                        int B, int Hdim, int C, float scale, uint16_t* dlogits, float* block_loss,
                        int32_t* block_correct, float* logits_out, hipStream_t s);
int har_softmax_ce_head_blocks(int B);

// Fused Adam(W) over a flat fp32 parameter buffer; also writes the bf16 compute copy.
// Gradient = grad[i] (if slabs == null) or sum_s slabs[s*n + i] (fused split-K reduction).
// The step counter (*step, device int32) is incremented on the stream before the update
// (by this call when tick != 0, else by an earlier kernel such as har_reduce_slabs_grouped).
// Flat-gradient reduction (+ Adam) of the MLP step (mlp.hip): mode bits 1 = reduce the regions' slabs,
// 2 = store G, 4 = Adam with t = *step (tick != 0: *step += 1 first, in its own launch).  Regions:
// sorted, disjoint, 4-aligned [start, start + len), S slabs at src + s * lds.
// MFMA-fragment-ordered bf16 copies of the step's W0 / W1 (mlp.hip frag_pos): dst = [W0 frag (H*K0) |
// W1 frag (H*H) | W1^T frag (H*H)], refreshed by every Adam update that is given the spec.
typedef struct MlpFragSpec {
  uint16_t* dst;
  int64_t w0_off, w1_off;  // flat offsets of W0 [H][K0] and W1 [H][H]
  int K0, H;
  int w1t;                 // the Adam update also writes the W1^T copy (paths with no step forward)
} MlpFragSpec;
// Small-batch step (mlp_small.hip): the whole forward + backward of a 32-row tile per workgroup (B / 32
// of them, B <= har_mlp_small_step_max_batch()), each writing its partial gradient to slab blockIdx.x in
// the flat parameter layout (segment offsets off_*), loss / #correct per workgroup; `tick` (optional)
// advances Adam's step counter.  Wf: the MlpFragSpec fragment copies (W0 | W1 | W1^T, all read).
typedef struct MlpSmallStepArgs {
  const uint16_t* X;        // [B][K0] bf16 (padded inputs)
  const uint16_t* Wf;       // fragment copies
  const float* b0;
  const float* b1;
  const uint16_t* Wo;       // [16][H] bf16
  const float* bo;          // [16]
  const int32_t* labels;    // [B]
  int B, C;
  float scale;              // 1 / global batch
  float* slab;              // [B / 32][total]
  int64_t total, off_w0, off_b0, off_w1, off_b1, off_wo, off_bo;
  float* block_loss;        // [B / 32]
  int32_t* block_correct;   // [B / 32]
  int32_t* tick;
} MlpSmallStepArgs;
int har_mlp_small_step(const MlpSmallStepArgs* args, int K0, int H, hipStream_t s);
int har_mlp_small_step_max_batch();
int har_grad_reduce_adam(int nreg, const float* const* src, const int64_t* start, const int64_t* len,
                         const int64_t* lds, const int* S, int64_t n, float* G, float* param, float* m, float* v,
                         uint16_t* pb, float lr, float b1, float b2, float eps, float wd, int32_t* step, int tick,
                         int mode, const MlpFragSpec* frag, hipStream_t s, const void* pf = nullptr,
                         int64_t pf_bytes = 0, uint32_t* pf_sink = nullptr, const void* pf1 = nullptr,
                         int64_t pf1_bytes = 0);
int har_mlp_pack_frag(const uint16_t* pb, const MlpFragSpec* f, hipStream_t s);
int har_adam_step(float* param, const float* grad, const float* slabs, int nslabs, float* m, float* v,
                  uint16_t* param_bf16, int64_t n, float lr, float beta1, float beta2, float eps,
                  float weight_decay, float grad_scale, int32_t* step, int tick, hipStream_t s);

// Fused head + last hidden layer's data gradient: logits/softmax/CE/dlogits as above plus
// dH = (dlogits . Wout) * (H > 0) written as bf16 [B][D].  Per-workgroup partials (64 rows each).
int har_head_fused(const uint16_t* H, const uint16_t* W, const float* bias, const int32_t* labels, int B, int D,
                   int C, float scale, uint16_t* dlogits, uint16_t* dH, float* block_loss, int32_t* block_correct,
                   hipStream_t s);
int har_head_fused_blocks(int B);

// Fused 2-hidden-layer MLP forward + head + head weight gradient (mlp_fused.hip):
// X [B][K0] bf16 (K0 = 32/64), W0 [H][K0], W1 [H][H], Wo [>=16][H] bf16 (H = 128/256),
// fp32 biases, C <= 16 classes, B % 16 == 0.  Writes h1 and dact2 = (dz . Wo) * (h2 > 0)
// ([B][H] bf16), per-workgroup slabs [grid][16*H + 16] (dWout rows 0..15, dbout 0..15)
// and per-workgroup loss / #correct.  Grid size: har_mlp_fwd_head_grid(B).
int har_mlp_fwd_head(const uint16_t* X, int K0, const uint16_t* W0, const float* b0, const uint16_t* W1,
                     const float* b1, int H, const uint16_t* Wo, const float* bo, const int32_t* labels, int B,
                     int C, float scale, uint16_t* h1, uint16_t* dact, float* slab, float* block_loss,
                     int32_t* block_correct, hipStream_t s);
int har_mlp_fwd_head_grid(int B);
// Fused training step of the H = 256 MLP (mlp_step.hip; K0 = 32/64, C <= 16, B % 64 == 0):
// har_mlp_step_fwd writes dact2 [B][256] bf16 (the layer-2 gradient (dz . Wout) * relu'(h2), 16-byte
// chunks of rows with bit 2 set swapped in pairs), per workgroup slabs
// [har_mlp_step_grid(B)][har_mlp_step_fwd_slab_width(H)] (dWout rows 0..15, dbout) and per-workgroup
// loss / #correct; har_mlp_step_bwd reads dact2 and X and writes per row slice
// s < har_mlp_step_slices(B) the partials of dW1, dW0, db0, db1 at gw1 / gw0 / gb0 / gb1 + s * slab_stride
// (h1 recomputed from X).
// Wf: the MlpFragSpec::dst fragment copies of W0 / W1 (the step's weight operands); the forward
// (re)writes the W1^T part from its W1 registers, the backward of the same step reads it.
int har_mlp_step_fwd(const uint16_t* X, int K0, uint16_t* Wf, const float* b0, const float* b1, int H,
                     const uint16_t* Wo, const float* bo, const int32_t* labels, int B, int C, float scale,
                     uint16_t* dact2, float* slab, float* block_loss, int32_t* block_correct, hipStream_t s);
// serving forward on the same pipeline: logits [B][C] fp32 + argmax [B] (B % 64 == 0, H == 256)
int har_mlp_step_fwd_infer(const uint16_t* X, int K0, const uint16_t* Wf, const float* b0, const float* b1, int H,
                           const uint16_t* Wo, const float* bo, int B, int C, float* logits, int32_t* pred,
                           hipStream_t s);
int har_mlp_step_bwd(const uint16_t* dact2, const uint16_t* X, int K0, const uint16_t* Wf, int H, const float* b0,
                     int B, float* gw1, float* gw0, float* gb0, float* gb1, int64_t slab_stride, int32_t* tick,
                     const float* fslab, int fslab_w, float* gwo, float* gbo, hipStream_t s);
int har_mlp_step_grid(int B);
int har_mlp_step_slices(int B);
int har_mlp_step_fwd_slab_width(int H);
// diagnostic phase stamps of the step kernels (nullptr = off); see mlp_step.hip
void har_mlp_set_stamps(uint64_t* p);
// Serving variant of the same kernel: logits [B][C] fp32 + argmax class [B] int32, nothing else.
int har_mlp_fwd_infer_f32(const float* X, int ldx, int F, int K0, const uint16_t* W0, const float* b0,
                          const uint16_t* W1, const float* b1, int H, const uint16_t* Wo, const float* bo, int B, int C,
                          float* logits, int32_t* pred, hipStream_t s);
int har_mlp_fwd_infer(const uint16_t* X, int K0, const uint16_t* W0, const float* b0, const uint16_t* W1,
                      const float* b1, int H, const uint16_t* Wo, const float* bo, int B, int C, float* logits,
                      int32_t* pred, hipStream_t s);

// dst[g*n + i] = sum of slabs[s*n + i] over the g-th group of ceil(S/G) slabs (deterministic).
// A non-null tick is incremented once by the first workgroup (the optimizer step counter).
// Up to 4 independent grouped slab reductions in one launch (per-segment slabs / S / n / lds / dst / ldd).
int har_reduce_slabs_multi(int nseg, const float* const* slabs, const int* S, const int64_t* n, const int64_t* lds,
                           float* const* dst, const int64_t* ldd, int G, int32_t* tick, hipStream_t s);
int har_reduce_slabs_grouped(const float* slabs, int S, int64_t n, int64_t lds, float* dst, int G, int64_t ldd,
                             int32_t* tick, hipStream_t s);

// dst[i] = sum_s slabs[s*n + i]  (deterministic split-K reduction)
int har_reduce_slabs(const float* slabs, int nslabs, int64_t n, float* dst, hipStream_t s);

// fp32 -> bf16 cast with row padding: out[r][0:cols_out] = in[r][0:cols_in], zero fill.
int har_cast_pad_bf16(const float* in, int rows, int cols_in, int ld_in, uint16_t* out, int cols_out,
                      hipStream_t s);

// ---- randomness (Philox4x32-10 keyed by global row id) ----
int har_philox_buckets(uint64_t seed, uint32_t stream, int64_t row0, int64_t n, const uint32_t* thr,
                       int nthr, int32_t* out, hipStream_t s);
// Per-fit init (tree.hip): W [T][N] = bootstrap draw from the CDF table (or 1) x optional rw [T][N]; node_of [T][N]
// = 0 / -1 (zero weight); root class counts added into stats + t * stats_tree_stride; *bad = 1 on a
// label outside [0, K).
// cdf: HOST array of ncdf (<= 16) uint32 bootstrap CDF thresholds (ncdf = 0: every weight 1).
int har_tree_init(uint64_t seed, int tree0, int ntrees, int64_t row0, int64_t n, const uint32_t* cdf, int ncdf,
                  const float* rw, const int32_t* y, int K, float* W, int32_t* node_of, float* stats,
                  int64_t stats_tree_stride, int32_t* bad, hipStream_t s);
// findSplits cut points from the per-feature sorted sample [F][n] (NaN last), n <= 16384, ns <= 63:
// out [F][ns + 1] = thresholds then their count.
int har_find_splits_post_sort(const float* sorted, int F, int n, int ns, float* out, hipStream_t s);
// findSplits sample sort: columns of the row-major X [n][ld] (F of them) -> out [F][n] ascending, NaN
// last (n <= 16384: one LDS bitonic sort per column).
int har_sort_columns(const float* X, int n, int F, int ld, float* out, hipStream_t s);
int har_poisson_bootstrap(uint64_t seed, int tree0, int ntrees, int64_t row0, int64_t n, uint8_t* out,
                          hipStream_t s);

// ---- statistics / metrics ----
// Column count/sum/sumsq/min/max (optional row weights, NaN skipped) -> stats[5][ncols] (double);
// workspace: har_column_stats_workspace(n, ncols) doubles.
int har_column_stats(const float* X, int64_t n, int ncols, int ld, const float* w, double* stats,
                     double* workspace, hipStream_t s);
int har_column_stats_f64(const double* X, int64_t n, int ncols, const double* center, double* stats,
                         double* workspace, hipStream_t s);
int64_t har_column_stats_workspace(int64_t n, int ncols);
// bins[f][i] = #{b < nthr[f] : thr[f][b] < X[i][f]}  (uint8, feature-major)
int har_bin_features(const float* X, int64_t n, int F, int ld, const float* thr, int maxb, const int32_t* nthr,
                     uint8_t* bins, hipStream_t s);
// counts of codes in [0, V) (V <= 32768; -1 / out-of-range ignored) into out[V] (zeroed here)
int har_value_counts(const int64_t* codes, int64_t n, int V, int64_t* out, hipStream_t s);
int har_confusion_matrix(const int32_t* label, const int32_t* pred, int64_t n, int K, int64_t* cm,
                         hipStream_t s);
int har_regression_moments(const float* y, const float* yhat, int64_t n, double* out6, hipStream_t s);
// B models' confusion matrices over masked rows: pred / mask [B][n] (mask != 0 = scored), cm [B][K][K]
// (zeroed here)
// DP forest level wire format (tree_dp.hip): per-node present classes / field widths packed into
// int32 words (sum-exact), and the owner's unpack back to an fp32 [n][mb][K] store
int har_tree_dp_pack(const float* store, int A, int64_t slot, int mb, int K, const int32_t* cls, const int32_t* kp,
                     const int32_t* bw, const int64_t* woff, int32_t* out, hipStream_t s);
int har_tree_dp_unpack(const int32_t* in, int a0, int n, int64_t slot, int mb, int K, const int32_t* cls,
                       const int32_t* kp, const int32_t* bw, const int64_t* woff, int64_t base, float* local,
                       hipStream_t s);
int har_confusion_matrix_batched(const int32_t* label, const int32_t* pred, const uint8_t* mask, int64_t n, int B,
                                 int K, int64_t* cm, hipStream_t s);
// scores sorted descending, labels permuted alike (positive iff > 0.5):
// out4 = {sum dFP (TP + TP_prev), sum dTP (prec + prec_prev), P, N} over tie-group end points
int har_roc_pr_sums(const float* sorted_scores, const float* labels, int64_t n, double* out4, hipStream_t s);
int har_roc_pr_sums_batched(const float* sorted_scores, const float* labels, const int32_t* ns, int B, int64_t ld,
                            double* out, hipStream_t s);

// ---- logistic regression (batched over B models, K classes padded to 8) ----
// ---- device logistic regression + batched L-BFGS / OWL-QN (logreg_qn.hip) ----
typedef struct LogregEvalArgs {
  const float* dense;       // [N][ldd] dense feature columns (Fd used)
  int64_t ldd;
  int Fd;
  const int32_t* dense_cols;  // [Fd] global column id of each dense column
  const int32_t* cat;       // [N][C] global column id of each row's one-hot entry, -1 = none
  int C;
  const int32_t* y;         // [N] labels (mode 0)
  const float* rw;          // [S][N] row weights per spec (null = 1)
  const float* inv_wsum;    // [S]
  const float* W;           // [n_trial_models][F+1][KP] effective weights (row F = intercept)
  int64_t N;
  int F, K, T, tstride;     // model bt = model0 + blockIdx.y * tstride, spec = bt / T
  int model0;               // first model of the launch (R holds one [N][KP] slot per launched model)
  int mode;                 // 0 = loss/gradient, 1 = margins into R
  float* R;                 // [n_trial_models][N][KP] residuals (mode 0, needed when C > 0) / margins
  float* slab;              // [n_trial_models][tiles][Fd*KP + KP + 1]
} LogregEvalArgs;

typedef struct LogregGradArgs {
  const float* slab;
  const float* R;
  const int32_t* col_map;   // [F+1]: >= 0 dense index, -1 intercept, <= -2 one-hot (CSC rows)
  const int32_t* csc_rows;  // row ids of the one-hot columns, column-major, ascending per column
  const int32_t* csc_off;   // [F+2] CSC offsets of every column
  const int32_t* col_slice; // [F+2] first row slice of each column (har_logreg_col_slices)
  int SL;                   // rows per slice
  const float* inv_std;     // [S][F]
  const float* pmask;       // [S][K][F+1]
  int64_t N;
  int F, Fd, K, T, tstride, ntiles;
  int model0;               // as LogregEvalArgs: model bt = model0 + blockIdx.y * tstride, R slot blockIdx.y
  float* G;                 // [n_trial_models][K][F+1]
  double* loss;             // [n_trial_models] (loss_fx == null)
  float* loss_fx;           // [n_trial_models][5] fixed-point loss pieces for the DP bucket, or null
  const int32_t* col_blk;   // [nblk][4] column blocks (c0, c1, first slice, end slice): <= 256 columns and
  int nblk;                 // <= 256 slices each (a lone heavier column excepted), or null: fixed 256 columns
  const int32_t* srow;      // [slices + 1] first CSC row of every slice (with col_blk)
} LogregGradArgs;

typedef struct QnArgs {
  int B, T, K, F, m, head, filled, init, nch;
  int fin_it;               // phase 2: hist row of the objective it leaves (0 for the init update)
  int64_t D;                // K * (F + 1)
  float* x;                 // [B][D] standardized parameters
  float* g;                 // [B][D] smooth gradient at x
  double* fobj;             // [B] objective at x (smooth + regularization)
  const float* l1;          // [B][D] per-element L1 weights (null = pure L-BFGS)
  const float* l2;          // [B][D] per-element L2 weights
  const float* pmask;       // [B][D]
  const float* inv_std;     // [B][F]
  float* S;                 // [m][B][D]
  float* Y;                 // [m][B][D]
  double* rho;              // [m][B] (0 = empty / rejected slot)
  double* SY;               // [B][m][m] history Gram matrix s_i . y_j
  double* YY;               // [B][m][m] history Gram matrix y_i . y_j
  double* P1;               // [B][nch][2m+1] chunk partials of the next direction's dots (phase 2)
  double* P2;               // [B][nch][3T+2] chunk partials (phase 1)
  double* P3;               // [B][nch][5+3m] chunk partials (phase 2)
  float* xtrial;            // [B*T][D]
  float* weff;              // [B*T][F+1][KP]
  double* reg;              // [B*T]
  double* decr;             // [B*T]
  const float* G;           // [B*T][D] data gradient of each trial (masked, scaled)
  const double* loss;       // [B*T] data loss of each trial
  float* step_scale;        // [B]
  int32_t* active;          // [B]
  int32_t* fails;           // [B]
  int32_t* iters;           // [B]
  int32_t* steep;           // [B] steepest descent this iteration (the last direction was not descent)
  int32_t* pick;            // [B] trial taken by the last phase 2 (-1 none, -2 non-descent)
  double* hist;             // [max_iter + 1][B] objective per iteration (nullable)
  int32_t* done;            // [B] phase-2 chunks done (zeroed; the last chunk resets it)
  double c1, tol;
} QnArgs;

int har_logreg_eval(const LogregEvalArgs* a, int KP, int n_models, hipStream_t s);
int har_logreg_eval_tiles(int64_t n);
int har_logreg_grad(const LogregGradArgs* a, int KP, int n_models, hipStream_t s);
typedef struct LogregSummaryArgs {
  const float* dense;       // [N][ldd] dense feature columns
  int64_t ldd;
  int Fd;
  const int32_t* y;         // [N]
  const float* rw;          // [S][N] row weights (null = 1)
  int64_t N;
  int F, K, S;
  const int32_t* col_map;   // [F+1] (HybridMatrix.col_map)
  const int32_t* csc_rows;
  const int32_t* csc_off;   // [F+2]
  const int32_t* col_slice; // [F+2] (har_logreg_col_slices)
  int SL;
  int ntiles;               // har_logreg_summary_tiles(N)
  const int32_t* srow;      // [slices + 1] first CSC row of every slice, or null (search the slice's column)
  double* part;             // [S][ntiles][2 Fd + K + 1] tile partials
  double* summ;             // [S][1 + 2F + K] (sum w, sum w x, sum w x^2, class sums)
} LogregSummaryArgs;

typedef struct LogregPrepareArgs {
  const double* summ;       // [B][1 + 2F + K] (all-reduced in data-parallel fits)
  const float* reg;         // [B] regParam
  const float* alpha;       // [B] elasticNetParam
  int B, F, K, Kp;
  int standardization, fit_intercept, binomial;
  float* inv_std;           // [B][F]
  float* inv_wsum;          // [B]
  float* pmask;             // [B][Kp][F+1]
  float* l2;                // [B][Kp (F+1)]
  float* l1;                // [B][Kp (F+1)] or null (no L1 term)
  float* x0;                // [B][Kp][F+1]
} LogregPrepareArgs;

// phase 0: tile partials, phase 1: column sums
int har_logreg_summary(const LogregSummaryArgs* a, int phase, hipStream_t s);
int har_logreg_summary_tiles(int64_t n);
int har_logreg_prepare(const LogregPrepareArgs* a, hipStream_t s);
int har_logreg_col_slices(const int32_t* csc_off, int F, int SL, int32_t* col_slice, hipStream_t s);
int har_logreg_loss_decode(const float* fx, double* loss, int n, hipStream_t s);
int har_qn_chunks(int64_t D, int B);
int har_lbfgs_phase(const QnArgs* a, int KP, int phase, hipStream_t s);
// the whole L-BFGS / OWL-QN solve as one cooperative launch: 0 ran, -4 not available here (use
// the launch sequence), -2 invalid; sync = 2 device words (barrier counter, timeout flag)
uint32_t har_logreg_set_spin_limit(uint32_t n);
// diagnostic phase stamps of the evaluation / direction / update kernels (tools/lr_stamps.py); null = off
void har_lr_set_stamps(uint64_t* ev, uint64_t* dir, uint64_t* upd, uint64_t* grd);
int har_logreg_solve_persistent(const QnArgs* q, const LogregEvalArgs* evT, const LogregGradArgs* grT, int nT,
                                const LogregEvalArgs* ev1, const LogregGradArgs* gr1, int n1, int KP, int max_iter,
                                uint32_t* sync, int max_grid, hipStream_t s);



// ---- windowed feature extraction over raw [S, A] streams ----
// Training-input variant: bf16 ((isnan(v) ? nan_value : v) - mean) * inv_std rows, zero-padded to ld_out.
int har_window_features_mlp(const float* stream, int64_t n_samples, int axes, int window, int stride,
                            int64_t n_windows, float hz, const float* mean, const float* inv_std, float nan_value,
                            uint16_t* out, int ld_out, hipStream_t s);
int har_window_features(const float* stream, int64_t n_samples, int axes, int window, int stride,
                        int64_t n_windows, float hz, int nbins, float* out, int ld_out, hipStream_t s);
// Probe switch: 1 = the pre-v3 (per-sample LDS reads) window kernels only, 0 = default selection.
void har_window_set_legacy(int on);

// ---- trees ----
// Fused per-level histogram + best split; grid (feature chunks, active nodes).
// rows/row_w list each node's rows contiguously (node_start/node_count); feats [A][m].
// Outputs per (node, chunk): gain (-inf = none), global feature, bin, left class counts [K];
// out_total [A][K] = node class counts.  mode 0 fused; 1 histogram only -> ghist [A][m][maxbins][K];
// 2 split search from ghist (after a cross-rank reduction).  row_chunks > 1 (mode 1 only): each node's
// rows are split over that many workgroups that atomically merge into a ZEROED ghist.
// One-hot-aware histograms (tree.hip SPARSE): cat [N][ncat] int32 = the global column of each row's 1 in
// every one-hot block (-1 none), onehot [F] uint8 = 1 for the one-hot columns; F = the feature count.
typedef struct TreeSparse {
  const int32_t* cat;
  int ncat;
  const uint8_t* onehot;
  int F;
} TreeSparse;
// bins [F][n] of a hybrid matrix (numeric block dense [n][Fd] at columns dense_cols, one-hot entries cat)
// findSplits of a hybrid matrix (its sampled rows: cat [n][ncat]; colmap [F] = numeric index or < 0 for
// one-hot; dthr [Fd][ns + 1] = find_splits_post_sort of the numeric block) -> thr_mat [F][maxb], nbins [F]
int har_tree_thresholds_hybrid(const int32_t* cat, int64_t n, int ncat, int F, const int32_t* colmap, const float* dthr,
                               int ns, int maxb, int32_t* ones, float* thr_mat, int32_t* nbins, hipStream_t s);
int har_tree_bins_hybrid(const float* dense, int64_t n, int Fd, const int32_t* dense_cols, const int32_t* cat, int ncat,
                         int F, const float* thr, int maxb, const int32_t* nbins, uint8_t* bins, hipStream_t s);
int har_tree_hist_split(const uint8_t* bins, int64_t N, int F, int row_major, const int32_t* nbins_feat, const int32_t* rows,
                        const float* row_w, const int32_t* node_start, const int32_t* node_count, int A,
                        const int32_t* feats, int m, int fc, const int32_t* label, int K, int maxbins,
                        float min_inst, float min_gain, int impurity, float* out_gain, int32_t* out_feat,
                        int32_t* out_bin, float* out_left, float* out_total, int mode, float* ghist,
                        int row_chunks, const TreeSparse* sparse, hipStream_t s);
// Device-count convention of the level kernels below: a non-null a_dev / p_dev / s_dev points at the
// level's real count on the device and the host's A / P / S is then only an upper bound (grid size
// and array stride), so a whole fit can be enqueued without reading counts back per level.
// Load-balanced level (tree.hip): har_tree_plan builds the work plan from the node row counts
// (nodes of > prows rows become ceil(count / prows) chunk items with a merged-histogram slot, zeroed
// here for at most max_big slots of slot_elems floats); then har_tree_hist_split_planned mode 3
// (grid.y = an upper bound of the items: fused small nodes + chunk histograms) and mode 4 (grid.y
// = max_big: split search of the merged big nodes).  by_node = 1 keeps every node's histogram in
// ghist = a per-node store [A][m][bins][K]; mode 5 then derives the nodes marked derive_from[a] >= 0
// (sibling subtraction, parents in hprev, frontier-provided parent_of / derive_from).
int har_tree_plan(const int32_t* counts, int A, int prows, int32_t* plan, int64_t slot_elems, float* ghist,
                  int max_big, int by_node, const int32_t* a_dev, hipStream_t s);
int har_tree_hist_split_planned(const uint8_t* bins, int64_t N, int F, int row_major, const int32_t* nbins_feat,
                                const int32_t* rows, const float* row_w, const int32_t* node_start,
                                const int32_t* node_count, int A, const int32_t* feats, int m, int fc,
                                const int32_t* label, int K, int maxbins, float min_inst, float min_gain, int impurity,
                                float* out_gain, int32_t* out_feat, int32_t* out_bin, float* out_left,
                                float* out_total, int mode, float* ghist, int row_chunks, const int32_t* plan,
                                int prows, int bound, int by_node, const float* hprev, const int32_t* derive_from,
                                const int32_t* parent_of, const TreeSparse* sparse, hipStream_t s);
// Sum over trees of (normalized) leaf statistics; trees as SoA [T][maxn] arrays, feature < 0 = leaf.
// Level bookkeeping of the forest builder (tree_level.hip): Floyd feature subsets per (tree, node)
// (bit-identical to har/ops/rng.py), per-(tree,row) candidate keys, and the row -> child partition.
int har_tree_feature_subsets(uint64_t seed, const int32_t* trees, const int32_t* nodes, int64_t P, int F, int m,
                             int32_t* out, const int32_t* p_dev, hipStream_t s);
int har_tree_level_keys(const int32_t* node_of, const int32_t* cand_idx, int T, int64_t N, int maxn, int32_t* key,
                        hipStream_t s);
// Stable grouping of the level's (tree, row) pairs by candidate node (no sort); cnt_ws holds
// har_tree_level_group_chunks(N) x A ints.  -4: a tree has more than 4096 candidates.
int har_tree_level_group(const int32_t* node_of, const int32_t* cand_idx, const int32_t* tree_lo, const float* W,
                         int T, int64_t N, int maxn, int A, int nt_max, int32_t* cnt_ws, int32_t* counts,
                         int32_t* starts, int32_t* rows, float* row_w, const int32_t* a_dev, hipStream_t s);
int har_tree_level_group_chunks(int64_t N);
// Commit the level's splits (feature / bin / threshold / children / gain / child stats) in one launch,
// then move rows with the committed arrays (no per-level temporaries).
int har_tree_commit_level(int S, const int64_t* ti, const int64_t* ni, const int64_t* cl, const int64_t* dsi,
                          const int32_t* rfeat, const int32_t* rbin, const float* rgain, const float* rleft,
                          const float* rtotal, int K, const float* thr_mat, int ldthr, int maxn, int32_t* feature,
                          int32_t* split_bin, float* thresh, int32_t* left, int32_t* right, float* gains,
                          float* stats, const int32_t* s_dev, hipStream_t s);
int har_tree_partition_split(int32_t* node_of, const int32_t* feature, const int32_t* split_bin, const int32_t* left,
                             const uint8_t* bins, int T, int64_t N, int maxn, hipStream_t s);
int har_tree_level_decide(int A, const float* gain, const float* left, const float* total, int K, int impurity,
                          float min2, float* out, const int32_t* a_dev, hipStream_t s);
// Device-resident frontier update from the level decisions (see tree_level.hip): commit records
// ti/ni/cl/dsi [<= A], next candidates ct/cn [<= 2A], tree starts [Tn + 1], cand_idx entries, and
// scal = [splits, next candidates, max per tree, max weight float bits] (the level's one D2H).
int har_tree_frontier(int A, int Tn, int maxn, const int32_t* ct, const int32_t* cn, const int32_t* tlo,
                      const float* dec, const int32_t* n_nodes, int32_t* n_nodes_next, int32_t* pos_ws, int64_t* ti,
                      int64_t* ni, int64_t* cl, int64_t* dsi, float* front, int32_t* q_ws, int32_t* ct_next,
                      int32_t* cn_next, int32_t* tlo_next, int32_t* cand_idx, int32_t* scal, const int32_t* a_dev,
                      int32_t* parent_of, int32_t* derive_from, hipStream_t s);
// Root frontier (candidate roots, tree starts, cand_idx, scal = [0, A, 1, max weight bits]) from the
// root class counts stats[t * tree_stride .. + K), on the device.
int har_tree_root_frontier(const float* stats, int Tn, int K, int64_t tree_stride, int impurity, float min2,
                           int maxn, int32_t* ct, int32_t* cn, int32_t* tlo, int32_t* cand_idx, int32_t* scal,
                           hipStream_t s);
int har_tree_partition(int32_t* node_of, const int32_t* lvl_feat, const int32_t* lvl_bin, const int32_t* lvl_left,
                       const uint8_t* bins, int T, int64_t N, int maxn, hipStream_t s);
int har_forest_predict(const float* X, int64_t n, int F, int ld, const int32_t* feat, const float* thr,
                       const int32_t* left, const int32_t* right, const float* leaf, int ntrees, int maxn, int K,
                       int max_depth, int normalize, float* raw_out, hipStream_t s);

// ---- CSV on device (4 KiB chunks per workgroup) ----
int har_csv_count_newlines(const uint8_t* buf, int64_t n, int32_t* counts, hipStream_t s);
int har_csv_newline_pos(const uint8_t* buf, int64_t n, const int64_t* block_off, int64_t* pos, hipStream_t s);
// Per (col, row) outputs ([ncols][nrows]): fp64 value (NaN if not numeric), FNV-1a hash,
// flags (bit0 present, bit1 int literal, bit2 float literal, bit3 quoted), byte span.
int har_csv_parse_rows(const uint8_t* buf, const int64_t* starts, const int64_t* ends, int64_t nrows, int ncols,
                       double* vals, uint64_t* hashes, uint8_t* flags, int64_t* fstart, int32_t* flen,
                       hipStream_t s);

#ifdef __cplusplus
}
#endif
