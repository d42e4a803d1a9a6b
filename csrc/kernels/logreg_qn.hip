// Device-resident multinomial logistic regression + batched L-BFGS / OWL-QN.
//
// Reference: LogisticRegression(maxIter=20, regParam=0.3) and the 3x3 x 5-fold CrossValidator
// (Main/main.py:115-124, 202-215).  Spark runs Breeze L-BFGS on the JVM driver with one
// treeAggregate of (loss, gradient) over the executors per evaluation; here every model of a
// batch (the 45 CV fits) and every trial step of its line search advance in lock step on the
// device and the host only enqueues kernels:
//
//   lbfgs_direction  one workgroup per model: OWL-QN pseudo-gradient, two-loop recursion over
//                    the m-slot history, orthant projection, then T trial points
//                    x + a0 2^-t d (t < T) and, for each, the standardized effective weights
//                    W_eff = x * inv_std * mask laid out [F+1][KP] for the evaluator, the
//                    regularization value and the Armijo decrease term (padded classes
//                    k >= K of W_eff are zero from allocation and never written)
//   logreg_eval      one workgroup per (256-row tile, trial model): margins from the HYBRID
//                    feature layout (C one-hot columns gathered by index + Fd dense columns
//                    staged in LDS), softmax, cross entropy, residual R = w (p - onehot(y));
//                    the dense-column / intercept gradient and the loss of the tile are
//                    reduced in LDS and written to a per-tile slab (no atomics)
//   logreg_grad      one lane per (feature column, trial model): sums the slabs in tile order,
//                    or the residuals of the rows holding a one-hot column (CSC row lists),
//                    and scales by inv_std * mask — every sum in a fixed order, so a fit is
//                    bitwise reproducible
//   lbfgs_update     one workgroup per model: picks the largest trial step that satisfies the
//                    Armijo condition, updates x / g / objective and the history slot,
//                    convergence flags (frozen models stop moving; nothing reads back to host)
//
// A one-hot feature of the reference's 3,100-dim encoding (Main/main.py:51-66) is one gathered
// weight column per row instead of 3,090 multiplications by zero: the WISDM objective reads
// ~60 bytes per row instead of 12.4 KB.
#include <algorithm>
#include <cstdlib>

#include "common.h"
#include "wave_ops.h"
#include "../har_kernels.h"

// Diagnostic phase stamps (tools/lr_stamps.py): a STAMP instantiation of the evaluation / direction /
// update kernels, launched only while har_lr_set_stamps() holds a buffer, has thread 0 of every
// workgroup store s_memtime at fixed points into its 16-slot row (workgroup = y * gridDim.x + x).
uint64_t* g_lr_stamps = nullptr;       // evaluation kernel rows
uint64_t* g_lr_stamps_dir = nullptr;   // direction kernel rows
uint64_t* g_lr_stamps_upd = nullptr;   // update kernel rows
uint64_t* g_lr_stamps_grd = nullptr;   // gradient kernel rows
namespace {
#define HAR_LR_STAMP(k)                                                                                  \
  if constexpr (STAMP) {                                                                                 \
    if (threadIdx.x == 0)                                                                                \
      st[((size_t)blockIdx.y * gridDim.x + blockIdx.x) * 16 + (k)] = __builtin_amdgcn_s_memtime();      \
  }

constexpr int EVAL_ROWS = 256;

// ---------------------------------------------------------------------------------------------
// logreg_eval: one workgroup = EVAL_ROWS rows x one (trial) model.  The dense columns go through
// LDS in chunks of EVAL_DCH (any width: a 165-column 9-axis design or an un-one-hot numeric design
// uses the same kernel as the 10 dense columns of the reference encoding): pass A accumulates the
// margins chunk by chunk (column order = the order of one unchunked sweep), pass B re-stages the
// chunks newest-first (the last one is still in LDS) for the tile's dense gradient R^T X.
// ---------------------------------------------------------------------------------------------
constexpr int EVAL_DCH = 32;                       // dense columns per LDS chunk
// LDS row stride of the dense tile (a compile-time constant: the tile's row addresses fold into
// immediate offsets): 33 in general, 11 for designs of at most 10 dense columns (the reference
// encoding) — an 11 KB tile instead of 34 KB, so three times as many evaluation workgroups fit a CU
// (the 54-model CrossValidator batch: 62 -> 49 us per evaluation)
constexpr int EVAL_XLD_NARROW = 11;
__host__ __device__ constexpr int eval_xld(int Fd) { return Fd <= EVAL_XLD_NARROW - 1 ? EVAL_XLD_NARROW : EVAL_DCH + 1; }
// Dense designs wider than the narrow tile run both dense products on the matrix cores (MF kernels,
// v_mfma_f32_16x16x4_f32: fp32 operands, fp32 accumulation): the margins of the tile's 256 rows as
// W^T . X^T (16 classes x 4 columns per step; KP = 8 pads the class rows with zeros) and the tile's
// dense gradient R^T . X (16 classes x 16 columns, the rows split over the 4 waves, their partials
// added in a fixed order: still bitwise reproducible).  Row pitch 36: the chunk zero-padded to a
// multiple of 4 columns, and the 16 rows x 4 columns of an operand read hit 64 distinct banks.
constexpr int EVAL_XLD_MF = 36;
// ... and the narrow designs (<= 10 dense columns, the reference encoding) on the matrix cores too, at
// row pitch 12 (the chunk padded to 12 columns; 16 rows x 4 columns of a pass-A operand read still hit
// 64 distinct banks): pass B's 80 scalar 256-long LDS chains (~5.3k cycles, eval stamps) become 16
// MFMAs per wave (4.7k -> 2.5k cycles).  With the row-owned staging of the narrow tile it is the default
// for both the single fit and the 54-model CrossValidator batch (same-box A/B: LR 0.93 vs 0.94-0.99 ms,
// LR-CV 4.28-4.34 vs 4.36-4.60 ms, profiles/r5/lr_grad_blocks.md); HAR_LR_EVAL_MFN=0 keeps the scalar
// narrow kernel, -1 uses the MFMA one for launches of <= 256 workgroups only
constexpr int EVAL_XLD_MFN = 12;
template <int XLD> constexpr bool eval_mf() { return XLD == EVAL_XLD_MF || XLD == EVAL_XLD_MFN; }

template <int KP, int XLD>
__device__ __forceinline__ void eval_stage_chunk(const LogregEvalArgs& a, const float* W, float* wd, float* xs,
                                                 int c0, int nc, int64_t r0, int64_t nrow_tile, bool weights) {
  const int tid = threadIdx.x;
  // (MF pitch: columns nc .. nc4 - 1 of the chunk staged as zeros, the MFMA k steps are 4 wide)
  const int ncs = eval_mf<XLD>() ? (nc + 3) & ~3 : nc;
  if (weights)
    for (int e = tid; e < ncs * KP; e += EVAL_ROWS)
      wd[e] = e / KP < nc ? W[(int64_t)a.dense_cols[c0 + e / KP] * KP + (e % KP)] : 0.f;
  if constexpr (XLD == EVAL_XLD_NARROW || XLD == EVAL_XLD_MFN) {
    // narrow tile (<= 10 columns): thread = row, its nc values in ONE round of loads (the flat loop
    // below takes two rounds of 8 for the 10 x 256 tile, with an integer division per element);
    // the MFMA pitch's columns nc .. ncs - 1 as zeros
    constexpr int NW = EVAL_XLD_NARROW - 1;
    const bool in = tid < nrow_tile;
    const float* rp = a.dense + (r0 + (in ? tid : 0)) * a.ldd + c0;
    float v[NW];
#pragma unroll
    for (int j = 0; j < NW; ++j) v[j] = j < nc ? rp[j] : 0.f;
#pragma unroll
    for (int j = 0; j < XLD; ++j)
      if (j < ncs) xs[tid * XLD + j] = in && j < nc ? v[j < NW ? j : 0] : 0.f;
    return;
  }
  // U loads in flight per thread (clamped to a valid element, zeroed by a select), then the U stores:
  // the plain loop waited out one global round trip per element (10 per tile at 10 dense columns,
  // most of the evaluation's latency)
  constexpr int U = 8;
  const int tot = EVAL_ROWS * ncs;
  for (int e0 = tid; e0 < tot; e0 += U * EVAL_ROWS) {
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = e0 + u * EVAL_ROWS;
      const int rr = e / ncs, j = e % ncs;
      const bool in = e < tot && rr < nrow_tile && j < nc;
      const float x = a.dense[(r0 + (in ? rr : 0)) * a.ldd + c0 + (in ? j : 0)];
      v[u] = in ? x : 0.f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = e0 + u * EVAL_ROWS;
      if (e < tot) xs[(e / ncs) * XLD + (e % ncs)] = v[u];
    }
  }
}

__device__ __forceinline__ f32x4_t mfma4(float a, float b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// The kernel bodies below take their workgroup coordinates as arguments: the stand-alone kernels pass
// blockIdx / gridDim, the persistent solve (logreg_solve_persistent_kernel) its virtual blocks.
template <int KP, int XLD, bool STAMP = false>
__device__ __forceinline__ void logreg_eval_body(const LogregEvalArgs& a, int bx, int by, int gdx, float* smem,
                                                 uint64_t* st = nullptr) {
  HAR_LR_STAMP(0)
  const int Fd = a.Fd;
  float* wd = smem;                                // [EVAL_DCH][KP] dense weights of the chunk
  constexpr int xld = XLD;
  float* xs = wd + EVAL_DCH * KP;                  // [EVAL_ROWS][xld] dense row tile, one chunk
  float* rs = xs + EVAL_ROWS * xld;                // [EVAL_ROWS][KP]
  float* red = rs + EVAL_ROWS * KP;                // [EVAL_ROWS / 64]
  constexpr bool MF = eval_mf<XLD>();              // matrix-core dense products
  float* pb = red + EVAL_ROWS / 64;                // MF: [4 waves][EVAL_DCH][KP] gradient partials
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int l16 = lane & 15, kq = lane >> 4;

  const int tid = threadIdx.x;
  const int bt = a.model0 + by * a.tstride;  // trial model (its residual rows: R slot by)
  const int s = bt / a.T;                          // spec (row-weight vector) of the model
  const int64_t r0 = (int64_t)bx * EVAL_ROWS;
  const int64_t row = r0 + tid;
  const bool ok = row < a.N;
  const float* W = a.W + (int64_t)bt * (a.F + 1) * KP;
  const int64_t nrow_tile = min((int64_t)EVAL_ROWS, a.N - r0);
  const int nchunk = (Fd + EVAL_DCH - 1) / EVAL_DCH;

  // designs with <= 4 one-hot features (the reference encoding: 3): this row's category indices and
  // their weight rows are loaded now, under the dense staging (added below in the same order as the
  // grouped gathers: the same sums)
  constexpr int CP = 4;
  const bool cpre = a.C <= CP;
  f32x4_t wpre[CP][KP / 4];
  bool onp[CP];
  if (cpre) {
    const int32_t* cr = a.cat + (ok ? row : 0) * a.C;
    int cp[CP];
#pragma unroll
    for (int u = 0; u < CP; ++u) cp[u] = u < a.C ? cr[u] : -1;
#pragma unroll
    for (int u = 0; u < CP; ++u) {
      onp[u] = ok && cp[u] >= 0;
      const f32x4_t* wp = reinterpret_cast<const f32x4_t*>(W + (int64_t)max(cp[u], 0) * KP);
#pragma unroll
      for (int q = 0; q < KP / 4; ++q) wpre[u][q] = wp[q];
    }
  }
  // ---- pass A: margins ----
  float z[KP];
#pragma unroll
  for (int k = 0; k < KP; ++k) z[k] = W[(int64_t)a.F * KP + k];  // intercept row
  f32x4_t za[4] = {f32x4_t{0.f, 0.f, 0.f, 0.f}, f32x4_t{0.f, 0.f, 0.f, 0.f}, f32x4_t{0.f, 0.f, 0.f, 0.f},
                   f32x4_t{0.f, 0.f, 0.f, 0.f}};  // MF: z^T of the wave's 4 row blocks (lane: row l16, classes 4 kq + r)
  for (int ch = 0; ch < nchunk; ++ch) {
    const int c0 = ch * EVAL_DCH, nc = min(EVAL_DCH, Fd - c0);
    if (ch) __syncthreads();                       // the previous chunk is consumed
    eval_stage_chunk<KP, XLD>(a, W, wd, xs, c0, nc, r0, nrow_tile, true);
    __syncthreads();
    if constexpr (MF) {
      const int nc4 = (nc + 3) & ~3;
      for (int j0 = 0; j0 < nc4; j0 += 4) {
        const float av = l16 < KP ? wd[(j0 + kq) * KP + l16] : 0.f;  // A = W^T [class l16][column j0 + kq]
#pragma unroll
        for (int rb = 0; rb < 4; ++rb)                                   // B = X^T [column j0 + kq][row l16]
          za[rb] = mfma4(av, xs[(wv * 64 + rb * 16 + l16) * XLD + j0 + kq], za[rb]);
      }
    } else if (ok) {
      for (int j = 0; j < nc; ++j) {
        const float xv = xs[tid * xld + j];
#pragma unroll
        for (int k = 0; k < KP; ++k) z[k] = fmaf(xv, wd[j * KP + k], z[k]);
      }
    }
  }
  HAR_LR_STAMP(1)
  if constexpr (MF) {  // the margins through LDS to their rows' threads
#pragma unroll
    for (int rb = 0; rb < 4; ++rb)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (4 * kq + r < KP) rs[(wv * 64 + rb * 16 + l16) * KP + 4 * kq + r] = za[rb][r];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < KP; ++k) z[k] += rs[tid * KP + k];
    __syncthreads();                               // rs is rewritten with the residuals below
  }
  float lossv = 0.f;
  if (ok) {
    // one-hot columns in groups of CG: the group's indices in one round of independent loads, then its
    // weight rows in another (clamped, unconditional), added in column order with a select — two
    // round trips per group instead of two dependent ones per column (a per-column `if (col >= 0)`
    // load serialized ~2 C L2 round trips per evaluation; the sums and their order are unchanged)
    constexpr int CG = 8;  // (16: slower, r5 stamps)
    const int32_t* cr = a.cat + row * a.C;
    if (cpre) {
#pragma unroll
      for (int u = 0; u < CP; ++u) {
#pragma unroll
        for (int q = 0; q < KP / 4; ++q) {
          z[4 * q + 0] = onp[u] ? z[4 * q + 0] + wpre[u][q][0] : z[4 * q + 0];
          z[4 * q + 1] = onp[u] ? z[4 * q + 1] + wpre[u][q][1] : z[4 * q + 1];
          z[4 * q + 2] = onp[u] ? z[4 * q + 2] + wpre[u][q][2] : z[4 * q + 2];
          z[4 * q + 3] = onp[u] ? z[4 * q + 3] + wpre[u][q][3] : z[4 * q + 3];
        }
      }
    }
    for (int c0 = 0; c0 < (cpre ? 0 : a.C); c0 += CG) {
      int cols[CG];
#pragma unroll
      for (int u = 0; u < CG; ++u) {
        const int cu = min(c0 + u, a.C - 1);
        const int v = cr[cu];
        cols[u] = c0 + u < a.C ? v : -1;
      }
      f32x4_t w4[CG][KP / 4];
#pragma unroll
      for (int u = 0; u < CG; ++u) {
        const f32x4_t* wp = reinterpret_cast<const f32x4_t*>(W + (int64_t)max(cols[u], 0) * KP);
#pragma unroll
        for (int q = 0; q < KP / 4; ++q) w4[u][q] = wp[q];
      }
#pragma unroll
      for (int u = 0; u < CG; ++u) {
        const bool on = cols[u] >= 0;
#pragma unroll
        for (int q = 0; q < KP / 4; ++q) {
          z[4 * q + 0] = on ? z[4 * q + 0] + w4[u][q][0] : z[4 * q + 0];
          z[4 * q + 1] = on ? z[4 * q + 1] + w4[u][q][1] : z[4 * q + 1];
          z[4 * q + 2] = on ? z[4 * q + 2] + w4[u][q][2] : z[4 * q + 2];
          z[4 * q + 3] = on ? z[4 * q + 3] + w4[u][q][3] : z[4 * q + 3];
        }
      }
    }
  }
  HAR_LR_STAMP(2)
  float rv[KP];
  if (a.mode == 1) {  // prediction: raw margins out
#pragma unroll
    for (int k = 0; k < KP; ++k) rv[k] = z[k];
  } else {
    const float w = ok ? (a.rw ? a.rw[(int64_t)s * a.N + row] : 1.f) * a.inv_wsum[s] : 0.f;
    const int yi = ok ? a.y[row] : 0;
    float mx = -INFINITY;
#pragma unroll
    for (int k = 0; k < KP; ++k)
      if (k < a.K) mx = fmaxf(mx, z[k]);
    float se = 0.f;
#pragma unroll
    for (int k = 0; k < KP; ++k) {
      const float e = k < a.K ? __expf(z[k] - mx) : 0.f;
      rv[k] = e;
      se += e;
    }
    const float inv = 1.f / se;
    float zy = 0.f;
#pragma unroll
    for (int k = 0; k < KP; ++k) {
      zy = (k == yi) ? z[k] : zy;
      rv[k] = (ok && k < a.K) ? w * (rv[k] * inv - (k == yi ? 1.f : 0.f)) : 0.f;
    }
    lossv = (ok && w != 0.f) ? w * ((mx + __logf(se)) - zy) : 0.f;
  }
#pragma unroll
  for (int k = 0; k < KP; ++k) rs[tid * KP + k] = rv[k];
  if (a.R != nullptr && ok) {
    f32x4_t* rp = reinterpret_cast<f32x4_t*>(a.R + ((int64_t)by * a.N + row) * KP);
#pragma unroll
    for (int q = 0; q < KP / 4; ++q) rp[q] = f32x4_t{rv[4 * q], rv[4 * q + 1], rv[4 * q + 2], rv[4 * q + 3]};
  }
  if (a.mode == 1) return;
  HAR_LR_STAMP(3)
  // tile loss: wave sums, then the 4 wave partials in a fixed order
  lossv = wops::wave_sum_f_dpp(lossv);
  if ((tid & 63) == 0) red[tid >> 6] = lossv;
  __syncthreads();                                 // rs / red complete; the last chunk is in xs
  const int SW = Fd * KP + KP + 1;
  float* slab = a.slab + ((int64_t)bt * gdx + bx) * SW;
  HAR_LR_STAMP(4)
  // ---- pass B: dense gradient R^T X of the tile, chunks newest-first (fixed row order) ----
  for (int ch = nchunk - 1; ch >= 0; --ch) {
    const int c0 = ch * EVAL_DCH, nc = min(EVAL_DCH, Fd - c0);
    if (ch != nchunk - 1) {
      __syncthreads();
      eval_stage_chunk<KP, XLD>(a, W, wd, xs, c0, nc, r0, nrow_tile, false);
      __syncthreads();
    }
    if constexpr (MF) {
      // wave wv: rows 64 wv .. + 63 of R^T . X for every 16-column block of the chunk -> pb[wv]
      for (int fb = 0; fb * 16 < nc; ++fb) {
        f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
        for (int i0 = 0; i0 < 64; i0 += 4) {
          const int row = wv * 64 + i0 + kq;
          const float av = l16 < KP ? rs[row * KP + l16] : 0.f;   // A = R^T [class l16][row]
          acc = mfma4(av, xs[row * XLD + fb * 16 + l16], acc);     // B = X [row][column fb 16 + l16]
        }
        const int j = fb * 16 + l16;                               // D: column j, classes 4 kq + r
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (j < nc && 4 * kq + r < KP) pb[(wv * EVAL_DCH + j) * KP + 4 * kq + r] = acc[r];
      }
      __syncthreads();
      for (int o = tid; o < nc * KP; o += EVAL_ROWS)
        slab[(int64_t)c0 * KP + o] = (pb[o] + pb[EVAL_DCH * KP + o]) + (pb[2 * EVAL_DCH * KP + o] + pb[3 * EVAL_DCH * KP + o]);
    } else {
      // (one 256-row chain per output: four interleaved chains and row ranges on more threads both
      // measured slower, the reads being the bound — r5 stamps)
      for (int o = tid; o < nc * KP; o += EVAL_ROWS) {
        const int j = o / KP, k = o % KP;
        float acc = 0.f;
        for (int i = 0; i < EVAL_ROWS; ++i) acc = fmaf(rs[i * KP + k], xs[i * xld + j], acc);
        slab[(int64_t)c0 * KP + o] = acc;
      }
    }
  }
  HAR_LR_STAMP(5)
  // intercept gradient sum R of the tile
  // intercept: the 8 class sums over the 256 rows on 32 threads per class (8-row chains, then a
  // fixed-order tree of the 32 through LDS), not one 256-long chain per class
  {
    const int k = tid & (KP - 1), part = tid / KP;  // KP classes x (EVAL_ROWS / KP) parts of KP rows
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < KP; ++i) acc += rs[(part * KP + i) * KP + k];
    __syncthreads();  // (every thread's pass-B reads of rs / xs are done: red2 reuses xs)
    float* red2 = xs;
    red2[tid] = acc;
    __syncthreads();
    if (tid < KP) {
      float t = 0.f;
      for (int q = 0; q < EVAL_ROWS / KP; ++q) t += red2[q * KP + tid];
      slab[Fd * KP + tid] = t;
    }
  }
  if (tid == 0) slab[SW - 1] = (red[0] + red[1]) + (red[2] + red[3]);
  HAR_LR_STAMP(6)
}

template <int KP, int XLD, bool STAMP = false>
__global__ __launch_bounds__(EVAL_ROWS) void logreg_eval_kernel(LogregEvalArgs a, uint64_t* st) {
  extern __shared__ float smem[];
  logreg_eval_body<KP, XLD, STAMP>(a, blockIdx.x, blockIdx.y, gridDim.x, smem, st);
}

// ---------------------------------------------------------------------------------------------
// logreg_grad: G[bt][k][col], loss[bt].  Workgroup w owns the columns [256 w, 256 w + 256) and the
// row SLICES of its one-hot columns: a column's CSC row list is cut into slices of a.SL rows
// (col_slice = exclusive scan of ceil(rows / SL), built on the device by logreg_col_slices), so a
// frequent category — '?' in XPEAK, hundreds of rows — is spread over many lanes instead of
// serializing one.  The workgroup walks its slices in rounds of 256: one lane per slice sums its
// rows' residuals into LDS, then one lane per column adds its slices of the round in order (or
// the tile slabs of a dense column / the intercept).  Fixed summation order everywhere: bitwise
// reproducible, and no host-side partition (the grid is ceil((F+1) / 256) x models).
// ---------------------------------------------------------------------------------------------
// Exact loss transport for the data-parallel bucket: a rank's fp64 loss as a 2^-40 fixed-point
// int64 in four 16-bit pieces (three unsigned, the top one signed) carried as fp32 integers, plus
// a non-finite flag.  The fp32 SUM all-reduce adds every piece exactly (|sum| < 2^24 for up to
// 256 ranks), so the decoded total is the exact sum of the ranks' fixed-point losses: one
// collective per evaluation carries the gradient AND a loss good to ~1e-12.
constexpr double LOSS_FX = 1099511627776.0;  // 2^40

__device__ __forceinline__ void loss_encode(double l, float* out) {
  if (!(fabs(l) < 8388608.0)) {  // non-finite or out of range: flag it
    out[0] = out[1] = out[2] = out[3] = 0.f;
    out[4] = 1.f;
    return;
  }
  long long q = llrint(l * LOSS_FX);
  out[0] = (float)(q & 0xffff);
  q >>= 16;
  out[1] = (float)(q & 0xffff);
  q >>= 16;
  out[2] = (float)(q & 0xffff);
  q >>= 16;
  out[3] = (float)q;
  out[4] = 0.f;
}

__device__ __forceinline__ double loss_decode(const float* in) {
  if (in[4] != 0.f) return __builtin_nan("");
  const long long q = (long long)in[0] + ((long long)in[1] << 16) + ((long long)in[2] << 32) +
                      ((long long)in[3] << 48);
  return (double)q / LOSS_FX;
}

// TB trial models per workgroup (TB = 4, opt-in: the four trials of one spec, launches with tstride 1):
// the slice row lists, the column metadata and inv_std / pmask loaded once for the TB models and their
// residual rows gathered together.  The sums per model and their order are those of TB = 1.
template <int KP, bool STAMP = false, int TB = 1>
__device__ __forceinline__ void logreg_grad_body(const LogregGradArgs& a, int bx, int by, uint64_t* st = nullptr) {
  HAR_LR_STAMP(0)
  __shared__ float part[256 * KP * TB];
  __shared__ int cs_l[257];                        // col_slice[c0 .. c1] of the block
  __shared__ float tl[256];                        // tile losses (block 0)
  const int bt0 = a.model0 + TB * by * a.tstride;  // model of trial slot 0 (slot tt: bt0 + tt * tstride)
  const int s = bt0 / a.T;                         // (TB > 1: the TB models share the spec)
  const int Fp1 = a.F + 1;
  const int SW = a.Fd * KP + KP + 1;
  // col_blk (balanced blocks, ops/logreg.py LogregDesign.col_blocks): block bx = columns [c0, c1), slices
  // [s0, s1), and slice sl covers the CSC rows [srow[sl], srow[sl + 1]) — no slice -> column search;
  // everything a lane needs is loaded in ONE round at entry (its slice's rows, its column's slice range,
  // inv_std and pmask).  Without it: fixed 256-column blocks, the slice's column searched in LDS
  const bool fast = a.col_blk != nullptr;
  int c0, c1, s0 = 0, s1 = 0;
  if (fast) {
    const int4 bk = reinterpret_cast<const int4*>(a.col_blk)[bx];
    c0 = bk.x; c1 = bk.y; s0 = bk.z; s1 = bk.w;
  } else {
    c0 = bx * 256;
    c1 = min(Fp1, c0 + 256);
  }
  const int col = c0 + threadIdx.x;
  int cs0 = 0, cs1 = 0, r0f = 0, r1f = 0;
  if (fast) {
    if (col < c1) { cs0 = a.col_slice[col]; cs1 = a.col_slice[col + 1]; }
    if (s0 + (int)threadIdx.x < s1) { r0f = a.srow[s0 + threadIdx.x]; r1f = a.srow[s0 + threadIdx.x + 1]; }
  } else {
    if (c0 + (int)threadIdx.x <= c1) cs_l[threadIdx.x] = a.col_slice[c0 + threadIdx.x];
    if (threadIdx.x == 0 && c1 - c0 == 256) cs_l[256] = a.col_slice[c1];
  }
  // the output scaling of this lane's column, loaded now (its latency hides behind the sums)
  const int64_t D = (int64_t)a.K * Fp1;
  float sc = 1.f, pmv[KP];
#pragma unroll
  for (int k = 0; k < KP; ++k) pmv[k] = 0.f;
  if (col < c1) {
    if (col < a.F) sc = a.inv_std[(int64_t)s * a.F + col];
    const float* pm = a.pmask + (int64_t)s * D;
#pragma unroll
    for (int k = 0; k < KP; ++k)
      if (k < a.K) pmv[k] = pm[(int64_t)k * Fp1 + col];
  }
  const bool loss_block = bx == 0;
#pragma unroll
  for (int tt = 0; tt < TB; ++tt) {
    const int bt = bt0 + tt * a.tstride;
    const float* slab = a.slab + (int64_t)bt * a.ntiles * SW;
    if (tt) __syncthreads();  // tl consumed
    if (loss_block && (int)threadIdx.x < a.ntiles) tl[threadIdx.x] = slab[(int64_t)threadIdx.x * SW + SW - 1];
    __syncthreads();
    if (loss_block && threadIdx.x == 0) {
      double l = 0.0;
      for (int t = 0; t < a.ntiles; ++t)  // tile order (ntiles > 256: the rest straight from the slabs)
        l += (double)(t < 256 ? tl[t] : slab[(int64_t)t * SW + SW - 1]);
      if (a.loss_fx)
        loss_encode(l, a.loss_fx + (int64_t)bt * 5);
      else
        a.loss[bt] = l;
    }
  }
  HAR_LR_STAMP(1)
  if (!fast) {
    s0 = cs_l[0];
    s1 = cs_l[c1 - c0];
    cs0 = col < c1 ? cs_l[threadIdx.x] : 0;
    cs1 = col < c1 ? cs_l[threadIdx.x + 1] : 0;
  }
  const float* R = a.R + (int64_t)TB * by * a.N * KP;  // this launch's residual slots of the TB models
  float g[TB][KP];
#pragma unroll
  for (int tt = 0; tt < TB; ++tt)
#pragma unroll
    for (int k = 0; k < KP; ++k) g[tt][k] = 0.f;
  for (int base = s0; base < s1; base += 256) {
    if (base > s0) __syncthreads();  // the previous round's partials are consumed
    const int sl = base + threadIdx.x;
    if (sl < s1) {
      int r0, r1;
      if (fast) {
        r0 = base == s0 ? r0f : a.srow[sl];
        r1 = base == s0 ? r1f : a.srow[sl + 1];
      } else {
        // the slice's column: the last column of the block whose first slice is <= sl
        int lo = 0, hi = c1 - c0 - 1;
        while (lo < hi) {
          const int mid = (lo + hi + 1) >> 1;
          if (cs_l[mid] <= sl) lo = mid; else hi = mid - 1;
        }
        r0 = a.csc_off[c0 + lo] + (sl - cs_l[lo]) * a.SL;
        r1 = min(r0 + a.SL, a.csc_off[c0 + lo + 1]);
      }
      float gs[TB][KP];
#pragma unroll
      for (int tt = 0; tt < TB; ++tt)
#pragma unroll
        for (int k = 0; k < KP; ++k) gs[tt][k] = 0.f;
      // groups of RG rows: RG row indices, then their RG residual rows (of each of the TB models) in
      // flight (two dependent round trips per group, the slice's last partial group included: rows past
      // r1 re-read row r1 - 1 and add +0, an exact identity since gs is never -0 — the sums are bitwise
      // the row-by-row ones; a row-at-a-time tail cost two round trips PER ROW: grad stamps)
      constexpr int RG = TB > 1 ? 4 : (KP == 8 ? 8 : 4);
      for (int i0 = r0; i0 < r1; i0 += RG) {
        int rid[RG];
#pragma unroll
        for (int j = 0; j < RG; ++j) rid[j] = a.csc_rows[min(i0 + j, r1 - 1)];
        f32x4_t rr[TB][RG][KP / 4];
#pragma unroll
        for (int tt = 0; tt < TB; ++tt)
#pragma unroll
          for (int j = 0; j < RG; ++j)
#pragma unroll
            for (int q = 0; q < KP / 4; ++q)
              rr[tt][j][q] = reinterpret_cast<const f32x4_t*>(R + ((int64_t)tt * a.N + rid[j]) * KP)[q];
#pragma unroll
        for (int j = 0; j < RG; ++j) {
          const bool on = i0 + j < r1;
#pragma unroll
          for (int tt = 0; tt < TB; ++tt)
#pragma unroll
            for (int q = 0; q < KP / 4; ++q) {
              gs[tt][4 * q + 0] += on ? rr[tt][j][q][0] : 0.f;
              gs[tt][4 * q + 1] += on ? rr[tt][j][q][1] : 0.f;
              gs[tt][4 * q + 2] += on ? rr[tt][j][q][2] : 0.f;
              gs[tt][4 * q + 3] += on ? rr[tt][j][q][3] : 0.f;
            }
        }
      }
#pragma unroll
      for (int tt = 0; tt < TB; ++tt)
#pragma unroll
        for (int k = 0; k < KP; ++k) part[(threadIdx.x * TB + tt) * KP + k] = gs[tt][k];
    }
    __syncthreads();
    const int e0 = max(cs0, base), e1 = min(cs1, base + 256);
    for (int e = e0; e < e1; ++e) {  // this column's slices of the round, in order
#pragma unroll
      for (int tt = 0; tt < TB; ++tt)
#pragma unroll
        for (int k = 0; k < KP; ++k) g[tt][k] += part[((e - base) * TB + tt) * KP + k];
    }
  }
  HAR_LR_STAMP(2)
  if (col >= c1) return;
  const int cm = a.col_map[col];
  if (cm >= 0 || cm == -1) {  // dense column j = cm, or the intercept (slab entries after the dense block)
    const int off = cm >= 0 ? cm * KP : a.Fd * KP;
#pragma unroll
    for (int tt = 0; tt < TB; ++tt) {
      const float* slab = a.slab + (int64_t)(bt0 + tt * a.tstride) * a.ntiles * SW;
#pragma unroll 8
      for (int t = 0; t < a.ntiles; ++t) {
        const float* p = slab + (int64_t)t * SW + off;
#pragma unroll
        for (int k = 0; k < KP; ++k) g[tt][k] += p[k];
      }
    }
  }
  HAR_LR_STAMP(3)
#pragma unroll
  for (int tt = 0; tt < TB; ++tt) {
    float* G = a.G + (int64_t)(bt0 + tt * a.tstride) * D;
#pragma unroll
    for (int k = 0; k < KP; ++k)
      if (k < a.K) G[(int64_t)k * Fp1 + col] = g[tt][k] * sc * pmv[k];
  }
  HAR_LR_STAMP(4)
}

template <int KP, bool STAMP = false, int TB = 1>
__global__ __launch_bounds__(256) void logreg_grad_kernel(LogregGradArgs a, uint64_t* st) {
  logreg_grad_body<KP, STAMP, TB>(a, blockIdx.x, blockIdx.y, st);
}
// the same body held to 5+ waves per SIMD (94 VGPRs): more resident workgroups for the batched
// CrossValidator launch — opt-in (HAR_LR_GRAD_WPE=5): LR-CV 4.07-4.24 vs 4.12-4.17 ms, within noise
// (profiles/r5/lr_grad_blocks.md)
template <int KP>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5))) void logreg_grad_kernel_w5(LogregGradArgs a,
                                                                                                  uint64_t* st) {
  logreg_grad_body<KP, false, 1>(a, blockIdx.x, blockIdx.y, st);
}

// after the data-parallel all-reduce of the bucket: the summed fixed-point losses -> fp64
__global__ void logreg_loss_decode_kernel(const float* __restrict__ fx, double* __restrict__ loss, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) loss[i] = loss_decode(fx + (int64_t)i * 5);
}

// col_slice [F+2] = exclusive scan over the F+1 columns of ceil((csc_off[c+1] - csc_off[c]) / SL):
// one 1024-thread workgroup, chunked block scan (integer: exact)
__global__ __launch_bounds__(1024) void logreg_col_slices_kernel(const int32_t* __restrict__ off, int F1, int SL,
                                                                 int32_t* __restrict__ col_slice) {
  __shared__ int wsum[16];
  __shared__ int carry;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (tid == 0) carry = 0;
  __syncthreads();
  for (int base = 0; base < F1; base += 1024) {
    const int c = base + tid;
    const int n = c < F1 ? (off[c + 1] - off[c] + SL - 1) / SL : 0;
    int v = n;  // inclusive wave scan
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int t = __shfl_up(v, o, 64);
      if (lane >= o) v += t;
    }
    if (lane == 63) wsum[w] = v;
    __syncthreads();
    int pre = carry;
    for (int i = 0; i < w; ++i) pre += wsum[i];
    if (c < F1) col_slice[c] = pre + v - n;
    __syncthreads();
    if (tid == 1023) carry = pre + v;
    __syncthreads();
  }
  if (tid == 0) col_slice[F1] = carry;
}

// ---------------------------------------------------------------------------------------------
// Batched L-BFGS / OWL-QN, chunked over the whole chip.
//
// Every model's parameter vector (D = K (F+1) = 18,606 for WISDM) is cut into har_qn_chunks(D, B)
// chunks and each phase runs one 256-thread workgroup per (chunk, model), so a single fit
// streams its history (m = 10 pairs of D floats) with tens of CUs instead of one.  Cross-chunk
// sums go through per-chunk fp64 partial slabs reduced in chunk order by the consumer (fixed
// order: bitwise reproducible).  The two-loop recursion runs in coefficient space on the history
// Gram matrices SY[i][j] = s_i.y_j and YY[i][j] = y_i.y_j (maintained as pairs enter), so a
// direction costs two streaming sweeps instead of 4m dependent ones.
//
//   phase 1  (chunks x B)  reduce P1 -> recursion coefficients (lane 0) -> per element
//                          d = -(gamma pg + sum cY_j y_j + cS_j s_j) (orthant-restricted), the T
//                          trial points x + a0 2^-t d and their W_eff; partial reg / decrease /
//                          pg.d -> P2
//   (logreg_eval + logreg_grad evaluate the B*T trials)
//   phase 2  (chunks x B)  reduce P2 -> pick the largest Armijo-satisfying trial (or reject a
//                          non-descent direction: steepest descent next iteration) -> per element
//                          s, y into the history slot, x, g; partial dots of the new pair with
//                          every slot -> P3, and the NEXT direction's dots s_j.pg, y_j.pg, pg.pg
//                          (new pg, new pair in its slot) -> P1.  The last chunk of a model to
//                          finish (a device-scope counter: release fence + atomic, no spinning)
//                          finalizes the model: Gram rows of the new pair, rho, objective,
//                          convergence / failure flags.  A rejected step (no trial taken) changes
//                          neither x, g nor the history, so the P1 of the previous update stays
//                          exact.  Two launches per iteration between the evaluations, no
//                          separate dots / finalize pass.
// ---------------------------------------------------------------------------------------------
constexpr int QN_BLOCK = 256;
constexpr int QN_MAX_TRIALS = 4;
constexpr int QN_MAX_M = 10;
constexpr int NP1 = 2 * QN_MAX_M + 1;        // s_j.pg, y_j.pg, pg.pg
constexpr int NP2 = 3 * QN_MAX_TRIALS + 2;   // per trial: 0.5 l2 x^2, l1 |x|, pg.(xt - x); then pg.d, pg.pg
constexpr int NP3 = 5 + 3 * QN_MAX_M;        // s.y, s.s, y.y, x.x, pg.pg, then s.y_j, s_j.y, y.y_j


constexpr int QN_MAX_CHUNKS = 32;

// Block sum of fp32 per-lane partials, fp64 totals into the shared tot[NV], through an LDS transpose:
// every thread stores its NV partials, then thread 4 q + w adds value q over the 64 threads of
// segment w (four fp64 chains of 16, fixed order), and thread q adds the four segments in order.
// (Per-value wave reductions — 6 butterfly steps each, 56 values in the update pass — took 12-20k
// cycles with LDS shuffles or fp64 DPP, profiles/r5/lr_stamps.md.)  `sh` holds the [NV][4] segment
// sums; WIDE is kept for the call sites' signatures.
template <int NV, bool WIDE = false>
__device__ __forceinline__ void block_sum_f(const float (&p)[NV], double* sh, double* tot) {
  static_assert(QN_BLOCK == 256 && 4 * NV <= QN_BLOCK, "four 64-thread segments, one thread per (value, segment)");
  constexpr int TP = QN_BLOCK + 4;  // row pitch (16-byte rows)
  __shared__ __attribute__((aligned(16))) float tr[NV * TP];
  const int t = threadIdx.x;
#pragma unroll
  for (int q = 0; q < NV; ++q) tr[q * TP + t] = p[q];
  __syncthreads();
  if (t < 4 * NV) {
    const int q = t >> 2, w = t & 3;
    const float4* r = reinterpret_cast<const float4*>(tr + q * TP + 64 * w);
    double c0 = 0.0, c1 = 0.0, c2 = 0.0, c3 = 0.0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float4 v = r[i];
      c0 += (double)v.x;
      c1 += (double)v.y;
      c2 += (double)v.z;
      c3 += (double)v.w;
    }
    sh[q * 4 + w] = (c0 + c1) + (c2 + c3);
  }
  __syncthreads();
  if (t < NV) tot[t] = (sh[t * 4] + sh[t * 4 + 1]) + (sh[t * 4 + 2] + sh[t * 4 + 3]);
  __syncthreads();
}

// reduce_chunks_shared of two partial slabs at once (agent-scope loads, one round, one barrier): threads
// q < NA sum slab A into va, threads 64 + q (q < NB) slab B into vb, side by side in chunk order
template <int NA, int NB>
__device__ __forceinline__ void reduce_chunks2_shared(const double* PA, const double* PB, int nch, double* va,
                                                      double* vb, double* stage) {
  static_assert(NA <= 64 && NB <= 64, "one wave per slab");
  for (int i = threadIdx.x; i < nch * (NA + NB); i += QN_BLOCK)
    stage[i] = i < nch * NA ? __hip_atomic_load(PA + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                            : __hip_atomic_load(PB + (i - nch * NA), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const int t = threadIdx.x;
  if (t < NA) {
    double acc = 0.0;
#pragma unroll 8
    for (int c = 0; c < nch; ++c) acc += stage[c * NA + t];
    va[t] = acc;
  } else if (t >= 64 && t < 64 + NB) {
    const double* sb = stage + nch * NA;
    double acc = 0.0;
#pragma unroll 8
    for (int c = 0; c < nch; ++c) acc += sb[c * NB + (t - 64)];
    vb[t - 64] = acc;
  }
}

// block_sum_f with the totals handed to out(q, total) by thread q < NV (all in wave 0 for NV <= 64: the
// caller's stores then need no barrier before wave 0 publishes them) instead of a shared array + barrier
template <int NV, typename Out>
__device__ __forceinline__ void block_sum_out(const float (&p)[NV], double* sh, Out&& out) {
  static_assert(QN_BLOCK == 256 && 4 * NV <= QN_BLOCK && NV <= 64, "four 64-thread segments; totals in wave 0");
  constexpr int TP = QN_BLOCK + 4;
  __shared__ __attribute__((aligned(16))) float tr[NV * TP];
  const int t = threadIdx.x;
#pragma unroll
  for (int q = 0; q < NV; ++q) tr[q * TP + t] = p[q];
  __syncthreads();
  if (t < 4 * NV) {
    const int q = t >> 2, w = t & 3;
    const float4* r = reinterpret_cast<const float4*>(tr + q * TP + 64 * w);
    double c0 = 0.0, c1 = 0.0, c2 = 0.0, c3 = 0.0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float4 v = r[i];
      c0 += (double)v.x;
      c1 += (double)v.y;
      c2 += (double)v.z;
      c3 += (double)v.w;
    }
    sh[q * 4 + w] = (c0 + c1) + (c2 + c3);
  }
  __syncthreads();
  if (t < NV) out(t, (sh[t * 4] + sh[t * 4 + 1]) + (sh[t * 4 + 2] + sh[t * 4 + 3]));
}

// Chunk sums in chunk order (fixed: bitwise reproducible) into the shared vs[NV]: every lane of the
// block loads part of the nch x NV partials into LDS (ONE round of independent loads, not a chain of
// nch / 8 dependent rounds per lane), then one lane per value q adds them in chunk order.  AGENT:
// agent-scope (write-through, cross-XCD coherent) loads, for partials stored earlier in the same
// launch.  The caller synchronizes before reading vs.
template <int NV, bool AGENT = false>
__device__ __forceinline__ void reduce_chunks_shared(const double* P, int nch, double* vs, double* stage) {
  for (int i = threadIdx.x; i < nch * NV; i += QN_BLOCK)
    stage[i] = AGENT ? __hip_atomic_load(P + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : P[i];
  __syncthreads();
  const int q = threadIdx.x;
  if (q < NV) {
    double t = 0.0;
#pragma unroll 8
    for (int c = 0; c < nch; ++c) t += stage[c * NV + q];  // LDS reads pipelined, adds in chunk order
    vs[q] = t;
  }
}


// The phase-2 chunk partials P3 cross workgroups inside the kernel (the model's last chunk reduces
// them): agent-scope stores / loads (write-through, coherent across the XCDs' L2s) instead of a
// device-scope release fence, whose L2 write-back of every dirty line cost more than the pass it saves

__device__ __forceinline__ float pseudo_grad(float x, float g, float l1) {
  if (l1 == 0.f) return g;
  const float gp = g + l1, gm = g - l1;
  if (x > 0.f) return gp;
  if (x < 0.f) return gm;
  return gp < 0.f ? gp : (gm > 0.f ? gm : 0.f);
}

__device__ __forceinline__ float sgnf(float v) { return v > 0.f ? 1.f : (v < 0.f ? -1.f : 0.f); }

// phase 2 of model b, completed by one lane of its last chunk (p: >= 0 accepted trial, -1 no
// trial accepted / inactive, -2 non-descent direction; regp: the regularization of trial p, from the
// block's own P2 sums — reg[] is stored by chunk 0 of this launch, not visible to the last chunk);
// the objective goes to hist row fin_it
// The per-model scalars phase 2 reads (objective, trial losses, step scale, flags, counters) are
// loaded at the start of the launch, uniform (scalar loads): their round trip overlaps the P2
// partials' instead of following the pick and again the last-chunk count.
struct QnScalars {
  double F0, L0, L1, L2, L3;  // objective at x, data loss of trials 0..3
  float step_scale;
  int steep, active, fails, iters;
};

__device__ __forceinline__ double trial_loss(const QnScalars& q, int t) {
  return t == 0 ? q.L0 : t == 1 ? q.L1 : t == 2 ? q.L2 : q.L3;
}

__device__ __forceinline__ QnScalars qn_load_scalars(const QnArgs& a, int b) {
  const double* L = a.loss + b * a.T;
  return QnScalars{a.fobj[b], L[0], a.T > 1 ? L[1] : 0.0, a.T > 2 ? L[2] : 0.0, a.T > 3 ? L[3] : 0.0,
                   a.step_scale[b], a.steep[b], a.active[b], a.fails[b], a.iters[b]};
}

// Run by the first three waves (t = threadIdx.x): thread j < m writes row / column j of the history Gram
// matrices, thread 64 (wave 1) the curvature test, thread 128 (wave 2) the objective and the flags, so
// the three parts run side by side instead of as one lane's serial ~35 stores + fp64 square roots and
// divisions (~5k cycles of the update kernel's last chunk, profiles/r5/lr_kernel_medians.md)
__device__ __forceinline__ void qn_finalize(const QnArgs& a, int b, int p, double regp, const QnScalars& q,
                                            const double* v, int t) {
  const int mm = a.m;
  if (a.init) {
    if (t == 128) {
      const double F = q.L0 + regp;
      a.fobj[b] = F;
      if (a.hist) a.hist[b] = F;
    }
    return;
  }
  const int h = a.head;
  double Fout = q.F0;
  if (p >= 0) {  // v: the P3 chunk sums (LDS)
    double* SY = a.SY + (int64_t)b * mm * mm;
    double* YY = a.YY + (int64_t)b * mm * mm;
    if (t < mm) {
      const int j = t;
      if (j == h) {
        SY[h * mm + h] = v[0];
        YY[h * mm + h] = v[2];
      } else {
        SY[h * mm + j] = v[5 + 3 * j];
        SY[j * mm + h] = v[6 + 3 * j];
        YY[h * mm + j] = YY[j * mm + h] = v[7 + 3 * j];
      }
    }
    if (t == 64) {
      const bool good = v[0] > 1e-10 * fmax(sqrt(v[1]) * sqrt(v[2]), 1e-300);
      a.rho[h * a.B + b] = good ? 1.0 / v[0] : 0.0;
    }
    if (t == 128) {
      const double Fn = trial_loss(q, p) + regp;
      const double F0 = q.F0;
      const double rel = fabs(F0 - Fn) / fmax(fmax(fabs(F0), fabs(Fn)), 1.0);
      a.fobj[b] = Fout = Fn;
      a.iters[b] = q.iters + 1;
      a.fails[b] = 0;
      a.steep[b] = 0;
      a.step_scale[b] = 1.0f;
      if (rel < a.tol || sqrt(v[4]) <= a.tol * fmax(sqrt(v[3]), 1.0)) a.active[b] = 0;
    }
  } else if (t == 128) {
    if (p == -2) {  // the recursion produced no descent direction: steepest descent next
      a.rho[h * a.B + b] = 0.0;
      a.steep[b] = 1;
    } else {
      a.rho[h * a.B + b] = 0.0;
      if (q.active) {
        a.step_scale[b] = q.step_scale * (1.0f / 16.0f);
        a.fails[b] = q.fails + 1;
        if (q.fails + 1 >= 2) a.active[b] = 0;
      }
    }
  }
  if (t == 128 && a.hist) a.hist[(int64_t)a.fin_it * a.B + b] = Fout;
}

// One parameter element's operands for phase 1 (x, g, L1 / L2 weights, the W_eff scale and the
// m history values), loaded at a clamped (always valid) index so the loads are unconditional: the
// kernel keeps the next element's loads in flight while it computes the current one, and the
// first element's while lane 0 runs the recursion.
struct DirElem {
  float x, g, l1, hl2, wsc;
  float s[QN_MAX_M], y[QN_MAX_M];
};

__device__ __forceinline__ DirElem dir_load(const QnArgs& a, int b, int k, int col) {
  const int64_t D = a.D, sstride = (int64_t)a.B * D;
  const int Fp1 = a.F + 1;
  const int e = k * Fp1 + col;
  DirElem v;
  v.x = a.x[b * D + e];
  v.g = a.g[b * D + e];
  v.l1 = a.l1 ? a.l1[b * D + e] : 0.f;
  v.hl2 = 0.5f * a.l2[b * D + e];
  const float isd = a.inv_std[(int64_t)b * a.F + min(col, a.F - 1)];
  v.wsc = a.pmask[b * D + e] * (col < a.F ? isd : 1.f);
#pragma unroll
  for (int j = 0; j < QN_MAX_M; ++j) {
    // slots not filled yet (j >= filled; the ring fills 0, 1, ... before it wraps) re-read slot 0: the
    // same lines, so they cost no HBM traffic (the batched CV direction is bandwidth-bound while the
    // history fills), and their coefficients cS / cY are 0; slots >= m are never valid either
    const int jj = j < a.filled ? j : 0;
    v.s[j] = a.S[jj * sstride + b * D + e];
    v.y[j] = a.Y[jj * sstride + b * D + e];
  }
  return v;
}

// phase 1
template <int KP, bool FULLM, bool STAMP = false>
__device__ __forceinline__ void qn_direction_body(const QnArgs& a, int c, int b, uint64_t* st = nullptr,
                                                  float* wt = nullptr) {
  HAR_LR_STAMP(0)
  __shared__ double sh[4 * NP2];
  __shared__ float cS[QN_MAX_M], cY[QN_MAX_M];
  __shared__ float gam;
  const int D = (int)a.D;
  const int mm = a.m;
  const int Fp1 = a.F + 1;
  const bool steep = a.steep[b] != 0;
  // the recursion's operands live in LDS: the P1 chunk sums (reduced by NP1 lanes), the Gram
  // matrices, rho and the coefficient vectors (per-lane arrays indexed by slot would spill to scratch)
  __shared__ double p1v[NP1], SY[QN_MAX_M * QN_MAX_M], YY[QN_MAX_M * QN_MAX_M], rho_s[QN_MAX_M];
  const bool rec = !a.init && !steep;  // block-uniform
  // chunk c = the columns [cc0, cc0 + ccn) x every class k (element e = k (F+1) + col), walked k-major
  // (i = k ccn + j: consecutive lanes, consecutive columns -> coalesced loads and xtrial stores); with
  // `wt` (an LDS tile [T][KP][ccs]) the chunk's W_eff rows are assembled on chip and stored as whole
  // 32-byte rows — written per element they were 4-byte stores 32 bytes apart, the batched CV
  // direction's bound (profiles/r5/lr_grad_blocks.md)
  const int ccs = (Fp1 + a.nch - 1) / a.nch, cc0 = c * ccs, ccn = max(0, min(Fp1, cc0 + ccs) - cc0);
  const int nel = ccn * a.K;
  const uint32_t cmag = 0xffffffffu / (uint32_t)max(ccn, 1) + 1u;  // i / ccn = umulhi(i, cmag) (i ccn < 2^32)
  const int e0 = threadIdx.x, e1 = nel;
  auto kof = [&](int i) { return (int)__umulhi((uint32_t)i, cmag); };
  // each thread's first three elements in flight during the prologue + recursion (a refill three ahead),
  // issued AFTER the recursion's operand loads (Gram, rho, P1 totals): a counted wait for those then
  // does not also wait for the 75 element loads behind them
  auto dclamp = [&](int e) { return max(min(e, e1 - 1), 0); };
  auto dload = [&](int i) {
    const int k = ccn ? kof(i) : 0;
    return dir_load(a, b, k, cc0 + (ccn ? i - k * ccn : 0));
  };
  const int i = threadIdx.x;
  double syv = 0.0, yyv = 0.0, rhv = 0.0, p1x = 0.0;
  if (rec) {
    // the Gram matrices and rho (one element per lane: m^2 <= 100 < QN_BLOCK)
    if (i < mm * mm) {
      syv = a.SY[(int64_t)b * mm * mm + i];
      yyv = a.YY[(int64_t)b * mm * mm + i];
    }
    if (i < mm) rhv = a.rho[i * a.B + b];
    if (i < NP1) p1x = a.P1[(int64_t)b * a.nch * NP1 + i];  // the totals (the last update's last chunk)
  }
  __builtin_amdgcn_sched_barrier(0);
  DirElem d0 = dload(dclamp(e0)), d1 = dload(dclamp(e0 + QN_BLOCK)), d2 = dload(dclamp(e0 + 2 * QN_BLOCK));
  __builtin_amdgcn_sched_barrier(0);
  if (rec) {
    // every entry of the [QN_MAX_M]^2 images written (zeros past m^2): the recursion below reads whole
    // rows / columns unconditionally, its products with the zero coefficients of unused slots exact
    if (i < NP1) p1v[i] = p1x;
    if (i < QN_MAX_M * QN_MAX_M) {
      SY[i] = syv;
      YY[i] = yyv;
    }
    if (i < QN_MAX_M) rho_s[i] = rhv;
    __syncthreads();
  }
  HAR_LR_STAMP(1)
  if (threadIdx.x < 64) {
    // the two-loop recursion on coefficients, lane L of each 16-lane row of wave 0 owning STEP L (slot
    // j_L = head - 1 - L mod m): both loops are triangular recurrences, so each lane keeps the running dot
    // product of its own step — step i's coefficient is computed on lane i, broadcast by readlane, and
    // every lane adds its product with its Gram element (one fp64 fma).  A step is then readlane + fma +
    // the next lane's update instead of a 10-term product and a 4-stage fp64 DPP row sum (recursion
    // 6.9k -> see profiles/r5/lr_grad_blocks.md).  The loop-2 products with the final q (y_j . q for
    // every j) do not depend on loop 2 and run as independent per-lane dots.  Fixed order on every run.
    const int L = threadIdx.x & 15;
    if (threadIdx.x < QN_MAX_M) cS[threadIdx.x] = cY[threadIdx.x] = 0.f;
    float gamma = 0.f;
    if (rec) {
      auto readlane_d = [](double v, int lane) {
        const uint64_t u = __builtin_bit_cast(uint64_t, v);
        return __builtin_bit_cast(double, ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(u >> 32), lane) << 32) |
                                              (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, lane));
      };
      // slot index j_i = head - 1 - i mod m by a conditional add (an integer modulo by the runtime m is a
      // ~40-instruction division); steps i >= filled may run below slot 0: any slot, unused
      auto slot = [&](int i) {
        int j = a.head - 1 - i;
        j = j < 0 ? j + mm : j;
        return j < 0 ? 0 : j;
      };
      const int jL = slot(L);
      // every Gram element this lane's step needs, read before the dependent steps
      double m1[QN_MAX_M], m2[QN_MAX_M], m3[QN_MAX_M];
#pragma unroll
      for (int i = 0; i < QN_MAX_M; ++i) {
        const int ji = slot(i);
        m1[i] = SY[jL * mm + ji];  // s_jL . y_ji
        m2[i] = YY[jL * mm + ji];  // y_jL . y_ji
        m3[i] = SY[ji * mm + jL];  // s_ji . y_jL
      }
      const double paL = p1v[jL], pbL = p1v[QN_MAX_M + jL], rhL = rho_s[jL];
      // loop 1, newest -> oldest: al_i = rho_i s_i . q, q = pg - sum al_l y_l (a rejected pair: rho = 0, al 0)
      double acc = 0.0, alL = 0.0, als[QN_MAX_M];
#pragma unroll
      for (int i = 0; i < QN_MAX_M; ++i) {
        als[i] = 0.0;
        if (i < a.filled) {
          const double ali = readlane_d(rhL == 0.0 ? 0.0 : rhL * (paL + acc), i);
          als[i] = ali;
          alL = L == i ? ali : alL;
          acc = fma(-ali, m1[i], acc);
        }
      }
      double gm;
      if (a.filled == 0) {
        gm = 1.0 / fmax(sqrt(p1v[2 * QN_MAX_M]), 1e-12);
      } else {
        const int n = slot(0);
        const double yy = YY[n * mm + n];
        gm = (rho_s[n] > 0.0 && yy > 0.0) ? SY[n * mm + n] / yy : 1.0;
      }
      // y_jL . q with the final q
      double yq = pbL;
#pragma unroll
      for (int l = 0; l < QN_MAX_M; ++l)
        if (l < a.filled) yq = fma(-als[l], m2[l], yq);
      // loop 2, oldest -> newest: w_i = al_i - rho_i y_i . r, r = gm q + sum w_l s_l
      double acc2 = 0.0, wL = 0.0;
#pragma unroll
      for (int i = QN_MAX_M - 1; i >= 0; --i) {
        if (i < a.filled) {
          const double wi = readlane_d(rhL == 0.0 ? 0.0 : als[i] - rhL * fma(gm, yq, acc2), i);
          wL = L == i ? wi : wL;
          acc2 = fma(wi, m3[i], acc2);
        }
      }
      if (threadIdx.x < 16 && L < a.filled) {
        cY[jL] = (float)(gm * -alL);
        cS[jL] = (float)wL;
      }
      gamma = (float)gm;
    }
    if (threadIdx.x == 0) {
      gam = gamma;
    }
  }
  __syncthreads();
  HAR_LR_STAMP(2)
  const bool l1on = a.l1 != nullptr;
  const bool active = a.active[b] != 0;
  const int T = a.init ? 1 : a.T;
  const float s0 = a.init ? 0.f : a.step_scale[b];
  const float gamma = gam;
  float r[NP2];
#pragma unroll
  for (int t = 0; t < NP2; ++t) r[t] = 0.f;
  auto proc = [&](const DirElem& cur, int i) __attribute__((always_inline)) {
    const int k = kof(i), jc = i - k * ccn, col = cc0 + jc, e = k * Fp1 + col;
    const float xe = cur.x;
    const float l1e = cur.l1;
    const float pg = a.init ? 0.f : pseudo_grad(xe, cur.g, l1e);
    float d = 0.f;
    if (!a.init) {
      if (steep) {
        d = -pg;
      } else {
        float acc = gamma * pg;
#pragma unroll
        for (int j = 0; j < QN_MAX_M; ++j) {
          if (FULLM || j < mm) {
            acc = fmaf(cY[j], cur.y[j], acc);
            acc = fmaf(cS[j], cur.s[j], acc);
          }
        }
        d = -acc;
        if (l1on && d * pg >= 0.f) d = 0.f;  // OWL-QN: keep the direction in pg's orthant
      }
    }
    r[3 * QN_MAX_TRIALS] = fmaf(pg, d, r[3 * QN_MAX_TRIALS]);
    r[3 * QN_MAX_TRIALS + 1] = fmaf(pg, pg, r[3 * QN_MAX_TRIALS + 1]);
    const float xi = xe != 0.f ? sgnf(xe) : sgnf(-pg);
    const float hl2 = cur.hl2;
    const float wsc = cur.wsc;
#pragma unroll
    for (int t = 0; t < QN_MAX_TRIALS; ++t) {
      if (t < T) {
        float xn = xe + s0 * ldexpf(1.f, -t) * d;
        if (l1on && !a.init) {  // stay in the orthant of x (or of -pg where x == 0)
          if (sgnf(xn) != xi) xn = 0.f;
          r[3 * t + 2] = fmaf(pg, xn - xe, r[3 * t + 2]);
        }
        if (!active) xn = xe;
        const int bt = b * a.T + t;
        a.xtrial[(int64_t)bt * D + e] = xn;
        r[3 * t] = fmaf(hl2, xn * xn, r[3 * t]);
        r[3 * t + 1] = fmaf(l1e, fabsf(xn), r[3 * t + 1]);
        if (wt)
          wt[(t * KP + k) * ccs + jc] = xn * wsc;
        else
          a.weff[((int64_t)bt * Fp1 + col) * KP + k] = xn * wsc;
      }
    }
  };
  for (int e = e0; e < e1; e += 3 * QN_BLOCK) {
    proc(d0, e);
    if (e + 3 * QN_BLOCK < e1) d0 = dload(e + 3 * QN_BLOCK);
    if (e + QN_BLOCK < e1) {
      proc(d1, e + QN_BLOCK);
      if (e + 4 * QN_BLOCK < e1) d1 = dload(e + 4 * QN_BLOCK);
    }
    if (e + 2 * QN_BLOCK < e1) {
      proc(d2, e + 2 * QN_BLOCK);
      if (e + 5 * QN_BLOCK < e1) d2 = dload(e + 5 * QN_BLOCK);
    }
  }
  if (wt) {  // the chunk's W_eff rows from the tile, 8 lanes per 32-byte row (classes >= K: zeros)
    __syncthreads();
    for (int t = 0; t < T; ++t) {
      float* wrow = a.weff + ((int64_t)(b * a.T + t) * Fp1 + cc0) * KP;
      for (int idx = threadIdx.x; idx < ccn * KP; idx += QN_BLOCK) {
        const int jc = idx / KP, k = idx % KP;
        wrow[idx] = k < a.K ? wt[(t * KP + k) * ccs + jc] : 0.f;
      }
    }
  }
  HAR_LR_STAMP(3)
  __shared__ double tot2[NP2];
  block_sum_f<NP2>(r, sh, tot2);
  HAR_LR_STAMP(4)
  if (threadIdx.x == 0) {
    double* P2 = a.P2 + ((int64_t)b * a.nch + c) * NP2;
#pragma unroll
    for (int q = 0; q < NP2; ++q) P2[q] = tot2[q];
  }
  HAR_LR_STAMP(5)
}

template <int KP, bool FULLM, bool STAMP = false>
__global__ __launch_bounds__(QN_BLOCK) void qn_direction_kernel(QnArgs a, uint64_t* st, int use_wt) {
  extern __shared__ float wtile[];
  qn_direction_body<KP, FULLM, STAMP>(a, blockIdx.x, blockIdx.y, st, use_wt ? wtile : nullptr);
}

// One parameter element's phase-2 operands that do not depend on the picked trial (x, g, L1 / L2
// weights, the history values), loaded at a clamped (valid) index: the first three elements of every
// thread go out at the start of the launch, under the P2 reduction and the pick, and a refill three
// elements ahead while the current ones are processed (the history stores of an element may alias the
// next element's loads for the compiler, so a plain loop waited out one round trip per element)
struct UpdElem {
  float x, g, l2, l1;
  float s[QN_MAX_M], y[QN_MAX_M];
};

template <bool FULLM>
__device__ __forceinline__ UpdElem upd_load(const QnArgs& a, int b, int e) {
  const int64_t D = a.D, sstride = (int64_t)a.B * D, o = (int64_t)b * D + e;
  UpdElem v;
  v.x = a.x[o];
  v.g = a.g[o];
  v.l2 = a.l2[o];
  v.l1 = a.l1 ? a.l1[o] : 0.f;
#pragma unroll
  for (int j = 0; j < QN_MAX_M; ++j) {
    v.s[j] = v.y[j] = 0.f;
    // FULLM also loads slot `head` (its OLD pair) and accumulates its P3 sums, which finalize never reads;
    // unfilled slots re-read slot 0 (cached lines; their dots are never read)
    if (!a.init && (FULLM || (j < a.m && j != a.head))) {
      const int jl = j < a.filled ? j : 0;
      v.s[j] = a.S[jl * sstride + o];
      v.y[j] = a.Y[jl * sstride + o];
    }
  }
  return v;
}

// phase 2
template <bool FULLM, bool WIDE, bool STAMP = false>
__device__ __forceinline__ void qn_update_body(const QnArgs& a, int c, int b, uint64_t* st = nullptr) {
  HAR_LR_STAMP(0)
  __shared__ double sh[4 * (NP3 + 2 * QN_MAX_M)];
  __shared__ double p2v[NP2];
  __shared__ double fin_v[NP3], p1t[NP1];
  __shared__ double stage[QN_MAX_CHUNKS * (NP3 + NP1)];
  __shared__ int pick, last;
  const int D = (int)a.D;
  const int mm = a.m;
  const QnScalars qs = qn_load_scalars(a, b);  // uniform (scalar) loads, in flight with the P2 partials
  const int csz = (D + a.nch - 1) / a.nch, e1 = min(D, (c + 1) * csz), eb = c * csz + (int)threadIdx.x;
  auto eclamp = [&](int e) { return max(min(e, e1 - 1), 0); };
  // the P2 partials (reduce_chunks_shared, its loads split out) BEFORE the element prefetch, so the
  // counted wait for them does not also wait for the element loads
  static_assert(QN_MAX_CHUNKS * NP2 <= 2 * QN_BLOCK, "two P2 partials per thread at most");
  const double* P2b = a.P2 + (int64_t)b * a.nch * NP2;
  const int n2 = a.nch * NP2, t2 = (int)threadIdx.x;
  const double p2a = t2 < n2 ? P2b[t2] : 0.0, p2b = t2 + QN_BLOCK < n2 ? P2b[t2 + QN_BLOCK] : 0.0;
  __builtin_amdgcn_sched_barrier(0);
  UpdElem u0 = upd_load<FULLM>(a, b, eclamp(eb));
  UpdElem u1 = upd_load<FULLM>(a, b, eclamp(eb + QN_BLOCK));
  UpdElem u2 = upd_load<FULLM>(a, b, eclamp(eb + 2 * QN_BLOCK));
  __builtin_amdgcn_sched_barrier(0);
  if (t2 < n2) stage[t2] = p2a;
  if (t2 + QN_BLOCK < n2) stage[t2 + QN_BLOCK] = p2b;
  __syncthreads();
  if (t2 < NP2) {
    double acc = 0.0;
#pragma unroll 8
    for (int cc = 0; cc < a.nch; ++cc) acc += stage[cc * NP2 + t2];  // chunk order
    p2v[t2] = acc;
  }
  __syncthreads();
  HAR_LR_STAMP(1)
  if (threadIdx.x == 0) {
    const bool steep = qs.steep != 0;
    const double dd = steep ? -p2v[3 * QN_MAX_TRIALS + 1] : p2v[3 * QN_MAX_TRIALS];
    const int T = a.init ? 1 : a.T;
    const float s0 = a.init ? 0.f : qs.step_scale;
    int p = -1;
    if (a.init) {
      p = 0;
    } else if (qs.active) {
      if (dd >= 0.0) {
        p = steep ? -1 : -2;
      } else {
#pragma unroll
        for (int t = 0; t < QN_MAX_TRIALS; ++t) {
          if (t < T && p < 0) {
            const double decr = a.l1 ? p2v[3 * t + 2] : (double)(s0 * ldexpf(1.f, -t)) * dd;
            const double Ft = trial_loss(qs, t) + p2v[3 * t] + p2v[3 * t + 1];
            if (isfinite(Ft) && Ft <= qs.F0 + a.c1 * decr) p = t;
          }
        }
      }
    }
    if (c == 0) {
      a.pick[b] = p;
      for (int t = 0; t < T; ++t) {
        a.reg[b * a.T + t] = p2v[3 * t] + p2v[3 * t + 1];
        a.decr[b * a.T + t] = a.l1 ? p2v[3 * t + 2] : (double)(s0 * ldexpf(1.f, -t)) * dd;
      }
    }
    pick = p;
  }
  __syncthreads();
  HAR_LR_STAMP(2)
  const int p = pick;
  if (p >= 0) {  // block-uniform
    const int64_t sstride = (int64_t)a.B * D;
    float* __restrict__ x = a.x + (int64_t)b * D;
    float* __restrict__ g = a.g + (int64_t)b * D;
    float* Sh = a.S + (int64_t)a.head * sstride + (int64_t)b * D;  // aliases slot `head` of the history
    float* Yh = a.Y + (int64_t)a.head * sstride + (int64_t)b * D;
    const int bt = b * a.T + p;
    const float* __restrict__ xt = a.xtrial + (int64_t)bt * D;
    const float* __restrict__ Gt = a.G + (int64_t)bt * D;
    float ps[NP3];
    float pd[2 * QN_MAX_M];  // the next direction's s_j.pg, y_j.pg (pg.pg is ps[4])
#pragma unroll
    for (int q = 0; q < NP3; ++q) ps[q] = 0.f;
#pragma unroll
    for (int q = 0; q < 2 * QN_MAX_M; ++q) pd[q] = 0.f;
    auto proc = [&](const UpdElem& u, int e, float xn, float gt) __attribute__((always_inline)) {
      const float gn = gt + u.l2 * xn;  // data gradient (masked, scaled) + L2 term
      const float pg = pseudo_grad(xn, gn, u.l1);
      if (!a.init) {
        const float se = xn - u.x, ye = gn - u.g;
        ps[0] = fmaf(se, ye, ps[0]);
        ps[1] = fmaf(se, se, ps[1]);
        ps[2] = fmaf(ye, ye, ps[2]);
#pragma unroll
        for (int j = 0; j < QN_MAX_M; ++j) {
          if (FULLM || j < mm) {
            const bool hj = j == a.head;
            const float sj = u.s[j], yj = u.y[j];
            if (FULLM || !hj) {
              ps[5 + 3 * j] = fmaf(se, yj, ps[5 + 3 * j]);
              ps[6 + 3 * j] = fmaf(sj, ye, ps[6 + 3 * j]);
              ps[7 + 3 * j] = fmaf(ye, yj, ps[7 + 3 * j]);
            }
            pd[j] = fmaf(hj ? se : sj, pg, pd[j]);
            pd[QN_MAX_M + j] = fmaf(hj ? ye : yj, pg, pd[QN_MAX_M + j]);
          }
        }
        Sh[e] = se;
        Yh[e] = ye;
      }
      ps[3] = fmaf(xn, xn, ps[3]);
      ps[4] = fmaf(pg, pg, ps[4]);
      x[e] = xn;
      g[e] = gn;
    };
    // three elements per thread and round: their trial values in one round of loads, then each processed
    // and its slot refilled three elements ahead (the element order and every sum's order are unchanged)
    for (int e = eb; e < e1; e += 3 * QN_BLOCK) {
      const int ea = eclamp(e), eb1 = eclamp(e + QN_BLOCK), eb2 = eclamp(e + 2 * QN_BLOCK);
      const float xn0 = xt[ea], gt0 = Gt[ea], xn1 = xt[eb1], gt1 = Gt[eb1], xn2 = xt[eb2], gt2 = Gt[eb2];
      proc(u0, e, xn0, gt0);
      if (e + 3 * QN_BLOCK < e1) u0 = upd_load<FULLM>(a, b, e + 3 * QN_BLOCK);
      if (e + QN_BLOCK < e1) {
        proc(u1, e + QN_BLOCK, xn1, gt1);
        if (e + 4 * QN_BLOCK < e1) u1 = upd_load<FULLM>(a, b, e + 4 * QN_BLOCK);
      }
      if (e + 2 * QN_BLOCK < e1) {
        proc(u2, e + 2 * QN_BLOCK, xn2, gt2);
        if (e + 5 * QN_BLOCK < e1) u2 = upd_load<FULLM>(a, b, e + 5 * QN_BLOCK);
      }
    }
    HAR_LR_STAMP(3)
    // the P3 and P1 partials in ONE block sum (one LDS transpose and barrier pair), each total stored
    // by its own wave-0 thread (P3: agent-scope, read by the model's last chunk in this launch)
    float pc[NP3 + 2 * QN_MAX_M];
#pragma unroll
    for (int q = 0; q < NP3; ++q) pc[q] = ps[q];
#pragma unroll
    for (int q = 0; q < 2 * QN_MAX_M; ++q) pc[NP3 + q] = pd[q];
    double* P3 = a.P3 + ((int64_t)b * a.nch + c) * NP3;
    double* P1 = a.P1 + ((int64_t)b * a.nch + c) * NP1;
    block_sum_out<NP3 + 2 * QN_MAX_M>(pc, sh, [&](int q, double v) {
      // (P1 too is reduced by the model's last chunk in this launch: agent-scope as well)
      if (q < NP3) __hip_atomic_store(P3 + q, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else __hip_atomic_store(P1 + (q - NP3), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (q == 4) __hip_atomic_store(P1 + 2 * QN_MAX_M, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // pg.pg
    });
  }
  // the last chunk of model b to get here finalizes the model.  Memory model: lane 0 publishes the
  // chunk's P3 / P1 partials with an agent-scope RELEASE fence before counting it (the stores are
  // complete and written back past this XCD's L2), and the block that counts last takes an agent-scope
  // ACQUIRE fence before reading any other chunk's partials (its own L2 / L1 copies invalidated), so
  // the handoff holds across the 8 XCDs without relying on the counter's relaxed ordering
  HAR_LR_STAMP(4)
  // every storing wave drains its partial-total stores, then the workgroup barrier orders them before
  // lane 0's release (the stores come from lanes 0-54 of wave 0, not from lane 0 alone); the wait after
  // the fence keeps the counter add behind the write-back (MI355X_MICROARCH: compiler hazard)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    last = __hip_atomic_fetch_add(a.done + b, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == a.nch - 1;
    if (last) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __syncthreads();
  HAR_LR_STAMP(5)
  if (!last) return;
  // the P3 sums (finalize) and the next direction's P1 sums, side by side; the P1 totals replace chunk
  // 0's partials (P1[b][0]), which the direction kernel then reads as they are — one load round instead
  // of every direction workgroup reducing the nch partials again (a rejected step writes no partials:
  // the totals of the last accepted one stay, as the history does)
  if (p >= 0) {
    double* P1b = a.P1 + (int64_t)b * a.nch * NP1;
    if (!a.init)
      reduce_chunks2_shared<NP3, NP1>(a.P3 + (int64_t)b * a.nch * NP3, P1b, a.nch, fin_v, p1t, stage);
    else
      reduce_chunks2_shared<0, NP1>(nullptr, P1b, a.nch, fin_v, p1t, stage);
    __syncthreads();
    if (threadIdx.x < NP1) P1b[threadIdx.x] = p1t[threadIdx.x];
  }
  __syncthreads();
  HAR_LR_STAMP(6)
  if (threadIdx.x <= 128) {
    qn_finalize(a, b, p, p >= 0 ? p2v[3 * p] + p2v[3 * p + 1] : 0.0, qs, fin_v, threadIdx.x);
    if (threadIdx.x == 0) __hip_atomic_store(a.done + b, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  HAR_LR_STAMP(7)
}

template <bool FULLM, bool WIDE, bool STAMP = false>
__global__ __launch_bounds__(QN_BLOCK) void qn_update_kernel(QnArgs a, uint64_t* st) {
  qn_update_body<FULLM, WIDE, STAMP>(a, blockIdx.x, blockIdx.y, st);
}

// ---------------------------------------------------------------------------------------------
// Persistent solve: the whole fit's launch sequence (logreg_solve_run in bind.cpp: init direction,
// evaluate, gradient, init update, then max_iter x [direction, evaluate, gradient, update]) as ONE
// cooperative launch.  Every phase runs the SAME body as its stand-alone kernel over virtual blocks
// (workgroup g takes blocks g, g + grid, ...), so the solve is bitwise the launch sequence's; a
// grid barrier replaces each kernel boundary.  Barrier: an agent-scope release fence (this XCD's
// L2 written back), one counter increment, a bounded spin on the counter, an agent-scope acquire
// fence (stale L1 / L2 lines dropped).  The spin is bounded and a timed-out barrier raises a flag
// that every later barrier checks first, so a fault can never leave waves spinning: the launcher
// reports the flag and the caller falls back to the launch sequence.
// ---------------------------------------------------------------------------------------------
struct SolvePersistArgs {
  QnArgs q;
  LogregEvalArgs evT, ev1;  // the init evaluation (trial 0 of every model) / the per-iteration one
  LogregGradArgs grT, gr1;
  int nT, n1, max_iter;
  uint32_t* sync;           // [0] barrier counter (zeroed by the launcher), [1] timeout flag
  uint32_t spin_limit;      // polls per barrier before the timeout flag is raised
};

constexpr uint32_t SOLVE_SPIN_LIMIT = 1u << 22;
// (tests shrink it to force the timeout path: har_logreg_set_spin_limit)
uint32_t g_solve_spin_limit = SOLVE_SPIN_LIMIT;

__device__ __forceinline__ void grid_barrier(uint32_t* sync, uint32_t& gen, uint32_t spin_limit) {
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __hip_atomic_fetch_add(sync, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t target = (gen + 1) * gridDim.x;
    uint32_t spins = 0;
    while (__hip_atomic_load(sync, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      if (__hip_atomic_load(sync + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) break;
      if (++spins > spin_limit) {
        __hip_atomic_store(sync + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  ++gen;
  __syncthreads();
}

template <int KP, int XLD, bool FULLM>
__global__ __launch_bounds__(QN_BLOCK) void logreg_solve_persistent_kernel(SolvePersistArgs p) {
  extern __shared__ float smem[];
  uint32_t gen = 0;
  const int G = gridDim.x, g0 = blockIdx.x;
  const int nqb = p.q.nch * p.q.B;
  const int tiles = (int)((p.ev1.N + EVAL_ROWS - 1) / EVAL_ROWS);
  const int cols = p.gr1.col_blk ? p.gr1.nblk : (p.gr1.F + 1 + 255) / 256;  // (grT: the same design)
  auto qn = [&](int phase, int head, int filled, int init, int fin_it) {
    QnArgs a = p.q;
    a.head = head;
    a.filled = filled;
    a.init = init;
    a.fin_it = fin_it;
    for (int v = g0; v < nqb; v += G) {
      if (phase == 1)
        qn_direction_body<KP, FULLM>(a, v % a.nch, v / a.nch);
      else
        qn_update_body<FULLM, FULLM>(a, v % a.nch, v / a.nch);
      __syncthreads();  // the next virtual block reuses the LDS
    }
    grid_barrier(p.sync, gen, p.spin_limit);
  };
  auto evaluate = [&](const LogregEvalArgs& ev, const LogregGradArgs& gr, int n) {
    for (int v = g0; v < tiles * n; v += G) {
      logreg_eval_body<KP, XLD>(ev, v % tiles, v / tiles, tiles, smem);
      __syncthreads();
    }
    grid_barrier(p.sync, gen, p.spin_limit);
    for (int v = g0; v < cols * n; v += G) {
      logreg_grad_body<KP>(gr, v % cols, v / cols);
      __syncthreads();
    }
    grid_barrier(p.sync, gen, p.spin_limit);
  };
  qn(1, 0, 0, 1, 0);
  evaluate(p.evT, p.grT, p.nT);
  qn(2, 0, 0, 1, 0);
  const int mm = p.q.m;
  int head = 0, filled = 0;
  for (int it = 0; it < p.max_iter; ++it) {
    qn(1, head, filled, 0, 0);
    evaluate(p.ev1, p.gr1, p.n1);
    qn(2, head, filled, 0, it + 1);
    head = (head + 1) % mm;
    filled = filled + 1 < mm ? filled + 1 : mm;
  }
}

}  // namespace

extern "C" int har_logreg_eval(const LogregEvalArgs* args, int KP, int n_models, hipStream_t s) {
  const LogregEvalArgs& a = *args;
  if (a.Fd < 0 || a.K < 1 || a.K > KP || (KP != 8 && KP != 16) || a.T < 1 ||
      a.tstride < 1 || (a.mode == 0 && a.slab == nullptr) || (a.C > 0 && a.cat == nullptr))
    return -2;
  if (a.N == 0 || n_models == 0) return 0;
  const int tiles = (int)((a.N + EVAL_ROWS - 1) / EVAL_ROWS);
  static const bool mf_on = [] {
    const char* e = std::getenv("HAR_LR_EVAL_MFMA");
    return !e || std::atoi(e) != 0;
  }();
  static const int mfn_mode = [] {  // narrow designs on the MFMA kernel: 1 always, 0 never, -1 small launches
    const char* e = std::getenv("HAR_LR_EVAL_MFN");
    return e ? std::atoi(e) : 1;
  }();
  const bool narrow = eval_xld(a.Fd) == EVAL_XLD_NARROW;
  const bool mf = mf_on && (!narrow || mfn_mode == 1 || (mfn_mode < 0 && (int64_t)tiles * n_models <= 256));
  const int xld = mf ? (narrow ? EVAL_XLD_MFN : EVAL_XLD_MF) : eval_xld(a.Fd);
  const size_t lds = sizeof(float) * (EVAL_DCH * KP + EVAL_ROWS * xld + EVAL_ROWS * KP + EVAL_ROWS / 64 +
                                      (mf ? 4 * EVAL_DCH * KP : 0));
  dim3 grid(tiles, n_models);
  if (mf && narrow && KP == 8)
    if (g_lr_stamps)
      logreg_eval_kernel<8, EVAL_XLD_MFN, true><<<grid, EVAL_ROWS, lds, s>>>(a, g_lr_stamps);
    else
      logreg_eval_kernel<8, EVAL_XLD_MFN><<<grid, EVAL_ROWS, lds, s>>>(a, nullptr);
  else if (mf && narrow)
    logreg_eval_kernel<16, EVAL_XLD_MFN><<<grid, EVAL_ROWS, lds, s>>>(a, nullptr);
  else if (mf && KP == 8)
    logreg_eval_kernel<8, EVAL_XLD_MF><<<grid, EVAL_ROWS, lds, s>>>(a, nullptr);
  else if (mf)
    logreg_eval_kernel<16, EVAL_XLD_MF><<<grid, EVAL_ROWS, lds, s>>>(a, nullptr);
  else if (KP == 8 && narrow)
    if (g_lr_stamps)
      logreg_eval_kernel<8, EVAL_XLD_NARROW, true><<<grid, EVAL_ROWS, lds, s>>>(a, g_lr_stamps);
    else
      logreg_eval_kernel<8, EVAL_XLD_NARROW><<<grid, EVAL_ROWS, lds, s>>>(a, nullptr);
  else if (KP == 8)
    logreg_eval_kernel<8, EVAL_DCH + 1><<<grid, EVAL_ROWS, lds, s>>>(a, nullptr);
  else if (narrow)
    logreg_eval_kernel<16, EVAL_XLD_NARROW><<<grid, EVAL_ROWS, lds, s>>>(a, nullptr);
  else
    logreg_eval_kernel<16, EVAL_DCH + 1><<<grid, EVAL_ROWS, lds, s>>>(a, nullptr);
  HAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int har_logreg_eval_tiles(int64_t n) { return (int)((n + EVAL_ROWS - 1) / EVAL_ROWS); }

extern "C" int har_logreg_grad(const LogregGradArgs* args, int KP, int n_models, hipStream_t s) {
  const LogregGradArgs& a = *args;
  if (a.K < 1 || a.K > KP || (KP != 8 && KP != 16) || a.T < 1 || a.tstride < 1 || a.SL < 1 ||
      a.col_slice == nullptr || a.csc_off == nullptr || (a.loss == nullptr && a.loss_fx == nullptr))
    return -2;
  if (n_models == 0) return 0;
  if (a.col_blk && (a.nblk < 1 || a.srow == nullptr)) return -2;
  // opt-in (HAR_LR_GRAD_TB=4): four trial models per workgroup for large launches of consecutive trials
  // of one spec — measured SLOWER for the batched CrossValidator (grad 54.8 vs 35.6 us per launch, LR-CV
  // 4.8-5.3 vs 4.1-4.5 ms: a quarter of the workgroups, each with 4x the gathers in flight per lane,
  // profiles/r5/lr_grad_blocks.md)
  static const int tb_env = [] {
    const char* e = std::getenv("HAR_LR_GRAD_TB");
    return e ? std::atoi(e) : 1;
  }();
  const bool tb4 = tb_env == 4 && KP == 8 && a.T == 4 && a.tstride == 1 && a.model0 % 4 == 0 && n_models % 4 == 0 &&
                   n_models >= 64;
  if (tb4) {
    dim3 g4(a.col_blk ? a.nblk : (a.F + 1 + 255) / 256, n_models / 4);
    logreg_grad_kernel<8, false, 4><<<g4, 256, 0, s>>>(a, nullptr);
    HAR_CHECK_LAUNCH();
    return 0;
  }
  dim3 grid(a.col_blk ? a.nblk : (a.F + 1 + 255) / 256, n_models);
  static const int wpe_env = [] {
    const char* e = std::getenv("HAR_LR_GRAD_WPE");
    return e ? std::atoi(e) : 0;
  }();
  if (KP == 8 && wpe_env == 5 && (int64_t)grid.x * grid.y >= 1024 && !g_lr_stamps_grd) {
    logreg_grad_kernel_w5<8><<<grid, 256, 0, s>>>(a, nullptr);
    HAR_CHECK_LAUNCH();
    return 0;
  }
  if (KP == 8)
    if (g_lr_stamps_grd)
      logreg_grad_kernel<8, true><<<grid, 256, 0, s>>>(a, g_lr_stamps_grd);
    else
      logreg_grad_kernel<8><<<grid, 256, 0, s>>>(a, nullptr);
  else
    logreg_grad_kernel<16><<<grid, 256, 0, s>>>(a, nullptr);
  HAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int har_logreg_col_slices(const int32_t* csc_off, int F, int SL, int32_t* col_slice, hipStream_t s) {
  if (F < 0 || SL < 1) return -2;
  logreg_col_slices_kernel<<<1, 1024, 0, s>>>(csc_off, F + 1, SL, col_slice);
  HAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int har_logreg_loss_decode(const float* fx, double* loss, int n, hipStream_t s) {
  if (n <= 0) return n < 0 ? -2 : 0;
  logreg_loss_decode_kernel<<<(n + 255) / 256, 256, 0, s>>>(fx, loss, n);
  HAR_CHECK_LAUNCH();
  return 0;
}

// Chunks per model: at most HAR_QN_WORKGROUPS (default 512) workgroups over the B models of a
// solve and at most QN_MAX_CHUNKS per model, at least 256 elements per chunk.  Measured (rocprofv3,
// WISDM): a 54-model CrossValidator batch at 9 chunks per model beats 14 and 19 (update 42 / 50 /
// 59 us, direction 68 / 66 / 87 us), and a single fit at 32 chunks beats 64 (the last-chunk
// finalize and the chunk reductions grow with the chunk count).
extern "C" int har_qn_chunks(int64_t D, int B) {
  static const int64_t budget = [] {
    const char* e = std::getenv("HAR_QN_WORKGROUPS");
    const long v = e ? std::atol(e) : 512;
    return (int64_t)(v > 0 ? v : 512);
  }();
  const int64_t by_b = budget / std::max(B, 1), by_d = (D + 255) / 256;
  return (int)std::max<int64_t>(1, std::min<int64_t>(QN_MAX_CHUNKS, std::min(by_b, by_d)));
}

// Host-side validation of one evaluation's arguments (the checks of har_logreg_eval / har_logreg_grad).
static bool eval_args_ok(const LogregEvalArgs& a, const LogregGradArgs& g, int KP, int n) {
  return a.Fd >= 0 && a.K >= 1 && a.K <= KP && a.T >= 1 && a.tstride >= 1 && a.slab != nullptr &&
         (a.C == 0 || a.cat != nullptr) && a.mode == 0 && g.K == a.K && g.T == a.T && g.SL >= 1 &&
         g.col_slice != nullptr && g.csc_off != nullptr && g.loss != nullptr && g.loss_fx == nullptr &&
         g.N == a.N && g.F == a.F && g.Fd == a.Fd && g.tstride == a.tstride && g.model0 == a.model0 &&
         g.ntiles == (int)((a.N + EVAL_ROWS - 1) / EVAL_ROWS) && (g.col_blk == nullptr || (g.nblk >= 1 && g.srow != nullptr)) && n >= 1 && a.N > 0 && (a.C == 0 || a.R != nullptr);
}

// The whole solve as one cooperative launch (logreg_solve_persistent_kernel).  Returns 0 when it ran
// (the caller then checks the timeout flag sync[1] with its results), -4 when this configuration
// has no persistent instantiation (m != QN_MAX_M) or the grid cannot be co-resident (the caller uses
// the launch sequence), -2 on invalid arguments.
extern "C" int har_logreg_solve_persistent(const QnArgs* q, const LogregEvalArgs* evT, const LogregGradArgs* grT,
                                           int nT, const LogregEvalArgs* ev1, const LogregGradArgs* gr1, int n1,
                                           int KP, int max_iter, uint32_t* sync, int max_grid, hipStream_t s) {
  const QnArgs& a = *q;
  if ((KP != 8 && KP != 16) || a.K > KP || a.m < 1 || a.m > QN_MAX_M || a.T < 1 || a.T > QN_MAX_TRIALS ||
      a.D != (int64_t)a.K * (a.F + 1) || a.D >= (1LL << 31) || a.nch != har_qn_chunks(a.D, a.B) || a.B < 1 ||
      a.done == nullptr || sync == nullptr || max_iter < 0 || !eval_args_ok(*evT, *grT, KP, nT) ||
      !eval_args_ok(*ev1, *gr1, KP, n1) || grT->col_blk != gr1->col_blk || grT->nblk != gr1->nblk || evT->N != ev1->N || evT->Fd != ev1->Fd || ev1->F != a.F ||
      ev1->K != a.K || n1 != a.B * a.T || nT != a.B || ev1->tstride != 1 || evT->tstride != a.T)
    return -2;
  if (a.m != QN_MAX_M) return -4;
  SolvePersistArgs p{*q, *evT, *ev1, *grT, *gr1, nT, n1, max_iter, sync, g_solve_spin_limit};
  p.q.head = p.q.filled = p.q.init = p.q.fin_it = 0;
  static const bool mf_on = [] {
    const char* e = std::getenv("HAR_LR_EVAL_MFMA");
    return !e || std::atoi(e) != 0;
  }();
  static const int mfn_mode = [] {
    const char* e = std::getenv("HAR_LR_EVAL_MFN");
    return e ? std::atoi(e) : 1;
  }();
  const bool narrow = eval_xld(ev1->Fd) == EVAL_XLD_NARROW;
  const bool mf = mf_on && (!narrow || mfn_mode == 1);
  const int xld = mf ? (narrow ? EVAL_XLD_MFN : EVAL_XLD_MF) : eval_xld(ev1->Fd);
  const size_t lds = sizeof(float) * (EVAL_DCH * KP + EVAL_ROWS * xld + EVAL_ROWS * KP + EVAL_ROWS / 64 +
                                      (mf ? 4 * EVAL_DCH * KP : 0));
  const void* fn;
  if (KP == 8)
    fn = mf && narrow ? (const void*)logreg_solve_persistent_kernel<8, EVAL_XLD_MFN, true>
       : mf ? (const void*)logreg_solve_persistent_kernel<8, EVAL_XLD_MF, true>
            : narrow ? (const void*)logreg_solve_persistent_kernel<8, EVAL_XLD_NARROW, true>
                     : (const void*)logreg_solve_persistent_kernel<8, EVAL_DCH + 1, true>;
  else
    fn = mf && narrow ? (const void*)logreg_solve_persistent_kernel<16, EVAL_XLD_MFN, true>
       : mf ? (const void*)logreg_solve_persistent_kernel<16, EVAL_XLD_MF, true>
            : narrow ? (const void*)logreg_solve_persistent_kernel<16, EVAL_XLD_NARROW, true>
                     : (const void*)logreg_solve_persistent_kernel<16, EVAL_DCH + 1, true>;
  // grid: every phase's virtual blocks once if they fit co-resident, else as many as are
  int dev = 0, cus = 0, per_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, QN_BLOCK, lds) != hipSuccess || per_cu < 1)
    return -4;
  const int tiles = (int)((ev1->N + EVAL_ROWS - 1) / EVAL_ROWS), cols = gr1->col_blk ? gr1->nblk : (a.F + 1 + 255) / 256;
  const int64_t want = std::max<int64_t>({(int64_t)a.nch * a.B, (int64_t)tiles * n1, (int64_t)cols * n1});
  if (max_grid < 0 && want > (int64_t)per_cu * cus) return -4;  // one co-resident round required
  int64_t grid = std::min<int64_t>(want, (int64_t)per_cu * cus);
  if (max_grid > 0) grid = std::min<int64_t>(grid, max_grid);
  if (grid < 1) return -4;
  if (hipMemsetAsync(sync, 0, 2 * sizeof(uint32_t), s) != hipSuccess) return -4;
  void* kargs[] = {&p};
  if (hipLaunchCooperativeKernel(fn, dim3((unsigned)grid), dim3(QN_BLOCK), kargs, (unsigned)lds, s) != hipSuccess) {
    (void)hipGetLastError();
    return -4;
  }
  return 0;
}

extern "C" uint32_t har_logreg_set_spin_limit(uint32_t n) {
  const uint32_t old = g_solve_spin_limit;
  g_solve_spin_limit = n ? n : SOLVE_SPIN_LIMIT;
  return old;
}

extern "C" int har_lbfgs_phase(const QnArgs* args, int KP, int phase, hipStream_t s) {
  const QnArgs& a = *args;
  if ((KP != 8 && KP != 16) || a.K > KP || a.m < 1 || a.m > QN_MAX_M || a.T < 1 || a.T > QN_MAX_TRIALS ||
      a.D != (int64_t)a.K * (a.F + 1) || a.D >= (1LL << 31) || a.nch != har_qn_chunks(a.D, a.B) || phase < 1 ||
      phase > 2 || a.head < 0 || a.head >= a.m || a.done == nullptr)
    return -2;
  if (a.B == 0) return 0;
  const bool full = a.m == QN_MAX_M;
  const dim3 grid(a.nch, a.B);
  if (phase == 1) {
    // the W_eff tile [T][KP][columns per chunk] in LDS when it fits 64 KB and the launch is a batch of
    // >= 256 workgroups (CV direction 42.7 -> 26.0 us; a single fit's 32 workgroups are latency-bound and
    // the tile's extra pass cost ~1 us there, profiles/r5/lr_grad_blocks.md); HAR_LR_WTILE=0: never
    static const bool wt_on = [] {
      const char* e = std::getenv("HAR_LR_WTILE");
      return !e || std::atoi(e) != 0;
    }();
    const int ccs = (a.F + 1 + a.nch - 1) / a.nch;
    const size_t wb = (size_t)(a.init ? 1 : a.T) * KP * ccs * sizeof(float);
    const int uw = wt_on && wb <= 64 * 1024 && (int64_t)a.nch * a.B >= 256 ? 1 : 0;
    const size_t lds = uw ? wb : 0;
    if (KP == 8 && full)
      if (g_lr_stamps)
        qn_direction_kernel<8, true, true><<<grid, QN_BLOCK, lds, s>>>(a, g_lr_stamps_dir, uw);
      else
        qn_direction_kernel<8, true><<<grid, QN_BLOCK, lds, s>>>(a, nullptr, uw);
    else if (KP == 8)
      qn_direction_kernel<8, false><<<grid, QN_BLOCK, lds, s>>>(a, nullptr, uw);
    else if (full)
      qn_direction_kernel<16, true><<<grid, QN_BLOCK, lds, s>>>(a, nullptr, uw);
    else
      qn_direction_kernel<16, false><<<grid, QN_BLOCK, lds, s>>>(a, nullptr, uw);
  } else {
    if (full)  // 170 VGPRs: the 54-model CV batch at 9 chunks still fits one round (40.6 us vs 42.5 lean)
      if (g_lr_stamps)
        qn_update_kernel<true, true, true><<<grid, QN_BLOCK, 0, s>>>(a, g_lr_stamps_upd);
      else
        qn_update_kernel<true, true><<<grid, QN_BLOCK, 0, s>>>(a, nullptr);
    else
      qn_update_kernel<false, false><<<grid, QN_BLOCK, 0, s>>>(a, nullptr);
  }
  HAR_CHECK_LAUNCH();
  return 0;
}

extern "C" void har_lr_set_stamps(uint64_t* ev, uint64_t* dir, uint64_t* upd, uint64_t* grd) {
  g_lr_stamps_grd = grd;
  g_lr_stamps = ev;
  g_lr_stamps_dir = dir;
  g_lr_stamps_upd = upd;
}
