// LogisticRegression fit setup on the device (SURVEY.md K4 / K8, N7's summarizer pass):
//
//   logreg_summary_tiles  one workgroup per (256-row tile, spec): fp64 partial sums of w, w x and
//                         w x^2 of every dense column (chunks of 32 columns staged in LDS) and the
//                         class weight sums of the tile
//   logreg_summary_cols   one lane per (column | class) and spec: the tile partials of a dense
//                         column in tile order, or w over the CSC rows of a one-hot column (x = x^2
//                         = 1), walked as row slices in rounds of 256 like logreg_grad -> the
//                         summary row [sum w, sum w x (F), sum w x^2 (F), class sums (K)]
//   logreg_prepare        one lane per (column, model): standardization (1 / std, unbiased
//                         variance), the frozen-column / pivot / intercept mask, the L2 and L1
//                         weight vectors and the initial point (log class priors as intercepts)
//
// Spark runs this as a MultivariateOnlineSummarizer + MultiClassSummarizer treeAggregate before
// L-BFGS (Main/main.py:115-117); here it is three launches with no host round trip (the data-
// parallel all-reduce of the summary rows sits between the first two and the third).  Every sum
// is fp64 in a fixed order: bitwise reproducible.
#include "common.h"
#include "../har_kernels.h"

namespace {

constexpr int SROWS = 256;
constexpr int SDCH = 32;
constexpr int SXLD = SDCH + 1;

// thread = row: a chunk's values of the row in one round of loads (the flat element loop was one
// dependent round trip per element); each sum is 4 chains of 64 rows added in a fixed order (a single
// 256-long fp64 chain per value was most of the kernel's ~36 us, profiles/r5/lr_grad_blocks.md)
__global__ __launch_bounds__(SROWS) void logreg_summary_tiles_kernel(LogregSummaryArgs a) {
  constexpr int NP = 4, PR = SROWS / NP;  // row parts per sum, rows per part
  __shared__ float xs[SROWS * SXLD];
  __shared__ double ws[SROWS];
  __shared__ int ys[SROWS];
  __shared__ double red[SROWS];  // >= NP * 2 * SDCH partial chains
  const int tid = threadIdx.x, s = blockIdx.y;
  const int64_t r0 = (int64_t)blockIdx.x * SROWS, row = r0 + tid;
  const int64_t nrow = min((int64_t)SROWS, a.N - r0);
  const int PW = 2 * a.Fd + a.K + 1;
  double* out = a.part + ((int64_t)s * gridDim.x + blockIdx.x) * PW;
  ws[tid] = row < a.N ? (a.rw ? (double)a.rw[(int64_t)s * a.N + row] : 1.0) : 0.0;
  ys[tid] = row < a.N ? a.y[row] : -1;
  for (int c0 = 0; c0 < a.Fd; c0 += SDCH) {
    const int nc = min(SDCH, a.Fd - c0);
    __syncthreads();
    {
      const bool in = tid < nrow;
      const float* rp = a.dense + (r0 + (in ? tid : 0)) * a.ldd + c0;
      float v[SDCH];
#pragma unroll
      for (int j = 0; j < SDCH; ++j) v[j] = j < nc ? rp[j] : 0.f;
#pragma unroll
      for (int j = 0; j < SDCH; ++j)
        if (j < nc) xs[tid * SXLD + j] = in ? v[j] : 0.f;
    }
    __syncthreads();
    if (tid < NP * 2 * nc) {
      const int q = tid / NP, part = tid % NP, j = q >> 1, sq = q & 1;
      double acc = 0.0;
      for (int i = part * PR; i < (part + 1) * PR; ++i) {
        const double x = (double)xs[i * SXLD + j];
        acc = fma(ws[i], sq ? x * x : x, acc);
      }
      red[tid] = acc;
    }
    __syncthreads();
    if (tid < 2 * nc) {
      const double* r = red + NP * tid;
      out[2 * c0 + tid] = (r[0] + r[1]) + (r[2] + r[3]);  // value tid = 2 j + sq
    }
  }
  __syncthreads();
  // class sums (k < K) and the weight sum (k == K): 4 row parts each (one 256-row chain when K >= 64)
  const int npk = NP * (a.K + 1) <= SROWS ? NP : 1, prk = SROWS / npk;
  if (tid < npk * (a.K + 1)) {
    const int k = tid / npk, part = tid % npk;
    double acc = 0.0;
    for (int i = part * prk; i < (part + 1) * prk; ++i) acc += (k == a.K || ys[i] == k) ? ws[i] : 0.0;
    red[tid] = acc;
  }
  __syncthreads();
  if (tid <= a.K) {
    const double* r = red + npk * tid;
    out[2 * a.Fd + tid] = npk == NP ? (r[0] + r[1]) + (r[2] + r[3]) : r[0];
  }
}

__global__ __launch_bounds__(256) void logreg_summary_cols_kernel(LogregSummaryArgs a) {
  __shared__ double part[256];
  const int s = blockIdx.y, F = a.F, K = a.K;
  const int PW = 2 * a.Fd + K + 1;
  const double* tp = a.part + (int64_t)s * a.ntiles * PW;
  double* out = a.summ + (int64_t)s * (1 + 2 * F + K);
  const int c0 = blockIdx.x * 256, c1 = min(F, c0 + 256);
  const int col = c0 + threadIdx.x;
  // one-hot columns: row slices of the block's columns in rounds of 256 (fixed order)
  double g = 0.0;
  if (c0 < F) {
    const int s0 = a.col_slice[c0], s1 = a.col_slice[c1];
    const int cs0 = col < c1 ? a.col_slice[col] : 0, cs1 = col < c1 ? a.col_slice[col + 1] : 0;
    for (int base = s0; base < s1; base += 256) {
      if (base > s0) __syncthreads();
      const int sl = base + threadIdx.x;
      if (sl < s1) {
        int r0, r1;
        if (a.srow) {  // the slice's rows from the per-slice table: no dependent search
          r0 = a.srow[sl];
          r1 = a.srow[sl + 1];
        } else {  // the slice's column by a binary search over col_slice (a chain of global loads)
          int lo = c0, hi = c1 - 1;
          while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (a.col_slice[mid] <= sl) lo = mid; else hi = mid - 1;
          }
          r0 = a.csc_off[lo] + (sl - a.col_slice[lo]) * a.SL;
          r1 = min(r0 + a.SL, a.csc_off[lo + 1]);
        }
        double acc = 0.0;
        for (int i = r0; i < r1; ++i) acc += a.rw ? (double)a.rw[(int64_t)s * a.N + a.csc_rows[i]] : 1.0;
        part[threadIdx.x] = acc;
      }
      __syncthreads();
      const int e0 = max(cs0, base), e1 = min(cs1, base + 256);
      for (int e = e0; e < e1; ++e) g += part[e - base];
    }
  }
  if (col < F) {
    const int cm = a.col_map[col];
    if (cm >= 0) {  // dense column: tile partials in tile order
      double s1 = 0.0, s2 = 0.0;
      for (int t = 0; t < a.ntiles; ++t) {
        s1 += tp[(int64_t)t * PW + 2 * cm];
        s2 += tp[(int64_t)t * PW + 2 * cm + 1];
      }
      out[1 + col] = s1;
      out[1 + F + col] = s2;
    } else {
      out[1 + col] = g;
      out[1 + F + col] = g;
    }
  }
  if (blockIdx.x == 0 && threadIdx.x <= K) {  // class sums, then the weight sum (slot 0)
    double acc = 0.0;
    for (int t = 0; t < a.ntiles; ++t) acc += tp[(int64_t)t * PW + 2 * a.Fd + threadIdx.x];
    if ((int)threadIdx.x < K) out[1 + 2 * F + threadIdx.x] = acc; else out[0] = acc;
  }
}

__global__ __launch_bounds__(256) void logreg_prepare_kernel(LogregPrepareArgs a) {
  const int b = blockIdx.y, F = a.F, Kp = a.Kp, K = a.K;
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j > F) return;
  const double* sm = a.summ + (int64_t)b * (1 + 2 * F + K);
  const double wsum = sm[0];
  float feat = 1.f;
  if (j < F) {
    const double mean = sm[1 + j] / wsum, ex2 = sm[1 + F + j] / wsum;
    const double var = (ex2 - mean * mean) * (wsum / fmax(wsum - 1.0, 1.0));
    const float sd = (float)sqrt(fmax(var, 0.0));
    const float inv = sd > 0.f ? (a.standardization ? 1.f / fmaxf(sd, 1e-30f) : 1.f) : 0.f;
    a.inv_std[(int64_t)b * F + j] = inv;
    feat = inv > 0.f ? 1.f : 0.f;
  }
  if (j == 0) a.inv_wsum[b] = (float)(1.0 / wsum);
  const float reg = a.reg[b], alpha = a.alpha[b];
  const int64_t D = (int64_t)Kp * (F + 1);
  // initial intercepts: log class priors (binomial: the logit of class 1; multinomial: centred)
  float prior_mean = 0.f, csum = 0.f;
  if (j == F && a.fit_intercept) {
    for (int k = 0; k < K; ++k) {
      const float c = (float)sm[1 + 2 * F + k];
      csum += c;
      prior_mean += log1pf(c);
    }
    prior_mean /= (float)Kp;
  }
  for (int k = 0; k < Kp; ++k) {
    const float coef = ((!a.fit_intercept && j == F) || (a.binomial && k == 0)) ? 0.f : 1.f;
    const float pm = coef * feat;
    const int64_t e = (int64_t)b * D + (int64_t)k * (F + 1) + j;
    a.pmask[e] = pm;
    const float notb = j == F ? 0.f : 1.f;
    a.l2[e] = reg * (1.f - alpha) * pm * notb;
    if (a.l1) a.l1[e] = reg * alpha * pm * notb;
    float x0 = 0.f;
    if (j == F && a.fit_intercept) {
      if (a.binomial) {
        if (k == 1) {
          const float p1 = fminf(fmaxf((float)sm[1 + 2 * F + 1] / csum, 1e-12f), 1.f - 1e-12f);
          x0 = logf(p1 / (1.f - p1));
        }
      } else {
        x0 = log1pf((float)sm[1 + 2 * F + k]) - prior_mean;
      }
    }
    a.x0[e] = x0 * pm;
  }
}

}  // namespace

extern "C" int har_logreg_summary(const LogregSummaryArgs* args, int phase, hipStream_t s) {
  const LogregSummaryArgs& a = *args;
  if (a.N < 0 || a.F < 1 || a.K < 1 || a.K > 255 || a.Fd < 0 || a.S < 1 || a.SL < 1 || !a.part || !a.summ ||
      !a.col_slice || !a.csc_off || !a.col_map || (a.Fd > 0 && !a.dense) || !a.y ||
      a.ntiles != (int)((a.N + SROWS - 1) / SROWS))
    return -2;
  if (phase == 0) {
    if (a.ntiles == 0) return 0;
    logreg_summary_tiles_kernel<<<dim3(a.ntiles, a.S), SROWS, 0, s>>>(a);
  } else {
    logreg_summary_cols_kernel<<<dim3((a.F + 255) / 256, a.S), 256, 0, s>>>(a);
  }
  HAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int har_logreg_summary_tiles(int64_t n) { return (int)((n + SROWS - 1) / SROWS); }

extern "C" int har_logreg_prepare(const LogregPrepareArgs* args, hipStream_t s) {
  const LogregPrepareArgs& a = *args;
  if (a.B < 1 || a.F < 1 || a.K < 1 || a.Kp < 1 || a.Kp > a.K + 1 || !a.summ || !a.inv_std || !a.inv_wsum ||
      !a.pmask || !a.l2 || !a.x0 || !a.reg || !a.alpha)
    return -2;
  logreg_prepare_kernel<<<dim3((a.F + 1 + 255) / 256, a.B), 256, 0, s>>>(a);
  HAR_CHECK_LAUNCH();
  return 0;
}
