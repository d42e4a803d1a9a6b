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
#include "common.h"
#include "../har_kernels.h"

namespace {

constexpr int EVAL_ROWS = 256;
constexpr int QN_THREADS = 1024;

// ---------------------------------------------------------------------------------------------
// logreg_eval: one workgroup = EVAL_ROWS rows x one (trial) model
// ---------------------------------------------------------------------------------------------
template <int KP>
__global__ __launch_bounds__(EVAL_ROWS) void logreg_eval_kernel(LogregEvalArgs a) {
  extern __shared__ float smem[];
  const int Fd = a.Fd;
  const int xs_ld = Fd | 1;                        // odd row stride: conflict-free row reads
  float* wd = smem;                                // [Fd + 1][KP] dense weights + intercept
  float* xs = wd + (Fd + 1) * KP;                  // [EVAL_ROWS][xs_ld]
  float* rs = xs + EVAL_ROWS * xs_ld;              // [EVAL_ROWS][KP]
  float* red = rs + EVAL_ROWS * KP;                // [EVAL_ROWS / 64]

  const int tid = threadIdx.x;
  const int bt = blockIdx.y * a.tstride;           // trial model
  const int s = bt / a.T;                          // spec (row-weight vector) of the model
  const int64_t r0 = (int64_t)blockIdx.x * EVAL_ROWS;
  const int64_t row = r0 + tid;
  const bool ok = row < a.N;
  const float* W = a.W + (int64_t)bt * (a.F + 1) * KP;

  // stage the dense weights (+ intercept row) and the dense row tile
  for (int e = tid; e < Fd * KP; e += EVAL_ROWS) wd[e] = W[(int64_t)a.dense_cols[e / KP] * KP + (e % KP)];
  if (tid < KP) wd[Fd * KP + tid] = W[(int64_t)a.F * KP + tid];
  const int64_t nrow_tile = min((int64_t)EVAL_ROWS, a.N - r0);
  for (int64_t e = tid; e < nrow_tile * Fd; e += EVAL_ROWS) {
    const int64_t rr = e / Fd, j = e % Fd;
    xs[rr * xs_ld + j] = a.dense[(r0 + rr) * a.ldd + j];
  }
  for (int64_t e = nrow_tile * Fd + tid; e < (int64_t)EVAL_ROWS * Fd; e += EVAL_ROWS) {
    const int64_t rr = e / Fd, j = e % Fd;
    xs[rr * xs_ld + j] = 0.f;
  }
  __syncthreads();

  float z[KP];
#pragma unroll
  for (int k = 0; k < KP; ++k) z[k] = wd[Fd * KP + k];
  float lossv = 0.f;
  if (ok) {
    for (int j = 0; j < Fd; ++j) {
      const float xv = xs[tid * xs_ld + j];
#pragma unroll
      for (int k = 0; k < KP; ++k) z[k] = fmaf(xv, wd[j * KP + k], z[k]);
    }
    for (int c = 0; c < a.C; ++c) {
      const int col = a.cat[row * a.C + c];
      if (col >= 0) {
        const f32x4_t* wp = reinterpret_cast<const f32x4_t*>(W + (int64_t)col * KP);
#pragma unroll
        for (int q = 0; q < KP / 4; ++q) {
          const f32x4_t w4 = wp[q];
          z[4 * q + 0] += w4[0];
          z[4 * q + 1] += w4[1];
          z[4 * q + 2] += w4[2];
          z[4 * q + 3] += w4[3];
        }
      }
    }
  }
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
    f32x4_t* rp = reinterpret_cast<f32x4_t*>(a.R + ((int64_t)bt * a.N + row) * KP);
#pragma unroll
    for (int q = 0; q < KP / 4; ++q) rp[q] = f32x4_t{rv[4 * q], rv[4 * q + 1], rv[4 * q + 2], rv[4 * q + 3]};
  }
  if (a.mode == 1) return;
  // tile loss: wave sums, then the 4 wave partials in a fixed order
  lossv = wave_sum(lossv);
  if ((tid & 63) == 0) red[tid >> 6] = lossv;
  __syncthreads();
  const int SW = Fd * KP + KP + 1;
  float* slab = a.slab + ((int64_t)bt * gridDim.x + blockIdx.x) * SW;
  // dense gradient R^T X and intercept gradient sum R of the tile (fixed row order)
  for (int o = tid; o < Fd * KP + KP; o += EVAL_ROWS) {
    const int k = o % KP;
    float acc = 0.f;
    if (o < Fd * KP) {
      const int j = o / KP;
      for (int i = 0; i < EVAL_ROWS; ++i) acc = fmaf(rs[i * KP + k], xs[i * xs_ld + j], acc);
    } else {
      for (int i = 0; i < EVAL_ROWS; ++i) acc += rs[i * KP + k];
    }
    slab[o] = acc;
  }
  if (tid == 0) slab[SW - 1] = (red[0] + red[1]) + (red[2] + red[3]);
}

// ---------------------------------------------------------------------------------------------
// logreg_grad: one lane per (column, trial model); G[bt][k][col], loss[bt]
// ---------------------------------------------------------------------------------------------
template <int KP>
__global__ __launch_bounds__(256) void logreg_grad_kernel(LogregGradArgs a) {
  const int bt = blockIdx.y * a.tstride;
  const int s = bt / a.T;
  const int col = blockIdx.x * 256 + threadIdx.x;
  const int Fp1 = a.F + 1;
  const int SW = a.Fd * KP + KP + 1;
  const float* slab = a.slab + (int64_t)bt * a.ntiles * SW;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    double l = 0.0;
    for (int t = 0; t < a.ntiles; ++t) l += (double)slab[(int64_t)t * SW + SW - 1];
    a.loss[bt] = l;
  }
  if (col >= Fp1) return;
  const int cm = a.col_map[col];
  float g[KP];
#pragma unroll
  for (int k = 0; k < KP; ++k) g[k] = 0.f;
  if (cm >= 0 || cm == -1) {  // dense column j = cm, or the intercept (slab entries after the dense block)
    const int off = cm >= 0 ? cm * KP : a.Fd * KP;
    for (int t = 0; t < a.ntiles; ++t) {
      const float* p = slab + (int64_t)t * SW + off;
#pragma unroll
      for (int k = 0; k < KP; ++k) g[k] += p[k];
    }
  } else {  // one-hot column: its rows (CSC list, ascending row order)
    const int lo = a.csc_off[col], hi = a.csc_off[col + 1];
    const float* R = a.R + (int64_t)bt * a.N * KP;
    for (int i = lo; i < hi; ++i) {
      const f32x4_t* rp = reinterpret_cast<const f32x4_t*>(R + (int64_t)a.csc_rows[i] * KP);
#pragma unroll
      for (int q = 0; q < KP / 4; ++q) {
        const f32x4_t r4 = rp[q];
        g[4 * q + 0] += r4[0];
        g[4 * q + 1] += r4[1];
        g[4 * q + 2] += r4[2];
        g[4 * q + 3] += r4[3];
      }
    }
  }
  const float sc = col < a.F ? a.inv_std[(int64_t)s * a.F + col] : 1.f;
  const int64_t D = (int64_t)a.K * Fp1;
  float* G = a.G + (int64_t)bt * D;
  const float* pm = a.pmask + (int64_t)s * D;
  for (int k = 0; k < a.K; ++k) G[(int64_t)k * Fp1 + col] = g[k] * sc * pm[(int64_t)k * Fp1 + col];
}

// ---------------------------------------------------------------------------------------------
// block reductions for the QN kernels (1024 threads = 16 waves)
// ---------------------------------------------------------------------------------------------
template <int NV>
__device__ __forceinline__ void block_sum(double (&v)[NV], double* sh) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int q = 0; q < NV; ++q) v[q] = wave_sum_d(v[q]);
  __syncthreads();
  if (lane == 0) {
#pragma unroll
    for (int q = 0; q < NV; ++q) sh[w * NV + q] = v[q];
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < NV; ++q) {
    double t = 0.0;
    for (int i = 0; i < QN_THREADS / 64; ++i) t += sh[i * NV + q];  // fixed order
    v[q] = t;
  }
  __syncthreads();
}

__device__ __forceinline__ float pseudo_grad(float x, float g, float l1) {
  if (l1 == 0.f) return g;
  const float gp = g + l1, gm = g - l1;
  if (x > 0.f) return gp;
  if (x < 0.f) return gm;
  return gp < 0.f ? gp : (gm > 0.f ? gm : 0.f);
}

__device__ __forceinline__ float sgnf(float v) { return v > 0.f ? 1.f : (v < 0.f ? -1.f : 0.f); }

// ---------------------------------------------------------------------------------------------
// lbfgs_direction: one workgroup per model b
// ---------------------------------------------------------------------------------------------
template <int KP>
__global__ __launch_bounds__(QN_THREADS) void lbfgs_direction_kernel(QnArgs a) {
  __shared__ double sh[16 * 4];
  __shared__ double alph[32];
  const int b = blockIdx.x;
  const int64_t D = a.D;
  const int Fp1 = a.F + 1;
  const float* x = a.x + b * D;
  const float* g = a.g + b * D;
  const float* l1v = a.l1 ? a.l1 + b * D : nullptr;
  float* q = a.work + b * D;  // q, then r, then the direction
  const int tid = threadIdx.x;
  const bool active = a.active[b] != 0;

  double dd = 0.0, gamma = 1.0;
  if (a.init) {
    for (int64_t e = tid; e < D; e += QN_THREADS) q[e] = 0.f;
  } else {
    // pseudo-gradient -> q
    double pn[1] = {0.0};
    for (int64_t e = tid; e < D; e += QN_THREADS) {
      const float pg = pseudo_grad(x[e], g[e], l1v ? l1v[e] : 0.f);
      q[e] = pg;
      pn[0] += (double)pg * pg;
    }
    block_sum<1>(pn, sh);
    // first loop: newest -> oldest
    for (int i = 0; i < a.filled; ++i) {
      const int j = (a.head - 1 - i + a.m) % a.m;
      const float* S = a.S + ((int64_t)j * a.B + b) * D;
      const float* Y = a.Y + ((int64_t)j * a.B + b) * D;
      const double rho = a.rho[j * a.B + b];
      double v[1] = {0.0};
      if (rho != 0.0)
        for (int64_t e = tid; e < D; e += QN_THREADS) v[0] += (double)S[e] * q[e];
      block_sum<1>(v, sh);
      const double al = rho * v[0];
      if (tid == 0) alph[i] = al;
      if (rho != 0.0)
        for (int64_t e = tid; e < D; e += QN_THREADS) q[e] = (float)((double)q[e] - al * Y[e]);
    }
    if (a.filled > 0) {
      const int j = (a.head - 1 + a.m) % a.m;
      const float* S = a.S + ((int64_t)j * a.B + b) * D;
      const float* Y = a.Y + ((int64_t)j * a.B + b) * D;
      const double rho = a.rho[j * a.B + b];
      double v[2] = {0.0, 0.0};
      for (int64_t e = tid; e < D; e += QN_THREADS) {
        v[0] += (double)Y[e] * Y[e];
        v[1] += (double)S[e] * Y[e];
      }
      block_sum<2>(v, sh);
      gamma = (rho > 0.0 && v[0] > 0.0) ? v[1] / v[0] : 1.0;
    } else {
      gamma = 1.0 / fmax(sqrt(pn[0]), 1e-12);
    }
    for (int64_t e = tid; e < D; e += QN_THREADS) q[e] = (float)(gamma * q[e]);
    __syncthreads();
    // second loop: oldest -> newest
    for (int i = a.filled - 1; i >= 0; --i) {
      const int j = (a.head - 1 - i + a.m) % a.m;
      const float* S = a.S + ((int64_t)j * a.B + b) * D;
      const float* Y = a.Y + ((int64_t)j * a.B + b) * D;
      const double rho = a.rho[j * a.B + b];
      double v[1] = {0.0};
      if (rho != 0.0)
        for (int64_t e = tid; e < D; e += QN_THREADS) v[0] += (double)Y[e] * q[e];
      block_sum<1>(v, sh);
      const double coef = alph[i] - rho * v[0];
      if (rho != 0.0)
        for (int64_t e = tid; e < D; e += QN_THREADS) q[e] = (float)((double)q[e] + coef * S[e]);
    }
    __syncthreads();
    // direction d = -r, orthant-restricted for OWL-QN; descent check
    double v[2] = {0.0, 0.0};
    for (int64_t e = tid; e < D; e += QN_THREADS) {
      const float pg = pseudo_grad(x[e], g[e], l1v ? l1v[e] : 0.f);
      float d = -q[e];
      if (l1v && d * pg >= 0.f) d = 0.f;
      q[e] = d;
      v[0] += (double)pg * d;
      v[1] += (double)pg * pg;
    }
    block_sum<2>(v, sh);
    dd = v[0];
    if (dd >= 0.0) {  // not a descent direction: steepest descent on the pseudo-gradient
      for (int64_t e = tid; e < D; e += QN_THREADS) q[e] = -pseudo_grad(x[e], g[e], l1v ? l1v[e] : 0.f);
      dd = -v[1];
    }
    __syncthreads();
  }
  // trial points, their effective weights, regularization and Armijo decrease terms
  const int T = a.init ? 1 : a.T;
  for (int t = 0; t < T; ++t) {
    const float step = a.init ? 0.f : a.step_scale[b] * ldexpf(1.f, -t);
    const int bt = b * a.T + t;
    float* xt = a.xtrial + (int64_t)bt * D;
    float* W = a.weff + (int64_t)bt * Fp1 * KP;
    double v[3] = {0.0, 0.0, 0.0};  // 0.5 l2 |beta|^2, l1 |x|_1, pg . (xt - x)
    for (int64_t e = tid; e < D; e += QN_THREADS) {
      const float xe = x[e];
      float xn = xe + step * q[e];
      const float l1e = l1v ? l1v[e] : 0.f;
      if (l1v && !a.init) {  // stay in the orthant of x (or of -pg where x == 0)
        const float pg = pseudo_grad(xe, g[e], l1e);
        const float xi = xe != 0.f ? sgnf(xe) : sgnf(-pg);
        if (sgnf(xn) != xi) xn = 0.f;
        v[2] += (double)pg * (xn - xe);
      }
      if (!active) xn = xe;
      xt[e] = xn;
      const float l2e = a.l2[b * D + e];
      v[0] += 0.5 * (double)l2e * xn * xn;
      v[1] += (double)l1e * fabsf(xn);
      const int k = (int)(e / Fp1), col = (int)(e % Fp1);
      const float pm = a.pmask[b * D + e];
      const float sc = col < a.F ? a.inv_std[(int64_t)b * a.F + col] : 1.f;
      W[(int64_t)col * KP + k] = xn * sc * pm;
    }
    block_sum<3>(v, sh);
    if (tid == 0) {
      a.reg[bt] = v[0] + v[1];
      a.decr[bt] = l1v ? v[2] : (double)step * dd;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// lbfgs_update: one workgroup per model b
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(QN_THREADS) void lbfgs_update_kernel(QnArgs a) {
  __shared__ double sh[16 * 5];
  __shared__ int pick;
  const int b = blockIdx.x;
  const int64_t D = a.D;
  const int tid = threadIdx.x;
  float* x = a.x + b * D;
  float* g = a.g + b * D;
  const float* l1v = a.l1 ? a.l1 + b * D : nullptr;
  const bool active = a.active[b] != 0;
  if (tid == 0) {
    int p = -1;
    if (a.init) {
      p = 0;
    } else if (active) {
      const double F0 = a.fobj[b];
      for (int t = 0; t < a.T && p < 0; ++t) {
        const int bt = b * a.T + t;
        const double Ft = a.loss[bt] + a.reg[bt];
        if (isfinite(Ft) && Ft <= F0 + a.c1 * a.decr[bt]) p = t;
      }
    }
    pick = p;
  }
  __syncthreads();
  const int p = pick;
  float* S = a.S + ((int64_t)a.head * a.B + b) * D;
  float* Y = a.Y + ((int64_t)a.head * a.B + b) * D;
  if (p < 0) {  // inactive, or no trial accepted: keep x; disable the slot; shrink the next steps
    if (!a.init) {
      if (tid == 0) {
        a.rho[a.head * a.B + b] = 0.0;
        if (active) {
          a.step_scale[b] *= 1.0f / 16.0f;
          if (++a.fails[b] >= 2) a.active[b] = 0;
        }
      }
    }
    return;
  }
  const int bt = b * a.T + p;
  const float* xt = a.xtrial + (int64_t)bt * D;
  const float* Gt = a.G + (int64_t)bt * D;
  double v[5] = {0.0, 0.0, 0.0, 0.0, 0.0};  // s.y, |s|^2, |y|^2, |x_new|^2, |pg_new|^2
  for (int64_t e = tid; e < D; e += QN_THREADS) {
    const float xn = xt[e];
    const float gn = Gt[e] + a.l2[b * D + e] * xn;  // data gradient (masked, scaled) + L2 term
    if (!a.init) {
      const float se = xn - x[e], ye = gn - g[e];
      S[e] = se;
      Y[e] = ye;
      v[0] += (double)se * ye;
      v[1] += (double)se * se;
      v[2] += (double)ye * ye;
    }
    const float pg = pseudo_grad(xn, gn, l1v ? l1v[e] : 0.f);
    v[3] += (double)xn * xn;
    v[4] += (double)pg * pg;
    x[e] = xn;
    g[e] = gn;
  }
  block_sum<5>(v, sh);
  if (tid == 0) {
    const double Fn = a.loss[bt] + a.reg[bt];
    if (a.init) {
      a.fobj[b] = Fn;
    } else {
      const bool good = v[0] > 1e-10 * fmax(sqrt(v[1]) * sqrt(v[2]), 1e-300);
      a.rho[a.head * a.B + b] = good ? 1.0 / v[0] : 0.0;
      const double F0 = a.fobj[b];
      const double rel = fabs(F0 - Fn) / fmax(fmax(fabs(F0), fabs(Fn)), 1.0);
      a.fobj[b] = Fn;
      a.iters[b] += 1;
      a.fails[b] = 0;
      a.step_scale[b] = 1.0f;
      if (rel < a.tol || sqrt(v[4]) <= a.tol * fmax(sqrt(v[3]), 1.0)) a.active[b] = 0;
    }
    if (a.hist) a.hist[(int64_t)a.it * a.B + b] = a.fobj[b];
  }
}

}  // namespace

extern "C" int har_logreg_eval(const LogregEvalArgs* args, int KP, int n_models, hipStream_t s) {
  const LogregEvalArgs& a = *args;
  if (a.Fd < 0 || a.Fd > HAR_LOGREG_MAX_DENSE || a.K < 1 || a.K > KP || (KP != 8 && KP != 16) || a.T < 1 ||
      a.tstride < 1 || (a.mode == 0 && a.slab == nullptr) || (a.C > 0 && a.cat == nullptr))
    return -2;
  if (a.N == 0 || n_models == 0) return 0;
  const int tiles = (int)((a.N + EVAL_ROWS - 1) / EVAL_ROWS);
  const size_t lds = sizeof(float) * ((a.Fd + 1) * KP + EVAL_ROWS * (a.Fd | 1) + EVAL_ROWS * KP + EVAL_ROWS / 64);
  dim3 grid(tiles, n_models);
  if (KP == 8)
    logreg_eval_kernel<8><<<grid, EVAL_ROWS, lds, s>>>(a);
  else
    logreg_eval_kernel<16><<<grid, EVAL_ROWS, lds, s>>>(a);
  HAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int har_logreg_eval_tiles(int64_t n) { return (int)((n + EVAL_ROWS - 1) / EVAL_ROWS); }

extern "C" int har_logreg_grad(const LogregGradArgs* args, int KP, int n_models, hipStream_t s) {
  const LogregGradArgs& a = *args;
  if (a.K < 1 || a.K > KP || (KP != 8 && KP != 16) || a.T < 1 || a.tstride < 1) return -2;
  if (n_models == 0) return 0;
  dim3 grid((a.F + 1 + 255) / 256, n_models);
  if (KP == 8)
    logreg_grad_kernel<8><<<grid, 256, 0, s>>>(a);
  else
    logreg_grad_kernel<16><<<grid, 256, 0, s>>>(a);
  HAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int har_lbfgs_direction(const QnArgs* args, int KP, hipStream_t s) {
  const QnArgs& a = *args;
  if ((KP != 8 && KP != 16) || a.K > KP || a.m > 32 || a.T < 1 || a.D != (int64_t)a.K * (a.F + 1)) return -2;
  if (a.B == 0) return 0;
  if (KP == 8)
    lbfgs_direction_kernel<8><<<a.B, QN_THREADS, 0, s>>>(a);
  else
    lbfgs_direction_kernel<16><<<a.B, QN_THREADS, 0, s>>>(a);
  HAR_CHECK_LAUNCH();
  return 0;
}

extern "C" int har_lbfgs_update(const QnArgs* args, hipStream_t s) {
  const QnArgs& a = *args;
  if (a.m > 32 || a.T < 1) return -2;
  if (a.B == 0) return 0;
  lbfgs_update_kernel<<<a.B, QN_THREADS, 0, s>>>(a);
  HAR_CHECK_LAUNCH();
  return 0;
}
