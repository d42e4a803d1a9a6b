// areaUnderROC / areaUnderPR (BinaryClassificationEvaluator at
// Main/main.py:135-143) over scores already sorted descending (the sort is the
// rocPRIM radix sort behind torch.sort).
//
// One workgroup streams the sorted array in chunks of ROC_T * ROC_I entries, carrying the
// running positive count and the last curve point across chunks.  A curve point is the end of
// a tie group (s[i] != s[i+1]); its (TP, FP) come from a block scan of the positive flags and
// the previous point from a second block scan with the "latest point wins" operator, so ties
// that straddle threads or chunks are grouped exactly as in BinaryClassificationMetrics.
// ROC sums exact integer products (sum dFP * (TP + TP_prev)), PR sums in fp64; the host
// divides by 2PN / 2P and adds the (1, 1) end point.
#include "common.h"
#include "../har_kernels.h"

namespace {

constexpr int ROC_T = 1024, ROC_I = 4, ROC_W = ROC_T / 64;

__global__ __launch_bounds__(ROC_T) void roc_pr_kernel(const float* __restrict__ s, const float* __restrict__ y,
                                                      int n, double* __restrict__ out, const int32_t* __restrict__ ns,
                                                      int64_t ld) {
  // batched (grid = models): model b's scores / labels at + b * ld, its first ns[b] entries
  if (ns) {
    s += (size_t)blockIdx.x * ld;
    y += (size_t)blockIdx.x * ld;
    n = ns[blockIdx.x];
    out += 4 * (size_t)blockIdx.x;
  }
  __shared__ int wtot[ROC_W], whas[ROC_W], wtp[ROC_W], wfp[ROC_W];
  __shared__ int carry[4];  // has point, TP, FP of the last point; positives so far
  __shared__ double wred[2][ROC_W];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (tid < 4) carry[tid] = 0;
  double roc = 0.0, pr = 0.0;
  __syncthreads();
  for (int base = 0; base < n; base += ROC_T * ROC_I) {
    const int i0 = base + tid * ROC_I;
    float sv[ROC_I + 1];
    int pos[ROC_I], cnt = 0;
#pragma unroll
    for (int k = 0; k <= ROC_I; ++k) sv[k] = i0 + k < n ? s[i0 + k] : 0.f;
#pragma unroll
    for (int k = 0; k < ROC_I; ++k) {
      pos[k] = (i0 + k < n && y[i0 + k] > 0.5f) ? 1 : 0;
      cnt += pos[k];
    }
    int inc = cnt;  // wave inclusive scan of the positive counts
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int t = __shfl_up(inc, o, 64);
      if (lane >= o) inc += t;
    }
    if (lane == 63) wtot[w] = inc;
    __syncthreads();
    int woff = 0;
    for (int j = 0; j < w; ++j) woff += wtot[j];
    const int c0 = carry[3];
    int tp = c0 + woff + inc - cnt;
    int tpk[ROC_I];
    bool endk[ROC_I];
    int lh = 0, ltp = 0, lfp = 0;  // this thread's last point
#pragma unroll
    for (int k = 0; k < ROC_I; ++k) {
      const int idx = i0 + k;
      tp += pos[k];
      tpk[k] = tp;
      endk[k] = idx < n && (idx == n - 1 || sv[k] != sv[k + 1]);
      if (endk[k]) { lh = 1; ltp = tp; lfp = idx + 1 - tp; }
    }
    int vh = lh, vtp = ltp, vfp = lfp;  // wave inclusive scan: the latest point wins
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int h = __shfl_up(vh, o, 64), a = __shfl_up(vtp, o, 64), b = __shfl_up(vfp, o, 64);
      if (lane >= o && !vh) { vh = h; vtp = a; vfp = b; }
    }
    if (lane == 63) { whas[w] = vh; wtp[w] = vtp; wfp[w] = vfp; }
    int eh = __shfl_up(vh, 1, 64), etp = __shfl_up(vtp, 1, 64), efp = __shfl_up(vfp, 1, 64);
    if (lane == 0) eh = 0;
    __syncthreads();
    for (int j = w - 1; j >= 0 && !eh; --j)
      if (whas[j]) { eh = 1; etp = wtp[j]; efp = wfp[j]; }
    if (!eh) { eh = carry[0]; etp = carry[1]; efp = carry[2]; }
    // trapezoids between consecutive points; the first point's PR predecessor is itself
    bool has = eh != 0;
    int ptp = has ? etp : 0, pfp = has ? efp : 0;
    double pprec = has ? (double)ptp / (double)(ptp + pfp) : 0.0;
#pragma unroll
    for (int k = 0; k < ROC_I; ++k) {
      if (!endk[k]) continue;
      const int ctp = tpk[k], cfp = i0 + k + 1 - ctp;
      const double prec = (double)ctp / (double)(i0 + k + 1);
      roc += (double)(cfp - pfp) * (double)(ctp + ptp);
      pr += (double)(ctp - ptp) * (prec + (has ? pprec : prec));
      ptp = ctp; pfp = cfp; pprec = prec; has = true;
    }
    __syncthreads();  // every thread has read the old carry
    if (tid == ROC_T - 1) {
      if (vh) { carry[0] = 1; carry[1] = vtp; carry[2] = vfp; }
      else { carry[0] = eh; carry[1] = etp; carry[2] = efp; }
      carry[3] = c0 + woff + inc;
    }
    __syncthreads();
  }
  roc = wave_sum_d(roc);
  pr = wave_sum_d(pr);
  if (lane == 0) { wred[0][w] = roc; wred[1][w] = pr; }
  __syncthreads();
  if (tid == 0) {
    double a = 0.0, b = 0.0;
    for (int j = 0; j < ROC_W; ++j) { a += wred[0][j]; b += wred[1][j]; }
    out[0] = a;
    out[1] = b;
    out[2] = (double)carry[3];
    out[3] = (double)(n - carry[3]);
  }
}

}  // namespace

extern "C" int har_roc_pr_sums(const float* sorted_scores, const float* labels, int64_t n, double* out4,
                               hipStream_t s) {
  if (n < 0 || n >= ((int64_t)1 << 30)) return -2;
  roc_pr_kernel<<<1, ROC_T, 0, s>>>(sorted_scores, labels, (int)n, out4, nullptr, 0);
  HAR_CHECK_LAUNCH();
  return 0;
}

// B models: row b of sorted_scores / labels ([B][ld], scores descending) holds ns[b] valid entries
// (a CrossValidator fold's validation rows, sorted to the front); out [B][4].
extern "C" int har_roc_pr_sums_batched(const float* sorted_scores, const float* labels, const int32_t* ns, int B,
                                       int64_t ld, double* out, hipStream_t s) {
  if (B <= 0 || ld < 0 || ld >= ((int64_t)1 << 30) || !ns) return -2;
  roc_pr_kernel<<<B, ROC_T, 0, s>>>(sorted_scores, labels, 0, out, ns, ld);
  HAR_CHECK_LAUNCH();
  return 0;
}
