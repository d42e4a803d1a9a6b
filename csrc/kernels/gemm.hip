// LDS-tiled MFMA GEMM with fused epilogues (bf16 and exact-fp32 inputs).
//
//   C[M,N] (op)= sum_k A(m,k) * B(k,n)
//
// A is stored K-major ([M][lda], k contiguous) or M-major ([K][lda], m contiguous);
// B is stored K-major ([N][ldb]) or N-major ([K][ldb]).  With those two flags one
// kernel covers every product of an MLP / logistic-regression step without
// materialising a transpose:
//   forward      Y  = X  . W^T   A=X  (K-major)   B=W  (K-major)
//   data grad    dX = dY . W     A=dY (K-major)   B=W  (N-major)
//   weight grad  dW = dY^T . X   A=dY (M-major)   B=X  (N-major), split-K over the batch
//
// Tiles: BM x BN per workgroup, BK = 32, (WM x WN) waves of 64 lanes, each wave
// owning a (BM/WM) x (BN/WN) sub-tile of 16x16 MFMA accumulators.
//   bf16 : v_mfma_f32_16x16x32_bf16  (lane l: A[l&15][8(l>>4)+j], j<8)
//   fp32 : v_mfma_f32_16x16x4_f32    (lane l: A[l&15][l>>4]) — exact fp32, used by LR
// C/D map (both): col = lane&15, row = 4*(lane>>4) + reg.
//
// Epilogues:
//   EPI_F32        C(f32)  = alpha*acc
//   EPI_F32_ATOMIC C(f32) += alpha*acc           (split-K partials, grid.z = splits)
//   EPI_BIAS_RELU  C(bf16) = relu(acc + bias[n])
//   EPI_BIAS       C(bf16) = acc + bias[n]
//   EPI_RELU_GRAD  C(bf16) = acc * (mask(m,n) > 0);  colsum[n] += sum_m C   (fused bias grad)
//   EPI_BIAS_F32   C(f32)  = acc + bias[n]
#include "common.h"
#include "../har_kernels.h"

namespace {

enum { EPI_F32 = 0, EPI_F32_ATOMIC = 1, EPI_BIAS_RELU = 2, EPI_BIAS = 3, EPI_RELU_GRAD = 4, EPI_BIAS_F32 = 5 };

constexpr int BK = 32;

template <typename T> struct Mfma;
template <> struct Mfma<bf16_t> {
  static constexpr int KPER = 32;  // k per instruction
  static constexpr int VEC = 8;    // elements per lane per instruction
  typedef bf16x8_t frag;
  __device__ static inline f32x4_t mma(const bf16_t* a, const bf16_t* b, f32x4_t c) {
    bf16x8_t fa = *reinterpret_cast<const bf16x8_t*>(a);
    bf16x8_t fb = *reinterpret_cast<const bf16x8_t*>(b);
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb, c, 0, 0, 0);
  }
};
template <> struct Mfma<float> {
  static constexpr int KPER = 4;
  static constexpr int VEC = 1;
  __device__ static inline f32x4_t mma(const float* a, const float* b, f32x4_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(*a, *b, c, 0, 0, 0);
  }
};

// LDS row pitch (elements): BK + one 16-byte pad breaks the power-of-two stride.
template <typename T> constexpr int pitch() { return BK + 16 / (int)sizeof(T); }

template <typename T, int ROWS, int NT, bool KMAJOR>
__device__ __forceinline__ void stage_tile(T* __restrict__ lds, const T* __restrict__ g, int ld,
                                           int row0, int nrows, int k0, int K, int tid) {
  constexpr int EPV = 16 / sizeof(T);  // elements per 16-byte vector
  constexpr int P = pitch<T>();
  if (KMAJOR) {
    // [row][k] source: 16-byte vectors along k
    constexpr int VPR = BK / EPV;
#pragma unroll
    for (int v = tid; v < ROWS * VPR; v += NT) {
      int r = v / VPR, kv = (v % VPR) * EPV;
      int gr = row0 + r, gk = k0 + kv;
      uint4 val = make_uint4(0, 0, 0, 0);
      if (gr < nrows && gk < K) val = *reinterpret_cast<const uint4*>(g + (size_t)gr * ld + gk);
      *reinterpret_cast<uint4*>(lds + r * P + kv) = val;
    }
  } else {
    // [k][row] source: 16-byte vectors along rows, transposed on the LDS write
    constexpr int VPK = ROWS / EPV;
#pragma unroll
    for (int v = tid; v < BK * VPK; v += NT) {
      int k = v / VPK, rv = (v % VPK) * EPV;
      int gk = k0 + k, gr = row0 + rv;
      union { uint4 u; T e[EPV]; } val;
      val.u = make_uint4(0, 0, 0, 0);
      if (gk < K && gr < nrows) val.u = *reinterpret_cast<const uint4*>(g + (size_t)gk * ld + gr);
#pragma unroll
      for (int i = 0; i < EPV; ++i) lds[(rv + i) * P + k] = val.e[i];
    }
  }
}

template <typename T, int BM, int BN, int WM, int WN, bool A_KMAJOR, bool B_KMAJOR, int EPI>
__global__ __launch_bounds__(WM * WN * 64) void gemm_kernel(GemmParams p) {
  constexpr int NT = WM * WN * 64;
  constexpr int P = pitch<T>();
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int RM = TM / 16, RN = TN / 16;
  constexpr int KPER = Mfma<T>::KPER, VEC = Mfma<T>::VEC;
  __shared__ __attribute__((aligned(16))) T As[BM * P];
  __shared__ __attribute__((aligned(16))) T Bs[BN * P];

  const T* __restrict__ A = reinterpret_cast<const T*>(p.A);
  const T* __restrict__ B = reinterpret_cast<const T*>(p.B);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int r16 = lane & 15, q = lane >> 4;

  // XCD-aware tile order over the (n, m) tile grid
  const int ntn = gridDim.x, ntm = gridDim.y;
  const int lin = xcd_remap(blockIdx.y * ntn + blockIdx.x, ntn * ntm);
  const int m0 = (lin / ntn) * BM, n0 = (lin % ntn) * BN;

  int kb = 0, ke = p.K;
  if (EPI == EPI_F32_ATOMIC) {
    kb = blockIdx.z * p.k_split;
    ke = min(p.K, kb + p.k_split);
  }

  f32x4_t acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  for (int k0 = kb; k0 < ke; k0 += BK) {
    // the K bound of the tile clamps to this split's range
    stage_tile<T, BM, NT, A_KMAJOR>(As, A, p.lda, m0, p.M, k0, ke, tid);
    stage_tile<T, BN, NT, B_KMAJOR>(Bs, B, p.ldb, n0, p.N, k0, ke, tid);
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < BK; kk += KPER) {
      const int kl = kk + q * VEC;
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j)
          acc[i][j] = Mfma<T>::mma(&As[(wm * TM + i * 16 + r16) * P + kl],
                                   &Bs[(wn * TN + j * 16 + r16) * P + kl], acc[i][j]);
    }
    __syncthreads();
  }

  // ---- epilogue ----
  float* Cf = reinterpret_cast<float*>(p.C);
  bf16_t* Cb = reinterpret_cast<bf16_t*>(p.C);
  const bf16_t* mask = reinterpret_cast<const bf16_t*>(p.mask);
#pragma unroll
  for (int j = 0; j < RN; ++j) {
    const int n = n0 + wn * TN + j * 16 + r16;
    const bool nok = n < p.N;
    float bias = 0.f;
    if ((EPI == EPI_BIAS_RELU || EPI == EPI_BIAS || EPI == EPI_BIAS_F32) && nok && p.bias) bias = p.bias[n];
    float csum = 0.f;
#pragma unroll
    for (int i = 0; i < RM; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * TM + i * 16 + q * 4 + r;
        if (!(nok && m < p.M)) continue;
        float v = acc[i][j][r];
        size_t off = (size_t)m * p.ldc + n;
        if (EPI == EPI_F32) Cf[off] = p.alpha * v;
        else if (EPI == EPI_F32_ATOMIC) atomicAdd(Cf + off, p.alpha * v);
        else if (EPI == EPI_BIAS_RELU) Cb[off] = f2bf(fmaxf(v + bias, 0.f));
        else if (EPI == EPI_BIAS) Cb[off] = f2bf(v + bias);
        else if (EPI == EPI_BIAS_F32) Cf[off] = v + bias;
        else if (EPI == EPI_RELU_GRAD) {
          bf16_t mk = mask[(size_t)m * p.ldmask + n];
          float g = ((mk & 0x8000u) == 0 && mk != 0) ? v : 0.f;
          bf16_t gb = f2bf(g);
          Cb[off] = gb;
          csum += bf2f(gb);
        }
      }
    }
    if (EPI == EPI_RELU_GRAD && p.colsum) {
      // lanes r16, r16+16, r16+32, r16+48 share the column
      csum += __shfl_xor(csum, 16, 64);
      csum += __shfl_xor(csum, 32, 64);
      if (q == 0 && nok) atomicAdd(p.colsum + n, csum);
    }
  }
}

template <typename T, int BM, int BN, int WM, int WN, bool AK, bool BKm>
int launch_epi(const GemmParams& p, int epi, hipStream_t s) {
  dim3 grid((p.N + BN - 1) / BN, (p.M + BM - 1) / BM, 1);
  if (epi == EPI_F32_ATOMIC) grid.z = (p.K + p.k_split - 1) / p.k_split;
  dim3 block(WM * WN * 64);
  switch (epi) {
    case EPI_F32: gemm_kernel<T, BM, BN, WM, WN, AK, BKm, EPI_F32><<<grid, block, 0, s>>>(p); break;
    case EPI_F32_ATOMIC: gemm_kernel<T, BM, BN, WM, WN, AK, BKm, EPI_F32_ATOMIC><<<grid, block, 0, s>>>(p); break;
    case EPI_BIAS_RELU: gemm_kernel<T, BM, BN, WM, WN, AK, BKm, EPI_BIAS_RELU><<<grid, block, 0, s>>>(p); break;
    case EPI_BIAS: gemm_kernel<T, BM, BN, WM, WN, AK, BKm, EPI_BIAS><<<grid, block, 0, s>>>(p); break;
    case EPI_RELU_GRAD: gemm_kernel<T, BM, BN, WM, WN, AK, BKm, EPI_RELU_GRAD><<<grid, block, 0, s>>>(p); break;
    case EPI_BIAS_F32: gemm_kernel<T, BM, BN, WM, WN, AK, BKm, EPI_BIAS_F32><<<grid, block, 0, s>>>(p); break;
    default: return -1;
  }
  HAR_CHECK_LAUNCH();
  return 0;
}

template <typename T, bool AK, bool BKm>
int launch_tile(const GemmParams& p, int epi, hipStream_t s) {
  // tile choice: wide tiles when both dims are large, narrow-N tiles for heads / thin outputs
  if (p.N <= 32) return launch_epi<T, 128, 32, 4, 1, AK, BKm>(p, epi, s);
  if (p.N <= 64) return launch_epi<T, 128, 64, 2, 2, AK, BKm>(p, epi, s);
  if (p.M <= 64) return launch_epi<T, 64, 128, 1, 4, AK, BKm>(p, epi, s);
  return launch_epi<T, 128, 128, 2, 2, AK, BKm>(p, epi, s);
}

template <typename T>
int gemm_dispatch(const GemmParams& p, int layout, int epi, hipStream_t s) {
  // layout bit0: A is M-major; bit1: B is N-major
  const int EPV = 16 / sizeof(T);
  bool a_mmajor = layout & 1, b_nmajor = layout & 2;
  // vector-load alignment contract (checked on the host side as well)
  if ((a_mmajor ? p.M : p.K) % EPV || (b_nmajor ? p.N : p.K) % EPV || p.lda % EPV || p.ldb % EPV) return -2;
  if (epi == EPI_F32_ATOMIC && (p.k_split <= 0 || p.k_split % BK)) return -3;
  if (!a_mmajor && !b_nmajor) return launch_tile<T, true, true>(p, epi, s);
  if (!a_mmajor && b_nmajor) return launch_tile<T, true, false>(p, epi, s);
  if (a_mmajor && b_nmajor) return launch_tile<T, false, false>(p, epi, s);
  return launch_tile<T, false, true>(p, epi, s);
}

}  // namespace

extern "C" int har_gemm_bf16(const GemmParams* p, int layout, int epi, hipStream_t s) {
  return gemm_dispatch<bf16_t>(*p, layout, epi, s);
}

extern "C" int har_gemm_f32(const GemmParams* p, int layout, int epi, hipStream_t s) {
  return gemm_dispatch<float>(*p, layout, epi, s);
}
