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
// Tiles: BM x BN x BK per workgroup (BK = 32/64/128), (WM x WN) waves of 64 lanes, each wave
// owning a (BM/WM) x (BN/WN) sub-tile of 16x16 MFMA accumulators.
//   bf16 : v_mfma_f32_16x16x32_bf16  (lane l: A[l&15][8(l>>4)+j], j<8)
//   fp32 : v_mfma_f32_16x16x4_f32    (lane l: A[l&15][l>>4]) — exact fp32, used by LR
// C/D map (both): col = lane&15, row = 4*(lane>>4) + reg.
//
// LDS images are copies of the global tiles in their own orientation (16-byte
// vector writes only): K-major operands as [rows][BK], M/N-major operands as
// [BK][rows].  Fragments of a [BK][rows] bf16 image are read with the gfx950
// transposing LDS read ds_read_b64_tr_b16 (guide §5.5 T10): two reads give a
// lane the 8 consecutive k of its row, exactly the MFMA operand map — no
// scalar transposing stores.  Main loop: register-staged prefetch (the global
// loads of tile k+1 are issued before the MFMAs of tile k, guide §6 G15/T14).
// bf16 epilogues go through LDS and leave as 16-byte row vectors.
//
// Epilogues:
//   EPI_F32        C(f32)  = alpha*acc
//   EPI_F32_ATOMIC C(f32) += alpha*acc                 (split-K, grid.z = splits)
//   EPI_BIAS_RELU  C(bf16) = relu(acc + bias[n])
//   EPI_BIAS       C(bf16) = acc + bias[n]
//   EPI_RELU_GRAD  C(bf16) = acc * (mask(m,n) > 0)
//   EPI_BIAS_F32   C(f32)  = acc + bias[n]
//   EPI_F32_SLAB   C[z](f32) = alpha*acc   plain stores into split slab z = blockIdx.z
//                  (deterministic split-K: a later pass sums the slabs, no atomics)
// Optional fused A-row sums (bias gradients of a weight-grad product): blocks of
// the first N tile sum the k-slots of the A fragments they feed to the MFMAs and
// store sum_k A(m,k) over their K range to rowsum[z * slab_stride_rowsum + m]
// (atomicAdd for EPI_F32_ATOMIC).
#include "common.h"
#include "../har_kernels.h"

namespace {

enum { EPI_F32 = 0, EPI_F32_ATOMIC = 1, EPI_BIAS_RELU = 2, EPI_BIAS = 3, EPI_RELU_GRAD = 4, EPI_BIAS_F32 = 5,
       EPI_F32_SLAB = 6 };


typedef __attribute__((ext_vector_type(4))) short s16x4_t;
typedef __attribute__((address_space(3))) s16x4_t lds_s16x4_t;

template <typename T> __device__ __forceinline__ float to_f(T v);
template <> __device__ __forceinline__ float to_f<bf16_t>(bf16_t v) { return bf2f(v); }
template <> __device__ __forceinline__ float to_f<float>(float v) { return v; }

// LDS pitches (elements): one 16-byte pad per row breaks power-of-two strides.
template <typename T, int ROWS, bool KMAJOR, int BK>
struct Img {
  static constexpr int EPV = 16 / sizeof(T);
  static constexpr int PITCH = KMAJOR ? BK + EPV : ROWS + EPV;
  static constexpr int SIZE = KMAJOR ? ROWS * PITCH : BK * PITCH;  // elements
};

// Global -> registers -> LDS stager for one ROWS x BK operand tile.
template <typename T, int ROWS, int NT, bool KMAJOR, int BK>
struct Stager {
  static constexpr int EPV = 16 / sizeof(T);
  static constexpr int NVEC = ROWS * BK / EPV;
  static constexpr int NV = (NVEC + NT - 1) / NT;  // 16-byte vectors per thread
  static constexpr int P = Img<T, ROWS, KMAJOR, BK>::PITCH;
  uint4 r[NV];

  __device__ __forceinline__ void load(const T* __restrict__ g, int ld, int row0, int nrows, int k0, int K, int tid) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int v = tid + i * NT;
      r[i] = make_uint4(0, 0, 0, 0);
      if (v < NVEC) {
        if (KMAJOR) {
          constexpr int VPR = BK / EPV;
          const int rr = v / VPR, kv = (v % VPR) * EPV;
          const int gr = row0 + rr, gk = k0 + kv;
          if (gr < nrows && gk < K) r[i] = *reinterpret_cast<const uint4*>(g + (size_t)gr * ld + gk);
        } else {
          constexpr int VPK = ROWS / EPV;
          const int k = v / VPK, rv = (v % VPK) * EPV;
          const int gk = k0 + k, gr = row0 + rv;
          if (gk < K && gr < nrows) r[i] = *reinterpret_cast<const uint4*>(g + (size_t)gk * ld + gr);
        }
      }
    }
  }

  __device__ __forceinline__ void store(T* __restrict__ lds, int tid) const {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int v = tid + i * NT;
      if (v < NVEC) {
        if (KMAJOR) {
          constexpr int VPR = BK / EPV;
          const int rr = v / VPR, kv = (v % VPR) * EPV;
          *reinterpret_cast<uint4*>(lds + rr * P + kv) = r[i];
        } else {
          constexpr int VPK = ROWS / EPV;
          const int k = v / VPK, rv = (v % VPK) * EPV;
          *reinterpret_cast<uint4*>(lds + k * P + rv) = r[i];
        }
      }
    }
  }
};

// MFMA operand fragment of rows row0..row0+15, k = kk + (k-slot of this lane).
template <typename T, int ROWS, bool KMAJOR, int BK> struct Frag;

template <int ROWS, int BK> struct Frag<bf16_t, ROWS, true, BK> {
  static constexpr int P = Img<bf16_t, ROWS, true, BK>::PITCH;
  __device__ __forceinline__ static bf16x8_t get(const bf16_t* lds, int row0, int kk, int lane) {
    return *reinterpret_cast<const bf16x8_t*>(lds + (row0 + (lane & 15)) * P + kk + (lane >> 4) * 8);
  }
};

template <int ROWS, int BK> struct Frag<bf16_t, ROWS, false, BK> {
  static constexpr int P = Img<bf16_t, ROWS, false, BK>::PITCH;
  // [BK][rows] image: lane 4q+p of each 16-lane group addresses row k0+q, columns 4p..4p+3 of a
  // 4x16 block; the transposing read returns column (lane&15) of the 4 rows.  Two reads cover
  // k = 8g .. 8g+7 for lane group g = lane>>4.
  __device__ __forceinline__ static bf16x8_t get(const bf16_t* lds, int row0, int kk, int lane) {
    const int li = lane & 15, g = lane >> 4;
    const int kq = kk + 8 * g + (li >> 2);
    const int col = row0 + 4 * (li & 3);
    const bf16_t* p0 = lds + kq * P + col;
    const bf16_t* p1 = p0 + 4 * P;
    s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(p0));
    s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(p1));
    typedef __attribute__((ext_vector_type(8))) short s16x8_t;
    s16x8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8_t, v);
  }
};

template <int ROWS, int BK> struct Frag<float, ROWS, true, BK> {
  static constexpr int P = Img<float, ROWS, true, BK>::PITCH;
  __device__ __forceinline__ static float get(const float* lds, int row0, int kk, int lane) {
    return lds[(row0 + (lane & 15)) * P + kk + (lane >> 4)];
  }
};

template <int ROWS, int BK> struct Frag<float, ROWS, false, BK> {
  static constexpr int P = Img<float, ROWS, false, BK>::PITCH;
  __device__ __forceinline__ static float get(const float* lds, int row0, int kk, int lane) {
    return lds[(kk + (lane >> 4)) * P + row0 + (lane & 15)];
  }
};

// Sum of the k-values a lane holds in an A fragment (fused bias-gradient row sums).
__device__ __forceinline__ float frag_sum(bf16x8_t a) {
  typedef __attribute__((ext_vector_type(4))) uint32_t u32x4_t;
  const u32x4_t w = __builtin_bit_cast(u32x4_t, a);
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) s += __uint_as_float(w[j] << 16) + __uint_as_float(w[j] & 0xffff0000u);
  return s;
}
__device__ __forceinline__ float frag_sum(float a) { return a; }

__device__ __forceinline__ f32x4_t mma(bf16x8_t a, bf16x8_t b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4_t mma(float a, float b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

template <typename T> struct KPerMma;
template <> struct KPerMma<bf16_t> { static constexpr int v = 32; };
template <> struct KPerMma<float> { static constexpr int v = 4; };

constexpr bool is_bf16_epi(int e) { return e == EPI_BIAS_RELU || e == EPI_BIAS || e == EPI_RELU_GRAD; }

template <typename T, int BM, int BN, int BK, int WM, int WN, bool A_KMAJOR, bool B_KMAJOR, int EPI>
__global__ __launch_bounds__(WM * WN * 64) void gemm_kernel(GemmParams p) {
  constexpr int NT = WM * WN * 64;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int RM = TM / 16, RN = TN / 16;
  constexpr int KPER = KPerMma<T>::v;
  using ImgA = Img<T, BM, A_KMAJOR, BK>;
  using ImgB = Img<T, BN, B_KMAJOR, BK>;
  constexpr int STAGE_BYTES = (ImgA::SIZE + ImgB::SIZE) * (int)sizeof(T);
  constexpr int CPITCH = BN + 8;  // bf16 epilogue image [BM][BN+8]
  constexpr int EPI_BYTES = is_bf16_epi(EPI) ? BM * CPITCH * 2 : 0;
  constexpr int SMEM = STAGE_BYTES > EPI_BYTES ? STAGE_BYTES : EPI_BYTES;
  __shared__ __attribute__((aligned(16))) unsigned char smem[SMEM];
  T* As = reinterpret_cast<T*>(smem);
  T* Bs = As + ImgA::SIZE;

  const T* __restrict__ A = reinterpret_cast<const T*>(p.A);
  const T* __restrict__ B = reinterpret_cast<const T*>(p.B);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int r16 = lane & 15, q = lane >> 4;

  // XCD-aware tile order over the (n, m) tile grid
  const int ntn = gridDim.x, ntm = gridDim.y;
  const int lin = xcd_remap(blockIdx.y * ntn + blockIdx.x, ntn * ntm);
  const int tn = lin % ntn;
  const int m0 = (lin / ntn) * BM, n0 = tn * BN;

  int kb = 0, ke = p.K;
  if (EPI == EPI_F32_ATOMIC || EPI == EPI_F32_SLAB) {
    kb = blockIdx.z * p.k_split;
    ke = min(p.K, kb + p.k_split);
  }
  // bias-gradient row sums come from the A fragments already in registers: waves of the
  // first N-column (wn == 0) of the first N tile add up their k-slots (free VALU work next
  // to the MFMAs), one cross-lane reduction at the end
  const bool rs_wave = p.rowsum != nullptr && tn == 0 && wn == 0;
  float rs[RM];
#pragma unroll
  for (int i = 0; i < RM; ++i) rs[i] = 0.f;

  f32x4_t acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  Stager<T, BM, NT, A_KMAJOR, BK> sa;
  Stager<T, BN, NT, B_KMAJOR, BK> sb;
  if (kb < ke) {
    sa.load(A, p.lda, m0, p.M, kb, ke, tid);
    sb.load(B, p.ldb, n0, p.N, kb, ke, tid);
  }
  for (int k0 = kb; k0 < ke; k0 += BK) {
    sa.store(As, tid);
    sb.store(Bs, tid);
    __syncthreads();
    if (k0 + BK < ke) {  // prefetch the next tile into registers while the MFMAs run
      sa.load(A, p.lda, m0, p.M, k0 + BK, ke, tid);
      sb.load(B, p.ldb, n0, p.N, k0 + BK, ke, tid);
    }
#pragma unroll
    for (int kk = 0; kk < BK; kk += KPER) {
#pragma unroll
      for (int i = 0; i < RM; ++i) {
        const auto a = Frag<T, BM, A_KMAJOR, BK>::get(As, wm * TM + i * 16, kk, lane);
        if (rs_wave) rs[i] += frag_sum(a);
#pragma unroll
        for (int j = 0; j < RN; ++j)
          acc[i][j] = mma(a, Frag<T, BN, B_KMAJOR, BK>::get(Bs, wn * TN + j * 16, kk, lane), acc[i][j]);
      }
    }
    __syncthreads();
  }

  if (rs_wave) {
#pragma unroll
    for (int i = 0; i < RM; ++i) {  // lanes r16, r16+16, r16+32, r16+48 hold the same row
      float v = rs[i];
      v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 32);
      const int m = m0 + wm * TM + i * 16 + r16;
      if (q == 0 && m < p.M) {
        if (EPI == EPI_F32_ATOMIC) atomicAdd(p.rowsum + m, p.alpha * v);
        else p.rowsum[(size_t)blockIdx.z * p.slab_stride_rowsum + m] = p.alpha * v;
      }
    }
  }

  // ---- epilogue ----
  if constexpr (is_bf16_epi(EPI)) {
    // 1) registers -> LDS image [BM][BN+8] (bias / relu applied here), 2) 16-byte row vectors out
    bf16_t* Cs = reinterpret_cast<bf16_t*>(smem);
#pragma unroll
    for (int j = 0; j < RN; ++j) {
      const int cl = wn * TN + j * 16 + r16;
      float bias = 0.f;
      if (EPI != EPI_RELU_GRAD && p.bias && n0 + cl < p.N) bias = p.bias[n0 + cl];
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = acc[i][j][r] + bias;
          if (EPI == EPI_BIAS_RELU) v = fmaxf(v, 0.f);
          Cs[(wm * TM + i * 16 + q * 4 + r) * CPITCH + cl] = f2bf(v);
        }
    }
    __syncthreads();
    bf16_t* Cb = reinterpret_cast<bf16_t*>(p.C);
    const bf16_t* mask = reinterpret_cast<const bf16_t*>(p.mask);
    constexpr int VPR = BN / 8;
    for (int v = tid; v < BM * VPR; v += NT) {
      const int rl = v / VPR, cl = (v % VPR) * 8;
      const int m = m0 + rl, n = n0 + cl;
      if (m >= p.M || n >= p.N) continue;
      union { uint4 u; bf16_t e[8]; } val;
      val.u = *reinterpret_cast<const uint4*>(Cs + rl * CPITCH + cl);
      if (EPI == EPI_RELU_GRAD) {
        union { uint4 u; bf16_t e[8]; } mk;
        mk.u = *reinterpret_cast<const uint4*>(mask + (size_t)m * p.ldmask + n);
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (!((mk.e[e] & 0x8000u) == 0 && mk.e[e] != 0)) val.e[e] = 0;
      }
      *reinterpret_cast<uint4*>(Cb + (size_t)m * p.ldc + n) = val.u;  // N % 8 == 0 (host contract)
    }
  } else {
    float* Cf = reinterpret_cast<float*>(p.C);
    if (EPI == EPI_F32_SLAB) Cf += (size_t)blockIdx.z * p.slab_stride;
#pragma unroll
    for (int j = 0; j < RN; ++j) {
      const int n = n0 + wn * TN + j * 16 + r16;
      const bool nok = n < p.N;
      float bias = 0.f;
      if (EPI == EPI_BIAS_F32 && nok && p.bias) bias = p.bias[n];
#pragma unroll
      for (int i = 0; i < RM; ++i) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm * TM + i * 16 + q * 4 + r;
          if (!(nok && m < p.M)) continue;
          const float v = acc[i][j][r];
          const size_t off = (size_t)m * p.ldc + n;
          if (EPI == EPI_F32 || EPI == EPI_F32_SLAB) Cf[off] = p.alpha * v;
          else if (EPI == EPI_F32_ATOMIC) atomicAdd(Cf + off, p.alpha * v);
          else if (EPI == EPI_BIAS_F32) Cf[off] = v + bias;
        }
      }
    }
  }
}

template <typename T, int BM, int BN, int BK, int WM, int WN, bool AK, bool BKm>
int launch_epi(const GemmParams& p, int epi, hipStream_t s) {
  dim3 grid((p.N + BN - 1) / BN, (p.M + BM - 1) / BM, 1);
  if (epi == EPI_F32_ATOMIC || epi == EPI_F32_SLAB) {
    if (p.k_split % BK) return -3;
    grid.z = (p.K + p.k_split - 1) / p.k_split;
  }
  dim3 block(WM * WN * 64);
  switch (epi) {
    case EPI_F32: gemm_kernel<T, BM, BN, BK, WM, WN, AK, BKm, EPI_F32><<<grid, block, 0, s>>>(p); break;
    case EPI_F32_ATOMIC: gemm_kernel<T, BM, BN, BK, WM, WN, AK, BKm, EPI_F32_ATOMIC><<<grid, block, 0, s>>>(p); break;
    case EPI_BIAS_F32: gemm_kernel<T, BM, BN, BK, WM, WN, AK, BKm, EPI_BIAS_F32><<<grid, block, 0, s>>>(p); break;
    case EPI_F32_SLAB: gemm_kernel<T, BM, BN, BK, WM, WN, AK, BKm, EPI_F32_SLAB><<<grid, block, 0, s>>>(p); break;
    default:
      if constexpr (sizeof(T) == 2) {
        if (p.N % 8) return -6;  // bf16 epilogues store 16-byte row vectors
        switch (epi) {
          case EPI_BIAS_RELU: gemm_kernel<T, BM, BN, BK, WM, WN, AK, BKm, EPI_BIAS_RELU><<<grid, block, 0, s>>>(p); break;
          case EPI_BIAS: gemm_kernel<T, BM, BN, BK, WM, WN, AK, BKm, EPI_BIAS><<<grid, block, 0, s>>>(p); break;
          case EPI_RELU_GRAD: gemm_kernel<T, BM, BN, BK, WM, WN, AK, BKm, EPI_RELU_GRAD><<<grid, block, 0, s>>>(p); break;
          default: return -1;
        }
      } else {
        return -1;  // bf16-output epilogues need bf16 inputs
      }
  }
  HAR_CHECK_LAUNCH();
  return 0;
}

// Tile ids (ops/gemm.py mirrors this table to size split-K):
//   0: 128x128 (2x2 waves)  1: 128x64 (2x2)  2: 128x32 (4x1)  3: 64x128 (1x4)  4: 64x64 (2x2)  5: 32x64 (1x2)
//   6: 128x256 (2x4, 512 threads)  7: 64x256 (1x4)            (all BK = 32)
//   8: 64x64 BK128  9: 128x128 BK64  10: 128x256 BK64  11: 32x64 BK128  12: 64x128 BK64  13: 128x64 BK128
//   18: 128x128 BK64 with 8 waves (4 x 2)   20: 64x64 BK128 with 8 waves (4 x 2) — the split-K
//   weight-gradient tiles (profiles/gemm_tile_sweep_v2.md: 8 waves of 32-row slices beat 4 waves,
//   2 x 4 and 4 x 4 arrangements)
template <typename T, bool AK, bool BKm>
int launch_tile(const GemmParams& p, int epi, hipStream_t s) {
  int tile = p.tile;
  if (tile < 0) {
    if (p.N <= 32) tile = 2;
    else if (p.N <= 64) tile = 1;
    else if (p.M <= 64) tile = 3;
    else tile = 0;
  }
  switch (tile) {
    case 0: return launch_epi<T, 128, 128, 32, 2, 2, AK, BKm>(p, epi, s);
    case 1: return launch_epi<T, 128, 64, 32, 2, 2, AK, BKm>(p, epi, s);
    case 2: return launch_epi<T, 128, 32, 32, 4, 1, AK, BKm>(p, epi, s);
    case 3: return launch_epi<T, 64, 128, 32, 1, 4, AK, BKm>(p, epi, s);
    case 4: return launch_epi<T, 64, 64, 32, 2, 2, AK, BKm>(p, epi, s);
    case 5: return launch_epi<T, 32, 64, 32, 1, 2, AK, BKm>(p, epi, s);
    case 6: return launch_epi<T, 128, 256, 32, 2, 4, AK, BKm>(p, epi, s);
    case 7: return launch_epi<T, 64, 256, 32, 1, 4, AK, BKm>(p, epi, s);
    case 8: return launch_epi<T, 64, 64, 128, 2, 2, AK, BKm>(p, epi, s);
    case 9: return launch_epi<T, 128, 128, 64, 2, 2, AK, BKm>(p, epi, s);
    case 10: return launch_epi<T, 128, 256, 64, 2, 4, AK, BKm>(p, epi, s);
    case 11: return launch_epi<T, 32, 64, 128, 1, 2, AK, BKm>(p, epi, s);
    case 12: return launch_epi<T, 64, 128, 64, 1, 4, AK, BKm>(p, epi, s);
    case 13: return launch_epi<T, 128, 64, 128, 2, 2, AK, BKm>(p, epi, s);
    case 18: return launch_epi<T, 128, 128, 64, 4, 2, AK, BKm>(p, epi, s);
    case 20: return launch_epi<T, 64, 64, 128, 4, 2, AK, BKm>(p, epi, s);
    default: return -4;
  }
}

template <typename T>
int gemm_dispatch(const GemmParams& p, int layout, int epi, hipStream_t s) {
  // layout bit0: A is M-major; bit1: B is N-major
  const int EPV = 16 / sizeof(T);
  bool a_mmajor = layout & 1, b_nmajor = layout & 2;
  // vector-load alignment contract (checked on the host side as well)
  if ((a_mmajor ? p.M : p.K) % EPV || (b_nmajor ? p.N : p.K) % EPV || p.lda % EPV || p.ldb % EPV) return -2;
  if ((epi == EPI_F32_ATOMIC || epi == EPI_F32_SLAB) && (p.k_split <= 0 || p.k_split % 32)) return -3;
  if (!a_mmajor && !b_nmajor) return launch_tile<T, true, true>(p, epi, s);
  if (!a_mmajor && b_nmajor) return launch_tile<T, true, false>(p, epi, s);
  if (a_mmajor && b_nmajor) return launch_tile<T, false, false>(p, epi, s);
  return -5;  // (A M-major, B K-major) is never needed
}

}  // namespace

extern "C" int har_gemm_bf16(const GemmParams* p, int layout, int epi, hipStream_t s) {
  return gemm_dispatch<bf16_t>(*p, layout, epi, s);
}

extern "C" int har_gemm_f32(const GemmParams* p, int layout, int epi, hipStream_t s) {
  return gemm_dispatch<float>(*p, layout, epi, s);
}
