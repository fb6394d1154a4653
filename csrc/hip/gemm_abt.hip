// Skinny bf16 GEMMs of psi_2's SplineConv:  C[N, M] = A[N, K] . Bt[M, K]^T
//
//   forward       Y  = X  . [W_0 | ... | W_25]   (K = 128,  M = 3328)
//   input grad    dX = dY . W^T                  (K = 3328, M = 128)
//
// Both are memory-bound (61 MB of Y written / dY read per layer); hipBLASLt
// picks MT256x192 / MT128x64 kernels that reach ~2.5-2.9 TB/s on them
// (tools/gemm_layouts.py).  Measured: this kernel reaches 2.2 / 1.4 TB/s
// (27.8 / 43.6 us vs hipBLASLt 22 / 21 us), so the model keeps hipBLASLt;
// the op stays available (bit-identical results, beta=1 accumulation).
// It is a plain LDS-tiled MFMA GEMM
// (v_mfma_f32_32x32x16_bf16, fp32 accumulators) specialised for the two
// shapes:
//
// * Bt is [M, K] row-major (contiguous in K) so both operands are read as
//   16-byte row chunks and the MFMA B fragment is an LDS row read;
// * 4 waves; each owns a WM x WN sub-tile of 32 x 32 MFMA tiles;
// * K is consumed in BK-wide tiles staged through two LDS buffers, the next
//   tile's global loads are issued into registers before the MFMAs of the
//   current one (one barrier per tile);
// * XCD-aware block order (blocks sharing A rows land on one XCD's L2);
// * epilogue: optional beta = 1 accumulation into C (gradient sums without
//   an add kernel), bf16 or fp32 output.
#include "common.h"

namespace dgmc {

typedef __bf16 gab_bf16x8 __attribute__((ext_vector_type(8)));
typedef float gab_f32x16 __attribute__((ext_vector_type(16)));
#define GAB_LDS __attribute__((address_space(3)))

template <int BM, int BN, int BK, int WM, int WN, int NBUF, typename TC>
__global__ __launch_bounds__(256) void gemm_abt_kernel(
    const __bf16* __restrict__ A, const __bf16* __restrict__ Bt,
    TC* __restrict__ C, int N, int M, int K, int64_t lda, int64_t ldb,
    int64_t ldc, int accumulate) {
  constexpr int KP = BK + 8;                 // padded LDS row
  constexpr int TM = WM / 32, TN = WN / 32;  // MFMA tiles per wave
  constexpr int WAVES_N = BN / WN;
  static_assert((BM / WM) * (BN / WN) == 4, "4 waves");
  constexpr int CH = BK / 8;                 // 16-byte chunks per row
  constexpr int A_CH = BM * CH, B_CH = BN * CH;
  constexpr int A_PT = (A_CH + 255) / 256, B_PT = (B_CH + 255) / 256;

  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  GAB_LDS __bf16* sA = (GAB_LDS __bf16*)smem_raw;   // [NBUF][BM][KP]
  GAB_LDS __bf16* sB = sA + NBUF * BM * KP;         // [NBUF][BN][KP]

  const int tid = threadIdx.x;
  const int nbm = (N + BM - 1) / BM, nbn = (M + BN - 1) / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int bm = bid / nbn, bn = bid % nbn;
  if (bm >= nbm) return;
  const int m0 = bm * BM, n0 = bn * BN;

  gab_bf16x8 ra[A_PT], rb[B_PT];
  auto load = [&](int k0) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < A_PT; ++i) {
      const int c = tid + i * 256;
      const int r = c / CH, kk = k0 + (c % CH) * 8;
      gab_bf16x8 v = {};
      if (c < A_CH && m0 + r < N && kk < K)
        v = *reinterpret_cast<const gab_bf16x8*>(A + (size_t)(m0 + r) * lda +
                                                 kk);
      ra[i] = v;
    }
#pragma unroll
    for (int i = 0; i < B_PT; ++i) {
      const int c = tid + i * 256;
      const int r = c / CH, kk = k0 + (c % CH) * 8;
      gab_bf16x8 v = {};
      if (c < B_CH && n0 + r < M && kk < K)
        v = *reinterpret_cast<const gab_bf16x8*>(Bt + (size_t)(n0 + r) * ldb +
                                                 kk);
      rb[i] = v;
    }
  };
  auto store = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < A_PT; ++i) {
      const int c = tid + i * 256;
      if (c < A_CH)
        *reinterpret_cast<GAB_LDS gab_bf16x8*>(
            sA + buf * BM * KP + (c / CH) * KP + (c % CH) * 8) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < B_PT; ++i) {
      const int c = tid + i * 256;
      if (c < B_CH)
        *reinterpret_cast<GAB_LDS gab_bf16x8*>(
            sB + buf * BN * KP + (c / CH) * KP + (c % CH) * 8) = rb[i];
    }
  };

  const int wave = tid / 64, lane = tid % 64;
  const int wm = (wave / WAVES_N) * WM, wn = (wave % WAVES_N) * WN;
  const int lr = lane & 31, lh = lane >> 5;
  gab_f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int nk = (K + BK - 1) / BK;
  load(0);
  store(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = NBUF == 2 ? (kt & 1) : 0;
    if (kt + 1 < nk) load((kt + 1) * BK);   // in flight during the MFMAs
    GAB_LDS const __bf16* a0 = sA + buf * BM * KP + (wm + lr) * KP + 8 * lh;
    GAB_LDS const __bf16* b0 = sB + buf * BN * KP + (wn + lr) * KP + 8 * lh;
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      gab_bf16x8 af[TM], bf[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        af[i] = *reinterpret_cast<GAB_LDS const gab_bf16x8*>(
            a0 + i * 32 * KP + 16 * s);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bf[j] = *reinterpret_cast<GAB_LDS const gab_bf16x8*>(
            b0 + j * 32 * KP + 16 * s);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          // Operands swapped (Bt . A^T): the accumulator's lane index is
          // the C row and its registers run along C columns, so the
          // epilogue writes 4 consecutive columns per 8-byte LDS store.
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
              bf[j], af[i], acc[i][j], 0, 0, 0);
    }
    if (NBUF == 2) {
      if (kt + 1 < nk) store(buf ^ 1);  // other buffer: free since last barrier
      __syncthreads();
    } else if (kt + 1 < nk) {
      __syncthreads();                  // single buffer: all reads done
      store(0);
      __syncthreads();
    }
  }

  // Epilogue through LDS: the C tile is assembled row-major in LDS (8-byte
  // writes of 4 consecutive columns), then written with coalesced 16-byte
  // row stores (2-byte scattered stores ran at ~1.7 TB/s).
  constexpr int CP = BN + (16 / (int)sizeof(TC));   // padded C row
  static_assert((size_t)BM * CP * sizeof(TC) <=
                    (size_t)NBUF * (BM + BN) * KP * 2,
                "C tile must fit in the operand LDS");
  GAB_LDS TC* sC = (GAB_LDS TC*)smem_raw;
  __syncthreads();   // operand tiles no longer read
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        // lane -> row wm + 32i + lr; regs 4g..4g+3 -> columns
        // wn + 32j + 8g + 4lh + 0..3
        const int row = wm + i * 32 + lr;
        const int col = wn + j * 32 + 8 * g + 4 * lh;
        TC pk[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) pk[e] = Cvt<TC>::from_f(acc[i][j][4 * g + e]);
        typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
        typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));
        if constexpr (sizeof(TC) == 2) {
          *reinterpret_cast<GAB_LDS u32x2*>(sC + row * CP + col) =
              *reinterpret_cast<const u32x2*>(pk);
        } else {
          *reinterpret_cast<GAB_LDS u32x4v*>(sC + row * CP + col) =
              *reinterpret_cast<const u32x4v*>(pk);
        }
      }
  __syncthreads();
  constexpr int VC = 16 / sizeof(TC);              // elements per 16 bytes
  constexpr int RCH = BN / VC;                     // 16-byte chunks per row
  for (int c = tid; c < BM * RCH; c += 256) {
    const int r = c / RCH, cc = (c % RCH) * VC;
    const int row = m0 + r, col = n0 + cc;
    if (row >= N || col >= M) continue;
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 raw = *reinterpret_cast<GAB_LDS const u32x4*>(sC + r * CP + cc);
    const TC* ev = reinterpret_cast<const TC*>(&raw);
    float v[VC], o[VC];
#pragma unroll
    for (int e = 0; e < VC; ++e) v[e] = Cvt<TC>::to_f(ev[e]);
    TC* p = C + (size_t)row * ldc + col;
    if (col + VC <= M && aligned16(p)) {
      if (accumulate) {
        load_vec<TC, VC>(p, o);
#pragma unroll
        for (int e = 0; e < VC; ++e) v[e] += o[e];
      }
      store_vec<TC, VC>(p, v);
    } else {
      for (int e = 0; e < VC && col + e < M; ++e)
        p[e] = Cvt<TC>::from_f(v[e] + (accumulate ? Cvt<TC>::to_f(p[e]) : 0.f));
    }
  }
}

template <int BM, int BN, int BK, int WM, int WN, int NBUF, typename TC>
static void launch_gab(const at::Tensor& A, const at::Tensor& Bt,
                       at::Tensor& C, bool accumulate) {
  const int N = A.size(0), K = A.size(1), M = Bt.size(0);
  const size_t lds = (size_t)NBUF * (BM + BN) * (BK + 8) * 2;
  auto kern = gemm_abt_kernel<BM, BN, BK, WM, WN, NBUF, TC>;
  static bool attr_set = false;
  if (!attr_set) {
    DGMC_CHECK_HIP(hipFuncSetAttribute(
        reinterpret_cast<const void*>(kern),
        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr_set = true;
  }
  const int blocks = ((N + BM - 1) / BM) * ((M + BN - 1) / BN);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), lds, stream(),
                     reinterpret_cast<const __bf16*>(A.data_ptr()),
                     reinterpret_cast<const __bf16*>(Bt.data_ptr()),
                     reinterpret_cast<TC*>(C.data_ptr()), N, M, K, A.stride(0),
                     Bt.stride(0), C.stride(0), accumulate ? 1 : 0);
}

// C = A . Bt^T (or C += ... with `out` given and accumulate).  A [N, K],
// Bt [M, K] bf16 with unit inner stride; rows 16-byte aligned.
at::Tensor gemm_abt(const at::Tensor& A, const at::Tensor& Bt,
                    const c10::optional<at::Tensor>& out, bool accumulate,
                    c10::optional<at::ScalarType> out_dtype) {
  TORCH_CHECK(A.is_cuda() && A.dim() == 2 && Bt.dim() == 2 &&
                  A.scalar_type() == at::kBFloat16 &&
                  Bt.scalar_type() == at::kBFloat16,
              "gemm_abt: bf16 2-D operands expected");
  TORCH_CHECK(A.stride(1) == 1 && Bt.stride(1) == 1 && A.size(1) == Bt.size(1),
              "gemm_abt: A [N, K], Bt [M, K] with unit inner stride");
  TORCH_CHECK(A.size(1) % 8 == 0 && A.stride(0) % 8 == 0 &&
                  Bt.stride(0) % 8 == 0 && aligned16(A.data_ptr()) &&
                  aligned16(Bt.data_ptr()),
              "gemm_abt: 16-byte aligned rows required");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(A.device());
  const int64_t N = A.size(0), M = Bt.size(0), K = A.size(1);
  at::Tensor C;
  if (out.has_value() && out->defined()) {
    C = *out;
    TORCH_CHECK(C.dim() == 2 && C.size(0) == N && C.size(1) == M &&
                    C.stride(1) == 1,
                "gemm_abt: out must be [N, M] with unit inner stride");
  } else {
    C = at::empty({N, M}, A.options().dtype(out_dtype.value_or(at::kBFloat16)));
    accumulate = false;
  }
  if (N == 0 || M == 0) return C;
  const bool f32 = C.scalar_type() == at::kFloat;
  TORCH_CHECK(f32 || C.scalar_type() == at::kBFloat16, "gemm_abt: out dtype");
  if (K <= 128) {
    // Other short K: one K tile, 128 x 128 output tiles, one LDS buffer.
    if (f32)
      launch_gab<128, 128, 128, 64, 64, 1, float>(A, Bt, C, accumulate);
    else
      launch_gab<128, 128, 128, 64, 64, 1, __hip_bfloat16>(A, Bt, C,
                                                           accumulate);
  } else {
    // Long K, narrow output (input gradient dX = dY W^T).
    // Double-buffered 64-wide K tiles (55 KB -> 2 blocks per CU).
    if (f32)
      launch_gab<64, 128, 64, 32, 64, 2, float>(A, Bt, C, accumulate);
    else
      launch_gab<64, 128, 64, 32, 64, 2, __hip_bfloat16>(A, Bt, C,
                                                         accumulate);
  }
  DGMC_CHECK_LAUNCH();
  return C;
}

}  // namespace dgmc
