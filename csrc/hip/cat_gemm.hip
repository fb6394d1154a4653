// Concatenate-and-project for the consensus MLP's first layer:
//
//   out[M, 128] = [X_0 | X_1 | ... ] @ W^T,   W: [128, K], K = sum_i K_i
//   (optionally also writing the concatenation O = [X_0 | X_1 | ...])
//
// In DGMC's consensus loop (reference dgmc.py:174-179 with psi_2 =
// SplineCNN(cat=True), spline.py:51) the MLP's first Linear - folded with
// psi_2's final Linear (models/dgmc.py) - is applied to the concatenation of
// psi_2's input and its two layer outputs.  Eager: a cat kernel writing the
// [M, 384] features plus a library GEMM whose [M, 128] output has only
// ceil(M / 160) = 128 output tiles for 256 CUs (12.8 us measured).  Here:
// one workgroup (8 waves) per CU, each wave taking 16-row tiles, W staged
// once per workgroup in LDS (row pitch K + 8 bf16: conflict-free ds_read_b128 fragment reads),
// each wave's 16 rows x K read straight from the three inputs into A
// fragments of v_mfma_f32_16x16x32_bf16 (16-byte loads), 8 column blocks x
// K/32 MFMAs per wave.  The concatenation, needed only by the loop-shared
// weight gradient, is written from the same A fragments into the loop's
// stacked buffer (no cat, no later cat_rows).
#include "common.h"

namespace dgmc {

namespace {

typedef __bf16 cg_bf16x8 __attribute__((ext_vector_type(8)));
typedef float cg_f32x4 __attribute__((ext_vector_type(4)));

constexpr int kCgN = 128;          // output columns
constexpr int kCgWaves = 8;
constexpr int kCgMaxIn = 4;
constexpr int kCgMaxKs = 16;       // K <= 512 (LDS: N x (K + 8) bf16)

struct CatGemmArgs {
  const __bf16* x[kCgMaxIn];
  int64_t ldx[kCgMaxIn];
  int koff[kCgMaxIn + 1];          // column offset of each input in [0, K]
  int nin;
};

}  // namespace

template <int KS, int NC>
__global__ __launch_bounds__(kCgWaves * 64, 1) void cat_gemm_kernel(
    const CatGemmArgs args, const __bf16* __restrict__ W,
    __bf16* __restrict__ out, __bf16* __restrict__ ocat, int M) {
  constexpr int K = 32 * KS;
  constexpr int N = kCgN * NC;              // output columns
  constexpr int WP = K + 8;                 // LDS row pitch (bf16)
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  DGMC_LDS __bf16* Ws = (DGMC_LDS __bf16*)smem_raw;   // [N][WP]
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;

  const int rl = lane & 15, kq = 8 * (lane >> 4);
  // 16-row tiles dealt wave-major across the grid: tile t goes to workgroup
  // t % grid, so every CU gets work even when M / 16 < 8 x grid.
  const int ntiles = (M + 15) / 16;
  cg_bf16x8 a[KS];
  auto load_a = [&](int tile) __attribute__((always_inline)) {
    const int row = 16 * tile + rl;
    const bool rv = row < M;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int k = 32 * ks + kq;
      int i = 0;
#pragma unroll
      for (int q = 1; q < kCgMaxIn; ++q)
        if (q < args.nin && k >= args.koff[q]) i = q;
      const cg_bf16x8 z = {};
      a[ks] = rv ? *reinterpret_cast<const cg_bf16x8*>(
                       args.x[i] + (int64_t)row * args.ldx[i] +
                       (k - args.koff[i]))
                 : z;
    }
  };
  // The first tile's A fragments are requested before the W staging so
  // both memory round trips overlap.
  const int tile0 = wave * gridDim.x + blockIdx.x;
  if (tile0 < ntiles) load_a(tile0);

  // Stage W [N, K] (16-byte chunks): every chunk of this thread is requested
  // before the first LDS store (one memory round trip instead of one per
  // chunk - the loop form waited on each load before its store).
  {
    constexpr int kChunks = N * K / 8;
    constexpr int kPer = (kChunks + kCgWaves * 64 - 1) / (kCgWaves * 64);
    cg_bf16x8 wv[kPer];
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int c = tid + u * kCgWaves * 64;
      if (c < kChunks) {
        const int n = c / (K / 8), k8 = c - n * (K / 8);
        wv[u] = *reinterpret_cast<const cg_bf16x8*>(W + (int64_t)n * K +
                                                     8 * k8);
      }
    }
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int c = tid + u * kCgWaves * 64;
      if (c < kChunks) {
        const int n = c / (K / 8), k8 = c - n * (K / 8);
        *reinterpret_cast<DGMC_LDS cg_bf16x8*>(Ws + n * WP + 8 * k8) = wv[u];
      }
    }
  }
  __syncthreads();

  for (int tile = tile0; tile < ntiles; tile += kCgWaves * gridDim.x) {
    if (tile != tile0) load_a(tile);
    const int row = 16 * tile + rl;
    const bool rv = row < M;
    if (ocat && rv) {
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
        *reinterpret_cast<cg_bf16x8*>(ocat + (int64_t)row * K + 32 * ks +
                                      kq) = a[ks];
    }
#pragma unroll
    for (int nc = 0; nc < NC; ++nc) {       // 128-column chunks of the output
      cg_f32x4 acc[8];
#pragma unroll
      for (int nb = 0; nb < 8; ++nb) acc[nb] = cg_f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        cg_bf16x8 b[8];
#pragma unroll
        for (int nb = 0; nb < 8; ++nb)
          b[nb] = *reinterpret_cast<DGMC_LDS const cg_bf16x8*>(
              Ws + (kCgN * nc + 16 * nb + rl) * WP + 32 * ks + kq);
#pragma unroll
        for (int nb = 0; nb < 8; ++nb)
          acc[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[ks], b[nb],
                                                            acc[nb], 0, 0, 0);
        // One k-step of B fragments in flight: without this fence the
        // scheduler hoists all K/32 x 8 fragment reads (spills at K = 384).
        __builtin_amdgcn_sched_barrier(0);
      }
      // lane holds C[(lane >> 4) * 4 + r][128 nc + 16 nb + (lane & 15)]
      const int r0 = 16 * tile + 4 * (lane >> 4);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (r0 + r >= M) continue;
        __bf16* orow = out + (int64_t)(r0 + r) * N + kCgN * nc + rl;
#pragma unroll
        for (int nb = 0; nb < 8; ++nb) orow[16 * nb] = (__bf16)acc[nb][r];
      }
    }
  }
}

// xs: inputs [M, K_i] bf16 (unit column stride, 16-byte aligned rows,
// K_i % 32 == 0); W [128, K] bf16 contiguous; ocat: optional [M, K] bf16
// contiguous receiving the concatenation.  Returns out [M, 128] bf16.
at::Tensor cat_gemm(at::TensorList xs, const at::Tensor& W,
                    const c10::optional<at::Tensor>& ocat) {
  const int nin = (int)xs.size();
  TORCH_CHECK(nin >= 1 && nin <= kCgMaxIn, "cat_gemm: 1..4 inputs");
  TORCH_CHECK(W.is_cuda() && W.scalar_type() == at::kBFloat16 && W.dim() == 2 &&
                  W.size(0) % kCgN == 0 && W.size(0) <= 3 * kCgN &&
                  W.is_contiguous() && aligned16(W.data_ptr()),
              "cat_gemm: W contiguous bf16 [128 | 256 | 384, K]");
  const int NC = (int)W.size(0) / kCgN;
  const int64_t M = xs[0].size(0);
  CatGemmArgs args{};
  int K = 0;
  for (int i = 0; i < nin; ++i) {
    const at::Tensor& x = xs[i];
    TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 &&
                    x.dim() == 2 && x.size(0) == M && x.stride(1) == 1 &&
                    x.size(1) % 32 == 0 && x.stride(0) % 8 == 0 &&
                    aligned16(x.data_ptr()) && x.device() == W.device(),
                "cat_gemm: inputs bf16 [M, K_i], K_i % 32 == 0, 16-byte "
                "aligned rows");
    args.x[i] = reinterpret_cast<const __bf16*>(x.data_ptr());
    args.ldx[i] = x.stride(0);
    args.koff[i] = K;
    K += (int)x.size(1);
  }
  args.koff[nin] = K;
  args.nin = nin;
  TORCH_CHECK(W.size(1) == K, "cat_gemm: W [N, sum K_i]");
  const int KS = K / 32;
  TORCH_CHECK(KS >= 1 && KS <= kCgMaxKs, "cat_gemm: K in [32, 512]");
  __bf16* op = nullptr;
  if (ocat.has_value() && ocat->defined()) {
    TORCH_CHECK(ocat->scalar_type() == at::kBFloat16 && ocat->is_contiguous() &&
                    ocat->numel() == M * K && aligned16(ocat->data_ptr()),
                "cat_gemm: ocat contiguous bf16 [M, K]");
    op = reinterpret_cast<__bf16*>(ocat->data_ptr());
  }
  TORCH_CHECK(M < INT32_MAX, "cat_gemm: M range");
  at::Tensor out = at::empty({M, (int64_t)kCgN * NC}, W.options());
  if (M == 0) return out;
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(W.device());
  const size_t lds = (size_t)kCgN * NC * (K + 8) * 2;
  TORCH_CHECK(lds <= 160 * 1024, "cat_gemm: W too large for LDS staging");
  // One workgroup per CU (W fills ~100 KB of LDS), waves over 16-row tiles.
  const int tiles = (int)((M + 15) / 16);
  const int grid = std::max(1, std::min((tiles + kCgWaves - 1) / kCgWaves *
                                            kCgWaves, 256));
#define DGMC_CG_CASE(ks, nc)                                                  \
  if (KS == ks && NC == nc) {                                                 \
    static bool attr = false;                                                 \
    if (!attr) {                                                              \
      DGMC_CHECK_HIP(hipFuncSetAttribute(                                     \
          reinterpret_cast<const void*>(cat_gemm_kernel<ks, nc>),             \
          hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));           \
      attr = true;                                                            \
    }                                                                         \
    hipLaunchKernelGGL((cat_gemm_kernel<ks, nc>), dim3(grid),                 \
                       dim3(kCgWaves * 64), lds, stream(), args,              \
                       reinterpret_cast<const __bf16*>(W.data_ptr()),         \
                       reinterpret_cast<__bf16*>(out.data_ptr()), op,         \
                       (int)M);                                               \
    launched = true;                                                          \
  }
  bool launched = false;
  DGMC_CG_CASE(4, 1)
  DGMC_CG_CASE(8, 1)
  DGMC_CG_CASE(12, 1)
  DGMC_CG_CASE(16, 1)
  DGMC_CG_CASE(4, 2)
  DGMC_CG_CASE(4, 3)
  DGMC_CG_CASE(8, 2)
  TORCH_CHECK(launched, "cat_gemm: unsupported (K, N) = (", K, ", ",
              kCgN * NC, ")");
#undef DGMC_CG_CASE
  DGMC_CHECK_LAUNCH();
  return out;
}

}  // namespace dgmc
