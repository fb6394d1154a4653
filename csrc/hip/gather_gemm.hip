// Fused gather + MFMA GEMM for slot-structured message passing.
//
//   out[i, :] = act( sum_k Z_k[i, :] @ W_k + bias ),
//   Z_k[i, :] = sum_{e in (i, k)} a_e * X[j_e, :]
//
// is SplineConv (k = B-spline slot, 25 + root for psi_2) and RelConv (k in
// {in-flow, out-flow, root}) - see /root/reference/dgmc/models/spline.py:49
// and rel.py:26-31.  The unfused formulation (nn/conv.py) materialises
// Y = X @ [W_0 | ... | W_{S-1}] ([N, S*C], 61 MB for psi_2 at PascalVOC
// batch 512) and gathers it back; both passes ran at ~2.2 TB/s in hipBLASLt's
// skinny-GEMM kernels and the SpMM (45 us per layer).  Here Z never leaves
// the CU:
//
// * block = 64 destination rows x 128 output columns; 8 MFMA waves (tiles
//   of 32 x 32, v_mfma_f32_32x32x16_bf16, fp32 accumulators in registers)
//   and 4 gather waves;
// * the block's slot-CSR metadata (row pointers, source ids, coefficients)
//   and, when the sources are local, the window of X rows they touch are
//   staged in LDS once;
// * per slot: the gather waves build the Z_k tile (16-byte bf16 reads, fp32
//   FMA, one bf16 rounding) in one LDS buffer while the MFMA waves consume
//   the other - one barrier per slot; W_k^T slices stream through LDS
//   (coalesced loads two slots ahead).  W is re-read by every block, so
//   rows per block (64) set the L2 traffic: 144 blocks x 852 KB for psi_2;
// * epilogue: + bias, ReLU, store (bf16/fp32).
//
// The backward of the same layer is the same kernel on the transposed
// operator (slot-CSR of A^T has rows j*S + k) with W_k^T read in place, and
// it can write the gathered tiles (= dY = A^T G) for the weight-gradient
// GEMM (runtime/loopgrad.py stacks them across consensus steps).
#include "common.h"

#include <climits>

namespace dgmc {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));


constexpr int kGG_BM = 64;              // destination rows per block
constexpr int kGG_BN = 128;             // output columns per block
constexpr int kGG_ECAP = 2048;          // staged (col, val) entries per block
constexpr int kGG_LDS_MAX = 160 * 1024;
constexpr int kGG_MFMA_WAVES = 8;       // 2 row halves x 4 column quarters
constexpr int kGG_GATHER_THREADS = 256; // 4 gather waves
constexpr int kGG_THREADS = kGG_MFMA_WAVES * 64 + kGG_GATHER_THREADS;
__device__ long long g_gg_stamps[16];
#define GG_STAMP(i)                                                   \
  if ((dbg & 4) && blockIdx.x == 0 && blockIdx.y == 0 && tid == 0)    \
    g_gg_stamps[i] = wall_clock64();

__device__ __forceinline__ bf16x8_t pack_bf16x8(const float* v) {
  bf16x8_t r;
#pragma unroll
  for (int c = 0; c < 8; ++c) r[c] = (__bf16)v[c];
  return r;
}

// Block-shared state, all in the dynamic LDS region carved at 16-byte
// multiples (a static __shared__ in front of it would misalign every
// ds_*_b128 access) and typed address_space(3) so every access is a ds_*
// instruction (generic pointers become flat_* loads that wait on vmcnt and
// lgkmcnt together - measured 2x slower here).
struct GGShared {
  DGMC_LDS int* minmax;     // [2]
  DGMC_LDS __bf16* zbuf;    // [2][BM][KP]   gathered Z_k tiles
  DGMC_LDS __bf16* bbuf;    // [2][BN][KP]   W_k^T slices (B operand)
  DGMC_LDS __bf16* xwin;    // [wcap][KP]    source window of X
  DGMC_LDS int* srp;        // [BM*S + 1]
  DGMC_LDS int* ecol;       // [ECAP]
  DGMC_LDS float* eval;     // [ECAP]
};

// Gather Z_k of the block's rows into `zb` (gather waves).  Branch-free in
// the entry loop: every row slot of a thread issues its read each iteration
// (exhausted slots read a valid dummy with weight 0), so all of a thread's
// reads are in flight together.
template <int K, bool STAGED, bool WINDOWED, bool WRITE_Z>
__device__ __forceinline__ void gg_gather(
    const GGShared& sh, DGMC_LDS __bf16* zb, int k, int S, int rows,
    int ebase, int wlo, const __hip_bfloat16* __restrict__ X,
    const int* __restrict__ ecol, const float* __restrict__ eval,
    __hip_bfloat16* __restrict__ Z, int i0, int gt) {
  constexpr int BM = kGG_BM;
  constexpr int KP = K + 8;
  constexpr int LPR = K / 8;
  constexpr int RPP = kGG_GATHER_THREADS / LPR;
  constexpr int PASSES = BM >= RPP ? BM / RPP : 1;
  const int q = gt % LPR, rg = gt / LPR;
  int eb[PASSES], cnt[PASSES];
  int mx = 0;
#pragma unroll
  for (int p = 0; p < PASSES; ++p) {
    const int r = p * RPP + rg;
    eb[p] = 0;
    cnt[p] = 0;
    if (r < rows) {
      eb[p] = sh.srp[r * S + k] - ebase;
      cnt[p] = sh.srp[r * S + k + 1] - ebase - eb[p];
    }
    mx = max(mx, cnt[p]);
  }
  float acc[PASSES][8];
#pragma unroll
  for (int p = 0; p < PASSES; ++p)
#pragma unroll
    for (int c = 0; c < 8; ++c) acc[p][c] = 0.f;
  for (int t = 0; t < mx; ++t) {
    int j[PASSES];
    float a[PASSES];
#pragma unroll
    for (int p = 0; p < PASSES; ++p) {
      const bool v = t < cnt[p];
      const int e = v ? eb[p] + t : 0;
      if constexpr (STAGED) {
        j[p] = sh.ecol[e];
        a[p] = sh.eval[e];
      } else {
        j[p] = ecol[ebase + e];
        a[p] = eval[ebase + e];
      }
      if (!v) a[p] = 0.f;
    }
    bf16x8_t xv[PASSES];
#pragma unroll
    for (int p = 0; p < PASSES; ++p) {
      if constexpr (WINDOWED)
        xv[p] = *reinterpret_cast<DGMC_LDS const bf16x8_t*>(
            sh.xwin + (j[p] - wlo) * KP + q * 8);
      else
        xv[p] = *reinterpret_cast<const bf16x8_t*>(
            reinterpret_cast<const __bf16*>(X) + (size_t)j[p] * K + q * 8);
    }
#pragma unroll
    for (int p = 0; p < PASSES; ++p)
#pragma unroll
      for (int c = 0; c < 8; ++c)
        acc[p][c] = fmaf(a[p], (float)xv[p][c], acc[p][c]);
  }
#pragma unroll
  for (int p = 0; p < PASSES; ++p) {
    const int r = p * RPP + rg;
    if (r < BM) {
      const bf16x8_t v = pack_bf16x8(acc[p]);
      *reinterpret_cast<DGMC_LDS bf16x8_t*>(zb + r * KP + q * 8) = v;
      if constexpr (WRITE_Z) {
        if (r < rows)
          *reinterpret_cast<bf16x8_t*>(reinterpret_cast<__bf16*>(Z) +
                                       ((size_t)(i0 + r) * S + k) * K +
                                       q * 8) = v;
      }
    }
  }
}

// Warp-specialised: 8 MFMA waves run slot k while 4 gather waves build slot
// k+1 in the other Z buffer (one barrier per slot).  The W_k^T slice
// (BN x K) is streamed through LDS: coalesced 16-B loads of slot k+2 go to
// registers during slot k and are written to the free B buffer during slot
// k+1, so W (re-read by every block) moves at full cache-line efficiency.
// When the block's source rows span a small window (graphs batched as
// disjoint unions keep their edges local) that window of X is staged in LDS
// once and every gather is an LDS read; otherwise gathers read L2.
template <int K, bool WRITE_Z, typename TOUT>
__global__ __launch_bounds__(kGG_THREADS) void gather_gemm_kernel(
    const __hip_bfloat16* __restrict__ X, const int* __restrict__ srp,
    const int* __restrict__ ecol, const float* __restrict__ eval,
    const __hip_bfloat16* __restrict__ Wb, int64_t ss, int64_t sn,
    const float* __restrict__ bias, int relu, TOUT* __restrict__ out,
    __hip_bfloat16* __restrict__ Z, int Ndst, int S, int M, int wcap,
    int dbg) {
  constexpr int BM = kGG_BM, BN = kGG_BN;
  constexpr int KP = K + 8;          // padded LDS row (bf16 elements)
  constexpr int LPR = K / 8;         // 16-byte chunks per row
  constexpr int KS = K / 16;         // MFMA k-steps per slot
  constexpr int MT = kGG_MFMA_WAVES * 64;
  constexpr int BCH = BN * LPR;      // 16-byte chunks of one W_k^T slice
  constexpr int BPT = (BCH + MT - 1) / MT;  // chunks per MFMA thread

  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  DGMC_LDS char* smem = (DGMC_LDS char*)smem_raw;
  GGShared sh;
  sh.minmax = (DGMC_LDS int*)smem;
  sh.zbuf = (DGMC_LDS __bf16*)(smem + 16);
  sh.bbuf = sh.zbuf + 2 * BM * KP;
  sh.xwin = sh.bbuf + 2 * BN * KP;
  sh.srp = (DGMC_LDS int*)(sh.xwin + (size_t)wcap * KP);
  const int srp_n = BM * S + 1;
  sh.ecol = sh.srp + ((srp_n + 3) & ~3);
  sh.eval = (DGMC_LDS float*)(sh.ecol + kGG_ECAP);

  const int tid = threadIdx.x;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int i0 = tile * BM;
  const int n0 = blockIdx.y * BN;
  const int rows = min(BM, Ndst - i0);
  const int wave = tid / 64, lane = tid % 64;
  const bool mfma_role = wave < kGG_MFMA_WAVES;

  // W_k^T slice loads (MFMA threads): chunk c -> row n0 + c / LPR.
  const __bf16* W = reinterpret_cast<const __bf16*>(Wb);
  bf16x8_t breg[BPT];
  auto load_w = [&](int k) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < BPT; ++i) {
      const int c = tid + i * MT;
      const int n = n0 + c / LPR;
      if (c < BCH && n < M)
        breg[i] = *reinterpret_cast<const bf16x8_t*>(
            W + (size_t)k * ss + (size_t)n * sn + (c % LPR) * 8);
    }
  };
  auto store_w = [&](int buf) __attribute__((always_inline)) {
    DGMC_LDS __bf16* bb = sh.bbuf + buf * BN * KP;
#pragma unroll
    for (int i = 0; i < BPT; ++i) {
      const int c = tid + i * MT;
      if (c < BCH && n0 + c / LPR < M)
        *reinterpret_cast<DGMC_LDS bf16x8_t*>(bb + (c / LPR) * KP +
                                              (c % LPR) * 8) = breg[i];
    }
  };
  GG_STAMP(0);
  if (mfma_role) load_w(0);   // in flight during the metadata staging

  // ---- stage the block's slot-CSR metadata (+ source window) -----------
  const int nsrp = rows * S + 1;
  for (int t = tid; t < nsrp; t += kGG_THREADS)
    sh.srp[t] = srp[(size_t)i0 * S + t];
  if (tid == 0) {
    sh.minmax[0] = INT_MAX;
    sh.minmax[1] = -1;
  }
  __syncthreads();
  const int ebase = sh.srp[0];
  const int ecount = sh.srp[rows * S] - ebase;
  const bool staged = ecount <= kGG_ECAP;
  if (staged) {
    int lo = INT_MAX, hi = -1;
    for (int t = tid; t < ecount; t += kGG_THREADS) {
      const int j = ecol[ebase + t];
      sh.ecol[t] = j;
      sh.eval[t] = eval[ebase + t];
      lo = min(lo, j);
      hi = max(hi, j);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      lo = min(lo, __shfl_xor(lo, o));
      hi = max(hi, __shfl_xor(hi, o));
    }
    if (lane == 0 && hi >= 0) {
      atomicMin((int*)&sh.minmax[0], lo);
      atomicMax((int*)&sh.minmax[1], hi);
    }
  }
  __syncthreads();
  const int wlo = sh.minmax[0];
  const int whi = sh.minmax[1];
  const bool windowed = staged && whi >= 0 && whi - wlo + 1 <= wcap;
  if (windowed) {
    const int wrows = whi - wlo + 1;
    for (int t = tid; t < wrows * LPR; t += kGG_THREADS) {
      const int r = t / LPR, c = t % LPR;
      *reinterpret_cast<DGMC_LDS bf16x8_t*>(sh.xwin + r * KP + c * 8) =
          *reinterpret_cast<const bf16x8_t*>(
              reinterpret_cast<const __bf16*>(X) + (size_t)(wlo + r) * K +
              c * 8);
    }
  }
  if (mfma_role) {
    store_w(0);
    if (S > 1) load_w(1);
  }
  __syncthreads();

  const bool write_z = WRITE_Z && blockIdx.y == 0;
  const int gt = tid - MT;
  auto gather = [&](int k, int buf) __attribute__((always_inline)) {
    DGMC_LDS __bf16* zb = sh.zbuf + buf * BM * KP;
    if (write_z) {
      if (windowed)
        gg_gather<K, true, true, WRITE_Z>(sh, zb, k, S, rows, ebase, wlo, X,
                                          ecol, eval, Z, i0, gt);
      else if (staged)
        gg_gather<K, true, false, WRITE_Z>(sh, zb, k, S, rows, ebase, wlo, X,
                                           ecol, eval, Z, i0, gt);
      else
        gg_gather<K, false, false, WRITE_Z>(sh, zb, k, S, rows, ebase, wlo,
                                            X, ecol, eval, Z, i0, gt);
    } else {
      if (windowed)
        gg_gather<K, true, true, false>(sh, zb, k, S, rows, ebase, wlo, X,
                                        ecol, eval, Z, i0, gt);
      else if (staged)
        gg_gather<K, true, false, false>(sh, zb, k, S, rows, ebase, wlo, X,
                                         ecol, eval, Z, i0, gt);
      else
        gg_gather<K, false, false, false>(sh, zb, k, S, rows, ebase, wlo, X,
                                          ecol, eval, Z, i0, gt);
    }
  };

  // ---- MFMA tiles: wave (rh, cq) owns rows 32rh.., columns 32cq.. -------
  const int rh = (wave >> 2) & 1, cq = wave & 3;
  const int lr = lane & 31, lh = lane >> 5;
  const int col = n0 + cq * 32 + lr;
  const bool wave_active = mfma_role && n0 + cq * 32 < M;  // wave-uniform
  f32x16_t acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;

  GG_STAMP(1);
  if (!mfma_role) gather(0, 0);
  __syncthreads();
  GG_STAMP(2);
  for (int k = 0; k < S; ++k) {
    const int buf = k & 1;
    if (mfma_role && !(dbg & 2)) {
      // W_{k+1}: registers (loaded during slot k-1) -> the free B buffer;
      // then start W_{k+2}.
      if (k + 1 < S) store_w(buf ^ 1);
      if (k + 2 < S) load_w(k + 2);
      if (wave_active) {
        DGMC_LDS const __bf16* za =
            sh.zbuf + buf * BM * KP + (rh * 32 + lr) * KP + 8 * lh;
        DGMC_LDS const __bf16* zbp =
            sh.bbuf + buf * BN * KP + (cq * 32 + lr) * KP + 8 * lh;
#pragma unroll
        for (int s2 = 0; s2 < KS; ++s2) {
          const bf16x8_t a =
              *reinterpret_cast<DGMC_LDS const bf16x8_t*>(za + 16 * s2);
          const bf16x8_t b =
              *reinterpret_cast<DGMC_LDS const bf16x8_t*>(zbp + 16 * s2);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
        }
      }
    } else if (!mfma_role && k + 1 < S && !(dbg & 1)) {
      gather(k + 1, buf ^ 1);
    }
    __syncthreads();
  }

  GG_STAMP(3);
  // ---- epilogue ----------------------------------------------------------
  if (!wave_active || col >= M) return;
  const float b = bias ? bias[col] : 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = rh * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
    if (row < rows) {
      float v = acc[r] + b;
      if (relu) v = fmaxf(v, 0.f);
      out[(size_t)(i0 + row) * M + col] = Cvt<TOUT>::from_f(v);
    }
  }
}

static int gg_debug() {  // DGMC_GG_DEBUG: 1 = skip gathers, 2 = skip MFMA
  static int v = [] {
    const char* e = getenv("DGMC_GG_DEBUG");
    return e ? atoi(e) : 0;
  }();
  return v;
}

template <int K>
static size_t gg_fixed_lds(int S) {
  const size_t row_bytes = (size_t)(K + 8) * 2;
  const size_t srp_n = (size_t)kGG_BM * S + 1;
  return 16 + (size_t)2 * (kGG_BM + kGG_BN) * row_bytes +
         ((srp_n + 3) & ~size_t(3)) * 4 + (size_t)kGG_ECAP * 8;
}

template <int K, bool WRITE_Z, typename TOUT>
static void launch_gg(const at::Tensor& X, const at::Tensor& srp,
                      const at::Tensor& ecol, const at::Tensor& eval,
                      const at::Tensor& W, int64_t ss, int64_t sn,
                      const float* bias, bool relu, at::Tensor& out,
                      __hip_bfloat16* Z, int Ndst, int S, int M) {
  const size_t row_bytes = (size_t)(K + 8) * 2;
  const size_t fixed = gg_fixed_lds<K>(S);
  TORCH_CHECK(fixed <= (size_t)kGG_LDS_MAX,
              "gather_gemm: LDS budget exceeded (S=", S, ")");
  // Source window: whatever LDS is left (beyond it the block reads L2).
  const int wcap =
      (int)std::min<size_t>((kGG_LDS_MAX - fixed) / row_bytes, 1024);
  const size_t lds = fixed + (size_t)wcap * row_bytes;
  auto kern = gather_gemm_kernel<K, WRITE_Z, TOUT>;
  static bool attr_set = false;
  if (!attr_set) {
    DGMC_CHECK_HIP(hipFuncSetAttribute(
        reinterpret_cast<const void*>(kern),
        hipFuncAttributeMaxDynamicSharedMemorySize, kGG_LDS_MAX));
    attr_set = true;
  }
  dim3 grid((Ndst + kGG_BM - 1) / kGG_BM, (M + kGG_BN - 1) / kGG_BN);
  hipLaunchKernelGGL(kern, grid, dim3(kGG_THREADS), lds, stream(),
                     reinterpret_cast<const __hip_bfloat16*>(X.data_ptr()),
                     srp.data_ptr<int>(), ecol.data_ptr<int>(),
                     eval.data_ptr<float>(),
                     reinterpret_cast<const __hip_bfloat16*>(W.data_ptr()), ss,
                     sn, bias, relu ? 1 : 0,
                     reinterpret_cast<TOUT*>(out.data_ptr()), Z, Ndst, S, M,
                     wcap, gg_debug());
}

template <int K>
static void dispatch_gg(const at::Tensor& X, const at::Tensor& srp,
                        const at::Tensor& ecol, const at::Tensor& eval,
                        const at::Tensor& W, int64_t ss, int64_t sn,
                        const float* bias, bool relu, at::Tensor& out,
                        __hip_bfloat16* Z, int Ndst, int S, int M) {
  const bool f32 = out.scalar_type() == at::kFloat;
  if (Z) {
    if (f32)
      launch_gg<K, true, float>(X, srp, ecol, eval, W, ss, sn, bias, relu,
                                out, Z, Ndst, S, M);
    else
      launch_gg<K, true, __hip_bfloat16>(X, srp, ecol, eval, W, ss, sn, bias,
                                         relu, out, Z, Ndst, S, M);
  } else {
    if (f32)
      launch_gg<K, false, float>(X, srp, ecol, eval, W, ss, sn, bias, relu,
                                 out, Z, Ndst, S, M);
    else
      launch_gg<K, false, __hip_bfloat16>(X, srp, ecol, eval, W, ss, sn, bias,
                                          relu, out, Z, Ndst, S, M);
  }
}

// X [Nsrc, K] bf16; srp [Ndst*S + 1] int32 slot-CSR (row i*S + k);
// ecol/eval entries; W bf16 with element (slot k, out col n, in kk) at
// W[k*ss + n*sn + kk]; optional bias [M]; optional Z [Ndst*S, K] bf16 output.
// Debug: block (0,0) wall-clock stamps of the last launch with
// DGMC_GG_DEBUG & 4 (prologue start, metadata staged, slot 0 gathered, loop
// done).
at::Tensor gather_gemm_stamps() {
  long long h[16];
  DGMC_CHECK_HIP(hipMemcpyFromSymbol(h, HIP_SYMBOL(g_gg_stamps), sizeof(h)));
  at::Tensor t = at::empty({16}, at::kLong);
  memcpy(t.data_ptr<int64_t>(), h, sizeof(h));
  return t;
}

at::Tensor gather_gemm(const at::Tensor& X, const at::Tensor& srp,
                       const at::Tensor& ecol, const at::Tensor& eval,
                       const at::Tensor& W, int64_t ss, int64_t sn,
                       int64_t num_slots, int64_t M,
                       const c10::optional<at::Tensor>& bias, bool relu,
                       at::ScalarType out_dtype,
                       const c10::optional<at::Tensor>& Z) {
  TORCH_CHECK(X.is_cuda() && X.dim() == 2 && X.is_contiguous() &&
                  X.scalar_type() == at::kBFloat16,
              "gather_gemm: X must be contiguous bf16 [N, K]");
  TORCH_CHECK(W.scalar_type() == at::kBFloat16 && W.is_cuda(),
              "gather_gemm: W must be bf16");
  TORCH_CHECK(srp.scalar_type() == at::kInt && ecol.scalar_type() == at::kInt &&
                  eval.scalar_type() == at::kFloat,
              "gather_gemm: int32 index / fp32 value expected");
  TORCH_CHECK(out_dtype == at::kBFloat16 || out_dtype == at::kFloat,
              "gather_gemm: bf16 or fp32 output");
  const int K = X.size(1);
  const int S = num_slots;
  TORCH_CHECK(S >= 1 && (srp.numel() - 1) % S == 0,
              "gather_gemm: srp size must be Ndst*S + 1");
  const int Ndst = (srp.numel() - 1) / S;
  TORCH_CHECK(M > 0 && M % 32 == 0, "gather_gemm: M % 32 == 0");
  TORCH_CHECK(ss % 8 == 0 && sn % 8 == 0 && aligned16(W.data_ptr()) &&
                  aligned16(X.data_ptr()),
              "gather_gemm: 16-byte aligned operand rows required");
  // Bounds of the strided W reads.
  TORCH_CHECK((S - 1) * ss + (M - 1) * sn + K <= W.numel(),
              "gather_gemm: W too small for (S, M, K, strides)");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(X.device());
  at::Tensor out = at::empty({Ndst, M}, X.options().dtype(out_dtype));
  at::Tensor b_c;
  const float* bp = nullptr;
  if (bias.has_value() && bias->defined()) {
    b_c = bias->to(at::kFloat).contiguous();
    TORCH_CHECK(b_c.numel() == M, "gather_gemm: bias size");
    bp = b_c.data_ptr<float>();
  }
  __hip_bfloat16* zp = nullptr;
  if (Z.has_value() && Z->defined()) {
    TORCH_CHECK(Z->scalar_type() == at::kBFloat16 && Z->is_contiguous() &&
                    Z->numel() == (int64_t)Ndst * S * K &&
                    aligned16(Z->data_ptr()),
                "gather_gemm: Z must be contiguous bf16 [Ndst*S, K]");
    zp = reinterpret_cast<__hip_bfloat16*>(Z->data_ptr());
  }
  if (Ndst == 0) return out;
  switch (K) {
    case 32: dispatch_gg<32>(X, srp, ecol, eval, W, ss, sn, bp, relu, out, zp, Ndst, S, M); break;
    case 64: dispatch_gg<64>(X, srp, ecol, eval, W, ss, sn, bp, relu, out, zp, Ndst, S, M); break;
    case 128: dispatch_gg<128>(X, srp, ecol, eval, W, ss, sn, bp, relu, out, zp, Ndst, S, M); break;
    default: TORCH_CHECK(false, "gather_gemm: K must be 32, 64 or 128");
  }
  DGMC_CHECK_LAUNCH();
  return out;
}

}  // namespace dgmc
