// Split-K TN GEMM for weight gradients, fp32 in / fp32 out:
//
//   C[M, N] (+)= [A_0 | A_1 | ...]^T [B_0 | B_1 | ...],   A_p [K, m_p],
//                                                          B_q [K, n_q]
//
// K is the (long) node dimension and M x N the (small) weight: the weight
// gradients of RelConv's stacked node map (dY [N, 3C]^T x [N, C_in],
// /root/reference/dgmc/models/rel.py:28-31), of the encoders' final Linear
// on the concatenated features (g [N, C]^T x [x | h1 | h2 | h3], rel.py:92,
// spline.py:53) and of GIN / MLP Linears (gin.py:49, mlp.py:35) - the
// products that fell to hipBLASLt split-K batched GEMMs.  Parts are read in
// place (any row stride, widths % 4): the concatenations are never formed,
// and widths that are not multiples of the tile (300, 1068) read a zero page
// past their last column.
//
// Kernel: 128 x 128 output tiles of 4 waves (64 x 64 each, 2 x 2 MFMA blocks
// of 32 x 32), the K range of the grid split into equal 16-row-aligned
// chunks so that tiles x splits fills two workgroups per CU.  Each step
// stages 16 rows of both operand column blocks as k-major fp32 images
// ([16][128] floats, 8 KB each) by global_load_lds_dwordx4 into a ring of
// four LDS stages (three steps in flight while one is multiplied: HBM
// latency is hidden at two workgroups per CU); the MFMA operand of lane
// (i, h) is column i of rows 8 h .. + 7 (bf16x6) or row 2 s + h (exact f32):
// 32 consecutive floats per half wave, conflict-free ds_read_b32.
//
// Arithmetic: bf16x6 (each fp32 operand split into three bf16 terms in
// registers, six v_mfma_f32_32x32x16_bf16 per 16-deep step into a large-
// and a small-term accumulator - the scheme of slot_gemm_x6.hip, error at or
// below the exact fp32 chain's) or exact fp32 (v_mfma_f32_32x32x2_f32).
//
// Each (split, tile) writes its partial tile in the accumulator-native
// layout (float4 per lane, 1 KB per store instruction); the fold kernel sums
// the splits in index order (deterministic, no atomics) and writes or adds
// the [M, N] result with any row stride.
#include "common.h"

namespace dgmc {

namespace {

typedef float tn_f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 tn_bf16x8 __attribute__((ext_vector_type(8)));

constexpr int kTnT = 128;               // tile rows / columns
constexpr int kTnAlign = 32;            // split chunks: multiples of this
constexpr int kTnTile = kTnT * kTnT;    // floats per partial tile
constexpr int kTnMaxParts = 8;

struct TnParts {
  const float* p[kTnMaxParts];
  int ld[kTnMaxParts];
  int off[kTnMaxParts + 1];             // first column of each part
  int n;
};

__device__ __attribute__((aligned(16))) float g_tn_zero[4] = {0.f, 0.f, 0.f,
                                                             0.f};

__device__ __forceinline__ void tn_dma16(const float* g, DGMC_LDS float* l) {
  const unsigned m0 = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)l);
  asm volatile(
      "s_mov_b32 m0, %1\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %0, off"
      :: "v"(g), "s"(m0) : "memory", "m0");
}

// Barrier that also drains this wave's LDS operations: the MFMAs that
// consume a fragment may be scheduled after the barrier (they touch no
// memory), and with them the wait for the fragment's ds_read - which could
// then still be in flight when another wave overwrites the image after the
// barrier (observed as rare result differences of the cooperative-split
// kernel, whose plane images are rewritten right after it).
__device__ __forceinline__ void tn_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Row-0 address and row stride of logical column c (c % 4 == 0); null past
// the last part.
__device__ __forceinline__ const float* tn_col(const TnParts& P, int c,
                                               int& ld) {
  ld = 0;
  const float* r = nullptr;
#pragma unroll
  for (int q = 0; q < kTnMaxParts; ++q)
    if (r == nullptr && q < P.n && c >= P.off[q] && c < P.off[q + 1]) {
      r = P.p[q] + (c - P.off[q]);
      ld = P.ld[q];
    }
  return r;
}

template <int N>
__device__ __forceinline__ void tn_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" :: "n"(N) : "memory");
}

// Wait until at most `younger` stages' DMAs (D per stage and thread) are
// outstanding.
template <int D>
__device__ __forceinline__ void tn_wait_stages(int younger) {
  switch (younger) {
    case 0: tn_vmcnt<0>(); break;
    case 1: tn_vmcnt<D>(); break;
    case 2: tn_vmcnt<2 * D>(); break;
    case 3: tn_vmcnt<3 * D>(); break;
    case 4: tn_vmcnt<4 * D>(); break;
    default: tn_vmcnt<5 * D>(); break;
  }
}

// KR rows per staged step, NST stages in the LDS ring (NST - 1 steps in
// flight while one is multiplied).
template <bool X6, int KR, int NST, bool SCHED = false>
__global__ __launch_bounds__(256, 2) void gemm_tn_kernel(
    TnParts A, TnParts B, int K, int kchunk, int tiles_n, int tiles,
    float* __restrict__ part) {
  static_assert(KR % 16 == 0 && NST >= 2 && NST <= 6, "tn config");
  constexpr int IMG = KR * kTnT;              // floats per operand image
  constexpr int DJ = KR / 8;                  // DMAs per operand, thread
  __shared__ __attribute__((aligned(16))) float sA_[NST * IMG];
  __shared__ __attribute__((aligned(16))) float sB_[NST * IMG];
  DGMC_LDS float* sA = (DGMC_LDS float*)sA_;
  DGMC_LDS float* sB = (DGMC_LDS float*)sB_;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  // consecutive logical blocks = the tiles of one k chunk: they share its
  // operand rows in their XCD's L2
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int split = wg / tiles, tile = wg - split * tiles;
  const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
  const int k0 = split * kchunk;
  const int k1 = min(K, k0 + kchunk);
  const int nsteps = k1 > k0 ? (k1 - k0 + KR - 1) / KR : 0;

  // Staging: wave w's DMA j covers rows (KR / 4) w + 2 j (lanes 0-31) and
  // + 1 (lanes 32-63), 16-byte chunk lane % 32 of the 128 columns.
  const int cc = 4 * (lane & 31);
  int lda, ldb;
  const float* acol = tn_col(A, tm * kTnT + cc, lda);
  const float* bcol = tn_col(B, tn * kTnT + cc, ldb);
  const int wrow = (KR / 4) * wave;
  const int rbase = wrow + (lane >> 5);
  const float* zero = g_tn_zero;
  auto stage = [&](int s) {
    const int kb = k0 + s * KR;
    DGMC_LDS float* da = sA + (s % NST) * IMG;
    DGMC_LDS float* db = sB + (s % NST) * IMG;
#pragma unroll
    for (int j = 0; j < DJ; ++j) {
      const int row = kb + rbase + 2 * j;
      const bool in = row < k1;
      tn_dma16(in && acol ? acol + (size_t)row * lda : zero,
               da + (wrow + 2 * j) * kTnT);
      tn_dma16(in && bcol ? bcol + (size_t)row * ldb : zero,
               db + (wrow + 2 * j) * kTnT);
    }
  };

  const int i = lane & 31, h = lane >> 5;
  tn_f32x16 acc[2][2], acs[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = acs[a][b][r] = 0.f;
  const int am = wm * 64 + i, bn = wn * 64 + i;
  // SCHED: the splits of each 32 x 32 block's fragments are placed right
  // before their first MFMA and overlap the previous block's MFMAs
  // (scheduling regions fenced by sched_barrier): a0 b0 | MFMA(0,0) + b1 |
  // MFMA(0,1) + a1 | MFMA(1,0) MFMA(1,1) + the next 16 rows' a0 b0 | ...
  auto ld_split = [&](const DGMC_LDS float* img, int kr, int col,
                      tn_bf16x8 (&v)[3]) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      __bf16 hh, mm, ll;
      split3_bf16(img[(kr + j) * kTnT + col], hh, mm, ll);
      v[0][j] = hh;
      v[1][j] = mm;
      v[2][j] = ll;
    }
  };
  auto mfma6 = [&](int a, int b, const tn_bf16x8 (&av)[3],
                   const tn_bf16x8 (&bv)[3]) {
    tn_f32x16 sm = acs[a][b];
    sm = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[2], bv[0], sm, 0, 0, 0);
    sm = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[0], bv[2], sm, 0, 0, 0);
    sm = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[1], bv[1], sm, 0, 0, 0);
    sm = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[1], bv[0], sm, 0, 0, 0);
    sm = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[0], bv[1], sm, 0, 0, 0);
    acs[a][b] = sm;
    acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[0], bv[0],
                                                        acc[a][b], 0, 0, 0);
  };
  auto compute = [&](const DGMC_LDS float* la, const DGMC_LDS float* lb) {
    if (X6 && SCHED) {
      tn_bf16x8 a0[3], a1[3], b0[3], b1[3];
      ld_split(la, 8 * h, am, a0);
      ld_split(lb, 8 * h, bn, b0);
#pragma unroll
      for (int st = 0; st < KR / 16; ++st) {
        const int kr = 16 * st + 8 * h;
        __builtin_amdgcn_sched_barrier(0);
        mfma6(0, 0, a0, b0);
        ld_split(lb, kr, bn + 32, b1);
        __builtin_amdgcn_sched_barrier(0);
        mfma6(0, 1, a0, b1);
        ld_split(la, kr, am + 32, a1);
        __builtin_amdgcn_sched_barrier(0);
        mfma6(1, 0, a1, b0);
        mfma6(1, 1, a1, b1);
        if (st + 1 < KR / 16) {
          ld_split(la, kr + 16, am, a0);
          ld_split(lb, kr + 16, bn, b0);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      return;
    }
    if (X6) {
#pragma unroll
     for (int st = 0; st < KR / 16; ++st) {
      // one 16-deep step: lane (i, h) supplies rows 8 h .. 8 h + 7
      tn_bf16x8 av[2][3], bv[2][3];
      const int kr = 16 * st + 8 * h;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
#pragma unroll
        for (int a = 0; a < 2; ++a) {
          __bf16 hh, mm, ll;
          split3_bf16(la[(kr + j) * kTnT + am + 32 * a], hh, mm, ll);
          av[a][0][j] = hh;
          av[a][1][j] = mm;
          av[a][2][j] = ll;
        }
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          __bf16 hh, mm, ll;
          split3_bf16(lb[(kr + j) * kTnT + bn + 32 * b], hh, mm, ll);
          bv[b][0][j] = hh;
          bv[b][1][j] = mm;
          bv[b][2][j] = ll;
        }
      }
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          tn_f32x16 sm = acs[a][b];
          sm = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[a][2], bv[b][0], sm, 0, 0, 0);
          sm = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[a][0], bv[b][2], sm, 0, 0, 0);
          sm = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[a][1], bv[b][1], sm, 0, 0, 0);
          sm = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[a][1], bv[b][0], sm, 0, 0, 0);
          sm = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[a][0], bv[b][1], sm, 0, 0, 0);
          acs[a][b] = sm;
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
              av[a][0], bv[b][0], acc[a][b], 0, 0, 0);
        }
     }
      return;
    }
#pragma unroll
    for (int s = 0; s < KR / 2; ++s) {
      const int kk = 2 * s + h;
      float av[2], bv[2];
#pragma unroll
      for (int a = 0; a < 2; ++a) av[a] = la[kk * kTnT + am + 32 * a];
#pragma unroll
      for (int b = 0; b < 2; ++b) bv[b] = lb[kk * kTnT + bn + 32 * b];
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[a], bv[b],
                                                           acc[a][b], 0, 0, 0);
    }
  };

  // NST-stage ring: NST - 1 steps in flight while one is multiplied; the
  // stage refilled at step s was consumed at step s - 1 (its trailing
  // barrier orders the refill after every wave's reads).
  const int pro = min(nsteps, NST - 1);
  for (int s = 0; s < pro; ++s) stage(s);
  for (int s = 0; s < nsteps; ++s) {
    if (s + NST - 1 < nsteps) stage(s + NST - 1);
    tn_wait_stages<2 * DJ>(min(NST - 1, nsteps - 1 - s));
    tn_barrier();
    compute(sA + (s % NST) * IMG, sB + (s % NST) * IMG);
    tn_barrier();
  }

  // acc[a][b] register 4 q + r of lane (i, h): row m = tm 128 + wm 64 +
  // 32 a + 8 q + 4 h + r, column n = tn 128 + wn 64 + 32 b + i.  Stored as
  // [wave][a 2 + b][q][lane][r] (float4 per lane).
  float* out = part + ((size_t)split * tiles + tile) * kTnTile + wave * 4096;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float4 v;
        if (X6)
          v = make_float4(acc[a][b][4 * q] + acs[a][b][4 * q],
                          acc[a][b][4 * q + 1] + acs[a][b][4 * q + 1],
                          acc[a][b][4 * q + 2] + acs[a][b][4 * q + 2],
                          acc[a][b][4 * q + 3] + acs[a][b][4 * q + 3]);
        else
          v = make_float4(acc[a][b][4 * q], acc[a][b][4 * q + 1],
                          acc[a][b][4 * q + 2], acc[a][b][4 * q + 3]);
        *reinterpret_cast<float4*>(out + (((a * 2 + b) * 4 + q) * 64 + lane) *
                                             4) = v;
      }
}

// C[m, n] (+)= sum over splits (in order) of the partial tiles.
__global__ __launch_bounds__(256) void gemm_tn_fold_kernel(
    const float* __restrict__ part, int splits, int tiles, int tiles_n, int M,
    int N, float* __restrict__ C, int64_t ldc, int accumulate) {
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;   // float4 id
  if (g >= (int64_t)tiles * (kTnTile / 4)) return;
  const int tile = (int)(g / (kTnTile / 4));
  const int w = (int)(g - (int64_t)tile * (kTnTile / 4));
  const int wave = w >> 10, x = w & 1023;
  const int lane = x & 63, bq = x >> 6, blk = bq >> 2, q = bq & 3;
  const int a = blk >> 1, b = blk & 1;
  const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
  const int n = tn * kTnT + (wave & 1) * 64 + 32 * b + (lane & 31);
  const int m0 = tm * kTnT + (wave >> 1) * 64 + 32 * a + 8 * q +
                 4 * (lane >> 5);
  if (n >= N || m0 >= M) return;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  const float* p = part + (size_t)tile * kTnTile + 4 * (size_t)w;
  for (int sp = 0; sp < splits; ++sp) {
    const float4 v =
        *reinterpret_cast<const float4*>(p + (size_t)sp * tiles * kTnTile);
    s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
  }
  const float vv[4] = {s.x, s.y, s.z, s.w};
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int m = m0 + r;
    if (m < M) {
      float* dst = C + (size_t)m * ldc + n;
      *dst = accumulate ? *dst + vv[r] : vv[r];
    }
  }
}

TnParts tn_parts(at::TensorList parts, int64_t K, const char* what,
                 int64_t& width) {
  TORCH_CHECK(parts.size() >= 1 && parts.size() <= (size_t)kTnMaxParts,
              "gemm_tn_f32: 1..8 ", what, " parts");
  TnParts P{};
  width = 0;
  P.off[0] = 0;
  for (const at::Tensor& t : parts) {
    TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat &&
                    t.dim() == 2 && t.size(0) == K && t.stride(1) == 1 &&
                    t.size(1) % 4 == 0 && (t.stride(0) % 4 == 0 ||
                                           t.size(0) <= 1) &&
                    aligned16(t.data_ptr()),
                "gemm_tn_f32: ", what,
                " parts fp32 [K, w % 4] with 16-byte rows");
    P.p[P.n] = t.data_ptr<float>();
    P.ld[P.n] = (int)t.stride(0);
    width += t.size(1);
    ++P.n;
    P.off[P.n] = (int)width;
  }
  return P;
}


}  // namespace

// C = [a_parts]^T [b_parts] (fp32 [M, N]; written, or added into `out` when
// `accumulate`).  splits <= 0: chosen to fill two workgroups per CU.
at::Tensor gemm_tn_f32(at::TensorList a_parts, at::TensorList b_parts,
                       const c10::optional<at::Tensor>& out, bool accumulate,
                       bool x6, int64_t splits, int64_t cfg) {
  TORCH_CHECK(!a_parts.empty(), "gemm_tn_f32: A parts");
  const int64_t K = a_parts[0].size(0);
  int64_t M = 0, N = 0;
  const TnParts A = tn_parts(a_parts, K, "A", M);
  const TnParts B = tn_parts(b_parts, K, "B", N);
  TORCH_CHECK(K < (int64_t)1 << 31 && M * N < (int64_t)1 << 31,
              "gemm_tn_f32: sizes");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(a_parts[0].device());
  at::Tensor C;
  if (out.has_value() && out->defined()) {
    C = *out;
    TORCH_CHECK(C.is_cuda() && C.scalar_type() == at::kFloat &&
                    C.dim() == 2 && C.size(0) == M && C.size(1) == N &&
                    (C.stride(1) == 1 || N <= 1),
                "gemm_tn_f32: out fp32 [M, N] with unit column stride");
  } else {
    TORCH_CHECK(!accumulate, "gemm_tn_f32: accumulate needs out");
    C = at::empty({M, N}, a_parts[0].options());
  }
  if (M == 0 || N == 0) return C;
  const int64_t tiles_n = (N + kTnT - 1) / kTnT;
  const int64_t tiles = ((M + kTnT - 1) / kTnT) * tiles_n;
  // (the split count fixes the summation order: sized from the physical
  // CU count, never the DP reserve)
  const int64_t cus = device_cus(a_parts[0].device().index());
  if (splits <= 0)
    splits = std::max<int64_t>(1, (2 * cus + tiles - 1) / tiles);
  // equal chunks of whole 32-row steps
  const int64_t steps = std::max<int64_t>(1, (K + kTnAlign - 1) / kTnAlign);
  splits = std::min(splits, steps);
  const int64_t kchunk = ((steps + splits - 1) / splits) * kTnAlign;
  splits = std::max<int64_t>(1, (K + kchunk - 1) / kchunk);
  at::Tensor part = at::empty({splits * tiles * kTnTile},
                              a_parts[0].options());
  // cfg (measurement hook, tools/bench_gemm_tn.py; profiles/
  // bench_gemm_tn_r6_*.json): 0 = default (32-row steps, 2 stages, bf16x6
  // splits scheduled against the previous block's MFMAs), 1 = 16 x 4,
  // 2 = 32 x 3 (one workgroup per CU), 4 = 32 x 2 unscheduled.  (A
  // cooperative split - each element split once per workgroup into LDS
  // bf16 planes - measured no faster: LDS waits replaced the split VALU.)
  using KernT = void (*)(TnParts, TnParts, int, int, int, int, float*);
  KernT kern;
  switch (cfg) {
    case 1: kern = x6 ? gemm_tn_kernel<true, 16, 4>
                      : gemm_tn_kernel<false, 16, 4>; break;
    case 2: kern = x6 ? gemm_tn_kernel<true, 32, 3>
                      : gemm_tn_kernel<false, 32, 3>; break;
    case 4: kern = x6 ? gemm_tn_kernel<true, 32, 2>
                      : gemm_tn_kernel<false, 32, 2>; break;
    default: kern = x6 ? gemm_tn_kernel<true, 32, 2, true>
                       : gemm_tn_kernel<false, 32, 2>; break;
  }
  hipLaunchKernelGGL(kern, dim3((unsigned)(splits * tiles)), dim3(256), 0,
                     stream(), A, B, (int)K, (int)kchunk, (int)tiles_n,
                     (int)tiles, part.data_ptr<float>());
  DGMC_CHECK_LAUNCH();
  const int64_t n4 = tiles * (kTnTile / 4);
  hipLaunchKernelGGL(gemm_tn_fold_kernel, dim3((unsigned)((n4 + 255) / 256)),
                     dim3(256), 0, stream(), part.data_ptr<float>(),
                     (int)splits, (int)tiles, (int)tiles_n, (int)M, (int)N,
                     C.data_ptr<float>(), (int64_t)C.stride(0),
                     accumulate ? 1 : 0);
  DGMC_CHECK_LAUNCH();
  return C;
}

}  // namespace dgmc
