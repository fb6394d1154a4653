// Exact-fp32 NT GEMM over column chunks read in place, with an optional bias
// / ReLU epilogue:
//
//   Y[M, Nn] = act([A_0 | A_1 | ...] Bt^T + bias),   Bt [Nn, K] k-contiguous
//
// The A operand is a list of fp32 row-major parts (any row stride, any
// width that is a multiple of 4) - the concatenation is never formed.  Each
// part is consumed in 32-wide steps; a step's columns past the part's
// width, and the matching Bt columns, read a zero page instead of memory,
// so no part or weight needs padding (e.g. the 300-wide DBP15K features
// and the 1068-wide [x | h1 | h2 | h3] of RelCNN's final Linear,
// /root/reference/dgmc/models/rel.py:90-92, read in place).
//
// Uses: RelConv's stacked node map x [W1 | W2 | Wr]^T (rel.py:28-31) and
// the encoders' final Linear on the concatenated features (rel.py:92,
// spline.py:53) - the fp32 node GEMMs that ran on hipBLASLt.
//
// Kernel: v_mfma_f32_32x32x2_f32 (a k-ordered fmaf chain - exact fp32),
// 128x128, 128x64 or 64x64 tiles of 4 waves (picked for whole rounds of
// tiles on the chip), k consumed in 32-wide steps (a part's last step only as
// wide as needed) through two LDS stages filled by
// global_load_lds_dwordx4 (XOR-swizzled [row][32] images read as
// ds_read_b128, conflict-free), persistent grid of up to 2 workgroups per
// CU walking tiles in an XCD-aware order.  Rows past M are clamped on load
// and not stored.
#include "common.h"

namespace dgmc {

namespace {

typedef float gf_f32x16 __attribute__((ext_vector_type(16)));
typedef float gf_f32x4 __attribute__((ext_vector_type(4)));

constexpr int kGfBK = 32;           // k per staged step
constexpr int kGfMaxSteps = 96;     // 32-wide k steps (K <= 3072)
constexpr size_t kGfEpiBytes = 4 * 32 * 32 * 4;   // epilogue transpose

// A zero page for the DMAs of columns past a part's width.
__device__ __attribute__((aligned(16))) float g_gf_zero[4] = {0.f, 0.f, 0.f,
                                                             0.f};

// The k range as 32-wide steps over the parts (a part's last step may be
// narrower: its missing columns read the zero page).
struct GfSteps {
  const float* a[kGfMaxSteps];    // step start (part base + 32 j)
  int lda[kGfMaxSteps];
  int width[kGfMaxSteps];         // valid columns (<= 32)
  int boff[kGfMaxSteps];          // first Bt column of the step
  int n;
};

__device__ __forceinline__ void gf_dma16(const float* g, DGMC_LDS float* l) {
  const unsigned m0 = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)l);
  asm volatile(
      "s_mov_b32 m0, %1\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %0, off"
      :: "v"(g), "s"(m0) : "memory", "m0");
}

__device__ __forceinline__ void gf_barrier() {
  // (drain this wave's LDS reads first: gfx950 barriers do not wait for
  // them, and their consumers - MFMAs, no memory operands - may be
  // scheduled past the barrier while another wave's DMA refills the stage)
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

typedef __bf16 gf_bf16x8 __attribute__((ext_vector_type(8)));

// fp32 -> three bf16 terms hi + mid + lo (slot_gemm_x6.hip's split)
__device__ __forceinline__ void gf_split8(const gf_f32x4 u0, const gf_f32x4 u1,
                                          gf_bf16x8 (&v)[3]) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float x = e < 4 ? u0[e] : u1[e - 4];
    const __bf16 hh = (__bf16)x;
    const float r1 = x - (float)hh;
    const __bf16 mm = (__bf16)r1;
    v[0][e] = hh;
    v[1][e] = mm;
    v[2][e] = (__bf16)(r1 - (float)mm);
  }
}

// X6: the same tiles, staging and epilogue with the products on the bf16
// matrix cores as bf16x6 (slot_gemm_x6.hip: each fp32 operand split into
// three bf16 terms in registers, six v_mfma_f32_32x32x16_bf16 per 16-deep
// step into a large- and a small-term accumulator; max error below the
// exact-f32 chain's, tests/test_gemm_f32.py) - 2.7x fewer matrix-core
// cycles than v_mfma_f32_32x32x2_f32.
template <int MB, int NB, bool X6 = false, bool SCHED = false>
__global__ __launch_bounds__(256, 2) void gemm_nt_f32_kernel(
    GfSteps A, int M, const float* __restrict__ bt, int ldb, int Nn,
    const float* __restrict__ bias, int relu, float* __restrict__ Y,
    int ldy, int accumulate) {
  constexpr int TM = 64 * MB, TN = 64 * NB;
  __shared__ __attribute__((aligned(16))) float sA0_[TM * kGfBK];
  __shared__ __attribute__((aligned(16))) float sA1_[TM * kGfBK];
  __shared__ __attribute__((aligned(16))) float sB0_[TN * kGfBK];
  __shared__ __attribute__((aligned(16))) float sB1_[TN * kGfBK];
  DGMC_LDS float* sA0 = (DGMC_LDS float*)sA0_;
  DGMC_LDS float* sA1 = (DGMC_LDS float*)sA1_;
  DGMC_LDS float* sB0 = (DGMC_LDS float*)sB0_;
  DGMC_LDS float* sB1 = (DGMC_LDS float*)sB1_;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave & 1, wm = wave >> 1;
  const int ntn = (Nn + TN - 1) / TN, nk = A.n;
  const int U = ((M + TM - 1) / TM) * ntn;
  const int G = gridDim.x;
  int u = xcd_remap(blockIdx.x, G);
  if (u >= U) return;

  // Staging: wave w's A pieces j < 2 MB cover rows 16 MB w + 8 j + lane / 8,
  // its B pieces j < 2 NB rows 16 NB w + 8 j + lane / 8; lane L loads the
  // 4 floats of physical chunk L % 8 = logical (L % 8) ^ ((row >> 1) & 7).
  const int prow = lane >> 3;
  auto swz = [&](int row) { return 4 * ((lane & 7) ^ ((row >> 1) & 7)); };
  int arow[2 * MB];
  int brow0;
  auto tile_ptrs = [&](int uu) {
    const int m0 = (uu / ntn) * TM, n0 = (uu % ntn) * TN;
#pragma unroll
    for (int j = 0; j < 2 * MB; ++j)
      arow[j] = min(m0 + 16 * MB * wave + 8 * j + prow, M - 1);
    brow0 = n0 + 16 * NB * wave + prow;
  };
  const float* zero = g_gf_zero;
  auto stage = [&](int kc, DGMC_LDS float* da, DGMC_LDS float* db) {
    const float* ap = A.a[kc];
    const int lda = A.lda[kc], wid = A.width[kc], bo = A.boff[kc];
#pragma unroll
    for (int j = 0; j < 2 * MB; ++j) {
      const int row = 16 * MB * wave + 8 * j + prow;
      const int k = swz(row);
      gf_dma16(k < wid ? ap + (size_t)arow[j] * lda + k : zero,
               da + (16 * MB * wave + 8 * j) * kGfBK);
    }
#pragma unroll
    for (int j = 0; j < 2 * NB; ++j) {
      const int row = 16 * NB * wave + 8 * j + prow;
      const int k = swz(row);
      gf_dma16(k < wid && brow0 + 8 * j < Nn
                   ? bt + (size_t)(brow0 + 8 * j) * ldb + bo + k
                   : zero,
               db + (16 * NB * wave + 8 * j) * kGfBK);
    }
  };
  const int i = lane & 31, h = lane >> 5, sw = (i >> 1) & 7;
  int qoff[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) qoff[g] = 4 * ((2 * g + h) ^ sw);
  const int offN = (wn * 32 * NB + i) * kGfBK;
  const int offM = (wm * 32 * MB + i) * kGfBK;
  gf_f32x16 acc[NB][MB], acs[NB][MB];
#pragma unroll
  for (int a = 0; a < NB; ++a)
#pragma unroll
    for (int b = 0; b < MB; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = acs[a][b][r] = 0.f;
  // SCHED (bf16x6): each fragment is split right before its first MFMA
  // and overlaps the previous block's MFMAs (regions fenced by
  // sched_barrier): w0 x0 | MFMA(0,0) + the next fragment | ... | the last
  // block's MFMAs + the next 16-deep step's w0 x0.
  auto wsplit = [&](const DGMC_LDS float* lb, int st, int a,
                    gf_bf16x8 (&v)[3]) {
    const int c0 = 4 * st + 2 * h;
    gf_split8(*reinterpret_cast<const DGMC_LDS gf_f32x4*>(
                  lb + offN + a * 32 * kGfBK + 4 * (c0 ^ sw)),
              *reinterpret_cast<const DGMC_LDS gf_f32x4*>(
                  lb + offN + a * 32 * kGfBK + 4 * ((c0 + 1) ^ sw)),
              v);
  };
  auto xsplit = [&](const DGMC_LDS float* la, int st, int b,
                    gf_bf16x8 (&v)[3]) {
    const int c0 = 4 * st + 2 * h;
    gf_split8(*reinterpret_cast<const DGMC_LDS gf_f32x4*>(
                  la + offM + b * 32 * kGfBK + 4 * (c0 ^ sw)),
              *reinterpret_cast<const DGMC_LDS gf_f32x4*>(
                  la + offM + b * 32 * kGfBK + 4 * ((c0 + 1) ^ sw)),
              v);
  };
  auto mfma6 = [&](int a, int b, const gf_bf16x8 (&w)[3],
                   const gf_bf16x8 (&x)[3]) {
    gf_f32x16 sm = acs[a][b];
    sm = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[2], x[0], sm, 0, 0, 0);
    sm = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[0], x[2], sm, 0, 0, 0);
    sm = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[1], x[1], sm, 0, 0, 0);
    sm = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[1], x[0], sm, 0, 0, 0);
    sm = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[0], x[1], sm, 0, 0, 0);
    acs[a][b] = sm;
    acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[0], x[0],
                                                        acc[a][b], 0, 0, 0);
  };
  auto compute = [&](const DGMC_LDS float* la, const DGMC_LDS float* lb) {
    if (X6 && SCHED) {
      gf_bf16x8 w[NB][3], x[MB][3];
      wsplit(lb, 0, 0, w[0]);
      xsplit(la, 0, 0, x[0]);
#pragma unroll
      for (int st = 0; st < 2; ++st) {
#pragma unroll
        for (int a = 0; a < NB; ++a)
#pragma unroll
          for (int b = 0; b < MB; ++b) {
            __builtin_amdgcn_sched_barrier(0);
            mfma6(a, b, w[a], x[b]);
            // the next fragment in consumption order
            if (a == 0 && b + 1 < MB) {
              xsplit(la, st, b + 1, x[b + 1]);
            } else if (b == MB - 1 && a + 1 < NB) {
              wsplit(lb, st, a + 1, w[a + 1]);
            } else if (a == NB - 1 && b == MB - 1 && st == 0) {
              wsplit(lb, 1, 0, w[0]);
              xsplit(la, 1, 0, x[0]);
            }
          }
      }
      __builtin_amdgcn_sched_barrier(0);
      return;
    }
    if (X6) {
      // 16-deep step st: lane (i, h) supplies k = 16 st + 8 h .. + 7, the
      // logical chunks 4 st + 2 h and + 1 of its row image
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        gf_bf16x8 w[NB][3], x[MB][3];
        const int c0 = 4 * st + 2 * h;
        const int o0 = 4 * (c0 ^ sw), o1 = 4 * ((c0 + 1) ^ sw);
#pragma unroll
        for (int a = 0; a < NB; ++a)
          gf_split8(*reinterpret_cast<const DGMC_LDS gf_f32x4*>(
                        lb + offN + a * 32 * kGfBK + o0),
                    *reinterpret_cast<const DGMC_LDS gf_f32x4*>(
                        lb + offN + a * 32 * kGfBK + o1),
                    w[a]);
#pragma unroll
        for (int b = 0; b < MB; ++b)
          gf_split8(*reinterpret_cast<const DGMC_LDS gf_f32x4*>(
                        la + offM + b * 32 * kGfBK + o0),
                    *reinterpret_cast<const DGMC_LDS gf_f32x4*>(
                        la + offM + b * 32 * kGfBK + o1),
                    x[b]);
#pragma unroll
        for (int a = 0; a < NB; ++a)
#pragma unroll
          for (int b = 0; b < MB; ++b) {
            gf_f32x16 sm = acs[a][b];
            sm = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[a][2], x[b][0], sm, 0, 0, 0);
            sm = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[a][0], x[b][2], sm, 0, 0, 0);
            sm = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[a][1], x[b][1], sm, 0, 0, 0);
            sm = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[a][1], x[b][0], sm, 0, 0, 0);
            sm = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[a][0], x[b][1], sm, 0, 0, 0);
            acs[a][b] = sm;
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                w[a][0], x[b][0], acc[a][b], 0, 0, 0);
          }
      }
      return;
    }
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      gf_f32x4 fa[NB], fb[MB];
#pragma unroll
      for (int a = 0; a < NB; ++a)
        fa[a] = *reinterpret_cast<const DGMC_LDS gf_f32x4*>(
            lb + offN + a * 32 * kGfBK + qoff[g]);
#pragma unroll
      for (int b = 0; b < MB; ++b)
        fb[b] = *reinterpret_cast<const DGMC_LDS gf_f32x4*>(
            la + offM + b * 32 * kGfBK + qoff[g]);
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int a = 0; a < NB; ++a)
#pragma unroll
          for (int b = 0; b < MB; ++b)
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(
                fa[a][t], fb[b][t], acc[a][b], 0, 0, 0);
    }
  };
  // acc[a][b]: accumulator of Y^T block (n block a, m block b): lane i is
  // row m0 + 32 b + i, registers 4 q + r columns n0 + 32 a + 8 q + 4 h + r.
  // Each 32 x 32 block leaves through a wave-private LDS transpose (16-byte
  // chunk c of row r at c ^ (r & 7): conflict-free ds_write_b128 columns and
  // ds_read_b128 rows), so a store instruction writes 8 whole 128-byte row
  // segments instead of 32 rows x 32 bytes.
  extern __shared__ __attribute__((aligned(16))) float gf_epi_[];  // [4][32][32]
  DGMC_LDS float* epi = (DGMC_LDS float*)gf_epi_ + wave * 32 * 32;
  auto epilogue = [&](int uu) {
    const int mb = (uu / ntn) * TM + wm * 32 * MB;
    const int nb = (uu % ntn) * TN + wn * 32 * NB;
#pragma unroll
    for (int a = 0; a < NB; ++a) {
      float4 bv[4];
#pragma unroll
      for (int q = 0; q < 4; ++q)
        bv[q] = bias && nb + 4 * h + 32 * a + 8 * q < Nn
                    ? *reinterpret_cast<const float4*>(bias + nb + 4 * h +
                                                       32 * a + 8 * q)
                    : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int b = 0; b < MB; ++b) {
        asm volatile("" ::: "memory");
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float4 v;
          if (X6)
            v = make_float4(acc[a][b][4 * q] + acs[a][b][4 * q] + bv[q].x,
                            acc[a][b][4 * q + 1] + acs[a][b][4 * q + 1] +
                                bv[q].y,
                            acc[a][b][4 * q + 2] + acs[a][b][4 * q + 2] +
                                bv[q].z,
                            acc[a][b][4 * q + 3] + acs[a][b][4 * q + 3] +
                                bv[q].w);
          else
            v = make_float4(acc[a][b][4 * q] + bv[q].x,
                            acc[a][b][4 * q + 1] + bv[q].y,
                            acc[a][b][4 * q + 2] + bv[q].z,
                            acc[a][b][4 * q + 3] + bv[q].w);
          if (relu) {
            v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f);
            v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f);
          }
          *reinterpret_cast<DGMC_LDS gf_f32x4*>(
              epi + i * 32 + 4 * ((2 * q + h) ^ (i & 7))) =
              gf_f32x4{v.x, v.y, v.z, v.w};
#pragma unroll
          for (int r = 0; r < 4; ++r)
            acc[a][b][4 * q + r] = acs[a][b][4 * q + r] = 0.f;
        }
        asm volatile("" ::: "memory");
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int r = 8 * k + (lane >> 3);
          const gf_f32x4 v = *reinterpret_cast<const DGMC_LDS gf_f32x4*>(
              epi + r * 32 + 4 * ((lane & 7) ^ (r & 7)));
          const int m = mb + 32 * b + r;
          const int n = nb + 32 * a + 4 * (lane & 7);
          if (m < M && n < Nn) {
            float4* y = reinterpret_cast<float4*>(Y + (size_t)m * ldy + n);
            float4 o = make_float4(v[0], v[1], v[2], v[3]);
            if (accumulate) {
              const float4 p = *y;       // beta = 1 (e.g. a cat gradient)
              o.x += p.x; o.y += p.y; o.z += p.z; o.w += p.w;
            }
            *y = o;
          }
        }
      }
    }
  };
  tile_ptrs(u);
  stage(0, sA0, sB0);
  int kc = 0;
  auto step = [&](DGMC_LDS float* ca, DGMC_LDS float* cb, DGMC_LDS float* na,
                  DGMC_LDS float* nbuf) -> bool {
    const bool last_chunk = kc + 1 == nk;
    const int tu = last_chunk ? u + G : u;
    const int tkc = last_chunk ? 0 : kc + 1;
    const bool more = tu < U;
    if (more) {
      if (last_chunk) tile_ptrs(tu);
      stage(tkc, na, nbuf);
      // (this wave's 2 (MB + NB) pieces of the next chunk stay in flight)
      if constexpr (MB + NB == 4)
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else if constexpr (MB + NB == 3)
        asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    gf_barrier();
    compute(ca, cb);
    if (last_chunk) epilogue(u);
    gf_barrier();
    u = tu;
    kc = tkc;
    return more;
  };
  while (step(sA0, sB0, sA1, sB1) && step(sA1, sB1, sA0, sB0)) {
  }
}

int gf_num_cus(int dev) {
  static int cached[64] = {0};
  if (dev < 0 || dev >= 64) dev = 0;
  if (cached[dev] == 0) {
    hipDeviceProp_t prop;
    DGMC_CHECK_HIP(hipGetDeviceProperties(&prop, dev));
    cached[dev] = prop.multiProcessorCount;
  }
  return usable_cus(cached[dev]);
}

}  // namespace

// Y = act([parts] bt^T + bias).  parts: fp32 [M, K_p] views (unit column
// stride, 16-byte aligned rows, K_p % 4 == 0); bt: fp32 [Nn, sum K_p] with
// unit column stride (Nn % 4 == 0; a partial last tile column block is
// masked); out: optional [M, Nn] view to write, or to add into
// (accumulate: beta = 1).
at::Tensor gemm_nt_f32(at::TensorList parts, const at::Tensor& bt,
                       const c10::optional<at::Tensor>& bias, bool relu,
                       const c10::optional<at::Tensor>& out, bool x6,
                       bool accumulate, int64_t sched) {
  TORCH_CHECK(parts.size() >= 1, "gemm_nt_f32: at least one part");
  const int64_t M = parts[0].size(0);
  GfSteps A{};
  int64_t K = 0;
  for (const at::Tensor& p : parts) {
    TORCH_CHECK(p.is_cuda() && p.scalar_type() == at::kFloat &&
                    p.dim() == 2 && p.size(0) == M && p.stride(1) == 1 &&
                    p.size(1) % 4 == 0 && p.stride(0) % 4 == 0 &&
                    aligned16(p.data_ptr()),
                "gemm_nt_f32: parts fp32 [M, K_p % 4] with 16-byte rows");
    for (int64_t c0 = 0; c0 < p.size(1); c0 += kGfBK) {
      TORCH_CHECK(A.n < kGfMaxSteps, "gemm_nt_f32: K too large");
      A.a[A.n] = p.data_ptr<float>() + c0;
      A.lda[A.n] = (int)p.stride(0);
      A.width[A.n] = (int)std::min<int64_t>(kGfBK, p.size(1) - c0);
      A.boff[A.n] = (int)(K + c0);
      ++A.n;
    }
    K += p.size(1);
  }
  TORCH_CHECK(bt.is_cuda() && bt.scalar_type() == at::kFloat &&
                  bt.dim() == 2 && bt.size(1) == K && bt.stride(1) == 1 &&
                  bt.stride(0) % 4 == 0 && aligned16(bt.data_ptr()) &&
                  bt.size(0) % 4 == 0,
              "gemm_nt_f32: Bt fp32 [Nn % 4, K] with 16-byte rows");
  const int64_t Nn = bt.size(0);
  const float* bp = nullptr;
  if (bias.has_value() && bias->defined()) {
    TORCH_CHECK(bias->scalar_type() == at::kFloat && bias->is_contiguous() &&
                    bias->numel() == Nn && aligned16(bias->data_ptr()),
                "gemm_nt_f32: fp32 bias [Nn]");
    bp = bias->data_ptr<float>();
  }
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(bt.device());
  at::Tensor Y;
  if (out.has_value() && out->defined()) {
    Y = *out;
    TORCH_CHECK(Y.scalar_type() == at::kFloat && Y.dim() == 2 &&
                    Y.size(0) == M && Y.size(1) == Nn && Y.stride(1) == 1 &&
                    Y.stride(0) % 4 == 0 && aligned16(Y.data_ptr()),
                "gemm_nt_f32: out fp32 [M, Nn] with 16-byte rows");
  } else {
    TORCH_CHECK(!accumulate, "gemm_nt_f32: accumulate needs out");
    Y = at::empty({M, Nn}, bt.options());
  }
  if (M == 0 || Nn == 0) return Y;
  const int cus = gf_num_cus(bt.device().index());
  // Tile shape: the fewest tile-time units on 2 blocks per CU - whole
  // rounds of 2 * CUs tiles, each costing its MFMA work with the smaller
  // tiles' lower operand reuse (measured ~1.12x / ~1.3x per MAC).
  // bf16x6 (2.7x fewer matrix-core cycles) is bound by the operand
  // traffic: 128x64 tiles cost no more per MAC than 128x128 there
  // (tools/micro/bench_nt_f32_cfg.py, DBP15K final Linear 1068 -> 256:
  // 237 / 229 / 215 / 226 us for the picks / 128x128 / 128x64 / 64x64).
  struct Cfg { int mb, nb; double eff; };
  const Cfg cfgs[3] = {{2, 2, 1.0}, {2, 1, x6 ? 1.0 : 1.12},
                       {1, 1, 1.3}};
  int pick = -1;
  double best = 0.0;
  int64_t tiles = 0;
  const int forced = diag_env_int("DGMC_GEMM_F32_CFG", 0);   // diag build
  for (int c = 0; c < 3; ++c) {
    const int TM = 64 * cfgs[c].mb, TN = 64 * cfgs[c].nb;
    // (a tile column block past Nn is masked: its share of wasted MACs
    // counts against the shape)
    const int64_t tn = (Nn + TN - 1) / TN;
    const int64_t t = ((M + TM - 1) / TM) * tn;
    const int64_t rounds = (t + 2 * cus - 1) / (2 * cus);
    const double cost = (double)rounds * cfgs[c].mb * cfgs[c].nb *
                        cfgs[c].eff * ((double)(tn * TN) / (double)Nn);
    if (forced ? c == forced - 1 : (pick < 0 || cost < best - 1e-9)) {
      pick = c;
      best = cost;
      tiles = t;
    }
  }
  TORCH_CHECK(pick >= 0, "gemm_nt_f32: no tile shape for Nn = ", Nn);
  const int64_t blocks = std::min<int64_t>(tiles, 2 * (int64_t)cus);
  // sched (measurement hook): bf16x6 with the fragment splits scheduled
  // against the previous block's MFMAs.
  auto kern = x6 ? (sched ? (pick == 0 ? gemm_nt_f32_kernel<2, 2, true, true>
                             : pick == 1 ? gemm_nt_f32_kernel<2, 1, true, true>
                                         : gemm_nt_f32_kernel<1, 1, true, true>)
                          : (pick == 0 ? gemm_nt_f32_kernel<2, 2, true>
                             : pick == 1 ? gemm_nt_f32_kernel<2, 1, true>
                                         : gemm_nt_f32_kernel<1, 1, true>))
                 : (pick == 0 ? gemm_nt_f32_kernel<2, 2>
                              : pick == 1 ? gemm_nt_f32_kernel<2, 1>
                                          : gemm_nt_f32_kernel<1, 1>);
  DGMC_CHECK_HIP(hipFuncSetAttribute(
      reinterpret_cast<const void*>(kern),
      hipFuncAttributeMaxDynamicSharedMemorySize, (int)kGfEpiBytes));
  hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(256), kGfEpiBytes,
                     stream(), A,
                     (int)M, bt.data_ptr<float>(), (int)bt.stride(0),
                     (int)Nn, bp, relu ? 1 : 0, Y.data_ptr<float>(),
                     (int)Y.stride(0), accumulate ? 1 : 0);
  DGMC_CHECK_LAUNCH();
  return Y;
}

}  // namespace dgmc
