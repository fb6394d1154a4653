// Weight gradient of a slot-structured graph convolution WITHOUT the
// per-slot gradient stack:
//
//   dW_k = sum_u sum_{e in slot k} a_e X_u[j_e]^T G_u[i_e]      (128 x 128)
//
// for every slot k of SplineConv's operator (/root/reference/dgmc/models/
// spline.py:49; entry e = (target i, source j, slot k, value a)), summed over
// the U uses of the layer inside the consensus loop (runtime/loopgrad.py
// keeps each use's input X_u and output gradient G_u, [N, 128] each).
//
// The unfused backward writes dY = A^T G ([N*S, 128], 73 MB per psi_2 use)
// with an SpMM and contracts the 10-use stack with one long-K GEMM
// (X^T dY: 730 MB read).  Here the reduction runs directly over the
// (use, entry) pairs of each slot: rows X_u[j_e] (scaled by a_e) and
// G_u[i_e] are gathered (L2/MALL-resident: the stacks are 28 MB) into LDS
// and contracted on MFMA - no dY is ever written.
//
// Mapping (gfx950): one workgroup = 8 waves (2 per SIMD) = one (slot,
// split) pair; K = 32 pairs per step; the 128 x 128 fp32 result is split
// 2 (channels) x 4 (outputs) over the waves (64 x 32 each).  Operands are
// staged row-major ([pair][channel], 256-B rows, XOR-swizzled) and read
// K-contiguous with ds_read_b64_tr_b16 (CDNA4 transposed LDS read) for both
// the A (X^T) and B (G) fragments of v_mfma_f32_16x16x32_bf16.  Row loads
// are register-prefetched two steps ahead; LDS is double-buffered; pairs
// iterate entry-chunk-major / use-minor so each thread's (j, i, a) is loaded
// once per U steps.  Per-split partials are folded by reduce_add_rows
// (deterministic; no float atomics).
#include "common.h"

#include <type_traits>

namespace dgmc {

namespace {

typedef __bf16 sw_bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 sw_bf16x4 __attribute__((ext_vector_type(4)));
typedef float sw_f32x4 __attribute__((ext_vector_type(4)));
typedef short sw_i16x4 __attribute__((ext_vector_type(4)));

constexpr int kSwC = 128;          // channels (in == out)
constexpr int kSwK = 32;           // pairs per step
constexpr int kSwThreads = 512;    // 8 waves
constexpr int kSwTile = kSwK * kSwC;   // bf16 elements per staged operand
constexpr int kSwEB = 1024;        // entries staged in LDS per batch
constexpr int kSwMaxU = 16;        // uses addressed through the pointer table

// Per-use row bases of X and G (kernel argument: captured by value in a
// hipGraph; the uses' tensors are read in place, no stacking copy).
struct SwUses {
  const __bf16* x[kSwMaxU];
  const __bf16* g[kSwMaxU];
};

// Byte offset of 16-byte chunk `ch` of row `row` in a [rows][128 bf16]
// image (256-B rows): the XOR keeps both ds_write_b128 row stores and the
// 4-row transposed reads bank-conflict free (cdna_hip_programming.md T10,
// image (b)).
__device__ __forceinline__ int sw_off(int row, int ch) {
  return 256 * row + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}

// 16x16x32 operand fragment (8 K-consecutive elements of one column) of a
// row-major [K][128] LDS image: rows 8g..8g+7 of column block `cb` (16
// columns) for lane group g - two transposed 4-row reads.
__device__ __forceinline__ sw_bf16x8 sw_frag(const DGMC_LDS char* img,
                                             int cb, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  sw_bf16x4 v[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int row = 8 * g + 4 * h + q;
    const DGMC_LDS char* a = img + sw_off(row, 2 * cb + (p >> 1)) + 8 * (p & 1);
    // Whole-vector bit casts: element-wise short->bf16 conversion of the
    // v4i16 result was miscompiled (lanes 2-3 replaced by 0-1).
    v[h] = __builtin_bit_cast(
        sw_bf16x4, __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                       (DGMC_LDS sw_i16x4*)a));
  }
  return __builtin_shufflevector(v[0], v[1], 0, 1, 2, 3, 4, 5, 6, 7);
}

}  // namespace

__global__ __launch_bounds__(kSwThreads, 1) void slot_wgrad_kernel(
    const SwUses P, const int* __restrict__ esrc, const int* __restrict__ edst,
    const float* __restrict__ evals, const int* __restrict__ soff, int S,
    int U, int N, int nsplit, float* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) char lds[2][2][kSwTile * 2];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int k = blockIdx.x / nsplit, s = blockIdx.x % nsplit;
  const int e_lo = soff[k], Ek = soff[k + 1] - e_lo;
  const int nch = (Ek + kSwK - 1) / kSwK;
  const int ch0 = (int)((long long)nch * s / nsplit);
  const int ch1 = (int)((long long)nch * (s + 1) / nsplit);

  // Staging role: thread -> (pair row r, 16-byte chunk c) of both operands.
  const int r = tid >> 4, c = tid & 15;
  // The split's entries (source, target, value) are staged in LDS once per
  // batch of kSwEB, so the step loop issues only the row gathers (no
  // dependent index loads, no branches: the compiler keeps the register
  // prefetch two steps deep instead of draining vmcnt every step).
  __shared__ int ej_s[kSwEB], ei_s[kSwEB];
  __shared__ float ea_s[kSwEB];
  sw_bf16x8 xr[2], gr[2];
  float ar[2];

  // Accumulators: wave (mi, nw) owns channels 64mi.., outputs 32nw...
  const int mi = wave >> 2, nw = wave & 3;
  sw_f32x4 acc[4][2];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = sw_f32x4{0.f, 0.f, 0.f, 0.f};

  for (int cb0 = ch0; cb0 < ch1; cb0 += kSwEB / kSwK) {
    const int cb1 = min(ch1, cb0 + kSwEB / kSwK);
    const int nent = (cb1 - cb0) * kSwK;
    __syncthreads();                      // previous batch fully consumed
    for (int i = tid; i < kSwEB; i += kSwThreads) {
      const int e = cb0 * kSwK + i;
      const bool v = i < nent && e < Ek;   // the rest: row 0, weight 0
      ej_s[i] = v ? esrc[e_lo + e] : 0;
      ei_s[i] = v ? edst[e_lo + e] : 0;
      ea_s[i] = v ? evals[e_lo + e] : 0.f;
    }
    __syncthreads();
    const int steps = (cb1 - cb0) * U;
    // (chunk, use) of the step being issued, advanced without division.
    int iu = 0, ic = 0;
    // Register slots are compile-time (the step loop is unrolled by two):
    // a runtime slot index turns the prefetch registers into a dynamically
    // indexed array, which the compiler resolves with selects that wait on
    // every load.
    auto issue = [&](auto slot_c) __attribute__((always_inline)) {
      constexpr int slot = decltype(slot_c)::value;
      const int e = ic * kSwK + r;
      const bool in = e < nent;           // past the batch: weight 0, row 0
      const int ee = in ? e : 0;
      // iu is wave-uniform: the table lookup is a scalar load.
      xr[slot] = *reinterpret_cast<const sw_bf16x8*>(
          P.x[iu] + (size_t)ej_s[ee] * kSwC + 8 * c);
      gr[slot] = *reinterpret_cast<const sw_bf16x8*>(
          P.g[iu] + (size_t)ei_s[ee] * kSwC + 8 * c);
      ar[slot] = in ? ea_s[ee] : 0.f;
      const bool wrap = iu + 1 == U;
      iu = wrap ? 0 : iu + 1;
      ic += wrap ? 1 : 0;
    };
    auto stage = [&](auto slot_c) __attribute__((always_inline)) {
      constexpr int slot = decltype(slot_c)::value, buf = slot;
      sw_bf16x8 xs;
#pragma unroll
      for (int q = 0; q < 8; ++q)
        xs[q] = (__bf16)((float)xr[slot][q] * ar[slot]);
      *reinterpret_cast<DGMC_LDS sw_bf16x8*>(
          (DGMC_LDS char*)lds[buf][0] + sw_off(r, c)) = xs;
      *reinterpret_cast<DGMC_LDS sw_bf16x8*>(
          (DGMC_LDS char*)lds[buf][1] + sw_off(r, c)) = gr[slot];
    };
    using S0 = std::integral_constant<int, 0>;
    using S1 = std::integral_constant<int, 1>;
    issue(S0{});
    issue(S1{});
    stage(S0{});
    __syncthreads();
    // One step: MFMAs on buffer BUF while the rows of step t+2 load into the
    // registers just staged, then stage step t+1 into the other buffer.
    auto step = [&](auto buf_c) __attribute__((always_inline)) {
      constexpr int buf = decltype(buf_c)::value;
      issue(buf_c);
      const DGMC_LDS char* A = (const DGMC_LDS char*)lds[buf][0];
      const DGMC_LDS char* B = (const DGMC_LDS char*)lds[buf][1];
      sw_bf16x8 af[4], bf[2];
#pragma unroll
      for (int a = 0; a < 4; ++a) af[a] = sw_frag(A, 4 * mi + a, lane);
#pragma unroll
      for (int b = 0; b < 2; ++b) bf[b] = sw_frag(B, 2 * nw + b, lane);
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[a], bf[b],
                                                              acc[a][b], 0, 0,
                                                              0);
      stage(std::integral_constant<int, buf ^ 1>{});
      __syncthreads();
    };
    // Steps past `steps` (odd count) carry zero weights.
    for (int t = 0; t < steps; t += 2) {
      step(S0{});
      step(S1{});
    }
  }

  // Partial [split][slot][channel][output] (fp32): lane holds rows
  // 4(lane/16) + r of column lane%16 of each 16x16 block.
  float* out = part + ((size_t)s * S + k) * kSwC * kSwC;
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = 64 * mi + 16 * a + 4 * (lane >> 4) + q;
        const int colo = 32 * nw + 16 * b + (lane & 15);
        out[(size_t)row * kSwC + colo] = acc[a][b][q];
      }
}

static void check_pairs(const at::Tensor& esrc, const at::Tensor& edst,
                        const at::Tensor& evals, const at::Tensor& soff) {
  TORCH_CHECK(esrc.scalar_type() == at::kInt &&
                  edst.scalar_type() == at::kInt &&
                  evals.scalar_type() == at::kFloat &&
                  soff.scalar_type() == at::kInt && esrc.is_contiguous() &&
                  edst.is_contiguous() && evals.is_contiguous() &&
                  soff.is_contiguous() && esrc.numel() == edst.numel() &&
                  esrc.numel() == evals.numel(),
              "slot_wgrad: int32 esrc/edst/soff, fp32 evals");
}

static at::Tensor launch_slot_wgrad(const SwUses& P, int U, int64_t N,
                                    const at::Tensor& like,
                                    const at::Tensor& esrc,
                                    const at::Tensor& edst,
                                    const at::Tensor& evals,
                                    const at::Tensor& soff, int64_t nsplit) {
  check_pairs(esrc, edst, evals, soff);
  const int64_t S = soff.numel() - 1;
  TORCH_CHECK(S >= 1 && nsplit >= 1 && S * nsplit < (1 << 30),
              "slot_wgrad: slots / splits");
  TORCH_CHECK(N < INT32_MAX / kSwC, "slot_wgrad: size range");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(like.device());
  at::Tensor part = at::empty({nsplit, S * kSwC * kSwC},
                              like.options().dtype(at::kFloat));
  hipLaunchKernelGGL(slot_wgrad_kernel, dim3(S * nsplit), dim3(kSwThreads), 0,
                     stream(), P, esrc.data_ptr<int>(), edst.data_ptr<int>(),
                     evals.data_ptr<float>(), soff.data_ptr<int>(), (int)S,
                     U, (int)N, (int)nsplit, part.data_ptr<float>());
  DGMC_CHECK_LAUNCH();
  return part;
}

// X, G [U*N, 128] bf16 (use-major stacks); esrc/edst [E] int32 source /
// target node of each operator entry, evals [E] fp32, all grouped by slot
// with offsets soff [S+1]; returns per-split partials [nsplit, S*128*128]
// fp32 of dW [S, 128, 128] (channel, output).
at::Tensor slot_wgrad(const at::Tensor& X, const at::Tensor& G,
                      const at::Tensor& esrc, const at::Tensor& edst,
                      const at::Tensor& evals, const at::Tensor& soff,
                      int64_t U, int64_t nsplit) {
  TORCH_CHECK(X.is_cuda() && X.scalar_type() == at::kBFloat16 &&
                  X.is_contiguous() && X.dim() == 2 && X.size(1) == kSwC &&
                  G.sizes() == X.sizes() &&
                  G.scalar_type() == at::kBFloat16 && G.is_contiguous(),
              "slot_wgrad: X, G contiguous bf16 [U*N, 128]");
  TORCH_CHECK(U >= 1 && U <= kSwMaxU && X.size(0) % U == 0,
              "slot_wgrad: 1 <= U <= 16, rows % U");
  TORCH_CHECK(aligned16(X.data_ptr()) && aligned16(G.data_ptr()),
              "slot_wgrad: 16-byte aligned operands");
  const int64_t N = X.size(0) / U;
  SwUses P{};
  const __bf16* xb = reinterpret_cast<const __bf16*>(X.data_ptr());
  const __bf16* gb = reinterpret_cast<const __bf16*>(G.data_ptr());
  for (int u = 0; u < U; ++u) {
    P.x[u] = xb + (size_t)u * N * kSwC;
    P.g[u] = gb + (size_t)u * N * kSwC;
  }
  return launch_slot_wgrad(P, (int)U, N, X, esrc, edst, evals, soff, nsplit);
}

// Same, with the U uses' X_u / G_u [N, 128] read in place (no stacks).
at::Tensor slot_wgrad_list(at::TensorList xs, at::TensorList gs,
                           const at::Tensor& esrc, const at::Tensor& edst,
                           const at::Tensor& evals, const at::Tensor& soff,
                           int64_t nsplit) {
  const int64_t U = (int64_t)xs.size();
  TORCH_CHECK(U >= 1 && U <= kSwMaxU && (int64_t)gs.size() == U,
              "slot_wgrad_list: 1 <= uses <= 16, one G per X");
  const int64_t N = xs[0].size(0);
  SwUses P{};
  for (int u = 0; u < U; ++u) {
    for (const at::Tensor* t : {&xs[u], &gs[u]})
      TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kBFloat16 &&
                      t->is_contiguous() && t->dim() == 2 &&
                      t->size(0) == N && t->size(1) == kSwC &&
                      aligned16(t->data_ptr()),
                  "slot_wgrad_list: contiguous 16-B aligned bf16 [N, 128]");
    P.x[u] = reinterpret_cast<const __bf16*>(xs[u].data_ptr());
    P.g[u] = reinterpret_cast<const __bf16*>(gs[u].data_ptr());
  }
  return launch_slot_wgrad(P, (int)U, N, xs[0], esrc, edst, evals, soff,
                           nsplit);
}

}  // namespace dgmc

namespace dgmc {

// ---------------------------------------------------------------------------
// Dense TN weight gradient over loop uses, the same MFMA pipeline without the
// entry lists:
//
//   dW_s = sum_u X_u[:, 128 s : 128 s + 128]^T G_u          (s < S, 128x128)
//
// for X_u [N, 128 S] (row stride ldx) and G_u [N, 128] (row stride 128): the
// weight gradient of a K = 128 S -> 128 projection summed over the loop's
// uses (the folded consensus projection, ops/dense.py::_CatMatmul), read in
// place (no concatenation of the kept gradients, no split-K GEMM over a
// 10x-long K at hipBLASLt's 0.16 PF/s on this skinny shape).  Workgroup =
// (block s, split); each split walks a contiguous row-chunk range, all uses
// per chunk.
// ---------------------------------------------------------------------------
struct DwUses {
  const __bf16* x[kSwMaxU];
  const __bf16* g[kSwMaxU];
};

__global__ __launch_bounds__(kSwThreads, 1) void dense_wgrad_kernel(
    const DwUses P, int U, int N, int64_t ldx, int64_t ldg, int Sx, int Sg,
    int nsplit, float* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) char lds[2][2][kSwTile * 2];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int k = blockIdx.x / nsplit, s = blockIdx.x % nsplit;
  const int kx = k / Sg, kg = k - kx * Sg;   // 128x128 output block
  const int nch = (N + kSwK - 1) / kSwK;
  const int ch0 = (int)((long long)nch * s / nsplit);
  const int ch1 = (int)((long long)nch * (s + 1) / nsplit);
  const int r = tid >> 4, c = tid & 15;
  const int mi = wave >> 2, nw = wave & 3;
  sw_f32x4 acc[4][2];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = sw_f32x4{0.f, 0.f, 0.f, 0.f};
  sw_bf16x8 xr[2], gr[2];
  const int steps = (ch1 - ch0) * U;
  int iu = 0, ic = ch0;
  auto issue = [&](auto slot_c) __attribute__((always_inline)) {
    constexpr int slot = decltype(slot_c)::value;
    const int row = ic * kSwK + r;
    const bool in = row < N && ic < ch1;     // padding rows contribute 0
    const int rr = in ? row : 0;
    const sw_bf16x8 z = {};
    const sw_bf16x8 xv = *reinterpret_cast<const sw_bf16x8*>(
        P.x[iu] + (size_t)rr * ldx + 128 * kx + 8 * c);
    const sw_bf16x8 gv = *reinterpret_cast<const sw_bf16x8*>(
        P.g[iu] + (size_t)rr * ldg + 128 * kg + 8 * c);
    xr[slot] = in ? xv : z;
    gr[slot] = in ? gv : z;
    const bool wrap = iu + 1 == U;
    iu = wrap ? 0 : iu + 1;
    ic += wrap ? 1 : 0;
  };
  auto stage = [&](auto slot_c) __attribute__((always_inline)) {
    constexpr int slot = decltype(slot_c)::value, buf = slot;
    *reinterpret_cast<DGMC_LDS sw_bf16x8*>(
        (DGMC_LDS char*)lds[buf][0] + sw_off(r, c)) = xr[slot];
    *reinterpret_cast<DGMC_LDS sw_bf16x8*>(
        (DGMC_LDS char*)lds[buf][1] + sw_off(r, c)) = gr[slot];
  };
  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  issue(S0{});
  issue(S1{});
  stage(S0{});
  __syncthreads();
  auto step = [&](auto buf_c) __attribute__((always_inline)) {
    constexpr int buf = decltype(buf_c)::value;
    issue(buf_c);
    const DGMC_LDS char* A = (const DGMC_LDS char*)lds[buf][0];
    const DGMC_LDS char* B = (const DGMC_LDS char*)lds[buf][1];
    sw_bf16x8 af[4], bf[2];
#pragma unroll
    for (int a = 0; a < 4; ++a) af[a] = sw_frag(A, 4 * mi + a, lane);
#pragma unroll
    for (int b = 0; b < 2; ++b) bf[b] = sw_frag(B, 2 * nw + b, lane);
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
        acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[a], bf[b],
                                                            acc[a][b], 0, 0,
                                                            0);
    stage(std::integral_constant<int, buf ^ 1>{});
    __syncthreads();
  };
  // Steps past `steps` (odd count) read past ch1: zero rows.
  for (int t = 0; t < steps; t += 2) {
    step(S0{});
    step(S1{});
  }
  // Partial [split][128 Sx][128 Sg] (row-major dW block).
  const int Kg = kSwC * Sg;
  float* out = part + (size_t)s * kSwC * Sx * Kg + (size_t)kSwC * kx * Kg +
               kSwC * kg;
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = 64 * mi + 16 * a + 4 * (lane >> 4) + q;
        const int colo = 32 * nw + 16 * b + (lane & 15);
        out[(size_t)row * Kg + colo] = acc[a][b][q];
      }
}

// xs[u] [N, 128 Sx], gs[u] [N, 128 Sg] bf16 (unit column stride, equal
// 16-byte aligned row strides per list); returns per-split partials
// [nsplit, 128 Sx * 128 Sg] fp32 of dW = sum_u xs[u]^T gs[u].
at::Tensor dense_wgrad(at::TensorList xs, at::TensorList gs, int64_t nsplit) {
  const int64_t U = (int64_t)xs.size();
  TORCH_CHECK(U >= 1 && U <= kSwMaxU && (int64_t)gs.size() == U,
              "dense_wgrad: 1 <= uses <= 16, one G per X");
  const int64_t N = xs[0].size(0);
  TORCH_CHECK(xs[0].dim() == 2 && xs[0].size(1) % kSwC == 0 &&
                  xs[0].size(1) >= kSwC && gs[0].dim() == 2 &&
                  gs[0].size(1) % kSwC == 0 && gs[0].size(1) >= kSwC,
              "dense_wgrad: X [N, 128 Sx], G [N, 128 Sg]");
  const int64_t Sx = xs[0].size(1) / kSwC, Sg = gs[0].size(1) / kSwC;
  const int64_t ldx = xs[0].stride(0), ldg = gs[0].stride(0);
  DwUses P{};
  for (int u = 0; u < U; ++u) {
    const at::Tensor& x = xs[u];
    const at::Tensor& g = gs[u];
    for (const at::Tensor* t : {&x, &g}) {
      const bool isx = t == &x;
      TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kBFloat16 &&
                      t->dim() == 2 && t->size(0) == N &&
                      t->size(1) == (isx ? Sx : Sg) * kSwC &&
                      t->stride(1) == 1 && t->stride(0) == (isx ? ldx : ldg) &&
                      t->stride(0) % 8 == 0 && aligned16(t->data_ptr()),
                  "dense_wgrad: bf16 operands with equal 16-byte row strides");
    }
    P.x[u] = reinterpret_cast<const __bf16*>(x.data_ptr());
    P.g[u] = reinterpret_cast<const __bf16*>(g.data_ptr());
  }
  TORCH_CHECK(nsplit >= 1 && Sx * Sg * nsplit < (1 << 30) &&
                  N < INT32_MAX / kSwC,
              "dense_wgrad: size range");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(xs[0].device());
  at::Tensor part = at::empty({nsplit, Sx * Sg * kSwC * kSwC},
                              xs[0].options().dtype(at::kFloat));
  hipLaunchKernelGGL(dense_wgrad_kernel, dim3(Sx * Sg * nsplit),
                     dim3(kSwThreads), 0, stream(), P, (int)U, (int)N, ldx,
                     ldg, (int)Sx, (int)Sg, (int)nsplit,
                     part.data_ptr<float>());
  DGMC_CHECK_LAUNCH();
  return part;
}

// Probe of ds_read_b64_tr_b16 semantics (tools/debug/wgrad_debug.py): LDS
// tile [16 rows][16 cols] int16 = 100 * row + col; lane 4q+p of each 16-lane
// group addresses row (q + 4 * (group & 1)), columns 4p..4p+3.  Returns the
// four elements every lane receives.
__global__ void tr16_probe_kernel(short* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) short tile[16 * 16];
  const int lane = threadIdx.x;
  for (int i = lane; i < 256; i += 64) tile[i] = (short)(100 * (i / 16) + i % 16);
  __syncthreads();
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int row = q + 4 * (g & 1);
  typedef short i16x4 __attribute__((ext_vector_type(4)));
  const i16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (DGMC_LDS i16x4*)((DGMC_LDS short*)tile + row * 16 + 4 * p));
  for (int j = 0; j < 4; ++j) out[lane * 4 + j] = v[j];
}

at::Tensor tr16_probe(const at::Tensor& like) {
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(like.device());
  at::Tensor out = at::empty({64, 4}, like.options().dtype(at::kShort));
  hipLaunchKernelGGL(tr16_probe_kernel, dim3(1), dim3(64), 0, stream(),
                     out.data_ptr<short>());
  DGMC_CHECK_LAUNCH();
  return out;
}

}  // namespace dgmc

namespace dgmc {

// ---------------------------------------------------------------------------
// Entries of a slot-structured CSR operator grouped by slot, in entry order
// inside each slot (a deterministic, stable counting sort - the weight
// gradient's summation order is fixed run to run).  Entries past rowptr[N]
// (the inert tail of a fixed-capacity operator) are dropped.
constexpr int kPlBlock = 1024;    // entries per block
constexpr int kPlThreads = 256;
constexpr int kPlMaxS = 64;

__global__ __launch_bounds__(kPlThreads) void pair_count_kernel(
    const int* __restrict__ rowptr, const int* __restrict__ col, int N,
    int S, int* __restrict__ cnt) {
  __shared__ int hist[kPlMaxS];
  const int tid = threadIdx.x, blk = blockIdx.x;
  const int E = rowptr[N];
  if (tid < S) hist[tid] = 0;
  __syncthreads();
  for (int i = 0; i < kPlBlock / kPlThreads; ++i) {
    const int e = blk * kPlBlock + i * kPlThreads + tid;
    if (e < E) atomicAdd(&hist[col[e] % S], 1);
  }
  __syncthreads();
  if (tid < S) cnt[blk * S + tid] = hist[tid];
}

// off[blk][k] = (entries of slots < k) + (entries of slot k in blocks < blk).
// The counts are staged in LDS first (a serial scan over global memory would
// pay one load latency per block).
constexpr int kPlScanLds = 16384;   // ints

__global__ __launch_bounds__(kPlThreads) void pair_scan_kernel(
    const int* __restrict__ cnt, int nblk, int S, int* __restrict__ off,
    int* __restrict__ soff) {
  __shared__ int c_s[kPlScanLds];
  __shared__ int total[kPlMaxS + 1];
  const int tid = threadIdx.x;
  const bool staged = nblk * S <= kPlScanLds;
  if (staged)
    for (int i = tid; i < nblk * S; i += kPlThreads) c_s[i] = cnt[i];
  __syncthreads();
  const int k = tid;
  int run = 0;
  if (k < S) {
    for (int b = 0; b < nblk; ++b) {
      const int c = staged ? c_s[b * S + k] : cnt[b * S + k];
      if (staged) c_s[b * S + k] = run; else off[b * S + k] = run;
      run += c;
    }
    total[k] = run;
  }
  __syncthreads();
  if (tid == 0) {
    int acc = 0;
    for (int kk = 0; kk < S; ++kk) {
      soff[kk] = acc;
      const int t = total[kk];
      total[kk] = acc;
      acc += t;
    }
    soff[S] = acc;
  }
  __syncthreads();
  for (int i = tid; i < nblk * S; i += kPlThreads)
    off[i] = (staged ? c_s[i] : off[i]) + total[i % S];
}

__global__ __launch_bounds__(kPlThreads) void pair_scatter_kernel(
    const int* __restrict__ rowptr, const int* __restrict__ col,
    const float* __restrict__ val, const int64_t* __restrict__ row, int N,
    int S, const int* __restrict__ off, int* __restrict__ esrc,
    int* __restrict__ edst, float* __restrict__ evals) {
  constexpr int R = kPlBlock / kPlThreads;   // rounds
  constexpr int W = kPlThreads / 64;         // waves
  __shared__ int wcnt[R * W][kPlMaxS];
  const int tid = threadIdx.x, blk = blockIdx.x, wave = tid >> 6,
            lane = tid & 63;
  const int E = rowptr[N];
  const unsigned long long lt = (1ull << lane) - 1ull;
  int key[R], rank[R];
  for (int i = 0; i < R; ++i) {
    const int e = blk * kPlBlock + i * kPlThreads + tid;
    key[i] = e < E ? col[e] % S : -1;
    rank[i] = 0;
    for (int k = 0; k < S; ++k) {           // stable rank inside the wave
      const unsigned long long m = __ballot(key[i] == k);
      if (key[i] == k) rank[i] = __popcll(m & lt);
      if (lane == 0) wcnt[i * W + wave][k] = __popcll(m);
    }
  }
  __syncthreads();
  if (tid < S) {                            // exclusive prefix in entry order
    int run = 0;
    for (int g = 0; g < R * W; ++g) {
      const int c = wcnt[g][tid];
      wcnt[g][tid] = run;
      run += c;
    }
  }
  __syncthreads();
  for (int i = 0; i < R; ++i) {
    if (key[i] < 0) continue;
    const int e = blk * kPlBlock + i * kPlThreads + tid;
    const int k = key[i];
    const int pos = off[blk * S + k] + wcnt[i * W + wave][k] + rank[i];
    esrc[pos] = col[e] / S;
    edst[pos] = (int)row[e];
    evals[pos] = val[e];
  }
}

std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> slot_pair_lists(
    const at::Tensor& rowptr, const at::Tensor& col, const at::Tensor& val,
    const at::Tensor& row, int64_t S) {
  TORCH_CHECK(rowptr.is_cuda() && rowptr.scalar_type() == at::kInt &&
                  col.scalar_type() == at::kInt &&
                  val.scalar_type() == at::kFloat &&
                  row.scalar_type() == at::kLong && rowptr.is_contiguous() &&
                  col.is_contiguous() && val.is_contiguous() &&
                  row.is_contiguous() && col.numel() == val.numel() &&
                  row.numel() == col.numel(),
              "slot_pair_lists: int32 rowptr/col, fp32 val, int64 row");
  TORCH_CHECK(S >= 1 && S <= kPlMaxS, "slot_pair_lists: 1 <= S <= 64");
  const int64_t N = rowptr.numel() - 1, E = col.numel();
  TORCH_CHECK(E < INT32_MAX, "slot_pair_lists: size range");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(col.device());
  const int nblk = (int)std::max<int64_t>((E + kPlBlock - 1) / kPlBlock, 1);
  auto i32 = col.options();
  at::Tensor cnt = at::empty({nblk, S}, i32);
  at::Tensor off = at::empty({nblk, S}, i32);
  at::Tensor soff = at::empty({S + 1}, i32);
  // Only the first rowptr[N] entries are written - and read (through soff).
  at::Tensor esrc = at::empty({E}, i32);
  at::Tensor edst = at::empty({E}, i32);
  at::Tensor evals = at::empty({E}, val.options());
  hipLaunchKernelGGL(pair_count_kernel, dim3(nblk), dim3(kPlThreads), 0,
                     stream(), rowptr.data_ptr<int>(), col.data_ptr<int>(),
                     (int)N, (int)S, cnt.data_ptr<int>());
  hipLaunchKernelGGL(pair_scan_kernel, dim3(1), dim3(kPlThreads), 0, stream(),
                     cnt.data_ptr<int>(), nblk, (int)S, off.data_ptr<int>(),
                     soff.data_ptr<int>());
  hipLaunchKernelGGL(pair_scatter_kernel, dim3(nblk), dim3(kPlThreads), 0,
                     stream(), rowptr.data_ptr<int>(), col.data_ptr<int>(),
                     val.data_ptr<float>(), row.data_ptr<int64_t>(), (int)N,
                     (int)S, off.data_ptr<int>(), esrc.data_ptr<int>(),
                     edst.data_ptr<int>(), evals.data_ptr<float>());
  DGMC_CHECK_LAUNCH();
  return {esrc, edst, evals, soff};
}

}  // namespace dgmc
