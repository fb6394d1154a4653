// Initial dense correspondence scores per graph pair (DGMC Stage I):
//
//   S_hat[b, i, j] = < h_s[ptr_s[b] + i], h_t[ptr_t[b] + j] >
//                    for i < n_s[b], j < n_t[b];  0 elsewhere in [N_s, N_t]
//
// Reference: /root/reference/dgmc/models/dgmc.py:154-163 - to_dense_batch of
// both embeddings, then one batched GEMM ``h_s @ h_t^T``.  The dense path of
// the reference (and our generic path) pads both [sum N, C] embeddings into
// fp32 [B, N_max, C] tensors (fill + index_copy each, plus the fp32 cast) and
// runs a batched GEMM of tiny 19 x 256 x 19 products; the backward scatters
// the dense gradients back through index_copy / slice backward (zero fills
// and copies).  Here one workgroup per pair reads the packed embedding rows
// straight from the encoder output (bf16 under autocast, fp32 accumulation)
// and writes the padded [N_s, N_t] score tile; the backward writes the
// gradient of the whole joint [h_s; h_t] encoder output (padding rows zero).
//
// Forward mapping (N_t <= 64): the pair's target rows are staged transposed
// in LDS (htT[c][j], lane j reads consecutive words: conflict-free), source
// rows row-major (hs[i][c] is a wave broadcast); wave w computes rows
// i = w, w + 4, ... with lane j = column j.
#include "common.h"

namespace dgmc {

namespace {

constexpr int kPsThreads = 256;
constexpr int kPsMaxN = 64;

template <typename T>
__device__ __forceinline__ float ps_load(const T* p) {
  return (float)*p;
}

template <typename T>
__global__ __launch_bounds__(kPsThreads) void pair_scores_kernel(
    const T* __restrict__ h, int64_t t_off, const int* __restrict__ ptr_s,
    const int* __restrict__ ptr_t, float* __restrict__ S, int Ns, int Nt,
    int C, int ldt) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  DGMC_LDS float* sm = (DGMC_LDS float*)smem_raw;
  DGMC_LDS float* hs = sm;                        // [Ns][C]
  DGMC_LDS float* htT = sm + Ns * C;              // [C][ldt], ldt odd
  const int b = blockIdx.x, tid = threadIdx.x;
  const int s0 = ptr_s[b], ns = min(ptr_s[b + 1] - s0, Ns);
  const int t0 = ptr_t[b], nt = min(ptr_t[b + 1] - t0, Nt);
  const T* hs_g = h + (int64_t)s0 * C;
  const T* ht_g = h + (t_off + t0) * C;
  for (int e = tid; e < ns * C; e += kPsThreads) hs[e] = ps_load(hs_g + e);
  for (int e = tid; e < nt * C; e += kPsThreads) {
    const int j = e / C, c = e - j * C;   // consecutive lanes: consecutive c,
    htT[c * ldt + j] = ps_load(ht_g + e); // odd stride -> distinct banks
  }
  __syncthreads();
  const int wave = tid >> 6, lane = tid & 63;
  float* Sb = S + (int64_t)b * Ns * Nt;
  for (int i = wave; i < Ns; i += kPsThreads / 64) {
    float acc = 0.f;
    if (i < ns && lane < nt) {
      DGMC_LDS const float* a = hs + i * C;
#pragma unroll 8
      for (int c = 0; c < C; ++c) acc += a[c] * htT[c * ldt + lane];
    }
    if (lane < Nt) Sb[i * Nt + lane] = acc;
  }
}

// Pairs with N_s, N_t <= 32 (PascalVOC / WILLOW): ONE wave per pair on
// v_mfma_f32_32x32x16_bf16 (4 pairs per workgroup).  Lane l (r = l & 31,
// q = l >> 5) loads A[r][16s + 8q .. +7] = h_s row r and B[..][r] = h_t row r
// straight from global (16-byte loads, rows past the pair's count read as
// zero), 16 k-steps for C = 256; the accumulator holds
// S[(reg & 3) + 8 (reg >> 2) + 4q][r].
typedef __bf16 ps_bf16x8 __attribute__((ext_vector_type(8)));
typedef float ps_f32x16 __attribute__((ext_vector_type(16)));

__global__ __launch_bounds__(256) void pair_scores_mfma_kernel(
    const __hip_bfloat16* __restrict__ hg, int64_t t_off,
    const int* __restrict__ ptr_s, const int* __restrict__ ptr_t,
    float* __restrict__ S, int B, int Ns, int Nt, int C) {
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  const int lane = threadIdx.x & 63, r = lane & 31, q = lane >> 5;
  const __bf16* h = reinterpret_cast<const __bf16*>(hg);
  const int s0 = ptr_s[b], ns = min(ptr_s[b + 1] - s0, Ns);
  const int t0 = ptr_t[b], nt = min(ptr_t[b + 1] - t0, Nt);
  const __bf16* arow = h + (int64_t)(s0 + min(r, max(ns - 1, 0))) * C + 8 * q;
  const __bf16* brow =
      h + (t_off + t0 + min(r, max(nt - 1, 0))) * C + 8 * q;
  const bool av = r < ns, bv = r < nt;
  ps_f32x16 acc = {};
  const ps_bf16x8 z = {};
  for (int k = 0; k < C; k += 16) {
    const ps_bf16x8 a = av ? *reinterpret_cast<const ps_bf16x8*>(arow + k) : z;
    const ps_bf16x8 bb =
        bv ? *reinterpret_cast<const ps_bf16x8*>(brow + k) : z;
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bb, acc, 0, 0, 0);
  }
  float* Sb = S + (int64_t)b * Ns * Nt;
  if (r < Nt) {
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const int i = (reg & 3) + 8 * (reg >> 2) + 4 * q;
      if (i < Ns) Sb[i * Nt + r] = acc[reg];
    }
  }
}

// dh for the joint [h_s; h_t]: block b handles pair b's rows and a
// grid-stride share of the padding rows [ptr_s[B], t_off) and
// [t_off + ptr_t[B], rows) (zeroed with 8-byte stores).
//   dh_s[i, c] = sum_j dS[i, j] h_t[j, c],  dh_t[j, c] = sum_i dS[i, j] h_s[i, c]
template <typename T>
__device__ __forceinline__ void ps_stage(DGMC_LDS float* dst, const T* src,
                                         int n, int tid) {
  // n % 4 == 0; 4 elements per thread and pass.
  for (int e = 4 * tid; e < n; e += 4 * kPsThreads) {
    float v[4];
    if constexpr (sizeof(T) == 2) {
      typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));
      const u16x4 w = *reinterpret_cast<const u16x4*>(src + e);
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = __uint_as_float((unsigned)w[k] << 16);
    } else {
      const float4 w = *reinterpret_cast<const float4*>(src + e);
      v[0] = w.x; v[1] = w.y; v[2] = w.z; v[3] = w.w;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) dst[e + k] = v[k];
  }
}

template <typename T>
__global__ __launch_bounds__(kPsThreads) void pair_scores_bwd_kernel(
    const float* __restrict__ dS, const float* __restrict__ dS2,
    const T* __restrict__ h, int64_t t_off,
    int64_t rows, const int* __restrict__ ptr_s, const int* __restrict__ ptr_t,
    T* __restrict__ dh, int B, int Ns, int Nt, int C) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  DGMC_LDS float* sm = (DGMC_LDS float*)smem_raw;
  DGMC_LDS float* g = sm;                          // [Ns][Nt]
  DGMC_LDS float* hsL = g + ((Ns * Nt + 3) & ~3);  // [Ns][C]
  DGMC_LDS float* htL = hsL + Ns * C;              // [Nt][C]
  const int b = blockIdx.x, tid = threadIdx.x;
  {
    // padding rows (4-element groups; C % 4 == 0 keeps rows aligned)
    const int64_t a0 = (int64_t)ptr_s[B] * C, a1 = t_off * C;
    const int64_t b0 = (t_off + ptr_t[B]) * C, b1 = rows * C;
    const int64_t na = (a1 - a0) / 4, nb = (b1 - b0) / 4;
    typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));
    for (int64_t q = (int64_t)b * kPsThreads + tid; q < na + nb;
         q += (int64_t)gridDim.x * kPsThreads) {
      T* p = dh + (q < na ? a0 + 4 * q : b0 + 4 * (q - na));
      if constexpr (sizeof(T) == 2) {
        const u16x4 z = {0, 0, 0, 0};
        *reinterpret_cast<u16x4*>(p) = z;
      } else {
        *reinterpret_cast<float4*>(p) = make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
  }
  const int s0 = ptr_s[b], ns = min(ptr_s[b + 1] - s0, Ns);
  const int t0 = ptr_t[b], nt = min(ptr_t[b + 1] - t0, Nt);
  const float* dSb = dS + (int64_t)b * Ns * Nt;
  const T* hs_g = h + (int64_t)s0 * C;
  const T* ht_g = h + (t_off + t0) * C;
  // Two consumers' gradients of S_hat (loss + consensus loop) are summed
  // here instead of by an autograd add kernel.
  if (dS2) {
    const float* dSb2 = dS2 + (int64_t)b * Ns * Nt;
    for (int e = tid; e < Ns * Nt; e += kPsThreads) g[e] = dSb[e] + dSb2[e];
  } else {
    for (int e = tid; e < Ns * Nt; e += kPsThreads) g[e] = dSb[e];
  }
  ps_stage(hsL, hs_g, ns * C, tid);
  ps_stage(htL, ht_g, nt * C, tid);
  __syncthreads();
  T* dhs = dh + (int64_t)s0 * C;
  T* dht = dh + (t_off + t0) * C;
  // One (row, 4 channels) item per thread and pass: lanes of a wave share
  // the row (g broadcast) and read consecutive 16-byte LDS chunks.
  const int C4 = C / 4;
  for (int it = tid; it < (ns + nt) * C4; it += kPsThreads) {
    const int row = it / C4, c = (it - row * C4) * 4;
    const bool src = row < ns;
    const int i = src ? row : row - ns;
    DGMC_LDS const float* other = src ? htL : hsL;
    const int n = src ? nt : ns;
    typedef float f32x4 __attribute__((ext_vector_type(4)));
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int j = 0; j < n; ++j) {
      const float w = src ? g[i * Nt + j] : g[j * Nt + i];
      const f32x4 v =
          *reinterpret_cast<DGMC_LDS const f32x4*>(other + j * C + c);
      acc += w * v;
    }
    T* dst = (src ? dhs : dht) + (int64_t)i * C + c;
#pragma unroll
    for (int e = 0; e < 4; ++e) dst[e] = (T)acc[e];
  }
}

}  // namespace

// h: [rows, C] joint encoder output (source rows first; target rows start at
// t_off), bf16 or fp32; ptr_s / ptr_t int32 [B + 1] pair row offsets (target
// offsets relative to t_off).  Returns S_hat fp32 [B, Ns, Nt].
at::Tensor pair_scores(const at::Tensor& h, int64_t t_off,
                       const at::Tensor& ptr_s, const at::Tensor& ptr_t,
                       int64_t Ns, int64_t Nt) {
  TORCH_CHECK(h.is_cuda() && h.dim() == 2 && h.is_contiguous() &&
                  (h.scalar_type() == at::kBFloat16 ||
                   h.scalar_type() == at::kFloat),
              "pair_scores: contiguous bf16/fp32 h [rows, C]");
  TORCH_CHECK(ptr_s.scalar_type() == at::kInt && ptr_t.scalar_type() == at::kInt &&
                  ptr_s.numel() == ptr_t.numel() && ptr_s.numel() >= 1 &&
                  ptr_s.is_contiguous() && ptr_t.is_contiguous(),
              "pair_scores: int32 ptr_s / ptr_t [B + 1]");
  TORCH_CHECK(Ns >= 1 && Nt >= 1 && Ns <= kPsMaxN && Nt <= kPsMaxN,
              "pair_scores: 1 <= N_s, N_t <= 64");
  TORCH_CHECK(t_off >= 0 && t_off <= h.size(0), "pair_scores: t_off range");
  const int B = (int)ptr_s.numel() - 1;
  const int C = (int)h.size(1);
  const int ldt = (int)Nt | 1;     // odd transposed stride (no bank conflicts)
  const size_t lds = ((size_t)Ns * C + (size_t)C * ldt) * sizeof(float);
  TORCH_CHECK(lds <= 160 * 1024, "pair_scores: C too large for LDS staging");
  at::Tensor S = at::empty({B, Ns, Nt}, h.options().dtype(at::kFloat));
  if (B == 0) return S;
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(h.device());
  static bool attr = false;
  if (!attr) {
    DGMC_CHECK_HIP(hipFuncSetAttribute(
        reinterpret_cast<const void*>(pair_scores_kernel<__hip_bfloat16>),
        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    DGMC_CHECK_HIP(hipFuncSetAttribute(
        reinterpret_cast<const void*>(pair_scores_kernel<float>),
        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr = true;
  }
  if (h.scalar_type() == at::kBFloat16 && Ns <= 32 && Nt <= 32 &&
      C % 16 == 0 && aligned16(h.data_ptr()) && (t_off * C) % 8 == 0) {
    hipLaunchKernelGGL(pair_scores_mfma_kernel, dim3((B + 3) / 4), dim3(256),
                       0, stream(),
                       reinterpret_cast<const __hip_bfloat16*>(h.data_ptr()),
                       t_off, ptr_s.data_ptr<int>(), ptr_t.data_ptr<int>(),
                       S.data_ptr<float>(), B, (int)Ns, (int)Nt, C);
  } else if (h.scalar_type() == at::kBFloat16) {
    auto k = pair_scores_kernel<__hip_bfloat16>;
    hipLaunchKernelGGL(k, dim3(B), dim3(kPsThreads), lds, stream(),
                       reinterpret_cast<const __hip_bfloat16*>(h.data_ptr()),
                       t_off, ptr_s.data_ptr<int>(), ptr_t.data_ptr<int>(),
                       S.data_ptr<float>(), (int)Ns, (int)Nt, C, ldt);
  } else {
    auto k = pair_scores_kernel<float>;
    hipLaunchKernelGGL(k, dim3(B), dim3(kPsThreads), lds, stream(),
                       h.data_ptr<float>(), t_off, ptr_s.data_ptr<int>(),
                       ptr_t.data_ptr<int>(), S.data_ptr<float>(), (int)Ns,
                       (int)Nt, C, ldt);
  }
  DGMC_CHECK_LAUNCH();
  return S;
}

at::Tensor pair_scores_bwd(const at::Tensor& dS, const at::Tensor& h,
                           int64_t t_off, const at::Tensor& ptr_s,
                           const at::Tensor& ptr_t,
                           const c10::optional<at::Tensor>& dS2) {
  TORCH_CHECK(dS.is_cuda() && dS.scalar_type() == at::kFloat && dS.dim() == 3 &&
                  dS.is_contiguous(),
              "pair_scores_bwd: contiguous fp32 dS [B, Ns, Nt]");
  const float* d2 = nullptr;
  if (dS2.has_value() && dS2->defined()) {
    TORCH_CHECK(dS2->scalar_type() == at::kFloat && dS2->is_contiguous() &&
                    dS2->sizes() == dS.sizes(),
                "pair_scores_bwd: dS2 like dS");
    d2 = dS2->data_ptr<float>();
  }
  TORCH_CHECK(h.is_cuda() && h.dim() == 2 && h.is_contiguous() &&
                  (h.scalar_type() == at::kBFloat16 ||
                   h.scalar_type() == at::kFloat),
              "pair_scores_bwd: contiguous bf16/fp32 h [rows, C]");
  const int B = (int)dS.size(0), Ns = (int)dS.size(1), Nt = (int)dS.size(2);
  TORCH_CHECK(ptr_s.numel() == B + 1 && ptr_t.numel() == B + 1 &&
                  ptr_s.scalar_type() == at::kInt &&
                  ptr_t.scalar_type() == at::kInt,
              "pair_scores_bwd: int32 ptr_s / ptr_t [B + 1]");
  TORCH_CHECK(Ns <= kPsMaxN && Nt <= kPsMaxN, "pair_scores_bwd: N <= 64");
  TORCH_CHECK(h.size(1) % 4 == 0 && aligned16(h.data_ptr()),
              "pair_scores_bwd: C % 4 != 0 or unaligned h");
  if (dS.size(0) == 0) return at::zeros_like(h);
  const int C = (int)h.size(1);
  at::Tensor dh = at::empty_like(h);
  const size_t lds =
      ((size_t)((Ns * Nt + 3) & ~3) + (size_t)(Ns + Nt) * C) * sizeof(float);
  TORCH_CHECK(lds <= 160 * 1024, "pair_scores_bwd: C too large for LDS");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(h.device());
  const int64_t rows = h.size(0);
  static bool attr = false;
  if (!attr) {
    DGMC_CHECK_HIP(hipFuncSetAttribute(
        reinterpret_cast<const void*>(pair_scores_bwd_kernel<__hip_bfloat16>),
        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    DGMC_CHECK_HIP(hipFuncSetAttribute(
        reinterpret_cast<const void*>(pair_scores_bwd_kernel<float>),
        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr = true;
  }
  if (h.scalar_type() == at::kBFloat16)
    hipLaunchKernelGGL(pair_scores_bwd_kernel<__hip_bfloat16>, dim3(B),
                       dim3(kPsThreads), lds, stream(), dS.data_ptr<float>(),
                       d2,
                       reinterpret_cast<const __hip_bfloat16*>(h.data_ptr()),
                       t_off, rows, ptr_s.data_ptr<int>(),
                       ptr_t.data_ptr<int>(),
                       reinterpret_cast<__hip_bfloat16*>(dh.data_ptr()), B,
                       Ns, Nt, C);
  else
    hipLaunchKernelGGL(pair_scores_bwd_kernel<float>, dim3(B),
                       dim3(kPsThreads), lds, stream(), dS.data_ptr<float>(),
                       d2, h.data_ptr<float>(), t_off, rows,
                       ptr_s.data_ptr<int>(),
                       ptr_t.data_ptr<int>(), dh.data_ptr<float>(), B, Ns, Nt,
                       C);
  DGMC_CHECK_LAUNCH();
  return dh;
}

}  // namespace dgmc
