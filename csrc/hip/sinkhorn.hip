// Masked log-domain Sinkhorn normalisation of the dense correspondence
// scores, one workgroup per graph pair (opt-in `normalization='sinkhorn'`
// of DGMC; the reference itself only row-normalises with a masked softmax,
// /root/reference/dgmc/models/dgmc.py:15-19 - BASELINE.json config 3 names
// the dense Sinkhorn variant).
//
//   L0 = S_hat / tau on the valid n_s x n_t block of each pair
//   repeat iters times:   a_i = LSE_j(L0_ij - b_j)      (rows sum to 1)
//                         b_j = LSE_i(L0_ij - a_i)      (columns sum to 1)
//   final row step:       a_i = LSE_j(L0_ij - b_j)
//   P_ij = exp(L0_ij - a_i - b_j)  (0 outside the valid block)
//
// In the log domain every half-step's potential is a closed form of the
// other one (no accumulation), so the forward keeps only the potentials of
// every half-step ([B, iters + 1, Ns] and [B, iters, Nt]); the backward
// rebuilds each half-step's output from them and applies the normalisation
// Jacobians in reverse:  row step  D_ij -= exp(out_ij) sum_k D_ik,
//                        column step D_ij -= exp(out_ij) sum_k D_kj.
// The pair tile lives in LDS (N <= 64).  ONE wave per pair: in a row step
// lane i owns row i and reduces it sequentially (the tile's odd pitch keeps
// the lanes' reads of one column conflict-free), in a column step lane j
// owns column j - no cross-lane reductions, no multi-wave barriers (a
// half-step is ~20 LDS reads + exps per lane; was one wave-wide LSE per row
// with 4 waves and a block barrier per half-step: 63 -> see
// docs/performance.md).  Deterministic, no atomics.
#include "common.h"

namespace dgmc {

namespace {
constexpr int kShMaxN = 64;
constexpr int kShPitch = kShMaxN + 1;

// LSE_k (row[k * stride] - pot[k]) over k < n (0 for an empty set).
__device__ __forceinline__ float lse_line(const DGMC_LDS float* row,
                                          int stride,
                                          const DGMC_LDS float* pot, int n) {
  float m = -INFINITY;
  for (int k = 0; k < n; ++k) m = fmaxf(m, row[k * stride] - pot[k]);
  if (m == -INFINITY) return 0.f;
  float sum = 0.f;
  for (int k = 0; k < n; ++k) sum += __expf(row[k * stride] - pot[k] - m);
  return m + __logf(sum);
}


// Loads L0 = S_hat / tau of pair tile S (row pitch NP) into LDS.
__device__ __forceinline__ void sk_load(DGMC_LDS float* L0, const float* S,
                                        int Ns, int Nt, int NP, float inv_tau,
                                        int lane) {
  for (int e = lane; e < Ns * Nt; e += kWave) {
    const int i = e / Nt, j = e - i * Nt;
    L0[i * NP + j] = S[e] * inv_tau;
  }
}

// The forward iterations on the LDS tile: leaves the final potentials in
// a / b and records every half-step's in ah ([iters + 1, Ns]) / bh
// ([iters, Nt]).  Ends with a barrier.
__device__ __forceinline__ void sk_iterate(const DGMC_LDS float* L0,
                                           DGMC_LDS float* a,
                                           DGMC_LDS float* b, int ns, int nt,
                                           int Ns, int Nt, int NP, int iters,
                                           float* ah, float* bh, int lane) {
  b[lane] = 0.f;
  a[lane] = 0.f;
  __syncthreads();
  for (int it = 0; it <= iters; ++it) {
    // Row step: lane i.
    if (lane < Ns) {
      const float r = lane < ns ? lse_line(L0 + lane * NP, 1, b, nt) : 0.f;
      a[lane] = r;
      ah[it * Ns + lane] = r;
    }
    __syncthreads();
    if (it == iters) break;
    // Column step: lane j.
    if (lane < Nt) {
      const float c = lane < nt ? lse_line(L0 + lane, NP, a, ns) : 0.f;
      b[lane] = c;
      bh[it * Nt + lane] = c;
    }
    __syncthreads();
  }
}

// The backward half-steps in reverse on D (holding dL/d(final row-step
// output) on entry, dL/dL0 on exit).  Ends with a barrier.
__device__ __forceinline__ void sk_reverse(const DGMC_LDS float* L0,
                                           DGMC_LDS float* D,
                                           DGMC_LDS float* a,
                                           DGMC_LDS float* b, int ns, int nt,
                                           int Ns, int Nt, int NP, int iters,
                                           const float* ah, const float* bh,
                                           int lane) {
  for (int step = 2 * iters; step >= 0; --step) {
    const bool row = (step & 1) == 0;     // even: row step, odd: column step
    const int it = step >> 1;
    // Potentials defining this half-step's output L0 - a - b.
    if (lane < Ns) a[lane] = ah[it * Ns + lane];
    if (lane < Nt)
      b[lane] = row ? (it > 0 ? bh[(it - 1) * Nt + lane] : 0.f)
                    : bh[it * Nt + lane];
    __syncthreads();
    if (row) {
      // Lane i: D_ij -= exp(out_ij) sum_k D_ik over its row.
      if (lane < ns) {
        DGMC_LDS float* Dr = D + lane * NP;
        const DGMC_LDS float* Lr = L0 + lane * NP;
        float sum = 0.f;
        for (int j = 0; j < Nt; ++j) sum += Dr[j];
        const float ai = a[lane];
        for (int j = 0; j < nt; ++j)
          Dr[j] -= __expf(Lr[j] - ai - b[j]) * sum;
      }
    } else {
      // Lane j: D_ij -= exp(out_ij) sum_k D_kj over its column.
      if (lane < nt) {
        float sum = 0.f;
        for (int i = 0; i < Ns; ++i) sum += D[i * NP + lane];
        const float bj = b[lane];
        for (int i = 0; i < ns; ++i)
          D[i * NP + lane] -= __expf(L0[i * NP + lane] - a[i] - bj) * sum;
      }
    }
    __syncthreads();
  }
}

// Loads the final potentials (row step iters, column step iters - 1).
__device__ __forceinline__ void sk_final_pot(DGMC_LDS float* a,
                                             DGMC_LDS float* b, int Ns,
                                             int Nt, int iters,
                                             const float* ah, const float* bh,
                                             int lane) {
  if (lane < Ns) a[lane] = ah[iters * Ns + lane];
  if (lane < Nt) b[lane] = iters > 0 ? bh[(iters - 1) * Nt + lane] : 0.f;
}
}  // namespace

__global__ __launch_bounds__(kWave) void sinkhorn_fwd_kernel(
    const float* __restrict__ S_hat, const int* __restrict__ n_s,
    const int* __restrict__ n_t, int Ns, int Nt, int iters, float inv_tau,
    float* __restrict__ P, float* __restrict__ a_hist,
    float* __restrict__ b_hist) {
  __shared__ float L0_[kShMaxN * kShPitch];
  __shared__ float a_[kShMaxN], b_[kShMaxN];
  DGMC_LDS float* L0 = (DGMC_LDS float*)L0_;
  DGMC_LDS float* a = (DGMC_LDS float*)a_;
  DGMC_LDS float* b = (DGMC_LDS float*)b_;
  const int pb = xcd_remap(blockIdx.x, gridDim.x);
  const int lane = threadIdx.x;
  const int ns = n_s[pb], nt = n_t[pb];
  const int NP = Nt + 1 + (Nt & 1);      // odd pitch (<= 65)
  sk_load(L0, S_hat + (size_t)pb * Ns * Nt, Ns, Nt, NP, inv_tau, lane);
  sk_iterate(L0, a, b, ns, nt, Ns, Nt, NP, iters,
             a_hist + (size_t)pb * (iters + 1) * Ns,
             b_hist + (size_t)pb * iters * Nt, lane);
  float* Pb = P + (size_t)pb * Ns * Nt;
  for (int e = lane; e < Ns * Nt; e += kWave) {
    const int i = e / Nt, j = e - i * Nt;
    Pb[e] = (i < ns && j < nt) ? __expf(L0[i * NP + j] - a[i] - b[j]) : 0.f;
  }
}

__global__ __launch_bounds__(kWave) void sinkhorn_bwd_kernel(
    const float* __restrict__ G, const float* __restrict__ S_hat,
    const int* __restrict__ n_s, const int* __restrict__ n_t, int Ns, int Nt,
    int iters, float inv_tau, const float* __restrict__ a_hist,
    const float* __restrict__ b_hist, float* __restrict__ dS) {
  __shared__ float L0_[kShMaxN * kShPitch];
  __shared__ float D_[kShMaxN * kShPitch];
  __shared__ float a_[kShMaxN], b_[kShMaxN];
  DGMC_LDS float* L0 = (DGMC_LDS float*)L0_;
  DGMC_LDS float* D = (DGMC_LDS float*)D_;
  DGMC_LDS float* a = (DGMC_LDS float*)a_;
  DGMC_LDS float* b = (DGMC_LDS float*)b_;
  const int pb = xcd_remap(blockIdx.x, gridDim.x);
  const int lane = threadIdx.x;
  const int ns = n_s[pb], nt = n_t[pb];
  const int NP = Nt + 1 + (Nt & 1);      // odd pitch (<= 65)
  const float* Gb = G + (size_t)pb * Ns * Nt;
  const float* ah = a_hist + (size_t)pb * (iters + 1) * Ns;
  const float* bh = b_hist + (size_t)pb * iters * Nt;
  sk_final_pot(a, b, Ns, Nt, iters, ah, bh, lane);
  sk_load(L0, S_hat + (size_t)pb * Ns * Nt, Ns, Nt, NP, inv_tau, lane);
  __syncthreads();
  // dL of the final output: G * P (P = exp(out of the final row step)).
  for (int e = lane; e < Ns * Nt; e += kWave) {
    const int i = e / Nt, j = e - i * Nt;
    const bool v = i < ns && j < nt;
    D[i * NP + j] = v ? Gb[e] * __expf(L0[i * NP + j] - a[i] - b[j]) : 0.f;
  }
  __syncthreads();
  sk_reverse(L0, D, a, b, ns, nt, Ns, Nt, NP, iters, ah, bh, lane);
  float* out = dS + (size_t)pb * Ns * Nt;
  for (int e = lane; e < Ns * Nt; e += kWave) {
    const int i = e / Nt, j = e - i * Nt;
    out[e] = D[i * NP + j] * inv_tau;
  }
}

// ---------------------------------------------------------------------------
// Sinkhorn + transport in one kernel (the consensus step's input, Sinkhorn
// counterpart of dense_consensus.hip's softmax transport; dgmc.py:168-171
// with the normaliser swapped):
//   joint[ps + i]          = r_s[ps + i]                  (i < n_s)
//   joint[rows_s + pt + j] = sum_i P_ij r_s[ps + i]       (j < n_t)
// P is formed in place of L0 (and optionally written out, step 0's S_0).
// Lane c owns channels c + 64 q, q < CPL (R = 64 CPL); the target rows run
// in chunks of kSkJ with the P column entries read as LDS broadcasts.
constexpr int kSkJ = 8;

template <int CPL>
__global__ __launch_bounds__(kWave) void sinkhorn_transport_kernel(
    const float* __restrict__ S_hat, const int* __restrict__ ptr_s,
    const int* __restrict__ ptr_t, int Ns, int Nt, int iters, float inv_tau,
    const float* __restrict__ r_s, int rows_s, float* __restrict__ joint,
    float* __restrict__ P, float* __restrict__ a_hist,
    float* __restrict__ b_hist) {
  constexpr int R = kWave * CPL;
  __shared__ float L0_[kShMaxN * kShPitch];
  __shared__ float a_[kShMaxN], b_[kShMaxN];
  DGMC_LDS float* L0 = (DGMC_LDS float*)L0_;
  DGMC_LDS float* a = (DGMC_LDS float*)a_;
  DGMC_LDS float* b = (DGMC_LDS float*)b_;
  const int pb = xcd_remap(blockIdx.x, gridDim.x);
  const int lane = threadIdx.x;
  const int ps = ptr_s[pb], ns = ptr_s[pb + 1] - ps;
  const int pt = ptr_t[pb], nt = ptr_t[pb + 1] - pt;
  const int NP = Nt + 1 + (Nt & 1);      // odd pitch (<= 65)
  sk_load(L0, S_hat + (size_t)pb * Ns * Nt, Ns, Nt, NP, inv_tau, lane);
  sk_iterate(L0, a, b, ns, nt, Ns, Nt, NP, iters,
             a_hist + (size_t)pb * (iters + 1) * Ns,
             b_hist + (size_t)pb * iters * Nt, lane);
  float* Pb = P ? P + (size_t)pb * Ns * Nt : nullptr;
  for (int e = lane; e < Ns * Nt; e += kWave) {
    const int i = e / Nt, j = e - i * Nt;
    const float v =
        (i < ns && j < nt) ? __expf(L0[i * NP + j] - a[i] - b[j]) : 0.f;
    L0[i * NP + j] = v;      // each entry read and rewritten by one lane
    if (Pb) Pb[e] = v;
  }
  __syncthreads();
  const float* rs = r_s + (size_t)ps * R + lane;
  float* js = joint + (size_t)ps * R + lane;
  for (int i = 0; i < ns; ++i)
#pragma unroll
    for (int q = 0; q < CPL; ++q) js[i * R + q * kWave] = rs[i * R + q * kWave];
  float* jt = joint + ((size_t)rows_s + pt) * R + lane;
  for (int j0 = 0; j0 < nt; j0 += kSkJ) {
    float acc[kSkJ][CPL];
#pragma unroll
    for (int jj = 0; jj < kSkJ; ++jj)
#pragma unroll
      for (int q = 0; q < CPL; ++q) acc[jj][q] = 0.f;
    for (int i = 0; i < ns; ++i) {
      float rv[CPL];
#pragma unroll
      for (int q = 0; q < CPL; ++q) rv[q] = rs[i * R + q * kWave];
      const DGMC_LDS float* Pr = L0 + i * NP + j0;
#pragma unroll
      for (int jj = 0; jj < kSkJ; ++jj) {
        const float p = j0 + jj < nt ? Pr[jj] : 0.f;
#pragma unroll
        for (int q = 0; q < CPL; ++q) acc[jj][q] = fmaf(p, rv[q], acc[jj][q]);
      }
    }
#pragma unroll
    for (int jj = 0; jj < kSkJ; ++jj)
      if (j0 + jj < nt)
#pragma unroll
        for (int q = 0; q < CPL; ++q)
          jt[(j0 + jj) * R + q * kWave] = acc[jj][q];
  }
}

// Backward of sinkhorn_transport: with g_t = d joint[rows_s + pt + j] and
// G_P = dL/dP (optional: step 0's S_0 loss),
//   dL/dP_ij = G_P_ij + <r_s[ps + i], g_t[j]>,
// then the Sinkhorn Jacobians as in sinkhorn_bwd_kernel; dS = D / tau
// (+ add, the gradient of S_hat's other consumer).  The inner products run
// over kSkC-channel chunks of r_s / g_t staged in LDS, lane per (i, j).
constexpr int kSkC = 32;
constexpr int kSkCP = kSkC + 4;       // 16-byte rows, bank-shifted
typedef float sk_f4 __attribute__((ext_vector_type(4)));

template <int CPL>
__global__ __launch_bounds__(kWave) void sinkhorn_transport_bwd_kernel(
    const float* __restrict__ G, const float* __restrict__ g_joint,
    const float* __restrict__ r_s, const float* __restrict__ S_hat,
    const int* __restrict__ ptr_s, const int* __restrict__ ptr_t, int Ns,
    int Nt, int iters, float inv_tau, int rows_s,
    const float* __restrict__ a_hist, const float* __restrict__ b_hist,
    const float* __restrict__ add, float* __restrict__ dS) {
  constexpr int R = kWave * CPL;
  __shared__ float L0_[kShMaxN * kShPitch];
  __shared__ float D_[kShMaxN * kShPitch];
  __shared__ __attribute__((aligned(16))) float rc_[kShMaxN * kSkCP];
  __shared__ __attribute__((aligned(16))) float gc_[kShMaxN * kSkCP];
  __shared__ float a_[kShMaxN], b_[kShMaxN];
  DGMC_LDS float* L0 = (DGMC_LDS float*)L0_;
  DGMC_LDS float* D = (DGMC_LDS float*)D_;
  DGMC_LDS float* rc = (DGMC_LDS float*)rc_;
  DGMC_LDS float* gc = (DGMC_LDS float*)gc_;
  DGMC_LDS float* a = (DGMC_LDS float*)a_;
  DGMC_LDS float* b = (DGMC_LDS float*)b_;
  const int pb = xcd_remap(blockIdx.x, gridDim.x);
  const int lane = threadIdx.x;
  const int ps = ptr_s[pb], ns = ptr_s[pb + 1] - ps;
  const int pt = ptr_t[pb], nt = ptr_t[pb + 1] - pt;
  const int NP = Nt + 1 + (Nt & 1);      // odd pitch (<= 65)
  const size_t off = (size_t)pb * Ns * Nt;
  const float* ah = a_hist + (size_t)pb * (iters + 1) * Ns;
  const float* bh = b_hist + (size_t)pb * iters * Nt;
  sk_final_pot(a, b, Ns, Nt, iters, ah, bh, lane);
  sk_load(L0, S_hat + off, Ns, Nt, NP, inv_tau, lane);
  for (int e = lane; e < Ns * Nt; e += kWave) {
    const int i = e / Nt, j = e - i * Nt;
    D[i * NP + j] = G ? G[off + e] : 0.f;
  }
  // <r_s[i], g_t[j]> over channel chunks: 8 lanes stage one 32-float row.
  const float* rs = r_s + (size_t)ps * R;
  const float* gt = g_joint + ((size_t)rows_s + pt) * R;
  const int sr = lane >> 3, sc = (lane & 7) * 4;
  for (int c0 = 0; c0 < R; c0 += kSkC) {
    __syncthreads();                     // previous chunk's readers done
    for (int i = sr; i < ns; i += kWave / 8)
      *(DGMC_LDS sk_f4*)(rc + i * kSkCP + sc) =
          *(const sk_f4*)(rs + (size_t)i * R + c0 + sc);
    for (int j = sr; j < nt; j += kWave / 8)
      *(DGMC_LDS sk_f4*)(gc + j * kSkCP + sc) =
          *(const sk_f4*)(gt + (size_t)j * R + c0 + sc);
    __syncthreads();
    for (int e = lane; e < ns * nt; e += kWave) {
      const int i = e / nt, j = e - i * nt;
      const DGMC_LDS sk_f4* x = (const DGMC_LDS sk_f4*)(rc + i * kSkCP);
      const DGMC_LDS sk_f4* y = (const DGMC_LDS sk_f4*)(gc + j * kSkCP);
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < kSkC / 4; ++k) {
        const sk_f4 u = x[k], v = y[k];
        s = fmaf(u.x, v.x, s);
        s = fmaf(u.y, v.y, s);
        s = fmaf(u.z, v.z, s);
        s = fmaf(u.w, v.w, s);
      }
      D[i * NP + j] += s;
    }
  }
  __syncthreads();
  // dL of the final output -> times P.
  for (int e = lane; e < Ns * Nt; e += kWave) {
    const int i = e / Nt, j = e - i * Nt;
    const bool v = i < ns && j < nt;
    D[i * NP + j] =
        v ? D[i * NP + j] * __expf(L0[i * NP + j] - a[i] - b[j]) : 0.f;
  }
  __syncthreads();
  sk_reverse(L0, D, a, b, ns, nt, Ns, Nt, NP, iters, ah, bh, lane);
  float* out = dS + off;
  for (int e = lane; e < Ns * Nt; e += kWave) {
    const int i = e / Nt, j = e - i * Nt;
    out[e] = D[i * NP + j] * inv_tau + (add ? add[off + e] : 0.f);
  }
}

static void sh_check(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat &&
                  t.is_contiguous() && t.dim() == 3,
              name, " must be a contiguous fp32 [B, Ns, Nt] GPU tensor");
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> sinkhorn_fwd(
    const at::Tensor& S_hat, const at::Tensor& n_s, const at::Tensor& n_t,
    int64_t iters, double tau) {
  sh_check(S_hat, "S_hat");
  const int64_t B = S_hat.size(0), Ns = S_hat.size(1), Nt = S_hat.size(2);
  TORCH_CHECK(Ns <= kShMaxN && Nt <= kShMaxN, "sinkhorn: pair tile > 64");
  TORCH_CHECK(n_s.scalar_type() == at::kInt && n_t.scalar_type() == at::kInt &&
                  n_s.numel() == B && n_t.numel() == B,
              "sinkhorn: int32 node counts [B]");
  TORCH_CHECK(iters >= 0 && tau > 0, "sinkhorn: iters >= 0, tau > 0");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(S_hat.device());
  at::Tensor P = at::empty_like(S_hat);
  at::Tensor ah = at::empty({B, iters + 1, Ns}, S_hat.options());
  at::Tensor bh = at::empty({B, std::max<int64_t>(iters, 1), Nt},
                            S_hat.options());
  if (B == 0) return {P, ah, bh};
  hipLaunchKernelGGL(sinkhorn_fwd_kernel, dim3(B), dim3(kWave), 0,
                     stream(), S_hat.data_ptr<float>(), n_s.data_ptr<int>(),
                     n_t.data_ptr<int>(), (int)Ns, (int)Nt, (int)iters,
                     (float)(1.0 / tau), P.data_ptr<float>(),
                     ah.data_ptr<float>(), bh.data_ptr<float>());
  DGMC_CHECK_LAUNCH();
  return {P, ah, bh};
}

at::Tensor sinkhorn_bwd(const at::Tensor& G, const at::Tensor& S_hat,
                        const at::Tensor& n_s, const at::Tensor& n_t,
                        const at::Tensor& a_hist, const at::Tensor& b_hist,
                        int64_t iters, double tau) {
  sh_check(G, "grad");
  sh_check(S_hat, "S_hat");
  TORCH_CHECK(G.sizes() == S_hat.sizes(), "sinkhorn_bwd: grad shape");
  const int64_t B = S_hat.size(0), Ns = S_hat.size(1), Nt = S_hat.size(2);
  TORCH_CHECK(Ns <= kShMaxN && Nt <= kShMaxN, "sinkhorn: pair tile > 64");
  TORCH_CHECK(a_hist.is_contiguous() && b_hist.is_contiguous() &&
                  a_hist.numel() == B * (iters + 1) * Ns &&
                  b_hist.numel() >= B * iters * Nt,
              "sinkhorn_bwd: potentials of the forward");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(S_hat.device());
  at::Tensor dS = at::empty_like(S_hat);
  if (B == 0) return dS;
  hipLaunchKernelGGL(sinkhorn_bwd_kernel, dim3(B), dim3(kWave), 0,
                     stream(), G.data_ptr<float>(), S_hat.data_ptr<float>(),
                     n_s.data_ptr<int>(), n_t.data_ptr<int>(), (int)Ns,
                     (int)Nt, (int)iters, (float)(1.0 / tau),
                     a_hist.data_ptr<float>(), b_hist.data_ptr<float>(),
                     dS.data_ptr<float>());
  DGMC_CHECK_LAUNCH();
  return dS;
}

static void sk_ptr_check(const at::Tensor& ptr, int64_t B, const char* name) {
  TORCH_CHECK(ptr.is_cuda() && ptr.scalar_type() == at::kInt &&
                  ptr.is_contiguous() && ptr.numel() == B + 1,
              name, " must be int32 [B + 1] pair offsets on the GPU");
}

static void sk_rows_check(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat &&
                  t.is_contiguous() && t.dim() == 2 &&
                  t.data_ptr() != nullptr &&
                  reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0,
              name, " must be a contiguous 16-byte aligned fp32 [rows, R]");
}

template <typename F>
static void sk_dispatch_cpl(int64_t R, F&& f) {
  switch (R) {
    case 64: f(std::integral_constant<int, 1>()); break;
    case 128: f(std::integral_constant<int, 2>()); break;
    case 256: f(std::integral_constant<int, 4>()); break;
    default: TORCH_CHECK(false, "sinkhorn_transport: R in {64, 128, 256}");
  }
}

std::vector<at::Tensor> sinkhorn_transport(const at::Tensor& S_hat,
                                           const at::Tensor& r_s,
                                           const at::Tensor& ptr_s,
                                           const at::Tensor& ptr_t,
                                           int64_t rows_t, int64_t iters,
                                           double tau, bool with_prob) {
  sh_check(S_hat, "S_hat");
  sk_rows_check(r_s, "r_s");
  const int64_t B = S_hat.size(0), Ns = S_hat.size(1), Nt = S_hat.size(2);
  const int64_t R = r_s.size(1), rows_s = r_s.size(0);
  TORCH_CHECK(Ns <= kShMaxN && Nt <= kShMaxN, "sinkhorn: pair tile > 64");
  TORCH_CHECK(iters >= 0 && tau > 0, "sinkhorn: iters >= 0, tau > 0");
  sk_ptr_check(ptr_s, B, "ptr_s");
  sk_ptr_check(ptr_t, B, "ptr_t");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(S_hat.device());
  at::Tensor joint = at::empty({rows_s + rows_t, R}, r_s.options());
  at::Tensor P = with_prob ? at::empty_like(S_hat) : at::Tensor();
  at::Tensor ah = at::empty({B, iters + 1, Ns}, S_hat.options());
  at::Tensor bh = at::empty({B, std::max<int64_t>(iters, 1), Nt},
                            S_hat.options());
  if (B == 0) return {joint, P, ah, bh};
  sk_dispatch_cpl(R, [&](auto cpl) {
    hipLaunchKernelGGL(sinkhorn_transport_kernel<decltype(cpl)::value>,
                       dim3(B), dim3(kWave), 0, stream(),
                       S_hat.data_ptr<float>(), ptr_s.data_ptr<int>(),
                       ptr_t.data_ptr<int>(), (int)Ns, (int)Nt, (int)iters,
                       (float)(1.0 / tau), r_s.data_ptr<float>(), (int)rows_s,
                       joint.data_ptr<float>(),
                       with_prob ? P.data_ptr<float>() : nullptr,
                       ah.data_ptr<float>(), bh.data_ptr<float>());
  });
  DGMC_CHECK_LAUNCH();
  return {joint, P, ah, bh};
}

at::Tensor sinkhorn_transport_bwd(const c10::optional<at::Tensor>& G,
                                  const at::Tensor& g_joint,
                                  const at::Tensor& r_s,
                                  const at::Tensor& S_hat,
                                  const at::Tensor& ptr_s,
                                  const at::Tensor& ptr_t,
                                  const at::Tensor& a_hist,
                                  const at::Tensor& b_hist, int64_t iters,
                                  double tau,
                                  const c10::optional<at::Tensor>& add) {
  sh_check(S_hat, "S_hat");
  sk_rows_check(r_s, "r_s");
  sk_rows_check(g_joint, "grad joint");
  const int64_t B = S_hat.size(0), Ns = S_hat.size(1), Nt = S_hat.size(2);
  const int64_t R = r_s.size(1), rows_s = r_s.size(0);
  TORCH_CHECK(Ns <= kShMaxN && Nt <= kShMaxN, "sinkhorn: pair tile > 64");
  TORCH_CHECK(g_joint.size(1) == R && g_joint.size(0) >= rows_s,
              "sinkhorn_transport_bwd: grad joint shape");
  sk_ptr_check(ptr_s, B, "ptr_s");
  sk_ptr_check(ptr_t, B, "ptr_t");
  TORCH_CHECK(a_hist.is_contiguous() && b_hist.is_contiguous() &&
                  a_hist.numel() == B * (iters + 1) * Ns &&
                  b_hist.numel() >= B * iters * Nt,
              "sinkhorn_transport_bwd: potentials of the forward");
  const float* gp = nullptr;
  if (G.has_value() && G->defined()) {
    sh_check(*G, "grad P");
    TORCH_CHECK(G->sizes() == S_hat.sizes(), "grad P shape");
    gp = G->data_ptr<float>();
  }
  const float* ad = nullptr;
  if (add.has_value() && add->defined()) {
    sh_check(*add, "addend");
    TORCH_CHECK(add->sizes() == S_hat.sizes(), "addend shape");
    ad = add->data_ptr<float>();
  }
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(S_hat.device());
  at::Tensor dS = at::empty_like(S_hat);
  if (B == 0) return dS;
  sk_dispatch_cpl(R, [&](auto cpl) {
    hipLaunchKernelGGL(sinkhorn_transport_bwd_kernel<decltype(cpl)::value>,
                       dim3(B), dim3(kWave), 0, stream(), gp,
                       g_joint.data_ptr<float>(), r_s.data_ptr<float>(),
                       S_hat.data_ptr<float>(), ptr_s.data_ptr<int>(),
                       ptr_t.data_ptr<int>(), (int)Ns, (int)Nt, (int)iters,
                       (float)(1.0 / tau), (int)rows_s,
                       a_hist.data_ptr<float>(), b_hist.data_ptr<float>(), ad,
                       dS.data_ptr<float>());
  });
  DGMC_CHECK_LAUNCH();
  return dS;
}

}  // namespace dgmc
