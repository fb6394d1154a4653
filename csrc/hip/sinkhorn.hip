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
  const float* S = S_hat + (size_t)pb * Ns * Nt;
  for (int e = lane; e < Ns * Nt; e += kWave) {
    const int i = e / Nt, j = e - i * Nt;
    L0[i * NP + j] = S[e] * inv_tau;
  }
  b[lane] = 0.f;
  a[lane] = 0.f;
  __syncthreads();
  float* ah = a_hist + (size_t)pb * (iters + 1) * Ns;
  float* bh = b_hist + (size_t)pb * iters * Nt;
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
  const float* S = S_hat + (size_t)pb * Ns * Nt;
  const float* Gb = G + (size_t)pb * Ns * Nt;
  const float* ah = a_hist + (size_t)pb * (iters + 1) * Ns;
  const float* bh = b_hist + (size_t)pb * iters * Nt;
  if (lane < Ns) a[lane] = ah[iters * Ns + lane];
  if (lane < Nt) b[lane] = iters > 0 ? bh[(iters - 1) * Nt + lane] : 0.f;
  for (int e = lane; e < Ns * Nt; e += kWave) {
    const int i = e / Nt, j = e - i * Nt;
    L0[i * NP + j] = S[e] * inv_tau;
  }
  __syncthreads();
  // dL of the final output: G * P (P = exp(out of the final row step)).
  for (int e = lane; e < Ns * Nt; e += kWave) {
    const int i = e / Nt, j = e - i * Nt;
    const bool v = i < ns && j < nt;
    D[i * NP + j] = v ? Gb[e] * __expf(L0[i * NP + j] - a[i] - b[j]) : 0.f;
  }
  __syncthreads();
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
  float* out = dS + (size_t)pb * Ns * Nt;
  for (int e = lane; e < Ns * Nt; e += kWave) {
    const int i = e / Nt, j = e - i * Nt;
    out[e] = D[i * NP + j] * inv_tau;
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

}  // namespace dgmc
