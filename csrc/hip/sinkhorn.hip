// Masked log-domain Sinkhorn normalisation of the dense correspondence
// scores, one wave per graph pair (opt-in `normalization='sinkhorn'` of
// DGMC; the reference itself only row-normalises with a masked softmax,
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
//
// Register-resident (N <= 64, compile-time bucket NM in {16, 24, 32, 48, 64}):
// lane i holds row i of L0 (r[]) and lane j column j (c[]) in VGPRs; the
// potentials live one per lane (a in lane i, b in lane j) and reach the
// other lanes by v_readlane (scalar broadcast) - a half-step is NM
// unrolled sub / max / exp per lane with no LDS traffic and no barrier.
// The backward keeps D in registers too and switches it between the row and
// the column layout through a conflict-free LDS transpose (odd pitch).
// Was: the tile in LDS with a sequential LSE loop per lane (~20 dependent
// LDS reads per half-step); before that one wave-wide LSE per row with a
// block barrier per half-step (docs/performance.md).  Deterministic, no
// atomics.
#include "common.h"

namespace dgmc {

namespace {
constexpr int kShMaxN = 64;
typedef float sk_f4 __attribute__((ext_vector_type(4)));
typedef float sk_f16v __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float sk_rl(float v, int l) {
  return __builtin_bit_cast(
      float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}

// LSE_k (x[k] - pot of lane k) over k < NM (x = -inf excluded); 0 if empty.
// (Fully unrolled over the bucket: wave-uniform early exits at the pair's
// own size measured SLOWER - 50 -> 77 us per backward - the per-k branch
// serialises the readlane / exp chains.)
template <int NM>
__device__ __forceinline__ float sk_lse(const float (&x)[NM], float pot) {
  float t[NM];
  float m = -INFINITY;
#pragma unroll
  for (int k = 0; k < NM; ++k) {
    t[k] = x[k] - sk_rl(pot, k);
    m = fmaxf(m, t[k]);
  }
  if (m == -INFINITY) return 0.f;
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < NM; ++k) s += __expf(t[k] - m);
  return m + __logf(s);
}

// Row copy (lane i: r[j] = L0_ij) and column copy (lane j: c[i] = L0_ij) of
// a pair tile S [Ns, Nt]; -inf outside the valid n_s x n_t block.
template <int NM>
__device__ __forceinline__ void sk_load_regs(const float* S, int Nt, int ns,
                                             int nt, float inv_tau, int lane,
                                             float (&r)[NM], float (&c)[NM]) {
  const bool rv = lane < ns, cv = lane < nt;
#pragma unroll
  for (int k = 0; k < NM; ++k) {
    r[k] = (rv && k < nt) ? S[lane * Nt + k] * inv_tau : -INFINITY;
    c[k] = (cv && k < ns) ? S[k * Nt + lane] * inv_tau : -INFINITY;
  }
}

// The forward iterations: final potentials in a (lane i) / b (lane j),
// every half-step's recorded in ah ([iters + 1, Ns]) / bh ([iters, Nt]).
template <int NM>
__device__ __forceinline__ void sk_iterate(const float (&r)[NM],
                                           const float (&c)[NM], int ns,
                                           int nt, int Ns, int Nt, int iters,
                                           float* ah, float* bh, int lane,
                                           float& a, float& b) {
  a = 0.f;
  b = 0.f;
  for (int it = 0; it <= iters; ++it) {
    const float x = sk_lse<NM>(r, b);       // row step: lane i
    a = lane < ns ? x : 0.f;
    if (lane < Ns) ah[it * Ns + lane] = a;
    if (it == iters) break;
    const float y = sk_lse<NM>(c, a);       // column step: lane j
    b = lane < nt ? y : 0.f;
    if (lane < Nt) bh[it * Nt + lane] = b;
  }
}

// r[] <- row of P = exp(L0 - a - b) (0 outside the valid block).
template <int NM>
__device__ __forceinline__ void sk_prob_row(float (&r)[NM], float a, float b,
                                            int ns, int nt, int lane) {
#pragma unroll
  for (int k = 0; k < NM; ++k) {
    const float p = __expf(r[k] - a - sk_rl(b, k));
    r[k] = (lane < ns && k < nt) ? p : 0.f;
  }
}

// D between the row layout (lane i: d[j] = D_ij) and the column layout
// (lane j: d[i] = D_ij) through the LDS tile Dl [NM][NM + 1].
template <int NM>
__device__ __forceinline__ void sk_transpose(float (&d)[NM], DGMC_LDS float* Dl,
                                             int lane, bool row_to_col) {
  constexpr int DP = NM + 1;
  if (lane < NM) {
#pragma unroll
    for (int k = 0; k < NM; ++k)
      Dl[row_to_col ? lane * DP + k : k * DP + lane] = d[k];
  }
  __syncthreads();
  if (lane < NM) {
#pragma unroll
    for (int k = 0; k < NM; ++k)
      d[k] = Dl[row_to_col ? k * DP + lane : lane * DP + k];
  }
  __syncthreads();
}
}  // namespace

template <int NM>
__global__ __launch_bounds__(kWave) void sinkhorn_fwd_kernel(
    const float* __restrict__ S_hat, const int* __restrict__ n_s,
    const int* __restrict__ n_t, int Ns, int Nt, int iters, float inv_tau,
    float* __restrict__ P, float* __restrict__ a_hist,
    float* __restrict__ b_hist) {
  const int pb = xcd_remap(blockIdx.x, gridDim.x);
  const int lane = threadIdx.x;
  const int ns = n_s[pb], nt = n_t[pb];
  const size_t off = (size_t)pb * Ns * Nt;
  float r[NM], c[NM], a, b;
  sk_load_regs<NM>(S_hat + off, Nt, ns, nt, inv_tau, lane, r, c);
  sk_iterate<NM>(r, c, ns, nt, Ns, Nt, iters,
                 a_hist + (size_t)pb * (iters + 1) * Ns,
                 b_hist + (size_t)pb * iters * Nt, lane, a, b);
  sk_prob_row<NM>(r, a, b, ns, nt, lane);
  if (lane < Ns) {
    float* Pr = P + off + (size_t)lane * Nt;
#pragma unroll
    for (int k = 0; k < NM; ++k)
      if (k < Nt) Pr[k] = r[k];
  }
}

// ---------------------------------------------------------------------------
// Sinkhorn + transport in one kernel (the consensus step's input, Sinkhorn
// counterpart of dense_consensus.hip's softmax transport; dgmc.py:168-171
// with the normaliser swapped):
//   joint[ps + i]          = r_s[ps + i]                  (i < n_s)
//   joint[rows_s + pt + j] = sum_i P_ij r_s[ps + i]       (j < n_t)
// P is formed in place of the row copy (and optionally written out, step
// 0's S_0).  Lane c owns channels c + 64 q, q < CPL (R = 64 CPL); P_ij
// reaches the channel lanes by v_readlane from lane i, kSkJ target rows of
// accumulators at a time.
constexpr int kSkJ = 16;

template <int NM, int CPL>
__global__ __launch_bounds__(kWave) void sinkhorn_transport_kernel(
    const float* __restrict__ S_hat, const int* __restrict__ ptr_s,
    const int* __restrict__ ptr_t, int Ns, int Nt, int iters, float inv_tau,
    const float* __restrict__ r_s, int rows_s, float* __restrict__ joint,
    float* __restrict__ P, float* __restrict__ a_hist,
    float* __restrict__ b_hist) {
  constexpr int R = kWave * CPL;
  constexpr int JC = NM % kSkJ == 0 ? kSkJ : 8;     // divides NM
  const int pb = xcd_remap(blockIdx.x, gridDim.x);
  const int lane = threadIdx.x;
  const int ps = ptr_s[pb], ns = ptr_s[pb + 1] - ps;
  const int pt = ptr_t[pb], nt = ptr_t[pb + 1] - pt;
  const size_t off = (size_t)pb * Ns * Nt;
  float r[NM], c[NM], a, b;
  sk_load_regs<NM>(S_hat + off, Nt, ns, nt, inv_tau, lane, r, c);
  sk_iterate<NM>(r, c, ns, nt, Ns, Nt, iters,
                 a_hist + (size_t)pb * (iters + 1) * Ns,
                 b_hist + (size_t)pb * iters * Nt, lane, a, b);
  sk_prob_row<NM>(r, a, b, ns, nt, lane);
  if (P && lane < Ns) {
    float* Pr = P + off + (size_t)lane * Nt;
#pragma unroll
    for (int k = 0; k < NM; ++k)
      if (k < Nt) Pr[k] = r[k];
  }
  const float* rs = r_s + (size_t)ps * R + lane;
  float* js = joint + (size_t)ps * R + lane;
  for (int i = 0; i < ns; ++i)
#pragma unroll
    for (int q = 0; q < CPL; ++q) js[i * R + q * kWave] = rs[i * R + q * kWave];
  if constexpr (NM <= 32) {
    // r_t^T blocks on the matrix cores (v_mfma_f32_32x32x2_f32): A = P^T
    // (lane l: row j = l % 32, k = i of the pair 2 t + l / 32, read from the
    // transposed P tile), B = r_s (k = i, 32 channels), one 32 x 32 output
    // block per 32 channels.
    constexpr int DP = NM + 1;
    __shared__ float Pt_[NM * DP];
    DGMC_LDS float* Pt = (DGMC_LDS float*)Pt_;
    if (lane < NM) {
#pragma unroll
      for (int k = 0; k < NM; ++k) Pt[lane * DP + k] = r[k];   // P[i][j]
    }
    __syncthreads();
    const int lj = lane & 31, hh = lane >> 5;
    const float* rb = r_s + (size_t)ps * R + lj;
    sk_f16v acc[CPL * 2];
#pragma unroll
    for (int b = 0; b < 2 * CPL; ++b)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[b][q] = 0.f;
    for (int i0 = 0; i0 < ns; i0 += 2) {
      const int i = i0 + hh;
      const bool vi = i < ns;
      const float a = (vi && lj < NM) ? Pt[i * DP + lj] : 0.f;
#pragma unroll
      for (int b = 0; b < 2 * CPL; ++b) {
        const float bv = vi ? rb[(size_t)i * R + 32 * b] : 0.f;
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bv, acc[b], 0, 0,
                                                      0);
      }
    }
    float* jt = joint + ((size_t)rows_s + pt) * R + lj;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int j = 8 * (q >> 2) + 4 * hh + (q & 3);
      if (j < nt)
#pragma unroll
        for (int b = 0; b < 2 * CPL; ++b) jt[(size_t)j * R + 32 * b] = acc[b][q];
    }
  } else {
    float* jt = joint + ((size_t)rows_s + pt) * R + lane;
#pragma unroll
    for (int j0 = 0; j0 < NM; j0 += JC) {
      if (j0 >= nt) break;
      float acc[JC][CPL];
#pragma unroll
      for (int jj = 0; jj < JC; ++jj)
#pragma unroll
        for (int q = 0; q < CPL; ++q) acc[jj][q] = 0.f;
      for (int i = 0; i < ns; ++i) {
        float rv[CPL];
#pragma unroll
        for (int q = 0; q < CPL; ++q) rv[q] = rs[i * R + q * kWave];
#pragma unroll
        for (int jj = 0; jj < JC; ++jj) {
          const float p = sk_rl(r[j0 + jj], i);
#pragma unroll
          for (int q = 0; q < CPL; ++q)
            acc[jj][q] = fmaf(p, rv[q], acc[jj][q]);
        }
      }
#pragma unroll
      for (int jj = 0; jj < JC; ++jj)
        if (j0 + jj < nt)
#pragma unroll
          for (int q = 0; q < CPL; ++q)
            jt[(j0 + jj) * R + q * kWave] = acc[jj][q];
    }
  }
}

// Backward, plain (TR = false: G = dL/dP, counts n_s / n_t) or of
// sinkhorn_transport (TR = true: ptr_s / ptr_t, g_t = d joint[rows_s + pt +
// j], optional G_P):
//   dL/dP_ij = G_P_ij + <r_s[ps + i], g_t[j]>
// (inner products over kSkC-channel chunks staged in LDS, lane per (i, j)),
// then the Sinkhorn Jacobians in reverse; dS = D / tau (+ add, the gradient
// of S_hat's other consumer).  The potentials of every half-step are staged
// in LDS once (dynamic, (iters + 1) Ns + iters Nt floats).
constexpr int kSkC = 32;
constexpr int kSkCP = kSkC + 4;       // 16-byte rows, bank-shifted

template <int NM, bool TR, int CPL>
__global__ __launch_bounds__(kWave) void sinkhorn_bwd_kernel(
    const float* __restrict__ G, const float* __restrict__ g_joint,
    const float* __restrict__ r_s, const float* __restrict__ S_hat,
    const int* __restrict__ cnt_s, const int* __restrict__ cnt_t, int Ns,
    int Nt, int iters, float inv_tau, int rows_s,
    const float* __restrict__ a_hist, const float* __restrict__ b_hist,
    const float* __restrict__ add, float* __restrict__ dS) {
  constexpr int R = kWave * CPL;
  constexpr int DP = NM + 1;
  constexpr int CH = (TR && NM > 32) ? NM * kSkCP : 1;
  __shared__ float Dl_[NM * DP];
  __shared__ __attribute__((aligned(16))) float rc_[CH];
  __shared__ __attribute__((aligned(16))) float gc_[CH];
  extern __shared__ float hist_[];
  DGMC_LDS float* Dl = (DGMC_LDS float*)Dl_;
  DGMC_LDS float* ahs = (DGMC_LDS float*)hist_;
  DGMC_LDS float* bhs = ahs + (iters + 1) * Ns;
  const int pb = xcd_remap(blockIdx.x, gridDim.x);
  const int lane = threadIdx.x;
  int ns, nt, ps = 0, pt = 0;
  if (TR) {   // cnt_* are the pair offsets
    ps = cnt_s[pb];
    ns = cnt_s[pb + 1] - ps;
    pt = cnt_t[pb];
    nt = cnt_t[pb + 1] - pt;
  } else {
    ns = cnt_s[pb];
    nt = cnt_t[pb];
  }
  const size_t off = (size_t)pb * Ns * Nt;
  {
    const float* ah = a_hist + (size_t)pb * (iters + 1) * Ns;
    const float* bh = b_hist + (size_t)pb * iters * Nt;
    for (int e = lane; e < (iters + 1) * Ns; e += kWave) ahs[e] = ah[e];
    for (int e = lane; e < iters * Nt; e += kWave) bhs[e] = bh[e];
  }
  float r[NM], c[NM], d[NM];
  sk_load_regs<NM>(S_hat + off, Nt, ns, nt, inv_tau, lane, r, c);
  if (TR && NM <= 32) {
    // D = G_P + <r_s[i], g_t[j]>: the 32 x 32 product block on the matrix
    // cores (v_mfma_f32_32x32x2_f32; lane l feeds row l % 32 of r_s and of
    // g_t, channel half l / 32 of each k pair).
    for (int e = lane; e < Ns * Nt; e += kWave) {
      const int i = e / Nt, j = e - i * Nt;
      Dl[i * DP + j] = G ? G[off + e] : 0.f;
    }
    const int li = lane & 31, hh = lane >> 5;
    const bool va = li < ns, vb = li < nt;
    const float* ra = r_s + ((size_t)ps + li) * R + hh * (R / 2);
    const float* gb = g_joint + ((size_t)rows_s + pt + li) * R + hh * (R / 2);
    sk_f16v acc;
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[q] = 0.f;
    for (int c0 = 0; c0 < R / 2; c0 += 16) {
      sk_f4 av[4], bv[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        av[q] = va ? *(const sk_f4*)(ra + c0 + 4 * q) : sk_f4{0.f, 0.f, 0.f, 0.f};
        bv[q] = vb ? *(const sk_f4*)(gb + c0 + 4 * q) : sk_f4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int t = 0; t < 4; ++t)
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[q][t], bv[q][t], acc,
                                                     0, 0, 0);
    }
    __syncthreads();                     // G staged
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int i = 8 * (q >> 2) + 4 * hh + (q & 3);
      if (i < NM && li < NM) Dl[i * DP + li] += acc[q];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NM; ++k)
      d[k] = (lane < Ns && k < Nt) ? Dl[lane * DP + k] : 0.f;
    __syncthreads();
  } else if (TR) {
    // D = G_P + <r_s[i], g_t[j]> in the LDS tile (8 lanes stage one row).
    DGMC_LDS float* rc = (DGMC_LDS float*)rc_;
    DGMC_LDS float* gc = (DGMC_LDS float*)gc_;
    for (int e = lane; e < Ns * Nt; e += kWave) {
      const int i = e / Nt, j = e - i * Nt;
      Dl[i * DP + j] = G ? G[off + e] : 0.f;
    }
    const float* rs = r_s + (size_t)ps * R;
    const float* gt = g_joint + ((size_t)rows_s + pt) * R;
    const int sr = lane >> 3, sc = (lane & 7) * 4;
    for (int c0 = 0; c0 < R; c0 += kSkC) {
      __syncthreads();                   // previous chunk's readers done
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
        Dl[i * DP + j] += s;
      }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NM; ++k)
      d[k] = (lane < Ns && k < Nt) ? Dl[lane * DP + k] : 0.f;
    __syncthreads();
  } else {
    __syncthreads();
    const float* Gr = G + off + (size_t)lane * Nt;
#pragma unroll
    for (int k = 0; k < NM; ++k) d[k] = (lane < Ns && k < Nt) ? Gr[k] : 0.f;
  }
  // dL of the final output -> times P (final row step's potentials).
  float a = lane < Ns ? ahs[iters * Ns + lane] : 0.f;
  float b = (lane < Nt && iters > 0) ? bhs[(iters - 1) * Nt + lane] : 0.f;
#pragma unroll
  for (int k = 0; k < NM; ++k) {
    const float p = __expf(r[k] - a - sk_rl(b, k));
    d[k] = (lane < ns && k < nt) ? d[k] * p : 0.f;
  }
  for (int step = 2 * iters; step >= 0; --step) {
    const bool row = (step & 1) == 0;     // even: row step, odd: column step
    const int it = step >> 1;
    a = lane < Ns ? ahs[it * Ns + lane] : 0.f;
    b = lane < Nt ? (row ? (it > 0 ? bhs[(it - 1) * Nt + lane] : 0.f)
                         : bhs[it * Nt + lane])
                  : 0.f;
    // (d: row layout in a row step, column layout in a column step; zero
    // outside the valid block)
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < NM; ++k) s += d[k];
    if (row) {
      // lane i: D_ij -= exp(out_ij) sum_k D_ik
#pragma unroll
      for (int k = 0; k < NM; ++k) {
        const float e = __expf(r[k] - a - sk_rl(b, k));
        d[k] = lane < ns ? fmaf(-e, s, d[k]) : d[k];
      }
      if (step > 0) sk_transpose<NM>(d, Dl, lane, true);
    } else {
      // lane j: D_ij -= exp(out_ij) sum_k D_kj
#pragma unroll
      for (int k = 0; k < NM; ++k) {
        const float e = __expf(c[k] - sk_rl(a, k) - b);
        d[k] = lane < nt ? fmaf(-e, s, d[k]) : d[k];
      }
      sk_transpose<NM>(d, Dl, lane, false);
    }
  }
  if (lane < Ns) {
    float* out = dS + off + (size_t)lane * Nt;
    const float* ad = add ? add + off + (size_t)lane * Nt : nullptr;
#pragma unroll
    for (int k = 0; k < NM; ++k)
      if (k < Nt)
        out[k] = (lane < ns && k < nt ? d[k] * inv_tau : 0.f) +
                 (ad ? ad[k] : 0.f);
  }
}

// ---------------------------------------------------------------------------
static void sh_check(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat &&
                  t.is_contiguous() && t.dim() == 3,
              name, " must be a contiguous fp32 [B, Ns, Nt] GPU tensor");
}

// Compile-time tile bucket of the register-resident kernels.
template <typename F>
static void sk_dispatch_nm(int64_t Ns, int64_t Nt, F&& f) {
  const int64_t n = std::max(Ns, Nt);
  TORCH_CHECK(n <= kShMaxN, "sinkhorn: pair tile > 64");
  if (n <= 16)
    f(std::integral_constant<int, 16>());
  else if (n <= 24)
    f(std::integral_constant<int, 24>());
  else if (n <= 32)
    f(std::integral_constant<int, 32>());
  else if (n <= 48)
    f(std::integral_constant<int, 48>());
  else
    f(std::integral_constant<int, 64>());
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

// Dynamic LDS of the backward (the potentials of every half-step).
template <typename K>
static size_t sk_hist_lds(K kern, int64_t iters, int64_t Ns, int64_t Nt) {
  const size_t bytes =
      (size_t)((iters + 1) * Ns + iters * Nt) * sizeof(float);
  TORCH_CHECK(bytes <= 96 * 1024, "sinkhorn_bwd: too many iterations (",
              iters, ") for the LDS-staged potentials");
  if (bytes > 48 * 1024)
    DGMC_CHECK_HIP(hipFuncSetAttribute(
        reinterpret_cast<const void*>(kern),
        hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
  return bytes;
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
  sk_dispatch_nm(Ns, Nt, [&](auto nm) {
    hipLaunchKernelGGL(sinkhorn_fwd_kernel<decltype(nm)::value>, dim3(B),
                       dim3(kWave), 0, stream(), S_hat.data_ptr<float>(),
                       n_s.data_ptr<int>(), n_t.data_ptr<int>(), (int)Ns,
                       (int)Nt, (int)iters, (float)(1.0 / tau),
                       P.data_ptr<float>(), ah.data_ptr<float>(),
                       bh.data_ptr<float>());
  });
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
  TORCH_CHECK(n_s.scalar_type() == at::kInt && n_t.scalar_type() == at::kInt &&
                  n_s.numel() == B && n_t.numel() == B,
              "sinkhorn: int32 node counts [B]");
  TORCH_CHECK(a_hist.is_contiguous() && b_hist.is_contiguous() &&
                  a_hist.numel() == B * (iters + 1) * Ns &&
                  b_hist.numel() >= B * iters * Nt,
              "sinkhorn_bwd: potentials of the forward");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(S_hat.device());
  at::Tensor dS = at::empty_like(S_hat);
  if (B == 0) return dS;
  sk_dispatch_nm(Ns, Nt, [&](auto nm) {
    auto kern = sinkhorn_bwd_kernel<decltype(nm)::value, false, 1>;
    const size_t lds = sk_hist_lds(kern, iters, Ns, Nt);
    hipLaunchKernelGGL(kern, dim3(B), dim3(kWave), lds, stream(),
                       G.data_ptr<float>(), nullptr, nullptr,
                       S_hat.data_ptr<float>(), n_s.data_ptr<int>(),
                       n_t.data_ptr<int>(), (int)Ns, (int)Nt, (int)iters,
                       (float)(1.0 / tau), 0, a_hist.data_ptr<float>(),
                       b_hist.data_ptr<float>(), nullptr,
                       dS.data_ptr<float>());
  });
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
  sk_dispatch_nm(Ns, Nt, [&](auto nm) {
    sk_dispatch_cpl(R, [&](auto cpl) {
      hipLaunchKernelGGL(
          (sinkhorn_transport_kernel<decltype(nm)::value,
                                     decltype(cpl)::value>),
          dim3(B), dim3(kWave), 0, stream(), S_hat.data_ptr<float>(),
          ptr_s.data_ptr<int>(), ptr_t.data_ptr<int>(), (int)Ns, (int)Nt,
          (int)iters, (float)(1.0 / tau), r_s.data_ptr<float>(), (int)rows_s,
          joint.data_ptr<float>(), with_prob ? P.data_ptr<float>() : nullptr,
          ah.data_ptr<float>(), bh.data_ptr<float>());
    });
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
  sk_dispatch_nm(Ns, Nt, [&](auto nm) {
    sk_dispatch_cpl(R, [&](auto cpl) {
      auto kern = sinkhorn_bwd_kernel<decltype(nm)::value, true,
                                      decltype(cpl)::value>;
      const size_t lds = sk_hist_lds(kern, iters, Ns, Nt);
      hipLaunchKernelGGL(kern, dim3(B), dim3(kWave), lds, stream(), gp,
                         g_joint.data_ptr<float>(), r_s.data_ptr<float>(),
                         S_hat.data_ptr<float>(), ptr_s.data_ptr<int>(),
                         ptr_t.data_ptr<int>(), (int)Ns, (int)Nt, (int)iters,
                         (float)(1.0 / tau), (int)rows_s,
                         a_hist.data_ptr<float>(), b_hist.data_ptr<float>(),
                         ad, dS.data_ptr<float>());
    });
  });
  DGMC_CHECK_LAUNCH();
  return dS;
}

}  // namespace dgmc
