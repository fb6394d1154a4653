// Per-pair fused kernels of the dense DGMC consensus loop
// (reference dgmc.py:161-183).  One workgroup (4 waves) per graph pair; the
// padded pair tile (N_s, N_t <= 64) lives in LDS, masks are derived from the
// per-pair node counts n_s[b], n_t[b] (valid nodes occupy the leading rows).
//
//   dense_masked_softmax      S = masked_softmax(S_hat)          (dgmc.py:15-19)
//   dense_softmax_transport   S, r_t = S^T r_s                   (dgmc.py:168-171)
//   dense_consensus           S_hat + mask*(relu(P_i - Q_j).w2 + b2)
//                             = S_hat + mask*MLP(o_s_i - o_t_j)  (dgmc.py:178-179)
// and their backward kernels.  The consensus backward recomputes relu(P-Q)
// instead of storing the [B, N_s, N_t, R] activation the reference keeps.
//
// LDS tiles use a row pitch of 65 floats so that lanes reading different rows
// of the same column (ds_read_b32, 32-bank groups) are conflict-free.
#include "common.h"

namespace dgmc {

constexpr int kMaxN = 64;      // max padded nodes per graph of a pair
constexpr int kPitch = 65;     // LDS row pitch (floats)
constexpr int kCh = 64;        // channel chunk staged per pass
constexpr int kWaves = 4;      // waves per workgroup
constexpr int kRowsPerWave = kMaxN / kWaves;

// Zero rows [row0, rows) of a packed [rows, R] tensor (padding rows of static
// batches; executed by the last workgroup of a launch).
template <typename T>
__device__ __forceinline__ void zero_tail(T* __restrict__ x, int row0,
                                          int rows, int R) {
  const size_t begin = (size_t)row0 * R, end = (size_t)rows * R;
  for (size_t e = begin + threadIdx.x; e < end; e += blockDim.x)
    x[e] = Cvt<T>::from_f(0.f);
}

// ---------------------------------------------------------------------------
// Row-wise masked softmax (+ backward).  One wave per (b, i) row.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void masked_softmax_kernel(
    const float* __restrict__ S_hat, const int* __restrict__ n_s,
    const int* __restrict__ n_t, float* __restrict__ S, int B, int Ns,
    int Nt) {
  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  const int row = blockIdx.x * kWaves + wave;
  if (row >= B * Ns) return;
  const int b = row / Ns, i = row % Ns;
  const float* src = S_hat + (size_t)row * Nt;
  float* dst = S + (size_t)row * Nt;
  const int nt = i < n_s[b] ? n_t[b] : 0;
  float m = -INFINITY;
  for (int j = lane; j < nt; j += kWave) m = fmaxf(m, src[j]);
  m = wave_max(m);
  float s = 0.f;
  for (int j = lane; j < nt; j += kWave) s += __expf(src[j] - m);
  s = wave_sum(s);
  const float inv = nt > 0 ? 1.f / s : 0.f;
  for (int j = lane; j < Nt; j += kWave)
    dst[j] = j < nt ? __expf(src[j] - m) * inv : 0.f;
}

__global__ __launch_bounds__(256) void masked_softmax_bwd_kernel(
    const float* __restrict__ S, const float* __restrict__ G,
    float* __restrict__ out, int rows, int Nt) {
  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  const int row = blockIdx.x * kWaves + wave;
  if (row >= rows) return;
  const float* s = S + (size_t)row * Nt;
  const float* g = G + (size_t)row * Nt;
  float dot = 0.f;
  for (int j = lane; j < Nt; j += kWave) dot += s[j] * g[j];
  dot = wave_sum(dot);
  for (int j = lane; j < Nt; j += kWave)
    out[(size_t)row * Nt + j] = s[j] * (g[j] - dot);
}

// ---------------------------------------------------------------------------
// Softmax + transport:  S = masked_softmax(S_hat[b]);  r_t[b] = S^T r_s[b].
// ---------------------------------------------------------------------------
template <typename TR>
__global__ __launch_bounds__(256) void softmax_transport_kernel(
    const float* __restrict__ S_hat, const TR* __restrict__ r_s,
    const int* __restrict__ ptr_s, const int* __restrict__ ptr_t,
    float* __restrict__ S, TR* __restrict__ r_t, int Ns, int Nt, int R,
    int rows_t, TR* __restrict__ r_s_copy, int rows_s) {
  __shared__ float sS[kMaxN * kPitch];
  __shared__ float sR[kMaxN * kPitch];
  const int b = xcd_remap(blockIdx.x, gridDim.x);
  if (blockIdx.x == gridDim.x - 1) zero_tail(r_t, ptr_t[gridDim.x], rows_t, R);
  if (r_s_copy) {
    // r_s rows past the last pair (static-batch padding), spread over the
    // whole grid: one element per thread instead of a serial loop in one
    // block (which put ~60 us on the kernel's critical path).
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t e = (size_t)ptr_s[gridDim.x] * R +
                    (size_t)blockIdx.x * blockDim.x + threadIdx.x;
         e < (size_t)rows_s * R; e += stride)
      r_s_copy[e] = r_s[e];
  }
  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  const int ns = ptr_s[b + 1] - ptr_s[b], nt = ptr_t[b + 1] - ptr_t[b];
  const float* Sh = S_hat + (size_t)b * Ns * Nt;
  float* Sb = S + (size_t)b * Ns * Nt;

  for (int i = wave; i < Ns; i += kWaves) {
    const bool valid = i < ns && lane < nt;
    const float v = valid ? Sh[i * Nt + lane] : -INFINITY;
    const float m = wave_max(v);
    const float e = valid ? __expf(v - m) : 0.f;
    const float s = wave_sum(e);
    const float p = valid ? e / s : 0.f;
    if (lane < Nt) {
      sS[i * kPitch + lane] = p;
      Sb[i * Nt + lane] = p;
    }
  }

  const TR* rs = r_s + (size_t)ptr_s[b] * R;
  TR* rt = r_t + (size_t)ptr_t[b] * R;
  for (int c0 = 0; c0 < R; c0 += kCh) {
    const int c = c0 + lane;
    __syncthreads();
    for (int i = wave; i < ns; i += kWaves) {
      const TR v = c < R ? rs[(size_t)i * R + c] : Cvt<TR>::from_f(0.f);
      sR[i * kPitch + lane] = Cvt<TR>::to_f(v);
      // Joint output [r_s; r_t]: psi_2's input without a concatenation.
      if (r_s_copy && c < R) r_s_copy[(size_t)(ptr_s[b] + i) * R + c] = v;
    }
    __syncthreads();
    for (int j = wave; j < nt; j += kWaves) {
      float acc = 0.f;
      for (int i = 0; i < ns; ++i)
        acc = fmaf(sS[i * kPitch + j], sR[i * kPitch + lane], acc);
      if (c < R) rt[(size_t)j * R + c] = Cvt<TR>::from_f(acc);
    }
  }
}

// dS_hat = softmax_bwd(S, dS),  dS[i][j] = sum_c r_s[i][c] * g[j][c].
template <typename TR>
__global__ __launch_bounds__(256) void softmax_transport_bwd_kernel(
    const float* __restrict__ S, const TR* __restrict__ r_s,
    const TR* __restrict__ g, const int* __restrict__ ptr_s,
    const int* __restrict__ ptr_t, float* __restrict__ dS_hat, int Ns,
    int Nt, int R) {
  __shared__ float sR[kMaxN * kPitch];
  __shared__ float sG[kMaxN * kPitch];
  const int b = xcd_remap(blockIdx.x, gridDim.x);
  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  const int ns = ptr_s[b + 1] - ptr_s[b], nt = ptr_t[b + 1] - ptr_t[b];
  const TR* rs = r_s + (size_t)ptr_s[b] * R;
  const TR* gb = g + (size_t)ptr_t[b] * R;

  float acc[kRowsPerWave];
#pragma unroll
  for (int q = 0; q < kRowsPerWave; ++q) acc[q] = 0.f;

  for (int c0 = 0; c0 < R; c0 += kCh) {
    const int c = c0 + lane;
    __syncthreads();
    for (int i = wave; i < ns; i += kWaves)
      sR[i * kPitch + lane] = c < R ? Cvt<TR>::to_f(rs[(size_t)i * R + c]) : 0.f;
    for (int j = wave; j < nt; j += kWaves)
      sG[j * kPitch + lane] = c < R ? Cvt<TR>::to_f(gb[(size_t)j * R + c]) : 0.f;
    __syncthreads();
    const int cmax = min(kCh, R - c0);
    if (lane < nt) {
#pragma unroll
      for (int q = 0; q < kRowsPerWave; ++q) {
        const int i = wave + q * kWaves;
        if (i < ns) {
          float a = acc[q];
          for (int cc = 0; cc < cmax; ++cc)
            a = fmaf(sR[i * kPitch + cc], sG[lane * kPitch + cc], a);
          acc[q] = a;
        }
      }
    }
  }
  const float* Sb = S + (size_t)b * Ns * Nt;
  float* out = dS_hat + (size_t)b * Ns * Nt;
#pragma unroll
  for (int q = 0; q < kRowsPerWave; ++q) {
    const int i = wave + q * kWaves;
    if (i < Ns) {
      const float s = lane < Nt ? Sb[i * Nt + lane] : 0.f;
      const float dot = wave_sum(s * acc[q]);
      if (lane < Nt) out[i * Nt + lane] = s * (acc[q] - dot);
    }
  }
}

// ---------------------------------------------------------------------------
// Consensus update: out = S_hat + mask * (sum_c relu(P_ic - Q_jc) w2_c + b2)
// ---------------------------------------------------------------------------
template <typename TPQ>
__global__ __launch_bounds__(256) void consensus_fwd_kernel(
    const float* __restrict__ S_hat, const TPQ* __restrict__ P,
    const TPQ* __restrict__ Q, const float* __restrict__ b1,
    const float* __restrict__ w2, const float* __restrict__ b2,
    const int* __restrict__ ptr_s, const int* __restrict__ ptr_t,
    float* __restrict__ out, int Ns, int Nt, int R) {
  __shared__ float sP[kMaxN * kPitch];
  __shared__ float sQ[kMaxN * kPitch];
  __shared__ float sW[kCh];
  const int b = xcd_remap(blockIdx.x, gridDim.x);
  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  const int ns = ptr_s[b + 1] - ptr_s[b], nt = ptr_t[b + 1] - ptr_t[b];
  const TPQ* Pb = P + (size_t)ptr_s[b] * R;
  const TPQ* Qb = Q + (size_t)ptr_t[b] * R;

  float acc[kRowsPerWave];
#pragma unroll
  for (int q = 0; q < kRowsPerWave; ++q) acc[q] = 0.f;

  for (int c0 = 0; c0 < R; c0 += kCh) {
    const int c = c0 + lane;
    __syncthreads();
    const float bias1 = c < R ? b1[c] : 0.f;
    for (int i = wave; i < ns; i += kWaves)
      sP[i * kPitch + lane] =
          c < R ? Cvt<TPQ>::to_f(Pb[(size_t)i * R + c]) + bias1 : 0.f;
    for (int j = wave; j < nt; j += kWaves)
      sQ[j * kPitch + lane] =
          c < R ? Cvt<TPQ>::to_f(Qb[(size_t)j * R + c]) : 0.f;
    if (wave == 0) sW[lane] = c < R ? w2[c] : 0.f;
    __syncthreads();
    const int cmax = min(kCh, R - c0);
    if (lane < nt) {
#pragma unroll
      for (int q = 0; q < kRowsPerWave; ++q) {
        const int i = wave + q * kWaves;
        if (i < ns) {
          float a = acc[q];
          for (int cc = 0; cc < cmax; ++cc) {
            const float z = sP[i * kPitch + cc] - sQ[lane * kPitch + cc];
            a = fmaf(fmaxf(z, 0.f), sW[cc], a);
          }
          acc[q] = a;
        }
      }
    }
  }
  const float bias = b2[0];
  const float* Sb = S_hat + (size_t)b * Ns * Nt;
  float* ob = out + (size_t)b * Ns * Nt;
#pragma unroll
  for (int q = 0; q < kRowsPerWave; ++q) {
    const int i = wave + q * kWaves;
    if (i < Ns && lane < Nt) {
      const bool valid = i < ns && lane < nt;
      ob[i * Nt + lane] = Sb[i * Nt + lane] + (valid ? acc[q] + bias : 0.f);
    }
  }
}

template <typename TPQ>
__global__ __launch_bounds__(256) void consensus_bwd_kernel(
    const float* __restrict__ G, const TPQ* __restrict__ P,
    const TPQ* __restrict__ Q, const float* __restrict__ b1,
    const float* __restrict__ w2, const int* __restrict__ ptr_s,
    const int* __restrict__ ptr_t, TPQ* __restrict__ dP,
    TPQ* __restrict__ dQ, float* __restrict__ dw2_part,
    float* __restrict__ db2_part, int Ns, int Nt, int R, int rows_s,
    int rows_t) {
  __shared__ float sG[kMaxN * kPitch];
  __shared__ float sP[kMaxN * kPitch];
  __shared__ float sQ[kMaxN * kPitch];
  __shared__ float sRed[kWaves * kCh];
  const int b = xcd_remap(blockIdx.x, gridDim.x);
  if (blockIdx.x == gridDim.x - 1) {
    zero_tail(dP, ptr_s[gridDim.x], rows_s, R);
    zero_tail(dQ, ptr_t[gridDim.x], rows_t, R);
  }
  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  const int ns = ptr_s[b + 1] - ptr_s[b], nt = ptr_t[b + 1] - ptr_t[b];
  const float* Gb = G + (size_t)b * Ns * Nt;
  const TPQ* Pb = P + (size_t)ptr_s[b] * R;
  const TPQ* Qb = Q + (size_t)ptr_t[b] * R;
  TPQ* dPb = dP + (size_t)ptr_s[b] * R;
  TPQ* dQb = dQ + (size_t)ptr_t[b] * R;

  // Masked upstream gradient tile + db2 partial.
  float gsum = 0.f;
  for (int i = wave; i < ns; i += kWaves) {
    const float v = lane < nt ? Gb[i * Nt + lane] : 0.f;
    sG[i * kPitch + lane] = v;
    gsum += v;
  }
  gsum = wave_sum(gsum);
  if (lane == 0) sRed[wave] = gsum;
  __syncthreads();
  if (threadIdx.x == 0)
    db2_part[b] = sRed[0] + sRed[1] + sRed[2] + sRed[3];

  for (int c0 = 0; c0 < R; c0 += kCh) {
    const int c = c0 + lane;
    const bool cv = c < R;
    __syncthreads();
    const float bias1 = cv ? b1[c] : 0.f;
    for (int i = wave; i < ns; i += kWaves)
      sP[i * kPitch + lane] =
          cv ? Cvt<TPQ>::to_f(Pb[(size_t)i * R + c]) + bias1 : 0.f;
    for (int j = wave; j < nt; j += kWaves)
      sQ[j * kPitch + lane] = cv ? Cvt<TPQ>::to_f(Qb[(size_t)j * R + c]) : 0.f;
    __syncthreads();
    const float w = cv ? w2[c] : 0.f;

    // dP[i][c] and dw2 partial: rows owned by this wave, lane = channel.
    // Branch-free, 4 independent partial sums so the LDS reads of 4 j's are
    // in flight together (the loop is LDS-latency bound otherwise).
    float dw = 0.f;
    for (int i = wave; i < ns; i += kWaves) {
      const float p = sP[i * kPitch + lane];
      float dp[4] = {0.f, 0.f, 0.f, 0.f}, dwq[4] = {0.f, 0.f, 0.f, 0.f};
      int j = 0;
      for (; j + 4 <= nt; j += 4) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const float z = fmaxf(p - sQ[(j + u) * kPitch + lane], 0.f);
          const float gij = sG[i * kPitch + j + u];
          dp[u] += z > 0.f ? gij : 0.f;
          dwq[u] = fmaf(gij, z, dwq[u]);
        }
      }
      for (; j < nt; ++j) {
        const float z = fmaxf(p - sQ[j * kPitch + lane], 0.f);
        const float gij = sG[i * kPitch + j];
        dp[0] += z > 0.f ? gij : 0.f;
        dwq[0] = fmaf(gij, z, dwq[0]);
      }
      dw += (dwq[0] + dwq[1]) + (dwq[2] + dwq[3]);
      if (cv)
        dPb[(size_t)i * R + c] =
            Cvt<TPQ>::from_f(((dp[0] + dp[1]) + (dp[2] + dp[3])) * w);
    }
    // dQ[j][c] = -w * sum_i G[i][j] [P_ic > Q_jc]
    for (int j = wave; j < nt; j += kWaves) {
      const float qv = sQ[j * kPitch + lane];
      float dq[4] = {0.f, 0.f, 0.f, 0.f};
      int i = 0;
      for (; i + 4 <= ns; i += 4) {
#pragma unroll
        for (int u = 0; u < 4; ++u)
          dq[u] += sP[(i + u) * kPitch + lane] > qv
                       ? sG[(i + u) * kPitch + j] : 0.f;
      }
      for (; i < ns; ++i)
        dq[0] += sP[i * kPitch + lane] > qv ? sG[i * kPitch + j] : 0.f;
      if (cv)
        dQb[(size_t)j * R + c] =
            Cvt<TPQ>::from_f(-((dq[0] + dq[1]) + (dq[2] + dq[3])) * w);
    }
    // Reduce dw over the 4 waves.
    sRed[wave * kCh + lane] = dw;
    __syncthreads();
    if (wave == 0 && cv)
      dw2_part[(size_t)b * R + c] = sRed[lane] + sRed[kCh + lane] +
                                    sRed[2 * kCh + lane] +
                                    sRed[3 * kCh + lane];
  }
}

// ---------------------------------------------------------------------------
// Host wrappers
// ---------------------------------------------------------------------------
static void check_pair_tensor(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat &&
                  t.is_contiguous() && t.dim() == 3,
              name, " must be a contiguous fp32 [B, N, *] GPU tensor");
}

static void check_counts(const at::Tensor& n_s, const at::Tensor& n_t,
                         int64_t B) {
  TORCH_CHECK(n_s.scalar_type() == at::kInt && n_t.scalar_type() == at::kInt &&
                  n_s.numel() == B && n_t.numel() == B,
              "node counts must be int32 [B]");
}

static void check_ptr(const at::Tensor& ptr_s, const at::Tensor& ptr_t,
                      int64_t B) {
  TORCH_CHECK(ptr_s.scalar_type() == at::kInt && ptr_t.scalar_type() == at::kInt &&
                  ptr_s.numel() == B + 1 && ptr_t.numel() == B + 1 &&
                  ptr_s.is_cuda() && ptr_t.is_cuda(),
              "row offsets must be int32 [B + 1] GPU tensors");
}

static void check_packed(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.dim() == 2 && t.is_contiguous(), name,
              " must be a contiguous [rows, R] GPU tensor");
}

at::Tensor dense_masked_softmax(const at::Tensor& S_hat, const at::Tensor& n_s,
                                const at::Tensor& n_t) {
  check_pair_tensor(S_hat, "S_hat");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(S_hat.device());
  const int B = S_hat.size(0), Ns = S_hat.size(1), Nt = S_hat.size(2);
  check_counts(n_s, n_t, B);
  at::Tensor S = at::empty_like(S_hat);
  const int rows = B * Ns;
  if (rows == 0 || Nt == 0) return S.zero_();
  hipLaunchKernelGGL(masked_softmax_kernel, dim3((rows + 3) / 4), dim3(256), 0,
                     stream(), S_hat.data_ptr<float>(), n_s.data_ptr<int>(),
                     n_t.data_ptr<int>(), S.data_ptr<float>(), B, Ns, Nt);
  DGMC_CHECK_LAUNCH();
  return S;
}

at::Tensor dense_masked_softmax_bwd(const at::Tensor& S, const at::Tensor& G,
                                    const at::Tensor& n_s,
                                    const at::Tensor& n_t) {
  check_pair_tensor(S, "S");
  check_pair_tensor(G, "grad");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(S.device());
  const int B = S.size(0), Ns = S.size(1), Nt = S.size(2);
  check_counts(n_s, n_t, B);
  at::Tensor out = at::empty_like(S);
  const int rows = B * Ns;
  if (rows == 0 || Nt == 0) return out.zero_();
  hipLaunchKernelGGL(masked_softmax_bwd_kernel, dim3((rows + 3) / 4),
                     dim3(256), 0, stream(), S.data_ptr<float>(),
                     G.data_ptr<float>(), out.data_ptr<float>(), rows, Nt);
  DGMC_CHECK_LAUNCH();
  return out;
}

// r_s: packed [sum N_s, R]; returns (S [B, Ns, Nt], r_t packed [rows_t, R]).
std::tuple<at::Tensor, at::Tensor> dense_softmax_transport(
    const at::Tensor& S_hat, const at::Tensor& r_s, const at::Tensor& ptr_s,
    const at::Tensor& ptr_t, int64_t rows_t, bool joint_out) {
  check_pair_tensor(S_hat, "S_hat");
  check_packed(r_s, "r_s");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(S_hat.device());
  const int B = S_hat.size(0), Ns = S_hat.size(1), Nt = S_hat.size(2);
  const int R = r_s.size(1);
  TORCH_CHECK(Ns <= kMaxN && Nt <= kMaxN, "pair tile too large");
  check_ptr(ptr_s, ptr_t, B);
  at::Tensor S = at::empty_like(S_hat);
  at::Tensor r_t, joint;
  const int64_t rows_s = r_s.size(0);
  if (joint_out) {
    // Joint [r_s; r_t] (psi_2's fused input): r_s rows are copied by the
    // same kernel, so no concatenation kernel is needed afterwards.
    joint = at::empty({rows_s + rows_t, R}, r_s.options());
    r_t = joint.narrow(0, rows_s, rows_t);
  } else {
    r_t = at::empty({rows_t, R}, r_s.options());
  }
  if (B == 0) {
    if (joint_out) joint.narrow(0, 0, rows_s).copy_(r_s);
    return {S, joint_out ? joint : r_t};
  }
  DGMC_DISPATCH_FLOAT(r_s.scalar_type(), T, [&] {
    hipLaunchKernelGGL(softmax_transport_kernel<T>, dim3(B), dim3(256), 0,
                       stream(), S_hat.data_ptr<float>(),
                       reinterpret_cast<const T*>(r_s.data_ptr()),
                       ptr_s.data_ptr<int>(), ptr_t.data_ptr<int>(),
                       S.data_ptr<float>(), reinterpret_cast<T*>(r_t.data_ptr()),
                       Ns, Nt, R, (int)rows_t,
                       joint_out ? reinterpret_cast<T*>(joint.data_ptr())
                                 : nullptr,
                       (int)rows_s);
  });
  DGMC_CHECK_LAUNCH();
  return {S, joint_out ? joint : r_t};
}

at::Tensor dense_softmax_transport_bwd(const at::Tensor& S,
                                       const at::Tensor& r_s,
                                       const at::Tensor& g,
                                       const at::Tensor& ptr_s,
                                       const at::Tensor& ptr_t) {
  check_pair_tensor(S, "S");
  check_packed(r_s, "r_s");
  check_packed(g, "grad r_t");
  TORCH_CHECK(r_s.scalar_type() == g.scalar_type(), "r_s/grad dtype");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(S.device());
  const int B = S.size(0), Ns = S.size(1), Nt = S.size(2);
  const int R = r_s.size(1);
  TORCH_CHECK(Ns <= kMaxN && Nt <= kMaxN, "pair tile too large");
  TORCH_CHECK(g.size(1) == R, "grad shape");
  check_ptr(ptr_s, ptr_t, B);
  at::Tensor out = at::empty_like(S);
  if (B == 0) return out;
  DGMC_DISPATCH_FLOAT(r_s.scalar_type(), T, [&] {
    hipLaunchKernelGGL(softmax_transport_bwd_kernel<T>, dim3(B), dim3(256), 0,
                       stream(), S.data_ptr<float>(),
                       reinterpret_cast<const T*>(r_s.data_ptr()),
                       reinterpret_cast<const T*>(g.data_ptr()),
                       ptr_s.data_ptr<int>(), ptr_t.data_ptr<int>(),
                       out.data_ptr<float>(), Ns, Nt, R);
  });
  DGMC_CHECK_LAUNCH();
  return out;
}

// P: packed [sum N_s, R] (without bias), Q: packed [sum N_t, R]
at::Tensor dense_consensus(const at::Tensor& S_hat, const at::Tensor& P,
                           const at::Tensor& Q, const at::Tensor& b1,
                           const at::Tensor& w2, const at::Tensor& b2,
                           const at::Tensor& ptr_s, const at::Tensor& ptr_t) {
  check_pair_tensor(S_hat, "S_hat");
  check_packed(P, "P");
  check_packed(Q, "Q");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(S_hat.device());
  const int B = S_hat.size(0), Ns = S_hat.size(1), Nt = S_hat.size(2);
  const int R = P.size(1);
  TORCH_CHECK(Ns <= kMaxN && Nt <= kMaxN, "pair tile too large");
  TORCH_CHECK(Q.size(1) == R && Q.scalar_type() == P.scalar_type(), "P/Q");
  TORCH_CHECK(b1.numel() == R && w2.numel() == R && b2.numel() == 1 &&
                  b1.scalar_type() == at::kFloat &&
                  w2.scalar_type() == at::kFloat &&
                  b2.scalar_type() == at::kFloat,
              "b1/w2/b2 must be fp32");
  check_ptr(ptr_s, ptr_t, B);
  at::Tensor out = at::empty_like(S_hat);
  if (B == 0) return out;
  DGMC_DISPATCH_FLOAT(P.scalar_type(), T, [&] {
    hipLaunchKernelGGL(consensus_fwd_kernel<T>, dim3(B), dim3(256), 0,
                       stream(), S_hat.data_ptr<float>(),
                       reinterpret_cast<const T*>(P.data_ptr()),
                       reinterpret_cast<const T*>(Q.data_ptr()),
                       b1.data_ptr<float>(), w2.data_ptr<float>(),
                       b2.data_ptr<float>(), ptr_s.data_ptr<int>(),
                       ptr_t.data_ptr<int>(), out.data_ptr<float>(), Ns, Nt,
                       R);
  });
  DGMC_CHECK_LAUNCH();
  return out;
}

std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> dense_consensus_bwd(
    const at::Tensor& G, const at::Tensor& P, const at::Tensor& Q,
    const at::Tensor& b1, const at::Tensor& w2, const at::Tensor& ptr_s,
    const at::Tensor& ptr_t, const c10::optional<at::Tensor>& dpq_out) {
  check_pair_tensor(G, "grad");
  check_packed(P, "P");
  check_packed(Q, "Q");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(G.device());
  const int B = G.size(0), Ns = G.size(1), Nt = G.size(2);
  const int R = P.size(1);
  TORCH_CHECK(Ns <= kMaxN && Nt <= kMaxN, "pair tile too large");
  check_ptr(ptr_s, ptr_t, B);
  at::Tensor dP, dQ;
  if (dpq_out.has_value() && dpq_out->defined()) {
    // Joint [P; Q] gradient buffer: no slice-backward (fill + 2 copies).
    const at::Tensor& d = *dpq_out;
    TORCH_CHECK(d.is_contiguous() && d.scalar_type() == P.scalar_type() &&
                    d.size(0) == P.size(0) + Q.size(0) && d.size(1) == R,
                "dense_consensus_bwd: dpq_out must be [rows_s + rows_t, R]");
    dP = d.narrow(0, 0, P.size(0));
    dQ = d.narrow(0, P.size(0), Q.size(0));
  } else {
    dP = at::empty_like(P);
    dQ = at::empty_like(Q);
  }
  at::Tensor dw2 = at::empty({B, R}, G.options());
  at::Tensor db2 = at::empty({B}, G.options());
  if (B == 0) return {dP, dQ, dw2.zero_(), db2.zero_()};
  DGMC_DISPATCH_FLOAT(P.scalar_type(), T, [&] {
    hipLaunchKernelGGL(consensus_bwd_kernel<T>, dim3(B), dim3(256), 0,
                       stream(), G.data_ptr<float>(),
                       reinterpret_cast<const T*>(P.data_ptr()),
                       reinterpret_cast<const T*>(Q.data_ptr()),
                       b1.data_ptr<float>(), w2.data_ptr<float>(),
                       ptr_s.data_ptr<int>(), ptr_t.data_ptr<int>(),
                       reinterpret_cast<T*>(dP.data_ptr()),
                       reinterpret_cast<T*>(dQ.data_ptr()),
                       dw2.data_ptr<float>(), db2.data_ptr<float>(), Ns, Nt, R,
                       (int)P.size(0), (int)Q.size(0));
  });
  DGMC_CHECK_LAUNCH();
  return {dP, dQ, dw2, db2};
}

}  // namespace dgmc
