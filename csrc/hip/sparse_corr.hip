// Sparse (top-k candidate) correspondence kernels, reference dgmc.py:184-244.
//
// The candidate structure S_idx [B, N_s, k] is a CSR matrix over flattened
// source rows with global target columns (b * N_t + idx); its transpose (CSC)
// is built once per forward.  With that, every op of the sparse consensus
// loop is deterministic and atomic-free:
//
//   sddmm                  val[p] = <A[row p], B[col p]>      (gathered dot,
//                          dgmc.py:197-201, and d/dS of the transport)
//   spmm_csr (spmm.hip)    transport r_t = S^T r_s (dgmc.py:209-212) and the
//                          backward of the gathered dot
//   sparse_consensus_fwd   S_hat[p] += relu(P_row + b1 - Q_col) . w2 + b2
//                          (factored MLP(o_s[i] - o_t[idx]), dgmc.py:219-223)
//   sparse_consensus_bwd_rows / _cols   dP, dw2 partials / dQ
//
// Mapping: one wave64 per row (or column); lanes own channels, each lane
// keeps its slice of the row operand in registers, candidates are walked
// sequentially with one coalesced load of the partner row per candidate and
// a wave reduction per dot.  k is small (10-20), rows are many (15k+).
#include "common.h"

namespace dgmc {

constexpr int kSpWaves = 4;
constexpr int kMaxChanPerLane = 8;   // C <= 512

__global__ __launch_bounds__(256) void sddmm_kernel(
    const int* __restrict__ rowptr, const int* __restrict__ col,
    const float* __restrict__ A, const float* __restrict__ Bm,
    float* __restrict__ val, int rows, int C) {
  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  const int r = xcd_remap(blockIdx.x, gridDim.x) * kSpWaves + wave;
  if (r >= rows) return;
  float a[kMaxChanPerLane];
#pragma unroll
  for (int u = 0; u < kMaxChanPerLane; ++u) {
    const int c = lane + u * kWave;
    a[u] = c < C ? A[(size_t)r * C + c] : 0.f;
  }
  const int p0 = rowptr[r], p1 = rowptr[r + 1];
  for (int p = p0; p < p1; ++p) {
    const float* b = Bm + (size_t)col[p] * C;
    float s = 0.f;
#pragma unroll
    for (int u = 0; u < kMaxChanPerLane; ++u) {
      const int c = lane + u * kWave;
      if (c < C) s = fmaf(a[u], b[c], s);
    }
    s = wave_sum(s);
    if (lane == 0) val[p] = s;
  }
}

__global__ __launch_bounds__(256) void sparse_consensus_fwd_kernel(
    const int* __restrict__ rowptr, const int* __restrict__ col,
    const float* __restrict__ S_hat, const float* __restrict__ P,
    const float* __restrict__ Q, const float* __restrict__ b1,
    const float* __restrict__ w2, const float* __restrict__ b2,
    float* __restrict__ out, int rows, int R) {
  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  const int r = xcd_remap(blockIdx.x, gridDim.x) * kSpWaves + wave;
  if (r >= rows) return;
  float pv[kMaxChanPerLane], wv[kMaxChanPerLane];
#pragma unroll
  for (int u = 0; u < kMaxChanPerLane; ++u) {
    const int c = lane + u * kWave;
    pv[u] = c < R ? P[(size_t)r * R + c] + b1[c] : 0.f;
    wv[u] = c < R ? w2[c] : 0.f;
  }
  const float bias = b2[0];
  const int p0 = rowptr[r], p1 = rowptr[r + 1];
  for (int p = p0; p < p1; ++p) {
    const float* q = Q + (size_t)col[p] * R;
    float s = 0.f;
#pragma unroll
    for (int u = 0; u < kMaxChanPerLane; ++u) {
      const int c = lane + u * kWave;
      if (c < R) s = fmaf(fmaxf(pv[u] - q[c], 0.f), wv[u], s);
    }
    s = wave_sum(s);
    if (lane == 0) out[p] = S_hat[p] + s + bias;
  }
}

// dP[r] = w2 * sum_p g_p [z_p > 0];  dw2 partial per block.
__global__ __launch_bounds__(256) void sparse_consensus_bwd_rows_kernel(
    const int* __restrict__ rowptr, const int* __restrict__ col,
    const float* __restrict__ G, const float* __restrict__ P,
    const float* __restrict__ Q, const float* __restrict__ b1,
    const float* __restrict__ w2, float* __restrict__ dP,
    float* __restrict__ dw2_part, int rows, int R) {
  __shared__ float red[kSpWaves][kMaxChanPerLane * kWave];
  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  const int blk = blockIdx.x;
  float dw[kMaxChanPerLane];
#pragma unroll
  for (int u = 0; u < kMaxChanPerLane; ++u) dw[u] = 0.f;
  // grid-stride over rows so the dw2 partial count stays = gridDim.x
  for (int r = blk * kSpWaves + wave; r < rows;
       r += gridDim.x * kSpWaves) {
    float pv[kMaxChanPerLane], dp[kMaxChanPerLane];
#pragma unroll
    for (int u = 0; u < kMaxChanPerLane; ++u) {
      const int c = lane + u * kWave;
      pv[u] = c < R ? P[(size_t)r * R + c] + b1[c] : 0.f;
      dp[u] = 0.f;
    }
    const int p0 = rowptr[r], p1 = rowptr[r + 1];
    for (int p = p0; p < p1; ++p) {
      const float g = G[p];
      const float* q = Q + (size_t)col[p] * R;
#pragma unroll
      for (int u = 0; u < kMaxChanPerLane; ++u) {
        const int c = lane + u * kWave;
        if (c < R) {
          const float z = pv[u] - q[c];
          if (z > 0.f) {
            dp[u] += g;
            dw[u] = fmaf(g, z, dw[u]);
          }
        }
      }
    }
#pragma unroll
    for (int u = 0; u < kMaxChanPerLane; ++u) {
      const int c = lane + u * kWave;
      if (c < R) dP[(size_t)r * R + c] = dp[u] * w2[c];
    }
  }
#pragma unroll
  for (int u = 0; u < kMaxChanPerLane; ++u) red[wave][u * kWave + lane] = dw[u];
  __syncthreads();
  for (int c = threadIdx.x; c < R; c += blockDim.x) {
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < kSpWaves; ++w) s += red[w][c];
    dw2_part[(size_t)blk * R + c] = s;
  }
}

// dQ[j] = -w2 * sum_{p in col j} g_p [P_row(p) + b1 - Q_j > 0]  (CSC walk)
__global__ __launch_bounds__(256) void sparse_consensus_bwd_cols_kernel(
    const int* __restrict__ colptr, const int* __restrict__ row_of,
    const int64_t* __restrict__ perm, const float* __restrict__ G,
    const float* __restrict__ P, const float* __restrict__ Q,
    const float* __restrict__ b1, const float* __restrict__ w2,
    float* __restrict__ dQ, int cols, int R) {
  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  const int j = xcd_remap(blockIdx.x, gridDim.x) * kSpWaves + wave;
  if (j >= cols) return;
  float qv[kMaxChanPerLane], dq[kMaxChanPerLane], bb[kMaxChanPerLane];
#pragma unroll
  for (int u = 0; u < kMaxChanPerLane; ++u) {
    const int c = lane + u * kWave;
    qv[u] = c < R ? Q[(size_t)j * R + c] : 0.f;
    bb[u] = c < R ? b1[c] : 0.f;
    dq[u] = 0.f;
  }
  const int p0 = colptr[j], p1 = colptr[j + 1];
  for (int e = p0; e < p1; ++e) {
    const float g = G[perm[e]];
    const float* pr = P + (size_t)row_of[e] * R;
#pragma unroll
    for (int u = 0; u < kMaxChanPerLane; ++u) {
      const int c = lane + u * kWave;
      if (c < R && pr[c] + bb[u] - qv[u] > 0.f) dq[u] += g;
    }
  }
#pragma unroll
  for (int u = 0; u < kMaxChanPerLane; ++u) {
    const int c = lane + u * kWave;
    if (c < R) dQ[(size_t)j * R + c] = -dq[u] * w2[c];
  }
}

// ---------------------------------------------------------------------------
static void check_f32_2d(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.dim() == 2 && t.scalar_type() == at::kFloat &&
                  t.is_contiguous(),
              name, " must be a contiguous fp32 [rows, C] GPU tensor");
  TORCH_CHECK(t.size(1) <= kMaxChanPerLane * kWave, name, ": C <= 512");
}

static int sp_blocks(int64_t rows) {
  return (int)((rows + kSpWaves - 1) / kSpWaves);
}

at::Tensor sddmm(const at::Tensor& rowptr, const at::Tensor& col,
                 const at::Tensor& A, const at::Tensor& B) {
  check_f32_2d(A, "A");
  check_f32_2d(B, "B");
  TORCH_CHECK(A.size(1) == B.size(1), "sddmm: channel mismatch");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(A.device());
  const int64_t rows = rowptr.numel() - 1;
  TORCH_CHECK(rows == A.size(0), "sddmm: rowptr / A rows mismatch");
  at::Tensor val = at::empty({col.numel()}, A.options());
  if (rows == 0 || col.numel() == 0) return val.zero_();
  hipLaunchKernelGGL(sddmm_kernel, dim3(sp_blocks(rows)), dim3(256), 0,
                     stream(), rowptr.data_ptr<int>(), col.data_ptr<int>(),
                     A.data_ptr<float>(), B.data_ptr<float>(),
                     val.data_ptr<float>(), (int)rows, (int)A.size(1));
  DGMC_CHECK_LAUNCH();
  return val;
}

at::Tensor sparse_consensus_fwd(const at::Tensor& rowptr, const at::Tensor& col,
                                const at::Tensor& S_hat, const at::Tensor& P,
                                const at::Tensor& Q, const at::Tensor& b1,
                                const at::Tensor& w2, const at::Tensor& b2) {
  check_f32_2d(P, "P");
  check_f32_2d(Q, "Q");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(P.device());
  const int64_t rows = rowptr.numel() - 1;
  const int R = P.size(1);
  TORCH_CHECK(rows == P.size(0) && Q.size(1) == R && b1.numel() == R &&
                  w2.numel() == R && b2.numel() == 1,
              "sparse_consensus_fwd: shapes");
  TORCH_CHECK(S_hat.numel() == col.numel() && S_hat.is_contiguous(),
              "sparse_consensus_fwd: S_hat");
  at::Tensor out = at::empty_like(S_hat);
  if (rows == 0) return out;
  hipLaunchKernelGGL(sparse_consensus_fwd_kernel, dim3(sp_blocks(rows)),
                     dim3(256), 0, stream(), rowptr.data_ptr<int>(),
                     col.data_ptr<int>(), S_hat.data_ptr<float>(),
                     P.data_ptr<float>(), Q.data_ptr<float>(),
                     b1.data_ptr<float>(), w2.data_ptr<float>(),
                     b2.data_ptr<float>(), out.data_ptr<float>(), (int)rows,
                     R);
  DGMC_CHECK_LAUNCH();
  return out;
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> sparse_consensus_bwd(
    const at::Tensor& rowptr, const at::Tensor& col, const at::Tensor& colptr,
    const at::Tensor& row_of, const at::Tensor& perm, const at::Tensor& G,
    const at::Tensor& P, const at::Tensor& Q, const at::Tensor& b1,
    const at::Tensor& w2) {
  check_f32_2d(P, "P");
  check_f32_2d(Q, "Q");
  TORCH_CHECK(perm.scalar_type() == at::kLong, "perm must be int64");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(P.device());
  const int64_t rows = rowptr.numel() - 1, cols = colptr.numel() - 1;
  const int R = P.size(1);
  TORCH_CHECK(rows == P.size(0) && cols == Q.size(0), "shape mismatch");
  at::Tensor dP = at::empty_like(P), dQ = at::empty_like(Q);
  const int nb = std::max(1, std::min(sp_blocks(rows), 1024));
  at::Tensor dw2 = at::empty({nb, R}, P.options());
  if (rows > 0) {
    hipLaunchKernelGGL(sparse_consensus_bwd_rows_kernel, dim3(nb), dim3(256),
                       0, stream(), rowptr.data_ptr<int>(),
                       col.data_ptr<int>(), G.data_ptr<float>(),
                       P.data_ptr<float>(), Q.data_ptr<float>(),
                       b1.data_ptr<float>(), w2.data_ptr<float>(),
                       dP.data_ptr<float>(), dw2.data_ptr<float>(), (int)rows,
                       R);
    DGMC_CHECK_LAUNCH();
  } else {
    dw2.zero_();
  }
  if (cols > 0) {
    hipLaunchKernelGGL(sparse_consensus_bwd_cols_kernel, dim3(sp_blocks(cols)),
                       dim3(256), 0, stream(), colptr.data_ptr<int>(),
                       row_of.data_ptr<int>(), perm.data_ptr<int64_t>(),
                       G.data_ptr<float>(), P.data_ptr<float>(),
                       Q.data_ptr<float>(), b1.data_ptr<float>(),
                       w2.data_ptr<float>(), dQ.data_ptr<float>(), (int)cols,
                       R);
    DGMC_CHECK_LAUNCH();
  }
  return {dP, dQ, dw2};
}

}  // namespace dgmc
