// Objective-side fused kernels of the dense DGMC training step.
//
// * masked_softmax_packed      S_0 / S_L = to_sparse(masked_softmax(S_hat))
//                              (reference dgmc.py:15-19,165,181): the dense
//                              [B, Ns, Nt] scores go straight to the packed
//                              [rows, Nt] output through the layout's dense
//                              row index (no pack gather, and its backward is
//                              a plain row scatter - no index_add);
// * nll_fwd / nll_bwd          DGMC.loss (dgmc.py:246-267) with the optional
//                              ground-truth mask of padded static batches,
//                              plus the Hits@1 count of DGMC.acc (dgmc.py:
//                              269-288) in the same pass; deterministic
//                              block reduction, no host sync;
// * nonfinite_partials/_final  device-side "any non-finite gradient" flag
//                              read by the fused Adam (skipped steps).
// The reference path for all of these is ~80 small ATen launches per step
// (advanced-indexing backward sorts its indices).
#include "common.h"

namespace dgmc {

constexpr int kLossThreads = 1024;

// ---------------------------------------------------------------------------
// Packed masked softmax.  One wave per packed row r: dense row
// idx = dense_index[r] (>= B * Ns: padding row -> zeros).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void masked_softmax_packed_kernel(
    const float* __restrict__ S_hat, const int64_t* __restrict__ dense_index,
    const int* __restrict__ n_s, const int* __restrict__ n_t,
    float* __restrict__ out, int rows, int B, int Ns, int Nt) {
  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  const int r = blockIdx.x * 4 + wave;
  if (r >= rows) return;
  const int64_t idx = dense_index[r];
  float* dst = out + (size_t)r * Nt;
  int nt = 0;
  const float* src = S_hat;
  if (idx >= 0 && idx < (int64_t)B * Ns) {
    const int b = (int)(idx / Ns), i = (int)(idx - (int64_t)b * Ns);
    nt = i < n_s[b] ? n_t[b] : 0;
    src = S_hat + (size_t)idx * Nt;
  }
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

// dS_hat[idx] = S (g - <S, g>) for every non-padding packed row; dS_hat is
// zero-filled beforehand (rows no packed row maps to get no gradient).
__global__ __launch_bounds__(256) void masked_softmax_packed_bwd_kernel(
    const float* __restrict__ S, const float* __restrict__ G,
    const int64_t* __restrict__ dense_index, float* __restrict__ dS_hat,
    int rows, int64_t dense_rows, int Nt) {
  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  const int r = blockIdx.x * 4 + wave;
  if (r >= rows) return;
  const int64_t idx = dense_index[r];
  if (idx < 0 || idx >= dense_rows) return;
  const float* s = S + (size_t)r * Nt;
  const float* g = G + (size_t)r * Nt;
  float dot = 0.f;
  for (int j = lane; j < Nt; j += kWave) dot += s[j] * g[j];
  dot = wave_sum(dot);
  float* d = dS_hat + (size_t)idx * Nt;
  for (int j = lane; j < Nt; j += kWave) d[j] = s[j] * (g[j] - dot);
}

// ---------------------------------------------------------------------------
// NLL (+ Hits@1).  One workgroup; fixed-order reduction (deterministic).
//   loss = sum_g w_g * -log(S[y0_g, y1_g] + eps) / (mean ? max(sum w, 1) : 1)
//   aux  = [sum w, sum w * (argmax_j S[y0_g, j] == y1_g)]
// ---------------------------------------------------------------------------
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  float t = 0.f;
  for (int w = 0; w < kLossThreads / kWave; ++w) t += red[w];
  return t;
}

__global__ __launch_bounds__(kLossThreads) void nll_fwd_kernel(
    const float* __restrict__ S, const int64_t* __restrict__ y0,
    const int64_t* __restrict__ y1, const bool* __restrict__ mask,
    float* __restrict__ loss, float* __restrict__ aux, int G, int Nt,
    float eps, int mean, int with_correct) {
  __shared__ float red[kLossThreads / kWave];
  float acc = 0.f, cnt = 0.f, cor = 0.f;
  for (int g = threadIdx.x; g < G; g += kLossThreads) {
    if (mask != nullptr && !mask[g]) continue;
    const float* row = S + (size_t)y0[g] * Nt;
    const int64_t t = y1[g];
    acc += -__logf(row[t] + eps);
    cnt += 1.f;
    if (with_correct) {
      float best = -INFINITY;
      int64_t arg = 0;
      for (int j = 0; j < Nt; ++j) {
        const float v = row[j];
        if (v > best) { best = v; arg = j; }
      }
      cor += arg == t ? 1.f : 0.f;
    }
  }
  acc = block_sum(acc, red);
  cnt = block_sum(cnt, red);
  cor = block_sum(cor, red);
  if (threadIdx.x == 0) {
    loss[0] = mean ? acc / fmaxf(cnt, 1.f) : acc;
    aux[0] = cnt;
    aux[1] = cor;
  }
}

// dS[y0_g, y1_g] += -grad * w_g / (S + eps) / divisor   (dS zero-filled).
__global__ __launch_bounds__(256) void nll_bwd_kernel(
    const float* __restrict__ grad, const float* __restrict__ S,
    const int64_t* __restrict__ y0, const int64_t* __restrict__ y1,
    const bool* __restrict__ mask, const float* __restrict__ aux,
    float* __restrict__ dS, int G, int Nt, float eps, int mean) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= G) return;
  if (mask != nullptr && !mask[g]) return;
  const float div = mean ? fmaxf(aux[0], 1.f) : 1.f;
  const size_t e = (size_t)y0[g] * Nt + y1[g];
  atomicAdd(dS + e, -grad[0] / ((S[e] + eps) * div));
}

// ---------------------------------------------------------------------------
// Sparse NLL (+ Hits@1) over top-k candidate lists (reference dgmc.py:
// 258-266: val = S.__val__[y0][S.__idx__[y0] == y1]; nll = -log(val + eps)).
// Every candidate slot of row y0_g holding target y1_g contributes (a
// ground truth missing from the candidates contributes nothing, duplicates
// count per slot); 'mean' divides by the number of contributing slots.
//   aux = [hits, correct, ground truths]  (correct: the row's first maximal
//   candidate is y1_g).  Per-block partials + a one-wave fold (fixed order).
// The backward writes dval[y0_g, c] = -grad / ((val + eps) div) with atomics
// only where two ground truths name the same (row, target): identical
// addends, so the sum does not depend on their order (deterministic).  This
// replaces the ATen chain of advanced-indexing gathers and the sort-based
// index_put backward (~25 launches per DBP15K step).
// ---------------------------------------------------------------------------
constexpr int kSnllMaxBlocks = 256;

// Stage 1: one ground truth per thread; per-block partials
// part[block] = {sum nll, hits, correct, ground truths}.
__global__ __launch_bounds__(256) void sparse_nll_part_kernel(
    const float* __restrict__ val, const int64_t* __restrict__ idx,
    const int64_t* __restrict__ y0, const int64_t* __restrict__ y1,
    const bool* __restrict__ mask, float4* __restrict__ part, int G, int K,
    int64_t R, float eps) {
  __shared__ float4 red[4];
  float acc = 0.f, hits = 0.f, cor = 0.f, cnt = 0.f;
  for (int g = blockIdx.x * 256 + threadIdx.x; g < G; g += gridDim.x * 256) {
    if (mask != nullptr && !mask[g]) continue;
    const int64_t r = y0[g];
    if (r < 0 || r >= R) continue;       // (invalid source row: ignored)
    const size_t o = (size_t)r * K;
    const int64_t t = y1[g];
    float best = -INFINITY;
    int64_t pred = -1;
#pragma unroll 4
    for (int c = 0; c < K; ++c) {
      const float v = val[o + c];
      const int64_t j = idx[o + c];
      if (j == t) { acc += -__logf(v + eps); hits += 1.f; }
      if (v > best || pred < 0) { best = v; pred = j; }
    }
    cor += pred == t ? 1.f : 0.f;
    cnt += 1.f;
  }
  acc = wave_sum(acc);
  hits = wave_sum(hits);
  cor = wave_sum(cor);
  cnt = wave_sum(cnt);
  const int wave = threadIdx.x / kWave;
  if (threadIdx.x % kWave == 0) red[wave] = make_float4(acc, hits, cor, cnt);
  __syncthreads();
  if (threadIdx.x == 0) {
    float4 t = red[0];
#pragma unroll
    for (int w = 1; w < 4; ++w) {
      t.x += red[w].x; t.y += red[w].y; t.z += red[w].z; t.w += red[w].w;
    }
    part[blockIdx.x] = t;
  }
}

// Stage 2 (one wave, fixed order): loss and aux = [hits, correct, count].
__global__ __launch_bounds__(64) void sparse_nll_fold_kernel(
    const float4* __restrict__ part, int nparts, float* __restrict__ loss,
    float* __restrict__ aux, int mean) {
  float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int b = threadIdx.x; b < nparts; b += kWave) {
    const float4 q = part[b];
    t.x += q.x; t.y += q.y; t.z += q.z; t.w += q.w;
  }
  t.x = wave_sum(t.x);
  t.y = wave_sum(t.y);
  t.z = wave_sum(t.z);
  t.w = wave_sum(t.w);
  if (threadIdx.x == 0) {
    loss[0] = mean ? t.x / fmaxf(t.y, 1.f) : t.x;
    aux[0] = t.y;
    aux[1] = t.z;
    aux[2] = t.w;
  }
}

__global__ __launch_bounds__(256) void sparse_nll_bwd_kernel(
    const float* __restrict__ grad, const float* __restrict__ val,
    const int64_t* __restrict__ idx, const int64_t* __restrict__ y0,
    const int64_t* __restrict__ y1, const bool* __restrict__ mask,
    const float* __restrict__ aux, float* __restrict__ dval, int G, int K,
    int64_t R, float eps, int mean) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= G) return;
  if (mask != nullptr && !mask[g]) return;
  const int64_t r = y0[g];
  if (r < 0 || r >= R) return;
  const float div = mean ? fmaxf(aux[0], 1.f) : 1.f;
  const size_t o = (size_t)r * K;
  const int64_t t = y1[g];
  for (int c = 0; c < K; ++c)
    if (idx[o + c] == t)
      atomicAdd(dval + o + c, -grad[0] / ((val[o + c] + eps) * div));
}

// ---------------------------------------------------------------------------
// Fused masked row softmax + NLL + Hits@1 of the dense correspondences, for
// the training objective (DGMC.loss / DGMC.acc, dgmc.py:246-288, on
// masked_softmax(S_hat), dgmc.py:15-19,165,181).  Ground truth of packed row
// r = ptr_s[b] + i is column y[r] (weight mask[r]); rows are visited in the
// dense [B, Ns] grid, so the backward writes every dense row (zeros outside
// the valid n_s x n_t blocks) without a zero-fill pass.
//   fwd: per-block partials (sum -log(S_y + eps), count, correct) -> fold
//   bwd: dS_hat[b, i, j] = d S_j (delta_jy - S_y),  d = -g / ((S_y + eps) n)
// The packed probabilities themselves are never written (the training step
// does not read them).
// ---------------------------------------------------------------------------
constexpr int kSnWaves = 4;

// Blocks [0, nb) read tile S_hat, blocks [nb, 2 nb) the optional second
// tile S_hat2 (the objective's two outputs S_L and S_0 in one launch).
__global__ __launch_bounds__(kSnWaves * 64) void softmax_nll_fwd_kernel(
    const float* __restrict__ S_hat1, const float* __restrict__ S_hat2,
    const int* __restrict__ ptr_s, const int* __restrict__ n_t,
    const int64_t* __restrict__ y, const bool* __restrict__ mask,
    float* __restrict__ part, int B, int Ns, int Nt, int nb, float eps) {
  __shared__ float red[kSnWaves][3];
  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  const bool second = (int)blockIdx.x >= nb;
  const float* __restrict__ S_hat = second ? S_hat2 : S_hat1;
  const int row = (blockIdx.x - (second ? nb : 0)) * kSnWaves + wave;
  float l = 0.f, c = 0.f, k = 0.f;
  if (row < B * Ns) {
    const int b = row / Ns, i = row - b * Ns;
    const int r = ptr_s[b] + i;
    const int nt = n_t[b];
    if (r < ptr_s[b + 1] && nt > 0 && (mask == nullptr || mask[r])) {
      const float* src = S_hat + (size_t)row * Nt;
      const int t = (int)y[r];
      float m = -INFINITY;
      int arg = 0;
      for (int j = lane; j < nt; j += kWave) {
        const float v = src[j];
        if (v > m) { m = v; arg = j; }
      }
      // wave argmax (first index among equal maxima)
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const float mo = __shfl_xor(m, o);
        const int ao = __shfl_xor(arg, o);
        if (mo > m || (mo == m && ao < arg)) { m = mo; arg = ao; }
      }
      float s = 0.f;
      for (int j = lane; j < nt; j += kWave) s += __expf(src[j] - m);
      s = wave_sum(s);
      const float st = (t >= 0 && t < nt) ? __expf(src[t] - m) / s : 0.f;
      l = -__logf(st + eps);
      c = 1.f;
      k = arg == t ? 1.f : 0.f;
    }
  }
  if (lane == 0) {
    red[wave][0] = l;
    red[wave][1] = c;
    red[wave][2] = k;
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    float a = 0.f;
    for (int w = 0; w < kSnWaves; ++w) a += red[w][threadIdx.x];
    part[(size_t)blockIdx.x * 3 + threadIdx.x] = a;
  }
}

// Fixed-order fold of the block partials: loss = sum over tiles of the mean
// over counted rows, aux = [count, correct] of the first tile and the
// second tile's count.  ``stats`` (optional, fp64): += [loss, correct,
// count] (the trainer's running sums, no extra kernels).
__global__ __launch_bounds__(kLossThreads) void softmax_nll_fold_kernel(
    const float* __restrict__ part, int nblocks, int tiles,
    float* __restrict__ loss, float* __restrict__ aux,
    double* __restrict__ stats) {
  __shared__ float red[kLossThreads / kWave];
  float total = 0.f, c0 = 0.f, k0 = 0.f, c1 = 0.f;
  for (int tile = 0; tile < tiles; ++tile) {
    const float* pt = part + (size_t)tile * nblocks * 3;
    float a = 0.f, c = 0.f, k = 0.f;
    for (int i = threadIdx.x; i < nblocks; i += kLossThreads) {
      a += pt[3 * i];
      c += pt[3 * i + 1];
      k += pt[3 * i + 2];
    }
    a = block_sum(a, red);
    c = block_sum(c, red);
    k = block_sum(k, red);
    total += a / fmaxf(c, 1.f);
    if (tile == 0) {
      c0 = c;
      k0 = k;
    } else {
      c1 = c;
    }
  }
  if (threadIdx.x == 0) {
    loss[0] = total;
    aux[0] = c0;
    aux[1] = k0;
    aux[2] = c1;
    if (stats) {
      stats[0] += (double)total;
      stats[1] += (double)k0;
      stats[2] += (double)c0;
    }
  }
}

__global__ __launch_bounds__(kSnWaves * 64) void softmax_nll_bwd_kernel(
    const float* __restrict__ grad, const float* __restrict__ S_hat1,
    const float* __restrict__ S_hat2, const int* __restrict__ ptr_s,
    const int* __restrict__ n_t, const int64_t* __restrict__ y,
    const bool* __restrict__ mask, const float* __restrict__ aux,
    float* __restrict__ dS1, float* __restrict__ dS2, int B, int Ns, int Nt,
    int nb, float eps) {
  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  const bool second = (int)blockIdx.x >= nb;
  const float* __restrict__ S_hat = second ? S_hat2 : S_hat1;
  float* __restrict__ dS = second ? dS2 : dS1;
  const float count = second ? aux[2] : aux[0];
  const int row = (blockIdx.x - (second ? nb : 0)) * kSnWaves + wave;
  if (row >= B * Ns) return;
  const int b = row / Ns, i = row - b * Ns;
  const int r = ptr_s[b] + i;
  const int nt = n_t[b];
  float* d = dS + (size_t)row * Nt;
  const bool valid =
      r < ptr_s[b + 1] && nt > 0 && (mask == nullptr || mask[r]);
  const int t = valid ? (int)y[r] : -1;
  if (!valid || t < 0 || t >= nt) {
    for (int j = lane; j < Nt; j += kWave) d[j] = 0.f;
    return;
  }
  const float* src = S_hat + (size_t)row * Nt;
  float m = -INFINITY;
  for (int j = lane; j < nt; j += kWave) m = fmaxf(m, src[j]);
  m = wave_max(m);
  float s = 0.f;
  for (int j = lane; j < nt; j += kWave) s += __expf(src[j] - m);
  s = wave_sum(s);
  const float inv = 1.f / s;
  const float st = __expf(src[t] - m) * inv;
  const float dy = -grad[0] / ((st + eps) * fmaxf(count, 1.f));
  for (int j = lane; j < Nt; j += kWave) {
    float v = 0.f;
    if (j < nt) {
      const float sj = __expf(src[j] - m) * inv;
      v = dy * sj * ((j == t ? 1.f : 0.f) - st);
    }
    d[j] = v;
  }
}

// ---------------------------------------------------------------------------
// Non-finite check: per-block flags, then one block folds them into the
// found_inf scalar (fp32 0/1, read by fused Adam) and the skipped-step count.
// ---------------------------------------------------------------------------
constexpr int kFiniteBlocks = 512;

__global__ __launch_bounds__(256) void nonfinite_partials_kernel(
    const float* __restrict__ x, int64_t n, int* __restrict__ part) {
  __shared__ int any;
  if (threadIdx.x == 0) any = 0;
  __syncthreads();
  int bad = 0;
  const int64_t n4 = n / 4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
       i += stride) {
    const float4 v = reinterpret_cast<const float4*>(x)[i];
    bad |= !isfinite(v.x) | !isfinite(v.y) | !isfinite(v.z) | !isfinite(v.w);
  }
  for (int64_t i = n4 * 4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
       i < n; i += stride)
    bad |= !isfinite(x[i]);
  if (bad) any = 1;   // benign race: every writer stores 1
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = any;
}

__global__ __launch_bounds__(256) void nonfinite_final_kernel(
    const int* __restrict__ part, int nparts, float* __restrict__ found_inf,
    double* __restrict__ counter) {
  int bad = 0;
  for (int i = threadIdx.x; i < nparts; i += blockDim.x) bad |= part[i];
  bad = __syncthreads_or(bad);
  if (threadIdx.x == 0) {
    found_inf[0] = bad ? 1.f : 0.f;
    if (counter != nullptr) counter[0] += bad ? 1.0 : 0.0;
  }
}

// ---------------------------------------------------------------------------
// Host wrappers
// ---------------------------------------------------------------------------
at::Tensor masked_softmax_packed(const at::Tensor& S_hat,
                                 const at::Tensor& dense_index,
                                 const at::Tensor& n_s, const at::Tensor& n_t) {
  TORCH_CHECK(S_hat.is_cuda() && S_hat.scalar_type() == at::kFloat &&
                  S_hat.is_contiguous() && S_hat.dim() == 3,
              "masked_softmax_packed: contiguous fp32 [B, Ns, Nt] scores");
  TORCH_CHECK(dense_index.scalar_type() == at::kLong && dense_index.dim() == 1 &&
                  dense_index.is_contiguous(),
              "masked_softmax_packed: int64 dense row index");
  const int B = S_hat.size(0), Ns = S_hat.size(1), Nt = S_hat.size(2);
  TORCH_CHECK(n_s.scalar_type() == at::kInt && n_t.scalar_type() == at::kInt &&
                  n_s.numel() == B && n_t.numel() == B,
              "masked_softmax_packed: int32 [B] node counts");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(S_hat.device());
  const int rows = dense_index.numel();
  at::Tensor out = at::empty({rows, Nt}, S_hat.options());
  if (rows == 0 || Nt == 0) return out;
  hipLaunchKernelGGL(masked_softmax_packed_kernel, dim3((rows + 3) / 4),
                     dim3(256), 0, stream(), S_hat.data_ptr<float>(),
                     dense_index.data_ptr<int64_t>(), n_s.data_ptr<int>(),
                     n_t.data_ptr<int>(), out.data_ptr<float>(), rows, B, Ns,
                     Nt);
  DGMC_CHECK_LAUNCH();
  return out;
}

at::Tensor masked_softmax_packed_bwd(const at::Tensor& S, const at::Tensor& G,
                                     const at::Tensor& dense_index, int64_t B,
                                     int64_t Ns) {
  TORCH_CHECK(S.is_cuda() && S.scalar_type() == at::kFloat &&
                  S.is_contiguous() && S.dim() == 2 &&
                  G.scalar_type() == at::kFloat && G.is_contiguous() &&
                  G.sizes() == S.sizes(),
              "masked_softmax_packed_bwd: contiguous fp32 [rows, Nt] S / grad");
  TORCH_CHECK(dense_index.scalar_type() == at::kLong &&
                  dense_index.numel() == S.size(0),
              "masked_softmax_packed_bwd: int64 dense row index per row");
  const int rows = S.size(0), Nt = S.size(1);
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(S.device());
  at::Tensor dS = at::zeros({B, Ns, (int64_t)Nt}, S.options());
  if (rows == 0 || Nt == 0) return dS;
  hipLaunchKernelGGL(masked_softmax_packed_bwd_kernel, dim3((rows + 3) / 4),
                     dim3(256), 0, stream(), S.data_ptr<float>(),
                     G.data_ptr<float>(), dense_index.data_ptr<int64_t>(),
                     dS.data_ptr<float>(), rows, B * Ns, Nt);
  DGMC_CHECK_LAUNCH();
  return dS;
}

static void check_nll_args(const at::Tensor& S, const at::Tensor& y0,
                           const at::Tensor& y1,
                           const c10::optional<at::Tensor>& mask) {
  TORCH_CHECK(S.is_cuda() && S.scalar_type() == at::kFloat &&
                  S.is_contiguous() && S.dim() == 2,
              "nll: contiguous fp32 [rows, Nt] probabilities");
  TORCH_CHECK(y0.scalar_type() == at::kLong && y1.scalar_type() == at::kLong &&
                  y0.is_contiguous() && y1.is_contiguous() &&
                  y0.numel() == y1.numel(),
              "nll: int64 contiguous y0 / y1 of equal length");
  if (mask.has_value() && mask->defined())
    TORCH_CHECK(mask->scalar_type() == at::kBool && mask->is_contiguous() &&
                    mask->numel() == y0.numel(),
                "nll: bool mask per ground truth");
}

std::tuple<at::Tensor, at::Tensor> nll_fwd(const at::Tensor& S,
                                           const at::Tensor& y0,
                                           const at::Tensor& y1,
                                           const c10::optional<at::Tensor>& mask,
                                           double eps, bool mean,
                                           bool with_correct) {
  check_nll_args(S, y0, y1, mask);
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(S.device());
  at::Tensor loss = at::empty({}, S.options());
  at::Tensor aux = at::empty({2}, S.options());
  const bool* mp = (mask.has_value() && mask->defined())
                       ? mask->data_ptr<bool>() : nullptr;
  hipLaunchKernelGGL(nll_fwd_kernel, dim3(1), dim3(kLossThreads), 0, stream(),
                     S.data_ptr<float>(), y0.data_ptr<int64_t>(),
                     y1.data_ptr<int64_t>(), mp, loss.data_ptr<float>(),
                     aux.data_ptr<float>(), (int)y0.numel(), (int)S.size(1),
                     (float)eps, mean ? 1 : 0, with_correct ? 1 : 0);
  DGMC_CHECK_LAUNCH();
  return {loss, aux};
}

at::Tensor nll_bwd(const at::Tensor& grad, const at::Tensor& S,
                   const at::Tensor& y0, const at::Tensor& y1,
                   const c10::optional<at::Tensor>& mask, const at::Tensor& aux,
                   double eps, bool mean) {
  check_nll_args(S, y0, y1, mask);
  TORCH_CHECK(grad.numel() == 1 && grad.scalar_type() == at::kFloat &&
                  aux.numel() == 2 && aux.scalar_type() == at::kFloat,
              "nll_bwd: scalar fp32 grad, [2] aux");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(S.device());
  at::Tensor dS = at::zeros_like(S);
  const int G = y0.numel();
  if (G == 0) return dS;
  const bool* mp = (mask.has_value() && mask->defined())
                       ? mask->data_ptr<bool>() : nullptr;
  at::Tensor g = grad.contiguous();
  hipLaunchKernelGGL(nll_bwd_kernel, dim3((G + 255) / 256), dim3(256), 0,
                     stream(), g.data_ptr<float>(), S.data_ptr<float>(),
                     y0.data_ptr<int64_t>(), y1.data_ptr<int64_t>(), mp,
                     aux.data_ptr<float>(), dS.data_ptr<float>(), G,
                     (int)S.size(1), (float)eps, mean ? 1 : 0);
  DGMC_CHECK_LAUNCH();
  return dS;
}

static void check_sparse_nll_args(const at::Tensor& val,
                                  const at::Tensor& idx, const at::Tensor& y0,
                                  const at::Tensor& y1,
                                  const c10::optional<at::Tensor>& mask) {
  TORCH_CHECK(val.is_cuda() && val.scalar_type() == at::kFloat &&
                  val.is_contiguous() && val.dim() == 2,
              "sparse_nll: contiguous fp32 [rows, k] candidate values");
  TORCH_CHECK(idx.scalar_type() == at::kLong && idx.is_contiguous() &&
                  idx.sizes() == val.sizes(),
              "sparse_nll: int64 [rows, k] candidate indices like val");
  TORCH_CHECK(y0.scalar_type() == at::kLong && y1.scalar_type() == at::kLong &&
                  y0.is_contiguous() && y1.is_contiguous() &&
                  y0.numel() == y1.numel(),
              "sparse_nll: int64 contiguous y0 / y1 of equal length");
  if (mask.has_value() && mask->defined())
    TORCH_CHECK(mask->scalar_type() == at::kBool && mask->is_contiguous() &&
                    mask->numel() == y0.numel(),
                "sparse_nll: bool mask per ground truth");
}

std::tuple<at::Tensor, at::Tensor> sparse_nll_fwd(
    const at::Tensor& val, const at::Tensor& idx, const at::Tensor& y0,
    const at::Tensor& y1, const c10::optional<at::Tensor>& mask, double eps,
    bool mean) {
  check_sparse_nll_args(val, idx, y0, y1, mask);
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(val.device());
  at::Tensor loss = at::empty({}, val.options());
  at::Tensor aux = at::empty({3}, val.options());
  const bool* mp = (mask.has_value() && mask->defined())
                       ? mask->data_ptr<bool>() : nullptr;
  const int G = y0.numel();
  const int nb = std::max(1, std::min(kSnllMaxBlocks, (G + 255) / 256));
  at::Tensor part = at::empty({nb, 4}, val.options());
  float4* pp = reinterpret_cast<float4*>(part.data_ptr<float>());
  hipLaunchKernelGGL(sparse_nll_part_kernel, dim3(nb), dim3(256), 0, stream(),
                     val.data_ptr<float>(), idx.data_ptr<int64_t>(),
                     y0.data_ptr<int64_t>(), y1.data_ptr<int64_t>(), mp, pp,
                     G, (int)val.size(1), val.size(0), (float)eps);
  DGMC_CHECK_LAUNCH();
  hipLaunchKernelGGL(sparse_nll_fold_kernel, dim3(1), dim3(64), 0, stream(),
                     pp, nb, loss.data_ptr<float>(), aux.data_ptr<float>(),
                     mean ? 1 : 0);
  DGMC_CHECK_LAUNCH();
  return {loss, aux};
}

at::Tensor sparse_nll_bwd(const at::Tensor& grad, const at::Tensor& val,
                          const at::Tensor& idx, const at::Tensor& y0,
                          const at::Tensor& y1,
                          const c10::optional<at::Tensor>& mask,
                          const at::Tensor& aux, double eps, bool mean) {
  check_sparse_nll_args(val, idx, y0, y1, mask);
  TORCH_CHECK(grad.numel() == 1 && grad.scalar_type() == at::kFloat &&
                  aux.numel() == 3 && aux.scalar_type() == at::kFloat,
              "sparse_nll_bwd: scalar fp32 grad, [3] aux");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(val.device());
  at::Tensor dval = at::zeros_like(val);
  const int G = y0.numel();
  if (G == 0) return dval;
  const bool* mp = (mask.has_value() && mask->defined())
                       ? mask->data_ptr<bool>() : nullptr;
  at::Tensor g = grad.contiguous();
  hipLaunchKernelGGL(sparse_nll_bwd_kernel, dim3((G + 255) / 256), dim3(256),
                     0, stream(), g.data_ptr<float>(), val.data_ptr<float>(),
                     idx.data_ptr<int64_t>(), y0.data_ptr<int64_t>(),
                     y1.data_ptr<int64_t>(), mp, aux.data_ptr<float>(),
                     dval.data_ptr<float>(), G, (int)val.size(1),
                     val.size(0), (float)eps, mean ? 1 : 0);
  DGMC_CHECK_LAUNCH();
  return dval;
}

void nonfinite_flag(const at::Tensor& x, at::Tensor found_inf,
                    const c10::optional<at::Tensor>& counter) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kFloat && x.is_contiguous() &&
                  aligned16(x.data_ptr()),
              "nonfinite_flag: contiguous aligned fp32 tensor");
  TORCH_CHECK(found_inf.scalar_type() == at::kFloat && found_inf.numel() == 1,
              "nonfinite_flag: fp32 scalar found_inf");
  double* cp = nullptr;
  if (counter.has_value() && counter->defined()) {
    TORCH_CHECK(counter->scalar_type() == at::kDouble && counter->numel() == 1,
                "nonfinite_flag: fp64 scalar counter");
    cp = counter->data_ptr<double>();
  }
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  const int64_t n = x.numel();
  const int blocks = (int)std::max<int64_t>(
      1, std::min<int64_t>(kFiniteBlocks, (n / 4 + 255) / 256));
  at::Tensor part = at::empty({blocks}, x.options().dtype(at::kInt));
  hipLaunchKernelGGL(nonfinite_partials_kernel, dim3(blocks), dim3(256), 0,
                     stream(), x.data_ptr<float>(), n, part.data_ptr<int>());
  hipLaunchKernelGGL(nonfinite_final_kernel, dim3(1), dim3(256), 0, stream(),
                     part.data_ptr<int>(), blocks, found_inf.data_ptr<float>(),
                     cp);
  DGMC_CHECK_LAUNCH();
}

namespace {
void check_snll(const at::Tensor& S_hat, const at::Tensor& ptr_s,
                const at::Tensor& n_t, const at::Tensor& y,
                const c10::optional<at::Tensor>& mask) {
  TORCH_CHECK(S_hat.is_cuda() && S_hat.scalar_type() == at::kFloat &&
                  S_hat.dim() == 3 && S_hat.is_contiguous(),
              "softmax_nll: contiguous fp32 S_hat [B, Ns, Nt]");
  const int64_t B = S_hat.size(0);
  TORCH_CHECK(ptr_s.scalar_type() == at::kInt && ptr_s.numel() == B + 1 &&
                  n_t.scalar_type() == at::kInt && n_t.numel() == B,
              "softmax_nll: int32 ptr_s [B + 1] / n_t [B]");
  TORCH_CHECK(y.scalar_type() == at::kLong && y.is_contiguous(),
              "softmax_nll: int64 y per packed row");
  if (mask.has_value() && mask->defined())
    TORCH_CHECK(mask->scalar_type() == at::kBool &&
                    mask->numel() == y.numel() && mask->is_contiguous(),
                "softmax_nll: bool mask per packed row");
}
}  // namespace

// loss = NLL(S_hat) [+ NLL(S_hat2)], aux = [count, correct, count2]; the
// optional fp64 ``stats`` receives += [loss, correct, count].
std::tuple<at::Tensor, at::Tensor> softmax_nll_fwd(
    const at::Tensor& S_hat, const c10::optional<at::Tensor>& S_hat2,
    const at::Tensor& ptr_s, const at::Tensor& n_t, const at::Tensor& y,
    const c10::optional<at::Tensor>& mask, double eps,
    const c10::optional<at::Tensor>& stats) {
  check_snll(S_hat, ptr_s, n_t, y, mask);
  const bool two = S_hat2.has_value() && S_hat2->defined();
  if (two)
    TORCH_CHECK(S_hat2->sizes() == S_hat.sizes() &&
                    S_hat2->scalar_type() == at::kFloat &&
                    S_hat2->is_contiguous(),
                "softmax_nll: S_hat2 like S_hat");
  double* sp = nullptr;
  if (stats.has_value() && stats->defined()) {
    TORCH_CHECK(stats->scalar_type() == at::kDouble && stats->numel() >= 3 &&
                    stats->is_contiguous() && stats->device() == S_hat.device(),
                "softmax_nll: stats fp64 [>= 3] on the device");
    sp = stats->data_ptr<double>();
  }
  const int B = S_hat.size(0), Ns = S_hat.size(1), Nt = S_hat.size(2);
  auto opt = S_hat.options();
  at::Tensor loss = at::empty({}, opt);
  at::Tensor aux = at::empty({3}, opt);
  const int rows = B * Ns;
  const int nblocks = std::max(1, (rows + kSnWaves - 1) / kSnWaves);
  const int tiles = two ? 2 : 1;
  at::Tensor part = at::empty({tiles * nblocks * 3}, opt);
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(S_hat.device());
  const bool* mp = (mask.has_value() && mask->defined())
                       ? mask->data_ptr<bool>() : nullptr;
  hipLaunchKernelGGL(softmax_nll_fwd_kernel, dim3(tiles * nblocks),
                     dim3(kSnWaves * 64), 0, stream(), S_hat.data_ptr<float>(),
                     two ? S_hat2->data_ptr<float>() : nullptr,
                     ptr_s.data_ptr<int>(), n_t.data_ptr<int>(),
                     y.data_ptr<int64_t>(), mp, part.data_ptr<float>(), B, Ns,
                     Nt, nblocks, (float)eps);
  hipLaunchKernelGGL(softmax_nll_fold_kernel, dim3(1), dim3(kLossThreads), 0,
                     stream(), part.data_ptr<float>(), nblocks, tiles,
                     loss.data_ptr<float>(), aux.data_ptr<float>(), sp);
  DGMC_CHECK_LAUNCH();
  return {loss, aux};
}

// Gradients of both tiles (dS2 undefined without S_hat2).
std::tuple<at::Tensor, at::Tensor> softmax_nll_bwd(
    const at::Tensor& grad, const at::Tensor& S_hat,
    const c10::optional<at::Tensor>& S_hat2, const at::Tensor& ptr_s,
    const at::Tensor& n_t, const at::Tensor& y,
    const c10::optional<at::Tensor>& mask, const at::Tensor& aux,
    double eps) {
  check_snll(S_hat, ptr_s, n_t, y, mask);
  TORCH_CHECK(grad.scalar_type() == at::kFloat && grad.numel() == 1 &&
                  aux.scalar_type() == at::kFloat && aux.numel() == 3,
              "softmax_nll_bwd: fp32 scalar grad / aux [3]");
  const bool two = S_hat2.has_value() && S_hat2->defined();
  if (two)
    TORCH_CHECK(S_hat2->sizes() == S_hat.sizes() &&
                    S_hat2->scalar_type() == at::kFloat &&
                    S_hat2->is_contiguous(),
                "softmax_nll_bwd: S_hat2 like S_hat");
  const int B = S_hat.size(0), Ns = S_hat.size(1), Nt = S_hat.size(2);
  at::Tensor dS = at::empty_like(S_hat);
  at::Tensor dS2 = two ? at::empty_like(S_hat) : at::Tensor();
  const int rows = B * Ns;
  if (rows == 0) return {dS, dS2};
  const int nblocks = (rows + kSnWaves - 1) / kSnWaves;
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(S_hat.device());
  const bool* mp = (mask.has_value() && mask->defined())
                       ? mask->data_ptr<bool>() : nullptr;
  hipLaunchKernelGGL(softmax_nll_bwd_kernel, dim3((two ? 2 : 1) * nblocks),
                     dim3(kSnWaves * 64), 0, stream(), grad.data_ptr<float>(),
                     S_hat.data_ptr<float>(),
                     two ? S_hat2->data_ptr<float>() : nullptr,
                     ptr_s.data_ptr<int>(), n_t.data_ptr<int>(),
                     y.data_ptr<int64_t>(), mp, aux.data_ptr<float>(),
                     dS.data_ptr<float>(), two ? dS2.data_ptr<float>() : nullptr,
                     B, Ns, Nt, nblocks, (float)eps);
  DGMC_CHECK_LAUNCH();
  return {dS, dS2};
}

}  // namespace dgmc
