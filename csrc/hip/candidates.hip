// Training candidate set of the sparse correspondence path (K12):
//
//   S_idx = cat([top-k, randint(N_t, (B, N_s, k_r))], -1), then for every
//   ground-truth pair (row, col) whose col is not among the row's candidates,
//   the LAST candidate is replaced by col.
//
// Reference: /root/reference/dgmc/models/dgmc.py:190-195 (torch.randint +
// torch.cat + __include_gt__, ~9 ATen launches with a boolean-mask index).
// Here: one kernel writes the [R, k + k_r] candidate rows (top-k copied,
// negatives drawn from a counter-based Philox4x32-10 stream keyed by the
// default generator's graph-safe (seed, offset) - the same state ATen's
// randint consumes, so a captured step draws fresh negatives every replay),
// a second patches the ground-truth rows.  Both are deterministic for a given
// generator state.
#include "common.h"

#include <ATen/hip/HIPGeneratorImpl.h>
#include <ATen/hip/detail/UnpackRaw.cuh>
#include <rocprim/device/device_radix_sort.hpp>

#include <mutex>

namespace dgmc {

namespace {

// Philox4x32-10 (Salmon et al., SC'11): 10 rounds of the 4x32 bijection.
__device__ __forceinline__ uint4 philox4x32_10(uint4 c, uint2 k) {
  constexpr uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  constexpr uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = __umulhi(M0, c.x), lo0 = M0 * c.x;
    const uint32_t hi1 = __umulhi(M1, c.z), lo1 = M1 * c.z;
    c = make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
    k.x += W0;
    k.y += W1;
  }
  return c;
}

// One thread per candidate entry (r, j): j < k copies the top-k index, else
// a uniform index in [0, N_t) (multiply-shift of a 32-bit draw).
__global__ __launch_bounds__(256) void candidates_kernel(
    const int64_t* __restrict__ topk, int64_t R, int k, int kr, int64_t n_t,
    at::PhiloxCudaState rng, int64_t* __restrict__ out) {
  const int kk = k + kr;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= R * kk) return;
  const int64_t r = e / kk;
  const int j = (int)(e - r * kk);
  if (j < k) {
    out[e] = topk[r * k + j];
    return;
  }
  const auto so = at::cuda::philox::unpack(rng);
  const uint64_t seed = std::get<0>(so), off = std::get<1>(so);
  // ATen's Philox layout (curand_init(seed, subsequence, offset)): the low
  // 64 counter bits are the 128-bit block (offset / 4), the high 64 the
  // subsequence (this entry) - so another op drawing from the generator
  // after this one (offset advanced by 4 below) never reuses these blocks.
  const uint64_t sub = (uint64_t)(r * kr + (j - k));
  const uint64_t blk = off / 4;
  const uint4 v = philox4x32_10(
      make_uint4((uint32_t)blk, (uint32_t)(blk >> 32), (uint32_t)sub,
                 (uint32_t)(sub >> 32)),
      make_uint2((uint32_t)seed, (uint32_t)(seed >> 32)));
  out[e] = (int64_t)(((uint64_t)v.x * (uint64_t)n_t) >> 32);
}

// One thread per ground-truth pair: if its target is not among the row's
// candidates, it takes the last slot (rows hold at most one ground truth).
__global__ __launch_bounds__(256) void include_gt_kernel(
    const int64_t* __restrict__ gt_row, const int64_t* __restrict__ gt_col,
    int64_t G, int64_t R, int kk, int64_t* __restrict__ out) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= G) return;
  const int64_t r = gt_row[g];
  if (r < 0 || r >= R) return;               // (invalid row: never written)
  const int64_t col = gt_col[g];
  int64_t* row = out + r * kk;
  bool present = false;
  for (int j = 0; j < kk; ++j) present |= row[j] == col;
  if (!present) row[kk - 1] = col;
}

// Candidate CSR / CSC, step 1: global target column of every candidate
// entry (pair b's targets start at b * N_t), the identity permutation (the
// sort's values) and the CSR row pointer (k entries per row).
__global__ __launch_bounds__(256) void csc_prep_kernel(
    const int64_t* __restrict__ idx, int64_t n, int k, int64_t rows_per_pair,
    int64_t n_t, int* __restrict__ col, int* __restrict__ iota,
    int* __restrict__ rowptr, int64_t R) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e <= R) rowptr[e] = (int)(e * k);
  if (e >= n) return;
  const int64_t r = e / k;
  col[e] = (int)(idx[e] + (r / rows_per_pair) * n_t);
  iota[e] = (int)e;
}

// Step 3 (after the stable radix sort by column): column pointers from the
// sorted keys (position i starts every column in (key[i-1], key[i]]) and
// the source row of every CSC entry.
__global__ __launch_bounds__(256) void csc_finish_kernel(
    const int* __restrict__ keys, const int* __restrict__ perm, int64_t n,
    int k, int64_t C, int* __restrict__ colptr, int* __restrict__ row_of) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i > n) return;
  // (keys lie in [0, C); the clamps only keep a corrupt index in bounds)
  const int64_t lo = i == 0 ? -1 : max((int64_t)keys[i - 1], (int64_t)-1);
  const int64_t hi = i == n ? C : min((int64_t)keys[i], C);
  for (int64_t c = lo + 1; c <= hi; ++c) colptr[c] = (int)i;
  if (i < n) row_of[i] = perm[i] / k;
}

}  // namespace

// S_idx [B, N_s, k] int64 (targets local to each pair's N_t block) ->
// (col int32 [nnz] global targets, rowptr int32 [B N_s + 1], colptr int32
// [B N_t + 1], perm int32 [nnz] CSC -> CSR entry map (stable: row order
// inside a column), row_of int32 [nnz]).  Prep + rocprim's stable radix
// sort (default configuration: it merge-sorts up to 1 M keys; forcing
// onesweep faulted inside the captured step) + finish, instead of an argsort
// + histogram + scan chain.
std::vector<at::Tensor> candidate_csc(const at::Tensor& S_idx, int64_t n_t) {
  TORCH_CHECK(S_idx.is_cuda() && S_idx.scalar_type() == at::kLong &&
                  S_idx.is_contiguous() && S_idx.dim() == 3,
              "candidate_csc: contiguous int64 [B, N_s, k]");
  const int64_t B = S_idx.size(0), N_s = S_idx.size(1), k = S_idx.size(2);
  const int64_t R = B * N_s, n = R * k, C = B * n_t;
  TORCH_CHECK(k >= 1 && n < INT32_MAX && C < INT32_MAX && n_t >= 1,
              "candidate_csc: sizes");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(S_idx.device());
  auto i32 = S_idx.options().dtype(at::kInt);
  at::Tensor col = at::empty({n}, i32), iota = at::empty({n}, i32);
  at::Tensor rowptr = at::empty({R + 1}, i32);
  at::Tensor keys = at::empty({n}, i32), perm = at::empty({n}, i32);
  at::Tensor colptr = at::empty({C + 1}, i32), row_of = at::empty({n}, i32);
  const int64_t m = std::max(n, R + 1);
  hipLaunchKernelGGL(csc_prep_kernel, dim3((unsigned)((m + 255) / 256)),
                     dim3(256), 0, stream(), S_idx.data_ptr<int64_t>(), n,
                     (int)k, N_s, n_t, col.data_ptr<int>(),
                     iota.data_ptr<int>(), rowptr.data_ptr<int>(), R);
  DGMC_CHECK_LAUNCH();
  unsigned bits = 1;
  while (bits < 31 && (int64_t(1) << bits) < C) ++bits;
  size_t tmp_bytes = 0;
  DGMC_CHECK_HIP(rocprim::radix_sort_pairs(
      nullptr, tmp_bytes, col.data_ptr<int>(), keys.data_ptr<int>(),
      iota.data_ptr<int>(), perm.data_ptr<int>(), (size_t)n, 0, bits,
      stream()));
  at::Tensor tmp = at::empty({(int64_t)std::max<size_t>(tmp_bytes, 1)},
                             S_idx.options().dtype(at::kByte));
  DGMC_CHECK_HIP(rocprim::radix_sort_pairs(
      tmp.data_ptr(), tmp_bytes, col.data_ptr<int>(), keys.data_ptr<int>(),
      iota.data_ptr<int>(), perm.data_ptr<int>(), (size_t)n, 0, bits,
      stream()));
  hipLaunchKernelGGL(csc_finish_kernel, dim3((unsigned)((n + 256) / 256)),
                     dim3(256), 0, stream(), keys.data_ptr<int>(),
                     perm.data_ptr<int>(), n, (int)k, C,
                     colptr.data_ptr<int>(), row_of.data_ptr<int>());
  DGMC_CHECK_LAUNCH();
  return {col, rowptr, colptr, perm, row_of};
}

// topk [..., k] int64; gt_row / gt_col int64 [G] (flattened candidate row of
// each ground-truth source, its target).  Returns [..., k + kr] int64.
at::Tensor train_candidates(const at::Tensor& topk, int64_t n_t, int64_t kr,
                            const at::Tensor& gt_row,
                            const at::Tensor& gt_col) {
  TORCH_CHECK(topk.is_cuda() && topk.scalar_type() == at::kLong &&
                  topk.is_contiguous() && topk.dim() >= 1,
              "train_candidates: contiguous int64 top-k indices");
  TORCH_CHECK(gt_row.scalar_type() == at::kLong &&
                  gt_col.scalar_type() == at::kLong &&
                  gt_row.is_contiguous() && gt_col.is_contiguous() &&
                  gt_row.numel() == gt_col.numel() &&
                  gt_row.device() == topk.device() &&
                  gt_col.device() == topk.device(),
              "train_candidates: int64 ground-truth rows / cols on the device");
  TORCH_CHECK(kr >= 0 && n_t >= 1 && n_t < (int64_t(1) << 32),
              "train_candidates: 0 <= kr, 1 <= N_t < 2^32");
  const int64_t k = topk.size(-1);
  const int64_t R = k > 0 ? topk.numel() / k : 0;
  const int64_t kk = k + kr;
  TORCH_CHECK(kk >= 1 && kk < 4096, "train_candidates: k + kr in [1, 4096)");
  std::vector<int64_t> shape(topk.sizes().begin(), topk.sizes().end());
  shape.back() = kk;
  at::Tensor out = at::empty(shape, topk.options());
  const int64_t n = R * kk;
  if (n == 0) return out;
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(topk.device());
  at::PhiloxCudaState rng;
  {
    auto* gen = at::get_generator_or_default<at::CUDAGeneratorImpl>(
        c10::nullopt, at::cuda::detail::getDefaultCUDAGenerator());
    std::lock_guard<std::mutex> lock(gen->mutex_);
    rng = gen->philox_cuda_state(4);
  }
  hipLaunchKernelGGL(candidates_kernel, dim3((unsigned)((n + 255) / 256)),
                     dim3(256), 0, stream(), topk.data_ptr<int64_t>(), R,
                     (int)k, (int)kr, n_t, rng, out.data_ptr<int64_t>());
  DGMC_CHECK_LAUNCH();
  const int64_t G = gt_row.numel();
  if (G > 0) {
    hipLaunchKernelGGL(include_gt_kernel, dim3((unsigned)((G + 255) / 256)),
                       dim3(256), 0, stream(), gt_row.data_ptr<int64_t>(),
                       gt_col.data_ptr<int64_t>(), G, R, (int)kk,
                       out.data_ptr<int64_t>());
    DGMC_CHECK_LAUNCH();
  }
  return out;
}

}  // namespace dgmc
