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

// Stable LSD radix sort of (key, value) int32 pairs, 8-bit digits, for the
// candidate CSC (a few hundred thousand entries: rocprim merge-sorts that
// size in ~18 launches).  Per pass two launches over tiles of kRsTile
// items (4 waves, each a contiguous quarter, 32 items per lane loaded into
// registers up front - one memory round trip):
//   rs_hist     per-wave digit counts (64-item groups: the lanes with the
//               same digit found by 8 ballots; the digit's highest lane adds
//               the group's count) -> [tiles][4 waves][256];
//   rs_scatter  every tile derives its waves' digit offsets from the whole
//               (small) count table, then writes every item at its digit's
//               running position in the wave + its rank among the group's
//               lanes with that digit: tile, wave, group, lane order -
//               stable.
constexpr int kRsBins = 256;
constexpr int kRsPer = 32;                       // items per lane
constexpr int kRsWave = 64 * kRsPer;             // items per wave
constexpr int kRsTile = 4 * kRsWave;             // items per tile (8192)
constexpr int kRsChunk = 32;                     // count rows per load round

__device__ __forceinline__ unsigned long long rs_match(int d) {
  unsigned long long m = ~0ull;
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    const unsigned long long v = __ballot((d >> b) & 1);
    m &= ((d >> b) & 1) ? v : ~v;
  }
  return m;
}

// Digit counts of this wave's quarter into cnt[256] (LDS, zeroed).
__device__ __forceinline__ void rs_count(const int* kr, int64_t i0, int64_t n,
                                         int shift, int* cnt) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int q = 0; q < kRsPer; ++q) {
    const bool ok = i0 + 64 * q < n;
    const int d = ok ? (kr[q] >> shift) & (kRsBins - 1) : -1;
    const unsigned long long m = rs_match(d) & __ballot(ok);
    if (ok && (m >> lane) == 1ull) cnt[d] += __popcll(m);
    __builtin_amdgcn_wave_barrier();
  }
}

__global__ __launch_bounds__(256) void rs_hist_kernel(
    const int* __restrict__ keys, int64_t n, int shift,
    int* __restrict__ hist, int tiles) {
  __shared__ int cnt[4][kRsBins];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int t = blockIdx.x;
  for (int d = lane; d < kRsBins; d += 64) cnt[wave][d] = 0;
  const int64_t i0 = (int64_t)t * kRsTile + wave * kRsWave + lane;
  int kr[kRsPer];
#pragma unroll
  for (int q = 0; q < kRsPer; ++q) {
    const int64_t i = i0 + 64 * q;
    kr[q] = keys[i < n ? i : 0];
  }
  __builtin_amdgcn_wave_barrier();
  rs_count(kr, i0, n, shift, &cnt[wave][0]);
  __builtin_amdgcn_wave_barrier();
  // per (digit, tile, wave) counts: digit-major rows of 4 * tiles
  for (int d = lane; d < kRsBins; d += 64)
    hist[((int64_t)4 * t + wave) * kRsBins + d] = cnt[wave][d];
}

// Large inputs (more than kRsScanTiles tiles): the per-digit exclusive
// prefixes of the [4 tiles][256] count table, column by column (block =
// digit, 256-row chunks scanned by wave shuffles + LDS with a running carry),
// and each digit's total - so every scatter block reads only its own four
// count rows instead of the whole table (O(tiles) instead of O(tiles^2)
// count traffic per pass).
constexpr int kRsScanTiles = 256;

__global__ __launch_bounds__(256) void rs_scan_kernel(
    const int* __restrict__ hist, int R4, int* __restrict__ pre,
    int* __restrict__ tot) {
  __shared__ int wsum[4];
  const int d = blockIdx.x, tid = threadIdx.x, lane = tid & 63,
            wave = tid >> 6;
  int carry = 0;
  for (int r0 = 0; r0 < R4; r0 += 256) {
    const int r = r0 + tid;
    const int v = r < R4 ? hist[(int64_t)r * kRsBins + d] : 0;
    int inc = v;
#pragma unroll
    for (int e = 1; e < 64; e <<= 1) {
      const int t = __shfl_up(inc, e);
      if (lane >= e) inc += t;
    }
    if (lane == 63) wsum[wave] = inc;
    __syncthreads();
    int base = carry, all = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      base += w < wave ? wsum[w] : 0;
      all += wsum[w];
    }
    if (r < R4) pre[(int64_t)r * kRsBins + d] = base + inc - v;
    carry += all;
    __syncthreads();                       // wsum reused
  }
  if (tid == 0) tot[d] = carry;
}

__global__ __launch_bounds__(256) void rs_scatter_kernel(
    const int* __restrict__ keys, const int* __restrict__ vals, int64_t n,
    int shift, const int* __restrict__ offs, int tiles,
    int* __restrict__ keys_out, int* __restrict__ vals_out,
    const int* __restrict__ spre, const int* __restrict__ stot) {
  __shared__ int cnt[4][kRsBins];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int t = blockIdx.x;
  const int64_t i0 = (int64_t)t * kRsTile + wave * kRsWave + lane;
  int kr[kRsPer], vr[kRsPer];
#pragma unroll
  for (int q = 0; q < kRsPer; ++q) {
    const int64_t i = i0 + 64 * q;
    kr[q] = keys[i < n ? i : 0];
    vr[q] = vals[i < n ? i : 0];
  }
  if (spre != nullptr) {
    // scanned table: digit totals scanned over digits, plus this tile's
    // four exclusive prefixes
    __shared__ int wtot2[4];
    const int d = tid, r0 = 4 * t;
    const int tt = stot[d];
    int inc = tt;
#pragma unroll
    for (int e = 1; e < 64; e <<= 1) {
      const int v = __shfl_up(inc, e);
      if (lane >= e) inc += v;
    }
    if (lane == 63) wtot2[wave] = inc;
    __syncthreads();
    int run = inc - tt;
    for (int w = 0; w < wave; ++w) run += wtot2[w];
#pragma unroll
    for (int w = 0; w < 4; ++w)
      cnt[w][d] = run + spre[(int64_t)(r0 + w) * kRsBins + d];
    __syncthreads();
  } else {
    // Start of digit d = tid in each of this tile's 4 waves, from the whole
    // [tiles][4][256] count table (coalesced rows, 32 loads in flight): the
    // digit's total (scanned over digits), the counts of the rows before
    // this tile, and this tile's own 4 counts.
    __shared__ int wtot[4];
    const int d = tid, R4 = 4 * tiles, r0 = 4 * t;
    int tot = 0, pre = 0, own[4] = {0, 0, 0, 0};
    for (int q0 = 0; q0 < R4; q0 += kRsChunk) {
      int c[kRsChunk];
#pragma unroll
      for (int q = 0; q < kRsChunk; ++q)    // (clamped, unconditional)
        c[q] = offs[(int64_t)min(q0 + q, R4 - 1) * kRsBins + d];
#pragma unroll
      for (int q = 0; q < kRsChunk; ++q) {
        const int r = q0 + q;
        const int v = r < R4 ? c[q] : 0;
        tot += v;
        pre += r < r0 ? v : 0;
#pragma unroll
        for (int w = 0; w < 4; ++w) own[w] += r == r0 + w ? v : 0;
      }
    }
    int inc = tot;                                 // scan over digits
#pragma unroll
    for (int e = 1; e < 64; e <<= 1) {
      const int v = __shfl_up(inc, e);
      if (lane >= e) inc += v;
    }
    if (lane == 63) wtot[wave] = inc;
    __syncthreads();
    int run = inc - tot + pre;
    for (int w = 0; w < wave; ++w) run += wtot[w];
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      cnt[w][d] = run;
      run += own[w];
    }
    __syncthreads();
  }
  int* cur = &cnt[wave][0];
  const unsigned long long lt = (1ull << lane) - 1ull;
#pragma unroll
  for (int q = 0; q < kRsPer; ++q) {
    const bool ok = i0 + 64 * q < n;
    const int d = ok ? (kr[q] >> shift) & (kRsBins - 1) : -1;
    const unsigned long long m = rs_match(d) & __ballot(ok);
    const int pos = ok ? cur[d] + __popcll(m & lt) : 0;
    __builtin_amdgcn_wave_barrier();
    if (ok) {
      keys_out[pos] = kr[q];
      vals_out[pos] = vr[q];
      if ((m >> lane) == 1ull) cur[d] = pos + 1;   // digit's last lane
    }
    __builtin_amdgcn_wave_barrier();
  }
}

}  // namespace

// S_idx [B, N_s, k] int64 (targets local to each pair's N_t block) ->
// (col int32 [nnz] global targets, rowptr int32 [B N_s + 1], colptr int32
// [B N_t + 1], perm int32 [nnz] CSC -> CSR entry map (stable: row order
// inside a column), row_of int32 [nnz]).  Prep + the stable LSD radix sort
// above (3 launches per 8-bit digit: 2 digits up to 65536 columns; rocprim's
// default merge-sorts this size in ~18 launches, and forcing its onesweep
// faulted inside the captured step) + finish.
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
  const int passes = (int)((bits + 7) / 8);
  const int tiles = (int)((n + kRsTile - 1) / kRsTile);
  at::Tensor hist = at::empty({(int64_t)kRsBins * 4 * std::max(tiles, 1)},
                              i32);
  at::Tensor k2 = at::empty({n}, i32), v2 = at::empty({n}, i32);
  // (large inputs: a scanned count table, see rs_scan_kernel)
  const bool scan = tiles > kRsScanTiles;
  at::Tensor pre, tot;
  if (scan) {
    pre = at::empty({(int64_t)kRsBins * 4 * tiles}, i32);
    tot = at::empty({kRsBins}, i32);
  }
  // ping-pong so the last pass lands in keys / perm
  const int* ki = col.data_ptr<int>();
  const int* vi = iota.data_ptr<int>();
  for (int p = 0; p < passes && n > 0; ++p) {
    const bool last = p == passes - 1;
    const bool odd = ((passes - 1 - p) & 1) != 0;
    int* ko = last ? keys.data_ptr<int>()
                   : (odd ? k2.data_ptr<int>() : keys.data_ptr<int>());
    int* vo = last ? perm.data_ptr<int>()
                   : (odd ? v2.data_ptr<int>() : perm.data_ptr<int>());
    hipLaunchKernelGGL(rs_hist_kernel, dim3(tiles), dim3(256), 0, stream(), ki,
                       n, 8 * p, hist.data_ptr<int>(), tiles);
    DGMC_CHECK_LAUNCH();
    if (scan) {
      hipLaunchKernelGGL(rs_scan_kernel, dim3(kRsBins), dim3(256), 0,
                         stream(), hist.data_ptr<int>(), 4 * tiles,
                         pre.data_ptr<int>(), tot.data_ptr<int>());
      DGMC_CHECK_LAUNCH();
    }
    hipLaunchKernelGGL(rs_scatter_kernel, dim3(tiles), dim3(256), 0, stream(),
                       ki, vi, n, 8 * p, hist.data_ptr<int>(), tiles, ko, vo,
                       scan ? pre.data_ptr<int>() : nullptr,
                       scan ? tot.data_ptr<int>() : nullptr);
    DGMC_CHECK_LAUNCH();
    ki = ko;
    vi = vo;
  }
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
