// fp32 SplineConv on the (node, slot) pairs the edges actually use.
//
// Reference: /root/reference/dgmc/models/spline.py:21,49 (PyG SplineConv over
// torch_spline_conv's weighting kernels: one thread per (edge, channel),
// atomicAdd weight gradients).  Here the conv is
//
//   out = act( A (X W) + bias ),  A [N, N*S] with columns j*S + k (source
//                                  node j, B-spline slot k; root = slot S-1)
//
// and only the columns that carry an entry are ever formed: on PascalVOC
// batches 42 % of the N*S (node, slot) pairs (10.8 of 26 per node), so the
// GEMM work is 2.4x smaller than the dense X [W_0 | ... | W_25] projection.
//
//   compact plan  mark the used columns, rank them per slot (ballot scans),
//                 lay the slots out as BM-row segments of the "compact" row
//                 space p: src[p] = j, the column -> p map and A's columns
//                 re-indexed to p (4 launches, no host sync);
//   slot_gemm     Y[p] = X[src[p]] W_{slot(p)}  - a segmented gathered GEMM on
//                 v_mfma_f32_32x32x2_f32 (exact fp32: a k-ordered fmaf chain),
//                 128x128 tiles, every tile inside one slot segment;
//   (SpMM)        out = A_c Y + bias, ReLU (spmm.hip, A_c = re-indexed A);
//   backward      dY_c = A_c^T g' (rowmap SpMM over the assembled A^T),
//                 dX = sum_k (dY_c W_k^T)[p(j,k)] (slot_gemm with W^T, then a
//                 per-node gather-sum), dW_k = sum_p X[src p]^T dY_c[p]
//                 (gathered TN MFMA over slot segments, fixed-order fold -
//                 deterministic, no atomics).
//
// LDS layouts are chosen so every MFMA operand read (one fp32 per lane) is
// bank-conflict free: k-contiguous tiles use a pitch of BK + 1 (33 dwords:
// lanes of consecutive rows step 33 banks), m/n-contiguous tiles a pitch of
// BN + 32 (the two lane halves read rows k and k + 1 on disjoint banks).
#include "common.h"

namespace dgmc {

namespace {

typedef float sg_f32x16 __attribute__((ext_vector_type(16)));
typedef float sg_f32x4 __attribute__((ext_vector_type(4)));

constexpr int kSgBM = 128;               // compact rows per tile
constexpr int kSgSeg = 256;              // slot segment alignment (the bf16x6
                                         // kernels' 256-row tiles)
constexpr int kSgBN = 128;
constexpr int kSgBK = 32;
constexpr int kSgThreads = 256;          // 4 waves, 2 x 2 wave grid of 64x64
constexpr int kSgKP = kSgBK + 1;         // pitch of k-contiguous LDS tiles
constexpr int kSgNP = kSgBN + 32;        // pitch of m/n-contiguous LDS tiles
constexpr int kSgMaxS = 64;
constexpr int kSgMaxU = 16;              // uses per wgrad launch

__device__ __forceinline__ float4 ld4(const float* p) {
  return *reinterpret_cast<const float4*>(p);
}

// Slot of compact row m (segments [seg[s], seg[s+1]) are BM-aligned).
__device__ __forceinline__ int seg_slot(const int* __restrict__ seg, int S,
                                        int m) {
  int s = 0;
  while (s < S - 1 && seg[s + 1] <= m) ++s;
  return s;
}

// XCD-local row groups of the compact row space: the rows of every slot
// segment are ordered by source node, so the x-th eighth of each segment
// covers (about) the x-th eighth of the nodes; work dispatched to XCD x
// (block id % 8, round-robin dispatch) takes those rows of every slot, and
// the node rows it gathers (X at the sources, g' at their neighbours) stay
// within one eighth of the graph batch - XCD x's L2 (rowmap SpMM 40 -> 25
// us per psi_2 call).  Units are `unit` rows (a multiple dividing every
// segment length); returns the first row of XCD x's i-th unit (-1 past the
// end) and, in *total, XCD x's unit count.  Wave-wide: lane s holds slot
// s's count, an inclusive shuffle scan locates the slot (no serial loop).
__device__ __forceinline__ int sg_xcd_unit(const int* __restrict__ seg, int S,
                                           int x, int i, int unit,
                                           int* total = nullptr) {
  const int lane = threadIdx.x & 63;
  const int sv = lane <= S ? seg[lane] : 0;
  const int sn = __shfl_down(sv, 1);
  int lo = 0, cnt = 0;
  if (lane < S) {
    const int q = (sn - sv) / unit;
    lo = q * x / kNumXcd;
    cnt = q * (x + 1) / kNumXcd - lo;
  }
  int incl = cnt;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int v = __shfl_up(incl, o);
    if (lane >= o) incl += v;
  }
  if (total != nullptr) *total = __shfl(incl, S - 1);
  const unsigned long long hit = __ballot(lane < S && incl > i);
  if (hit == 0ull) return -1;
  const int sl = __ffsll((long long)hit) - 1;
  const int base = __shfl(sv, sl), first = __shfl(lo, sl),
            before = __shfl(incl - cnt, sl);
  return base + (first + i - before) * unit;
}

__device__ __forceinline__ const float* slot_weight(const float* weight,
                                                    const float* root,
                                                    int nw, int s,
                                                    size_t stride) {
  return s < nw ? weight + (size_t)s * stride : root;
}

int num_cus(int dev) {
  static int cached[64] = {0};
  if (dev < 0 || dev >= 64) dev = 0;
  if (cached[dev] == 0) {
    hipDeviceProp_t prop;
    DGMC_CHECK_HIP(hipGetDeviceProperties(&prop, dev));
    cached[dev] = prop.multiProcessorCount;
  }
  return usable_cus(cached[dev]);
}

}  // namespace

// ---------------------------------------------------------------------------
// Compact plan
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void sg_mark_kernel(
    const int* __restrict__ rowptr, int R, const int* __restrict__ col,
    int cap, int* __restrict__ mark) {
  const int nnz = rowptr[R];
  for (int e = blockIdx.x * 256 + threadIdx.x; e < min(cap, nnz);
       e += gridDim.x * 256)
    mark[col[e]] = 1;          // same value from every writer
}

// One block per slot: rank[j*S+k] = rank of j among the used sources of slot
// k (-1 if unused); cnt[k] = used count.  Rounds of 1024 x 16 sources: each
// thread loads its 16 consecutive marks in one round (clamped addresses),
// then a shuffle scan per wave and the 16 wave totals through LDS - two
// barriers per round instead of four per 1024 sources.
constexpr int kSgScanPer = 16;
__global__ __launch_bounds__(1024) void sg_scan_kernel(
    const int* __restrict__ mark, int Nsrc, int S, int* __restrict__ rank,
    int* __restrict__ cnt) {
  __shared__ int wtot[16];
  const int k = blockIdx.x, tid = threadIdx.x, lane = tid & 63,
            wave = tid >> 6;
  int base = 0;
  for (int j0 = 0; j0 < Nsrc; j0 += 1024 * kSgScanPer) {
    const int jt = j0 + tid * kSgScanPer;
    int v[kSgScanPer];
    int s = 0;
#pragma unroll
    for (int e = 0; e < kSgScanPer; ++e) {
      const int j = min(jt + e, Nsrc - 1);
      const int m = mark[(size_t)j * S + k];
      v[e] = (jt + e < Nsrc && m != 0) ? 1 : 0;
      s += v[e];
    }
    int inc = s;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int t = __shfl_up(inc, d);
      if (lane >= d) inc += t;
    }
    if (lane == 63) wtot[wave] = inc;
    __syncthreads();
    int off = base + inc - s, all = 0;
#pragma unroll
    for (int w = 0; w < 16; ++w) {
      const int t = wtot[w];
      off += w < wave ? t : 0;
      all += t;
    }
#pragma unroll
    for (int e = 0; e < kSgScanPer; ++e) {
      if (jt + e < Nsrc) rank[(size_t)(jt + e) * S + k] = v[e] ? off : -1;
      off += v[e];
    }
    base += all;
    __syncthreads();                     // wtot reused next round
  }
  if (tid == 0) cnt[k] = base;
}

// posmap / src / cinv over the column space, col_c over the entries, seg;
// src / cinv of the compact rows no source fills (segment padding, rows past
// the last segment) are set to -1 here as well (no separate fill launches).
__global__ __launch_bounds__(256) void sg_fill_kernel(
    const int* __restrict__ rank, const int* __restrict__ cnt, int Nsrc,
    int S, const int* __restrict__ rowptr, int R, const int* __restrict__ col,
    int cap, int P_cap, int* __restrict__ posmap, int* __restrict__ src,
    int* __restrict__ cinv, int* __restrict__ col_c, int* __restrict__ seg) {
  __shared__ int sseg[kSgMaxS + 1], scnt[kSgMaxS];
  if (threadIdx.x == 0) {
    int run = 0;
    for (int k = 0; k < S; ++k) {
      sseg[k] = run;
      scnt[k] = cnt[k];
      run += (cnt[k] + kSgSeg - 1) / kSgSeg * kSgSeg;
    }
    sseg[S] = run;
  }
  __syncthreads();
  {
    const int p = blockIdx.x * 256 + threadIdx.x;
    if (p < P_cap) {
      int k = 0;
      while (k < S && sseg[k + 1] <= p) ++k;
      if (k == S || p >= sseg[k] + scnt[k]) {
        src[p] = -1;
        cinv[p] = -1;
      }
    }
  }
  if (blockIdx.x == 0)
    for (int k = threadIdx.x; k <= S; k += 256) seg[k] = sseg[k];
  const int ncols = Nsrc * S;
  const int nnz = min(cap, rowptr[R]);
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < ncols) {
    const int r = rank[i];
    const int j = i / S, k = i - j * S;
    if (r >= 0) {
      const int p = sseg[k] + r;
      posmap[i] = p;
      src[p] = j;
      cinv[p] = i;
    } else {
      posmap[i] = -1;
    }
  }
  if (i < cap) {
    if (i < nnz) {
      const int c = col[i];
      const int k = c % S;
      col_c[i] = sseg[k] + rank[c];
    } else {
      col_c[i] = 0;            // inert tail entry (val 0 in static operators)
    }
  }
}

std::vector<at::Tensor> slot_compact_plan(const at::Tensor& rowptr,
                                          const at::Tensor& col, int64_t Nsrc,
                                          int64_t S, int64_t P_cap) {
  TORCH_CHECK(rowptr.is_cuda() && rowptr.scalar_type() == at::kInt &&
                  col.scalar_type() == at::kInt,
              "slot_compact_plan: int32 CSR expected");
  TORCH_CHECK(S >= 1 && S <= kSgMaxS, "slot_compact_plan: 1 <= S <= 64");
  TORCH_CHECK(P_cap % kSgSeg == 0, "slot_compact_plan: P_cap % 256");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(rowptr.device());
  const int R = (int)rowptr.numel() - 1;
  const int cap = (int)col.numel();
  const int64_t ncols = Nsrc * S;
  auto i32 = rowptr.options();
  at::Tensor mark = at::zeros({ncols}, i32);
  at::Tensor rank = at::empty({ncols}, i32);
  at::Tensor cnt = at::empty({S}, i32);
  at::Tensor posmap = at::empty({ncols}, i32);
  at::Tensor src = at::empty({P_cap}, i32);     // (padding: sg_fill_kernel)
  at::Tensor cinv = at::empty({P_cap}, i32);
  at::Tensor col_c = at::empty({cap}, i32);
  at::Tensor seg = at::empty({S + 1}, i32);
  if (cap > 0) {
    const int blocks = std::min((cap + 255) / 256, 4096);
    hipLaunchKernelGGL(sg_mark_kernel, dim3(blocks), dim3(256), 0, stream(),
                       rowptr.data_ptr<int>(), R, col.data_ptr<int>(), cap,
                       mark.data_ptr<int>());
    DGMC_CHECK_LAUNCH();
  }
  hipLaunchKernelGGL(sg_scan_kernel, dim3(S), dim3(1024), 0, stream(),
                     mark.data_ptr<int>(), (int)Nsrc, (int)S,
                     rank.data_ptr<int>(), cnt.data_ptr<int>());
  DGMC_CHECK_LAUNCH();
  const int64_t span = std::max<int64_t>(std::max<int64_t>(ncols, cap), P_cap);
  hipLaunchKernelGGL(sg_fill_kernel, dim3((span + 255) / 256), dim3(256), 0,
                     stream(), rank.data_ptr<int>(), cnt.data_ptr<int>(),
                     (int)Nsrc, (int)S, rowptr.data_ptr<int>(), R,
                     col.data_ptr<int>(), cap, (int)P_cap,
                     posmap.data_ptr<int>(),
                     src.data_ptr<int>(), cinv.data_ptr<int>(),
                     col_c.data_ptr<int>(), seg.data_ptr<int>());
  DGMC_CHECK_LAUNCH();
  return {src, seg, col_c, posmap, cinv, cnt};
}

// ---------------------------------------------------------------------------
// Segmented gathered GEMM (NN):  Y[m, :] = A_m W_{slot(m)}  with
//   TRANS_W = false: A_m = X[src[m], :K] (zero row if src < 0), W_s [K, Nn]
//   TRANS_W = true : A_m = X[m, :K] (dX pass: X = dY_c), B = W_s^T,
//                    W_s stored [Nn, K] (the forward's [in, out] weight).
// Persistent: each workgroup walks 128x128 output tiles (grid stride) as ONE
// stream of 32-deep k-chunks, so the next tile's first chunk (and, one tile
// ahead, its gather indices) is in flight while the current tile finishes -
// psi_2's K = 128 has only 4 chunks per tile, and a per-tile prologue of two
// dependent global round trips otherwise dominates.
// ---------------------------------------------------------------------------
template <bool TRANS_W>
__global__ __launch_bounds__(kSgThreads, 2) void slot_gemm_kernel(
    const float* __restrict__ X, const int* __restrict__ src,
    const int* __restrict__ seg, int S, const float* __restrict__ weight,
    const float* __restrict__ root, int nw, int K, int Nn,
    const int* __restrict__ tlist, int tcap, float* __restrict__ Y) {
  __shared__ float As[kSgBM * kSgKP];
  __shared__ float Bs[TRANS_W ? kSgBN * kSgKP : kSgBK * kSgNP];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  const int ntn = Nn / kSgBN, nk = K / kSgBK;
  // Active output tiles: every row tile of the slot segments, or the row
  // tiles listed in tlist (count at tlist[tcap]; dX of the rows a caller
  // needs, slot_dx_tiles).
  const int U = (tlist ? tlist[tcap] : seg[S] / kSgBM) * ntn;
  auto rtile = [&](int uu) { return tlist ? tlist[uu / ntn] : uu / ntn; };
  const int G = gridDim.x;
  int u = xcd_remap(blockIdx.x, G);
  if (u >= U) return;

  // This thread's A slots: rows (tid >> 3) + 32 i, k-quad (tid & 7).
  const int c4 = (tid & 7) * 4;
  auto rows_of = [&](int uu, int (&rr)[4]) {
    const int m0 = rtile(uu) * kSgBM;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + (tid >> 3) + 32 * i;
      rr[i] = TRANS_W ? m : src[m];
    }
  };
  auto wptr = [&](int uu) {
    const int s = seg_slot(seg, S, rtile(uu) * kSgBM);
    return slot_weight(weight, root, nw, s, (size_t)K * Nn);
  };
  int rcur[4], rnext[4];
  rows_of(u, rcur);
  const float* W = wptr(u);
  int n0 = (u % ntn) * kSgBN;
  int un = u + G;
  const float* Wn = W;
  if (un < U) {
    rows_of(un, rnext);
    Wn = wptr(un);
  }

  float4 ra[4], rb[4];
  auto load = [&](const int (&rr)[4], const float* Wt, int nn0, int kc) {
    const int k0 = kc * kSgBK;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = rr[i];
      const float4 v = ld4(X + (size_t)(r < 0 ? 0 : r) * K + k0 + c4);
      ra[i] = r < 0 ? make_float4(0.f, 0.f, 0.f, 0.f) : v;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int idx = tid + kSgThreads * i;
      if (TRANS_W) {
        // B(k, n) = W[n0 + n][k0 + k]: 128 n-rows x 32 k.
        rb[i] = ld4(Wt + (size_t)(nn0 + (idx >> 3)) * K + k0 + (idx & 7) * 4);
      } else {
        // B(k, n) = W[k0 + k][n0 + n]: 32 k-rows x 128 n.
        rb[i] =
            ld4(Wt + (size_t)(k0 + (idx >> 5)) * Nn + nn0 + (idx & 31) * 4);
      }
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int idx = tid + kSgThreads * i;
      float* a = As + ((tid >> 3) + 32 * i) * kSgKP + c4;
      a[0] = ra[i].x; a[1] = ra[i].y; a[2] = ra[i].z; a[3] = ra[i].w;
      if (TRANS_W) {
        float* b = Bs + (idx >> 3) * kSgKP + (idx & 7) * 4;
        b[0] = rb[i].x; b[1] = rb[i].y; b[2] = rb[i].z; b[3] = rb[i].w;
      } else {
        *reinterpret_cast<float4*>(Bs + (idx >> 5) * kSgNP + (idx & 31) * 4) =
            rb[i];
      }
    }
  };

  sg_f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  const int l32 = lane & 31, h = lane >> 5;
  load(rcur, W, n0, 0);
  int kc = 0;
  while (true) {
    store();
    __syncthreads();
    const bool last = kc + 1 == nk;
    if (!last) load(rcur, W, n0, kc + 1);
    else if (un < U) load(rnext, Wn, (un % ntn) * kSgBN, 0);
#pragma unroll
    for (int st = 0; st < kSgBK / 2; ++st) {
      const int kk = 2 * st + h;
      float av[2], bv[2];
#pragma unroll
      for (int a = 0; a < 2; ++a)
        av[a] = As[(wm * 64 + a * 32 + l32) * kSgKP + kk];
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int n = wn * 64 + b * 32 + l32;
        bv[b] = TRANS_W ? Bs[n * kSgKP + kk] : Bs[kk * kSgNP + n];
      }
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[a], bv[b],
                                                           acc[a][b], 0, 0, 0);
    }
    __syncthreads();
    if (!last) {
      ++kc;
      continue;
    }
    // C/D: col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 h.
    const int m0 = rtile(u) * kSgBM;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = wm * 64 + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
          const int c = wn * 64 + b * 32 + l32;
          Y[(size_t)(m0 + row) * Nn + n0 + c] = acc[a][b][r];
          acc[a][b][r] = 0.f;
        }
    if (un >= U) break;
    u = un;
    n0 = (u % ntn) * kSgBN;
    W = Wn;
#pragma unroll
    for (int i = 0; i < 4; ++i) rcur[i] = rnext[i];
    kc = 0;
    un = u + G;
    if (un < U) {
      rows_of(un, rnext);
      Wn = wptr(un);
    }
  }
}

at::Tensor slot_gemm(const at::Tensor& X, const at::Tensor& src,
                     const at::Tensor& seg, const at::Tensor& weight,
                     const c10::optional<at::Tensor>& root, bool trans_w,
                     const c10::optional<at::Tensor>& tiles) {
  TORCH_CHECK(X.is_cuda() && X.scalar_type() == at::kFloat &&
                  X.is_contiguous() && X.dim() == 2,
              "slot_gemm: contiguous fp32 X");
  TORCH_CHECK(weight.scalar_type() == at::kFloat && weight.is_contiguous() &&
                  weight.dim() == 3,
              "slot_gemm: fp32 weight [K, in, out]");
  const int64_t S = seg.numel() - 1;
  const int64_t nw = weight.size(0);
  const int64_t in = weight.size(1), out = weight.size(2);
  const bool has_root = root.has_value() && root->defined();
  TORCH_CHECK(S == nw + (has_root ? 1 : 0) && S <= kSgMaxS,
              "slot_gemm: slots = weight slots + root");
  if (has_root)
    TORCH_CHECK(root->scalar_type() == at::kFloat && root->is_contiguous() &&
                    root->size(0) == in && root->size(1) == out,
                "slot_gemm: root [in, out]");
  TORCH_CHECK(in % kSgBN == 0 && out % kSgBN == 0,
              "slot_gemm: in/out multiples of 128");
  const int64_t K = trans_w ? out : in;
  const int64_t Nn = trans_w ? in : out;
  TORCH_CHECK(X.size(1) == K && aligned16(X.data_ptr()), "slot_gemm: X [*, K]");
  const int64_t P = src.numel();
  TORCH_CHECK(P % kSgBM == 0 && src.scalar_type() == at::kInt,
              "slot_gemm: src [P_cap % 128]");
  if (trans_w) TORCH_CHECK(X.size(0) == P, "slot_gemm: dY_c rows == P_cap");
  const bool listed = tiles.has_value() && tiles->defined();
  if (listed)
    TORCH_CHECK(tiles->scalar_type() == at::kInt &&
                    tiles->numel() == P / kSgBM + 1,
                "slot_gemm: tile list [P_cap / 128 + 1] (count last)");
  const int* tl = listed ? tiles->data_ptr<int>() : nullptr;
  const int tcap = (int)(P / kSgBM);
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(X.device());
  at::Tensor Y = at::empty({P, Nn}, X.options());
  // Persistent grid: 2 resident workgroups per CU (VGPR-limited; measured
  // with 1 / 2 / 3 per CU: psi_2 70.8 / 56.6 / 74.7 us, the third one only
  // starts when others finish - tools/bench_slot_gemm.py).
  const int64_t blocks = std::min<int64_t>(
      (P / kSgBM) * (Nn / kSgBN), 2 * (int64_t)num_cus(X.device().index()));
  if (blocks == 0) return Y;
  const float* rp = has_root ? root->data_ptr<float>() : nullptr;
  if (trans_w)
    hipLaunchKernelGGL(slot_gemm_kernel<true>, dim3(blocks), dim3(kSgThreads),
                       0, stream(), X.data_ptr<float>(), src.data_ptr<int>(),
                       seg.data_ptr<int>(), (int)S, weight.data_ptr<float>(),
                       rp, (int)nw, (int)K, (int)Nn, tl, tcap,
                       Y.data_ptr<float>());
  else
    hipLaunchKernelGGL(slot_gemm_kernel<false>, dim3(blocks),
                       dim3(kSgThreads), 0, stream(), X.data_ptr<float>(),
                       src.data_ptr<int>(), seg.data_ptr<int>(), (int)S,
                       weight.data_ptr<float>(), rp, (int)nw, (int)K, (int)Nn,
                       tl, tcap, Y.data_ptr<float>());
  DGMC_CHECK_LAUNCH();
  return Y;
}

// Row tiles of the dX pass that hold sources j >= row0.  Slot k's compact
// rows list its used sources in ascending j, then padding (src -1), so its
// first row with src >= row0 is found by a 64-ary search of src over the
// segment - one probe per lane and round, <= 3 rounds up to 262k rows -
// instead of a serial walk over the sources.  One wave per slot; the tiles
// from that row's tile to the segment end are listed in slot order;
// out[tcap] = count.
__global__ __launch_bounds__(1024) void sg_dx_tiles_kernel(
    const int* __restrict__ src, const int* __restrict__ seg, int S,
    int row0, int tcap, int unit, int* __restrict__ out) {
  __shared__ int sfirst[kSgMaxS], scnt[kSgMaxS], sbase[kSgMaxS];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int k = wave; k < S; k += 16) {
    const int a = seg[k], b = seg[k + 1];
    // first p in [a, b] with p == b, src[p] >= row0 or src[p] < 0
    // (monotone over the segment)
    int lo = a, hi = b;
    while (lo < hi) {
      const int step = (hi - lo + 63) / 64;
      const int q = lo + lane * step;
      bool ok = true;
      if (q < hi) {
        const int v = src[q];
        ok = v >= row0 || v < 0;
      }
      const unsigned long long m = __ballot(ok);
      if (m == 0ull) {
        lo += 63 * step + 1;
        continue;
      }
      const int f = __ffsll((long long)m) - 1;
      if (f == 0) {
        hi = lo;
      } else {
        hi = min(lo + f * step, hi);
        lo = lo + (f - 1) * step + 1;
      }
    }
    // a padding row: no used source >= row0 in this slot
    const int p = (lo < b && src[lo] < 0) ? b : lo;
    int first = p / unit;
    const int last = b / unit;
    if (first > last) first = last;
    if (lane == 0) {
      sfirst[k] = first;
      scnt[k] = last - first;
    }
  }
  __syncthreads();
  if (wave == 0) {
    const int n = lane < S ? scnt[lane] : 0;
    int incl = n;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int v = __shfl_up(incl, o);
      if (lane >= o) incl += v;
    }
    if (lane < S) sbase[lane] = incl - n;
    if (lane == 63) out[tcap] = min(incl, tcap);
  }
  __syncthreads();
  for (int k = 0; k < S; ++k) {
    const int base = sbase[k], first = sfirst[k];
    for (int t = threadIdx.x; t < scnt[k] && base + t < tcap; t += 1024)
      out[base + t] = first + t;
  }
}

at::Tensor slot_dx_tiles(const at::Tensor& src, const at::Tensor& seg,
                         int64_t N, int64_t row0, int64_t P_cap,
                         int64_t unit) {
  TORCH_CHECK(src.is_cuda() && src.scalar_type() == at::kInt &&
                  seg.scalar_type() == at::kInt && src.is_contiguous(),
              "slot_dx_tiles: int32 plan");
  const int64_t S = seg.numel() - 1;
  TORCH_CHECK(S <= kSgMaxS && src.numel() == P_cap && (unit == 128 ||
              unit == 256) && P_cap % unit == 0,
              "slot_dx_tiles: plan shapes (src [P_cap]), unit 128 / 256");
  (void)N;
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(src.device());
  const int64_t tcap = P_cap / unit;
  at::Tensor out = at::empty({tcap + 1}, src.options());
  hipLaunchKernelGGL(sg_dx_tiles_kernel, dim3(1), dim3(1024), 0, stream(),
                     src.data_ptr<int>(), seg.data_ptr<int>(), (int)S,
                     (int)row0, (int)tcap, (int)unit, out.data_ptr<int>());
  DGMC_CHECK_LAUNCH();
  return out;
}

// ---------------------------------------------------------------------------
// Slot GEMM v2 (LDS-DMA, double-buffered, transposed output fragments):
//
//   Y[m, :] = A_m Bt_s^T,  Bt_s [Nn, K] k-contiguous (forward: the W^T images
//   of slot_weight_t; dX: the [in, out] weight itself), A_m = X[src[m]] when
//   GATHER else X[m].
//
// * both operand tiles are [128 rows][32 k] fp32 (128-B rows) staged global
//   -> LDS with global_load_lds (16 B per lane, no VGPR round trip); lane l of
//   a wave's 8-row piece fetches logical quad (l & 7) ^ swz(row) of its row,
//   swz(row) = (row >> 1) & 7, so the fragment reads below are conflict-free;
// * two buffers per operand (separate LDS objects, the loop unrolled by two):
//   chunk c + 1 lands while chunk c is multiplied;
// * each lane reads float4 fragments (4 consecutive k of one row: one
//   ds_read_b128 per operand block feeds 4 MFMA steps; MFMA step t pairs
//   k = 8g + t (lanes 0-31) with k = 8g + 4 + t (lanes 32-63) on both
//   operands);
// * the weights are the MFMA A operand and the rows the B operand, so the
//   32x32 accumulator holds Y^T: a lane owns one output row and 4 consecutive
//   columns per register quad - the epilogue is 16 float4 stores per lane.
// ---------------------------------------------------------------------------
constexpr int kG2BK = 32;
constexpr int kG2Tile = kSgBM * kG2BK;       // floats per operand buffer

typedef const void __attribute__((address_space(1)))* sg_gptr;

// One 16-byte-per-lane global -> LDS copy (global_load_lds_dwordx4; the LDS
// destination is M0 + 16 * lane).  Issued as inline asm so the compiler does
// not track it as an LDS write: its own alias model would otherwise drain
// vmcnt before every fragment read of the other buffer.  The kernel counts
// these loads itself (s_waitcnt vmcnt before each raw barrier).
__device__ __forceinline__ void sg_dma16(const float* g, DGMC_LDS float* l) {
  const unsigned m0 = __builtin_amdgcn_readfirstlane(
      (unsigned)(uintptr_t)l);
  asm volatile(
      "s_mov_b32 m0, %1\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %0, off"
      :: "v"(g), "s"(m0) : "memory", "m0");
}

// s_barrier without __syncthreads' workgroup fence (which drains vmcnt and
// would serialise the next chunk's LDS-DMA with this chunk's MFMAs); the
// empty asm statements keep the compiler from moving memory ops across it.
__device__ __forceinline__ void sg_raw_barrier() {
  // (drains this wave's LDS reads: see slot_gemm_x6.hip::x6_barrier)
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <bool GATHER>
__global__ __launch_bounds__(kSgThreads, 2) void slot_gemm2_kernel(
    const float* __restrict__ X, const int* __restrict__ src,
    const int* __restrict__ seg, int S, const float* __restrict__ bt,
    const float* __restrict__ broot, int nb, int K, int Nn,
    float* __restrict__ Y) {
  __shared__ __attribute__((aligned(16))) float sA0_[kG2Tile];
  __shared__ __attribute__((aligned(16))) float sA1_[kG2Tile];
  __shared__ __attribute__((aligned(16))) float sB0_[kG2Tile];
  __shared__ __attribute__((aligned(16))) float sB1_[kG2Tile];
  DGMC_LDS float* sA0 = (DGMC_LDS float*)sA0_;
  DGMC_LDS float* sA1 = (DGMC_LDS float*)sA1_;
  DGMC_LDS float* sB0 = (DGMC_LDS float*)sB0_;
  DGMC_LDS float* sB1 = (DGMC_LDS float*)sB1_;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave & 1, wm = wave >> 1;
  const int ntn = Nn / kSgBN, nk = K / kG2BK;
  // Segment starts in lane registers: slot(m) = #{1 <= s < S: seg[s] <= m}.
  const int segv = lane <= S ? seg[lane] : 0x7fffffff;
  const int U = (__builtin_amdgcn_readlane(segv, S) / kSgBM) * ntn;
  auto slot_of = [&](int m) {
    return __popcll(__ballot(lane >= 1 && lane < S && segv <= m));
  };
  const int G = gridDim.x;
  int u = xcd_remap(blockIdx.x, G);
  if (u >= U) return;

  // Staging: this lane's 4 rows (32 wave + 8 j + lane / 8) and the physical
  // -> logical quad map of each.
  const int prow = lane >> 3;
  int sq[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int row = 32 * wave + 8 * j + prow;
    sq[j] = 4 * ((lane & 7) ^ ((row >> 1) & 7));
  }
  // Gather indices of a tile's staged rows (loaded one tile ahead).
  auto load_idx = [&](int uu, int (&ix)[4]) {
    const int m0 = (uu / ntn) * kSgBM + 32 * wave + prow;
#pragma unroll
    for (int j = 0; j < 4; ++j) ix[j] = GATHER ? src[m0 + 8 * j] : m0 + 8 * j;
  };
  const float* arow[4];
  const float* brow;            // this lane's B row of piece 0 (+ 8 j rows)
  auto tile_ptrs = [&](int uu, const int (&ix)[4]) {
    const int m0 = (uu / ntn) * kSgBM;
    const int n0 = (uu % ntn) * kSgBN;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = ix[j] < 0 ? 0 : ix[j];   // padding rows: never read
      arow[j] = X + (size_t)r * K;
    }
    const int s = slot_of(m0);
    const float* b = s < nb ? bt + (size_t)s * Nn * K : broot;
    brow = b + (size_t)(n0 + 32 * wave + prow) * K;
  };
  auto stage = [&](int kc, DGMC_LDS float* da, DGMC_LDS float* db) {
    const int k0 = kc * kG2BK;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      sg_dma16(arow[j] + k0 + sq[j], da + (32 * wave + 8 * j) * kG2BK);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      sg_dma16(brow + (size_t)8 * j * K + k0 + sq[j],
               db + (32 * wave + 8 * j) * kG2BK);
  };

  // Fragment offsets (floats): row (wave block + 32 a + i), quad (2g+h)^sw.
  const int i = lane & 31, h = lane >> 5, sw = (i >> 1) & 7;
  int qoff[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) qoff[g] = 4 * ((2 * g + h) ^ sw);
  const int offN = (wn * 64 + i) * kG2BK;    // + 32 a rows
  const int offM = (wm * 64 + i) * kG2BK;    // + 32 b rows

  sg_f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  // Fragments double-buffered in registers: group g + 1's four float4
  // reads are interleaved with group g's 16 MFMAs (one read after every
  // four MFMAs), so no MFMA waits on a fragment read.
  auto compute = [&](const DGMC_LDS float* la, const DGMC_LDS float* lb) {
    sg_f32x4 fa[2][2], fb[2][2];
    auto frag = [&](int g, int st) {
#pragma unroll
      for (int a = 0; a < 2; ++a)
        fa[st][a] = *reinterpret_cast<const DGMC_LDS sg_f32x4*>(
            lb + offN + a * 32 * kG2BK + qoff[g]);
#pragma unroll
      for (int b = 0; b < 2; ++b)
        fb[st][b] = *reinterpret_cast<const DGMC_LDS sg_f32x4*>(
            la + offM + b * 32 * kG2BK + qoff[g]);
    };
    frag(0, 0);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int st = g & 1;
      if (g < 3) frag(g + 1, st ^ 1);
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int b = 0; b < 2; ++b)
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(
                fa[st][a][t], fb[st][b][t], acc[a][b], 0, 0, 0);
    }
    // Issue order: group 0's reads, then per group 4 x (2 MFMA, 1 read) +
    // 8 MFMA while a next group exists (its reads land >= 8 MFMAs before
    // use), then the last group's 16 MFMAs.
    __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
#pragma unroll
    for (int g = 0; g < 3; ++g) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 16, 0);
  };
  auto epilogue = [&](int uu) {
    const int m0 = (uu / ntn) * kSgBM + wm * 64 + i;
    const int n0 = (uu % ntn) * kSgBN + wn * 64 + 4 * h;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        float* yrow = Y + (size_t)(m0 + 32 * b) * Nn + n0 + 32 * a;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          *reinterpret_cast<float4*>(yrow + 8 * q) =
              make_float4(acc[a][b][4 * q], acc[a][b][4 * q + 1],
                          acc[a][b][4 * q + 2], acc[a][b][4 * q + 3]);
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[a][b][4 * q + r] = 0.f;
        }
      }
  };

  // One stream of (tile, chunk) work items: (u, kc) is multiplied while the
  // item after it is staged into the other buffer.  The next tile's gather
  // indices are loaded while the current tile's chunk 1 is staged (nk >= 4),
  // so they have landed long before that tile's chunk 0 is staged.
  int inext[4];
  {
    int icur[4];
    load_idx(u, icur);
    tile_ptrs(u, icur);
  }
  stage(0, sA0, sB0);
  int kc = 0;
  auto step = [&](DGMC_LDS float* ca, DGMC_LDS float* cb, DGMC_LDS float* na,
                  DGMC_LDS float* nbuf) -> bool {
    // Item after (u, kc).
    const bool last_chunk = kc + 1 == nk;
    const int tu = last_chunk ? u + G : u;
    const int tkc = last_chunk ? 0 : kc + 1;
    const bool more = tu < U;
    if (more) {
      if (last_chunk) tile_ptrs(tu, inext);
      else if (tkc == 1 && u + G < U) load_idx(u + G, inext);
      stage(tkc, na, nbuf);
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    sg_raw_barrier();
    compute(ca, cb);
    if (last_chunk) epilogue(u);
    sg_raw_barrier();
    u = tu;
    kc = tkc;
    return more;
  };
  while (step(sA0, sB0, sA1, sB1) && step(sA1, sB1, sA0, sB0)) {
  }
}

at::Tensor slot_gemm2(const at::Tensor& X, const at::Tensor& src,
                      const at::Tensor& seg, const at::Tensor& bt,
                      const c10::optional<at::Tensor>& broot, bool gather) {
  TORCH_CHECK(X.is_cuda() && X.scalar_type() == at::kFloat &&
                  X.is_contiguous() && X.dim() == 2 && aligned16(X.data_ptr()),
              "slot_gemm2: contiguous fp32 X");
  TORCH_CHECK(bt.scalar_type() == at::kFloat && bt.is_contiguous() &&
                  bt.dim() == 3 && aligned16(bt.data_ptr()),
              "slot_gemm2: fp32 images [S', Nn, K]");
  const int64_t S = seg.numel() - 1;
  const int64_t nb = bt.size(0), Nn = bt.size(1), K = bt.size(2);
  const bool has_root = broot.has_value() && broot->defined();
  TORCH_CHECK(S == nb + (has_root ? 1 : 0) && S <= kSgMaxS,
              "slot_gemm2: slots = images (+ root)");
  if (has_root)
    TORCH_CHECK(broot->scalar_type() == at::kFloat && broot->is_contiguous() &&
                    broot->size(0) == Nn && broot->size(1) == K &&
                    aligned16(broot->data_ptr()),
                "slot_gemm2: root image [Nn, K]");
  TORCH_CHECK(K % kSgBN == 0 && Nn % kSgBN == 0,
              "slot_gemm2: K / Nn multiples of 128");
  TORCH_CHECK(X.size(1) == K, "slot_gemm2: X [*, K]");
  const int64_t P = src.numel();
  TORCH_CHECK(P % kSgBM == 0 && src.scalar_type() == at::kInt,
              "slot_gemm2: src [P_cap % 128]");
  if (!gather) TORCH_CHECK(X.size(0) == P, "slot_gemm2: rows == P_cap");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(X.device());
  at::Tensor Y = at::empty({P, Nn}, X.options());
  // Persistent grid: one workgroup per CU for long K loops, two for K = 128
  // (tools/bench_slot_gemm.py, per CU 1 / 2: 1024->256 forward 504 / 562
  // us, 256->256 147 / 160 us, 128->128 53 / 50 us; one workgroup per tile
  // 866 / 250 / 82 us).
  const int per_cu = K >= 256 ? 1 : 2;
  const int64_t tiles = (P / kSgBM) * (Nn / kSgBN);
  const int64_t blocks =
      std::min<int64_t>(tiles, per_cu * (int64_t)num_cus(X.device().index()));
  if (blocks == 0) return Y;
  const float* rp = has_root ? broot->data_ptr<float>() : nullptr;
  auto go = [&](auto g) {
    constexpr bool GA = decltype(g)::value;
    hipLaunchKernelGGL(slot_gemm2_kernel<GA>, dim3(blocks), dim3(kSgThreads),
                       0, stream(), X.data_ptr<float>(), src.data_ptr<int>(),
                       seg.data_ptr<int>(), (int)S, bt.data_ptr<float>(), rp,
                       (int)nb, (int)K, (int)Nn, Y.data_ptr<float>());
  };
  if (gather) go(std::true_type());
  else go(std::false_type());
  DGMC_CHECK_LAUNCH();
  return Y;
}

// ---------------------------------------------------------------------------
// Dense fp32 NT GEMM on the same LDS-DMA pipeline:
//   Y[M, Nn] = [A_0 | A_1 | ...] Bt^T,  A_j [M, 128] contiguous (up to 4
//   parts read in place - psi_2's concatenated features never formed),
//   Bt [Nn, K] k-contiguous, K = 128 * parts.
// Rows past M are clamped on load and not stored.
// ---------------------------------------------------------------------------
struct DnParts {
  const float* p[4];
};

// MB / NB: 32-row blocks per wave along M / N (tile (64 MB) x (64 NB));
// 64 x 64 tiles for skinny products (the [M, 384] x [384, 128] projection
// has only M / 128 tiles of 128 x 128).
template <int MB, int NB>
__global__ __launch_bounds__(kSgThreads, 2) void dense_nt_f32_kernel(
    DnParts A, int M, const float* __restrict__ bt, int K, int Nn,
    float* __restrict__ Y) {
  constexpr int TM = 64 * MB, TN = 64 * NB;
  __shared__ __attribute__((aligned(16))) float sA0_[TM * kG2BK];
  __shared__ __attribute__((aligned(16))) float sA1_[TM * kG2BK];
  __shared__ __attribute__((aligned(16))) float sB0_[TN * kG2BK];
  __shared__ __attribute__((aligned(16))) float sB1_[TN * kG2BK];
  DGMC_LDS float* sA0 = (DGMC_LDS float*)sA0_;
  DGMC_LDS float* sA1 = (DGMC_LDS float*)sA1_;
  DGMC_LDS float* sB0 = (DGMC_LDS float*)sB0_;
  DGMC_LDS float* sB1 = (DGMC_LDS float*)sB1_;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave & 1, wm = wave >> 1;
  const int ntn = Nn / TN, nk = K / kG2BK;
  const int U = ((M + TM - 1) / TM) * ntn;
  const int G = gridDim.x;
  int u = xcd_remap(blockIdx.x, G);
  if (u >= U) return;

  // Staging: wave w's A pieces j < 2 MB cover rows (2 MB) 8 w + 8 j + lane /
  // 8, its B pieces j < 2 NB rows (2 NB) 8 w + 8 j + lane / 8.
  const int prow = lane >> 3;
  auto swz = [&](int row) { return 4 * ((lane & 7) ^ ((row >> 1) & 7)); };
  int arow[2 * MB];
  const float* brow;
  auto tile_ptrs = [&](int uu) {
    const int m0 = (uu / ntn) * TM, n0 = (uu % ntn) * TN;
#pragma unroll
    for (int j = 0; j < 2 * MB; ++j)
      arow[j] = min(m0 + 16 * MB * wave + 8 * j + prow, M - 1);
    brow = bt + (size_t)(n0 + 16 * NB * wave + prow) * K;
  };
  auto stage = [&](int kc, DGMC_LDS float* da, DGMC_LDS float* db) {
    const int k0 = kc * kG2BK;
    const float* part = A.p[k0 >> 7];
    const int kp = k0 & 127;
#pragma unroll
    for (int j = 0; j < 2 * MB; ++j) {
      const int row = 16 * MB * wave + 8 * j + prow;
      sg_dma16(part + (size_t)arow[j] * 128 + kp + swz(row),
               da + (16 * MB * wave + 8 * j) * kG2BK);
    }
#pragma unroll
    for (int j = 0; j < 2 * NB; ++j) {
      const int row = 16 * NB * wave + 8 * j + prow;
      sg_dma16(brow + (size_t)8 * j * K + k0 + swz(row),
               db + (16 * NB * wave + 8 * j) * kG2BK);
    }
  };
  const int i = lane & 31, h = lane >> 5, sw = (i >> 1) & 7;
  int qoff[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) qoff[g] = 4 * ((2 * g + h) ^ sw);
  const int offN = (wn * 32 * NB + i) * kG2BK;
  const int offM = (wm * 32 * MB + i) * kG2BK;
  sg_f32x16 acc[NB][MB];
#pragma unroll
  for (int a = 0; a < NB; ++a)
#pragma unroll
    for (int b = 0; b < MB; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  auto compute = [&](const DGMC_LDS float* la, const DGMC_LDS float* lb) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      sg_f32x4 fa[NB], fb[MB];
#pragma unroll
      for (int a = 0; a < NB; ++a)
        fa[a] = *reinterpret_cast<const DGMC_LDS sg_f32x4*>(
            lb + offN + a * 32 * kG2BK + qoff[g]);
#pragma unroll
      for (int b = 0; b < MB; ++b)
        fb[b] = *reinterpret_cast<const DGMC_LDS sg_f32x4*>(
            la + offM + b * 32 * kG2BK + qoff[g]);
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int a = 0; a < NB; ++a)
#pragma unroll
          for (int b = 0; b < MB; ++b)
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(
                fa[a][t], fb[b][t], acc[a][b], 0, 0, 0);
    }
  };
  auto epilogue = [&](int uu) {
    const int m0 = (uu / ntn) * TM + wm * 32 * MB + i;
    const int n0 = (uu % ntn) * TN + wn * 32 * NB + 4 * h;
#pragma unroll
    for (int a = 0; a < NB; ++a)
#pragma unroll
      for (int b = 0; b < MB; ++b) {
        const int m = m0 + 32 * b;
        float* yrow = Y + (size_t)m * Nn + n0 + 32 * a;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if (m < M)
            *reinterpret_cast<float4*>(yrow + 8 * q) =
                make_float4(acc[a][b][4 * q], acc[a][b][4 * q + 1],
                            acc[a][b][4 * q + 2], acc[a][b][4 * q + 3]);
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[a][b][4 * q + r] = 0.f;
        }
      }
  };
  tile_ptrs(u);
  stage(0, sA0, sB0);
  int kc = 0;
  auto step = [&](DGMC_LDS float* ca, DGMC_LDS float* cb, DGMC_LDS float* na,
                  DGMC_LDS float* nbuf) -> bool {
    const bool last_chunk = kc + 1 == nk;
    const int tu = last_chunk ? u + G : u;
    const int tkc = last_chunk ? 0 : kc + 1;
    const bool more = tu < U;
    if (more) {
      if (last_chunk) tile_ptrs(tu);
      stage(tkc, na, nbuf);
      // (this wave's 2 (MB + NB) pieces of the next chunk stay in flight)
      if constexpr (MB + NB == 4)
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else if constexpr (MB + NB == 3)
        asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    sg_raw_barrier();
    compute(ca, cb);
    if (last_chunk) epilogue(u);
    sg_raw_barrier();
    u = tu;
    kc = tkc;
    return more;
  };
  while (step(sA0, sB0, sA1, sB1) && step(sA1, sB1, sA0, sB0)) {
  }
}

at::Tensor dense_nt_f32(at::TensorList parts, const at::Tensor& bt) {
  const int64_t np = (int64_t)parts.size();
  TORCH_CHECK(np >= 1 && np <= 4, "dense_nt_f32: 1..4 parts");
  const int64_t M = parts[0].size(0);
  DnParts A{};
  for (int64_t j = 0; j < np; ++j) {
    const at::Tensor& p = parts[j];
    TORCH_CHECK(p.is_cuda() && p.scalar_type() == at::kFloat &&
                    p.is_contiguous() && p.dim() == 2 && p.size(0) == M &&
                    p.size(1) == 128 && aligned16(p.data_ptr()),
                "dense_nt_f32: parts contiguous fp32 [M, 128]");
    A.p[j] = p.data_ptr<float>();
  }
  TORCH_CHECK(bt.scalar_type() == at::kFloat && bt.is_contiguous() &&
                  bt.dim() == 2 && bt.size(1) == 128 * np &&
                  bt.size(0) % 64 == 0 && aligned16(bt.data_ptr()),
              "dense_nt_f32: Bt fp32 [Nn % 64, 128 * parts]");
  const int64_t Nn = bt.size(0), K = bt.size(1);
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(bt.device());
  at::Tensor Y = at::empty({M, Nn}, bt.options());
  if (M == 0) return Y;
  // 128 x 128 tiles when they fill the chip, else 64 x 64.
  const int cus = num_cus(bt.device().index());
  const int64_t big = ((M + 127) / 128) * (Nn / 128);
  const bool small = big < cus || Nn % 128 != 0;
  const int64_t tiles =
      small ? ((M + 63) / 64) * (Nn / 64) : big;
  const int per_cu = (small || K < 256) ? 2 : 1;     // as slot_gemm2
  const int64_t blocks = std::min<int64_t>(tiles, per_cu * (int64_t)cus);
  auto kern = small ? dense_nt_f32_kernel<1, 1> : dense_nt_f32_kernel<2, 2>;
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(kSgThreads), 0, stream(), A,
                     (int)M, bt.data_ptr<float>(), (int)K, (int)Nn,
                     Y.data_ptr<float>());
  DGMC_CHECK_LAUNCH();
  return Y;
}

// W^T images [S, out, in] of weight [S - 1 or S, in, out] (+ root [in, out]
// as the last slot): 32x32 tiles through LDS.
__global__ __launch_bounds__(256) void slot_weight_t_kernel(
    const float* __restrict__ weight, const float* __restrict__ root, int nw,
    int cin, int cout, float* __restrict__ out) {
  __shared__ float t[32][33];
  const int s = blockIdx.z;
  const float* w = s < nw ? weight + (size_t)s * cin * cout : root;
  const int i0 = blockIdx.y * 32, o0 = blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
#pragma unroll
  for (int r = 0; r < 32; r += 8)
    t[ty + r][tx] = w[(size_t)(i0 + ty + r) * cout + o0 + tx];
  __syncthreads();
  float* o = out + (size_t)s * cin * cout;
#pragma unroll
  for (int r = 0; r < 32; r += 8)
    o[(size_t)(o0 + ty + r) * cin + i0 + tx] = t[tx][ty + r];
}

at::Tensor slot_weight_t(const at::Tensor& weight,
                         const c10::optional<at::Tensor>& root) {
  TORCH_CHECK(weight.is_cuda() && weight.scalar_type() == at::kFloat &&
                  weight.is_contiguous() && weight.dim() == 3,
              "slot_weight_t: contiguous fp32 weight [K, in, out]");
  const int64_t nw = weight.size(0), cin = weight.size(1),
                cout = weight.size(2);
  const bool has_root = root.has_value() && root->defined();
  if (has_root)
    TORCH_CHECK(root->scalar_type() == at::kFloat && root->is_contiguous() &&
                    root->size(0) == cin && root->size(1) == cout,
                "slot_weight_t: root [in, out]");
  TORCH_CHECK(cin % 32 == 0 && cout % 32 == 0, "slot_weight_t: multiples of 32");
  const int64_t S = nw + (has_root ? 1 : 0);
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(weight.device());
  at::Tensor out = at::empty({S, cout, cin}, weight.options());
  hipLaunchKernelGGL(slot_weight_t_kernel, dim3(cout / 32, cin / 32, S),
                     dim3(256), 0, stream(), weight.data_ptr<float>(),
                     has_root ? root->data_ptr<float>() : nullptr, (int)nw,
                     (int)cin, (int)cout, out.data_ptr<float>());
  DGMC_CHECK_LAUNCH();
  return out;
}

// ---------------------------------------------------------------------------
// Row-mapped SpMM: out[p, :] = sum_{e in row cinv[p] of (rowptr, col, val)}
// val[e] * g[col[e], :]  (zero for cinv[p] < 0) - dY_c = A_c^T g' straight
// from the assembled A^T (rows j*S + k) without re-indexing it.
// ---------------------------------------------------------------------------
// (start, end) of every compact row's A^T entries (one int2 per row: one
// dependent load fewer than cinv -> rowptr in each rowmap SpMM of a step).
__global__ __launch_bounds__(256) void sg_rowmap_ranges_kernel(
    const int* __restrict__ rowptr, const int* __restrict__ cinv, int P,
    int2* __restrict__ out) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P) return;
  const int c = cinv[p];
  out[p] = c >= 0 ? make_int2(rowptr[c], rowptr[c + 1]) : make_int2(0, 0);
}

// Inline entry table ("ELL"), 32 bytes per compact row: {c0, c1, c2, n} and
// {v0, v1, v2, e0} (values as float bits).  Rows with n <= 3 entries (nearly
// all) need no (col, val) round after the table load; longer rows walk
// col / val from e0.
__global__ __launch_bounds__(256) void sg_rowmap_ell_kernel(
    const int* __restrict__ rowptr, const int* __restrict__ col,
    const float* __restrict__ val, const int* __restrict__ cinv, int P,
    int4* __restrict__ out) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P) return;
  const int c = cinv[p];
  const int e0 = c >= 0 ? rowptr[c] : 0, n = c >= 0 ? rowptr[c + 1] - e0 : 0;
  int cc[3] = {0, 0, 0};
  float vv[3] = {0.f, 0.f, 0.f};
  if (n <= 3) {
#pragma unroll
    for (int u = 0; u < 3; ++u)
      if (u < n) {
        cc[u] = col[e0 + u];
        vv[u] = val[e0 + u];
      }
  }
  out[2 * p] = make_int4(cc[0], cc[1], cc[2], n);
  out[2 * p + 1] = make_int4(__float_as_int(vv[0]), __float_as_int(vv[1]),
                             __float_as_int(vv[2]), e0);
}

typedef __bf16 sg_bf16x4 __attribute__((ext_vector_type(4)));

// fp32 -> three bf16 terms hi + mid + lo (round-to-nearest at each stage;
// the operand format of slot_gemm_x6.hip).
__device__ __forceinline__ void sg_split4(const float4 v, sg_bf16x4& h,
                                          sg_bf16x4& m, sg_bf16x4& l) {
  const float f[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const __bf16 he = (__bf16)f[e];
    const float r1 = f[e] - (float)he;
    const __bf16 me = (__bf16)r1;
    h[e] = he;
    m[e] = me;
    l[e] = (__bf16)(r1 - (float)me);
  }
}

template <int LPR, bool XL>
__global__ __launch_bounds__(256) void sg_spmm_rowmap_kernel(
    const int* __restrict__ rowptr, const int* __restrict__ col,
    const float* __restrict__ val, const int* __restrict__ cinv,
    const int2* __restrict__ ranges, const int4* __restrict__ ell,
    const int* __restrict__ seg, int S,
    const float* __restrict__ g, float* __restrict__ out,
    __bf16* __restrict__ out3, int P, int C) {
  constexpr int RPB = 256 / LPR;
  int p;
  if (XL) {
    const int r0 = sg_xcd_unit(seg, S, blockIdx.x % kNumXcd,
                               blockIdx.x / kNumXcd, RPB);
    if (r0 < 0) return;
    p = r0 + threadIdx.x / LPR;
  } else {
    const int blk = xcd_remap(blockIdx.x, gridDim.x);
    p = blk * RPB + threadIdx.x / LPR;
  }
  const int lane = threadIdx.x % LPR;
  // Rows past the last slot segment are never read (slot_gemm / wgrad stop
  // at seg[S]); padding rows inside segments are written as zeros.
  if (p >= P || (seg != nullptr && p >= seg[S])) return;
  int e0, e1;
  int4 ec = make_int4(0, 0, 0, 0), ev = make_int4(0, 0, 0, 0);
  bool inl = false;
  if (ell != nullptr) {
    ec = ell[2 * p];
    ev = ell[2 * p + 1];
    inl = ec.w <= 3;
    e0 = ev.w;
    e1 = inl ? e0 : e0 + ec.w;
  } else if (ranges != nullptr) {
    const int2 r = ranges[p];
    e0 = r.x;
    e1 = r.y;
  } else {
    const int c = cinv[p];
    e0 = c >= 0 ? rowptr[c] : 0;
    e1 = c >= 0 ? rowptr[c + 1] : 0;
  }
  for (int c0 = lane * 4; c0 < C; c0 += LPR * 4) {
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    if (inl) {     // entries from the table: one g round
      const int n = ec.w;
      const int cs[3] = {ec.x, ec.y, ec.z};
      const int vs[3] = {ev.x, ev.y, ev.z};
      float4 v[3];
#pragma unroll
      for (int u = 0; u < 3; ++u)
        v[u] = u < n ? ld4(g + (size_t)cs[u] * C + c0)
                     : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int u = 0; u < 3; ++u)
        if (u < n) {
          const float w = __int_as_float(vs[u]);
          acc.x = fmaf(w, v[u].x, acc.x);
          acc.y = fmaf(w, v[u].y, acc.y);
          acc.z = fmaf(w, v[u].z, acc.z);
          acc.w = fmaf(w, v[u].w, acc.w);
        }
    }
    int e = e0;
    for (; e + 4 <= e1; e += 4) {
      float4 v[4];
      float w[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        w[u] = val[e + u];
        v[u] = ld4(g + (size_t)col[e + u] * C + c0);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        acc.x = fmaf(w[u], v[u].x, acc.x);
        acc.y = fmaf(w[u], v[u].y, acc.y);
        acc.z = fmaf(w[u], v[u].z, acc.z);
        acc.w = fmaf(w[u], v[u].w, acc.w);
      }
    }
    // Remainder (most compact rows hold 1-3 entries): one predicated batch
    // - a single (col, val) then g latency round instead of one per entry.
    const int rem = e1 - e;
    if (rem > 0) {
      float w[3];
      float4 v[3];
#pragma unroll
      for (int u = 0; u < 3; ++u) {
        const bool ok = u < rem;
        const int eu = ok ? e + u : e;     // (clamped: never past the row)
        const float wv = val[eu];
        const int cv = col[eu];
        w[u] = ok ? wv : 0.f;
        v[u] = ld4(g + (size_t)(ok ? cv : 0) * C + c0);
      }
#pragma unroll
      for (int u = 0; u < 3; ++u)
        if (u < rem) {
          acc.x = fmaf(w[u], v[u].x, acc.x);
          acc.y = fmaf(w[u], v[u].y, acc.y);
          acc.z = fmaf(w[u], v[u].z, acc.z);
          acc.w = fmaf(w[u], v[u].w, acc.w);
        }
    }
    if (out3 != nullptr) {     // bf16x6 operand planes [3][P][C]
      sg_bf16x4 h, m, l;
      sg_split4(acc, h, m, l);
      const size_t o = (size_t)p * C + c0, plane = (size_t)P * C;
      *reinterpret_cast<sg_bf16x4*>(out3 + o) = h;
      *reinterpret_cast<sg_bf16x4*>(out3 + o + plane) = m;
      *reinterpret_cast<sg_bf16x4*>(out3 + o + 2 * plane) = l;
    } else {
      *reinterpret_cast<float4*>(out + (size_t)p * C + c0) = acc;
    }
  }
}

// Entry-table rowmap, RPL rows per lane group: the table loads of all RPL
// rows are issued together, then all their gathers (RPL independent
// latency chains per wave instead of one).  XCD-local row groups as above.
template <int LPR, int RPL>
__global__ __launch_bounds__(256) void sg_spmm_rowmap_ell_kernel(
    const int* __restrict__ col, const float* __restrict__ val,
    const int4* __restrict__ ell, const int* __restrict__ seg, int S,
    const float* __restrict__ g, float* __restrict__ out,
    __bf16* __restrict__ out3, int P, int C) {
  constexpr int RPB = 256 / LPR;
  const int r0 = sg_xcd_unit(seg, S, blockIdx.x % kNumXcd,
                             blockIdx.x / kNumXcd, RPB * RPL);
  if (r0 < 0) return;
  const int lane = threadIdx.x % LPR;
  const int pend = min(P, seg[S]);
  int pr[RPL];
  int4 ec[RPL], ev[RPL];
  // (table rows clamped, not predicated: a predicated load waits for its
  // own round trip; rows past pend are skipped below)
#pragma unroll
  for (int q = 0; q < RPL; ++q) {
    pr[q] = r0 + q * RPB + threadIdx.x / LPR;
    const int pc = max(min(pr[q], pend - 1), 0);
    ec[q] = ell[2 * pc];
    ev[q] = ell[2 * pc + 1];
  }
  for (int c0 = lane * 4; c0 < C; c0 += LPR * 4) {
    float4 v[RPL][3];
#pragma unroll
    for (int q = 0; q < RPL; ++q) {
      // unused table slots hold column 0: every gather is in bounds
      const int cs[3] = {ec[q].x, ec[q].y, ec[q].z};
#pragma unroll
      for (int u = 0; u < 3; ++u) v[q][u] = ld4(g + (size_t)cs[u] * C + c0);
    }
#pragma unroll
    for (int q = 0; q < RPL; ++q) {
      if (pr[q] >= pend) continue;
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
      const int n = ec[q].w;
      if (n <= 3) {
        const int vs[3] = {ev[q].x, ev[q].y, ev[q].z};
#pragma unroll
        for (int u = 0; u < 3; ++u)
          if (u < n) {
            const float w = __int_as_float(vs[u]);
            acc.x = fmaf(w, v[q][u].x, acc.x);
            acc.y = fmaf(w, v[q][u].y, acc.y);
            acc.z = fmaf(w, v[q][u].z, acc.z);
            acc.w = fmaf(w, v[q][u].w, acc.w);
          }
      } else {          // long row: walk col / val (entry order)
        for (int e = ev[q].w; e < ev[q].w + n; ++e) {
          const float w = val[e];
          const float4 x = ld4(g + (size_t)col[e] * C + c0);
          acc.x = fmaf(w, x.x, acc.x);
          acc.y = fmaf(w, x.y, acc.y);
          acc.z = fmaf(w, x.z, acc.z);
          acc.w = fmaf(w, x.w, acc.w);
        }
      }
      if (out3 != nullptr) {
        sg_bf16x4 h, m, l;
        sg_split4(acc, h, m, l);
        const size_t o = (size_t)pr[q] * C + c0, plane = (size_t)P * C;
        *reinterpret_cast<sg_bf16x4*>(out3 + o) = h;
        *reinterpret_cast<sg_bf16x4*>(out3 + o + plane) = m;
        *reinterpret_cast<sg_bf16x4*>(out3 + o + 2 * plane) = l;
      } else {
        *reinterpret_cast<float4*>(out + (size_t)pr[q] * C + c0) = acc;
      }
    }
  }
}

// Rows per lane group of the ELL rowmap SpMM (2; DGMC_ROWMAP_RPL=1 in the
// diagnostic build restores one row per group).
static int rowmap_rpl() {
  static const int v = diag_env_int("DGMC_ROWMAP_RPL", 2);
  return v;
}

at::Tensor slot_spmm_rowmap(const at::Tensor& rowptr, const at::Tensor& col,
                            const at::Tensor& val, const at::Tensor& cinv,
                            const at::Tensor& g,
                            const c10::optional<at::Tensor>& seg,
                            const c10::optional<at::Tensor>& ranges,
                            bool planes) {
  TORCH_CHECK(g.is_cuda() && g.scalar_type() == at::kFloat &&
                  g.is_contiguous() && g.dim() == 2 && g.size(1) % 4 == 0 &&
                  aligned16(g.data_ptr()),
              "slot_spmm_rowmap: contiguous fp32 g [N, C % 4]");
  TORCH_CHECK(val.scalar_type() == at::kFloat && cinv.scalar_type() == at::kInt,
              "slot_spmm_rowmap: dtypes");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(g.device());
  const int64_t P = cinv.numel(), C = g.size(1);
  at::Tensor out = planes ? at::empty({3, P, C}, g.options().dtype(at::kBFloat16))
                          : at::empty({P, C}, g.options());
  if (P == 0) return out;
  // (Rows past seg[S] are left unwritten in both formats: no consumer -
  // the GEMMs stop at seg[S], the weight gradient at its segments - reads
  // them.)
  float* op = planes ? nullptr : out.data_ptr<float>();
  __bf16* op3 = planes ? reinterpret_cast<__bf16*>(out.data_ptr()) : nullptr;
  const int* segp = nullptr;
  int S = 0;
  if (seg.has_value() && seg->defined()) {
    segp = seg->data_ptr<int>();
    S = (int)seg->numel() - 1;
  }
  const int2* rg = nullptr;
  const int4* el = nullptr;
  if (ranges.has_value() && ranges->defined()) {
    TORCH_CHECK(ranges->scalar_type() == at::kInt && ranges->is_contiguous() &&
                    (ranges->numel() == 2 * P || ranges->numel() == 8 * P),
                "slot_spmm_rowmap: int32 ranges [P, 2] or entry table [P, 8]");
    if (ranges->numel() == 8 * P)
      el = reinterpret_cast<const int4*>(ranges->data_ptr<int>());
    else
      rg = reinterpret_cast<const int2*>(ranges->data_ptr<int>());
  }
  const bool xl = segp != nullptr;      // XCD-local row groups (above)
  const int lanes = (int)(C / 4);
  const int rpl = rowmap_rpl();
  if (el != nullptr && xl && (rpl == 2 || rpl == 4) && lanes <= 64) {
    auto go2 = [&](auto lpr, auto rtag) {
      constexpr int L = decltype(lpr)::value, RP = decltype(rtag)::value;
      constexpr int RPB = 256 / L;
      const int64_t blocks = (P / (RPB * RP) / kNumXcd + S + 1) * kNumXcd;
      hipLaunchKernelGGL((sg_spmm_rowmap_ell_kernel<L, RP>), dim3(blocks),
                         dim3(256), 0, stream(), col.data_ptr<int>(),
                         val.data_ptr<float>(), el, segp, S,
                         g.data_ptr<float>(), op, op3, (int)P, (int)C);
    };
    auto pick = [&](auto rtag) {
      if (lanes <= 8) go2(std::integral_constant<int, 8>(), rtag);
      else if (lanes <= 16) go2(std::integral_constant<int, 16>(), rtag);
      else if (lanes <= 32) go2(std::integral_constant<int, 32>(), rtag);
      else go2(std::integral_constant<int, 64>(), rtag);
    };
    if (rpl == 4) pick(std::integral_constant<int, 4>());
    else pick(std::integral_constant<int, 2>());
    DGMC_CHECK_LAUNCH();
    return out;
  }
  auto go = [&](auto lpr) {
    constexpr int L = decltype(lpr)::value;
    constexpr int RPB = 256 / L;
    // XCD-local groups: every slot's eighth is a whole number of groups, so
    // per XCD at most P / RPB / 8 + S groups.
    const int64_t blocks = xl ? (P / RPB / kNumXcd + S + 1) * kNumXcd
                              : (P + RPB - 1) / RPB;
    auto kern = xl ? sg_spmm_rowmap_kernel<L, true>
                   : sg_spmm_rowmap_kernel<L, false>;
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, stream(),
                       rowptr.data_ptr<int>(), col.data_ptr<int>(),
                       val.data_ptr<float>(), cinv.data_ptr<int>(), rg, el,
                       segp,
                       S, g.data_ptr<float>(), op, op3, (int)P, (int)C);
  };
  if (lanes <= 8) go(std::integral_constant<int, 8>());
  else if (lanes <= 16) go(std::integral_constant<int, 16>());
  else if (lanes <= 32) go(std::integral_constant<int, 32>());
  else go(std::integral_constant<int, 64>());
  DGMC_CHECK_LAUNCH();
  return out;
}

// ---------------------------------------------------------------------------
// Per-node gather-sum over slots: out[j, :] = add[j, :] + sum_k Z[posmap[j*S
// + k], :]  (slot order fixed: deterministic).  dX of the slot GEMM.
//
// RB (fused ReLU / bias backward of the PRODUCING layer, whose output the
// gathered gradient belongs to): out = (relu_out > 0) ? sum : 0, and the
// bias gradient's column partials of 16-row blocks go to part[blk].  A
// block is 16 lane groups, one row each; the masked rows are stashed in LDS
// and summed in elementwise.hip::colsum_kernel<float, ..., LPR, true>'s
// order (its lane group q accumulates rows q, q + R, ... from 0 with
// R = 256 / LPR, then the groups are added in q order), so the partials
// are bit-identical to relu_bias_bwd on the unfused output.
// ---------------------------------------------------------------------------
template <int LPR, bool RB>
__global__ __launch_bounds__(RB ? 16 * LPR : 256) void sg_gather_sum_kernel(
    const int* __restrict__ posmap, const float* __restrict__ Z,
    const float* __restrict__ add, int lda, float* __restrict__ out, int N,
    int S, int C, int row0, const float* __restrict__ relu_out,
    float* __restrict__ part) {
  constexpr int RPB = RB ? 16 : 256 / LPR;      // rows per block
  const int blk = RB ? blockIdx.x : xcd_remap(blockIdx.x, gridDim.x);
  const int q = threadIdx.x / LPR;
  const int j = blk * RPB + q;
  const int lane = threadIdx.x % LPR;
  __shared__ float stash[RB ? 16 * 4 * LPR : 1];     // [16][C] masked rows
  if (RB && (j >= N || j < row0)) {     // (zero rows of the partials)
    for (int c0 = lane * 4; c0 < C; c0 += LPR * 4)
      *reinterpret_cast<float4*>(stash + q * C + c0) =
          make_float4(0.f, 0.f, 0.f, 0.f);
  }
  if (j < N && j < row0) {   // rows nobody reads the gradient of: zeros
    for (int c0 = lane * 4; c0 < C; c0 += LPR * 4)
      *reinterpret_cast<float4*>(out + (size_t)j * C + c0) =
          make_float4(0.f, 0.f, 0.f, 0.f);
  } else if (j < N) {
    // The row's S posmap entries are loaded once, lane-parallel (lane l of
    // the group holds entries l, l + LPR, ...), and broadcast by shuffles;
    // the Z rows are then gathered eight slots at a time, branch-free
    // (unused slots read row 0 and are not added), so a node's gathers are
    // in flight together instead of one dependent (posmap, Z) round per slot.
    constexpr int NP = (kSgMaxS + LPR - 1) / LPR;
    const int* pm = posmap + (size_t)j * S;
    int pl[NP];
#pragma unroll
    for (int u = 0; u < NP; ++u) {
      const int k = u * LPR + lane;
      const int v = pm[k < S ? k : 0];       // (clamped: never past the row)
      pl[u] = k < S ? v : -1;
    }
    for (int c0 = lane * 4; c0 < C; c0 += LPR * 4) {
      float4 acc = add ? ld4(add + (size_t)j * lda + c0)
                       : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int k0 = 0; k0 < kSgMaxS; k0 += 8) {
        if (k0 >= S) break;
        int p[8];
        float4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int k = k0 + u;
          p[u] = __shfl(pl[k / LPR], k % LPR, LPR);
          p[u] = k < S ? p[u] : -1;
          v[u] = ld4(Z + (size_t)(p[u] < 0 ? 0 : p[u]) * C + c0);
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (p[u] >= 0) {          // slot order: the same sums as before
            acc.x += v[u].x; acc.y += v[u].y; acc.z += v[u].z;
            acc.w += v[u].w;
          }
      }
      if (RB) {
        const float4 m = ld4(relu_out + (size_t)j * C + c0);
        acc.x = m.x > 0.f ? acc.x : 0.f;
        acc.y = m.y > 0.f ? acc.y : 0.f;
        acc.z = m.z > 0.f ? acc.z : 0.f;
        acc.w = m.w > 0.f ? acc.w : 0.f;
        *reinterpret_cast<float4*>(stash + q * C + c0) = acc;
      }
      *reinterpret_cast<float4*>(out + (size_t)j * C + c0) = acc;
    }
  }
  if (RB) {
    // (stash: the masked rows, 0 for rows < row0 - relu_bias_bwd sums
    // those zeros)
    __syncthreads();
    constexpr int R = 256 / LPR;              // colsum's lane groups
    for (int c = threadIdx.x; c < C; c += 16 * LPR) {
      float s = 0.f;
      for (int g = 0; g < R; ++g) {
        float a = 0.f;
        for (int r = g; r < 16; r += R)
          if (blk * 16 + r < N) a += stash[r * C + c];
        s += a;
      }
      part[(size_t)blk * C + c] = s;
    }
  }
}

at::Tensor slot_rowmap_ranges(const at::Tensor& rowptr,
                              const at::Tensor& cinv) {
  TORCH_CHECK(rowptr.is_cuda() && rowptr.scalar_type() == at::kInt &&
                  cinv.scalar_type() == at::kInt && cinv.is_contiguous() &&
                  rowptr.is_contiguous(),
              "slot_rowmap_ranges: int32 rowptr / cinv");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(cinv.device());
  const int64_t P = cinv.numel();
  at::Tensor out = at::empty({P, 2}, cinv.options());
  if (P == 0) return out;
  hipLaunchKernelGGL(sg_rowmap_ranges_kernel, dim3((unsigned)((P + 255) / 256)),
                     dim3(256), 0, stream(), rowptr.data_ptr<int>(),
                     cinv.data_ptr<int>(), (int)P,
                     reinterpret_cast<int2*>(out.data_ptr<int>()));
  DGMC_CHECK_LAUNCH();
  return out;
}

at::Tensor slot_rowmap_ell(const at::Tensor& rowptr, const at::Tensor& col,
                           const at::Tensor& val, const at::Tensor& cinv) {
  TORCH_CHECK(rowptr.is_cuda() && rowptr.scalar_type() == at::kInt &&
                  col.scalar_type() == at::kInt &&
                  val.scalar_type() == at::kFloat &&
                  cinv.scalar_type() == at::kInt && cinv.is_contiguous() &&
                  rowptr.is_contiguous() && col.is_contiguous() &&
                  val.is_contiguous(),
              "slot_rowmap_ell: int32 rowptr / col / cinv, fp32 val");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(cinv.device());
  const int64_t P = cinv.numel();
  at::Tensor out = at::empty({P, 8}, cinv.options());
  if (P == 0) return out;
  hipLaunchKernelGGL(sg_rowmap_ell_kernel, dim3((unsigned)((P + 255) / 256)),
                     dim3(256), 0, stream(), rowptr.data_ptr<int>(),
                     col.data_ptr<int>(), val.data_ptr<float>(),
                     cinv.data_ptr<int>(), (int)P,
                     reinterpret_cast<int4*>(out.data_ptr<int>()));
  DGMC_CHECK_LAUNCH();
  return out;
}

at::Tensor slot_gather_sum(const at::Tensor& posmap, const at::Tensor& Z,
                           int64_t N, int64_t S,
                           const c10::optional<at::Tensor>& add,
                           int64_t row0,
                           const c10::optional<at::Tensor>& relu_out,
                           const c10::optional<at::Tensor>& part) {
  TORCH_CHECK(Z.is_cuda() && Z.scalar_type() == at::kFloat &&
                  Z.is_contiguous() && Z.dim() == 2 && Z.size(1) % 4 == 0 &&
                  aligned16(Z.data_ptr()),
              "slot_gather_sum: contiguous fp32 Z [P, C % 4]");
  TORCH_CHECK(posmap.numel() == N * S, "slot_gather_sum: posmap [N * S]");
  const int64_t C = Z.size(1);
  const float* ap = nullptr;
  int64_t lda = 0;
  if (add.has_value() && add->defined()) {
    TORCH_CHECK(add->scalar_type() == at::kFloat && add->dim() == 2 &&
                    add->size(0) == N && add->size(1) == C &&
                    add->stride(1) == 1 && add->stride(0) % 4 == 0 &&
                    aligned16(add->data_ptr()),
                "slot_gather_sum: addend fp32 [N, C], 16-B aligned rows");
    ap = add->data_ptr<float>();
    lda = add->stride(0);
  }
  const bool rb = relu_out.has_value() && relu_out->defined();
  if (rb) {
    // (16-row partial blocks = relu_bias_bwd's blocks for these N)
    TORCH_CHECK(relu_out->scalar_type() == at::kFloat &&
                    relu_out->is_contiguous() && relu_out->size(0) == N &&
                    relu_out->size(1) == C && aligned16(relu_out->data_ptr()),
                "slot_gather_sum: relu_out contiguous fp32 [N, C]");
    TORCH_CHECK(N >= 256 && N <= 16 * 1024 && C >= 64 && C <= 256,
                "slot_gather_sum: fused ReLU / bias backward needs 256 <= N "
                "<= 16384, 64 <= C <= 256");
    TORCH_CHECK(part.has_value() && part->defined() &&
                    part->scalar_type() == at::kFloat && part->is_contiguous() &&
                    part->numel() == (N + 15) / 16 * C,
                "slot_gather_sum: part fp32 [ceil(N / 16), C]");
  }
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(Z.device());
  at::Tensor out = at::empty({N, C}, Z.options());
  if (N == 0) return out;
  const int lanes = (int)(C / 4);
  const float* rp = rb ? relu_out->data_ptr<float>() : nullptr;
  float* pp = rb ? part->data_ptr<float>() : nullptr;
  auto go = [&](auto lpr) {
    constexpr int L = decltype(lpr)::value;
    if (rb) {
      hipLaunchKernelGGL((sg_gather_sum_kernel<L, true>),
                         dim3((unsigned)((N + 15) / 16)), dim3(16 * L), 0,
                         stream(), posmap.data_ptr<int>(), Z.data_ptr<float>(),
                         ap, (int)lda, out.data_ptr<float>(), (int)N, (int)S,
                         (int)C, (int)row0, rp, pp);
      return;
    }
    const int64_t blocks = (N + 256 / L - 1) / (256 / L);
    hipLaunchKernelGGL((sg_gather_sum_kernel<L, false>), dim3(blocks),
                       dim3(256), 0, stream(), posmap.data_ptr<int>(),
                       Z.data_ptr<float>(), ap, (int)lda,
                       out.data_ptr<float>(), (int)N, (int)S, (int)C,
                       (int)row0, nullptr, nullptr);
  };
  if (lanes <= 8) go(std::integral_constant<int, 8>());
  else if (lanes <= 16) go(std::integral_constant<int, 16>());
  else if (lanes <= 32) go(std::integral_constant<int, 32>());
  else go(std::integral_constant<int, 64>());
  DGMC_CHECK_LAUNCH();
  return out;
}

// ---------------------------------------------------------------------------
// Weight gradient (TN):  dW_s[i, c] = sum_u sum_{p in slot s} X_u[src p][i]
// dY_u[p][c].  Work items = (slot, CH consecutive 128-row tiles of its
// segment), each a 128x128 output tile; the items' fp32 partials are folded
// per slot in item order (deterministic).
// ---------------------------------------------------------------------------
struct SgUses {
  const float* x[kSgMaxU];
  const float* g[kSgMaxU];
  const float* xp[kSgMaxU][4];    // dense mode: X_u as [M, 128] parts
};

// Item table: item i -> (slot, first step, end step); ib[s] = first item of
// slot s.  A slot's steps are its 32-row chunks x uses (chunk-major).  The
// steps per item Q balance the work: with `target` items (one or two rounds
// of resident workgroups) every slot is cut into ceil(steps / Q) pieces,
// Q = ceil(total / (target - S)) so that at most `target` items exist, capped
// by the LDS index buffer (qcap steps).  One wave: lane s owns slot s.
__global__ __launch_bounds__(64) void sg_items_kernel(
    const int* __restrict__ seg, int S, int nu, int target, int qcap,
    int G_cap, int* __restrict__ items, int* __restrict__ ib, int rows) {
  const int lane = threadIdx.x;
  int b = 0, steps = 0;
  if (lane < S) {
    b = seg[lane];
    steps = (seg[lane + 1] - b) / rows * nu;
  }
  int tot = steps;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o);
  int Q = target > S ? (tot + target - S - 1) / (target - S) : tot;
  Q = max(1, min(Q, qcap));
  const int n = (steps + Q - 1) / Q;
  int incl = n;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int v = __shfl_up(incl, o);
    if (lane >= o) incl += v;
  }
  const int first = incl - n;
  const int total = __shfl(incl, 63);
  if (lane < S) {
    ib[lane] = min(first, G_cap);
    for (int q = 0; q < n && first + q < G_cap; ++q) {
      items[3 * (first + q) + 0] = lane;
      items[3 * (first + q) + 1] = q * Q;
      items[3 * (first + q) + 2] = min((q + 1) * Q, steps);
    }
  }
  if (lane == 0) ib[S] = min(total, G_cap);
  for (int i = total + lane; i < G_cap; i += 64) items[3 * i + 0] = -1;
}

// Weight gradient: the TN product on LDS-DMA double-buffered operands.
// Work item (slot, CH row tiles) x output tile (i0, n0); the K loop runs over
// (32-row chunk, use) steps, chunk-major, so a chunk's gather indices (staged
// once per item in LDS) serve every use.  The accumulator holds dW^T (A
// operand = dY rows, B operand = X rows: a lane owns one input channel i and
// four consecutive output channels per register quad), so the partial tile
// is written with float4 stores.  Fragment reads are one ds_read_b32 per
// operand per MFMA step (lanes read 32 consecutive floats of one row: no
// bank conflicts on the lane-linear DMA image).
constexpr int kW2Rows = 32;                  // p rows per step
constexpr int kW2MaxRows = 3072;             // gathered rows per item (LDS)

template <bool DENSE>
__global__ __launch_bounds__(kSgThreads, 2) void slot_wgrad2_kernel(
    SgUses U, int nu, const int* __restrict__ src,
    const int* __restrict__ seg, const int* __restrict__ items, int Kin,
    int C, int ldxd, float* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) float sX0_[kW2Rows * 128];
  __shared__ __attribute__((aligned(16))) float sX1_[kW2Rows * 128];
  __shared__ __attribute__((aligned(16))) float sG0_[kW2Rows * 128];
  __shared__ __attribute__((aligned(16))) float sG1_[kW2Rows * 128];
  __shared__ int sidx[kW2MaxRows];
  DGMC_LDS float* sX0 = (DGMC_LDS float*)sX0_;
  DGMC_LDS float* sX1 = (DGMC_LDS float*)sX1_;
  DGMC_LDS float* sG0 = (DGMC_LDS float*)sG0_;
  DGMC_LDS float* sG1 = (DGMC_LDS float*)sG1_;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave & 1, wm = wave >> 1;
  const int tiles_n = C / kSgBN, tiles = (Kin / kSgBM) * tiles_n;
  const int item = blockIdx.x / tiles, t = blockIdx.x % tiles;
  const int i0 = (t / tiles_n) * kSgBM, n0 = (t % tiles_n) * kSgBN;
  const int s = items[3 * item];
  if (s < 0) return;
  // Steps [qb, qe) of slot s: chunk q / nu (32 rows from seg[s]), use
  // q % nu.  The gather indices of the item's chunks are staged once.
  const int qb = items[3 * item + 1], qe = items[3 * item + 2];
  const int c0 = qb / nu;
  const int pb = seg[s] + c0 * kW2Rows;
  const int nrows = ((qe - 1) / nu - c0 + 1) * kW2Rows;
  if (!DENSE) {
    for (int r = tid; r < nrows; r += kSgThreads) {
      const int j = src[pb + r];
      sidx[r] = j < 0 ? 0 : j;          // padding rows: dY row is zero
    }
    __syncthreads();
  }
  const int total = qe - qb;

  // Staging: wave w's pieces j = 0..3 cover rows 8 w + 2 j + (lane >> 5),
  // 16 B at column 4 (lane & 31) (lane-linear: no swizzle needed).
  const int prow = lane >> 5, pc = 4 * (lane & 31);
  auto stage = [&](int q, DGMC_LDS float* dx, DGMC_LDS float* dg) {
    const int qq = qb + q;
    const int ch = qq / nu - c0, u = qq - (qq / nu) * nu;
    const float* Xu = DENSE ? U.xp[u][i0 >> 7] + (i0 & 127) : U.x[u] + i0;
    const int ldx = DENSE ? ldxd : Kin;
    const float* Gu = U.g[u];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = 8 * wave + 2 * j + prow;
      const int row = ch * kW2Rows + r;
      sg_dma16(Xu + (size_t)(DENSE ? pb + row : sidx[row]) * ldx + pc,
               dx + (8 * wave + 2 * j) * 128);
      sg_dma16(Gu + (size_t)(pb + row) * C + n0 + pc,
               dg + (8 * wave + 2 * j) * 128);
    }
  };

  sg_f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  const int l32 = lane & 31, h = lane >> 5;
  auto compute = [&](const DGMC_LDS float* lx, const DGMC_LDS float* lg) {
#pragma unroll
    for (int st = 0; st < kW2Rows / 2; ++st) {
      const int kk = 2 * st + h;
      float av[2], bv[2];
#pragma unroll
      for (int a = 0; a < 2; ++a) av[a] = lg[kk * 128 + wn * 64 + a * 32 + l32];
#pragma unroll
      for (int b = 0; b < 2; ++b) bv[b] = lx[kk * 128 + wm * 64 + b * 32 + l32];
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[a], bv[b],
                                                           acc[a][b], 0, 0, 0);
    }
  };

  if (total > 0) stage(0, sX0, sG0);
  int q = 0;
  auto step = [&](DGMC_LDS float* cx, DGMC_LDS float* cg, DGMC_LDS float* nx,
                  DGMC_LDS float* ng) -> bool {
    const bool more = q + 1 < total;
    if (more) {
      stage(q + 1, nx, ng);
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    sg_raw_barrier();
    compute(cx, cg);
    sg_raw_barrier();
    ++q;
    return more;
  };
  if (total > 0)
    while (step(sX0, sG0, sX1, sG1) && step(sX1, sG1, sX0, sG0)) {
    }
  // acc[a][b]: rows c = wn 64 + 32 a + 8 qd + 4 h + e, column i = wm 64 +
  // 32 b + l32.
  float* outp = part + (size_t)item * Kin * C;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      float* row = outp + (size_t)(i0 + wm * 64 + b * 32 + l32) * C + n0 +
                   wn * 64 + a * 32 + 4 * h;
#pragma unroll
      for (int qd = 0; qd < 4; ++qd)
        *reinterpret_cast<float4*>(row + 8 * qd) =
            make_float4(acc[a][b][4 * qd], acc[a][b][4 * qd + 1],
                        acc[a][b][4 * qd + 2], acc[a][b][4 * qd + 3]);
    }
}

// out[s] = sum_{items of s, in order} part[item]  (float4 per thread).
__global__ __launch_bounds__(256) void sg_fold_kernel(
    const float* __restrict__ part, const int* __restrict__ ib, int S,
    int64_t per, float* __restrict__ out) {
  const int s = blockIdx.y;
  const int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  if (i >= per) return;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  const int ge = ib[s + 1];
  int g = ib[s];
  // (eight partial loads in flight; the sum keeps item order)
  for (; g + 8 <= ge; g += 8) {
    float4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = ld4(part + (size_t)(g + u) * per + i);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      acc.x += v[u].x; acc.y += v[u].y; acc.z += v[u].z; acc.w += v[u].w;
    }
  }
  for (; g < ge; ++g) {
    const float4 v = ld4(part + (size_t)g * per + i);
    acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
  }
  *reinterpret_cast<float4*>(out + (size_t)s * per + i) = acc;
}

// Work items (slot, step range) of `rows`-row steps for an external weight
// gradient kernel (slot_gemm_x6.hip) + the per-slot fold of its partials.
std::vector<at::Tensor> slot_wgrad_items(const at::Tensor& seg, int64_t nu,
                                         int64_t target, int64_t qcap,
                                         int64_t G_cap, int64_t rows) {
  const int64_t S = seg.numel() - 1;
  auto i32 = seg.options();
  at::Tensor items = at::empty({G_cap, 3}, i32);
  at::Tensor ib = at::empty({S + 1}, i32);
  hipLaunchKernelGGL(sg_items_kernel, dim3(1), dim3(64), 0, stream(),
                     seg.data_ptr<int>(), (int)S, (int)nu, (int)target,
                     (int)qcap, (int)G_cap, items.data_ptr<int>(),
                     ib.data_ptr<int>(), (int)rows);
  DGMC_CHECK_LAUNCH();
  return {items, ib};
}

at::Tensor slot_fold_parts(const at::Tensor& part, const at::Tensor& ib,
                           int64_t S, int64_t Kin, int64_t C) {
  const int64_t per = Kin * C;
  at::Tensor out = at::empty({S, Kin, C}, part.options());
  hipLaunchKernelGGL(sg_fold_kernel, dim3((per / 4 + 255) / 256, S), dim3(256),
                     0, stream(), part.data_ptr<float>(), ib.data_ptr<int>(),
                     (int)S, per, out.data_ptr<float>());
  DGMC_CHECK_LAUNCH();
  return out;
}

int slot_num_cus(int dev) { return num_cus(dev); }

at::Tensor slot_wgrad_f32(at::TensorList xs, at::TensorList gs,
                          const at::Tensor& src, const at::Tensor& seg,
                          int64_t rounds) {
  const int64_t nu = (int64_t)xs.size();
  TORCH_CHECK(nu >= 1 && nu <= kSgMaxU && (int64_t)gs.size() == nu,
              "slot_wgrad_f32: 1 <= uses <= 16, one G per X");
  const int64_t Kin = xs[0].size(1), C = gs[0].size(1);
  const int64_t P = src.numel(), S = seg.numel() - 1;
  TORCH_CHECK(Kin % kSgBM == 0 && C % kSgBN == 0 && P % kSgBM == 0 &&
                  rounds >= 1 && S <= kSgMaxS,
              "slot_wgrad_f32: in/out multiples of 128");
  SgUses U{};
  for (int64_t u = 0; u < nu; ++u) {
    const at::Tensor& x = xs[u];
    const at::Tensor& g = gs[u];
    TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kFloat &&
                    x.is_contiguous() && x.dim() == 2 && x.size(1) == Kin &&
                    aligned16(x.data_ptr()),
                "slot_wgrad_f32: X_u contiguous fp32 [N, in]");
    TORCH_CHECK(g.scalar_type() == at::kFloat && g.is_contiguous() &&
                    g.dim() == 2 && g.size(0) == P && g.size(1) == C &&
                    aligned16(g.data_ptr()),
                "slot_wgrad_f32: dY_u contiguous fp32 [P_cap, out]");
    U.x[u] = x.data_ptr<float>();
    U.g[u] = g.data_ptr<float>();
  }
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(src.device());
  // Items: `rounds` rounds of two resident workgroups per CU; steps per item
  // capped so an item's rows fit the LDS index buffer.
  const int64_t tiles = (Kin / kSgBM) * (C / kSgBN);
  const int64_t target = std::max<int64_t>(
      1, rounds * 2 * (int64_t)device_cus(src.device().index()) / tiles);
  const int64_t qcap = (kW2MaxRows / kW2Rows - 2) * nu;
  const int64_t G_cap = target + (P / kW2Rows * nu + qcap - 1) / qcap + S;
  auto i32 = src.options();
  at::Tensor items = at::empty({G_cap, 3}, i32);
  at::Tensor ib = at::empty({S + 1}, i32);
  hipLaunchKernelGGL(sg_items_kernel, dim3(1), dim3(64), 0, stream(),
                     seg.data_ptr<int>(), (int)S, (int)nu, (int)target,
                     (int)qcap, (int)G_cap, items.data_ptr<int>(),
                     ib.data_ptr<int>(), kW2Rows);
  DGMC_CHECK_LAUNCH();
  const int64_t per = Kin * C;
  at::Tensor part = at::empty({G_cap, per}, xs[0].options());
  hipLaunchKernelGGL(slot_wgrad2_kernel<false>, dim3(G_cap * tiles),
                     dim3(kSgThreads), 0, stream(), U, (int)nu,
                     src.data_ptr<int>(), seg.data_ptr<int>(),
                     items.data_ptr<int>(), (int)Kin, (int)C, 0,
                     part.data_ptr<float>());
  DGMC_CHECK_LAUNCH();
  at::Tensor out = at::empty({S, Kin, C}, xs[0].options());
  hipLaunchKernelGGL(sg_fold_kernel, dim3((per / 4 + 255) / 256, S), dim3(256),
                     0, stream(), part.data_ptr<float>(), ib.data_ptr<int>(),
                     (int)S, per, out.data_ptr<float>());
  DGMC_CHECK_LAUNCH();
  return out;
}

// Dense weight gradient sum_u [X_u,0 | X_u,1 | ...]^T G_u ([K, C], X parts
// [M, w] (w % 128, all parts alike) read in place, M % 32 == 0) on the slot
// kernel's dense mode: one "slot" [0, M), balanced step items, per-item
// partials folded in order.
at::Tensor dense_wgrad_f32(at::TensorList xparts, int64_t nparts,
                           at::TensorList gs, const at::Tensor& seg01) {
  const int64_t nu = (int64_t)gs.size();
  TORCH_CHECK(nu >= 1 && nu <= kSgMaxU && nparts >= 1 &&
                  (int64_t)xparts.size() == nu * nparts,
              "dense_wgrad_f32: 1..16 uses, nparts parts each");
  const int64_t M = gs[0].size(0), C = gs[0].size(1);
  const int64_t w = xparts[0].size(1), sub = w / 128;
  const int64_t Kin = w * nparts;
  TORCH_CHECK(w % 128 == 0 && nparts * sub <= 4,
              "dense_wgrad_f32: part widths % 128, K <= 512");
  TORCH_CHECK(M % kW2Rows == 0 && C % kSgBN == 0,
              "dense_wgrad_f32: M % 32, C % 128");
  TORCH_CHECK(seg01.scalar_type() == at::kInt && seg01.numel() == 2,
              "dense_wgrad_f32: seg [0, M] (device int32)");
  SgUses U{};
  for (int64_t u = 0; u < nu; ++u) {
    const at::Tensor& g = gs[u];
    TORCH_CHECK(g.is_cuda() && g.scalar_type() == at::kFloat &&
                    g.is_contiguous() && g.size(0) == M && g.size(1) == C &&
                    aligned16(g.data_ptr()),
                "dense_wgrad_f32: G_u contiguous fp32 [M, C]");
    U.g[u] = g.data_ptr<float>();
    for (int64_t j = 0; j < nparts; ++j) {
      const at::Tensor& x = xparts[u * nparts + j];
      TORCH_CHECK(x.scalar_type() == at::kFloat && x.is_contiguous() &&
                      x.dim() == 2 && x.size(0) == M && x.size(1) == w &&
                      aligned16(x.data_ptr()),
                  "dense_wgrad_f32: X parts contiguous fp32 [M, w]");
      for (int64_t q = 0; q < sub; ++q)
        U.xp[u][j * sub + q] = x.data_ptr<float>() + 128 * q;
    }
  }
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(seg01.device());
  const int64_t tiles = (Kin / kSgBM) * (C / kSgBN);
  // One round of resident workgroups: the outputs are small (<= 512 x 512)
  // and every item writes a full partial tile set for the fold.
  const int64_t target = std::max<int64_t>(
      2, 2 * (int64_t)device_cus(seg01.device().index()) / tiles);
  const int64_t qcap = (kW2MaxRows / kW2Rows - 2) * nu;
  const int64_t G_cap = target + (M / kW2Rows * nu + qcap - 1) / qcap + 1;
  auto i32 = seg01.options();
  at::Tensor items = at::empty({G_cap, 3}, i32);
  at::Tensor ib = at::empty({2}, i32);
  hipLaunchKernelGGL(sg_items_kernel, dim3(1), dim3(64), 0, stream(),
                     seg01.data_ptr<int>(), 1, (int)nu, (int)target,
                     (int)qcap, (int)G_cap, items.data_ptr<int>(),
                     ib.data_ptr<int>(), kW2Rows);
  DGMC_CHECK_LAUNCH();
  const int64_t per = Kin * C;
  at::Tensor part = at::empty({G_cap, per}, gs[0].options());
  hipLaunchKernelGGL(slot_wgrad2_kernel<true>, dim3(G_cap * tiles),
                     dim3(kSgThreads), 0, stream(), U, (int)nu, nullptr,
                     seg01.data_ptr<int>(), items.data_ptr<int>(), (int)Kin,
                     (int)C, (int)w, part.data_ptr<float>());
  DGMC_CHECK_LAUNCH();
  at::Tensor out = at::empty({Kin, C}, gs[0].options());
  hipLaunchKernelGGL(sg_fold_kernel, dim3((per / 4 + 255) / 256, 1), dim3(256),
                     0, stream(), part.data_ptr<float>(), ib.data_ptr<int>(),
                     1, per, out.data_ptr<float>());
  DGMC_CHECK_LAUNCH();
  return out;
}

}  // namespace dgmc
