// Fused similarity + top-k candidate search (reference dgmc.py:85-94, where
// KeOps LazyTensor.argKmin streams the N_s x N_t score matrix).
//
//   idx[b, i, :] = indices of the k largest <h_s[b,i], h_t[b,j]> over j,
//                  best first (ties: lower j first).
//
// One workgroup (4 waves) owns 64 source rows of one batch element; its rows
// stay resident in LDS while 64-row target tiles stream through LDS (the next
// tile is prefetched into registers while the current one is multiplied).
// Each wave computes a 32x32 score quadrant with exact-f32 MFMA
// (v_mfma_f32_32x32x2_f32).  K is consumed 8 at a time with a permuted k
// order so every operand fetch is one conflict-free ds_read_b128 (lane half h
// takes k = 8s + 4h .. 8s + 4h + 3 across four MFMAs).  Scores of a tile go
// through a small LDS tile into a per-row top-k list that lives in registers
// of lanes 0..k-1; candidates beating the current k-th score are inserted
// wave-parallel (ballot + popcount position + shfl_up shift).  The score matrix
// is never written to HBM.
#include "common.h"

namespace dgmc {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kTile = 64;
constexpr int kSPitch = 65;

template <int CT>
__global__ __launch_bounds__(256) void topk_dot_kernel(
    const float* __restrict__ h_s, const float* __restrict__ h_t,
    int64_t* __restrict__ out, int Ns, int Nt, int C, int k) {
  constexpr int CP = CT * 64;          // padded channel count
  constexpr int P = CP + 4;            // LDS row pitch (floats)
  constexpr int F4_ROW = CP / 4;       // float4 per padded row
  constexpr int PRE = kTile * F4_ROW / 256;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sA = smem;                    // [64][P]   source rows (resident)
  float* sB = sA + kTile * P;          // [64][P]   current target tile
  float* sS = sB + kTile * P;          // [64][65]  score tile

  const int b = blockIdx.y;
  const int row0 = blockIdx.x * kTile;
  const int tid = threadIdx.x;
  const int wave = tid / kWave, lane = tid % kWave;
  const float* hs = h_s + (size_t)b * Ns * C;
  const float* ht = h_t + (size_t)b * Nt * C;

  auto load_tile = [&](const float* base, int r0, int nrows, float4* regs) {
#pragma unroll
    for (int u = 0; u < PRE; ++u) {
      const int f = tid + 256 * u;
      const int r = f / F4_ROW, c = (f % F4_ROW) * 4;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (r0 + r < nrows && c < C)
        v = *reinterpret_cast<const float4*>(base + (size_t)(r0 + r) * C + c);
      regs[u] = v;
    }
  };
  auto store_tile = [&](float* dst, const float4* regs) {
#pragma unroll
    for (int u = 0; u < PRE; ++u) {
      const int f = tid + 256 * u;
      const int r = f / F4_ROW, c = (f % F4_ROW) * 4;
      *reinterpret_cast<float4*>(dst + r * P + c) = regs[u];
    }
  };

  float4 pre[PRE];
  load_tile(hs, row0, Ns, pre);
  store_tile(sA, pre);
  load_tile(ht, 0, Nt, pre);
  store_tile(sB, pre);
  __syncthreads();

  // Per-row top-k lists: wave owns rows wave*16 .. wave*16+15 of the block;
  // lane q < k holds entry q of each list.
  float lv[16];
  int li[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) { lv[q] = -INFINITY; li[q] = 0; }

  const int qr = (wave >> 1) * 32, qc = (wave & 1) * 32;
  const int h = lane >> 5, l32 = lane & 31;
  const float* aRow = sA + (qr + l32) * P + 4 * h;
  const float* bRow = sB + (qc + l32) * P + 4 * h;
  const int ntiles = (Nt + kTile - 1) / kTile;

  for (int t = 0; t < ntiles; ++t) {
    if (t + 1 < ntiles) load_tile(ht, (t + 1) * kTile, Nt, pre);

    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll 4
    for (int s = 0; s < CP / 8; ++s) {
      const float4 a = *reinterpret_cast<const float4*>(aRow + 8 * s);
      const float4 bb = *reinterpret_cast<const float4*>(bRow + 8 * s);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, bb.x, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, bb.y, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, bb.z, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, bb.w, acc, 0, 0, 0);
    }
    // C/D layout of 32x32: col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = qr + (r & 3) + 8 * (r >> 2) + 4 * h;
      sS[row * kSPitch + qc + l32] = acc[r];
    }
    __syncthreads();
    if (t + 1 < ntiles) store_tile(sB, pre);

    const int j = t * kTile + lane;
    const bool col_ok = j < Nt;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int row = wave * 16 + q;
      const float v = sS[row * kSPitch + lane];
      float thr = __shfl(lv[q], k - 1);
      unsigned long long mask = __ballot(col_ok && v > thr);
      while (mask) {
        const int src = __ffsll((long long)mask) - 1;
        mask &= mask - 1;
        const float cv = __shfl(v, src);
        if (!(cv > thr)) continue;
        const int pos =
            __popcll(__ballot(lane < k && lv[q] >= cv));
        const float pv = __shfl_up(lv[q], 1);
        const int pi = __shfl_up(li[q], 1);
        if (lane > pos && lane < k) { lv[q] = pv; li[q] = pi; }
        if (lane == pos) { lv[q] = cv; li[q] = t * kTile + src; }
        thr = __shfl(lv[q], k - 1);
      }
    }
    __syncthreads();
  }

#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int row = row0 + wave * 16 + q;
    if (row < Ns && lane < k)
      out[((size_t)b * Ns + row) * k + lane] = (int64_t)li[q];
  }
}

at::Tensor topk_dot(const at::Tensor& h_s, const at::Tensor& h_t, int64_t k) {
  TORCH_CHECK(h_s.is_cuda() && h_t.is_cuda() && h_s.dim() == 3 &&
                  h_t.dim() == 3 && h_s.scalar_type() == at::kFloat &&
                  h_t.scalar_type() == at::kFloat && h_s.is_contiguous() &&
                  h_t.is_contiguous(),
              "topk_dot: contiguous fp32 [B, N, C] inputs expected");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(h_s.device());
  const int B = h_s.size(0), Ns = h_s.size(1), C = h_s.size(2);
  const int Nt = h_t.size(1);
  TORCH_CHECK(h_t.size(0) == B && h_t.size(2) == C, "topk_dot: shape");
  TORCH_CHECK(k >= 1 && k <= 64 && k <= Nt, "topk_dot: need 1 <= k <= min(64, N_t)");
  TORCH_CHECK(C % 4 == 0 && C <= 256, "topk_dot: C % 4 == 0 and C <= 256");
  at::Tensor out = at::empty({B, Ns, k}, h_s.options().dtype(at::kLong));
  if (B == 0 || Ns == 0) return out;
  const int CT = (C + 63) / 64;
  const int P = CT * 64 + 4;
  const size_t lds = (size_t)(2 * kTile * P + kTile * kSPitch) * sizeof(float);
  dim3 grid((Ns + kTile - 1) / kTile, B);
  auto launch = [&](auto kernel) {
    DGMC_CHECK_HIP(hipFuncSetAttribute(
        reinterpret_cast<const void*>(kernel),
        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(kernel, grid, dim3(256), lds, stream(),
                       h_s.data_ptr<float>(), h_t.data_ptr<float>(),
                       out.data_ptr<int64_t>(), Ns, Nt, C, (int)k);
  };
  switch (CT) {
    case 1: launch(topk_dot_kernel<1>); break;
    case 2: launch(topk_dot_kernel<2>); break;
    case 3: launch(topk_dot_kernel<3>); break;
    default: launch(topk_dot_kernel<4>); break;
  }
  DGMC_CHECK_LAUNCH();
  return out;
}

}  // namespace dgmc
