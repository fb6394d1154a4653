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
    int64_t* __restrict__ out, int Ns, int Nt, int C, int k, int dbg) {
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
    for (int s = 0; s < ((kDiagBuild && (dbg & 2)) ? 0 : CP / 8); ++s) {
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
    const bool col_ok = j < Nt && !(kDiagBuild && (dbg & 1));
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


// ---------------------------------------------------------------------------
// Split-bf16 ("bf16x3") variant.  Each fp32 operand is split as x = hi + lo
// with hi = bf16(x), lo = bf16(x - hi) (16 mantissa bits together) and the
// score is accumulated in fp32 as hi_s.hi_t + hi_s.lo_t + lo_s.hi_t on
// v_mfma_f32_32x32x16_bf16 - 3 MFMA passes at 16x the f32-MFMA rate, i.e.
// ~5x fewer matrix-core cycles than exact f32, with score errors ~2^-16
// relative (only exact near-ties can order differently from fp32).
//
// Layout: a workgroup of 4 waves owns 128 source rows; every wave keeps the
// hi/lo A fragments of its 32 rows in registers for the whole kernel (128
// VGPRs at C=256), so only the 32-target B tiles stream through LDS (double
// buffered, one barrier per tile, next tile prefetched into registers during
// the MFMAs).  Two workgroups fit per CU (67.6 KB LDS, <=256 VGPRs), so one
// block's selection overlaps the other's MFMAs.  The 32x32 accumulator is
// used in place for selection: acc[r] of lanes 0..31 is source row
// R(r) = (r&3)+8(r>>2) over the 32 targets of the tile, lanes 32..63 hold row
// R(r)+4, so each half-wave keeps the top-k list of one row in lanes
// 0..k-1 of that half (k <= 32) and candidates are filtered with one
// compare against the half's k-th value (read with v_readlane).
// The target range can be split over gridDim.y blocks (to fill 256 CUs when
// N_s is small); per-split lists are then merged by topk_merge_kernel.
// ---------------------------------------------------------------------------
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// Source rows per workgroup: W waves x 32.  W = 8 (one 512-thread workgroup
// per CU) at C = 128 / 256: every streamed target tile serves 256 source rows
// - the kernel is bound by the target-plane stream (MALL / HBM), not the
// matrix cores, at 128 rows per tile load.
constexpr int kX3Tile = 32;    // targets per streamed tile

__device__ __forceinline__ float lane_f(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

// v of lane - 1 (DPP wave_shr:1); lane 0's result is undefined (no "old"
// operand to materialise: the callers never use it).
__device__ __forceinline__ int shr1(int v) {
  return __builtin_amdgcn_mov_dpp(v, 0x138, 0xf, 0xf, false);
}
__device__ __forceinline__ float shr1(float v) {
  return __int_as_float(shr1(__float_as_int(v)));
}

// h_t split once into bf16 hi / lo planes [B, Nt, CP] (CP = padded channels,
// zero tail), so the streaming loop of topk_x3_kernel moves 16-byte vectors
// straight into LDS with no per-block conversion work.
__global__ __launch_bounds__(256) void split_bf16_kernel(
    const float* __restrict__ x, __bf16* __restrict__ hi,
    __bf16* __restrict__ lo, int64_t rows, int C, int CP) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int vpr = CP / 4;
  const int64_t r = t / vpr;
  if (r >= rows) return;
  const int c = (int)(t % vpr) * 4;
  float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
  if (c < C) v = *reinterpret_cast<const float4*>(x + r * C + c);
  const float f[4] = {v.x, v.y, v.z, v.w};
  bf16x4 vh, vl;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const __bf16 h = (__bf16)f[e];
    vh[e] = h;
    vl[e] = (__bf16)(f[e] - (float)h);
  }
  *reinterpret_cast<bf16x4*>(hi + r * CP + c) = vh;
  *reinterpret_cast<bf16x4*>(lo + r * CP + c) = vl;
}

// Lane l ^ jj's value (jj = 1, 2, 4, 8 or 16, a constant after unrolling):
// DPP within the 16-lane row for 1, 2 (quad_perm) and 8 (row_ror:8), the
// LDS crossbar (ds_bpermute) otherwise.  (Same-box A/B, tools/gpu_r6_ah.sh:
// cold filter 1.077 -> 1.066 ms.)
__device__ __forceinline__ int xor_lane(int v, int jj) {
  if (jj == 1) return __builtin_amdgcn_mov_dpp(v, 0xB1, 0xf, 0xf, false);
  if (jj == 2) return __builtin_amdgcn_mov_dpp(v, 0x4E, 0xf, 0xf, false);
  if (jj == 8) return __builtin_amdgcn_mov_dpp(v, 0x128, 0xf, 0xf, false);
  return __shfl_xor(v, jj);
}

// Bitonic sort of (v, ix) over the 32 lanes of each half-wave into (value
// desc, index asc) order, from stage k2 = k2_0 (2: a full sort; 32: only the
// final merge of a bitonic sequence).
__device__ __forceinline__ void x3_bitonic32(float& v, int& ix, int hl,
                                             int k2_0) {
#pragma unroll
  for (int k2 = 2; k2 <= 32; k2 <<= 1) {
    if (k2 < k2_0) continue;
#pragma unroll
    for (int jj = k2 >> 1; jj > 0; jj >>= 1) {
      const float pv = __int_as_float(xor_lane(__float_as_int(v), jj));
      const int pix = xor_lane(ix, jj);
      const bool better = v > pv || (v == pv && ix < pix);
      const bool desc = (hl & k2) == 0, lower = (hl & jj) == 0;
      if ((lower == desc) != better) {
        v = pv;
        ix = pix;
      }
    }
  }
}

// Tiles (from the first) whose lists are updated by sort + merge instead of
// insertion rounds (the rounds win once few scores of a tile still enter).
// Same-box sweeps (tools/gpu_r6_ac.sh, gpu_r6_aj.sh): 4 with the first
// insertion rounds; 2 since the rounds got cheaper (1.12-1.14 ms against
// 1.15 at 4, 1.14 at 1, 1.14 at 3, 1.18 at 6).
constexpr int kX3MergeTiles = 2;

template <int NKS, int W>
__global__ __launch_bounds__(64 * W, 8 / W) void topk_x3_kernel(
    const float* __restrict__ h_s, const __bf16* __restrict__ t_hi,
    const __bf16* __restrict__ t_lo,
    float* __restrict__ part_v, int* __restrict__ part_i,
    int64_t* __restrict__ out, float* __restrict__ out_v, int Ns, int Nt,
    int C, int k, int span, int dbg, const float* __restrict__ warm) {
  constexpr int CP = NKS * 16;              // padded channels
  constexpr int BP = CP + 8;                // LDS row pitch (bf16)
  constexpr int TILE = kX3Tile * BP;        // one hi or lo tile (bf16)
  constexpr int V_ROW = CP / 8;             // 16-byte vectors per plane row
  constexpr int NT = 64 * W;                // threads
  constexpr int PRE = kX3Tile * V_ROW / NT;     // vectors per thread per plane
  static_assert(PRE >= 1 && kX3Tile * V_ROW % NT == 0, "tile split");
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  DGMC_LDS __bf16* sB = (DGMC_LDS __bf16*)smem_raw;   // [2 buf][hi, lo][TILE]

  const int b = blockIdx.z, split = blockIdx.y;
  const int tid = threadIdx.x, wave = tid / kWave, lane = tid % kWave;
  const int h = lane >> 5, hl = lane & 31, hb = lane & 32;
  const bool in_list = hl < k;
  // the list lanes of both halves as a ballot mask
  const unsigned long long in_mask =
      (((1ull << k) - 1ull) << 32) | ((1ull << k) - 1ull);
  const int row0 = blockIdx.x * (32 * W) + wave * 32;
  const int j_begin = split * span;
  const int j_end = min(Nt, j_begin + span);
  const float* hs = h_s + (size_t)b * Ns * C;
  const __bf16* th = t_hi + (size_t)b * Nt * CP;
  const __bf16* tl = t_lo + (size_t)b * Nt * CP;

  // A fragments (this wave's 32 source rows), split once.
  bf16x8 ahi[NKS], alo[NKS];
  {
    const int r = row0 + hl;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int c = ks * 16 + 8 * h + 4 * q;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (r < Ns && c < C)
          v = *reinterpret_cast<const float4*>(hs + (size_t)r * C + c);
        const float f[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const __bf16 hi = (__bf16)f[e];
          ahi[ks][4 * q + e] = hi;
          alo[ks][4 * q + e] = (__bf16)(f[e] - (float)hi);
        }
      }
    }
  }

  auto load_tile = [&](int j0, u32x4* regs) {
#pragma unroll
    for (int u = 0; u < PRE; ++u) {
      const int f = tid + NT * u;
      const int r = f / V_ROW, c = (f % V_ROW) * 8;
      u32x4 h = {0u, 0u, 0u, 0u}, l = h;
      if (j0 + r < j_end) {
        // (32-bit byte offsets from the uniform plane bases: saddr-form
        // loads, no per-lane 64-bit pointers held across the loop)
        const uint32_t off = (uint32_t)((j0 + r) * CP + c) * 2u;
        h = *reinterpret_cast<const u32x4*>(
            reinterpret_cast<const char*>(th) + off);
        l = *reinterpret_cast<const u32x4*>(
            reinterpret_cast<const char*>(tl) + off);
      }
      regs[u] = h;
      regs[PRE + u] = l;
    }
  };
  auto store_tile = [&](int buf, const u32x4* regs) {
    DGMC_LDS __bf16* hi_t = sB + buf * 2 * TILE;
    DGMC_LDS __bf16* lo_t = hi_t + TILE;
#pragma unroll
    for (int u = 0; u < PRE; ++u) {
      const int f = tid + NT * u;
      const int r = f / V_ROW, c = (f % V_ROW) * 8;
      *reinterpret_cast<DGMC_LDS u32x4*>(hi_t + r * BP + c) = regs[u];
      *reinterpret_cast<DGMC_LDS u32x4*>(lo_t + r * BP + c) = regs[PRE + u];
    }
  };

  float lv[16];
  int li[16];
  const int init_i = Nt + split * 64 + hl;    // unique sentinels (>= Nt)
  // k-th value of each row's list, kept per half-wave (lanes of half h hold
  // their row's threshold) - no readlane per candidate test.
  float thr[16];
  // Warm start (topk_warm_kernel): each list starts FULL of sentinel
  // entries valued just below a proven lower bound of the row's k-th
  // approximate score, so only targets that can still make the final list
  // are ever inserted.  Every member of the row's true top-k (by
  // approximate score) lies strictly above the start value and evicts the
  // sentinels; the selected lists are the same as from an empty start.
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    float t0 = -INFINITY;
    const int row = row0 + (r & 3) + 8 * (r >> 2) + 4 * h;
    if (warm && row < Ns) {
      const float w = warm[(size_t)b * Ns + row];
      t0 = w > -INFINITY ? nextafterf(w, -INFINITY) : -INFINITY;  // NaN too
    }
    lv[r] = t0;
    li[r] = init_i;
    thr[r] = t0;
  }

  const int ntiles = (j_end - j_begin + kX3Tile - 1) / kX3Tile;
  u32x4 pre[2 * PRE];
  if (ntiles > 0) {
    load_tile(j_begin, pre);
    store_tile(0, pre);
  }
  __syncthreads();

  int t_first = 0;
  if (ntiles > 0 && warm == nullptr && !(kDiagBuild && (dbg & 3))) {
    // The first tile fills the (empty) lists: every score of it would be
    // inserted one round at a time (32 rounds per row); instead each
    // half-wave sorts its row's 32 scores with a bitonic network (value
    // desc, index asc - the order the insertion rounds produce) and keeps
    // the first k.  Masked, -inf and NaN scores carry the lane's sentinel
    // index, as the rounds would leave them.  Same-box A/B on DBP15K zh_en
    // (tools/gpu_r6_ab.sh): filter 1.38 -> 1.30 ms, refinement step 4.91 ->
    // 4.82 ms.
    const int j0 = j_begin;
    if (1 < ntiles) load_tile(j0 + kX3Tile, pre);
    const DGMC_LDS __bf16* bh = sB + hl * BP + 8 * h;
    const DGMC_LDS __bf16* bl = bh + TILE;
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      const bf16x8 vh = *reinterpret_cast<const DGMC_LDS bf16x8*>(bh + 16 * ks);
      const bf16x8 vl = *reinterpret_cast<const DGMC_LDS bf16x8*>(bl + 16 * ks);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(alo[ks], vh, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ahi[ks], vl, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ahi[ks], vh, acc, 0, 0, 0);
    }
    if (1 < ntiles) store_tile(1, pre);
    __builtin_amdgcn_sched_barrier(0);     // (pre dead before the sort)
    const bool col_ok = j0 + hl < j_end;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const bool ok = col_ok && acc[r] > -INFINITY;
      float v = ok ? acc[r] : -INFINITY;
      int ix = ok ? j0 + hl : init_i;
      x3_bitonic32(v, ix, hl, 2);
      lv[r] = v;
      li[r] = ix;
      const float t_lo_half = lane_f(v, k - 1);
      const float t_hi_half = lane_f(v, 32 + k - 1);
      thr[r] = hb ? t_hi_half : t_lo_half;
      __builtin_amdgcn_sched_barrier(0);   // (one row at a time)
    }
    __syncthreads();
    t_first = 1;
  }

  auto step = [&](int t, auto merge_tag) {
    constexpr bool MERGE = decltype(merge_tag)::value;
    const int j0 = j_begin + t * kX3Tile;
    if (t + 1 < ntiles) load_tile(j0 + kX3Tile, pre);
    const DGMC_LDS __bf16* bh = sB + (t & 1) * 2 * TILE + hl * BP + 8 * h;
    const DGMC_LDS __bf16* bl = bh + TILE;
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    if (!(kDiagBuild && (dbg & 2))) {
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        const bf16x8 vh = *reinterpret_cast<const DGMC_LDS bf16x8*>(bh + 16 * ks);
        const bf16x8 vl = *reinterpret_cast<const DGMC_LDS bf16x8*>(bl + 16 * ks);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(alo[ks], vh, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ahi[ks], vl, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ahi[ks], vh, acc, 0, 0, 0);
      }
    }
    if (t + 1 < ntiles) store_tile((t + 1) & 1, pre);

    const bool col_ok = j0 + hl < j_end && !(kDiagBuild && (dbg & 1));
    if constexpr (MERGE) {
      // Early tiles still put about half their scores into the lists: sort
      // the tile's 32 scores per row-half (bitonic, value desc, index asc)
      // and merge them with the sorted 32-entry list (lanes >= k hold the
      // runners-up of the earlier tiles): the better of list[i] and
      // new[31 - i] gives the top 32 as a bitonic sequence, five more steps
      // sort it.  Every entry stays distinct - the tile's sentinels
      // (masked / non-finite scores) get indices of their own, >= Nt and
      // unique per (split, tile, lane) - so the split merge can rank them.
      const int sent = Nt + 64 * (split + (int)gridDim.y * t) + hl;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const bool ok = col_ok && acc[r] > -INFINITY;
        float v = ok ? acc[r] : -INFINITY;
        int ix = ok ? j0 + hl : sent;
        x3_bitonic32(v, ix, hl, 2);
        // reversed new list against the current list
        const float rv = __shfl(v, (lane & 32) + 31 - hl);
        const int rix = __shfl(ix, (lane & 32) + 31 - hl);
        float a = lv[r];
        int ai = li[r];
        if (rv > a || (rv == a && rix < ai)) {
          a = rv;
          ai = rix;
        }
        x3_bitonic32(a, ai, hl, 32);
        lv[r] = a;
        li[r] = ai;
        const float t_lo_half = lane_f(a, k - 1);
        const float t_hi_half = lane_f(a, 32 + k - 1);
        thr[r] = hb ? t_hi_half : t_lo_half;
        __builtin_amdgcn_sched_barrier(0);   // (one row at a time)
      }
      __syncthreads();
      return;
    }
    // Warm start: one wave vote for the whole tile first - the lists start
    // full, most tiles hold no candidate beating any row's k-th score, and
    // the 16 per-row votes below are skipped.  (Cold, some row of the
    // wave's 32 nearly always has a hit: the vote only costs - filter
    // 1.199 -> 1.163 ms without it, same box, tools/gpu_r6_ah.sh.)
    bool any = true;
    if (warm != nullptr) {
      bool hit = false;
#pragma unroll
      for (int r = 0; r < 16; ++r) hit |= col_ok && acc[r] > thr[r];
      any = __ballot(hit) != 0ull;
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      if (!any) break;
      const float v = col_ok ? acc[r] : -INFINITY;
      const unsigned long long mask = __ballot(v > thr[r]);
      // One candidate of each half-wave per round (the halves hold
      // different rows): max(hits_lo, hits_hi) rounds, not their sum.
      // (Interleaving two rows' rounds measured slower: 1.27 -> 1.39 ms.)
      // Scalar picks; an exhausted half proposes -inf, which its whole
      // list outranks (no insertion).  No threshold test per round: a
      // candidate that no longer beats the k-th entry ranks at pos = k and
      // changes nothing, so the threshold is re-read once per row, after
      // its rounds.  Branch-free list update (selects, no exec-mask
      // branches).  ~20 vector instructions a round against ~40 before
      // (hipcc -S; same-box filter 1.277 -> 1.196 ms, tools/gpu_r6_af.sh,
      // then 1.12 -> 1.08 ms for the ballot mask and DPP form,
      // tools/gpu_r6_ah.sh).
      unsigned lo = (unsigned)mask, hi = (unsigned)(mask >> 32);
      while (lo | hi) {
        float cv0 = -INFINITY, cv1 = -INFINITY;
        int s0 = 0, s1 = 0;
        if (lo) {
          s0 = __builtin_ctz(lo);
          cv0 = lane_f(v, s0);
          lo ^= 1u << s0;
        }
        if (hi) {
          s1 = __builtin_ctz(hi);
          cv1 = lane_f(v, 32 + s1);
          hi ^= 1u << s1;
        }
        const float cv = hb ? cv1 : cv0;
        // (list lanes masked in scalar: a ballot of a compound condition
        // is materialised through a VGPR first)
        const unsigned long long bm = __ballot(lv[r] >= cv) & in_mask;
        const int pos =
            hb ? __popc((unsigned)(bm >> 32)) : __popc((unsigned)bm);
        // shift the tail of the half's list down one lane (DPP wave_shr:1;
        // lane hl > pos >= 0 always reads a lane of its own half)
        const float pv = shr1(lv[r]);
        const int pi = shr1(li[r]);
        const bool at = in_list && hl == pos;
        const bool sh = in_list && hl > pos;
        const int ci = j0 + (hb ? s1 : s0);
        lv[r] = at ? cv : (sh ? pv : lv[r]);
        li[r] = at ? ci : (sh ? pi : li[r]);
      }
      if (mask) {
        const float t_lo_half = lane_f(lv[r], k - 1);
        const float t_hi_half = lane_f(lv[r], 32 + k - 1);
        thr[r] = hb ? t_hi_half : t_lo_half;
      }
    }
    __syncthreads();
  };
  // (two loops: the merge tiles' register use stays out of the main loop)
  int t = t_first;
  if (t_first == 1)
    for (; t < min(kX3MergeTiles, ntiles); ++t) step(t, std::true_type());
  for (; t < ntiles; ++t) step(t, std::false_type());

  if (hl < k) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = row0 + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (row >= Ns) continue;
      const size_t g = (size_t)b * Ns + row;
      if (part_v) {
        const size_t o = (g * gridDim.y + split) * k + hl;
        part_v[o] = lv[r];
        part_i[o] = li[r];
      } else {
        // (a sentinel can only survive a warm start whose bound did not
        // hold: it leaves as index 0 with value -inf, which the exact
        // re-score treats as a short list - the exhaustive fallback)
        const bool real = li[r] < Nt;
        out[g * k + hl] = real ? (int64_t)li[r] : 0;
        if (out_v) out_v[g * k + hl] = real ? lv[r] : -INFINITY;
      }
    }
  }
}

// Merge of per-split top-k lists: one thread per candidate computes its rank
// among the row's S*k candidates (value desc, index asc) and scatters itself.
__global__ __launch_bounds__(256) void topk_merge_kernel(
    const float* __restrict__ part_v, const int* __restrict__ part_i,
    int64_t* __restrict__ out, float* __restrict__ out_v, int64_t rows, int S,
    int k, int Nt) {
  const int n = S * k;
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t row = g / n;
  if (row >= rows) return;
  const float* v = part_v + row * n;
  const int* ix = part_i + row * n;
  const int c = (int)(g - row * n);
  const float mv = v[c];
  const int mj = ix[c];
  int rank = 0;
  for (int e = 0; e < n; ++e) {
    const float ov = v[e];
    const int oj = ix[e];
    rank += (ov > mv) || (ov == mv && oj < mj);
  }
  if (rank < k) {
    out[row * k + rank] = mj < Nt ? mj : 0;
    if (out_v) out_v[row * k + rank] = mj < Nt ? mv : -INFINITY;
  }
}

// The same merge with one wave per row (S * k <= 64): lane l holds
// candidate l, its rank from uniform-lane reads of the others (same
// comparisons, same output).
__global__ __launch_bounds__(256) void topk_merge_wave_kernel(
    const float* __restrict__ part_v, const int* __restrict__ part_i,
    int64_t* __restrict__ out, float* __restrict__ out_v, int64_t rows, int S,
    int k, int Nt) {
  const int n = S * k;
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;                     // wave-uniform
  const float* v = part_v + row * n;
  const int* ix = part_i + row * n;
  const bool on = lane < n;
  const float mv = on ? v[lane] : 0.f;
  const int mj = on ? ix[lane] : 0;
  int rank = 0;
  for (int e = 0; e < n; ++e) {
    const float ov = __int_as_float(
        __builtin_amdgcn_readlane(__float_as_int(mv), e));
    const int oj = __builtin_amdgcn_readlane(mj, e);
    rank += (ov > mv) || (ov == mv && oj < mj);
  }
  if (on && rank < k) {
    out[row * k + rank] = mj < Nt ? mj : 0;
    if (out_v) out_v[row * k + rank] = mj < Nt ? mv : -INFINITY;
  }
}

// ---------------------------------------------------------------------------
// Exact fp32 top-k at split-bf16 speed: filter + exact re-score.
//
// The bf16x3 pass keeps K2 = min(32, N_t, max(16, k + 6)) approximate
// candidates per row
// (scores s~_j, best first).  Its error against the exact-f32 MFMA score s_j
// (the k-ordered fmaf chain of topk_dot_kernel) is bounded per product by
// the dropped lo*lo term and the two split residuals (<= ~3 * 2^-18 |a b|)
// plus the fp32 accumulation of both (<= ~2^-16 sum |a b| at C = 256), so
// |s~_j - s_j| <= E = tau * |a| * max_j |b_j| (Cauchy-Schwarz) with
// tau = 2^-13, a >= 3x margin over the worst case.  Every member of the exact
// top-k then has s~_j >= T_k - 2E (T_k = the k-th approximate score): if
// j is in the exact top-k, s_j >= (exact k-th) >= T_k - E.  So
//   * candidates with s~_j >= T_k - 2E are re-scored with the exact chain
//     (bit-identical to topk_dot_kernel: k = 8s + t, then 8s + 4 + t) and
//     the k best by (exact score desc, index asc) are written;
//   * if the K2-th approximate candidate itself clears T_k - 2E the kept
//     list may be incomplete: that row (rare; hub-heavy near-ties) is
//     recomputed exactly over all N_t targets by its wave.
// One wave per row; the row of h_s is staged in LDS (zero-padded to a
// multiple of 8 channels) and broadcast to the lanes' chains.
// ---------------------------------------------------------------------------
constexpr float kTopkTau = 1.0f / 8192.0f;
// DGMC_TOPK_TAU_LOG2 (diagnostic build only): tau = 2^-value.
static float topk_tau() {
  static const float v = [] {
    const int e = diag_env_int("DGMC_TOPK_TAU_LOG2", 0);
    return e > 0 ? ldexpf(1.0f, -e) : kTopkTau;
  }();
  return v;
}

static at::Tensor topk_dot_x3(const at::Tensor& h_s, const at::Tensor& h_t,
                              int64_t k, at::Tensor* vals = nullptr,
                              const at::Tensor* warm = nullptr);
constexpr int kRefRows = 4;      // rows (waves) per block

// Per-block partial maxima of |h_t[b, j]|^2 (any summation order: the value
// only feeds the bound, with its own 1 + 2^-10 safety factor below).
__global__ __launch_bounds__(256) void row_sqnorm_max_kernel(
    const float* __restrict__ x, int Nt, int C, float* __restrict__ part) {
  __shared__ float red[4];
  const int b = blockIdx.y, j = blockIdx.x * 256 + threadIdx.x;
  float v = 0.f;
  if (j < Nt) {
    const float* r = x + ((size_t)b * Nt + j) * C;
    for (int c = 0; c < C; c += 4) {
      const float4 q = *reinterpret_cast<const float4*>(r + c);
      v += q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w;
    }
  }
  v = wave_max(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0)
    part[(size_t)b * gridDim.x + blockIdx.x] =
        fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

// Exact chain of topk_dot_kernel for one target row (a: LDS, zero-padded;
// C % 4 == 0).  The target row is fetched 64 channels at a time as 16
// independent 16-byte loads (clamped, zeroed past C) before that chunk's
// FMAs - the chain itself (k = 8s + t, then 8s + 4 + t) is unchanged.
__device__ __forceinline__ float exact_dot(const DGMC_LDS float* a,
                                           const float* __restrict__ b,
                                           int C, int C8) {
  float acc = 0.f;
  for (int s0 = 0; s0 < C8; s0 += 64) {
    float4 v[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int e = s0 + 4 * q;
      const float4 t =
          *reinterpret_cast<const float4*>(b + min(e, C - 4));
      v[q] = e < C ? t : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int s = s0 + 8 * u;
      if (s >= C8) break;
      const float bv[8] = {v[2 * u].x,     v[2 * u].y,     v[2 * u].z,
                           v[2 * u].w,     v[2 * u + 1].x, v[2 * u + 1].y,
                           v[2 * u + 1].z, v[2 * u + 1].w};
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        acc = __builtin_fmaf(a[s + t], bv[t], acc);
        acc = __builtin_fmaf(a[s + 4 + t], bv[4 + t], acc);
      }
    }
  }
  return acc;
}

__global__ __launch_bounds__(kRefRows * 64) void topk_refine_kernel(
    const float* __restrict__ h_s, const float* __restrict__ h_t,
    const int64_t* __restrict__ cand_i, const float* __restrict__ cand_v,
    const float* __restrict__ nmax_part, int nparts, int64_t* __restrict__ out,
    int* __restrict__ n_overflow, int Ns, int Nt, int C, int k, int K2,
    float tau) {
  __shared__ __attribute__((aligned(16))) float sa[kRefRows][264];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t g = (int64_t)blockIdx.x * kRefRows + wave;
  const int b = blockIdx.y;
  if (g >= Ns) return;                 // wave-uniform; no block barrier below
  const int C8 = (C + 7) & ~7;
  const float* arow = h_s + ((size_t)b * Ns + g) * C;
  DGMC_LDS float* a = (DGMC_LDS float*)sa[wave];
  float sq = 0.f;
  for (int c = lane; c < C8; c += 64) {
    const float v = c < C ? arow[c] : 0.f;
    a[c] = v;
    sq += v * v;
  }
  sq = wave_sum(sq);
  float bm = 0.f;
  for (int p = lane; p < nparts; p += 64)
    bm = fmaxf(bm, nmax_part[(size_t)b * nparts + p]);
  bm = wave_max(bm);
  // |a| |b|max with a relative safety factor for the (any-order) norms.
  const float E = tau * sqrtf(sq * bm) * (1.0f + 1.0f / 1024.0f);
  const size_t o = ((size_t)b * Ns + g);
  const int ci = lane < K2 ? (int)cand_i[o * K2 + lane] : 0;
  const float cv = lane < K2 ? cand_v[o * K2 + lane] : -INFINITY;
  const float Tk = __shfl(cv, k - 1);
  const float lim = Tk - 2.0f * E;
  const bool keep = lane < K2 && cv >= lim;
  // Fewer than k kept (non-finite scores: NaN compares false) or a possibly
  // incomplete list -> the exhaustive scan, which always writes k valid
  // indices.
  const bool overflow = (K2 < Nt && __shfl(cv, K2 - 1) >= lim) ||
                        __popcll(__ballot(keep)) < k;
  __builtin_amdgcn_wave_barrier();
  const float* tb = h_t + (size_t)b * Nt * C;
  int64_t* orow = out + o * k;
  if (!overflow) {
    const float ev = keep ? exact_dot(a, tb + (size_t)ci * C, C, C8)
                          : -INFINITY;
    // rank by (exact desc, index asc) among the kept candidates
    int rank = 0;
    for (int l = 0; l < K2; ++l) {
      const float ov = __shfl(ev, l);
      const int oj = __shfl(ci, l);
      const bool ok = __shfl((int)keep, l) != 0;
      rank += ok && (ov > ev || (ov == ev && oj < ci));
    }
    if (keep && rank < k) orow[rank] = ci;
    return;
  }
  // Incomplete list: exact scan of every target (wave-parallel over j),
  // insertion into a wave list like topk_dot_kernel (lanes 0..k-1).
  if (lane == 0) atomicAdd(n_overflow, 1);
  float lv = -INFINITY;
  int li = 0;
  for (int j0 = 0; j0 < Nt; j0 += 64) {
    const int j = j0 + lane;
    const float v =
        j < Nt ? exact_dot(a, tb + (size_t)j * C, C, C8) : -INFINITY;
    float thr = __shfl(lv, k - 1);
    unsigned long long mask = __ballot(j < Nt && v > thr);
    while (mask) {
      const int src = __ffsll((long long)mask) - 1;
      mask &= mask - 1;
      const float nv = __shfl(v, src);
      if (!(nv > thr)) continue;
      const int pos = __popcll(__ballot(lane < k && lv >= nv));
      const float pv = __shfl_up(lv, 1);
      const int pi = __shfl_up(li, 1);
      if (lane > pos && lane < k) { lv = pv; li = pi; }
      if (lane == pos) { lv = nv; li = j0 + src; }
      thr = __shfl(lv, k - 1);
    }
  }
  if (lane < k) orow[lane] = li;
}

// Exhaustive exact scan of one row by the whole wave (lanes 0..k-1 keep the
// list, as in topk_dot_kernel) - the fallback of both refine kernels.
__device__ __forceinline__ void refine_exhaustive(
    const DGMC_LDS float* a, const float* __restrict__ tb,
    int64_t* __restrict__ orow, int Nt, int C, int C8, int k) {
  const int lane = threadIdx.x & 63;
  float lv = -INFINITY;
  int li = 0;
  for (int j0 = 0; j0 < Nt; j0 += 64) {
    const int j = j0 + lane;
    const float v =
        j < Nt ? exact_dot(a, tb + (size_t)j * C, C, C8) : -INFINITY;
    float thr = __shfl(lv, k - 1);
    unsigned long long mask = __ballot(j < Nt && v > thr);
    while (mask) {
      const int src = __ffsll((long long)mask) - 1;
      mask &= mask - 1;
      const float nv = __shfl(v, src);
      if (!(nv > thr)) continue;
      const int pos = __popcll(__ballot(lane < k && lv >= nv));
      const float pv = __shfl_up(lv, 1);
      const int pi = __shfl_up(li, 1);
      if (lane > pos && lane < k) { lv = pv; li = pi; }
      if (lane == pos) { lv = nv; li = j0 + src; }
      thr = __shfl(lv, k - 1);
    }
  }
  if (lane < k) orow[lane] = li;
}

// K2 <= 16: four rows per wave (lane group r = lane / 16 re-scores row r's
// candidates, lane c of the group candidate c) - the same exact chains,
// margins, ranks and fallback as topk_refine_kernel, a quarter of the waves.
constexpr int kRef4Waves = 4;
__global__ __launch_bounds__(kRef4Waves * 64) void topk_refine4_kernel(
    const float* __restrict__ h_s, const float* __restrict__ h_t,
    const int64_t* __restrict__ cand_i, const float* __restrict__ cand_v,
    const float* __restrict__ nmax_part, int nparts, int64_t* __restrict__ out,
    int* __restrict__ n_overflow, int Ns, int Nt, int C, int k, int K2,
    float tau) {
  __shared__ __attribute__((aligned(16))) float sa[kRef4Waves][4][264];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int grp = lane >> 4, c = lane & 15;
  const int64_t g0 = ((int64_t)blockIdx.x * kRef4Waves + wave) * 4;
  const int b = blockIdx.y;
  if (g0 >= Ns) return;                  // wave-uniform; no block barrier
  const int64_t g = g0 + grp;
  const bool row_ok = g < Ns;
  const int C8 = (C + 7) & ~7;
  DGMC_LDS float* a = (DGMC_LDS float*)sa[wave][grp];
  float sq = 0.f;
  {
    const float* arow = h_s + ((size_t)b * Ns + (row_ok ? g : g0)) * C;
    for (int e = c; e < C8; e += 16) {
      const float v = e < C ? arow[e] : 0.f;
      a[e] = v;
      sq += v * v;
    }
  }
#pragma unroll
  for (int d = 8; d >= 1; d >>= 1) sq += __shfl_xor(sq, d);   // group sum
  float bm = 0.f;
  for (int p = lane; p < nparts; p += 64)
    bm = fmaxf(bm, nmax_part[(size_t)b * nparts + p]);
  bm = wave_max(bm);
  const float E = tau * sqrtf(sq * bm) * (1.0f + 1.0f / 1024.0f);
  const size_t o = (size_t)b * Ns + (row_ok ? g : g0);
  const bool has = row_ok && c < K2;
  const int ci = has ? (int)cand_i[o * K2 + c] : 0;
  const float cv = has ? cand_v[o * K2 + c] : -INFINITY;
  const int base = grp * 16;
  const float Tk = __shfl(cv, base + k - 1);
  const float lim = Tk - 2.0f * E;
  const bool keep = has && cv >= lim;
  const unsigned gmask = (unsigned)(__ballot(keep) >> base) & 0xffffu;
  const bool overflow = row_ok &&
      ((K2 < Nt && __shfl(cv, base + K2 - 1) >= lim) || __popc(gmask) < k);
  __builtin_amdgcn_wave_barrier();
  const float* tb = h_t + (size_t)b * Nt * C;
  const float ev = keep && !overflow
                       ? exact_dot(a, tb + (size_t)ci * C, C, C8) : -INFINITY;
  int rank = 0;
  for (int l = 0; l < 16; ++l) {
    const float ov = __shfl(ev, base + l);
    const int oj = __shfl(ci, base + l);
    const bool ok = ((gmask >> l) & 1u) != 0;
    rank += ok && (ov > ev || (ov == ev && oj < ci));
  }
  if (keep && !overflow && rank < k) out[o * k + rank] = ci;
  // Incomplete lists: each such row by the whole wave, in row order.
  const unsigned long long ovm = __ballot(overflow && c == 0);
  for (int r = 0; r < 4; ++r) {
    if (!((ovm >> (16 * r)) & 1ull)) continue;
    if (lane == 0) atomicAdd(n_overflow, 1);
    refine_exhaustive((DGMC_LDS float*)sa[wave][r], tb,
                      out + ((size_t)b * Ns + g0 + r) * k, Nt, C, C8, k);
  }
}

// Warm start of the filter from an earlier candidate list `prev` (row
// stride ld, e.g. the previous training step's filter output): per row,
// the K2 <= 16 listed targets are re-scored with the exact chain and
//   warm_i = min_j s_j - E_i    (E_i: the refine kernels' bound on
//                                |approximate - exact| score),
// a lower bound of the row's K2-th approximate score - K2 distinct targets
// have an approximate score >= min_j s_j - E_i.  Rows whose list is not K2
// distinct in-range indices (or any non-finite score) get -inf (cold).
// Four rows per wave, lane c of group r re-scores row r's candidate c.
__global__ __launch_bounds__(kRef4Waves * 64) void topk_warm_kernel(
    const float* __restrict__ h_s, const float* __restrict__ h_t,
    const int64_t* __restrict__ prev, int ld,
    const float* __restrict__ nmax_part, int nparts,
    float* __restrict__ warm, int Ns, int Nt, int C, int K2, float tau) {
  __shared__ __attribute__((aligned(16))) float sa[kRef4Waves][4][264];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int grp = lane >> 4, c = lane & 15;
  const int64_t g0 = ((int64_t)blockIdx.x * kRef4Waves + wave) * 4;
  const int b = blockIdx.y;
  if (g0 >= Ns) return;                  // wave-uniform; no block barrier
  const int64_t g = g0 + grp;
  const bool row_ok = g < Ns;
  const int C8 = (C + 7) & ~7;
  DGMC_LDS float* a = (DGMC_LDS float*)sa[wave][grp];
  float sq = 0.f;
  {
    const float* arow = h_s + ((size_t)b * Ns + (row_ok ? g : g0)) * C;
    for (int e = c; e < C8; e += 16) {
      const float v = e < C ? arow[e] : 0.f;
      a[e] = v;
      sq += v * v;
    }
  }
#pragma unroll
  for (int d = 8; d >= 1; d >>= 1) sq += __shfl_xor(sq, d);   // group sum
  float bm = 0.f;
  for (int p = lane; p < nparts; p += 64)
    bm = fmaxf(bm, nmax_part[(size_t)b * nparts + p]);
  bm = wave_max(bm);
  const float E = tau * sqrtf(sq * bm) * (1.0f + 1.0f / 1024.0f);
  const size_t o = (size_t)b * Ns + (row_ok ? g : g0);
  const bool has = c < K2;
  const int64_t cl = has ? prev[o * ld + c] : 0;
  bool ok = !has || (cl >= 0 && cl < Nt);
  const int ci = ok ? (int)cl : -1 - c;     // (invalid: unique, never used)
  // distinct: no earlier lane of the group holds the same index
  const int base = grp * 16;
  for (int l = 0; l < 16; ++l) {
    const int oj = __shfl(ci, base + l);
    if (has && l < c && oj == ci) ok = false;
  }
  __builtin_amdgcn_wave_barrier();
  const float* tb = h_t + (size_t)b * Nt * C;
  float s = has && ok ? exact_dot(a, tb + (size_t)ci * C, C, C8) : INFINITY;
  if (!has) s = INFINITY;
  if (!(s == s)) ok = false;             // NaN
  float m = ok ? s : -INFINITY;
#pragma unroll
  for (int d = 8; d >= 1; d >>= 1) m = fminf(m, __shfl_xor(m, d));
  const bool all_ok = (unsigned)(__ballot(!ok) >> base & 0xffffu) == 0u;
  if (row_ok && c == 0) {
    const float t = m - E;
    warm[o] = all_ok && t - t == 0.f ? t : -INFINITY;     // finite only
  }
}

static at::Tensor topk_dot_refined(const at::Tensor& h_s,
                                   const at::Tensor& h_t, int64_t k,
                                   at::Tensor* n_overflow,
                                   const at::Tensor* warm_state = nullptr) {
  const int B = h_s.size(0), Ns = h_s.size(1), C = h_s.size(2);
  const int Nt = h_t.size(1);
  // Candidates kept by the filter pass: k + 6 (>= 16), at most 32.  The
  // pass's insertion work grows ~K2 ln(Nt / K2); a row whose K2-th
  // candidate still clears the margin is recomputed exhaustively, so K2
  // only trades filter time against (rare) fallbacks.  DGMC_TOPK_K2
  // overrides (diagnostic build only).
  static const int k2_env = diag_env_int("DGMC_TOPK_K2", 0);
  int K2 = k2_env > 0 ? k2_env : std::max<int>(16, (int)k + 6);
  K2 = std::min(std::min(32, Nt), std::max<int>(K2, (int)k));
  at::Tensor out = at::empty({B, Ns, k}, h_s.options().dtype(at::kLong));
  at::Tensor cnt = at::zeros({1}, h_s.options().dtype(at::kInt));
  if (n_overflow) *n_overflow = cnt;
  const int nparts = (Nt + 255) / 256;
  at::Tensor part = at::empty({B, nparts}, h_s.options());
  if (B > 0 && Nt > 0) {
    hipLaunchKernelGGL(row_sqnorm_max_kernel, dim3(nparts, B), dim3(256), 0,
                       stream(), h_t.data_ptr<float>(), Nt, C,
                       part.data_ptr<float>());
    DGMC_CHECK_LAUNCH();
  }
  at::Tensor warm;
  const bool use_warm = warm_state != nullptr && K2 <= 16 && B > 0 && Ns > 0;
  if (use_warm) {
    warm = at::empty({B, Ns}, h_s.options());
    hipLaunchKernelGGL(topk_warm_kernel,
                       dim3((Ns + 4 * kRef4Waves - 1) / (4 * kRef4Waves), B),
                       dim3(kRef4Waves * 64), 0, stream(),
                       h_s.data_ptr<float>(), h_t.data_ptr<float>(),
                       warm_state->data_ptr<int64_t>(),
                       (int)warm_state->size(2), part.data_ptr<float>(),
                       nparts, warm.data_ptr<float>(), Ns, Nt, C, K2,
                       topk_tau());
    DGMC_CHECK_LAUNCH();
  }
  at::Tensor cv;
  at::Tensor ci = topk_dot_x3(h_s, h_t, K2, &cv, use_warm ? &warm : nullptr);
  if (warm_state != nullptr && B > 0 && Ns > 0)
    warm_state->narrow(2, 0, K2).copy_(ci);       // the next call's start
  if (B == 0 || Ns == 0) return out;
  if (K2 <= 16) {
    hipLaunchKernelGGL(topk_refine4_kernel,
                       dim3((Ns + 4 * kRef4Waves - 1) / (4 * kRef4Waves), B),
                       dim3(kRef4Waves * 64), 0, stream(),
                       h_s.data_ptr<float>(), h_t.data_ptr<float>(),
                       ci.data_ptr<int64_t>(), cv.data_ptr<float>(),
                       part.data_ptr<float>(), nparts,
                       out.data_ptr<int64_t>(), cnt.data_ptr<int>(), Ns, Nt, C,
                       (int)k, K2, topk_tau());
    DGMC_CHECK_LAUNCH();
    return out;
  }
  hipLaunchKernelGGL(topk_refine_kernel,
                     dim3((Ns + kRefRows - 1) / kRefRows, B),
                     dim3(kRefRows * 64), 0, stream(), h_s.data_ptr<float>(),
                     h_t.data_ptr<float>(), ci.data_ptr<int64_t>(),
                     cv.data_ptr<float>(), part.data_ptr<float>(), nparts,
                     out.data_ptr<int64_t>(), cnt.data_ptr<int>(), Ns, Nt, C,
                     (int)k, K2, topk_tau());
  DGMC_CHECK_LAUNCH();
  return out;
}

// (The kernels' dbg argument - 1 skip selection, 2 skip MFMA - is an
// ablation knob: DGMC_TOPK_DEBUG, diagnostic build only.)
static int topk_debug() {
  static const int v = diag_env_int("DGMC_TOPK_DEBUG", 0);
  return v;
}

// Target splits for the bf16x3 kernel: the smallest S whose blocks fill the
// per_cu-blocks-per-CU slots of the chip to >= 85% (a partial last wave of blocks
// idles CUs), keeping every split >= 2 tiles.
static int x3_splits(int64_t row_blocks, int Nt, int per_cu) {
  const int64_t slots = (int64_t)per_cu * 256;
  int best = 1;
  double best_eff = 0.0;
  for (int S = 1; S <= 16; ++S) {
    if (S > 1 && (int64_t)S * 2 * kX3Tile > Nt) break;
    const int64_t blocks = row_blocks * S;
    const double eff =
        (double)blocks / (double)(slots * ((blocks + slots - 1) / slots));
    if (eff >= 0.85) return S;
    if (eff > best_eff + 1e-9) { best_eff = eff; best = S; }
  }
  return best;
}

static at::Tensor topk_dot_x3(const at::Tensor& h_s, const at::Tensor& h_t,
                              int64_t k, at::Tensor* vals,
                              const at::Tensor* warm) {
  const int B = h_s.size(0), Ns = h_s.size(1), C = h_s.size(2);
  const int Nt = h_t.size(1);
  at::Tensor out = at::empty({B, Ns, k}, h_s.options().dtype(at::kLong));
  if (vals) *vals = at::empty({B, Ns, k}, h_s.options());
  float* out_v = vals ? vals->data_ptr<float>() : nullptr;
  if (B == 0 || Ns == 0) return out;
  const int NKS = (C + 63) / 64 * 4;
  const int CP = NKS * 16;
  TORCH_CHECK((int64_t)Nt * CP * 2 < ((int64_t)1 << 32),
              "topk_dot_x3: N_t x C too large for 32-bit plane offsets");
  const size_t lds = (size_t)4 * kX3Tile * (CP + 8) * sizeof(__bf16);
  const int W = (NKS == 8 || NKS == 16) ? 8 : 4;
  const int row_blocks = (Ns + 32 * W - 1) / (32 * W);
  int S = x3_splits((int64_t)row_blocks * B, Nt, W == 8 ? 1 : 2);
  {
    // DGMC_TOPK_SPLITS: diagnostic build only
    static const int s_env = diag_env_int("DGMC_TOPK_SPLITS", 0);
    if (s_env > 0) S = s_env;
  }
  int span = (Nt + S - 1) / S;
  span = (span + kX3Tile - 1) / kX3Tile * kX3Tile;
  S = (Nt + span - 1) / span;
  if (S > 1 && Nt - (S - 1) * span < (int)k) S = 1, span = Nt;  // tiny tails
  at::Tensor pv, pi;
  if (S > 1) {
    pv = at::empty({(int64_t)B * Ns * S * k}, h_s.options());
    pi = at::empty({(int64_t)B * Ns * S * k}, h_s.options().dtype(at::kInt));
  }
  // bf16 hi / lo planes of h_t (read by every row block: split once).
  at::Tensor planes = at::empty({2, (int64_t)B * Nt, CP},
                                h_s.options().dtype(at::kBFloat16));
  {
    const int64_t rows = (int64_t)B * Nt;
    const int64_t n = rows * (CP / 4);
    __bf16* hi = reinterpret_cast<__bf16*>(planes.data_ptr());
    hipLaunchKernelGGL(split_bf16_kernel, dim3((unsigned)((n + 255) / 256)),
                       dim3(256), 0, stream(), h_t.data_ptr<float>(), hi,
                       hi + rows * CP, rows, C, CP);
    DGMC_CHECK_LAUNCH();
  }
  const __bf16* t_hi = reinterpret_cast<const __bf16*>(planes.data_ptr());
  const __bf16* t_lo = t_hi + (int64_t)B * Nt * CP;
  dim3 grid(row_blocks, S, B);
  auto launch = [&](auto kernel) {
    DGMC_CHECK_HIP(hipFuncSetAttribute(
        reinterpret_cast<const void*>(kernel),
        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(kernel, grid, dim3(64 * W), lds, stream(),
                       h_s.data_ptr<float>(), t_hi, t_lo,
                       S > 1 ? pv.data_ptr<float>() : nullptr,
                       S > 1 ? pi.data_ptr<int>() : nullptr,
                       out.data_ptr<int64_t>(), out_v, Ns, Nt, C, (int)k,
                       span, topk_debug(),
                       warm ? warm->data_ptr<float>() : nullptr);
  };
  switch (NKS) {
    case 4: launch(topk_x3_kernel<4, 4>); break;
    case 8: launch(topk_x3_kernel<8, 8>); break;
    case 12: launch(topk_x3_kernel<12, 4>); break;
    default: launch(topk_x3_kernel<16, 8>); break;
  }
  DGMC_CHECK_LAUNCH();
  if (S > 1 && S * k <= 64) {
    const int64_t rows = (int64_t)B * Ns;
    hipLaunchKernelGGL(topk_merge_wave_kernel,
                       dim3((unsigned)((rows + 3) / 4)), dim3(256), 0,
                       stream(), pv.data_ptr<float>(), pi.data_ptr<int>(),
                       out.data_ptr<int64_t>(), out_v, rows, S, (int)k, Nt);
    DGMC_CHECK_LAUNCH();
  } else if (S > 1) {
    const int64_t rows = (int64_t)B * Ns;
    const int64_t n = rows * S * k;
    hipLaunchKernelGGL(topk_merge_kernel, dim3((unsigned)((n + 255) / 256)),
                       dim3(256), 0, stream(), pv.data_ptr<float>(),
                       pi.data_ptr<int>(), out.data_ptr<int64_t>(), out_v,
                       rows, S, (int)k, Nt);
    DGMC_CHECK_LAUNCH();
  }
  return out;
}

// mode 0: split-bf16 scores (~2^-16 relative); 1: brute-force exact-f32 MFMA;
// 2 (default): exact - the split-bf16 filter + exact re-score above, with
// the brute-force kernel where the filter does not apply (k > 32).
at::Tensor topk_dot(const at::Tensor& h_s, const at::Tensor& h_t, int64_t k,
                    int64_t mode, const c10::optional<at::Tensor>& warm) {
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
  if (mode == 0 && k <= 32) return topk_dot_x3(h_s, h_t, k);
  if (mode == 2 && k <= 16) {
    const at::Tensor* ws = nullptr;
    if (warm.has_value() && warm->defined()) {
      // int64 [B, N_s, >= K2] candidate state (any content: entries that are
      // not K2 distinct in-range indices only disable the warm start)
      TORCH_CHECK(warm->is_cuda() && warm->scalar_type() == at::kLong &&
                      warm->dim() == 3 && warm->size(0) == B &&
                      warm->size(1) == Ns && warm->size(2) >= 32 &&
                      warm->is_contiguous(),
                  "topk_dot: warm state int64 [B, N_s, 32]");
      ws = &*warm;
    }
    return topk_dot_refined(h_s, h_t, k, nullptr, ws);
  }
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
                       out.data_ptr<int64_t>(), Ns, Nt, C, (int)k,
                       topk_debug());
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

// Test hook: the refined result plus the number of rows that took the
// exhaustive exact path.
std::vector<at::Tensor> topk_dot_refined_stats(const at::Tensor& h_s,
                                               const at::Tensor& h_t,
                                               int64_t k) {
  TORCH_CHECK(h_s.is_cuda() && h_s.dim() == 3 && h_s.is_contiguous() &&
                  h_t.is_contiguous() && h_s.scalar_type() == at::kFloat &&
                  h_t.scalar_type() == at::kFloat && h_t.size(0) == h_s.size(0)
                  && h_t.size(2) == h_s.size(2),
              "topk_dot_refined_stats: contiguous fp32 [B, N, C]");
  TORCH_CHECK(k >= 1 && k <= 16 && k <= h_t.size(1) && h_s.size(2) % 4 == 0 &&
                  h_s.size(2) <= 256,
              "topk_dot_refined_stats: 1 <= k <= 16, C % 4 == 0, C <= 256");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(h_s.device());
  at::Tensor cnt;
  at::Tensor idx = topk_dot_refined(h_s, h_t, k, &cnt);
  return {idx, cnt};
}

}  // namespace dgmc
