// Fused slot-structured graph convolution on graph-closed row tiles:
//
//   out[i, :] = act( sum_k (A_k X)[i, :] W_k + bias )          (forward)
//   dX[j, :]  =      sum_k (A_k^T G)[j, :] W_k^T                (backward)
//
// A_k is the slot-k part of SplineConv's message operator (B-spline slot k of
// 5^dim, plus the root slot as the identity) - /root/reference/dgmc/models/
// spline.py:49 over PyG SplineConv / torch_spline_conv.  The unfused path
// (ops/sparse.py) writes Y = X [W_0 | .. | W_{S-1}] ([N, S*C], 73 MB for
// psi_2 at batch 512) and gathers it back (GEMM + SpMM); the backward writes
// dY = A^T G and reads it again for dX.
//
// Design (gfx950, v_mfma_f32_16x16x32_bf16, one workgroup = 4 waves = one
// tile of <= 64 rows):
//
// * Tiles are GRAPH-CLOSED: every entry of a tile row references a source row
//   inside the tile.  Batches are disjoint unions of small graphs, so tile t
//   is [first graph start >= t*window, first graph start >= (t+1)*window);
//   with window = 65 - n_max a tile never exceeds 64 rows.  The row flags
//   (1 = a graph starts here) come from the plan (csrc/hip/plan_assembly.hip).
// * slot_tile_plan (once per operator, i.e. once per training step for all
//   2 x 10 psi_2 uses and their backward): tile bounds and the tile's entries
//   bucketed by slot, packed (dst << 8 | src) + bf16 value.
// * slot_conv, per slot: the tile's part of A_k is scattered into a DENSE
//   64x64 bf16 LDS tile (triple-buffered, entries prefetched one slot ahead),
//   so the sparse gather is MFMA work:  Z_k^T = X^T A_k^T  (X^T fragments are
//   loaded once per tile and stay in registers).
// * The MFMA accumulator layout (lane holds 4 consecutive rows of one column)
//   is reused directly as the B operand of the second product
//   out^T += W_k^T Z_k^T  by permuting the K order inside each 32-wide chunk;
//   the weight image is pre-permuted the same way on the host
//   (ops/sparse.py::slot_conv_image), so Z never touches LDS or HBM.
// * W_k^T images (32 KB) stream global -> LDS with global_load_lds (no VGPR
//   round trip), double-buffered, XOR-swizzled through the source address so
//   the fragment reads are bank-conflict free.  One barrier per slot.
// * Backward: the same kernel with A_k^T (scatter transposed) and the
//   transposed weight image; optionally writes dY = A^T G (the Z_k tiles) for
//   the stacked weight-gradient GEMM.
#include "common.h"

#include <type_traits>

namespace dgmc {

namespace {

typedef __bf16 sc_bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 sc_bf16x4 __attribute__((ext_vector_type(4)));
typedef float sc_f32x4 __attribute__((ext_vector_type(4)));
typedef const void __attribute__((address_space(1)))* sc_gptr;

constexpr int kScC = 128;        // channels (in == out)
constexpr int kScT = 64;         // max rows per tile
constexpr int kScAP = 72;        // padded LDS row of the A / X^T tiles (bf16)
constexpr int kScThreads = 256;  // tile plan: 4 waves
constexpr int kScCT = 512;       // conv: 8 waves (2 per SIMD)
constexpr int kScWaves = kScCT / 64;
constexpr int kScMaxS = 63;      // slots per operator (one lane each)
constexpr int kScECap = 4096;    // tile entries staged in LDS
constexpr int kScWImg = kScC * kScC;               // bf16 elements per slot
constexpr int kScATile = kScT * kScAP;             // bf16 elements per A tile
constexpr size_t kScLds = (size_t)2 * kScWImg * 2 + (size_t)3 * kScATile * 2 +
                          (size_t)kScC * kScAP * 2 + (size_t)kScECap * 6 +
                          kScC * 4 + 16;

__device__ __forceinline__ int sc_first_flag(const uint8_t* __restrict__ flag,
                                             int b, int N, int lane) {
  // First row r >= b with flag[r] (N counts as flagged); -1 if none of the
  // 64 rows [b, b + 64) qualifies.
  if (b >= N) return N;
  const int r = b + lane;
  const bool f = r >= N || flag[r] != 0;
  const unsigned long long m = __ballot(f);
  return m ? min(b + (int)__builtin_ctzll(m), N) : -1;
}

}  // namespace

// In-kernel wall-clock stamps of workgroups 0 and 1 (DGMC_SC_DEBUG & 8):
// entry, prologue done, slot-0 tile ready, loop done, exit.
__device__ long long g_sc_stamps[16];
#define SC_STAMP(i)                                                      \
  if ((dbg & 8) && blockIdx.x < 2 && tid == 0)                           \
    g_sc_stamps[8 * blockIdx.x + (i)] = wall_clock64();

// ---------------------------------------------------------------------------
// Tile plan: tiles [T, 4] = (r0, r1, first entry, entries | largest slot
// bucket << 16); soff [T, S + 1] slot
// offsets inside the tile's entry range; ecode/eval [nnz] the tile's entries
// bucketed by slot (dst << 8 | src, bf16 value).  One workgroup per tile; the
// order inside a bucket is irrelevant (entries of a slot are distinct dense
// positions), so LDS atomics assign positions.
__global__ __launch_bounds__(kScThreads) void slot_tile_plan_kernel(
    const uint8_t* __restrict__ flag, const int* __restrict__ rowptr,
    const int* __restrict__ col, const float* __restrict__ val, int N,
    int window, int S, int* __restrict__ tiles, int* __restrict__ soff,
    int* __restrict__ ecode, __hip_bfloat16* __restrict__ eval,
    int* __restrict__ err) {
  __shared__ int rp[kScT + 1];
  __shared__ int cnt[kScMaxS + 1];
  __shared__ int bounds[2];
  const int t = blockIdx.x, tid = threadIdx.x;
  if (tid < 64) {
    const int b0 = t * window;
    const int r0 = sc_first_flag(flag, b0, N, tid);
    const int r1 = sc_first_flag(flag, b0 + window, N, tid);
    if (tid == 0) {
      bounds[0] = r0;
      bounds[1] = r1;
    }
  }
  for (int k = tid; k <= S; k += kScThreads) cnt[k] = 0;
  __syncthreads();
  int r0 = bounds[0], r1 = bounds[1];
  if (r0 < 0 || r1 < 0 || r1 - r0 > kScT) {
    if (tid == 0) atomicOr(err, 1);   // window too large for the graphs
    r0 = r1 = max(r0, 0);             // empty tile: its rows stay unwritten
  }
  const int rows = max(r1 - r0, 0);
  for (int i = tid; i <= rows; i += kScThreads) rp[i] = rowptr[r0 + i];
  __syncthreads();
  const int e0 = rp[0], E = rp[rows] - rp[0];
  if (E > 0xFFFF) {                   // E is packed into 16 bits below
    if (tid == 0) atomicOr(err, 4);
  }
  if (tid == 0) {
    tiles[4 * t + 0] = r0;
    tiles[4 * t + 1] = r0 + rows;
    tiles[4 * t + 2] = e0;
  }
  auto decode = [&](int e, int& k) -> int {
    int lo = 0, hi = rows;            // rp[lo] <= e0 + e < rp[hi]
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (rp[mid] <= e0 + e) lo = mid; else hi = mid;
    }
    const int c = col[e0 + e];
    const int j = c / S;
    k = c - j * S;
    const int sl = j - r0;
    if (sl < 0 || sl >= rows) {       // tile is not graph-closed
      atomicOr(err, 2);
      k = S;                          // parked in an unused bucket
    }
    return (lo << 8) | (sl & 255);
  };
  for (int e = tid; e < E; e += kScThreads) {
    int k;
    decode(e, k);
    atomicAdd(&cnt[k], 1);
  }
  __syncthreads();
  if (tid == 0) {
    int run = 0, most = 0;
    for (int k = 0; k <= S; ++k) {
      const int c = cnt[k];
      if (k < S) most = max(most, c);
      cnt[k] = run;
      soff[t * (S + 1) + k] = run;
      run += c;
    }
    tiles[4 * t + 3] = E | (most << 16);   // E, largest slot bucket
  }
  __syncthreads();
  for (int e = tid; e < E; e += kScThreads) {
    int k;
    const int code = decode(e, k);
    const int pos = atomicAdd(&cnt[k], 1);
    ecode[e0 + pos] = code;
    eval[e0 + pos] = __float2bfloat16(val[e0 + e]);
  }
}

// ---------------------------------------------------------------------------
template <bool TRANS, bool WRITE_Z, typename TOUT>
__global__ __launch_bounds__(kScCT, 1) void slot_conv_kernel(
    const __hip_bfloat16* __restrict__ Xg, const int* __restrict__ tiles,
    const int* __restrict__ soff, const int* __restrict__ ecode,
    const __hip_bfloat16* __restrict__ evalg, int S,
    const __hip_bfloat16* __restrict__ Wimg, const float* __restrict__ bias,
    int relu, TOUT* __restrict__ out, __hip_bfloat16* __restrict__ Zg,
    const __hip_bfloat16* __restrict__ addg, int ldadd, int dbg) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  DGMC_LDS char* smem = (DGMC_LDS char*)smem_raw;
  DGMC_LDS __bf16* wbuf = (DGMC_LDS __bf16*)smem;        // [2][128][128]
  DGMC_LDS __bf16* abuf = wbuf + 2 * kScWImg;             // [3][64][72]
  DGMC_LDS __bf16* xt = abuf + 3 * kScATile;              // [128][72]
  DGMC_LDS int* ecs = (DGMC_LDS int*)(xt + kScC * kScAP); // [kScECap]
  DGMC_LDS __bf16* evs = (DGMC_LDS __bf16*)(ecs + kScECap);  // [kScECap]
  DGMC_LDS float* bsh = (DGMC_LDS float*)(evs + kScECap);    // [128]
  DGMC_LDS __bf16* junk = (DGMC_LDS __bf16*)(bsh + kScC);    // [8] sink

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int ln = lane & 15, lq = lane >> 4;
  const __bf16* X = reinterpret_cast<const __bf16*>(Xg);
  const __bf16* W = reinterpret_cast<const __bf16*>(Wimg);
  const __bf16* ev = reinterpret_cast<const __bf16*>(evalg);

  SC_STAMP(0);
  const int t = blockIdx.x;
  const int r0 = tiles[4 * t], rows = tiles[4 * t + 1] - r0;
  const int e0 = tiles[4 * t + 2];
  const int E = tiles[4 * t + 3] & 0xffff, most = tiles[4 * t + 3] >> 16;
  if (rows <= 0) return;              // no graph starts in this window

  // W_k image -> wbuf[k & 1] (async).  LDS chunk p (16 B) of row p/16 holds
  // global chunk (p%16) ^ (row%16) of that row.
  int woff[kScWImg / 8 / kScCT];   // per-lane source offsets (loop-
#pragma unroll                           // invariant)
  for (int i = 0; i < kScWImg / 8 / kScCT; ++i) {
    const int p = (i * kScWaves + wave) * 64 + lane;
    const int row = p >> 4, jj = p & 15;
    woff[i] = row * kScC + ((jj ^ (row & 15)) << 3);
  }
  auto load_w = [&](int k) __attribute__((always_inline)) {
    const __bf16* src = W + (size_t)k * kScWImg;
    DGMC_LDS __bf16* dst = wbuf + (k & 1) * kScWImg;
#pragma unroll
    for (int i = 0; i < kScWImg / 8 / kScCT; ++i)
      __builtin_amdgcn_global_load_lds(
          (sc_gptr)(src + woff[i]),
          (DGMC_LDS void*)(dst + (i * kScWaves + wave) * 64 * 8), 16, 0, 0);
  };

  // ---- prologue ------------------------------------------------------------
  // Slot offsets: lane k of every wave holds soff[t][k] (read back with a
  // scalar readlane - no memory access in the slot loop).
  const int sof_v = lane <= S ? soff[t * (S + 1) + lane] : 0;
  auto sof = [&](int k) __attribute__((always_inline)) {
    return __builtin_amdgcn_readlane(sof_v, k);
  };
  const bool staged = E <= kScECap;   // entries in LDS (else read from L2)
  if (staged)
    for (int e = tid; e < E; e += kScCT) {
      ecs[e] = ecode[e0 + e];
      evs[e] = ev[e0 + e];
    }
  load_w(0);
  if (tid < kScC) bsh[tid] = bias ? bias[tid] : 0.f;
  {
    const sc_bf16x8 z = {};
    for (int i = tid; i < 3 * kScATile / 8; i += kScCT)
      *reinterpret_cast<DGMC_LDS sc_bf16x8*>(abuf + i * 8) = z;
  }
  // X rows r0..r0+63 -> xt[ch][row] (rows >= `rows` are zero).
#pragma unroll
  for (int i = 0; i < kScT * kScC / 8 / kScCT; ++i) {
    const int c = tid + i * kScCT;
    const int row = c & 63, cc = c >> 6;
    sc_bf16x8 v = {};
    if (row < rows)
      v = *reinterpret_cast<const sc_bf16x8*>(X + (size_t)(r0 + row) * kScC +
                                              cc * 8);
#pragma unroll
    for (int e = 0; e < 8; ++e) xt[(cc * 8 + e) * kScAP + row] = v[e];
  }
  __syncthreads();
  SC_STAMP(1);

  // X^T fragments (A operand of Z^T = X^T A_k^T): block m = channels
  // 16m..16m+15, chunk c = tile rows 32c..32c+31.
  sc_bf16x8 xa[8][2];
#pragma unroll
  for (int m = 0; m < 8; ++m)
#pragma unroll
    for (int c = 0; c < 2; ++c)
      xa[m][c] = *reinterpret_cast<DGMC_LDS const sc_bf16x8*>(
          xt + (16 * m + ln) * kScAP + 32 * c + 8 * lq);

  // A-tile maintenance: scatter (or clear) the entries of slot k into
  // buffer k % 3 (dense [dst][src], transposed for the backward).
  auto scatter = [&](int k, bool clear) __attribute__((always_inline)) {
    DGMC_LDS __bf16* tile = abuf + (k % 3) * kScATile;
    const int hi = sof(k + 1);
    for (int e = sof(k) + tid; e < hi; e += kScCT) {
      const int code = staged ? ecs[e] : ecode[e0 + e];
      const __bf16 v = clear ? (__bf16)0.f : (staged ? evs[e] : ev[e0 + e]);
      const int dl = code >> 8, sl = code & 255;
      tile[TRANS ? sl * kScAP + dl : dl * kScAP + sl] = v;
    }
  };
  scatter(0, false);

  sc_f32x4 ot[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) ot[m] = sc_f32x4{0.f, 0.f, 0.f, 0.f};
  // Wave w: tile rows 16 (w % 4) .. +15, output channels 64 (w / 4) .. +63
  // (Z_k is computed by both waves of a row block: MFMA is cheap, a second
  // wave per SIMD hides the LDS / DMA / barrier latencies of the first).
  const int node = 16 * (wave & 3) + ln;         // this lane's tile row
  const int oh = wave >> 2;                       // output-channel half
  __syncthreads();                                // W_0, A_0 ready
  SC_STAMP(2);

  // One slot step.  FAST (every slot bucket of the tile fits one entry per
  // thread): the A-tile maintenance is branch-free (idle lanes write a sink
  // word), so scatter, W DMA and MFMAs form one basic block that the
  // schedule below interleaves - one wave per SIMD has nothing else to
  // hide the LDS and issue latencies behind.
  auto step = [&](int k, auto fast_tag) __attribute__((always_inline)) {
    constexpr bool FAST = decltype(fast_tag)::value;
    if constexpr (FAST) {
      if (!(dbg & 4)) {
        // Before this step's LDS DMA, so the stores need no wait on it:
        // buffer (k-1)%3 is free (slot k-1 done before the last barrier),
        // buffer (k+1)%3 was cleared at step k-1.
        const int ec = (k >= 1 ? sof(k - 1) : 0) + tid;
        const bool vc = k >= 1 && ec < sof(k);
        const int es = sof(k + 1) + tid;
        const bool vs = k + 1 < S && es < sof(k + 2);
        const int cc = ecs[vc ? ec : 0];
        const int cs = ecs[vs ? es : 0];
        const __bf16 v = evs[vs ? es : 0];
        auto pos = [&](int code) {
          const int dl = code >> 8, sl = code & 255;
          return TRANS ? sl * kScAP + dl : dl * kScAP + sl;
        };
        DGMC_LDS __bf16* pc =
            vc ? abuf + ((k + 2) % 3) * kScATile + pos(cc) : junk;
        DGMC_LDS __bf16* ps =
            vs ? abuf + ((k + 1) % 3) * kScATile + pos(cs) : junk;
        *pc = (__bf16)0.f;
        *ps = v;
      }
      // Last step: a harmless reload of slot S-1 into the free buffer.
      load_w(min(k + 1, S - 1));
    } else {
      if (!(dbg & 4)) {
        if (k >= 1) scatter(k - 1, true);
        if (k + 1 < S) scatter(k + 1, false);
      }
      if (k + 1 < S) load_w(k + 1);
    }

    // Z_k^T = X^T A_k^T  (16 x 16 blocks: channels x this wave's rows).
    // Waves past the tile's rows multiply zero tiles (their SIMD is idle
    // otherwise; a uniform body keeps the accumulators in AGPRs).
    DGMC_LDS const __bf16* at =
        abuf + (k % 3) * kScATile + node * kScAP + 8 * lq;
    const sc_bf16x8 b0 = *reinterpret_cast<DGMC_LDS const sc_bf16x8*>(at);
    const sc_bf16x8 b1 = *reinterpret_cast<DGMC_LDS const sc_bf16x8*>(at + 32);
    DGMC_LDS const __bf16* wb = wbuf + (k & 1) * kScWImg + ln * kScC;
    sc_bf16x8 wf[2][4];
#pragma unroll
    for (int m = 0; m < 4; ++m)   // W fragments of chunk 0, in flight early
      wf[0][m] = *reinterpret_cast<DGMC_LDS const sc_bf16x8*>(
          wb + (4 * oh + m) * 16 * kScC + ((lq ^ ln) << 3));
    sc_f32x4 zt[8];
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      zt[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
          xa[m][0], b0, sc_f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      zt[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xa[m][1], b1, zt[m], 0,
                                                      0, 0);
    }
    // Accumulator -> B operand: chunk c covers channels
    // {32c + 4q + r} u {32c + 16 + 4q + r} in lane group q.
    sc_bf16x8 zb[4];
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        zb[c][r] = (__bf16)zt[2 * c][r];
        zb[c][4 + r] = (__bf16)zt[2 * c + 1][r];
      }
    if constexpr (WRITE_Z) {
      if (oh == 0 && node < rows) {
        __bf16* zr = reinterpret_cast<__bf16*>(Zg) +
                     ((size_t)(r0 + node) * S + k) * kScC + 4 * lq;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const sc_bf16x4 lo = {zb[c][0], zb[c][1], zb[c][2], zb[c][3]};
          const sc_bf16x4 hi = {zb[c][4], zb[c][5], zb[c][6], zb[c][7]};
          *reinterpret_cast<sc_bf16x4*>(zr + 32 * c) = lo;
          *reinterpret_cast<sc_bf16x4*>(zr + 32 * c + 16) = hi;
        }
      }
    }
    // out^T += W_k^T Z_k^T, W fragments of chunk c+1 read during chunk c.
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      if (c + 1 < 4) {
#pragma unroll
        for (int m = 0; m < 4; ++m)
          wf[(c + 1) & 1][m] = *reinterpret_cast<DGMC_LDS const sc_bf16x8*>(
              wb + (4 * oh + m) * 16 * kScC +
              (((4 * (c + 1) + lq) ^ ln) << 3));
      }
#pragma unroll
      for (int m = 0; m < 4; ++m)
        ot[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[c & 1][m], zb[c],
                                                        ot[m], 0, 0, 0);
    }
    // Schedule: LDS fragment reads run ahead of the MFMAs that consume them
    // (one wave per SIMD: nothing else hides their latency).
    if constexpr (FAST) {
      __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);  // entry codes
      __builtin_amdgcn_sched_group_barrier(0x200, 2, 0);  // A-tile stores
    }
    __builtin_amdgcn_sched_group_barrier(0x100, 6, 0);    // A + W chunk 0
#pragma unroll
    for (int i = 0; i < 4; ++i) {                          // MFMA1 + chunk 1
      __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);   // (+ W_{k+1} DMA)
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      if constexpr (FAST) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {                          // MFMA2 + chunks 2-3
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
    __syncthreads();   // drains W_{k+1} (vmcnt) and publishes A_{k+1}
  };
  if (staged && most <= kScCT) {
    for (int k = 0; k < S; ++k) step(k, std::true_type{});
  } else {
    for (int k = 0; k < S; ++k) step(k, std::false_type{});
  }

  SC_STAMP(3);
  // ---- epilogue: lane holds out[node][16m + 4q + r] ------------------------
  if (node >= rows) return;
  TOUT* orow = out + (size_t)(r0 + node) * kScC + 64 * oh + 4 * lq;
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    float v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      v[r] = ot[m][r] + bsh[64 * oh + 16 * m + 4 * lq + r];
    }
    if (addg) {   // fused gradient accumulation (a second consumer's dX)
      const sc_bf16x4 ad = *reinterpret_cast<const sc_bf16x4*>(
          reinterpret_cast<const __bf16*>(addg) +
          (size_t)(r0 + node) * ldadd + 64 * oh + 16 * m + 4 * lq);
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] += (float)ad[r];
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (relu) v[r] = fmaxf(v[r], 0.f);
    }
    if constexpr (sizeof(TOUT) == 2) {
      const sc_bf16x4 o = {(__bf16)v[0], (__bf16)v[1], (__bf16)v[2],
                           (__bf16)v[3]};
      *reinterpret_cast<sc_bf16x4*>(orow + 16 * m) = o;
    } else {
      *reinterpret_cast<sc_f32x4*>(orow + 16 * m) =
          sc_f32x4{v[0], v[1], v[2], v[3]};
    }
  }
  SC_STAMP(4);
}

// ---------------------------------------------------------------------------
// Wave-specialised variant (no Z output): waves 0-3 are MFMA waves, each owns
// 16 tile rows and ALL 128 output channels (Z_k computed once per row block,
// no duplicate), waves 4-7 are helpers that clear / scatter the A tiles and
// issue the W_{k+1} DMA while the MFMA waves run slot k.  One barrier per
// slot; the ablations of the 8-wave kernel (docs/performance.md) showed its
// DMA, scatter and MFMA phases adding up instead of overlapping.
constexpr size_t kScLdsWs = (size_t)3 * kScWImg * 2 +
                            (size_t)3 * kScATile * 2 + (size_t)kScECap * 6 +
                            kScC * 4 + 16;
static_assert(kScC * kScAP <= 3 * kScATile, "xt must fit the A tiles");

// Raw workgroup barrier of the wave-specialised kernel (no implicit
// waitcnt: each role drains exactly the counters it must before arriving).
// The empty asm statements with a memory clobber are compiler fences: no LDS
// access of one slot step may be scheduled across the barrier into another
// (s_barrier alone is not a memory operation to the optimiser).
__device__ __forceinline__ void sc_raw_barrier() {
  // (drains this wave's LDS reads: see slot_gemm_x6.hip::x6_barrier)
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <bool TRANS, typename TOUT>
__global__ __launch_bounds__(kScCT, 1) void slot_conv_ws_kernel(
    const __hip_bfloat16* __restrict__ Xg, const int* __restrict__ tiles,
    const int* __restrict__ soff, const int* __restrict__ ecode,
    const __hip_bfloat16* __restrict__ evalg, int S,
    const __hip_bfloat16* __restrict__ Wimg, const float* __restrict__ bias,
    int relu, TOUT* __restrict__ out, const __hip_bfloat16* __restrict__ addg,
    int ldadd, int ldx, const __hip_bfloat16* __restrict__ maskg,
    __hip_bfloat16* __restrict__ goutg, float* __restrict__ bpart) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  DGMC_LDS char* smem = (DGMC_LDS char*)smem_raw;
  DGMC_LDS __bf16* wbuf = (DGMC_LDS __bf16*)smem;        // [3][128][128]
  DGMC_LDS __bf16* abuf = wbuf + 3 * kScWImg;             // [3][64][72]
  DGMC_LDS __bf16* xt = abuf;                 // [128][72], prologue only
  DGMC_LDS int* ecs = (DGMC_LDS int*)(abuf + 3 * kScATile); // [kScECap]
  DGMC_LDS __bf16* evs = (DGMC_LDS __bf16*)(ecs + kScECap);  // [kScECap]
  DGMC_LDS float* bsh = (DGMC_LDS float*)(evs + kScECap);    // [128]

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int ln = lane & 15, lq = lane >> 4;
  // Roles: waves 0-3 MFMA, 4-5 A-tile maintenance (LDS only), 6-7 W DMA
  // (global_load_lds only, never an LDS read: nothing makes them wait on
  // their own DMA except the counted wait before the barrier).
  const bool mw = wave < 4;
  const bool sw = wave == 4 || wave == 5;
  const int sid = tid - 256, did = tid - 384;
  const __bf16* X = reinterpret_cast<const __bf16*>(Xg);
  const __bf16* W = reinterpret_cast<const __bf16*>(Wimg);
  const __bf16* ev = reinterpret_cast<const __bf16*>(evalg);

  const int t = blockIdx.x;
  const int r0 = tiles[4 * t], rows = tiles[4 * t + 1] - r0;
  const int e0 = tiles[4 * t + 2];
  const int E = tiles[4 * t + 3] & 0xffff;
  if (rows <= 0) {                    // empty tile (no graph starts in it)
    if constexpr (TRANS) {
      if (bpart && tid < kScC) bpart[(size_t)t * kScC + tid] = 0.f;
    }
    return;
  }

  const int sof_v = lane <= S ? soff[t * (S + 1) + lane] : 0;
  auto sof = [&](int k) __attribute__((always_inline)) {
    return __builtin_amdgcn_readlane(sof_v, k);
  };
  const bool staged = E <= kScECap;
  // W_k image (rows = output channels) -> wbuf[k & 1]; LDS chunk p (16 B)
  // of row p/16 holds global chunk (p%16) ^ (row%16).  nthr threads from
  // thread index i0 issue it (all 512 in the prologue, the helpers later).
  // The thread count is a compile-time constant: the unrolled pieces then
  // have provably disjoint LDS targets (a runtime count made the compiler
  // wait vmcnt(0) between consecutive global_load_lds).
  auto load_w = [&](int k, int i, auto nthr_c) __attribute__((always_inline)) {
    constexpr int nthr = decltype(nthr_c)::value;
    const __bf16* src = W + (size_t)k * kScWImg;
    DGMC_LDS __bf16* dst = wbuf + (k % 3) * kScWImg;
    const int wv = i >> 6;
    constexpr int nw = nthr >> 6;
#pragma unroll
    for (int j = 0; j < kScWImg / 8 / nthr; ++j) {
      const int p = (j * nw + wv) * 64 + (i & 63);
      const int row = p >> 4, jj = p & 15;
      __builtin_amdgcn_global_load_lds(
          (sc_gptr)(src + row * kScC + ((jj ^ (row & 15)) << 3)),
          (DGMC_LDS void*)(dst + (j * nw + wv) * 64 * 8), 16, 0, 0);
    }
  };
  auto scatter = [&](int k, bool clear, int i, int nthr)
      __attribute__((always_inline)) {
    DGMC_LDS __bf16* tile = abuf + (k % 3) * kScATile;
    const int hi = sof(k + 1);
    for (int e = sof(k) + i; e < hi; e += nthr) {
      const int code = staged ? ecs[e] : ecode[e0 + e];
      const __bf16 v = clear ? (__bf16)0.f : (staged ? evs[e] : ev[e0 + e]);
      const int dl = code >> 8, sl = code & 255;
      tile[TRANS ? sl * kScAP + dl : dl * kScAP + sl] = v;
    }
  };

  // ---- prologue (all waves) -------------------------------------------------
  if (staged)
    for (int e = tid; e < E; e += kScCT) {
      ecs[e] = ecode[e0 + e];
      evs[e] = ev[e0 + e];
    }
  using All = std::integral_constant<int, kScCT>;
  load_w(0, tid, All{});
  if (S > 1) load_w(1, tid, All{});
  if (tid < kScC) bsh[tid] = bias ? bias[tid] : 0.f;
  // Transposed pass with the fused ReLU/bias backward (maskg != null): the
  // tile's rows of g' = G * (out > 0) are formed here, written to goutg (the
  // slot weight gradient's operand) and summed per channel into bpart[t]
  // (the bias gradient's tile partial) - no separate relu_bias_bwd pass.
#pragma unroll
  for (int i = 0; i < kScT * kScC / 8 / kScCT; ++i) {
    const int c = tid + i * kScCT;
    const int row = c & 63, cc = c >> 6;
    sc_bf16x8 v = {};
    if (row < rows) {
      v = *reinterpret_cast<const sc_bf16x8*>(X + (size_t)(r0 + row) * ldx +
                                              cc * 8);
      if constexpr (TRANS) {
        const size_t o = (size_t)(r0 + row) * kScC + cc * 8;
        if (maskg) {
          const sc_bf16x8 m = *reinterpret_cast<const sc_bf16x8*>(
              reinterpret_cast<const __bf16*>(maskg) + o);
#pragma unroll
          for (int e = 0; e < 8; ++e)
            v[e] = (float)m[e] > 0.f ? v[e] : (__bf16)0.f;
        }
        if (goutg)
          *reinterpret_cast<sc_bf16x8*>(reinterpret_cast<__bf16*>(goutg) + o) =
              v;
      }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) xt[(cc * 8 + e) * kScAP + row] = v[e];
  }
  __syncthreads();
  sc_bf16x8 xa[8][2];
  if (mw) {
#pragma unroll
    for (int m = 0; m < 8; ++m)
#pragma unroll
      for (int c = 0; c < 2; ++c)
        xa[m][c] = *reinterpret_cast<DGMC_LDS const sc_bf16x8*>(
            xt + (16 * m + ln) * kScAP + 32 * c + 8 * lq);
  }
  if constexpr (TRANS) {
    if (bpart && sw) {
      // Helper waves 4-5: one channel per thread, rows in a fixed order
      // (deterministic).  xt is [channel][row]: a channel's 64 rows are
      // contiguous, read as eight 16-byte vectors (rows past `rows` were
      // staged as zeros).
      DGMC_LDS const __bf16* xr = xt + sid * kScAP;
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int r = 0; r < kScT; r += 8) {
        const sc_bf16x8 v =
            *reinterpret_cast<DGMC_LDS const sc_bf16x8*>(xr + r);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += (float)v[e];
      }
      bpart[(size_t)t * kScC + sid] = ((acc[0] + acc[1]) + (acc[2] + acc[3])) +
                                      ((acc[4] + acc[5]) + (acc[6] + acc[7]));
    }
  }
  __syncthreads();                                // xt (= A tiles) free
  {
    const sc_bf16x8 z = {};
    for (int i = tid; i < 3 * kScATile / 8; i += kScCT)
      *reinterpret_cast<DGMC_LDS sc_bf16x8*>(abuf + i * 8) = z;
  }
  __syncthreads();
  scatter(0, false, tid, kScCT);
  __syncthreads();                                // W_0, A_0 ready

  // MFMA wave w: tile rows 16 w .. +15, ALL 128 output channels (Z_k is
  // computed once per row block).
  const int node = 16 * (wave & 3) + ln;
  sc_f32x4 ot[8];
#pragma unroll
  for (int m = 0; m < 8; ++m) ot[m] = sc_f32x4{0.f, 0.f, 0.f, 0.f};

  for (int k = 0; k < S; ++k) {
    if (mw) {
      DGMC_LDS const __bf16* at =
          abuf + (k % 3) * kScATile + node * kScAP + 8 * lq;
      const sc_bf16x8 b0 = *reinterpret_cast<DGMC_LDS const sc_bf16x8*>(at);
      const sc_bf16x8 b1 =
          *reinterpret_cast<DGMC_LDS const sc_bf16x8*>(at + 32);
      DGMC_LDS const __bf16* wb = wbuf + (k % 3) * kScWImg + ln * kScC;
      sc_bf16x8 wf[2][8];
#pragma unroll
      for (int m = 0; m < 8; ++m)
        wf[0][m] = *reinterpret_cast<DGMC_LDS const sc_bf16x8*>(
            wb + m * 16 * kScC + ((lq ^ ln) << 3));
      sc_f32x4 zt[8];
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        zt[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
            xa[m][0], b0, sc_f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        zt[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xa[m][1], b1, zt[m],
                                                        0, 0, 0);
      }
      sc_bf16x8 zb[4];
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          zb[c][r] = (__bf16)zt[2 * c][r];
          zb[c][4 + r] = (__bf16)zt[2 * c + 1][r];
        }
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        if (c + 1 < 4) {
#pragma unroll
          for (int m = 0; m < 8; ++m)
            wf[(c + 1) & 1][m] = *reinterpret_cast<DGMC_LDS const sc_bf16x8*>(
                wb + m * 16 * kScC + (((4 * (c + 1) + lq) ^ ln) << 3));
        }
#pragma unroll
        for (int m = 0; m < 8; ++m)
          ot[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[c & 1][m], zb[c],
                                                          ot[m], 0, 0, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x100, 10, 0);  // A + W chunk 0
#pragma unroll
      for (int i = 0; i < 16; ++i)                          // Z_k
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
#pragma unroll
      for (int i = 0; i < 24; ++i) {                        // chunks 0-2
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);    // chunk 3
      sc_raw_barrier();
    } else if (sw) {
      // A tile of slot k-1 cleared, slot k+1 scattered (buffers the MFMA
      // waves do not read this step); stores visible before the barrier.
      if (k >= 1) scatter(k - 1, true, sid, 128);
      if (k + 1 < S) scatter(k + 1, false, sid, 128);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      sc_raw_barrier();
    } else {
      // W_{k+2} into the buffer of slot k-1 (two steps to land); before the
      // barrier only W_{k+1} (the previous step's 16 pieces) must be in.
      if (k + 2 < S) {
        load_w(k + 2, did, std::integral_constant<int, 128>{});
        asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      sc_raw_barrier();
    }
  }

  // ---- epilogue: MFMA lane holds out[node][16m + 4q + r] --------------------
  if (!mw || node >= rows) return;
  TOUT* orow = out + (size_t)(r0 + node) * kScC + 4 * lq;
#pragma unroll
  for (int m = 0; m < 8; ++m) {
    float v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = ot[m][r] + bsh[16 * m + 4 * lq + r];
    if (addg) {
      const sc_bf16x4 ad = *reinterpret_cast<const sc_bf16x4*>(
          reinterpret_cast<const __bf16*>(addg) +
          (size_t)(r0 + node) * ldadd + 16 * m + 4 * lq);
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] += (float)ad[r];
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (relu) v[r] = fmaxf(v[r], 0.f);
    }
    if constexpr (sizeof(TOUT) == 2) {
      const sc_bf16x4 o = {(__bf16)v[0], (__bf16)v[1], (__bf16)v[2],
                           (__bf16)v[3]};
      *reinterpret_cast<sc_bf16x4*>(orow + 16 * m) = o;
    } else {
      *reinterpret_cast<sc_f32x4*>(orow + 16 * m) =
          sc_f32x4{v[0], v[1], v[2], v[3]};
    }
  }
}

at::Tensor slot_conv_stamps() {
  long long h[16];
  DGMC_CHECK_HIP(hipMemcpyFromSymbol(h, HIP_SYMBOL(g_sc_stamps), sizeof(h)));
  at::Tensor t = at::empty({16}, at::kLong);
  memcpy(t.data_ptr<int64_t>(), h, sizeof(h));
  return t;
}

struct ScBwdFuse {          // fused ReLU/bias backward (ws kernel only)
  int ldx = kScC;
  const __hip_bfloat16* mask = nullptr;
  __hip_bfloat16* gout = nullptr;
  float* bpart = nullptr;
};

template <bool TRANS, bool WRITE_Z, typename TOUT>
static void launch_slot_conv(const at::Tensor& X, const at::Tensor& tiles,
                             const at::Tensor& soff, const at::Tensor& ecode,
                             const at::Tensor& eval, int S,
                             const at::Tensor& Wimg, const float* bias,
                             bool relu, at::Tensor& out, __hip_bfloat16* Z,
                             const __hip_bfloat16* add, int ldadd,
                             const ScBwdFuse& fz = ScBwdFuse()) {
  const int T = tiles.size(0);
  // Wave-specialised kernel for every pass; the 8-wave kernel only for the
  // transposed pass that also writes dY = A^T G (WRITE_Z).
  if constexpr (!WRITE_Z) {
    {
      auto kw = slot_conv_ws_kernel<TRANS, TOUT>;
      static bool ws_attr = false;
      if (!ws_attr) {
        DGMC_CHECK_HIP(hipFuncSetAttribute(
            reinterpret_cast<const void*>(kw),
            hipFuncAttributeMaxDynamicSharedMemorySize, (int)kScLdsWs));
        ws_attr = true;
      }
      hipLaunchKernelGGL(
          kw, dim3(T), dim3(kScCT), kScLdsWs, stream(),
          reinterpret_cast<const __hip_bfloat16*>(X.data_ptr()),
          tiles.data_ptr<int>(), soff.data_ptr<int>(), ecode.data_ptr<int>(),
          reinterpret_cast<const __hip_bfloat16*>(eval.data_ptr()), S,
          reinterpret_cast<const __hip_bfloat16*>(Wimg.data_ptr()), bias,
          relu ? 1 : 0, reinterpret_cast<TOUT*>(out.data_ptr()), add, ldadd,
          fz.ldx, fz.mask, fz.gout, fz.bpart);
      return;
    }
  }
  TORCH_CHECK(fz.ldx == kScC && !fz.mask && !fz.gout && !fz.bpart,
              "slot_conv: fused ReLU/bias backward needs the wave-specialised "
              "kernel");
  auto kern = slot_conv_kernel<TRANS, WRITE_Z, TOUT>;
  static bool attr_set = false;
  if (!attr_set) {
    DGMC_CHECK_HIP(hipFuncSetAttribute(
        reinterpret_cast<const void*>(kern),
        hipFuncAttributeMaxDynamicSharedMemorySize, (int)kScLds));
    attr_set = true;
  }
  hipLaunchKernelGGL(kern, dim3(T), dim3(kScCT), kScLds, stream(),
                     reinterpret_cast<const __hip_bfloat16*>(X.data_ptr()),
                     tiles.data_ptr<int>(), soff.data_ptr<int>(),
                     ecode.data_ptr<int>(),
                     reinterpret_cast<const __hip_bfloat16*>(eval.data_ptr()),
                     S,
                     reinterpret_cast<const __hip_bfloat16*>(Wimg.data_ptr()),
                     bias, relu ? 1 : 0,
                     reinterpret_cast<TOUT*>(out.data_ptr()), Z, add, ldadd,
                     0);
}

// flag [N] uint8 (1 = graph start); rowptr [N+1] / col / val: CSR of A with
// columns j*S + k; err [1] int32 (bit 0: a tile exceeds 64 rows, bit 1: an
// entry leaves its tile).  Returns (tiles [T, 4], soff [T, S+1], ecode [nnz],
// eval [nnz] bf16).
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> slot_tile_plan(
    const at::Tensor& flag, const at::Tensor& rowptr, const at::Tensor& col,
    const at::Tensor& val, int64_t window, int64_t S, at::Tensor err) {
  TORCH_CHECK(flag.is_cuda() && flag.scalar_type() == at::kByte &&
                  flag.is_contiguous(),
              "slot_tile_plan: uint8 flag [N]");
  const int64_t N = flag.numel();
  TORCH_CHECK(rowptr.scalar_type() == at::kInt && rowptr.numel() == N + 1 &&
                  rowptr.is_contiguous(),
              "slot_tile_plan: rowptr int32 [N + 1]");
  TORCH_CHECK(col.scalar_type() == at::kInt &&
                  val.scalar_type() == at::kFloat &&
                  col.numel() == val.numel() && col.is_contiguous() &&
                  val.is_contiguous(),
              "slot_tile_plan: int32 col / fp32 val entries");
  TORCH_CHECK(window >= 1 && window <= kScT,
              "slot_tile_plan: window in [1, 64]");
  TORCH_CHECK(S >= 1 && S <= kScMaxS - 1 && N * S < INT32_MAX,
              "slot_tile_plan: slot count / size range");
  TORCH_CHECK(err.is_cuda() && err.scalar_type() == at::kInt &&
                  err.numel() >= 1,
              "slot_tile_plan: err int32 [1]");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(flag.device());
  const int64_t T = std::max<int64_t>((N + window - 1) / window, 1);
  auto i32 = flag.options().dtype(at::kInt);
  // Every tile's row and slot offsets are written by the plan kernel.
  at::Tensor tiles = at::empty({T, 4}, i32);
  at::Tensor soff = at::empty({T, S + 1}, i32);
  at::Tensor ecode = at::empty({col.numel()}, i32);
  at::Tensor eval = at::empty({col.numel()}, flag.options().dtype(
      at::kBFloat16));
  if (N > 0)
    hipLaunchKernelGGL(slot_tile_plan_kernel, dim3(T), dim3(kScThreads), 0,
                       stream(), flag.data_ptr<uint8_t>(),
                       rowptr.data_ptr<int>(), col.data_ptr<int>(),
                       val.data_ptr<float>(), (int)N, (int)window, (int)S,
                       tiles.data_ptr<int>(), soff.data_ptr<int>(),
                       ecode.data_ptr<int>(),
                       reinterpret_cast<__hip_bfloat16*>(eval.data_ptr()),
                       err.data_ptr<int>());
  DGMC_CHECK_LAUNCH();
  return {tiles, soff, ecode, eval};
}

// X [N, 128] bf16; (tiles, soff, ecode, eval) from slot_tile_plan; Wimg
// [S, 128, 128] bf16 weight image (ops/sparse.py::slot_conv_image); bias
// [128] fp32; Z [N*S, 128] bf16 (trans only: dY = A^T X, rows j*S + k).
at::Tensor slot_conv(const at::Tensor& X, const at::Tensor& tiles,
                     const at::Tensor& soff, const at::Tensor& ecode,
                     const at::Tensor& eval, int64_t S, const at::Tensor& Wimg,
                     bool trans, const c10::optional<at::Tensor>& bias,
                     bool relu, at::ScalarType out_dtype,
                     const c10::optional<at::Tensor>& Z,
                     const c10::optional<at::Tensor>& addend) {
  TORCH_CHECK(X.is_cuda() && X.dim() == 2 && X.is_contiguous() &&
                  X.scalar_type() == at::kBFloat16 && X.size(1) == kScC &&
                  aligned16(X.data_ptr()),
              "slot_conv: X must be contiguous bf16 [N, 128]");
  const int64_t N = X.size(0);
  TORCH_CHECK(tiles.scalar_type() == at::kInt && tiles.dim() == 2 &&
                  tiles.size(1) == 4 && tiles.is_contiguous(),
              "slot_conv: tiles int32 [T, 4] (slot_tile_plan)");
  TORCH_CHECK(S >= 1 && S <= kScMaxS - 1 && N * S < INT32_MAX,
              "slot_conv: slot count / size range");
  TORCH_CHECK(soff.scalar_type() == at::kInt && soff.is_contiguous() &&
                  soff.numel() == tiles.size(0) * (S + 1),
              "slot_conv: soff int32 [T, S + 1]");
  TORCH_CHECK(ecode.scalar_type() == at::kInt &&
                  eval.scalar_type() == at::kBFloat16 &&
                  ecode.numel() == eval.numel() && ecode.is_contiguous() &&
                  eval.is_contiguous(),
              "slot_conv: int32 ecode / bf16 eval");
  TORCH_CHECK(Wimg.scalar_type() == at::kBFloat16 && Wimg.is_contiguous() &&
                  Wimg.numel() == S * kScWImg && aligned16(Wimg.data_ptr()),
              "slot_conv: Wimg must be contiguous bf16 [S, 128, 128]");
  TORCH_CHECK(out_dtype == at::kBFloat16 || out_dtype == at::kFloat,
              "slot_conv: bf16 or fp32 output");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(X.device());
  at::Tensor out = at::empty({N, kScC}, X.options().dtype(out_dtype));
  at::Tensor b_c;
  const float* bp = nullptr;
  if (bias.has_value() && bias->defined()) {
    b_c = bias->to(at::kFloat).contiguous();
    TORCH_CHECK(b_c.numel() == kScC, "slot_conv: bias [128]");
    bp = b_c.data_ptr<float>();
  }
  __hip_bfloat16* zp = nullptr;
  if (Z.has_value() && Z->defined()) {
    TORCH_CHECK(trans, "slot_conv: Z output only in the transposed pass");
    TORCH_CHECK(Z->scalar_type() == at::kBFloat16 && Z->is_contiguous() &&
                    Z->numel() == N * S * kScC && aligned16(Z->data_ptr()),
                "slot_conv: Z must be contiguous bf16 [N*S, 128]");
    zp = reinterpret_cast<__hip_bfloat16*>(Z->data_ptr());
  }
  const __hip_bfloat16* ap = nullptr;
  int lda = 0;
  if (addend.has_value() && addend->defined()) {
    TORCH_CHECK(addend->scalar_type() == at::kBFloat16 && addend->dim() == 2 &&
                    addend->size(0) == N && addend->size(1) == kScC &&
                    addend->stride(1) == 1 && addend->stride(0) % 4 == 0 &&
                    (reinterpret_cast<uintptr_t>(addend->data_ptr()) % 8) == 0,
                "slot_conv: addend bf16 [N, 128], unit column stride, 8-B "
                "aligned rows");
    ap = reinterpret_cast<const __hip_bfloat16*>(addend->data_ptr());
    lda = (int)addend->stride(0);
  }
  if (N == 0) return out;
  const int s = (int)S;
  const bool f32 = out_dtype == at::kFloat;
#define DGMC_SC_LAUNCH(TR, WZ)                                                \
  do {                                                                        \
    if (f32)                                                                  \
      launch_slot_conv<TR, WZ, float>(X, tiles, soff, ecode, eval, s, Wimg,  \
                                      bp, relu, out, zp, ap, lda);          \
    else                                                                      \
      launch_slot_conv<TR, WZ, __hip_bfloat16>(X, tiles, soff, ecode, eval,  \
                                               s, Wimg, bp, relu, out, zp,   \
                                               ap, lda);                      \
  } while (0)
  if (!trans)
    DGMC_SC_LAUNCH(false, false);
  else if (zp)
    DGMC_SC_LAUNCH(true, true);
  else
    DGMC_SC_LAUNCH(true, false);
#undef DGMC_SC_LAUNCH
  DGMC_CHECK_LAUNCH();
  return out;
}

// Transposed slot conv with the ReLU/bias backward fused into its prologue:
//   g' = G * (relu_out > 0)   (G: bf16 [N, 128], unit column stride, row
//                               stride ldg % 8 == 0 - e.g. a column slice of
//                               the concatenation's gradient)
//   g_out <- g'  (bf16 [N, 128] contiguous, the weight gradient's operand)
//   bias_part[t] <- sum of g' over tile t's rows (fp32 [T, 128], optional)
//   returns dX = sum_k (A_k^T g') W_k^T (+ addend)
at::Tensor slot_conv_relu_bwd(const at::Tensor& G,
                              const c10::optional<at::Tensor>& relu_out,
                              const at::Tensor& tiles, const at::Tensor& soff,
                              const at::Tensor& ecode, const at::Tensor& eval,
                              int64_t S, const at::Tensor& Wimg,
                              at::ScalarType out_dtype,
                              const c10::optional<at::Tensor>& addend,
                              at::Tensor g_out,
                              const c10::optional<at::Tensor>& bias_part) {
  TORCH_CHECK(G.is_cuda() && G.dim() == 2 && G.scalar_type() == at::kBFloat16 &&
                  G.size(1) == kScC && G.stride(1) == 1 &&
                  G.stride(0) >= kScC && G.stride(0) % 8 == 0 &&
                  aligned16(G.data_ptr()),
              "slot_conv_relu_bwd: G bf16 [N, 128], unit column stride, "
              "16-B aligned rows");
  const int64_t N = G.size(0);
  TORCH_CHECK(g_out.scalar_type() == at::kBFloat16 && g_out.is_contiguous() &&
                  g_out.numel() == N * kScC && aligned16(g_out.data_ptr()),
              "slot_conv_relu_bwd: g_out contiguous bf16 [N, 128]");
  const bool has_mask = relu_out.has_value() && relu_out->defined();
  if (has_mask)
    TORCH_CHECK(relu_out->scalar_type() == at::kBFloat16 &&
                    relu_out->is_contiguous() &&
                    relu_out->numel() == N * kScC &&
                    aligned16(relu_out->data_ptr()),
                "slot_conv_relu_bwd: relu_out contiguous bf16 [N, 128]");
  const bool has_bp = bias_part.has_value() && bias_part->defined();
  if (has_bp)
    TORCH_CHECK(bias_part->scalar_type() == at::kFloat &&
                    bias_part->is_contiguous() &&
                    bias_part->numel() == tiles.size(0) * kScC,
                "slot_conv_relu_bwd: bias_part fp32 [T, 128]");
  // Same checks as slot_conv for the shared operands (X validated above).
  TORCH_CHECK(tiles.scalar_type() == at::kInt && tiles.dim() == 2 &&
                  tiles.size(1) == 4 && tiles.is_contiguous(),
              "slot_conv_relu_bwd: tiles int32 [T, 4] (slot_tile_plan)");
  TORCH_CHECK(S >= 1 && S <= kScMaxS - 1 && N * S < INT32_MAX,
              "slot_conv_relu_bwd: slot count / size range");
  TORCH_CHECK(soff.scalar_type() == at::kInt && soff.is_contiguous() &&
                  soff.numel() == tiles.size(0) * (S + 1),
              "slot_conv_relu_bwd: soff int32 [T, S + 1]");
  TORCH_CHECK(ecode.scalar_type() == at::kInt &&
                  eval.scalar_type() == at::kBFloat16 &&
                  ecode.numel() == eval.numel() && ecode.is_contiguous() &&
                  eval.is_contiguous(),
              "slot_conv_relu_bwd: int32 ecode / bf16 eval");
  TORCH_CHECK(Wimg.scalar_type() == at::kBFloat16 && Wimg.is_contiguous() &&
                  Wimg.numel() == S * kScWImg && aligned16(Wimg.data_ptr()),
              "slot_conv_relu_bwd: Wimg contiguous bf16 [S, 128, 128]");
  TORCH_CHECK(out_dtype == at::kBFloat16 || out_dtype == at::kFloat,
              "slot_conv_relu_bwd: bf16 or fp32 output");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(G.device());
  at::Tensor out = at::empty({N, kScC}, G.options().dtype(out_dtype));
  const __hip_bfloat16* ap = nullptr;
  int lda = 0;
  if (addend.has_value() && addend->defined()) {
    TORCH_CHECK(addend->scalar_type() == at::kBFloat16 && addend->dim() == 2 &&
                    addend->size(0) == N && addend->size(1) == kScC &&
                    addend->stride(1) == 1 && addend->stride(0) % 4 == 0 &&
                    (reinterpret_cast<uintptr_t>(addend->data_ptr()) % 8) == 0,
                "slot_conv_relu_bwd: addend bf16 [N, 128], unit column "
                "stride, 8-B aligned rows");
    ap = reinterpret_cast<const __hip_bfloat16*>(addend->data_ptr());
    lda = (int)addend->stride(0);
  }
  if (N == 0) return out;
  ScBwdFuse fz;
  fz.ldx = (int)G.stride(0);
  fz.mask = has_mask
                ? reinterpret_cast<const __hip_bfloat16*>(relu_out->data_ptr())
                : nullptr;
  fz.gout = reinterpret_cast<__hip_bfloat16*>(g_out.data_ptr());
  // (Measured per transposed call: 25.9 us fused vs 23.6 + 5.4 us slot conv
  // + relu_bias_bwd unfused; docs/performance.md.)
  fz.bpart = has_bp ? bias_part->data_ptr<float>() : nullptr;
  if (out_dtype == at::kFloat)
    launch_slot_conv<true, false, float>(G, tiles, soff, ecode, eval, (int)S,
                                         Wimg, nullptr, false, out, nullptr,
                                         ap, lda, fz);
  else
    launch_slot_conv<true, false, __hip_bfloat16>(G, tiles, soff, ecode, eval,
                                                  (int)S, Wimg, nullptr, false,
                                                  out, nullptr, ap, lda, fz);
  DGMC_CHECK_LAUNCH();
  return out;
}

}  // namespace dgmc
