// fp32-accurate slot GEMM on the bf16 matrix cores ("bf16x6").
//
// Same products as slot_gemm.hip (reference: /root/reference/dgmc/models/
// spline.py:21,49 - PyG SplineConv, fp32):
//
//   Y[m, :] = A_m Bt_s^T    forward: A_m = X[src[m]], Bt_s = W_s^T images
//                           dX:      A_m = dY_c[m],   Bt_s = W_s ([in, out])
//
// but on v_mfma_f32_32x32x16_bf16 (16x the f32-MFMA rate) instead of the
// exact-f32 v_mfma_f32_32x32x2_f32.  Every fp32 operand is split once into
// three bf16 terms x = hi + mid + lo (round-to-nearest at each stage, so the
// residual is < 2^-26 |x|: 24 mantissa bits in three 8-bit pieces), and the
// six products whose order is >= 2^-16 are accumulated in fp32:
//
//   acc_hi += hi*hi,   acc_lo += lo*hi + hi*lo + mid*mid + mid*hi + hi*mid
//
// The three dropped terms (mid*lo, lo*mid, lo*lo) are < 2^-26 relative per
// product - below fp32's own rounding - and keeping the large and small
// partial sums in separate accumulators halves the accumulation error:
// measured on MI355X against an fp64 oracle (tools/micro/
// split_bf16_numerics.hip, profiles/split_bf16_numerics_r4.jsonl) the max
// error is 2.2-2.9x BELOW the exact-f32 MFMA chain at K = 128 ... 16384.
// Cost: 6 bf16 MFMAs (6 x 32 cycles) per 16-deep k step of a 32x32 block vs
// 8 f32 MFMAs (8 x 64 cycles): 2.7x fewer matrix-core cycles.
//
// Kernel: persistent grid over 256x128 output tiles (each inside one slot
// segment), 8 waves of 64x64, one workgroup per CU.  Operand planes are
// bf16 [3][rows][K]; each 16-deep k chunk of a tile is staged global -> LDS
// by global_load_lds_dwordx4 through a four-stage ring (raw s_barrier,
// hand-counted vmcnt), into [rows][32 B] images whose two 16-byte k-halves
// are XOR-swizzled by row bit 3 so every fragment read (ds_read_b128, 8
// consecutive k of one row) is bank-conflict free.  The weights are the
// MFMA A operand, so the accumulator holds Y^T: the epilogue writes float4
// rows (acc_hi + acc_lo).
#include "common.h"

namespace dgmc {

namespace {

typedef __bf16 x6_bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 x6_bf16x4 __attribute__((ext_vector_type(4)));
typedef float x6_f32x16 __attribute__((ext_vector_type(16)));
typedef float x6_f32x4 __attribute__((ext_vector_type(4)));

constexpr int kX6BN = 128;                 // output columns per tile
constexpr int kX6BK = 16;                  // k per staged chunk
constexpr int kX6MaxS = 64;

int x6_num_cus(int dev) {
  static int cached[64] = {0};
  if (dev < 0 || dev >= 64) dev = 0;
  if (cached[dev] == 0) {
    hipDeviceProp_t prop;
    DGMC_CHECK_HIP(hipGetDeviceProperties(&prop, dev));
    cached[dev] = prop.multiProcessorCount;
  }
  return usable_cus(cached[dev]);
}

// 16 bytes per lane global -> LDS (destination M0 + 16 * lane), issued as
// inline asm so the compiler does not model it as an LDS write (it would
// otherwise drain vmcnt before every fragment read); counted by hand below.
__device__ __forceinline__ void x6_dma16(const __bf16* g, DGMC_LDS __bf16* l) {
  const unsigned m0 =
      __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)l);
  asm volatile(
      "s_mov_b32 m0, %1\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %0, off"
      :: "v"(g), "s"(m0) : "memory", "m0");
}

// s_barrier without __syncthreads' fence (which would drain vmcnt and
// serialise the next chunk's DMA with this chunk's MFMAs).
__device__ __forceinline__ void x6_barrier() {
  // (drain this wave's LDS reads first: gfx950 barriers do not wait for
  // them, and their consumers - MFMAs, no memory operands - may be
  // scheduled past the barrier while another wave's DMA refills the stage)
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ void x6_split(float x, __bf16& h, __bf16& m,
                                         __bf16& l) {
  h = (__bf16)x;
  const float r1 = x - (float)h;      // exact
  m = (__bf16)r1;
  const float r2 = r1 - (float)m;     // exact
  l = (__bf16)r2;
}

}  // namespace

// ---------------------------------------------------------------------------
// Splits: fp32 [R, K] (row stride lda) -> bf16 planes [3][R][K].
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void split3_kernel(
    const float* __restrict__ x, int64_t R, int K, int64_t lda,
    __bf16* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int vpr = K / 4;
  const int64_t r = t / vpr;
  if (r >= R) return;
  const int c = (int)(t - r * vpr) * 4;
  const float4 v = *reinterpret_cast<const float4*>(x + r * lda + c);
  const float f[4] = {v.x, v.y, v.z, v.w};
  x6_bf16x4 h, m, l;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    __bf16 he, me, le;
    x6_split(f[e], he, me, le);
    h[e] = he;
    m[e] = me;
    l[e] = le;
  }
  const int64_t plane = R * K;
  __bf16* o = out + r * K + c;
  *reinterpret_cast<x6_bf16x4*>(o) = h;
  *reinterpret_cast<x6_bf16x4*>(o + plane) = m;
  *reinterpret_cast<x6_bf16x4*>(o + 2 * plane) = l;
}

// Weight images: slot s < nw is weight[s] ([in, out]), slot nw the root.
// TRANS: out[p][s][n][k] = W_s[k][n] (forward Bt = W^T, K = in, Nn = out);
// else   out[p][s][n][k] = W_s[n][k] (dX Bt = W, Nn = in, K = out).
template <bool TRANS>
__global__ __launch_bounds__(256) void weight_x3_kernel(
    const float* __restrict__ weight, const float* __restrict__ root, int nw,
    int in, int out, __bf16* __restrict__ img, int64_t plane) {
  const int Nn = TRANS ? out : in, K = TRANS ? in : out;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int vpr = K / 4;
  const int64_t per_slot = (int64_t)Nn * vpr;
  const int s = (int)(t / per_slot);
  const int64_t rem = t - (int64_t)s * per_slot;
  const int n = (int)(rem / vpr), k = (int)(rem - (int64_t)n * vpr) * 4;
  if (s > nw || (s == nw && root == nullptr)) return;
  const float* w = s < nw ? weight + (size_t)s * in * out : root;
  float f[4];
#pragma unroll
  for (int e = 0; e < 4; ++e)
    f[e] = TRANS ? w[(size_t)(k + e) * out + n] : w[(size_t)n * out + k + e];
  x6_bf16x4 h, m, l;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    __bf16 he, me, le;
    x6_split(f[e], he, me, le);
    h[e] = he;
    m[e] = me;
    l[e] = le;
  }
  __bf16* o = img + ((size_t)s * Nn + n) * K + k;
  *reinterpret_cast<x6_bf16x4*>(o) = h;
  *reinterpret_cast<x6_bf16x4*>(o + plane) = m;
  *reinterpret_cast<x6_bf16x4*>(o + 2 * plane) = l;
}

// TRANS images through a 64 x 64 LDS tile: W_s rows read as whole 256-byte
// segments (the per-element kernel above reads 4 floats 4 rows apart per
// thread - one 4-byte access per 1-KB row for psi_1's 1024 x 256 slots).
// grid (in / 64, out / 64, S); 256 threads.
__global__ __launch_bounds__(256) void weight_x3_t_kernel(
    const float* __restrict__ weight, const float* __restrict__ root, int nw,
    int in, int out, __bf16* __restrict__ img, int64_t plane) {
  __shared__ float tile[64][65];
  const int s = blockIdx.z;
  if (s == nw && root == nullptr) return;
  const float* w = s < nw ? weight + (size_t)s * in * out : root;
  const int k0 = blockIdx.x * 64, n0 = blockIdx.y * 64, t = threadIdx.x;
  const int r = t >> 4, c4 = 4 * (t & 15);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int kk = r + 16 * i;
    const float4 v = *reinterpret_cast<const float4*>(
        w + (size_t)(k0 + kk) * out + n0 + c4);
    tile[kk][c4] = v.x;
    tile[kk][c4 + 1] = v.y;
    tile[kk][c4 + 2] = v.z;
    tile[kk][c4 + 3] = v.w;
  }
  __syncthreads();
  // image row n = n0 + t / 4, 16 consecutive k = k0 + 16 (t % 4) ..
  const int n = t >> 2, kq = 16 * (t & 3);
  __bf16* o = img + ((size_t)s * out + n0 + n) * in + k0 + kq;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    x6_bf16x4 hv, mv, lv;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      __bf16 he, me, le;
      x6_split(tile[kq + 4 * g + e][n], he, me, le);
      hv[e] = he;
      mv[e] = me;
      lv[e] = le;
    }
    *reinterpret_cast<x6_bf16x4*>(o + 4 * g) = hv;
    *reinterpret_cast<x6_bf16x4*>(o + 4 * g + plane) = mv;
    *reinterpret_cast<x6_bf16x4*>(o + 4 * g + 2 * plane) = lv;
  }
}

// ---------------------------------------------------------------------------
// The GEMM.  A planes [3][*][K] (plane stride a_plane), B planes
// [3][S][Nn][K] (plane stride b_plane).  tiles (optional): 256-row tile list
// with its count at tiles[tcap] (dX of psi_2: only the target-source tiles).
//
// One workgroup per CU (8 waves = 2 per SIMD, 4 (rows) x 2 (cols) waves of
// 64 x 64), output tiles of 256 compact rows x 128 columns (slot segments
// are 256-aligned, so a tile is inside one slot), k consumed 32 at a time
// (48 MFMAs per wave between barriers) through two 72 KB LDS stages with
// ONE barrier per chunk: after it, the next chunk is staged into the buffer
// every wave has just finished reading.  Row segments are 64 B per plane
// (16 rows per 1 KB DMA instruction).  The 16-byte quads of a row are
// XOR-swizzled by f(row bits 2-4) so the ds_read_b128 fragment reads are
// bank-conflict free.  The next tile's gather indices are DMA'd into LDS
// (global_load_lds_dword): no compiler-visible vector load sits inside the
// hand-counted DMA pipeline.
// ---------------------------------------------------------------------------
constexpr int kXBM = 256;                        // rows per tile
constexpr int kXBK = 32;                         // k per chunk
constexpr int kXThreads = 512;
constexpr int kXAPlane = kXBM * kXBK;            // 8192 bf16 (16 KB)
constexpr int kXBPlane = kX6BN * kXBK;           // 4096 bf16 (8 KB)
constexpr int kXStage = 3 * kXAPlane + 3 * kXBPlane;   // bf16 per stage
constexpr size_t kXLds = (size_t)2 * kXStage * 2 + 2 * kXBM * 4;
constexpr int kXEpiPitch = 32;       // floats per row of the epilogue transpose
constexpr size_t kXEpiBytes = (size_t)8 * 32 * kXEpiPitch * 4;   // 8 waves

__device__ __forceinline__ void x6_dma4(const int* g, DGMC_LDS int* l) {
  const unsigned m0 =
      __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)l);
  asm volatile(
      "s_mov_b32 m0, %1\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dword %0, off"
      :: "v"(g), "s"(m0) : "memory", "m0");
}

// Quad swizzle of a 64-B row image: bits (2 ^ 4, 3 ^ 4) of the row.
__device__ __forceinline__ int x6_qswz(int r) {
  const int b4 = (r >> 4) & 1;
  return (((r >> 2) & 1) ^ b4) | ((((r >> 3) & 1) ^ b4) << 1);
}

// (An XCD-local tile order - workgroup b on XCD b % 8's node eighth of every
// slot - measured slower: 128->128 50.5 vs 44.3 us, 256->256 130 vs 111 us,
// profiles/bench_slot_gemm_x6_xl_r4.json; removed in round 5.)
// AF32 (fp32 A: the input gradient's dY_c, or the forward's gathered X):
// the A operand is staged
// as fp32 row images ([256][32] floats, 16-byte chunks XOR-swizzled by row
// bits 1-3 - conflict-free ds_read_b128) and split into the three bf16
// terms in registers: dY_c is stored at 4 instead of 6 bytes per element.
template <bool GATHER, bool AF32 = false>
__global__ __launch_bounds__(kXThreads, 1) void slot_gemm_x6_kernel(
    const __bf16* __restrict__ A, int64_t a_plane, const int* __restrict__ src,
    const int* __restrict__ seg, int S, const __bf16* __restrict__ B,
    int64_t b_plane, int K, int Nn, const int* __restrict__ tiles, int tcap,
    float* __restrict__ Y, const float* __restrict__ bias, int m_lim,
    int dbg) {
  // (stage sizes in bf16 units: A planes or the fp32 A image, then B)
  constexpr int AREG = AF32 ? 2 * kXBM * kXBK : 3 * kXAPlane;
  constexpr int STG = AREG + 3 * kXBPlane;
  extern __shared__ __attribute__((aligned(16))) char x6_smem[];
  DGMC_LDS __bf16* ring = (DGMC_LDS __bf16*)x6_smem;
  DGMC_LDS int* sidx =
      (DGMC_LDS int*)(x6_smem + (size_t)2 * STG * 2);   // [2][256]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave & 1, wm = wave >> 1;
  const int ntn = Nn / kX6BN, nk = K / kXBK;
  // Segment starts in lane registers: slot(m) = #{1 <= s < S: seg[s] <= m}.
  const int segv = lane <= S ? seg[lane] : 0x7fffffff;
  // (read here on every path: the compiler then waits for segv's load once,
  // before the DMA pipeline, instead of inside it - a vmcnt(0) there would
  // drain every DMA in flight at each tile start)
  const int seg_end = __builtin_amdgcn_readlane(segv, S);
  int nrt = tiles != nullptr ? tiles[tcap] : seg_end / kXBM;
  const int U = nrt * ntn;
  const int G = gridDim.x;
  const int u0 = xcd_remap(blockIdx.x, G);
  if (u0 >= U) return;
  const int my_tiles = (U - u0 + G - 1) / G;
  const int total = my_tiles * nk;
  auto slot_of = [&](int m) {
    return __popcll(__ballot(lane >= 1 && lane < S && segv <= m));
  };
  auto row_tile = [&](int j) {          // j-th tile of this workgroup
    const int q = (u0 + j * G) / ntn;
    return tiles != nullptr ? tiles[q] : q;
  };
  auto col_tile = [&](int j) { return (u0 + j * G) % ntn; };

  // Staging.  A: wave w fills rows 32 w + 16 e + L / 4 (e = 0, 1) of the
  // three plane images; B: DMA t = 3 w + e (e = 0..2) fills plane t / 8,
  // rows 16 (t % 8) + L / 4.  Lane L holds physical quad L % 4 of its row,
  // i.e. logical quad (L % 4) ^ swz(row).
  const int lr = lane >> 2;
  int ar[2], aq[2];
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    ar[e] = 32 * wave + 16 * e + lr;
    aq[e] = 8 * ((lane & 3) ^ x6_qswz(ar[e]));
  }
  int bp[3], br[3], bq[3];
#pragma unroll
  for (int e = 0; e < 3; ++e) {
    const int t = 3 * wave + e;
    bp[e] = t >> 3;
    br[e] = 16 * (t & 7) + lr;
    bq[e] = 8 * ((lane & 3) ^ x6_qswz(br[e]));
  }
  // AF32 staging: wave w fills rows 32 w + 8 e + L / 8 (e < 4), lane L
  // holds physical chunk L % 8 (4 floats) = logical (L % 8) ^ ((row >> 1) & 7).
  int fr[4], fq[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    fr[e] = 32 * wave + 8 * e + (lane >> 3);
    fq[e] = 4 * ((lane & 7) ^ ((fr[e] >> 1) & 7));
  }
  const float* Af = reinterpret_cast<const float*>(A);
  const float* frow[4] = {Af, Af, Af, Af};
  const bool bhi = wave >= 4;
  const __bf16* arow[2] = {A, A};
  const __bf16* brow = B;
  int bslot = 0;
  auto set_tile = [&](int j) {
    const int m0 = row_tile(j) * kXBM;
    if (AF32) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        int ix = m0 + fr[e];
        if (GATHER) ix = sidx[(j & 1) * kXBM + fr[e]];
        frow[e] = Af + (size_t)(ix < 0 ? 0 : ix) * K + fq[e];   // padding: row 0
      }
    }
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      int ix = m0 + ar[e];
      if (GATHER) ix = sidx[(j & 1) * kXBM + ar[e]];
      arow[e] = A + (size_t)(ix < 0 ? 0 : ix) * K + aq[e];   // padding: row 0
    }
    bslot = slot_of(m0);
    brow = B + ((size_t)bslot * Nn + col_tile(j) * kX6BN) * K;
  };
  // Gather indices of tile j into sidx[j & 1] (waves 4-7, one dword each).
  auto idx_dma = [&](int j) {
    if (GATHER && bhi && j < my_tiles)
      x6_dma4(src + row_tile(j) * kXBM + (tid - 256),
              sidx + (j & 1) * kXBM + 64 * (wave - 4));
  };
  auto stage = [&](int it) {
    const int j = it / nk, kc = it - j * nk;
    if (kc == 0) {
      set_tile(j);
      idx_dma(j + 1);
    }
    if (kDiagBuild && (dbg & 2)) return;
    DGMC_LDS __bf16* buf = ring + (it & 1) * STG;
    const int k0 = kc * kXBK;
    if (AF32) {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        x6_dma16(reinterpret_cast<const __bf16*>(frow[e] + k0),
                 buf + 2 * (32 * wave + 8 * e) * kXBK);
    } else {
#pragma unroll
      for (int p = 0; p < 3; ++p)
#pragma unroll
        for (int e = 0; e < 2; ++e)
          x6_dma16(arow[e] + p * a_plane + k0,
                   buf + p * kXAPlane + (32 * wave + 16 * e) * kXBK);
    }
    DGMC_LDS __bf16* bb = buf + AREG;
#pragma unroll
    for (int e = 0; e < 3; ++e)
      x6_dma16(brow + bp[e] * b_plane + (size_t)br[e] * K + k0 + bq[e],
               bb + bp[e] * kXBPlane + (br[e] - lr) * kXBK);
  };

  // Fragment offsets: row (block base + i), logical quad 2 s + h at physical
  // quad (2 s + h) ^ swz(i) (block bases are multiples of 32: swz of i).
  // Wave tiles: 64 x 64 on A planes; with fp32 A (fragments split in
  // registers) 32 rows x all 128 columns (FA = 4 W blocks, FB = 1 row
  // block), so no two waves read and split the same A rows.
  constexpr int FA = AF32 ? 4 : 2, FB = AF32 ? 1 : 2;
  const int xbase = AF32 ? 32 * wave : wm * 64;
  const int wbase = AF32 ? 0 : wn * 64;
  const int i = lane & 31, h = lane >> 5;
  const int fs = x6_qswz(i);
  const int offX = (xbase + i) * kXBK;
  const int offW = (wbase + i) * kXBK;

  x6_f32x16 acc[FA][FB], acs[FA][FB];
#pragma unroll
  for (int a = 0; a < FA; ++a)
#pragma unroll
    for (int b = 0; b < FB; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = acs[a][b][r] = 0.f;

  auto compute = [&](const DGMC_LDS __bf16* buf) {
    if (kDiagBuild && (dbg & 1)) return;
    const DGMC_LDS __bf16* la = buf;
    const DGMC_LDS __bf16* lb = buf + AREG;
    x6_bf16x8 w[2][3][FA], x[2][3][FB];
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      const int qo = 8 * ((2 * st + h) ^ fs);
#pragma unroll
      for (int p = 0; p < 3; ++p) {
#pragma unroll
        for (int a = 0; a < FA; ++a)
          w[st][p][a] = *reinterpret_cast<const DGMC_LDS x6_bf16x8*>(
              lb + p * kXBPlane + offW + a * 32 * kXBK + qo);
#pragma unroll
        for (int b = 0; b < FB; ++b)
          if (!AF32)
            x[st][p][b] = *reinterpret_cast<const DGMC_LDS x6_bf16x8*>(
                la + p * kXAPlane + offX + b * 32 * kXBK + qo);
      }
      if (AF32) {
        // 8 consecutive k of row r: logical chunks 4 st + 2 h, + 1.
        const DGMC_LDS float* lf = reinterpret_cast<const DGMC_LDS float*>(la);
#pragma unroll
        for (int a = 0; a < FB; ++a) {
          const int r = xbase + a * 32 + i;
          const int sw = (r >> 1) & 7, c0 = 4 * st + 2 * h;
          const x6_f32x4 u0 = *reinterpret_cast<const DGMC_LDS x6_f32x4*>(
              lf + r * kXBK + 4 * (c0 ^ sw));
          const x6_f32x4 u1 = *reinterpret_cast<const DGMC_LDS x6_f32x4*>(
              lf + r * kXBK + 4 * ((c0 + 1) ^ sw));
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            __bf16 hh, mm, ll;
            x6_split(e < 4 ? u0[e] : u1[e - 4], hh, mm, ll);
            x[st][0][a][e] = hh;
            x[st][1][a][e] = mm;
            x[st][2][a][e] = ll;
          }
        }
      }
    }
#pragma unroll
    for (int st = 0; st < 2; ++st)
#pragma unroll
      for (int a = 0; a < FA; ++a)
#pragma unroll
        for (int b = 0; b < FB; ++b) {
          x6_f32x16 sm = acs[a][b];
          sm = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[st][2][a], x[st][0][b], sm, 0, 0, 0);
          sm = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[st][0][a], x[st][2][b], sm, 0, 0, 0);
          sm = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[st][1][a], x[st][1][b], sm, 0, 0, 0);
          sm = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[st][1][a], x[st][0][b], sm, 0, 0, 0);
          sm = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[st][0][a], x[st][1][b], sm, 0, 0, 0);
          acs[a][b] = sm;
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
              w[st][0][a], x[st][0][b], acc[a][b], 0, 0, 0);
        }
  };
  // fp32-A kernels (32 x 128 wave tiles): the tile leaves through a
  // wave-private LDS transpose, so each store instruction writes 8 whole
  // 128-byte row segments instead of 32 rows x 32 bytes (4x fewer write
  // requests; the values and their order of summation are unchanged).
  // 16-byte chunk c of row r sits at chunk c ^ (r & 7): the column writes
  // (ds_write_b128: 8-lane groups = 8 rows of one chunk, 32 banks) and the
  // row reads (ds_read_b128: 16-lane groups over 4 rows x 4 chunks, 64
  // banks) are both bank-conflict free.
  DGMC_LDS float* epi = (DGMC_LDS float*)(x6_smem + (size_t)2 * STG * 2 +
                                          2 * kXBM * 4) +
                        wave * 32 * kXEpiPitch;
  auto epilogue_t = [&](int j) {
    const int rb = row_tile(j) * kXBM + xbase;      // the wave's first row
    const int cb = col_tile(j) * kX6BN;
    const int rr = lane >> 3, cc = 4 * (lane & 7);
#pragma unroll
    for (int a = 0; a < FA; ++a) {
      asm volatile("" ::: "memory");
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
        if (bias != nullptr)
          bv = *reinterpret_cast<const float4*>(bias + cb + 32 * a + 8 * q +
                                                4 * h);
        *reinterpret_cast<DGMC_LDS x6_f32x4*>(
            epi + i * kXEpiPitch + 4 * ((2 * q + h) ^ (i & 7))) =
            x6_f32x4{
            acc[a][0][4 * q] + acs[a][0][4 * q] + bv.x,
            acc[a][0][4 * q + 1] + acs[a][0][4 * q + 1] + bv.y,
            acc[a][0][4 * q + 2] + acs[a][0][4 * q + 2] + bv.z,
            acc[a][0][4 * q + 3] + acs[a][0][4 * q + 3] + bv.w};
#pragma unroll
        for (int r = 0; r < 4; ++r)
          acc[a][0][4 * q + r] = acs[a][0][4 * q + r] = 0.f;
      }
      asm volatile("" ::: "memory");
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int r = 8 * k + rr;
        const x6_f32x4 v = *reinterpret_cast<const DGMC_LDS x6_f32x4*>(
            epi + r * kXEpiPitch + 4 * ((lane & 7) ^ (r & 7)));
        if (rb + r < m_lim)
          *reinterpret_cast<float4*>(Y + (size_t)(rb + r) * Nn + cb +
                                     32 * a + cc) =
              make_float4(v[0], v[1], v[2], v[3]);
      }
    }
  };
  auto epilogue = [&](int j) {
    if (AF32) {
      epilogue_t(j);
      return;
    }
    const int m0 = row_tile(j) * kXBM + xbase + i;
    const int n0 = col_tile(j) * kX6BN + wbase + 4 * h;
#pragma unroll
    for (int a = 0; a < FA; ++a)
#pragma unroll
      for (int b = 0; b < FB; ++b) {
        float* yrow = Y + (size_t)(m0 + 32 * b) * Nn + n0 + 32 * a;
        const bool store = m0 + 32 * b < m_lim;    // (dense: rows past M)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
          if (bias != nullptr)
            bv = *reinterpret_cast<const float4*>(bias + n0 + 32 * a + 8 * q);
          if (store)
            *reinterpret_cast<float4*>(yrow + 8 * q) = make_float4(
              acc[a][b][4 * q] + acs[a][b][4 * q] + bv.x,
              acc[a][b][4 * q + 1] + acs[a][b][4 * q + 1] + bv.y,
              acc[a][b][4 * q + 2] + acs[a][b][4 * q + 2] + bv.z,
              acc[a][b][4 * q + 3] + acs[a][b][4 * q + 3] + bv.w);
#pragma unroll
          for (int r = 0; r < 4; ++r)
            acc[a][b][4 * q + r] = acs[a][b][4 * q + r] = 0.f;
        }
      }
  };

  if (GATHER) {                 // the first tile's gather indices
    idx_dma(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  stage(0);
  for (int it = 0; it < total; ++it) {
    // Item `it` (staged during the previous iteration) must have landed;
    // the previous tile's 16 epilogue stores, issued after it, need not.
    if (it > 0 && it % nk == 0)
      asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    x6_barrier();
    if (it + 1 < total) stage(it + 1);
    compute(ring + (it & 1) * STG);
    const int j = it / nk;
    if (it - j * nk == nk - 1) epilogue(j);
  }
}

// ---------------------------------------------------------------------------
// Weight gradient (TN) on bf16x6:
//   dW_s[i, c] = sum_u sum_{p in slot s} X_u[src p][i] * dY_u[p][c]
// Same work decomposition as slot_gemm.hip's slot_wgrad2_kernel - items =
// (slot, range of (16-row step, use) pairs, chunk-major) x 128 x 128 output
// tiles, per-item fp32 partials folded per slot in item order
// (deterministic) - with the contraction over compact rows p on
// v_mfma_f32_32x32x16_bf16: both operands are needed k(=p)-major per lane,
// so the row-major [16 p][128 ch] bf16 plane images are read with the
// gfx950 transposing ds_read_b64_tr_b16 (two per 8-row half fragment).  The
// images' 16-byte chunks are XOR-swizzled by ((row & 3) << 2 | (row >> 2) &
// 3), which makes the transposed reads bank-conflict free (guide T10 (b));
// the lane-linear LDS-DMA fill applies the same XOR to the global chunk each
// lane fetches.  Three-stage ring (2 x 24 KB in flight), two workgroups per
// CU, dual accumulators as in the forward kernel.
// ---------------------------------------------------------------------------
constexpr int kWXRows = 16;                      // rows per step
constexpr int kWXNst = 3;
constexpr int kWXPlane = kWXRows * 128;          // bf16 per plane image
constexpr int kWXStage = 6 * kWXPlane;           // X (3) + dY (3) planes
constexpr int kWXMaxRows = 1536;                 // gathered rows per item
constexpr int kWXMaxU = 16;
constexpr size_t kWXLds = (size_t)kWXNst * kWXStage * 2 + kWXMaxRows * 4;

struct X6Uses {
  const __bf16* x[kWXMaxU];     // X_u planes [3][N][Kin]
  const __bf16* g[kWXMaxU];     // dY_u planes [3][P][C]
};

typedef short x6_i16x4 __attribute__((ext_vector_type(4)));
typedef short x6_i16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ int wx_swz(int r) {
  return ((r & 3) << 2) | ((r >> 2) & 3);
}

// GF32: dY_u is fp32 [P][C] (4 instead of 6 bytes per element): staged as
// [16 rows][128 floats] images (16-byte chunks XOR 8 for rows 8-15, so the
// two half-waves' column reads hit disjoint banks), read column-wise
// (8 x ds_read_b32 per fragment) and split into bf16 terms in registers.
// XF32 (with GF32): X_u is fp32 [N][Kin] too - gathered rows staged as the
// same [16][128]-float images, B-operand columns read and split alike.
constexpr int kWXStageF = 3 * kWXPlane + 2 * kWXPlane;   // X planes + fp32 dY
constexpr int kWXStageFF = 2 * kWXPlane + 2 * kWXPlane;  // fp32 X + fp32 dY

// GG (with GF32, bf16 X planes): dY_c is never formed.  U.g[u] is the
// node-level output gradient g'_u [N, C] and the compact rows are built in
// the staging from the rowmap entry table (slot_gemm.hip::
// sg_rowmap_ell_kernel, 32 bytes per row: {c0, c1, c2, n}, {v0, v1, v2, e0}):
// dY_c[p] = sum_{e < n} v_e g'[c_e] (rows with n > 3 walk ecol / evl from
// e0), the same fmaf chain in the same entry order as the rowmap SpMM, so
// the result is bit-identical to the dY_c path.  Per step the 16 rows' table
// (512 B) is DMA'd into LDS ahead; each thread gathers its row's two 16-byte
// column chunks of up to three g' rows into registers before a step's MFMAs
// and combines and stores them into the ring after them.
// Measured (tools/bench_wgrad_gather.py, profiles/wgrad_gather_r5.json):
// psi_2's 10-use 128 -> 128 gradient 500 us vs 533 us for the rowmap SpMMs
// plus the dY_c kernel, psi_1's 256 -> 256 / 1024 -> 256 slower (180 vs
// 157, 588 vs 471 us: every 128-column X tile re-gathers the rows); two
// register sets (loads flying across two steps) measured 540 us.  Not on
// the training path: the input gradient still needs dY_c (docs/
// performance.md, "dY_c in the consumers").
template <bool GF32, bool XF32 = false, bool GG = false>
__global__ __launch_bounds__(256, 2) void slot_wgrad_x6_kernel(
    X6Uses U, int nu, int64_t xplane, int64_t gplane,
    const int* __restrict__ src, const int* __restrict__ seg,
    const int* __restrict__ items, int Kin, int C, float* __restrict__ part,
    const int* __restrict__ ell, const int* __restrict__ ecol,
    const float* __restrict__ evl) {
  static_assert(GF32 || !XF32, "fp32 X only with fp32 dY");
  static_assert(!GG || (GF32 && !XF32), "gathered dY: fp32 dY, X planes");
  constexpr int STG = XF32 ? kWXStageFF : GF32 ? kWXStageF : kWXStage;
  constexpr int XREG = XF32 ? 2 * kWXPlane : 3 * kWXPlane;   // X image size
  extern __shared__ __attribute__((aligned(16))) char wx_smem[];
  DGMC_LDS __bf16* ring = (DGMC_LDS __bf16*)wx_smem;
  DGMC_LDS int* sidx =
      (DGMC_LDS int*)(wx_smem + (size_t)kWXNst * STG * 2);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave & 1, wm = wave >> 1;
  const int tiles_n = C / 128, tiles = (Kin / 128) * tiles_n;
  const int item = blockIdx.x / tiles, t = blockIdx.x % tiles;
  const int i0 = (t / tiles_n) * 128, n0 = (t % tiles_n) * 128;
  const int s = items[3 * item];
  if (s < 0) return;
  const int qb = items[3 * item + 1], qe = items[3 * item + 2];
  const int c0 = qb / nu;
  const int pb = seg[s] + c0 * kWXRows;
  const int nrows = ((qe - 1) / nu - c0 + 1) * kWXRows;
  for (int r = tid; r < nrows; r += 256) {
    const int j = src[pb + r];
    sidx[r] = j < 0 ? 0 : j;            // padding rows: their dY row is zero
  }
  __syncthreads();
  const int total = qe - qb;

  // Staging: wave w fills rows 4 w .. 4 w + 3 of each plane image (1 KB per
  // DMA); lane L -> row 4 w + L / 16, physical chunk L % 16, which holds the
  // logical chunk (L % 16) ^ swz(row).
  const int srow = 4 * wave + (lane >> 4);
  const int schunk = (lane & 15) ^ wx_swz(srow);
  // GF32 dY staging: wave w fills rows 4 w + 2 e + L / 32 (e < 2); lane L
  // holds physical chunk L % 32 = logical (L % 32) ^ (8 (row >> 3 & 1)).
  int gfr[2], gfq[2];
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    gfr[e] = 4 * wave + 2 * e + (lane >> 5);
    gfq[e] = 4 * ((lane & 31) ^ (8 * ((gfr[e] >> 3) & 1)));
  }
  auto stage = [&](int q, DGMC_LDS __bf16* buf) {
    const int qq = qb + q;
    const int ch = qq / nu - c0, u = qq - (qq / nu) * nu;
    const int row = ch * kWXRows + srow;
    DGMC_LDS __bf16* d = buf + 4 * wave * 128;
    if (XF32) {
      const float* xf = reinterpret_cast<const float*>(U.x[u]);
#pragma unroll
      for (int e = 0; e < 2; ++e)
        x6_dma16(reinterpret_cast<const __bf16*>(
                     xf + (size_t)sidx[ch * kWXRows + gfr[e]] * Kin + i0 +
                     gfq[e]),
                 buf + 2 * (4 * wave + 2 * e) * 128);
    } else {
      const __bf16* xr = U.x[u] + (size_t)sidx[row] * Kin + i0 + 8 * schunk;
#pragma unroll
      for (int p = 0; p < 3; ++p) x6_dma16(xr + p * xplane, d + p * kWXPlane);
    }
    if (GF32) {
      const float* gf = reinterpret_cast<const float*>(U.g[u]) +
                        (size_t)(pb + ch * kWXRows) * C + n0;
      DGMC_LDS __bf16* dg = buf + XREG;
#pragma unroll
      for (int e = 0; e < 2; ++e)
        x6_dma16(reinterpret_cast<const __bf16*>(gf + (size_t)gfr[e] * C +
                                                 gfq[e]),
                 dg + 2 * (4 * wave + 2 * e) * 128);
    } else {
      const __bf16* gr = U.g[u] + (size_t)(pb + row) * C + n0 + 8 * schunk;
#pragma unroll
      for (int p = 0; p < 3; ++p)
        x6_dma16(gr + p * gplane, d + (3 + p) * kWXPlane);
    }
  };

  // Transposed fragment reads: 16-lane group g = lane / 16 covers columns
  // 16 (g & 1) .. + 15 of the 32-column block and rows 8 (g >> 1) .. + 7;
  // lane 4 q + p (of the group) addresses row q (+ 4 for the second read),
  // columns 4 p .. 4 p + 3.
  const int gq = (lane & 15) >> 2, gp = lane & 3, grp = lane >> 4;
  const int kb = 8 * (grp >> 1), cb = 16 * (grp & 1);
  auto tr_off = [&](int col0, int rr) {   // element offset in a plane image
    const int row = kb + rr + gq;
    const int chunk = (col0 + cb) / 8 + (gp >> 1);
    return row * 128 + 8 * (chunk ^ wx_swz(row)) + 4 * (gp & 1);
  };
  // Wave tile of the 128 x 128 output: 64 x 64 (NA = NB = 2) on planes; with
  // fp32 dY (column reads + splits) 32 dY columns x all 128 X columns
  // (NA = 1, NB = 4), so no two waves read and split the same dY columns.
  constexpr int NA = (GF32 && !XF32) ? 1 : 2, NB = 4 / NA;
  const int cbase = NA == 1 ? 32 * wave : wn * 64;
  const int ibase = NA == 1 ? 0 : wm * 64;
  int offG[NA][2], offX[NB][2];
#pragma unroll
  for (int rr = 0; rr < 2; ++rr) {
#pragma unroll
    for (int a = 0; a < NA; ++a) offG[a][rr] = tr_off(cbase + a * 32, 4 * rr);
#pragma unroll
    for (int b = 0; b < NB; ++b) offX[b][rr] = tr_off(ibase + b * 32, 4 * rr);
  }

  x6_f32x16 acc[NA][NB], acs[NA][NB];
#pragma unroll
  for (int a = 0; a < NA; ++a)
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = acs[a][b][r] = 0.f;

  // Two transposing reads (rows kb .. kb + 3 and kb + 4 .. kb + 7) make one
  // 8-element fragment.
  auto frag = [&](const DGMC_LDS __bf16* img, int o0, int o1) {
    const x6_i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (DGMC_LDS x6_i16x4*)(img + o0));
    const x6_i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (DGMC_LDS x6_i16x4*)(img + o1));
    // Whole-vector reinterpretation (a per-element bit_cast of the short
    // vector's lanes miscompiled to element 0 on this toolchain).
    const x6_i16x8 both = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5,
                                                  6, 7);
    return __builtin_bit_cast(x6_bf16x8, both);
  };
  auto compute = [&](const DGMC_LDS __bf16* buf) {
    x6_bf16x8 gv[3][NA], xv[3][NB];
#pragma unroll
    for (int p = 0; p < 3; ++p) {
#pragma unroll
      for (int a = 0; a < NA; ++a)
        if (!GF32)
          gv[p][a] = frag(buf + (3 + p) * kWXPlane, offG[a][0], offG[a][1]);
#pragma unroll
      for (int b = 0; b < NB; ++b)
        if (!XF32)
          xv[p][b] = frag(buf + p * kWXPlane, offX[b][0], offX[b][1]);
    }
    if (XF32) {
      // B operand X: lane l -> column i = ibase + 32 b + l % 32, rows
      // 8 (l / 32) + j, j < 8.
      const DGMC_LDS float* xf = reinterpret_cast<const DGMC_LDS float*>(buf);
      const int hl = lane >> 5;
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        const int c = ibase + b * 32 + (lane & 31);
        const int pc = 4 * ((c >> 2) ^ (8 * hl)) + (c & 3);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          __bf16 hh, mm, ll;
          x6_split(xf[(8 * hl + j) * 128 + pc], hh, mm, ll);
          xv[0][b][j] = hh;
          xv[1][b][j] = mm;
          xv[2][b][j] = ll;
        }
      }
    }
    if (GF32) {
      // A operand dY^T: lane l -> column c = cbase + 32 a + l % 32, rows
      // 8 (l / 32) + j, j < 8.
      const DGMC_LDS float* gf =
          reinterpret_cast<const DGMC_LDS float*>(buf + XREG);
      const int hl = lane >> 5;
#pragma unroll
      for (int a = 0; a < NA; ++a) {
        const int c = cbase + a * 32 + (lane & 31);
        const int pc = 4 * ((c >> 2) ^ (8 * hl)) + (c & 3);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          __bf16 hh, mm, ll;
          x6_split(gf[(8 * hl + j) * 128 + pc], hh, mm, ll);
          gv[0][a][j] = hh;
          gv[1][a][j] = mm;
          gv[2][a][j] = ll;
        }
      }
    }
#pragma unroll
    for (int a = 0; a < NA; ++a)
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        x6_f32x16 sm = acs[a][b];
        sm = __builtin_amdgcn_mfma_f32_32x32x16_bf16(gv[2][a], xv[0][b], sm, 0, 0, 0);
        sm = __builtin_amdgcn_mfma_f32_32x32x16_bf16(gv[0][a], xv[2][b], sm, 0, 0, 0);
        sm = __builtin_amdgcn_mfma_f32_32x32x16_bf16(gv[1][a], xv[1][b], sm, 0, 0, 0);
        sm = __builtin_amdgcn_mfma_f32_32x32x16_bf16(gv[1][a], xv[0][b], sm, 0, 0, 0);
        sm = __builtin_amdgcn_mfma_f32_32x32x16_bf16(gv[0][a], xv[1][b], sm, 0, 0, 0);
        acs[a][b] = sm;
        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
            gv[0][a], xv[0][b], acc[a][b], 0, 0, 0);
      }
  };

  if (GG) {
    DGMC_LDS int* tab = sidx + kWXMaxRows;          // [3][16 rows][8]
    auto prow = [&](int q) {                        // first compact row of q
      return pb + ((qb + q) / nu - c0) * kWXRows;
    };
    auto tab_dma = [&](int q) {                     // waves 0, 1: 512 B
      if (wave < 2)
        x6_dma4(ell + (size_t)prow(q) * 8 + 64 * wave + lane,
                tab + (q % 3) * 128 + 64 * wave);
    };
    const int gr = tid >> 4, gl = tid & 15;         // row, column chunk
    const int gsw = 8 * ((gr >> 3) & 1);
    auto gbase = [&](int q) {
      const int qq = qb + q, u = qq - (qq / nu) * nu;
      return reinterpret_cast<const float*>(U.g[u]) + n0 + 4 * gl;
    };
    float4 gv[3][2];
    auto gather = [&](int q) {                      // issue step q's gathers
      const float* g = gbase(q);
      const DGMC_LDS int* t = tab + (q % 3) * 128 + 8 * gr;
      // (unused entries hold column 0: every load is in bounds)
      const int cs[3] = {t[0], t[1], t[2]};
#pragma unroll
      for (int e = 0; e < 3; ++e)
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2)
          gv[e][h2] = *reinterpret_cast<const float4*>(
              g + (size_t)cs[e] * C + 64 * h2);
    };
    auto combine = [&](int q) {                     // dY rows into the ring
      const DGMC_LDS int* t = tab + (q % 3) * 128 + 8 * gr;
      const int n = t[3];
      float4 acc[2] = {make_float4(0.f, 0.f, 0.f, 0.f),
                       make_float4(0.f, 0.f, 0.f, 0.f)};
      if (n <= 3) {
#pragma unroll
        for (int e = 0; e < 3; ++e) {
          const float w = __int_as_float(t[4 + e]);
#pragma unroll
          for (int h2 = 0; h2 < 2; ++h2)
            if (e < n) {
              acc[h2].x = fmaf(w, gv[e][h2].x, acc[h2].x);
              acc[h2].y = fmaf(w, gv[e][h2].y, acc[h2].y);
              acc[h2].z = fmaf(w, gv[e][h2].z, acc[h2].z);
              acc[h2].w = fmaf(w, gv[e][h2].w, acc[h2].w);
            }
        }
      } else {                     // long row: walk (col, val) in entry order
        const float* g = gbase(q);
        const int e0 = t[7];
        for (int e = e0; e < e0 + n; ++e) {
          const float w = evl[e];
          const float* gr0 = g + (size_t)ecol[e] * C;
#pragma unroll
          for (int h2 = 0; h2 < 2; ++h2) {
            const float4 x = *reinterpret_cast<const float4*>(gr0 + 64 * h2);
            acc[h2].x = fmaf(w, x.x, acc[h2].x);
            acc[h2].y = fmaf(w, x.y, acc[h2].y);
            acc[h2].z = fmaf(w, x.z, acc[h2].z);
            acc[h2].w = fmaf(w, x.w, acc[h2].w);
          }
        }
      }
      DGMC_LDS float* dg = reinterpret_cast<DGMC_LDS float*>(
          ring + (q % kWXNst) * STG + XREG);
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
        const int pc = (gl + 16 * h2) ^ gsw;
        *reinterpret_cast<DGMC_LDS x6_f32x4*>(dg + gr * 128 + 4 * pc) =
            x6_f32x4{acc[h2].x, acc[h2].y, acc[h2].z, acc[h2].w};
      }
    };
    auto stage_x = [&](int q) {                     // X planes of step q
      const int qq = qb + q;
      const int ch = qq / nu - c0, u = qq - (qq / nu) * nu;
      const __bf16* xr = U.x[u] + (size_t)sidx[ch * kWXRows + srow] * Kin +
                         i0 + 8 * schunk;
      DGMC_LDS __bf16* d = ring + (q % kWXNst) * STG + 4 * wave * 128;
#pragma unroll
      for (int p = 0; p < 3; ++p) x6_dma16(xr + p * xplane, d + p * kWXPlane);
    };
    // Iteration q: X of q + 2 and the table of q + 3 DMA'd and q + 2's rows
    // gathered (registers) before step q's MFMAs, combined into the ring
    // after them; q = -2, -1 only fill the first two steps.
    tab_dma(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    x6_barrier();
    for (int q = -2; q < total; ++q) {
      const bool nxt = q + 2 < total;
      if (nxt) {
        gather(q + 2);
        stage_x(q + 2);
      }
      if (q + 3 < total) tab_dma(q + 3);
      if (q >= 0) {
        x6_barrier();
        compute(ring + (q % kWXNst) * STG);
      }
      if (nxt) combine(q + 2);
      // (X of q + 2 and the table of q + 3 landed: visible after the barrier)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      x6_barrier();
    }
  } else {
  const int pro = total < kWXNst - 1 ? total : kWXNst - 1;
  for (int q = 0; q < pro; ++q) stage(q, ring + (q % kWXNst) * STG);
  for (int q = 0; q < total; ++q) {
    if (q + kWXNst - 1 < total) {
      stage(q + kWXNst - 1, ring + ((q + kWXNst - 1) % kWXNst) * STG);
      // (this thread's DMAs of the two stages still in flight)
      if (XF32)
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else if (GF32)
        asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    x6_barrier();
    compute(ring + (q % kWXNst) * STG);
    x6_barrier();
  }
  }
  // acc[a][b]: rows c = cbase + 32 a + 8 qd + 4 h + e, column i = ibase +
  // 32 b + l32 (the dW^T layout of slot_wgrad2_kernel).  Each 32 x 32 block
  // leaves through a wave-private transpose in the (now idle) ring - the
  // swizzled image of the slot GEMM's epilogue - so a store instruction
  // writes 8 whole 128-byte row segments instead of 32 rows x 32 bytes.
  const int l32 = lane & 31, h = lane >> 5;
  float* outp = part + (size_t)item * Kin * C;
  DGMC_LDS float* epi = (DGMC_LDS float*)ring + wave * 32 * kXEpiPitch;
  const int rr = lane >> 3, cc = 4 * (lane & 7);
#pragma unroll
  for (int a = 0; a < NA; ++a)
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      asm volatile("" ::: "memory");
#pragma unroll
      for (int qd = 0; qd < 4; ++qd)
        *reinterpret_cast<DGMC_LDS x6_f32x4*>(
            epi + l32 * kXEpiPitch + 4 * ((2 * qd + h) ^ (l32 & 7))) =
            x6_f32x4{acc[a][b][4 * qd] + acs[a][b][4 * qd],
                     acc[a][b][4 * qd + 1] + acs[a][b][4 * qd + 1],
                     acc[a][b][4 * qd + 2] + acs[a][b][4 * qd + 2],
                     acc[a][b][4 * qd + 3] + acs[a][b][4 * qd + 3]};
      asm volatile("" ::: "memory");
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int r = 8 * k + rr;
        const x6_f32x4 v = *reinterpret_cast<const DGMC_LDS x6_f32x4*>(
            epi + r * kXEpiPitch + 4 * ((lane & 7) ^ (r & 7)));
        *reinterpret_cast<float4*>(outp + (size_t)(i0 + ibase + b * 32 + r) *
                                              C + n0 + cbase + a * 32 + cc) =
            make_float4(v[0], v[1], v[2], v[3]);
      }
    }
}

// ---------------------------------------------------------------------------
// Dense NT GEMM on bf16x6, fp32 operands split in registers:
//   Y[M, Nn] = [A_0 | A_1 | ...] Bt^T,  A_j fp32 [M, 128] read in place,
//   Bt fp32 [Nn, K] k-contiguous, K = 128 * parts.
// The consensus loop's folded projection (ops/dense.py::_CatMatmulF32) and
// its input gradient: skinny (M ~ 11k, K = 384 / 128) products that the
// 256x128 slot-GEMM tiles cannot spread over the chip.  One 64x64 tile per
// workgroup (4 waves of 32x32), k consumed 32 at a time through two LDS
// stages of fp32 row images ([64][32] floats, 16-byte chunks XOR-swizzled by
// row bits 1-3: conflict-free ds_read_b128), each fragment split into its
// three bf16 terms in registers.  Rows past M are clamped on load and not
// stored.  tools/micro/bench_dense_nt.py: [10944, 128] x [128, 384] 24.4 ->
// 14.9 us vs the exact-f32 kernel, [10944, 384] x [384, 128] 18.9 -> 15.1 us
// with B as pre-split planes (18.4 us splitting B in registers too; a
// four-stage ring, three chunks in flight, changed nothing).
// ---------------------------------------------------------------------------
struct NtParts {
  const float* p[4];
};

constexpr int kNtT = 64;                    // tile rows / columns
constexpr int kNtK = 32;                    // k per chunk
constexpr int kNtImg = kNtT * kNtK;         // floats per operand image

// B3: Bt given as bf16 planes [3][Nn][K] (split once per forward scope by the
// caller): only the A rows are split in registers.
template <bool B3>
__global__ __launch_bounds__(256, 4) void dense_nt_x6_kernel(
    NtParts A, int M, const float* __restrict__ bt,
    const __bf16* __restrict__ b3, int K, int Nn, float* __restrict__ Y) {
  constexpr int BIMG = B3 ? 3 * kNtT * kNtK / 2 : kNtImg;   // floats
  constexpr int STG = kNtImg + BIMG;
  __shared__ __attribute__((aligned(16))) float lds_[2 * STG];
  DGMC_LDS float* lds = (DGMC_LDS float*)lds_;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave & 1, wm = wave >> 1;
  const int ntn = Nn / kNtT, nk = K / kNtK;
  const int m0 = (blockIdx.x / ntn) * kNtT, n0 = (blockIdx.x % ntn) * kNtT;
  // Staging: wave w fills rows 16 w + 8 e + L / 8 (e < 2) of the fp32
  // images; lane L holds physical chunk L % 8 = logical (L % 8) ^ ((row >> 1)
  // & 7).  B3: DMA t = 3 w + e (e < 3) fills plane t / 4, rows 16 (t % 4) +
  // L / 4, lane L holding physical quad L % 4 = logical (L % 4) ^ swz(row).
  int srow[2], sq[2];
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    srow[e] = 16 * wave + 8 * e + (lane >> 3);
    sq[e] = 4 * ((lane & 7) ^ ((srow[e] >> 1) & 7));
  }
  int bpl[3], brw[3], bqd[3];
#pragma unroll
  for (int e = 0; e < 3; ++e) {
    const int t = 3 * wave + e;
    bpl[e] = t >> 2;
    brw[e] = 16 * (t & 3) + (lane >> 2);
    bqd[e] = 8 * ((lane & 3) ^ x6_qswz(brw[e]));
  }
  const int64_t bplane = (int64_t)Nn * K;
  auto stage = [&](int kc, DGMC_LDS float* buf) {
    const int k0 = kc * kNtK;
    const float* part = A.p[k0 >> 7];
    const int kp = k0 & 127;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int m = min(m0 + srow[e], M - 1);
      x6_dma16(reinterpret_cast<const __bf16*>(part + (size_t)m * 128 + kp +
                                               sq[e]),
               reinterpret_cast<DGMC_LDS __bf16*>(
                   buf + (16 * wave + 8 * e) * kNtK));
      if (!B3)
        x6_dma16(reinterpret_cast<const __bf16*>(
                     bt + (size_t)(n0 + srow[e]) * K + k0 + sq[e]),
                 reinterpret_cast<DGMC_LDS __bf16*>(
                     buf + kNtImg + (16 * wave + 8 * e) * kNtK));
    }
    if (B3) {
      DGMC_LDS __bf16* bb =
          reinterpret_cast<DGMC_LDS __bf16*>(buf + kNtImg);
#pragma unroll
      for (int e = 0; e < 3; ++e)
        x6_dma16(b3 + bpl[e] * bplane + (size_t)(n0 + brw[e]) * K + k0 +
                     bqd[e],
                 bb + bpl[e] * kNtT * kNtK + (brw[e] - (lane >> 2)) * kNtK);
    }
  };
  const int i = lane & 31, h = lane >> 5;
  const int ra = wm * 32 + i, rb = wn * 32 + i;   // A (m) / Bt (n) rows
  const int fs = x6_qswz(i);
  x6_f32x16 acc, acs;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = acs[r] = 0.f;
  auto frag = [&](const DGMC_LDS float* img, int row, int st,
                  x6_bf16x8 (&v)[3]) {
    const int sw = (row >> 1) & 7, c0 = 4 * st + 2 * h;
    const x6_f32x4 u0 = *reinterpret_cast<const DGMC_LDS x6_f32x4*>(
        img + row * kNtK + 4 * (c0 ^ sw));
    const x6_f32x4 u1 = *reinterpret_cast<const DGMC_LDS x6_f32x4*>(
        img + row * kNtK + 4 * ((c0 + 1) ^ sw));
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      __bf16 hh, mm, ll;
      x6_split(e < 4 ? u0[e] : u1[e - 4], hh, mm, ll);
      v[0][e] = hh;
      v[1][e] = mm;
      v[2][e] = ll;
    }
  };
  stage(0, lds);
  for (int kc = 0; kc < nk; ++kc) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    x6_barrier();
    if (kc + 1 < nk) stage(kc + 1, lds + ((kc + 1) & 1) * STG);
    const DGMC_LDS float* buf = lds + (kc & 1) * STG;
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      x6_bf16x8 x[3], w[3];
      frag(buf, ra, st, x);
      if (B3) {
        const DGMC_LDS __bf16* lb =
            reinterpret_cast<const DGMC_LDS __bf16*>(buf + kNtImg);
        const int qo = 8 * ((2 * st + h) ^ fs);
#pragma unroll
        for (int p = 0; p < 3; ++p)
          w[p] = *reinterpret_cast<const DGMC_LDS x6_bf16x8*>(
              lb + p * kNtT * kNtK + rb * kNtK + qo);
      } else {
        frag(buf + kNtImg, rb, st, w);
      }
      acs = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[2], x[0], acs, 0, 0, 0);
      acs = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[0], x[2], acs, 0, 0, 0);
      acs = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[1], x[1], acs, 0, 0, 0);
      acs = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[1], x[0], acs, 0, 0, 0);
      acs = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[0], x[1], acs, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[0], x[0], acc, 0, 0, 0);
    }
  }
  // acc: Y^T block - lane column i = row m, rows (r & 3) + 8 (r >> 2) + 4 h
  // = column n.  Out through a wave-private swizzled transpose in the ring
  // (after a barrier: other waves may still read the last chunk), 8 whole
  // 128-byte row segments per store instruction.
  x6_barrier();
  DGMC_LDS float* epi = lds + wave * 32 * 32;
#pragma unroll
  for (int q = 0; q < 4; ++q)
    *reinterpret_cast<DGMC_LDS x6_f32x4*>(
        epi + i * 32 + 4 * ((2 * q + h) ^ (i & 7))) =
        x6_f32x4{acc[4 * q] + acs[4 * q], acc[4 * q + 1] + acs[4 * q + 1],
                 acc[4 * q + 2] + acs[4 * q + 2],
                 acc[4 * q + 3] + acs[4 * q + 3]};
  asm volatile("" ::: "memory");
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int r = 8 * k + (lane >> 3);
    const x6_f32x4 v = *reinterpret_cast<const DGMC_LDS x6_f32x4*>(
        epi + r * 32 + 4 * ((lane & 7) ^ (r & 7)));
    const int m = m0 + wm * 32 + r;
    if (m < M)
      *reinterpret_cast<float4*>(Y + (size_t)m * Nn + n0 + wn * 32 +
                                 4 * (lane & 7)) =
          make_float4(v[0], v[1], v[2], v[3]);
  }
}

// ---------------------------------------------------------------------------
// Host wrappers
// ---------------------------------------------------------------------------
at::Tensor split3(const at::Tensor& x) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kFloat && x.dim() == 2 &&
                  x.stride(1) == 1 && x.size(1) % 4 == 0 &&
                  x.stride(0) % 4 == 0 && aligned16(x.data_ptr()),
              "split3: fp32 [R, K % 4] with 16-B aligned rows");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  const int64_t R = x.size(0), K = x.size(1);
  at::Tensor out = at::empty({3, R, K}, x.options().dtype(at::kBFloat16));
  const int64_t n = R * (K / 4);
  if (n == 0) return out;
  hipLaunchKernelGGL(split3_kernel, dim3((unsigned)((n + 255) / 256)),
                     dim3(256), 0, stream(), x.data_ptr<float>(), R, (int)K,
                     x.stride(0),
                     reinterpret_cast<__bf16*>(out.data_ptr()));
  DGMC_CHECK_LAUNCH();
  return out;
}

at::Tensor slot_weight_x3(const at::Tensor& weight,
                          const c10::optional<at::Tensor>& root,
                          bool transpose) {
  TORCH_CHECK(weight.is_cuda() && weight.scalar_type() == at::kFloat &&
                  weight.is_contiguous() && weight.dim() == 3,
              "slot_weight_x3: fp32 weight [K, in, out]");
  const bool has_root = root.has_value() && root->defined();
  const int64_t nw = weight.size(0), in = weight.size(1), out = weight.size(2);
  if (has_root)
    TORCH_CHECK(root->scalar_type() == at::kFloat && root->is_contiguous() &&
                    root->size(0) == in && root->size(1) == out,
                "slot_weight_x3: root [in, out]");
  TORCH_CHECK(in % 4 == 0 && out % 4 == 0, "slot_weight_x3: in/out % 4");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(weight.device());
  const int64_t S = nw + (has_root ? 1 : 0);
  const int64_t Nn = transpose ? out : in, K = transpose ? in : out;
  at::Tensor img =
      at::empty({3, S, Nn, K}, weight.options().dtype(at::kBFloat16));
  const int64_t n = S * Nn * (K / 4);
  if (n == 0) return img;
  const float* rp = has_root ? root->data_ptr<float>() : nullptr;
  if (transpose && in % 64 == 0 && out % 64 == 0) {
    hipLaunchKernelGGL(weight_x3_t_kernel,
                       dim3((unsigned)(in / 64), (unsigned)(out / 64),
                            (unsigned)S),
                       dim3(256), 0, stream(), weight.data_ptr<float>(), rp,
                       (int)nw, (int)in, (int)out,
                       reinterpret_cast<__bf16*>(img.data_ptr()),
                       S * Nn * K);
    DGMC_CHECK_LAUNCH();
    return img;
  }
  auto kern = transpose ? weight_x3_kernel<true> : weight_x3_kernel<false>;
  hipLaunchKernelGGL(kern, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     stream(), weight.data_ptr<float>(), rp, (int)nw, (int)in,
                     (int)out, reinterpret_cast<__bf16*>(img.data_ptr()),
                     S * Nn * K);
  DGMC_CHECK_LAUNCH();
  return img;
}

// DGMC_X6_DEBUG (diagnostic build only): bit 0 skips the MFMAs, bit 1 the
// operand DMAs.
static int x6_debug() {
  static const int v = diag_env_int("DGMC_X6_DEBUG", 0);
  return v;
}

at::Tensor slot_gemm_x6(const at::Tensor& a3, const at::Tensor& src,
                        const at::Tensor& seg, const at::Tensor& b3,
                        bool gather, const c10::optional<at::Tensor>& tiles) {
  // A: bf16 planes [3, R, K], or (input gradient, no gather) fp32 [R, K]
  // split in the kernel.
  const bool af32 = a3.scalar_type() == at::kFloat;
  TORCH_CHECK(a3.is_cuda() && a3.is_contiguous() &&
                  (af32 ? (a3.dim() == 2 && aligned16(a3.data_ptr()))
                        : (a3.scalar_type() == at::kBFloat16 &&
                           a3.dim() == 3 && a3.size(0) == 3)),
              "slot_gemm_x6: bf16 A planes [3, R, K] or fp32 A [R, K]");
  TORCH_CHECK(b3.scalar_type() == at::kBFloat16 && b3.is_contiguous() &&
                  b3.dim() == 4 && b3.size(0) == 3,
              "slot_gemm_x6: bf16 B planes [3, S, Nn, K]");
  const int64_t S = seg.numel() - 1;
  const int64_t Nn = b3.size(2), K = b3.size(3);
  TORCH_CHECK(b3.size(1) == S && S <= kX6MaxS, "slot_gemm_x6: slot count");
  TORCH_CHECK(a3.size(a3.dim() - 1) == K, "slot_gemm_x6: A [*, K]");
  TORCH_CHECK(K % 128 == 0 && Nn % kX6BN == 0,
              "slot_gemm_x6: K, Nn multiples of 128");
  const int64_t P = src.numel();
  TORCH_CHECK(P % kXBM == 0 && src.scalar_type() == at::kInt &&
                  seg.scalar_type() == at::kInt,
              "slot_gemm_x6: int32 src [P_cap % 256], seg");
  if (!gather) {
    TORCH_CHECK(a3.size(a3.dim() - 2) == P, "slot_gemm_x6: rows == P_cap");
  }
  const bool listed = tiles.has_value() && tiles->defined();
  if (listed)
    TORCH_CHECK(tiles->scalar_type() == at::kInt &&
                    tiles->numel() == P / kXBM + 1,
                "slot_gemm_x6: 256-row tile list [P_cap / 256 + 1] (count "
                "last)");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(a3.device());
  at::Tensor Y = at::empty({P, Nn}, a3.options().dtype(at::kFloat));
  const int64_t tiles_max = (P / kXBM) * (Nn / kX6BN);
  const int64_t blocks = std::min<int64_t>(
      tiles_max, (int64_t)x6_num_cus(a3.device().index()));
  if (blocks == 0) return Y;
  const __bf16* ap = reinterpret_cast<const __bf16*>(a3.data_ptr());
  const __bf16* bp = reinterpret_cast<const __bf16*>(b3.data_ptr());
  const int* tl = listed ? tiles->data_ptr<int>() : nullptr;
  auto kern = af32 ? (gather ? slot_gemm_x6_kernel<true, true>
                             : slot_gemm_x6_kernel<false, true>)
              : gather ? slot_gemm_x6_kernel<true, false>
                       : slot_gemm_x6_kernel<false, false>;
  const int64_t grid = blocks;
  const size_t lds = af32 ? (size_t)2 * (2 * kXBM * kXBK + 3 * kXBPlane) * 2 +
                                2 * kXBM * 4 + kXEpiBytes
                          : kXLds;
  DGMC_CHECK_HIP(hipFuncSetAttribute(
      reinterpret_cast<const void*>(kern),
      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL(kern, dim3(grid), dim3(kXThreads), lds, stream(), ap,
                     af32 ? 0 : a3.size(1) * K, src.data_ptr<int>(),
                     seg.data_ptr<int>(),
                     (int)S, bp, S * Nn * K, (int)K, (int)Nn, tl,
                     (int)(P / kXBM), Y.data_ptr<float>(), nullptr,
                     (int)P, x6_debug());
  DGMC_CHECK_LAUNCH();
  return Y;
}

std::vector<at::Tensor> slot_wgrad_items(const at::Tensor& seg, int64_t nu,
                                         int64_t target, int64_t qcap,
                                         int64_t G_cap, int64_t rows);
at::Tensor slot_fold_parts(const at::Tensor& part, const at::Tensor& ib,
                           int64_t S, int64_t Kin, int64_t C);

// dW [S, Kin, C] = sum_u X_u[src]^T dY_u per slot, operands as bf16 planes:
// xs[u] [3, N, Kin], gs[u] [3, P_cap, C].  `rounds`: rounds of resident
// workgroups the items are sized for (as slot_wgrad_f32).
at::Tensor slot_wgrad_x6(at::TensorList xs, at::TensorList gs,
                         const at::Tensor& src, const at::Tensor& seg,
                         int64_t rounds, const c10::optional<at::Tensor>& ell,
                         const c10::optional<at::Tensor>& ecol,
                         const c10::optional<at::Tensor>& evl) {
  // ell given: gs are node-level fp32 output gradients [N_g, out], and the
  // compact dY rows are gathered in the kernel (GG above).
  const bool gg = ell.has_value() && ell->defined();
  const int64_t nu = (int64_t)xs.size();
  TORCH_CHECK(nu >= 1 && nu <= kWXMaxU && (int64_t)gs.size() == nu,
              "slot_wgrad_x6: 1 <= uses <= 16, one dY per X");
  // dY_u: bf16 planes [3, P_cap, out] or fp32 [P_cap, out] (split in
  // the kernel).
  const bool gf32 = gs[0].scalar_type() == at::kFloat;
  const bool xf32 = xs[0].scalar_type() == at::kFloat;
  TORCH_CHECK(gf32 || !xf32, "slot_wgrad_x6: fp32 X needs fp32 dY");
  TORCH_CHECK(!gg || (gf32 && !xf32),
              "slot_wgrad_x6: gathered dY needs fp32 g' and X planes");
  const int64_t N = xf32 ? xs[0].size(0) : xs[0].size(1);
  const int64_t Kin = xf32 ? xs[0].size(1) : xs[0].size(2);
  const int64_t C = gf32 ? gs[0].size(1) : gs[0].size(2);
  const int64_t P = src.numel(), S = seg.numel() - 1;
  TORCH_CHECK(Kin % 128 == 0 && C % 128 == 0 && P % kWXRows == 0 &&
                  rounds >= 1 && S <= kX6MaxS && src.scalar_type() == at::kInt,
              "slot_wgrad_x6: in / out multiples of 128");
  X6Uses U{};
  for (int64_t u = 0; u < nu; ++u) {
    const at::Tensor& x = xs[u];
    const at::Tensor& g = gs[u];
    if (xf32) {
      TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kFloat &&
                      x.is_contiguous() && x.dim() == 2 && x.size(0) == N &&
                      x.size(1) == Kin && aligned16(x.data_ptr()),
                  "slot_wgrad_x6: X_u fp32 [N, in] (all uses alike)");
    } else {
      TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 &&
                      x.is_contiguous() && x.dim() == 3 && x.size(0) == 3 &&
                      x.size(1) == N && x.size(2) == Kin,
                  "slot_wgrad_x6: X_u bf16 planes [3, N, in]");
    }
    if (gg) {
      TORCH_CHECK(g.scalar_type() == at::kFloat && g.is_contiguous() &&
                      g.dim() == 2 && g.size(0) == gs[0].size(0) &&
                      g.size(1) == C && aligned16(g.data_ptr()),
                  "slot_wgrad_x6: g'_u fp32 [N_g, out] (all uses alike)");
    } else if (gf32) {
      TORCH_CHECK(g.scalar_type() == at::kFloat && g.is_contiguous() &&
                      g.dim() == 2 && g.size(0) == P && g.size(1) == C &&
                      aligned16(g.data_ptr()),
                  "slot_wgrad_x6: dY_u fp32 [P_cap, out] (all uses alike)");
    } else {
      TORCH_CHECK(g.scalar_type() == at::kBFloat16 && g.is_contiguous() &&
                      g.dim() == 3 && g.size(0) == 3 && g.size(1) == P &&
                      g.size(2) == C,
                  "slot_wgrad_x6: dY_u bf16 planes [3, P_cap, out]");
    }
    U.x[u] = reinterpret_cast<const __bf16*>(x.data_ptr());
    U.g[u] = reinterpret_cast<const __bf16*>(g.data_ptr());
  }
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(src.device());
  const int64_t tiles = (Kin / 128) * (C / 128);
  const int64_t target = std::max<int64_t>(
      1, rounds * 2 * (int64_t)device_cus(src.device().index()) / tiles);
  const int64_t qcap = (kWXMaxRows / kWXRows - 2) * nu;
  const int64_t G_cap = target + (P / kWXRows * nu + qcap - 1) / qcap + S;
  auto it = slot_wgrad_items(seg, nu, target, qcap, G_cap, kWXRows);
  const int64_t per = Kin * C;
  at::Tensor part =
      at::empty({G_cap, per}, xs[0].options().dtype(at::kFloat));
  const int *ep = nullptr, *cp = nullptr;
  const float* vp = nullptr;
  if (gg) {
    // entry table [P_cap, 8] of the same compact plan; long rows' (col, val)
    TORCH_CHECK(ell->scalar_type() == at::kInt && ell->is_contiguous() &&
                    ell->numel() == 8 * P && ecol.has_value() &&
                    evl.has_value() && ecol->scalar_type() == at::kInt &&
                    evl->scalar_type() == at::kFloat &&
                    ecol->is_contiguous() && evl->is_contiguous() &&
                    ecol->numel() == evl->numel(),
                "slot_wgrad_x6: int32 entry table [P_cap, 8] + col / val");
    ep = ell->data_ptr<int>();
    cp = ecol->data_ptr<int>();
    vp = evl->data_ptr<float>();
  }
  auto kern = gg ? slot_wgrad_x6_kernel<true, false, true>
              : xf32 ? slot_wgrad_x6_kernel<true, true>
              : gf32 ? slot_wgrad_x6_kernel<true> : slot_wgrad_x6_kernel<false>;
  const size_t lds =
      (size_t)kWXNst * (xf32 ? kWXStageFF : gf32 ? kWXStageF : kWXStage) * 2 +
      kWXMaxRows * 4 + (gg ? 3 * 128 * 4 : 0);
  DGMC_CHECK_HIP(hipFuncSetAttribute(
      reinterpret_cast<const void*>(kern),
      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL(kern, dim3(G_cap * tiles), dim3(256), lds, stream(), U,
                     (int)nu, N * Kin, P * C, src.data_ptr<int>(),
                     seg.data_ptr<int>(), it[0].data_ptr<int>(), (int)Kin,
                     (int)C, part.data_ptr<float>(), ep, cp, vp);
  DGMC_CHECK_LAUNCH();
  return slot_fold_parts(part, it[1], S, Kin, C);
}

at::Tensor dense_nt_x6(at::TensorList parts, const at::Tensor& bt,
                       const c10::optional<at::Tensor>& b3) {
  const int64_t np = (int64_t)parts.size();
  TORCH_CHECK(np >= 1 && np <= 4, "dense_nt_x6: 1..4 parts");
  const int64_t M = parts[0].size(0);
  NtParts A{};
  for (int64_t j = 0; j < np; ++j) {
    const at::Tensor& p = parts[j];
    TORCH_CHECK(p.is_cuda() && p.scalar_type() == at::kFloat &&
                    p.is_contiguous() && p.dim() == 2 && p.size(0) == M &&
                    p.size(1) == 128 && aligned16(p.data_ptr()),
                "dense_nt_x6: parts contiguous fp32 [M, 128]");
    A.p[j] = p.data_ptr<float>();
  }
  TORCH_CHECK(bt.is_cuda() && bt.scalar_type() == at::kFloat &&
                  bt.is_contiguous() && bt.dim() == 2 &&
                  bt.size(1) == 128 * np && bt.size(0) % kNtT == 0 &&
                  aligned16(bt.data_ptr()),
              "dense_nt_x6: Bt fp32 [Nn % 64, 128 * parts]");
  const int64_t Nn = bt.size(0), K = bt.size(1);
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(bt.device());
  at::Tensor Y = at::empty({M, Nn}, bt.options());
  if (M == 0) return Y;
  const bool planes = b3.has_value() && b3->defined();
  if (planes)
    TORCH_CHECK(b3->scalar_type() == at::kBFloat16 && b3->is_contiguous() &&
                    b3->dim() == 3 && b3->size(0) == 3 && b3->size(1) == Nn &&
                    b3->size(2) == K,
                "dense_nt_x6: Bt planes bf16 [3, Nn, K]");
  const int64_t tiles = ((M + kNtT - 1) / kNtT) * (Nn / kNtT);
  hipLaunchKernelGGL(planes ? dense_nt_x6_kernel<true>
                            : dense_nt_x6_kernel<false>,
                     dim3((unsigned)tiles), dim3(256), 0, stream(), A, (int)M,
                     bt.data_ptr<float>(),
                     planes ? reinterpret_cast<const __bf16*>(b3->data_ptr())
                            : nullptr,
                     (int)K, (int)Nn, Y.data_ptr<float>());
  DGMC_CHECK_LAUNCH();
  return Y;
}

}  // namespace dgmc
