// Per-pair fused kernels of the dense DGMC consensus loop
// (reference dgmc.py:161-183).  One workgroup (16 waves) per graph pair; the
// pair's node tiles live in LDS, masks are derived from the per-pair node
// counts (valid nodes occupy the leading rows of the padded tile).
//
//   dense_masked_softmax      S = masked_softmax(S_hat)          (dgmc.py:15-19)
//   dense_softmax_transport   S, r_t = S^T r_s                   (dgmc.py:168-171)
//   dense_consensus           S_hat + mask*(relu(P_i - Q_j).w2 + b2)
//                             = S_hat + mask*MLP(o_s_i - o_t_j)  (dgmc.py:178-179)
// and their backward kernels.  The consensus backward recomputes relu(P-Q)
// instead of storing the [B, N_s, N_t, R] activation the reference keeps.
//
// Latency design (MI355X): a pair is tiny (~9x9 nodes x 128 channels, a few
// kFLOP), so these kernels are bound by dependent memory round trips, not by
// bandwidth or ALU.  Every kernel therefore
//   * issues ALL loads of its operand tiles before the first LDS store
//     (`stage_rows`: up to 4 independent 16-byte loads per thread per batch,
//     P and Q tiles in the same batch) - one round trip per tile set instead
//     of one per row;
//   * computes from LDS with several independent partial sums per thread
//     (LDS latency overlapped), channel-parallel lanes (conflict-free rows) or
//     8 lanes per (i, j) entry with strided channels (odd LDS pitch);
//   * sizes LDS dynamically from the padded pair tile (Ns, Nt <= 64).
#include "common.h"

#include <type_traits>

namespace dgmc {

constexpr int kMaxN = 64;      // max padded nodes per graph of a pair
// Pair kernels run 16 waves per workgroup: the grid (one workgroup per pair,
// 512 for the PascalVOC batch) is a single dispatch wave, so the kernel time
// is the latency of the slowest pair - more lanes per pair = shorter
// per-thread loops.  2 workgroups/CU x 16 waves = full occupancy at <= 64
// VGPRs.
constexpr int kWaves = 8;
constexpr int kThreads = kWaves * kWave;
constexpr int kPrefetch = 4;   // S/G tile entries prefetched per thread
constexpr int kTPE = 8;        // lanes per (i, j) entry in channel dot loops
constexpr int kRowWaves = 4;   // row-softmax kernels: waves per 256 threads

// Zero rows [row0, rows) of a packed [rows, R] tensor (padding rows of static
// batches; executed by the last workgroup of a launch).
template <typename T>
__device__ __forceinline__ void zero_tail(T* __restrict__ x, int row0,
                                          int rows, int R) {
  const size_t begin = (size_t)row0 * R, end = (size_t)rows * R;
  for (size_t e = begin + threadIdx.x; e < end; e += blockDim.x)
    x[e] = Cvt<T>::from_f(0.f);
}

// Stage rows [0, na) of the packed row block a[na, R] and rows [0, nb) of
// b[nb, R] into LDS fp32 tiles dA / dB (row pitch `pitch`).  Each thread
// issues up to 4 independent loads before its first LDS store, so both tiles
// arrive in one memory round trip for pair-sized blocks.  `vec`: 16-byte
// aligned rows (R * sizeof(T) % 16 == 0 and aligned bases).
template <typename T>
__device__ __forceinline__ void stage_rows(DGMC_LDS float* dA,
                                           const T* __restrict__ a, int na,
                                           DGMC_LDS float* dB,
                                           const T* __restrict__ b, int nb,
                                           int pitch, int R, bool vec) {
  const int tid = threadIdx.x;
  if (vec) {
    constexpr int V = Vec16<T>::N;
    const int vpr = R / V;
    const int nva = na * vpr, nv = nva + nb * vpr;
    for (int base = tid; base < nv; base += 4 * kThreads) {
      float v[4][V];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int q = base + u * kThreads;
        if (q < nv)
          load_vec<T, V>(q < nva ? a + (size_t)q * V : b + (size_t)(q - nva) * V,
                         v[u]);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int q = base + u * kThreads;
        if (q < nv) {
          const bool in_a = q < nva;
          const int qq = in_a ? q : q - nva;
          const int r = qq / vpr, c = (qq - r * vpr) * V;
          DGMC_LDS float* d = (in_a ? dA : dB) + r * pitch + c;
#pragma unroll
          for (int k = 0; k < V; ++k) d[k] = v[u][k];
        }
      }
    }
  } else {
    const int nea = na * R, ne = nea + nb * R;
    for (int base = tid; base < ne; base += 4 * kThreads) {
      float v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int q = base + u * kThreads;
        v[u] = q < ne ? Cvt<T>::to_f(q < nea ? a[q] : b[q - nea]) : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int q = base + u * kThreads;
        if (q < ne) {
          const bool in_a = q < nea;
          const int qq = in_a ? q : q - nea;
          (in_a ? dA : dB)[(qq / R) * pitch + qq % R] = v[u];
        }
      }
    }
  }
}

// Prefetch the first kPrefetch * kThreads entries of a pair's fp32 [Ns, Nt]
// tile into registers (issued before the operand staging, consumed after).
__device__ __forceinline__ void prefetch_tile(const float* __restrict__ t,
                                              int NN, float (&v)[kPrefetch]) {
#pragma unroll
  for (int u = 0; u < kPrefetch; ++u) {
    const int e = threadIdx.x + u * kThreads;
    v[u] = e < NN ? t[e] : 0.f;
  }
}

// Channel mapping shared by the channel-parallel loops: chunk of up to
// kThreads channels; RP row groups when R < kThreads.
struct ChanMap {
  int cw, rp, c, r0;
  bool active;
  __device__ __forceinline__ ChanMap(int c0, int R) {
    cw = min(kThreads, R - c0);
    rp = kThreads / cw;
    const int tid = threadIdx.x;
    active = tid < rp * cw;
    c = c0 + tid % cw;
    r0 = tid / cw;
  }
};

// ---------------------------------------------------------------------------
// Row-wise masked softmax (+ backward).  One wave per (b, i) row.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void masked_softmax_kernel(
    const float* __restrict__ S_hat, const int* __restrict__ n_s,
    const int* __restrict__ n_t, float* __restrict__ S, int B, int Ns,
    int Nt) {
  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  const int row = blockIdx.x * kRowWaves + wave;
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
  const int row = blockIdx.x * kRowWaves + wave;
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
// LDS: sR [Ns][R] (r_s, fp32), sS [Ns][Nt] (S_hat, then S).
// ---------------------------------------------------------------------------
template <typename TR>
__global__ __launch_bounds__(kThreads) void softmax_transport_kernel(
    const float* __restrict__ S_hat, const TR* __restrict__ r_s,
    const int* __restrict__ ptr_s, const int* __restrict__ ptr_t,
    float* __restrict__ S, TR* __restrict__ r_t, int Ns, int Nt, int R,
    int rows_t, TR* __restrict__ r_s_copy, int rows_s, int vec) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  DGMC_LDS float* sR = (DGMC_LDS float*)smem_raw;
  DGMC_LDS float* sS = sR + Ns * R;
  const int b = xcd_remap(blockIdx.x, gridDim.x);
  const int tid = threadIdx.x;
  const int wave = tid / kWave, lane = tid % kWave;
  const int s0 = ptr_s[b], ns = ptr_s[b + 1] - s0;
  const int t0 = ptr_t[b], nt = ptr_t[b + 1] - t0;
  const int NN = Ns * Nt;
  const float* Sh = S_hat + (size_t)b * NN;
  float pre[kPrefetch];
  prefetch_tile(Sh, NN, pre);
  stage_rows<TR>(sR, r_s + (size_t)s0 * R, ns, sR, r_s, 0, R, R, vec != 0);
#pragma unroll
  for (int u = 0; u < kPrefetch; ++u) {
    const int e = tid + u * kThreads;
    if (e < NN) sS[e] = pre[u];
  }
  for (int e = tid + kPrefetch * kThreads; e < NN; e += kThreads) sS[e] = Sh[e];
  if (blockIdx.x == gridDim.x - 1) zero_tail(r_t, ptr_t[gridDim.x], rows_t, R);
  if (r_s_copy) {
    // r_s rows past the last pair (static-batch padding), spread over the
    // whole grid: one element per thread.
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t e = (size_t)ptr_s[gridDim.x] * R +
                    (size_t)blockIdx.x * blockDim.x + tid;
         e < (size_t)rows_s * R; e += stride)
      r_s_copy[e] = r_s[e];
  }
  __syncthreads();

  float* Sb = S + (size_t)b * NN;
  for (int i = wave; i < Ns; i += kWaves) {
    const bool valid = i < ns && lane < nt;
    const float v = valid ? sS[i * Nt + lane] : -INFINITY;
    const float m = wave_max(v);
    const float e = valid ? __expf(v - m) : 0.f;
    const float s = wave_sum(e);
    const float p = valid ? e / s : 0.f;
    if (lane < Nt) {
      sS[i * Nt + lane] = p;
      Sb[i * Nt + lane] = p;
    }
  }
  if (r_s_copy) {
    // Joint output [r_s; r_t]: psi_2's input without a concatenation
    // (bf16/fp32 -> fp32 -> same type is exact).
    TR* dst = r_s_copy + (size_t)s0 * R;
    for (int e = tid; e < ns * R; e += kThreads)
      dst[e] = Cvt<TR>::from_f(sR[e]);
  }
  __syncthreads();

  TR* rt = r_t + (size_t)t0 * R;
  for (int c0 = 0; c0 < R; c0 += kThreads) {
    const ChanMap cm(c0, R);
    if (!cm.active) continue;
    for (int j = cm.r0; j < nt; j += cm.rp) {
      float a[4] = {0.f, 0.f, 0.f, 0.f};
      int i = 0;
      for (; i + 4 <= ns; i += 4) {
#pragma unroll
        for (int u = 0; u < 4; ++u)
          a[u] = fmaf(sS[(i + u) * Nt + j], sR[(i + u) * R + cm.c], a[u]);
      }
      for (; i < ns; ++i) a[0] = fmaf(sS[i * Nt + j], sR[i * R + cm.c], a[0]);
      rt[(size_t)j * R + cm.c] = Cvt<TR>::from_f((a[0] + a[1]) + (a[2] + a[3]));
    }
  }
}

// dS_hat = softmax_bwd(S, dS),  dS[i][j] = sum_c r_s[i][c] * g[j][c].
// LDS: sR [Ns][R+1], sG [Nt][R+1], sD [Ns][Nt].
template <typename TR>
__global__ __launch_bounds__(kThreads) void softmax_transport_bwd_kernel(
    const float* __restrict__ S, const TR* __restrict__ r_s,
    const TR* __restrict__ g, const int* __restrict__ ptr_s,
    const int* __restrict__ ptr_t, float* __restrict__ dS_hat,
    const float* __restrict__ addend, int Ns, int Nt, int R, int vec) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  const int pitch = R + 1;
  DGMC_LDS float* sR = (DGMC_LDS float*)smem_raw;
  DGMC_LDS float* sG = sR + Ns * pitch;
  DGMC_LDS float* sD = sG + Nt * pitch;
  const int b = xcd_remap(blockIdx.x, gridDim.x);
  const int tid = threadIdx.x;
  const int wave = tid / kWave, lane = tid % kWave;
  const int s0 = ptr_s[b], ns = ptr_s[b + 1] - s0;
  const int t0 = ptr_t[b], nt = ptr_t[b + 1] - t0;
  const int NN = Ns * Nt;
  const float* Sb = S + (size_t)b * NN;
  // S rows of this wave (i = wave + kWaves * q), fetched up front.
  constexpr int QMAX = kMaxN / kWaves;
  float sv[QMAX];
#pragma unroll
  for (int q = 0; q < QMAX; ++q) {
    const int i = wave + q * kWaves;
    sv[q] = (i < Ns && lane < Nt) ? Sb[i * Nt + lane] : 0.f;
  }
  stage_rows<TR>(sR, r_s + (size_t)s0 * R, ns, sG, g + (size_t)t0 * R, nt,
                 pitch, R, vec != 0);
  __syncthreads();

  // dS[i][j]: kTPE lanes per entry, channels strided by kTPE.
  const int qd = tid % kTPE;
  const int pairs = ns * nt;
  for (int p0 = 0; p0 < pairs; p0 += kThreads / kTPE) {
    const int p = p0 + tid / kTPE;
    const bool valid = p < pairs;
    const int i = valid ? p / nt : 0;
    const int j = valid ? p - i * nt : 0;
    const DGMC_LDS float* rr = sR + i * pitch;
    const DGMC_LDS float* gr = sG + j * pitch;
    float a[4] = {0.f, 0.f, 0.f, 0.f};
    int c = qd;
    for (; c + 3 * kTPE < R; c += 4 * kTPE) {
#pragma unroll
      for (int u = 0; u < 4; ++u)
        a[u] = fmaf(rr[c + kTPE * u], gr[c + kTPE * u], a[u]);
    }
    for (; c < R; c += kTPE) a[0] = fmaf(rr[c], gr[c], a[0]);
    float acc = (a[0] + a[1]) + (a[2] + a[3]);
#pragma unroll
    for (int o = 1; o < kTPE; o <<= 1) acc += __shfl_xor(acc, o);
    if (valid && qd == 0) sD[i * Nt + j] = acc;
  }
  __syncthreads();

  float* out = dS_hat + (size_t)b * NN;
#pragma unroll
  for (int q = 0; q < QMAX; ++q) {
    const int i = wave + q * kWaves;
    if (i < Ns) {
      const float d = (i < ns && lane < nt) ? sD[i * Nt + lane] : 0.f;
      const float dot = wave_sum(sv[q] * d);
      if (lane < Nt) {
        // addend: S_hat's other consumer's gradient (the consensus
        // update's identity path), summed here instead of by a separate
        // kernel.
        const float a = addend ? addend[(size_t)b * NN + i * Nt + lane] : 0.f;
        out[i * Nt + lane] = sv[q] * (d - dot) + a;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Consensus update: out = S_hat + mask * (sum_c relu(P_ic + b1_c - Q_jc) w2_c
//                                         + b2)
// LDS: sP [Ns][R+1], sQ [Nt][R+1], sB [R] (b1), sW [R] (w2).
// ---------------------------------------------------------------------------
template <typename TPQ>
__global__ __launch_bounds__(kThreads) void consensus_fwd_kernel(
    const float* __restrict__ S_hat, const TPQ* __restrict__ P,
    const TPQ* __restrict__ Q, const float* __restrict__ b1,
    const float* __restrict__ w2, const float* __restrict__ b2,
    const int* __restrict__ ptr_s, const int* __restrict__ ptr_t,
    float* __restrict__ out, int Ns, int Nt, int R, int vec) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  const int pitch = R + 1;
  DGMC_LDS float* sP = (DGMC_LDS float*)smem_raw;
  DGMC_LDS float* sQ = sP + Ns * pitch;
  DGMC_LDS float* sB = sQ + Nt * pitch;
  DGMC_LDS float* sW = sB + R;
  const int b = xcd_remap(blockIdx.x, gridDim.x);
  const int tid = threadIdx.x;
  const int s0 = ptr_s[b], ns = ptr_s[b + 1] - s0;
  const int t0 = ptr_t[b], nt = ptr_t[b + 1] - t0;
  const int NN = Ns * Nt;
  const float* Sh = S_hat + (size_t)b * NN;
  float* ob = out + (size_t)b * NN;
  float bw[2] = {0.f, 0.f};
  if (tid < R) {
    bw[0] = b1[tid];
    bw[1] = w2[tid];
  }
  stage_rows<TPQ>(sP, P + (size_t)s0 * R, ns, sQ, Q + (size_t)t0 * R, nt,
                  pitch, R, vec != 0);
  if (tid < R) {
    sB[tid] = bw[0];
    sW[tid] = bw[1];
  }
  for (int c = tid + kThreads; c < R; c += kThreads) {
    sB[c] = b1[c];
    sW[c] = w2[c];
  }
  // Entries outside the valid ns x nt block pass S_hat through unchanged.
  for (int e = tid; e < NN; e += kThreads) {
    const int i = e / Nt, j = e - (e / Nt) * Nt;
    if (i >= ns || j >= nt) ob[e] = Sh[e];
  }
  const float bias2 = b2[0];
  __syncthreads();

  // kTPE lanes per (i, j) entry, channels strided by kTPE (odd pitch: the
  // rows of neighbouring entries fall on different banks).
  const int qd = tid % kTPE;
  const int pairs = ns * nt;
  for (int p0 = 0; p0 < pairs; p0 += kThreads / kTPE) {
    const int p = p0 + tid / kTPE;
    const bool valid = p < pairs;
    const int i = valid ? p / nt : 0;
    const int j = valid ? p - i * nt : 0;
    const float sh = (valid && qd == 0) ? Sh[i * Nt + j] : 0.f;
    const DGMC_LDS float* pr = sP + i * pitch;
    const DGMC_LDS float* qr = sQ + j * pitch;
    float a[4] = {0.f, 0.f, 0.f, 0.f};
    int c = qd;
    for (; c + 3 * kTPE < R; c += 4 * kTPE) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int cc = c + kTPE * u;
        a[u] = fmaf(fmaxf(pr[cc] + sB[cc] - qr[cc], 0.f), sW[cc], a[u]);
      }
    }
    for (; c < R; c += kTPE)
      a[0] = fmaf(fmaxf(pr[c] + sB[c] - qr[c], 0.f), sW[c], a[0]);
    float acc = (a[0] + a[1]) + (a[2] + a[3]);
#pragma unroll
    for (int o = 1; o < kTPE; o <<= 1) acc += __shfl_xor(acc, o);
    if (valid && qd == 0) ob[i * Nt + j] = sh + acc + bias2;
  }
}

// dP[i][c]  =  w2_c * sum_j G_ij [P_ic + b1_c > Q_jc]
// dQ[j][c]  = -w2_c * sum_i G_ij [P_ic + b1_c > Q_jc]
// dw2[c]    =  sum_ij G_ij relu(P_ic + b1_c - Q_jc)    (per-pair partial)
// db2       =  sum_ij G_ij                             (per-pair partial)
// LDS: sP [Ns][R], sQ [Nt][R] (lanes run along channels: conflict-free),
//      sG [Ns][Nt], sB [R], sW [R], sRed [kThreads].
template <typename TPQ>
__global__ __launch_bounds__(kThreads) void consensus_bwd_kernel(
    const float* __restrict__ G, const TPQ* __restrict__ P,
    const TPQ* __restrict__ Q, const float* __restrict__ b1,
    const float* __restrict__ w2, const int* __restrict__ ptr_s,
    const int* __restrict__ ptr_t, TPQ* __restrict__ dP,
    TPQ* __restrict__ dQ, float* __restrict__ dw2_part,
    float* __restrict__ db2_part, int Ns, int Nt, int R, int rows_s,
    int rows_t, int vec) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  DGMC_LDS float* sP = (DGMC_LDS float*)smem_raw;
  DGMC_LDS float* sQ = sP + Ns * R;
  DGMC_LDS float* sG = sQ + Nt * R;
  DGMC_LDS float* sB = sG + Ns * Nt;
  DGMC_LDS float* sW = sB + R;
  DGMC_LDS float* sRed = sW + R;
  const int b = xcd_remap(blockIdx.x, gridDim.x);
  const int tid = threadIdx.x;
  const int wave = tid / kWave, lane = tid % kWave;
  const int s0 = ptr_s[b], ns = ptr_s[b + 1] - s0;
  const int t0 = ptr_t[b], nt = ptr_t[b + 1] - t0;
  const int NN = Ns * Nt;
  const float* Gb = G + (size_t)b * NN;
  float pre[kPrefetch];
  prefetch_tile(Gb, NN, pre);
  float bw[2] = {0.f, 0.f};
  if (tid < R) {
    bw[0] = b1[tid];
    bw[1] = w2[tid];
  }
  stage_rows<TPQ>(sP, P + (size_t)s0 * R, ns, sQ, Q + (size_t)t0 * R, nt, R,
                  R, vec != 0);
  if (tid < R) {
    sB[tid] = bw[0];
    sW[tid] = bw[1];
  }
  for (int c = tid + kThreads; c < R; c += kThreads) {
    sB[c] = b1[c];
    sW[c] = w2[c];
  }
  // Masked upstream gradient tile + db2 partial.
  float gsum = 0.f;
#pragma unroll
  for (int u = 0; u < kPrefetch; ++u) {
    const int e = tid + u * kThreads;
    if (e < NN) {
      const int i = e / Nt, j = e - (e / Nt) * Nt;
      const float v = (i < ns && j < nt) ? pre[u] : 0.f;
      sG[e] = v;
      gsum += v;
    }
  }
  for (int e = tid + kPrefetch * kThreads; e < NN; e += kThreads) {
    const int i = e / Nt, j = e - (e / Nt) * Nt;
    const float v = (i < ns && j < nt) ? Gb[e] : 0.f;
    sG[e] = v;
    gsum += v;
  }
  gsum = wave_sum(gsum);
  if (lane == 0) sRed[wave] = gsum;
  if (blockIdx.x == gridDim.x - 1) {
    zero_tail(dP, ptr_s[gridDim.x], rows_s, R);
    zero_tail(dQ, ptr_t[gridDim.x], rows_t, R);
  }
  __syncthreads();
  if (tid == 0) {
    float t = 0.f;
    for (int w = 0; w < kWaves; ++w) t += sRed[w];
    db2_part[b] = t;
  }
  TPQ* dPb = dP + (size_t)s0 * R;
  TPQ* dQb = dQ + (size_t)t0 * R;

  for (int c0 = 0; c0 < R; c0 += kThreads) {
    const ChanMap cm(c0, R);
    const int c = cm.c;
    __syncthreads();   // sRed reuse
    float dw = 0.f;
    if (cm.active) {
      const float bias1 = sB[c], w = sW[c];
      // dP rows i = r0, r0 + rp, ...; dw2 partial over the same rows.
      for (int i = cm.r0; i < ns; i += cm.rp) {
        const float p = sP[i * R + c] + bias1;
        float dp[4] = {0.f, 0.f, 0.f, 0.f}, dwq[4] = {0.f, 0.f, 0.f, 0.f};
        int j = 0;
        for (; j + 4 <= nt; j += 4) {
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const float z = fmaxf(p - sQ[(j + u) * R + c], 0.f);
            const float gij = sG[i * Nt + j + u];
            dp[u] += z > 0.f ? gij : 0.f;
            dwq[u] = fmaf(gij, z, dwq[u]);
          }
        }
        for (; j < nt; ++j) {
          const float z = fmaxf(p - sQ[j * R + c], 0.f);
          const float gij = sG[i * Nt + j];
          dp[0] += z > 0.f ? gij : 0.f;
          dwq[0] = fmaf(gij, z, dwq[0]);
        }
        dw += (dwq[0] + dwq[1]) + (dwq[2] + dwq[3]);
        dPb[(size_t)i * R + c] =
            Cvt<TPQ>::from_f(((dp[0] + dp[1]) + (dp[2] + dp[3])) * w);
      }
      // dQ rows j = r0, r0 + rp, ...
      for (int j = cm.r0; j < nt; j += cm.rp) {
        // Same predicate as the forward: (P + b1) - Q > 0.
        const float qv = sQ[j * R + c];
        float dq[4] = {0.f, 0.f, 0.f, 0.f};
        int i = 0;
        for (; i + 4 <= ns; i += 4) {
#pragma unroll
          for (int u = 0; u < 4; ++u)
            dq[u] += (sP[(i + u) * R + c] + bias1) - qv > 0.f
                         ? sG[(i + u) * Nt + j] : 0.f;
        }
        for (; i < ns; ++i)
          dq[0] += (sP[i * R + c] + bias1) - qv > 0.f ? sG[i * Nt + j] : 0.f;
        dQb[(size_t)j * R + c] =
            Cvt<TPQ>::from_f(-((dq[0] + dq[1]) + (dq[2] + dq[3])) * w);
      }
    }
    // dw2: fixed-order reduction over the row groups (deterministic).
    sRed[tid] = dw;
    __syncthreads();
    if (tid < cm.cw) {
      float s = 0.f;
      for (int r = 0; r < cm.rp; ++r) s += sRed[r * cm.cw + tid];
      dw2_part[(size_t)b * R + c0 + tid] = s;
    }
  }
}

// ---------------------------------------------------------------------------
// Fused step boundary of the consensus loop: consensus update of step l
// followed by the softmax + transport of step l + 1, per pair in ONE
// workgroup (the updated S_hat tile never leaves LDS between the two):
//
//   S_hat' = S_hat + mask * (relu(P_i + b1 - Q_j) . w2 + b2)     (step l)
//   S      = masked_softmax(S_hat')                               (step l+1)
//   joint  = [r_s; S^T r_s]                                       (step l+1)
//
// Outputs S_hat' (the step's result), S (saved for the backward) and the
// joint psi_2 input.  LDS: sP, sQ [N][R+1], sB, sW [R], sR [Ns][R], sS [NN].
// ---------------------------------------------------------------------------
template <typename TPQ, typename TR>
__global__ __launch_bounds__(kThreads) void consensus_transport_kernel(
    const float* __restrict__ S_hat, const TPQ* __restrict__ P,
    const TPQ* __restrict__ Q, const float* __restrict__ b1,
    const float* __restrict__ w2, const float* __restrict__ b2,
    const TR* __restrict__ r_s, const int* __restrict__ ptr_s,
    const int* __restrict__ ptr_t, float* __restrict__ S_new,
    float* __restrict__ S_prob, TR* __restrict__ joint, int Ns, int Nt,
    int R, int rows_s, int rows_t, int vec_pq, int vec_r) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  const int pitch = R + 1;
  DGMC_LDS float* sP = (DGMC_LDS float*)smem_raw;
  DGMC_LDS float* sQ = sP + Ns * pitch;
  DGMC_LDS float* sB = sQ + Nt * pitch;
  DGMC_LDS float* sW = sB + R;
  DGMC_LDS float* sR = sW + R;
  DGMC_LDS float* sS = sR + Ns * R;
  const int b = xcd_remap(blockIdx.x, gridDim.x);
  const int tid = threadIdx.x;
  const int wave = tid / kWave, lane = tid % kWave;
  const int s0 = ptr_s[b], ns = ptr_s[b + 1] - s0;
  const int t0 = ptr_t[b], nt = ptr_t[b + 1] - t0;
  const int NN = Ns * Nt;
  const float* Sh = S_hat + (size_t)b * NN;
  float pre[kPrefetch];
  prefetch_tile(Sh, NN, pre);
  float bw[2] = {0.f, 0.f};
  if (tid < R) {
    bw[0] = b1[tid];
    bw[1] = w2[tid];
  }
  stage_rows<TPQ>(sP, P + (size_t)s0 * R, ns, sQ, Q + (size_t)t0 * R, nt,
                  pitch, R, vec_pq != 0);
  stage_rows<TR>(sR, r_s + (size_t)s0 * R, ns, sR, r_s, 0, R, R, vec_r != 0);
  if (tid < R) {
    sB[tid] = bw[0];
    sW[tid] = bw[1];
  }
  for (int c = tid + kThreads; c < R; c += kThreads) {
    sB[c] = b1[c];
    sW[c] = w2[c];
  }
#pragma unroll
  for (int u = 0; u < kPrefetch; ++u) {
    const int e = tid + u * kThreads;
    if (e < NN) sS[e] = pre[u];
  }
  for (int e = tid + kPrefetch * kThreads; e < NN; e += kThreads) sS[e] = Sh[e];
  // Static-batch padding rows: r_t tail zeroed, r_s tail copied (the joint
  // buffer covers every row of both graphs).
  if (blockIdx.x == gridDim.x - 1)
    zero_tail(joint + (size_t)rows_s * R, ptr_t[gridDim.x], rows_t, R);
  {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t e = (size_t)ptr_s[gridDim.x] * R +
                    (size_t)blockIdx.x * blockDim.x + tid;
         e < (size_t)rows_s * R; e += stride)
      joint[e] = r_s[e];
  }
  const float bias2 = b2[0];
  __syncthreads();

  // 1. consensus update of the valid ns x nt block (kTPE lanes per entry).
  float* ob = S_new + (size_t)b * NN;
  const int qd = tid % kTPE;
  const int pairs = ns * nt;
  for (int p0 = 0; p0 < pairs; p0 += kThreads / kTPE) {
    const int p = p0 + tid / kTPE;
    const bool valid = p < pairs;
    const int i = valid ? p / nt : 0;
    const int j = valid ? p - i * nt : 0;
    const DGMC_LDS float* pr = sP + i * pitch;
    const DGMC_LDS float* qr = sQ + j * pitch;
    float a[4] = {0.f, 0.f, 0.f, 0.f};
    int c = qd;
    for (; c + 3 * kTPE < R; c += 4 * kTPE) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int cc = c + kTPE * u;
        a[u] = fmaf(fmaxf(pr[cc] + sB[cc] - qr[cc], 0.f), sW[cc], a[u]);
      }
    }
    for (; c < R; c += kTPE)
      a[0] = fmaf(fmaxf(pr[c] + sB[c] - qr[c], 0.f), sW[c], a[0]);
    float acc = (a[0] + a[1]) + (a[2] + a[3]);
#pragma unroll
    for (int o = 1; o < kTPE; o <<= 1) acc += __shfl_xor(acc, o);
    if (valid && qd == 0) sS[i * Nt + j] += acc + bias2;
  }
  __syncthreads();

  // 2. Updated tile out (entries outside the valid block pass through) and
  //    its masked row softmax; each row belongs to one wave, so the in-place
  //    LDS update is race free.
  float* Sb = S_prob + (size_t)b * NN;
  for (int i = wave; i < Ns; i += kWaves) {
    const float raw = lane < Nt ? sS[i * Nt + lane] : 0.f;
    if (lane < Nt) ob[i * Nt + lane] = raw;
    const bool valid = i < ns && lane < nt;
    const float v = valid ? raw : -INFINITY;
    const float m = wave_max(v);
    const float e = valid ? __expf(v - m) : 0.f;
    const float sum = wave_sum(e);
    const float pv = valid ? e / sum : 0.f;
    if (lane < Nt) {
      Sb[i * Nt + lane] = pv;
      sS[i * Nt + lane] = pv;
    }
  }
  {
    TR* dst = joint + (size_t)s0 * R;
    for (int e = tid; e < ns * R; e += kThreads)
      dst[e] = Cvt<TR>::from_f(sR[e]);
  }
  __syncthreads();

  // 3. transport r_t = S^T r_s (channel-parallel lanes).
  TR* rt = joint + ((size_t)rows_s + t0) * R;
  for (int c0 = 0; c0 < R; c0 += kThreads) {
    const ChanMap cm(c0, R);
    if (!cm.active) continue;
    for (int j = cm.r0; j < nt; j += cm.rp) {
      float a[4] = {0.f, 0.f, 0.f, 0.f};
      int i = 0;
      for (; i + 4 <= ns; i += 4) {
#pragma unroll
        for (int u = 0; u < 4; ++u)
          a[u] = fmaf(sS[(i + u) * Nt + j], sR[(i + u) * R + cm.c], a[u]);
      }
      for (; i < ns; ++i) a[0] = fmaf(sS[i * Nt + j], sR[i * R + cm.c], a[0]);
      rt[(size_t)j * R + cm.c] =
          Cvt<TR>::from_f((a[0] + a[1]) + (a[2] + a[3]));
    }
  }
}

// Backward of the fused step boundary, per pair:
//   dS_hat' = softmax_bwd(S, r_s g_t^T) + addend          (step l+1 transport
//             + the next step's identity path)
//   then the consensus backward of step l with G = dS_hat':
//   dP, dQ (joint buffer), dw2 / db2 per-pair partials; G is also written
//   out as the gradient of step l's input S_hat (identity path).
// LDS: sR, sGt [N][R+1] (phase 1), sP, sQ [N][R] (phase 2), sD [NN],
//      sB, sW [R], sRed [kThreads].
template <typename TPQ, typename TR>
__global__ __launch_bounds__(kThreads) void transport_consensus_bwd_kernel(
    const float* __restrict__ S, const TR* __restrict__ r_s,
    const TR* __restrict__ g_t, const float* __restrict__ addend,
    const TPQ* __restrict__ P, const TPQ* __restrict__ Q,
    const float* __restrict__ b1, const float* __restrict__ w2,
    const int* __restrict__ ptr_s, const int* __restrict__ ptr_t,
    float* __restrict__ G_out, TPQ* __restrict__ dP, TPQ* __restrict__ dQ,
    float* __restrict__ dw2_part, float* __restrict__ db2_part, int Ns,
    int Nt, int R, int rows_s, int rows_t, int vec_r, int vec_pq) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  const int pitch = R + 1;
  DGMC_LDS float* sR = (DGMC_LDS float*)smem_raw;
  DGMC_LDS float* sGt = sR + Ns * pitch;
  DGMC_LDS float* sP = sGt + Nt * pitch;
  DGMC_LDS float* sQ = sP + Ns * R;
  DGMC_LDS float* sD = sQ + Nt * R;
  DGMC_LDS float* sB = sD + Ns * Nt;
  DGMC_LDS float* sW = sB + R;
  DGMC_LDS float* sRed = sW + R;
  const int b = xcd_remap(blockIdx.x, gridDim.x);
  const int tid = threadIdx.x;
  const int wave = tid / kWave, lane = tid % kWave;
  const int s0 = ptr_s[b], ns = ptr_s[b + 1] - s0;
  const int t0 = ptr_t[b], nt = ptr_t[b + 1] - t0;
  const int NN = Ns * Nt;
  const float* Sb = S + (size_t)b * NN;
  constexpr int QMAX = kMaxN / kWaves;
  float sv[QMAX], av[QMAX];
#pragma unroll
  for (int q = 0; q < QMAX; ++q) {
    const int i = wave + q * kWaves;
    const bool in = i < Ns && lane < Nt;
    sv[q] = in ? Sb[i * Nt + lane] : 0.f;
    av[q] = (in && addend) ? addend[(size_t)b * NN + i * Nt + lane] : 0.f;
  }
  float bw[2] = {0.f, 0.f};
  if (tid < R) {
    bw[0] = b1[tid];
    bw[1] = w2[tid];
  }
  stage_rows<TR>(sR, r_s + (size_t)s0 * R, ns, sGt, g_t + (size_t)t0 * R, nt,
                 pitch, R, vec_r != 0);
  stage_rows<TPQ>(sP, P + (size_t)s0 * R, ns, sQ, Q + (size_t)t0 * R, nt, R,
                  R, vec_pq != 0);
  if (tid < R) {
    sB[tid] = bw[0];
    sW[tid] = bw[1];
  }
  for (int c = tid + kThreads; c < R; c += kThreads) {
    sB[c] = b1[c];
    sW[c] = w2[c];
  }
  if (blockIdx.x == gridDim.x - 1) {
    zero_tail(dP, ptr_s[gridDim.x], rows_s, R);
    zero_tail(dQ, ptr_t[gridDim.x], rows_t, R);
  }
  __syncthreads();

  // Phase 1: dS[i][j] = <r_s[i], g_t[j]> (kTPE lanes per entry).
  {
    const int qd = tid % kTPE;
    const int pairs = ns * nt;
    for (int p0 = 0; p0 < pairs; p0 += kThreads / kTPE) {
      const int p = p0 + tid / kTPE;
      const bool valid = p < pairs;
      const int i = valid ? p / nt : 0;
      const int j = valid ? p - i * nt : 0;
      const DGMC_LDS float* rr = sR + i * pitch;
      const DGMC_LDS float* gr = sGt + j * pitch;
      float a[4] = {0.f, 0.f, 0.f, 0.f};
      int c = qd;
      for (; c + 3 * kTPE < R; c += 4 * kTPE) {
#pragma unroll
        for (int u = 0; u < 4; ++u)
          a[u] = fmaf(rr[c + kTPE * u], gr[c + kTPE * u], a[u]);
      }
      for (; c < R; c += kTPE) a[0] = fmaf(rr[c], gr[c], a[0]);
      float acc = (a[0] + a[1]) + (a[2] + a[3]);
#pragma unroll
      for (int o = 1; o < kTPE; o <<= 1) acc += __shfl_xor(acc, o);
      if (valid && qd == 0) sD[i * Nt + j] = acc;
    }
  }
  __syncthreads();
  // Softmax backward + addend -> G (global: step l's S_hat gradient; LDS:
  // the consensus backward's upstream tile, masked to the valid block).
  float* Gb = G_out + (size_t)b * NN;
  float gsum = 0.f;
#pragma unroll
  for (int q = 0; q < QMAX; ++q) {
    const int i = wave + q * kWaves;
    if (i < Ns) {
      const bool valid = i < ns && lane < nt;
      const float d = valid ? sD[i * Nt + lane] : 0.f;
      const float dot = wave_sum(sv[q] * d);
      const float gv = sv[q] * (d - dot) + av[q];
      if (lane < Nt) Gb[i * Nt + lane] = gv;
      const float gm = valid ? gv : 0.f;
      gsum += gm;
      sv[q] = gm;           // kept for the LDS store after the barrier
    }
  }
  __syncthreads();          // every wave has read its sD row
#pragma unroll
  for (int q = 0; q < QMAX; ++q) {
    const int i = wave + q * kWaves;
    if (i < Ns && lane < Nt) sD[i * Nt + lane] = sv[q];
  }
  gsum = wave_sum(gsum);
  if (lane == 0) sRed[wave] = gsum;
  __syncthreads();
  if (tid == 0) {
    float t = 0.f;
    for (int w = 0; w < kWaves; ++w) t += sRed[w];
    db2_part[b] = t;
  }

  // Phase 2: consensus backward with G = sD (as consensus_bwd_kernel).
  TPQ* dPb = dP + (size_t)s0 * R;
  TPQ* dQb = dQ + (size_t)t0 * R;
  for (int c0 = 0; c0 < R; c0 += kThreads) {
    const ChanMap cm(c0, R);
    const int c = cm.c;
    __syncthreads();   // sRed reuse
    float dw = 0.f;
    if (cm.active) {
      const float bias1 = sB[c], w = sW[c];
      for (int i = cm.r0; i < ns; i += cm.rp) {
        const float p = sP[i * R + c] + bias1;
        float dp[4] = {0.f, 0.f, 0.f, 0.f}, dwq[4] = {0.f, 0.f, 0.f, 0.f};
        int j = 0;
        for (; j + 4 <= nt; j += 4) {
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const float z = fmaxf(p - sQ[(j + u) * R + c], 0.f);
            const float gij = sD[i * Nt + j + u];
            dp[u] += z > 0.f ? gij : 0.f;
            dwq[u] = fmaf(gij, z, dwq[u]);
          }
        }
        for (; j < nt; ++j) {
          const float z = fmaxf(p - sQ[j * R + c], 0.f);
          const float gij = sD[i * Nt + j];
          dp[0] += z > 0.f ? gij : 0.f;
          dwq[0] = fmaf(gij, z, dwq[0]);
        }
        dw += (dwq[0] + dwq[1]) + (dwq[2] + dwq[3]);
        dPb[(size_t)i * R + c] =
            Cvt<TPQ>::from_f(((dp[0] + dp[1]) + (dp[2] + dp[3])) * w);
      }
      for (int j = cm.r0; j < nt; j += cm.rp) {
        const float qv = sQ[j * R + c];
        float dq[4] = {0.f, 0.f, 0.f, 0.f};
        int i = 0;
        for (; i + 4 <= ns; i += 4) {
#pragma unroll
          for (int u = 0; u < 4; ++u)
            dq[u] += (sP[(i + u) * R + c] + bias1) - qv > 0.f
                         ? sD[(i + u) * Nt + j] : 0.f;
        }
        for (; i < ns; ++i)
          dq[0] += (sP[i * R + c] + bias1) - qv > 0.f ? sD[i * Nt + j] : 0.f;
        dQb[(size_t)j * R + c] =
            Cvt<TPQ>::from_f(-((dq[0] + dq[1]) + (dq[2] + dq[3])) * w);
      }
    }
    sRed[tid] = dw;
    __syncthreads();
    if (tid < cm.cw) {
      float s = 0.f;
      for (int r = 0; r < cm.rp; ++r) s += sRed[r * cm.cw + tid];
      dw2_part[(size_t)b * R + c0 + tid] = s;
    }
  }
}

// ---------------------------------------------------------------------------
// Step-boundary kernels for a compile-time width R (32 / 64 / 128, bf16 rows).
//
// Same math as consensus_transport_kernel / transport_consensus_bwd_kernel,
// re-laid out for the LDS pipe (the generic kernels spend most of their time
// in ds_read_b32 with 4-way bank conflicts):
//   * (i, j) entry dots use 4 lanes per entry reading 16-byte quads of
//     channels (ds_read_b128); rows of the entry operands have the pitch
//     PP = R + ((16 - R) mod 64) dwords, so the 4 entries sharing one b128
//     lane group fall on disjoint banks for consecutive j;
//   * b1 / w2 of a lane's channels live in registers;
//   * channel-parallel loops (transport, dP / dQ) take one channel quad per
//     lane (b128 row reads, 8-byte bf16 stores);
//   * quad / wave reductions by DPP (no ds_bpermute);
//   * all operand loads of a pair issue in one batch, r_s rows are copied to
//     the joint output from the load registers, and static-batch padding
//     rows are handled by every workgroup with 16-byte accesses.
// ---------------------------------------------------------------------------
namespace {
typedef __bf16 ps_bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 ps_bf16x4 __attribute__((ext_vector_type(4)));
typedef float ps_f32x4 __attribute__((ext_vector_type(4)));

template <int R>
struct StepGeom {
  static constexpr int PP = R + ((16 - R) & 63);   // entry-operand row pitch
  static constexpr int RU = R / 16;                // b128 quads per lane/entry
  static constexpr int V8 = R / 8;                 // bf16x8 vectors per row
  static constexpr int CQ = R / 4;                 // channel quads
  static constexpr int RG = kThreads / CQ;         // row groups (channel loops)
};

// Node-level storage type of the step kernels: bf16 (autocast) or fp32
// (reference precision).  16-byte vectors: 8 bf16 / 4 fp32 channels.
template <typename T> struct StepIO;
template <> struct StepIO<__bf16> {
  typedef ps_bf16x8 vec;
  static constexpr int VN = 8;
  __device__ __forceinline__ static void to_lds(DGMC_LDS float* d,
                                                const vec& v) {
    reinterpret_cast<DGMC_LDS ps_f32x4*>(d)[0] =
        ps_f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
    reinterpret_cast<DGMC_LDS ps_f32x4*>(d)[1] =
        ps_f32x4{(float)v[4], (float)v[5], (float)v[6], (float)v[7]};
  }
  __device__ __forceinline__ static void store4(__bf16* p, ps_f32x4 a) {
    *reinterpret_cast<ps_bf16x4*>(p) =
        ps_bf16x4{(__bf16)a[0], (__bf16)a[1], (__bf16)a[2], (__bf16)a[3]};
  }
};
template <> struct StepIO<float> {
  typedef ps_f32x4 vec;
  static constexpr int VN = 4;
  __device__ __forceinline__ static void to_lds(DGMC_LDS float* d,
                                                const vec& v) {
    *reinterpret_cast<DGMC_LDS ps_f32x4*>(d) = v;
  }
  __device__ __forceinline__ static void store4(float* p, ps_f32x4 a) {
    *reinterpret_cast<ps_f32x4*>(p) = a;
  }
};

// Four fp32 values as their bf16x6 operand planes (common.h split3_bf16,
// the same split as slot_gemm_x6.hip's split3): p -> planes 0 / 1 / 2 at
// p, p + ps, p + 2 ps.
__device__ __forceinline__ void store_planes4(__bf16* p, size_t ps,
                                              ps_f32x4 a) {
  ps_bf16x4 h, m, l;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    __bf16 he, me, le;
    split3_bf16(a[e], he, me, le);
    h[e] = he;
    m[e] = me;
    l[e] = le;
  }
  *reinterpret_cast<ps_bf16x4*>(p) = h;
  *reinterpret_cast<ps_bf16x4*>(p + ps) = m;
  *reinterpret_cast<ps_bf16x4*>(p + 2 * ps) = l;
}

// One operand block staged by stage_blocks: rows [0, rows) of a packed
// [*, R] block (storage T) into an fp32 LDS tile of pitch `pitch`,
// optionally copied verbatim to `copy` (same row layout).
template <typename T>
struct StageBlk {
  const T* src;
  DGMC_LDS float* dst;
  T* copy;
  int rows, pitch;
};

// All loads of up to NB blocks are issued before the first LDS store (one
// memory round trip for pair-sized blocks).
template <int R, int NB, typename T>
__device__ __forceinline__ void stage_blocks(const StageBlk<T> (&blk)[NB]) {
  using IO = StepIO<T>;
  constexpr int VN = IO::VN;
  constexpr int V8 = R / VN;
  int end[NB];
  int total = 0;
#pragma unroll
  for (int k = 0; k < NB; ++k) {
    total += blk[k].rows * V8;
    end[k] = total;
  }
  for (int base = threadIdx.x; base < total; base += 4 * kThreads) {
    typename IO::vec v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int q = base + u * kThreads;
      if (q < total) {
        int k = 0, q0 = 0;
#pragma unroll
        for (int m = 0; m + 1 < NB; ++m)
          if (q >= end[m]) { k = m + 1; q0 = end[m]; }
        const T* src = blk[0].src;
#pragma unroll
        for (int m = 1; m < NB; ++m) if (k == m) src = blk[m].src;
        v[u] = *reinterpret_cast<const typename IO::vec*>(
            src + (size_t)(q - q0) * VN);
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int q = base + u * kThreads;
      if (q < total) {
        int k = 0, q0 = 0;
#pragma unroll
        for (int m = 0; m + 1 < NB; ++m)
          if (q >= end[m]) { k = m + 1; q0 = end[m]; }
        StageBlk<T> bk = blk[0];
#pragma unroll
        for (int m = 1; m < NB; ++m) if (k == m) bk = blk[m];
        const int qq = q - q0, r = qq / V8, c = (qq - r * V8) * VN;
        IO::to_lds(bk.dst + r * bk.pitch + c, v[u]);
        if (bk.copy)
          *reinterpret_cast<typename IO::vec*>(bk.copy + (size_t)qq * VN) =
              v[u];

      }
    }
  }
}

// Static-batch padding rows spread over the whole grid in 16-byte pieces:
// rows [z0, z1) of zdst zeroed and rows [c0, c1) of csrc copied to cdst
// (fp32 only: also as bf16x6 planes at pz / pc, rows laid out like zdst /
// cdst, plane stride ps).
template <int R, typename T>
__device__ __forceinline__ void pad_rows(T* zdst, int z0, int z1, T* cdst,
                                         const T* csrc, int c0, int c1,
                                         __bf16* pz = nullptr,
                                         __bf16* pc = nullptr, size_t ps = 0) {
  using V = typename StepIO<T>::vec;
  constexpr int VN = StepIO<T>::VN;
  constexpr int V8 = R / VN;
  const int nz = (z1 - z0) * V8, nc = cdst ? (c1 - c0) * V8 : 0;
  const int stride = gridDim.x * blockDim.x;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < nz + nc;
       e += stride) {
    if (e < nz) {
      const size_t off = (size_t)z0 * R + (size_t)e * VN;
      *reinterpret_cast<V*>(zdst + off) = V{};
      if constexpr (VN == 4)
        if (pz) store_planes4(pz + off, ps, V{});
    } else {
      const size_t off = (size_t)c0 * R + (size_t)(e - nz) * VN;
      const V v = *reinterpret_cast<const V*>(csrc + off);
      *reinterpret_cast<V*>(cdst + off) = v;
      if constexpr (VN == 4)
        if (pc) store_planes4(pc + off, ps, v);
    }
  }
}

__device__ __forceinline__ ps_f32x4 lds4(const DGMC_LDS float* p) {
  return *reinterpret_cast<const DGMC_LDS ps_f32x4*>(p);
}
}  // namespace

// Step kernels.  CONS: consensus update (forward) / its backward; TRANS:
// masked softmax + transport r_t = S^T r_s (forward) / its backward.  Both:
// the fused step boundary (consensus of step l, transport of step l + 1).
// Forward LDS: sP, sQ [N][PP] (CONS), sR [Ns][R] (TRANS), sS [Ns][Nt].
// Outputs: S_new (CONS: the updated S_hat), S_prob (TRANS), rt_out packed
// [rows_t, R] (TRANS) and, when rs_copy is given, r_s copied into it (the
// joint psi_2 input [r_s; r_t]).
template <int R, bool CONS, bool TRANS, typename T>
__global__ __launch_bounds__(kThreads) void pair_step_fwd_kernel(
    const float* __restrict__ S_hat, const T* __restrict__ P,
    const T* __restrict__ Q, const float* __restrict__ b1,
    const float* __restrict__ w2, const float* __restrict__ b2,
    const T* __restrict__ r_s, const int* __restrict__ ptr_s,
    const int* __restrict__ ptr_t, float* __restrict__ S_new,
    float* __restrict__ S_prob, T* __restrict__ rs_copy,
    T* __restrict__ rt_out, __bf16* __restrict__ planes, int Ns, int Nt,
    int rows_s, int rows_t) {
  using G = StepGeom<R>;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  DGMC_LDS float* sP = (DGMC_LDS float*)smem_raw;
  DGMC_LDS float* sQ = sP + (CONS ? Ns * G::PP : 0);
  DGMC_LDS float* sR = sQ + (CONS ? Nt * G::PP : 0);
  DGMC_LDS float* sS = sR + (TRANS ? Ns * R : 0);
  const int b = xcd_remap(blockIdx.x, gridDim.x);
  const int tid = threadIdx.x;
  const int wave = tid / kWave, lane = tid % kWave;
  const int s0 = ptr_s[b], ns = ptr_s[b + 1] - s0;
  const int t0 = ptr_t[b], nt = ptr_t[b + 1] - t0;
  const int NN = Ns * Nt;
  const float* Sh = S_hat + (size_t)b * NN;
  float pre[kPrefetch];
  prefetch_tile(Sh, NN, pre);
  // This lane's channels in the entry loop: 4 qd + 16 u + (0..3).
  const int qd = tid & 3;
  ps_f32x4 bv[CONS ? G::RU : 1], wv[CONS ? G::RU : 1];
  float bias2 = 0.f;
  if constexpr (CONS) {
#pragma unroll
    for (int u = 0; u < G::RU; ++u) {
      bv[u] = *reinterpret_cast<const ps_f32x4*>(b1 + 4 * qd + 16 * u);
      wv[u] = *reinterpret_cast<const ps_f32x4*>(w2 + 4 * qd + 16 * u);
    }
    bias2 = b2[0];
  }
  T* rsc = rs_copy ? rs_copy + (size_t)s0 * R : nullptr;
  // bf16x6 planes of the joint [r_s; r_t] (psi_2's operand; fp32 only, with
  // rs_copy): plane stride ps, r_t rows from row rows_s.  Written after the
  // last global load of the workgroup (vmcnt counts stores too: stores
  // issued during the staging would stall its load waits).
  const size_t ps = (size_t)(rows_s + rows_t) * R;
  if constexpr (CONS && TRANS) {
    const StageBlk<T> blk[3] = {{P + (size_t)s0 * R, sP, nullptr, ns, G::PP},
                             {Q + (size_t)t0 * R, sQ, nullptr, nt, G::PP},
                             {r_s + (size_t)s0 * R, sR, rsc, ns, R}};
    stage_blocks<R, 3>(blk);
  } else if constexpr (CONS) {
    const StageBlk<T> blk[2] = {{P + (size_t)s0 * R, sP, nullptr, ns, G::PP},
                                {Q + (size_t)t0 * R, sQ, nullptr, nt, G::PP}};
    stage_blocks<R, 2>(blk);
  } else {
    const StageBlk<T> blk[1] = {{r_s + (size_t)s0 * R, sR, rsc, ns, R}};
    stage_blocks<R, 1>(blk);
  }
#pragma unroll
  for (int u = 0; u < kPrefetch; ++u) {
    const int e = tid + u * kThreads;
    if (e < NN) sS[e] = pre[u];
  }
  for (int e = tid + kPrefetch * kThreads; e < NN; e += kThreads) sS[e] = Sh[e];
  __bf16* plt = (planes && rs_copy) ? planes + (size_t)rows_s * R : nullptr;
  if constexpr (TRANS)
    pad_rows<R, T>(rt_out, ptr_t[gridDim.x], rows_t, rs_copy, r_s,
                   ptr_s[gridDim.x], rows_s, plt, plt ? planes : nullptr, ps);
  __syncthreads();

  // 1. consensus update of the valid block: 4 lanes per (i, j) entry.
  if constexpr (CONS) {
    const int pairs = ns * nt;
    for (int p0 = 0; p0 < pairs; p0 += kThreads / 4) {
      const int p = p0 + (tid >> 2);
      const bool valid = p < pairs;
      const int i = valid ? p / nt : 0;
      const int j = valid ? p - i * nt : 0;
      const DGMC_LDS float* pr = sP + i * G::PP + 4 * qd;
      const DGMC_LDS float* qr = sQ + j * G::PP + 4 * qd;
      ps_f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int u = 0; u < G::RU; ++u) {
        const ps_f32x4 pv = lds4(pr + 16 * u), qv = lds4(qr + 16 * u);
#pragma unroll
        for (int k = 0; k < 4; ++k)
          acc[k] =
              fmaf(fmaxf(pv[k] + bv[u][k] - qv[k], 0.f), wv[u][k], acc[k]);
      }
      const float s = quad_sum((acc[0] + acc[1]) + (acc[2] + acc[3]));
      if (valid && qd == 0) sS[i * Nt + j] += s + bias2;
    }
    __syncthreads();
  }
  float* ob = S_new + (size_t)b * NN;
  if constexpr (!TRANS) {
    for (int e = tid; e < NN; e += kThreads) ob[e] = sS[e];
    return;
  }

  // 2. (updated tile out and) masked row softmax, one wave per row.
  float* Sb = S_prob + (size_t)b * NN;
  for (int i = wave; i < Ns; i += kWaves) {
    const float raw = lane < Nt ? sS[i * Nt + lane] : 0.f;
    if (CONS && lane < Nt) ob[i * Nt + lane] = raw;
    const bool valid = i < ns && lane < nt;
    const float v = valid ? raw : -INFINITY;
    const float m = wave_max_dpp(v);
    const float e = valid ? __expf(v - m) : 0.f;
    const float sum = wave_sum_dpp(e);
    const float pv = valid ? e / sum : 0.f;
    if (lane < Nt) {
      Sb[i * Nt + lane] = pv;
      sS[i * Nt + lane] = pv;
    }
  }
  __syncthreads();

  // 3. r_t = S^T r_s: one channel quad per lane, two rows j per pass.
  T* rt = rt_out + (size_t)t0 * R;
  const int cq = tid % G::CQ, rg = tid / G::CQ;
  for (int j0 = rg; j0 < nt; j0 += 2 * G::RG) {
    const int j1 = j0 + G::RG;
    const bool has1 = j1 < nt;
    ps_f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
    for (int i = 0; i < ns; ++i) {
      const ps_f32x4 rv = lds4(sR + i * R + 4 * cq);
      const float w0 = sS[i * Nt + j0];
      const float w1 = has1 ? sS[i * Nt + j1] : 0.f;
      a0 += w0 * rv;
      a1 += w1 * rv;
    }
    StepIO<T>::store4(rt + (size_t)j0 * R + 4 * cq, a0);
    if (has1) StepIO<T>::store4(rt + (size_t)j1 * R + 4 * cq, a1);
    if constexpr (std::is_same<T, float>::value) {
      if (plt) {
        __bf16* pj = plt + (size_t)t0 * R + 4 * cq;
        store_planes4(pj + (size_t)j0 * R, ps, a0);
        if (has1) store_planes4(pj + (size_t)j1 * R, ps, a1);
      }
    }
  }
  // the pair's r_s rows as planes, from their fp32 LDS image
  if constexpr (std::is_same<T, float>::value) {
    if (plt) {
      __bf16* pr = planes + (size_t)s0 * R;
      for (int q = tid; q < ns * (R / 4); q += kThreads)
        store_planes4(pr + (size_t)q * 4, ps, lds4(sR + q * 4));
    }
  }
}

// Backward.  TRANS: dS = softmax_bwd(S, r_s g_t^T) + addend -> G_out (the
// S_hat' gradient); CONS: the consensus backward with upstream G (TRANS: the
// G just formed; otherwise `S` is the upstream gradient tile) -> dP, dQ rows
// and per-pair dw2 / db2 partials.
// LDS: sR, sGt [N][PP] (TRANS; reused as sRed [RG][R]), sP, sQ [N][R]
// (CONS), sD [NN], sSum [kWaves].
template <int R, bool CONS, bool TRANS, typename T>
__global__ __launch_bounds__(kThreads) void pair_step_bwd_kernel(
    const float* __restrict__ S, const T* __restrict__ r_s,
    const T* __restrict__ g_t, const float* __restrict__ addend,
    const T* __restrict__ P, const T* __restrict__ Q,
    const float* __restrict__ b1, const float* __restrict__ w2,
    const int* __restrict__ ptr_s, const int* __restrict__ ptr_t,
    float* __restrict__ G_out, T* __restrict__ dP,
    T* __restrict__ dQ, float* __restrict__ dw2_part,
    float* __restrict__ db2_part, float* __restrict__ part, int accumulate,
    int Ns, int Nt, int rows_s, int rows_t) {
  using G = StepGeom<R>;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  DGMC_LDS float* sR = (DGMC_LDS float*)smem_raw;
  DGMC_LDS float* sGt = sR + Ns * G::PP;
  const int region1 =
      max(TRANS ? (Ns + Nt) * G::PP : 0, CONS ? 2 * G::RG * R : 0);
  DGMC_LDS float* sP = sR + region1;
  DGMC_LDS float* sQ = sP + (CONS ? Ns * R : 0);
  DGMC_LDS float* sD = sQ + (CONS ? Nt * R : 0);
  DGMC_LDS float* sRed = sR;                 // after phase 1
  DGMC_LDS float* sSum = sD + Ns * Nt;       // [kWaves]
  const int b = xcd_remap(blockIdx.x, gridDim.x);
  const int tid = threadIdx.x;
  const int wave = tid / kWave, lane = tid % kWave;
  const int s0 = ptr_s[b], ns = ptr_s[b + 1] - s0;
  const int t0 = ptr_t[b], nt = ptr_t[b + 1] - t0;
  const int NN = Ns * Nt;
  const float* Sb = S + (size_t)b * NN;
  constexpr int QMAX = kMaxN / kWaves;
  float sv[TRANS ? QMAX : 1], av[TRANS ? QMAX : 1];
  float pre[kPrefetch];
  if constexpr (TRANS) {
#pragma unroll
    for (int q = 0; q < QMAX; ++q) {
      const int i = wave + q * kWaves;
      const bool in = i < Ns && lane < Nt;
      sv[q] = in ? Sb[i * Nt + lane] : 0.f;
      av[q] = (in && addend) ? addend[(size_t)b * NN + i * Nt + lane] : 0.f;
    }
  } else {
    prefetch_tile(Sb, NN, pre);
  }
  const int cq = tid % G::CQ, rg = tid / G::CQ;
  ps_f32x4 bv = {0.f, 0.f, 0.f, 0.f}, wv = {0.f, 0.f, 0.f, 0.f};
  if constexpr (CONS) {
    bv = *reinterpret_cast<const ps_f32x4*>(b1 + 4 * cq);
    wv = *reinterpret_cast<const ps_f32x4*>(w2 + 4 * cq);
  }
  if constexpr (CONS && TRANS) {
    const StageBlk<T> blk[4] = {{r_s + (size_t)s0 * R, sR, nullptr, ns, G::PP},
                             {g_t + (size_t)t0 * R, sGt, nullptr, nt, G::PP},
                             {P + (size_t)s0 * R, sP, nullptr, ns, R},
                             {Q + (size_t)t0 * R, sQ, nullptr, nt, R}};
    stage_blocks<R, 4>(blk);
  } else if constexpr (TRANS) {
    const StageBlk<T> blk[2] = {{r_s + (size_t)s0 * R, sR, nullptr, ns, G::PP},
                             {g_t + (size_t)t0 * R, sGt, nullptr, nt, G::PP}};
    stage_blocks<R, 2>(blk);
  } else {
    const StageBlk<T> blk[2] = {{P + (size_t)s0 * R, sP, nullptr, ns, R},
                             {Q + (size_t)t0 * R, sQ, nullptr, nt, R}};
    stage_blocks<R, 2>(blk);
  }
  float gsum = 0.f;
  if constexpr (CONS) {
    pad_rows<R, T>(dP, ptr_s[gridDim.x], rows_s, nullptr, nullptr, 0, 0);
    pad_rows<R, T>(dQ, ptr_t[gridDim.x], rows_t, nullptr, nullptr, 0, 0);
  }
  if constexpr (!TRANS) {
    // Upstream gradient tile, masked to the valid block.
#pragma unroll
    for (int u = 0; u < kPrefetch; ++u) {
      const int e = tid + u * kThreads;
      if (e < NN) {
        const int i = e / Nt, j = e - (e / Nt) * Nt;
        const float v = (i < ns && j < nt) ? pre[u] : 0.f;
        sD[e] = v;
        gsum += v;
      }
    }
    for (int e = tid + kPrefetch * kThreads; e < NN; e += kThreads) {
      const int i = e / Nt, j = e - (e / Nt) * Nt;
      const float v = (i < ns && j < nt) ? Sb[e] : 0.f;
      sD[e] = v;
      gsum += v;
    }
  }
  __syncthreads();

  if constexpr (TRANS) {
    // Phase 1: dS[i][j] = <r_s[i], g_t[j]>, 4 lanes per entry.
    const int qd = tid & 3;
    const int pairs = ns * nt;
    for (int p0 = 0; p0 < pairs; p0 += kThreads / 4) {
      const int p = p0 + (tid >> 2);
      const bool valid = p < pairs;
      const int i = valid ? p / nt : 0;
      const int j = valid ? p - i * nt : 0;
      const DGMC_LDS float* rr = sR + i * G::PP + 4 * qd;
      const DGMC_LDS float* gr = sGt + j * G::PP + 4 * qd;
      ps_f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int u = 0; u < G::RU; ++u)
        acc += lds4(rr + 16 * u) * lds4(gr + 16 * u);
      const float s = quad_sum((acc[0] + acc[1]) + (acc[2] + acc[3]));
      if (valid && qd == 0) sD[i * Nt + j] = s;
    }
    __syncthreads();
    // Softmax backward + addend -> G (global) and, for CONS, the masked
    // upstream tile of the consensus backward (LDS, after the barrier).
    float* Gb = G_out + (size_t)b * NN;
#pragma unroll
    for (int q = 0; q < QMAX; ++q) {
      const int i = wave + q * kWaves;
      if (i < Ns) {
        const bool valid = i < ns && lane < nt;
        const float d = valid ? sD[i * Nt + lane] : 0.f;
        const float dot = wave_sum_dpp(sv[q] * d);
        const float gv = sv[q] * (d - dot) + av[q];
        if (lane < Nt) Gb[i * Nt + lane] = gv;
        const float gm = valid ? gv : 0.f;
        gsum += gm;
        sv[q] = gm;
      }
    }
    if constexpr (!CONS) return;
    __syncthreads();
#pragma unroll
    for (int q = 0; q < QMAX; ++q) {
      const int i = wave + q * kWaves;
      if (i < Ns && lane < Nt) sD[i * Nt + lane] = sv[q];
    }
  }
  gsum = wave_sum_dpp(gsum);
  if (lane == 0) sSum[wave] = gsum;
  __syncthreads();
  // Parameter-gradient partials of this pair: into [db1 | dw2 | db2] row b
  // of ``part`` (accumulated over the loop's uses in backward order: one
  // column sum at the end instead of per-use lists), else dw2 / db2 rows.
  float* pb = part ? part + (size_t)b * (2 * R + 1) : nullptr;
  if (tid == 0) {
    float t = 0.f;
    for (int w = 0; w < kWaves; ++w) t += sSum[w];
    if (pb)
      pb[2 * R] = (accumulate ? pb[2 * R] : 0.f) + t;
    else
      db2_part[b] = t;
  }

  // Phase 2: dP / dQ rows (one channel quad per lane), dw2 / db1 partials.
  ps_f32x4 dw = {0.f, 0.f, 0.f, 0.f}, db1v = {0.f, 0.f, 0.f, 0.f};
  for (int r = rg; r < ns + nt; r += G::RG) {
    ps_f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    if (r < ns) {
      const int i = r;
      const ps_f32x4 pv = lds4(sP + i * R + 4 * cq) + bv;
      for (int j = 0; j < nt; ++j) {
        const ps_f32x4 qv = lds4(sQ + j * R + 4 * cq);
        const float g = sD[i * Nt + j];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float z = fmaxf(pv[k] - qv[k], 0.f);
          acc[k] += z > 0.f ? g : 0.f;
          dw[k] = fmaf(g, z, dw[k]);
        }
      }
      acc *= wv;
      db1v += acc;
      StepIO<T>::store4(dP + ((size_t)s0 + i) * R + 4 * cq, acc);
    } else {
      const int j = r - ns;
      const ps_f32x4 qv = lds4(sQ + j * R + 4 * cq);
      for (int i = 0; i < ns; ++i) {
        const ps_f32x4 pv = lds4(sP + i * R + 4 * cq) + bv;
        const float g = sD[i * Nt + j];
#pragma unroll
        for (int k = 0; k < 4; ++k) acc[k] += pv[k] - qv[k] > 0.f ? g : 0.f;
      }
      acc *= -wv;
      StepIO<T>::store4(dQ + ((size_t)t0 + j) * R + 4 * cq, acc);
    }
  }
  *reinterpret_cast<DGMC_LDS ps_f32x4*>(sRed + rg * R + 4 * cq) = dw;
  *reinterpret_cast<DGMC_LDS ps_f32x4*>(sRed + (G::RG + rg) * R + 4 * cq) =
      db1v;
  __syncthreads();
  for (int c = tid; c < R; c += kThreads) {
    float s = 0.f, s1 = 0.f;
    for (int r = 0; r < G::RG; ++r) {
      s += sRed[r * R + c];
      s1 += sRed[(G::RG + r) * R + c];
    }
    if (pb) {
      pb[c] = (accumulate ? pb[c] : 0.f) + s1;
      pb[R + c] = (accumulate ? pb[R + c] : 0.f) + s;
    } else {
      dw2_part[(size_t)b * R + c] = s;
    }
  }
}

// LDS floats of the step kernels.
template <int R>
static size_t step_fwd_lds(bool cons, bool trans, int Ns, int Nt) {
  using G = StepGeom<R>;
  return (cons ? (size_t)(Ns + Nt) * G::PP : 0) +
         (trans ? (size_t)Ns * R : 0) + (size_t)Ns * Nt;
}
template <int R>
static size_t step_bwd_lds(bool cons, bool trans, int Ns, int Nt) {
  using G = StepGeom<R>;
  return (size_t)std::max(trans ? (Ns + Nt) * G::PP : 0,
                          cons ? 2 * G::RG * R : 0) +
         (cons ? (size_t)(Ns + Nt) * R : 0) + (size_t)Ns * Nt + kWaves;
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

// 16-byte vector loads possible for every pair's row block of t.
static bool rows_vec_ok(const at::Tensor& t) {
  return aligned16(t.data_ptr()) && (t.size(1) * t.element_size()) % 16 == 0;
}

// Dynamic LDS of a pair kernel; raises the per-kernel limit when needed.
template <typename K>
static size_t pair_lds(K kern, size_t floats) {
  const size_t bytes = floats * sizeof(float);
  TORCH_CHECK(bytes <= 160 * 1024, "pair tile exceeds the 160 KiB LDS (",
              bytes, " bytes)");
  if (bytes > 64 * 1024)
    DGMC_CHECK_HIP(hipFuncSetAttribute(
        reinterpret_cast<const void*>(kern),
        hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
  return bytes;
}

// Compile-time-width step kernels (pair_step_fwd/bwd_kernel): R in
// {32, 64, 128}, 16-byte aligned operand rows of ONE storage type (bf16 under
// autocast, fp32 at reference precision), aligned fp32 b1 / w2.
// Other widths / alignments use the generic kernels.
static bool fast_step_ok(int R, std::initializer_list<const at::Tensor*> rows,
                         std::initializer_list<const void*> vecs = {}) {
  if (!(R == 32 || R == 64 || R == 128)) return false;
  const at::ScalarType st = (*rows.begin())->scalar_type();
  if (st != at::kBFloat16 && st != at::kFloat) return false;
  for (const at::Tensor* t : rows)
    if (t->scalar_type() != st || !rows_vec_ok(*t)) return false;
  for (const void* v : vecs)
    if (!aligned16(v)) return false;
  return true;
}

static void* vp(const at::Tensor& t) { return t.data_ptr(); }

struct StepFwdArgs {
  const float* S_hat;
  const void *P, *Q;
  const float *b1, *w2, *b2;
  const void* r_s;
  const int *ptr_s, *ptr_t;
  float *S_new, *S_prob;
  void *rs_copy, *rt_out;
  int B, Ns, Nt, rows_s, rows_t;
  bool f32 = false;            // node-level storage fp32 (else bf16)
  __bf16* planes = nullptr;    // joint's bf16x6 planes (fp32, with rs_copy)
};

struct StepBwdArgs {
  const float* S;
  const void *r_s, *g_t;
  const float* addend;
  const void *P, *Q;
  const float *b1, *w2;
  const int *ptr_s, *ptr_t;
  float* G_out;
  void *dP, *dQ;
  float *dw2_part, *db2_part;
  int B, Ns, Nt, rows_s, rows_t;
  float* part = nullptr;       // [B, 2R + 1] loop-accumulated partials
  int accumulate = 0;
  bool f32 = false;
};

template <int R, bool C, bool T, typename E>
static void step_fwd_launch(const StepFwdArgs& a) {
  auto kern = pair_step_fwd_kernel<R, C, T, E>;
  const size_t lds = pair_lds(kern, step_fwd_lds<R>(C, T, a.Ns, a.Nt));
  hipLaunchKernelGGL(kern, dim3(a.B), dim3(kThreads), lds, stream(), a.S_hat,
                     (const E*)a.P, (const E*)a.Q, a.b1, a.w2, a.b2,
                     (const E*)a.r_s, a.ptr_s, a.ptr_t, a.S_new, a.S_prob,
                     (E*)a.rs_copy, (E*)a.rt_out,
                     std::is_same<E, float>::value ? a.planes : nullptr, a.Ns,
                     a.Nt, a.rows_s, a.rows_t);
  DGMC_CHECK_LAUNCH();
}

template <int R, bool C, bool T, typename E>
static void step_bwd_launch(const StepBwdArgs& a) {
  auto kern = pair_step_bwd_kernel<R, C, T, E>;
  const size_t lds = pair_lds(kern, step_bwd_lds<R>(C, T, a.Ns, a.Nt));
  hipLaunchKernelGGL(kern, dim3(a.B), dim3(kThreads), lds, stream(), a.S,
                     (const E*)a.r_s, (const E*)a.g_t, a.addend,
                     (const E*)a.P, (const E*)a.Q, a.b1, a.w2, a.ptr_s,
                     a.ptr_t, a.G_out, (E*)a.dP, (E*)a.dQ, a.dw2_part,
                     a.db2_part, a.part, a.accumulate, a.Ns, a.Nt, a.rows_s,
                     a.rows_t);
  DGMC_CHECK_LAUNCH();
}

template <bool C, bool T, typename E>
static void step_fwd_t(int R, const StepFwdArgs& a) {
  if (R == 32) step_fwd_launch<32, C, T, E>(a);
  else if (R == 64) step_fwd_launch<64, C, T, E>(a);
  else step_fwd_launch<128, C, T, E>(a);
}

template <bool C, bool T>
static void step_fwd(int R, const StepFwdArgs& a) {
  if (a.f32) step_fwd_t<C, T, float>(R, a);
  else step_fwd_t<C, T, __bf16>(R, a);
}

template <bool C, bool T, typename E>
static void step_bwd_t(int R, const StepBwdArgs& a) {
  if (R == 32) step_bwd_launch<32, C, T, E>(a);
  else if (R == 64) step_bwd_launch<64, C, T, E>(a);
  else step_bwd_launch<128, C, T, E>(a);
}

template <bool C, bool T>
static void step_bwd(int R, const StepBwdArgs& a) {
  if (a.f32) step_bwd_t<C, T, float>(R, a);
  else step_bwd_t<C, T, __bf16>(R, a);
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

at::Tensor split3(const at::Tensor& x);   // slot_gemm_x6.hip

// Optional bf16x6 planes output of the joint [r_s; r_t] ([3, rows, R] bf16,
// fp32 joint only); nullptr when absent.
static __bf16* joint_planes(const c10::optional<at::Tensor>& planes,
                            const at::Tensor& joint) {
  if (!planes.has_value() || !planes->defined()) return nullptr;
  const at::Tensor& p = *planes;
  TORCH_CHECK(joint.scalar_type() == at::kFloat &&
                  p.scalar_type() == at::kBFloat16 && p.is_contiguous() &&
                  p.dim() == 3 && p.size(0) == 3 &&
                  p.size(1) == joint.size(0) && p.size(2) == joint.size(1) &&
                  aligned16(p.data_ptr()) && p.device() == joint.device(),
              "joint planes: bf16 [3, rows_s + rows_t, R] of an fp32 joint");
  return reinterpret_cast<__bf16*>(p.data_ptr());
}

// (planes filled from the finished joint: the paths without the step kernel)
static void joint_planes_fill(const c10::optional<at::Tensor>& planes,
                              const at::Tensor& joint) {
  if (joint_planes(planes, joint) != nullptr && joint.numel() > 0)
    planes->copy_(split3(joint));
}

// r_s: packed [sum N_s, R]; returns (S [B, Ns, Nt], r_t packed [rows_t, R]).
// `planes` (with joint_out, fp32): also written with the joint's bf16x6
// operand planes (psi_2's first slot GEMM reads them; no split pass).
std::tuple<at::Tensor, at::Tensor> dense_softmax_transport(
    const at::Tensor& S_hat, const at::Tensor& r_s, const at::Tensor& ptr_s,
    const at::Tensor& ptr_t, int64_t rows_t, bool joint_out,
    const c10::optional<at::Tensor>& planes) {
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
  TORCH_CHECK(joint_out || !planes.has_value() || !planes->defined(),
              "dense_softmax_transport: planes need joint_out");
  if (B == 0) {
    if (joint_out) {
      joint.narrow(0, 0, rows_s).copy_(r_s);
      joint_planes_fill(planes, joint);
    }
    return {S, joint_out ? joint : r_t};
  }
  if (fast_step_ok(R, {&r_s})) {
    StepFwdArgs a{S_hat.data_ptr<float>(), nullptr, nullptr, nullptr,
                  nullptr, nullptr, vp(r_s), ptr_s.data_ptr<int>(),
                  ptr_t.data_ptr<int>(), nullptr, S.data_ptr<float>(),
                  joint_out ? vp(joint) : nullptr, vp(r_t), B, Ns,
                  Nt, (int)rows_s, (int)rows_t};
    a.f32 = r_s.scalar_type() == at::kFloat;
    if (joint_out) a.planes = joint_planes(planes, joint);
    step_fwd<false, true>(R, a);
    return {S, joint_out ? joint : r_t};
  }
  const int vec = rows_vec_ok(r_s) ? 1 : 0;
  DGMC_DISPATCH_FLOAT(r_s.scalar_type(), T, [&] {
    auto kern = softmax_transport_kernel<T>;
    const size_t lds = pair_lds(kern, (size_t)Ns * R + (size_t)Ns * Nt);
    hipLaunchKernelGGL(kern, dim3(B), dim3(kThreads), lds, stream(),
                       S_hat.data_ptr<float>(),
                       reinterpret_cast<const T*>(r_s.data_ptr()),
                       ptr_s.data_ptr<int>(), ptr_t.data_ptr<int>(),
                       S.data_ptr<float>(), reinterpret_cast<T*>(r_t.data_ptr()),
                       Ns, Nt, R, (int)rows_t,
                       joint_out ? reinterpret_cast<T*>(joint.data_ptr())
                                 : nullptr,
                       (int)rows_s, vec);
  });
  DGMC_CHECK_LAUNCH();
  if (joint_out) joint_planes_fill(planes, joint);
  return {S, joint_out ? joint : r_t};
}

at::Tensor dense_softmax_transport_bwd(const at::Tensor& S,
                                       const at::Tensor& r_s,
                                       const at::Tensor& g,
                                       const at::Tensor& ptr_s,
                                       const at::Tensor& ptr_t,
                                       const c10::optional<at::Tensor>& addend) {
  check_pair_tensor(S, "S");
  check_packed(r_s, "r_s");
  check_packed(g, "grad r_t");
  const float* add = nullptr;
  if (addend.has_value() && addend->defined()) {
    TORCH_CHECK(addend->scalar_type() == at::kFloat &&
                    addend->is_contiguous() && addend->sizes() == S.sizes() &&
                    addend->device() == S.device(),
                "dense_softmax_transport_bwd: addend fp32 like S");
    add = addend->data_ptr<float>();
  }
  TORCH_CHECK(r_s.scalar_type() == g.scalar_type(), "r_s/grad dtype");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(S.device());
  const int B = S.size(0), Ns = S.size(1), Nt = S.size(2);
  const int R = r_s.size(1);
  TORCH_CHECK(Ns <= kMaxN && Nt <= kMaxN, "pair tile too large");
  TORCH_CHECK(g.size(1) == R, "grad shape");
  check_ptr(ptr_s, ptr_t, B);
  at::Tensor out = at::empty_like(S);
  if (B == 0) return out;
  if (fast_step_ok(R, {&r_s, &g})) {
    StepBwdArgs a{S.data_ptr<float>(), vp(r_s), vp(g), add,
                  nullptr, nullptr, nullptr, nullptr, ptr_s.data_ptr<int>(),
                  ptr_t.data_ptr<int>(), out.data_ptr<float>(), nullptr,
                  nullptr, nullptr, nullptr, B, Ns, Nt, (int)r_s.size(0),
                  (int)g.size(0)};
    a.f32 = r_s.scalar_type() == at::kFloat;
    step_bwd<false, true>(R, a);
    return out;
  }
  const int vec = (rows_vec_ok(r_s) && rows_vec_ok(g)) ? 1 : 0;
  DGMC_DISPATCH_FLOAT(r_s.scalar_type(), T, [&] {
    auto kern = softmax_transport_bwd_kernel<T>;
    const size_t lds = pair_lds(
        kern, (size_t)(Ns + Nt) * (R + 1) + (size_t)Ns * Nt);
    hipLaunchKernelGGL(kern, dim3(B), dim3(kThreads), lds, stream(),
                       S.data_ptr<float>(),
                       reinterpret_cast<const T*>(r_s.data_ptr()),
                       reinterpret_cast<const T*>(g.data_ptr()),
                       ptr_s.data_ptr<int>(), ptr_t.data_ptr<int>(),
                       out.data_ptr<float>(), add, Ns, Nt, R, vec);
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
  if (fast_step_ok(R, {&P, &Q}, {b1.data_ptr(), w2.data_ptr()}) &&
      b1.is_contiguous() && w2.is_contiguous()) {
    StepFwdArgs a{S_hat.data_ptr<float>(), vp(P), vp(Q),
                  b1.data_ptr<float>(), w2.data_ptr<float>(),
                  b2.data_ptr<float>(), nullptr, ptr_s.data_ptr<int>(),
                  ptr_t.data_ptr<int>(), out.data_ptr<float>(), nullptr,
                  nullptr, nullptr, B, Ns, Nt, (int)P.size(0),
                  (int)Q.size(0)};
    a.f32 = P.scalar_type() == at::kFloat;
    step_fwd<true, false>(R, a);
    return out;
  }
  const int vec = (rows_vec_ok(P) && rows_vec_ok(Q)) ? 1 : 0;
  DGMC_DISPATCH_FLOAT(P.scalar_type(), T, [&] {
    auto kern = consensus_fwd_kernel<T>;
    const size_t lds =
        pair_lds(kern, (size_t)(Ns + Nt) * (R + 1) + 2 * (size_t)R);
    hipLaunchKernelGGL(kern, dim3(B), dim3(kThreads), lds, stream(),
                       S_hat.data_ptr<float>(),
                       reinterpret_cast<const T*>(P.data_ptr()),
                       reinterpret_cast<const T*>(Q.data_ptr()),
                       b1.data_ptr<float>(), w2.data_ptr<float>(),
                       b2.data_ptr<float>(), ptr_s.data_ptr<int>(),
                       ptr_t.data_ptr<int>(), out.data_ptr<float>(), Ns, Nt,
                       R, vec);
  });
  DGMC_CHECK_LAUNCH();
  return out;
}

// part (optional, fp32 [B, 2R + 1]): the fast kernels write the per-pair
// [db1 | dw2 | db2] partials there (added to the existing rows when
// ``accumulate``) and return undefined dw2 / db2.
static float* step_part(const c10::optional<at::Tensor>& part, int B, int R,
                        const at::Tensor& like) {
  if (!part.has_value() || !part->defined()) return nullptr;
  TORCH_CHECK(part->scalar_type() == at::kFloat && part->is_contiguous() &&
                  part->dim() == 2 && part->size(0) == B &&
                  part->size(1) == 2 * R + 1 &&
                  part->device() == like.device(),
              "pair step: part must be fp32 [B, 2R + 1]");
  return part->data_ptr<float>();
}

// Generic-kernel fallback of the ``part`` contract (only its column sums
// matter: the P-row sum of dP goes into row 0).
static void fold_part_generic(at::Tensor part, bool accumulate,
                              const at::Tensor& dP, const at::Tensor& dw2,
                              const at::Tensor& db2, int R) {
  if (!accumulate) part.zero_();
  part.select(0, 0).narrow(0, 0, R).add_(dP.to(at::kFloat).sum(0));
  part.narrow(1, R, R).add_(dw2);
  part.narrow(1, 2 * R, 1).add_(db2.view({-1, 1}));
}

std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> dense_consensus_bwd(
    const at::Tensor& G, const at::Tensor& P, const at::Tensor& Q,
    const at::Tensor& b1, const at::Tensor& w2, const at::Tensor& ptr_s,
    const at::Tensor& ptr_t, const c10::optional<at::Tensor>& dpq_out,
    const c10::optional<at::Tensor>& part, bool accumulate) {
  check_pair_tensor(G, "grad");
  check_packed(P, "P");
  check_packed(Q, "Q");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(G.device());
  const int B = G.size(0), Ns = G.size(1), Nt = G.size(2);
  const int R = P.size(1);
  TORCH_CHECK(Ns <= kMaxN && Nt <= kMaxN, "pair tile too large");
  TORCH_CHECK(b1.numel() == R && w2.numel() == R, "b1/w2 size");
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
  if (fast_step_ok(R, {&P, &Q, &dP, &dQ}, {b1.data_ptr(), w2.data_ptr()}) &&
      b1.is_contiguous() && w2.is_contiguous()) {
    StepBwdArgs a{G.data_ptr<float>(), nullptr, nullptr, nullptr,
                  vp(P), vp(Q), b1.data_ptr<float>(),
                  w2.data_ptr<float>(), ptr_s.data_ptr<int>(),
                  ptr_t.data_ptr<int>(), nullptr, vp(dP), vp(dQ),
                  dw2.data_ptr<float>(), db2.data_ptr<float>(), B, Ns, Nt,
                  (int)P.size(0), (int)Q.size(0)};
    a.part = step_part(part, B, R, G);
    a.accumulate = accumulate ? 1 : 0;
    a.f32 = P.scalar_type() == at::kFloat;
    step_bwd<true, false>(R, a);
    if (a.part) return {dP, dQ, at::Tensor(), at::Tensor()};
    return {dP, dQ, dw2, db2};
  }
  const int vec = (rows_vec_ok(P) && rows_vec_ok(Q)) ? 1 : 0;
  DGMC_DISPATCH_FLOAT(P.scalar_type(), T, [&] {
    auto kern = consensus_bwd_kernel<T>;
    const size_t lds = pair_lds(kern, (size_t)(Ns + Nt) * R +
                                          (size_t)Ns * Nt + 2 * (size_t)R +
                                          kThreads);
    hipLaunchKernelGGL(kern, dim3(B), dim3(kThreads), lds, stream(),
                       G.data_ptr<float>(),
                       reinterpret_cast<const T*>(P.data_ptr()),
                       reinterpret_cast<const T*>(Q.data_ptr()),
                       b1.data_ptr<float>(), w2.data_ptr<float>(),
                       ptr_s.data_ptr<int>(), ptr_t.data_ptr<int>(),
                       reinterpret_cast<T*>(dP.data_ptr()),
                       reinterpret_cast<T*>(dQ.data_ptr()),
                       dw2.data_ptr<float>(), db2.data_ptr<float>(), Ns, Nt, R,
                       (int)P.size(0), (int)Q.size(0), vec);
  });
  DGMC_CHECK_LAUNCH();
  if (step_part(part, B, R, G)) {
    fold_part_generic(*part, accumulate, dP, dw2, db2, R);
    return {dP, dQ, at::Tensor(), at::Tensor()};
  }
  return {dP, dQ, dw2, db2};
}

// Fused consensus update (step l) + softmax transport (step l + 1):
// returns (S_hat', S = masked_softmax(S_hat'), joint [r_s; S^T r_s]).
std::tuple<at::Tensor, at::Tensor, at::Tensor> dense_consensus_transport(
    const at::Tensor& S_hat, const at::Tensor& P, const at::Tensor& Q,
    const at::Tensor& b1, const at::Tensor& w2, const at::Tensor& b2,
    const at::Tensor& r_s, const at::Tensor& ptr_s, const at::Tensor& ptr_t,
    int64_t rows_t, const c10::optional<at::Tensor>& planes) {
  check_pair_tensor(S_hat, "S_hat");
  check_packed(P, "P");
  check_packed(Q, "Q");
  check_packed(r_s, "r_s");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(S_hat.device());
  const int B = S_hat.size(0), Ns = S_hat.size(1), Nt = S_hat.size(2);
  const int R = P.size(1);
  TORCH_CHECK(Ns <= kMaxN && Nt <= kMaxN, "pair tile too large");
  TORCH_CHECK(Q.size(1) == R && Q.scalar_type() == P.scalar_type() &&
                  r_s.size(1) == R,
              "dense_consensus_transport: P / Q / r_s widths");
  TORCH_CHECK(b1.numel() == R && w2.numel() == R && b2.numel() == 1 &&
                  b1.scalar_type() == at::kFloat &&
                  w2.scalar_type() == at::kFloat &&
                  b2.scalar_type() == at::kFloat,
              "b1/w2/b2 must be fp32");
  check_ptr(ptr_s, ptr_t, B);
  const int64_t rows_s = r_s.size(0);
  at::Tensor S_new = at::empty_like(S_hat);
  at::Tensor S_prob = at::empty_like(S_hat);
  at::Tensor joint = at::empty({rows_s + rows_t, R}, r_s.options());
  if (B == 0) {
    joint.narrow(0, 0, rows_s).copy_(r_s);
    joint.narrow(0, rows_s, rows_t).zero_();
    joint_planes_fill(planes, joint);
    return {S_new, S_prob, joint};
  }
  const int vec_pq = (rows_vec_ok(P) && rows_vec_ok(Q)) ? 1 : 0;
  const int vec_r = rows_vec_ok(r_s) ? 1 : 0;
  TORCH_CHECK(P.scalar_type() == r_s.scalar_type() &&
                  (P.scalar_type() == at::kBFloat16 ||
                   P.scalar_type() == at::kFloat),
              "dense_consensus_transport: P/Q and r_s both bf16 or fp32");
  if (fast_step_ok(R, {&P, &Q, &r_s}, {b1.data_ptr(), w2.data_ptr()})) {
    StepFwdArgs a{S_hat.data_ptr<float>(), vp(P), vp(Q),
                  b1.data_ptr<float>(), w2.data_ptr<float>(),
                  b2.data_ptr<float>(), vp(r_s), ptr_s.data_ptr<int>(),
                  ptr_t.data_ptr<int>(), S_new.data_ptr<float>(),
                  S_prob.data_ptr<float>(), vp(joint),
                  vp(joint.narrow(0, rows_s, rows_t)), B, Ns, Nt, (int)rows_s,
                  (int)rows_t};
    a.f32 = P.scalar_type() == at::kFloat;
    a.planes = joint_planes(planes, joint);
    step_fwd<true, true>(R, a);
    return {S_new, S_prob, joint};
  }
  DGMC_DISPATCH_FLOAT(P.scalar_type(), T, [&] {
  auto kern = consensus_transport_kernel<T, T>;
  const size_t lds = pair_lds(kern, (size_t)(Ns + Nt) * (R + 1) +
                                        2 * (size_t)R + (size_t)Ns * R +
                                        (size_t)Ns * Nt);
  hipLaunchKernelGGL(kern, dim3(B), dim3(kThreads), lds, stream(),
                     S_hat.data_ptr<float>(),
                     reinterpret_cast<const T*>(P.data_ptr()),
                     reinterpret_cast<const T*>(Q.data_ptr()),
                     b1.data_ptr<float>(), w2.data_ptr<float>(),
                     b2.data_ptr<float>(),
                     reinterpret_cast<const T*>(r_s.data_ptr()),
                     ptr_s.data_ptr<int>(), ptr_t.data_ptr<int>(),
                     S_new.data_ptr<float>(), S_prob.data_ptr<float>(),
                     reinterpret_cast<T*>(joint.data_ptr()), Ns, Nt, R,
                     (int)rows_s, (int)rows_t, vec_pq, vec_r);
  });
  DGMC_CHECK_LAUNCH();
  joint_planes_fill(planes, joint);
  return {S_new, S_prob, joint};
}

// Backward of dense_consensus_transport: returns (G = total gradient of
// S_hat' (also the gradient of S_hat through the identity path), dP, dQ,
// dw2 [B, R] / db2 [B] per-pair partials); dP / dQ live in dpq_out when
// given ([rows_s + rows_t, R]).
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor>
dense_transport_consensus_bwd(const at::Tensor& S_prob, const at::Tensor& r_s,
                              const at::Tensor& g_t,
                              const c10::optional<at::Tensor>& addend,
                              const at::Tensor& P, const at::Tensor& Q,
                              const at::Tensor& b1, const at::Tensor& w2,
                              const at::Tensor& ptr_s, const at::Tensor& ptr_t,
                              const c10::optional<at::Tensor>& dpq_out,
                              const c10::optional<at::Tensor>& part,
                              bool accumulate) {
  check_pair_tensor(S_prob, "S");
  check_packed(r_s, "r_s");
  check_packed(g_t, "grad r_t");
  check_packed(P, "P");
  check_packed(Q, "Q");
  const float* add = nullptr;
  if (addend.has_value() && addend->defined()) {
    TORCH_CHECK(addend->scalar_type() == at::kFloat &&
                    addend->is_contiguous() &&
                    addend->sizes() == S_prob.sizes(),
                "dense_transport_consensus_bwd: addend fp32 like S");
    add = addend->data_ptr<float>();
  }
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(S_prob.device());
  const int B = S_prob.size(0), Ns = S_prob.size(1), Nt = S_prob.size(2);
  const int R = P.size(1);
  TORCH_CHECK(Ns <= kMaxN && Nt <= kMaxN, "pair tile too large");
  TORCH_CHECK(r_s.size(1) == R && g_t.size(1) == R && Q.size(1) == R &&
                  (r_s.scalar_type() == at::kBFloat16 ||
                   r_s.scalar_type() == at::kFloat) &&
                  g_t.scalar_type() == r_s.scalar_type() &&
                  P.scalar_type() == r_s.scalar_type() &&
                  Q.scalar_type() == r_s.scalar_type(),
              "dense_transport_consensus_bwd: r_s / g_t / P / Q of width R, "
              "all bf16 or all fp32");
  TORCH_CHECK(b1.numel() == R && w2.numel() == R, "b1/w2 size");
  check_ptr(ptr_s, ptr_t, B);
  at::Tensor dP, dQ;
  if (dpq_out.has_value() && dpq_out->defined()) {
    const at::Tensor& d = *dpq_out;
    TORCH_CHECK(d.is_contiguous() && d.scalar_type() == P.scalar_type() &&
                    d.size(0) == P.size(0) + Q.size(0) && d.size(1) == R,
                "dense_transport_consensus_bwd: dpq_out [rows_s + rows_t, R]");
    dP = d.narrow(0, 0, P.size(0));
    dQ = d.narrow(0, P.size(0), Q.size(0));
  } else {
    dP = at::empty_like(P);
    dQ = at::empty_like(Q);
  }
  at::Tensor G = at::empty_like(S_prob);
  at::Tensor dw2 = at::empty({B, R}, S_prob.options());
  at::Tensor db2 = at::empty({B}, S_prob.options());
  if (B == 0) return {G, dP, dQ, dw2.zero_(), db2.zero_()};
  const int vec_r = (rows_vec_ok(r_s) && rows_vec_ok(g_t)) ? 1 : 0;
  const int vec_pq = (rows_vec_ok(P) && rows_vec_ok(Q)) ? 1 : 0;
  if (fast_step_ok(R, {&r_s, &g_t, &P, &Q, &dP, &dQ},
                   {b1.data_ptr(), w2.data_ptr()})) {
    StepBwdArgs a{S_prob.data_ptr<float>(), vp(r_s), vp(g_t), add,
                  vp(P), vp(Q), b1.data_ptr<float>(),
                  w2.data_ptr<float>(), ptr_s.data_ptr<int>(),
                  ptr_t.data_ptr<int>(), G.data_ptr<float>(), vp(dP),
                  vp(dQ), dw2.data_ptr<float>(), db2.data_ptr<float>(),
                  B, Ns, Nt, (int)P.size(0), (int)Q.size(0)};
    a.part = step_part(part, B, R, S_prob);
    a.accumulate = accumulate ? 1 : 0;
    a.f32 = P.scalar_type() == at::kFloat;
    step_bwd<true, true>(R, a);
    if (a.part) return {G, dP, dQ, at::Tensor(), at::Tensor()};
    return {G, dP, dQ, dw2, db2};
  }
  DGMC_DISPATCH_FLOAT(P.scalar_type(), T, [&] {
  auto kern = transport_consensus_bwd_kernel<T, T>;
  const size_t lds = pair_lds(kern, (size_t)(Ns + Nt) * (R + 1) +
                                        (size_t)(Ns + Nt) * R +
                                        (size_t)Ns * Nt + 2 * (size_t)R +
                                        kThreads);
  hipLaunchKernelGGL(kern, dim3(B), dim3(kThreads), lds, stream(),
                     S_prob.data_ptr<float>(),
                     reinterpret_cast<const T*>(r_s.data_ptr()),
                     reinterpret_cast<const T*>(g_t.data_ptr()), add,
                     reinterpret_cast<const T*>(P.data_ptr()),
                     reinterpret_cast<const T*>(Q.data_ptr()),
                     b1.data_ptr<float>(), w2.data_ptr<float>(),
                     ptr_s.data_ptr<int>(), ptr_t.data_ptr<int>(),
                     G.data_ptr<float>(), reinterpret_cast<T*>(dP.data_ptr()),
                     reinterpret_cast<T*>(dQ.data_ptr()),
                     dw2.data_ptr<float>(), db2.data_ptr<float>(), Ns, Nt, R,
                     (int)P.size(0), (int)Q.size(0), vec_r, vec_pq);
  });
  DGMC_CHECK_LAUNCH();
  if (step_part(part, B, R, S_prob)) {
    fold_part_generic(*part, accumulate, dP, dw2, db2, R);
    return {G, dP, dQ, at::Tensor(), at::Tensor()};
  }
  return {G, dP, dQ, dw2, db2};
}

}  // namespace dgmc
