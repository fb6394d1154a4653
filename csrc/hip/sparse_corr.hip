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
    float* __restrict__ dw2_part, int rows, int R, int ldp) {
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
    dw2_part[(size_t)blk * ldp + c] = s;
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
// Lane-group variants (channel count C a multiple of 4, C <= 256): a
// candidate is owned by G = pow2ceil(C / 4) lanes holding one float4 each, so
// a wave walks 64 / G candidates at once (R = 32: 8 candidates per step, the
// 20 candidates of a DBP15K row in one batch of loads) and a dot needs
// log2(G) xor steps instead of a whole-wave reduction per candidate.
// Summation order is fixed: results are reproducible run to run.
// ---------------------------------------------------------------------------
__device__ __forceinline__ float4 ld4(const float* __restrict__ p) {
  return *reinterpret_cast<const float4*>(p);
}

template <int G>
__device__ __forceinline__ float group_sum(float s) {
#pragma unroll
  for (int off = 1; off < G; off <<= 1) s += __shfl_xor(s, off);
  return s;
}

template <int G>
__global__ __launch_bounds__(256) void sddmm_g_kernel(
    const int* __restrict__ rowptr, const int* __restrict__ col,
    const float* __restrict__ A, const float* __restrict__ Bm,
    float* __restrict__ val, int rows, int C) {
  constexpr int NG = kWave / G;
  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  const int r = xcd_remap(blockIdx.x, gridDim.x) * kSpWaves + wave;
  if (r >= rows) return;
  const int g = lane / G, c = (lane % G) * 4;
  const bool cok = c < C;
  const float4 a = cok ? ld4(A + (size_t)r * C + c) : make_float4(0, 0, 0, 0);
  const int p0 = rowptr[r], p1 = rowptr[r + 1];
  for (int pb = p0; pb < p1; pb += 2 * NG) {
    float s[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int p = pb + u * NG + g;
      s[u] = 0.f;
      if (p < p1 && cok) {
        const float4 b = ld4(Bm + (size_t)col[p] * C + c);
        s[u] = fmaf(a.x, b.x, fmaf(a.y, b.y, fmaf(a.z, b.z, a.w * b.w)));
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const float t = group_sum<G>(s[u]);
      const int p = pb + u * NG + g;
      if ((lane % G) == 0 && p < p1) val[p] = t;
    }
  }
}

__device__ __forceinline__ float relu_dot4(float4 pv, float4 q, float4 w) {
  return fmaf(fmaxf(pv.x - q.x, 0.f), w.x,
              fmaf(fmaxf(pv.y - q.y, 0.f), w.y,
                   fmaf(fmaxf(pv.z - q.z, 0.f), w.z,
                        fmaxf(pv.w - q.w, 0.f) * w.w)));
}

// SOFT: also the row softmax of the updated scores, prob = softmax(out)
// over the row's candidates (the next step's S, reference dgmc.py:205,225),
// from registers: a row of k <= 8 * (64 / G) candidates is one wave.
template <int G, bool SOFT>
__global__ __launch_bounds__(256) void sparse_consensus_fwd_g_kernel(
    const int* __restrict__ rowptr, const int* __restrict__ col,
    const float* __restrict__ S_hat, const float* __restrict__ P,
    const float* __restrict__ Q, const float* __restrict__ b1,
    const float* __restrict__ w2, const float* __restrict__ b2,
    float* __restrict__ out, float* __restrict__ prob, int rows, int R) {
  constexpr int NG = kWave / G;
  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  const int r = xcd_remap(blockIdx.x, gridDim.x) * kSpWaves + wave;
  if (r >= rows) return;
  const int g = lane / G, c = (lane % G) * 4;
  const bool cok = c < R;
  float4 pv = make_float4(0, 0, 0, 0), wv = pv;
  if (cok) {
    const float4 p = ld4(P + (size_t)r * R + c), bb = ld4(b1 + c);
    pv = make_float4(p.x + bb.x, p.y + bb.y, p.z + bb.z, p.w + bb.w);
    wv = ld4(w2 + c);
  }
  const float bias = b2[0];
  const int p0 = rowptr[r], p1 = rowptr[r + 1];
  if constexpr (SOFT) {
    // the row's <= 8 * NG candidates in four unrolled batch pairs; every
    // lane of a group keeps its group's values for the softmax
    float vals[8];
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int pb = p0 + it * 2 * NG;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int p = pb + u * NG + g;
        float sv = 0.f;
        if (p < p1 && cok)
          sv = relu_dot4(pv, ld4(Q + (size_t)col[p] * R + c), wv);
        const float t = group_sum<G>(sv);
        const float o = p < p1 ? S_hat[p] + t + bias : -INFINITY;
        vals[2 * it + u] = o;
        if ((lane % G) == 0 && p < p1) out[p] = o;
      }
    }
    float m = -INFINITY;
#pragma unroll
    for (int j = 0; j < 8; ++j) m = fmaxf(m, vals[j]);
#pragma unroll
    for (int off = G; off < kWave; off <<= 1) m = fmaxf(m, __shfl_xor(m, off));
    float e[8], sum = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      e[j] = vals[j] == -INFINITY ? 0.f : __expf(vals[j] - m);
      sum += e[j];
    }
#pragma unroll
    for (int off = G; off < kWave; off <<= 1) sum += __shfl_xor(sum, off);
    const float inv = 1.f / sum;
    if ((lane % G) == 0) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int p = p0 + (j >> 1) * 2 * NG + (j & 1) * NG + g;
        if (p < p1) prob[p] = e[j] * inv;
      }
    }
    return;
  }
  for (int pb = p0; pb < p1; pb += 2 * NG) {
    float s2[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int p = pb + u * NG + g;
      s2[u] = 0.f;
      if (p < p1 && cok) s2[u] = relu_dot4(pv, ld4(Q + (size_t)col[p] * R + c), wv);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const float t = group_sum<G>(s2[u]);
      const int p = pb + u * NG + g;
      if ((lane % G) == 0 && p < p1) out[p] = S_hat[p] + t + bias;
    }
  }
}

// dP[r] = w2 * sum_p g_p [z_p > 0];  dw2 partial per block (fixed order).
// SOFT: the row also fed a softmax (prob, forward SOFT variant) whose
// gradient gS arrives here: the total score gradient is
// Gr + prob * (gS - <prob, gS>) (softmax backward + the pass-through add,
// one value per lane for k <= 64); it is written to Gtot (read by the
// column kernel and returned as the S_hat gradient).
template <int G, bool SOFT>
__global__ __launch_bounds__(256) void sparse_consensus_bwd_rows_g_kernel(
    const int* __restrict__ rowptr, const int* __restrict__ col,
    const float* __restrict__ Gr, const float* __restrict__ prob,
    const float* __restrict__ gS, float* __restrict__ Gtot,
    const float* __restrict__ P,
    const float* __restrict__ Q, const float* __restrict__ b1,
    const float* __restrict__ w2, float* __restrict__ dP,
    float* __restrict__ dw2_part, int ldp, int rows, int R) {
  constexpr int NG = kWave / G;
  __shared__ float4 red[kSpWaves][G];
  __shared__ float4 redb[kSpWaves][G];
  __shared__ float redg[kSpWaves];
  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  const int g = lane / G, gl = lane % G, c = gl * 4;
  const bool cok = c < R;
  const float4 bb = cok ? ld4(b1 + c) : make_float4(0, 0, 0, 0);
  const float4 wv = cok ? ld4(w2 + c) : make_float4(0, 0, 0, 0);
  float dw[4] = {0.f, 0.f, 0.f, 0.f};
  float db[4] = {0.f, 0.f, 0.f, 0.f};   // b1 gradient: sum of dP rows
  float gsum = 0.f;                      // b2 gradient: sum of the entries' g
  for (int r = blockIdx.x * kSpWaves + wave; r < rows;
       r += gridDim.x * kSpWaves) {
    float pv[4] = {0.f, 0.f, 0.f, 0.f}, dp[4] = {0.f, 0.f, 0.f, 0.f};
    if (cok) {
      const float4 p = ld4(P + (size_t)r * R + c);
      pv[0] = p.x + bb.x; pv[1] = p.y + bb.y;
      pv[2] = p.z + bb.z; pv[3] = p.w + bb.w;
    }
    const int p0 = rowptr[r], p1 = rowptr[r + 1];
    float gt = 0.f;     // SOFT: total gradient of candidate p0 + lane
    if constexpr (SOFT) {
      const int p = p0 + lane;
      float sp = 0.f, gs = 0.f, gg = 0.f;
      if (p < p1) { sp = prob[p]; gs = gS[p]; gg = Gr[p]; }
      float dot = sp * gs;
#pragma unroll
      for (int off = 1; off < kWave; off <<= 1) dot += __shfl_xor(dot, off);
      gt = gg + sp * (gs - dot);
      if (p < p1) Gtot[p] = gt;
    }
    for (int j = 0; j * NG < p1 - p0; ++j) {   // wave-uniform trip count
      const int p = p0 + g + NG * j;
      float gv;
      if constexpr (SOFT) gv = __shfl(gt, (g + NG * j) & (kWave - 1));
      if (p >= p1 || !cok) continue;
      if constexpr (!SOFT) gv = Gr[p];
      if (gl == 0) gsum += gv;
      const float4 q4 = ld4(Q + (size_t)col[p] * R + c);
      const float q[4] = {q4.x, q4.y, q4.z, q4.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float z = pv[k] - q[k];
        if (z > 0.f) {
          dp[k] += gv;
          dw[k] = fmaf(gv, z, dw[k]);
        }
      }
    }
#pragma unroll
    for (int off = G; off < kWave; off <<= 1)
#pragma unroll
      for (int k = 0; k < 4; ++k) dp[k] += __shfl_xor(dp[k], off);
    if (g == 0 && cok) {
      const float4 d =
          make_float4(dp[0] * wv.x, dp[1] * wv.y, dp[2] * wv.z, dp[3] * wv.w);
      *reinterpret_cast<float4*>(dP + (size_t)r * R + c) = d;
      db[0] += d.x; db[1] += d.y; db[2] += d.z; db[3] += d.w;
    }
  }
#pragma unroll
  for (int off = G; off < kWave; off <<= 1)
#pragma unroll
    for (int k = 0; k < 4; ++k) dw[k] += __shfl_xor(dw[k], off);
#pragma unroll
  for (int off = 1; off < kWave; off <<= 1) gsum += __shfl_xor(gsum, off);
  if (g == 0) {
    red[wave][gl] = make_float4(dw[0], dw[1], dw[2], dw[3]);
    redb[wave][gl] = make_float4(db[0], db[1], db[2], db[3]);
  }
  if (lane == 0) redg[wave] = gsum;
  __syncthreads();
  // block partial row: [dw2 (R) | db1 (R) | db2, 0, 0, 0]
  float* prow = dw2_part + (size_t)blockIdx.x * ldp;
  if (threadIdx.x < G && threadIdx.x * 4 < R) {
    float4 s = red[0][threadIdx.x], sb = redb[0][threadIdx.x];
#pragma unroll
    for (int w = 1; w < kSpWaves; ++w) {
      const float4 t = red[w][threadIdx.x], tb = redb[w][threadIdx.x];
      s.x += t.x; s.y += t.y; s.z += t.z; s.w += t.w;
      sb.x += tb.x; sb.y += tb.y; sb.z += tb.z; sb.w += tb.w;
    }
    *reinterpret_cast<float4*>(prow + threadIdx.x * 4) = s;
    *reinterpret_cast<float4*>(prow + R + threadIdx.x * 4) = sb;
  }
  if (threadIdx.x == 0) {
    float t = redg[0];
#pragma unroll
    for (int w = 1; w < kSpWaves; ++w) t += redg[w];
    *reinterpret_cast<float4*>(prow + 2 * R) = make_float4(t, 0.f, 0.f, 0.f);
  }
}

// dQ[j] = -w2 * sum_{e in col j} g_e [P_row(e) + b1 - Q_j > 0], walked in
// pieces of <= T entries (spmm.hip's piece plan), one G-lane group per piece:
// a target picked by thousands of source rows no longer serialises the
// kernel, and short columns are packed 64 / G to a wave.
template <int G>
__global__ __launch_bounds__(256) void sparse_consensus_bwd_cols_piece_kernel(
    const int* __restrict__ row_of, const int* __restrict__ perm,
    const int* __restrict__ prow, const int* __restrict__ pbeg,
    const int* __restrict__ pend, int npieces, const float* __restrict__ Gr,
    const float* __restrict__ P, const float* __restrict__ Q,
    const float* __restrict__ b1, const float* __restrict__ w2,
    float* __restrict__ dQ, float* __restrict__ part, int cols, int R) {
  constexpr int PPB = 256 / G;
  const int v = xcd_remap(blockIdx.x, gridDim.x) * PPB + threadIdx.x / G;
  const int c = (threadIdx.x % G) * 4;
  if (v >= npieces || c >= R) return;
  const int code = prow[v];
  if (code >= cols) return;
  const bool single = code >= 0;
  const int j = single ? code : ~code;
  const int beg = pbeg[v], end = pend[v];
  const float4 q = ld4(Q + (size_t)j * R + c), bb = ld4(b1 + c);
  const float qb[4] = {bb.x - q.x, bb.y - q.y, bb.z - q.z, bb.w - q.w};
  float dq[4] = {0.f, 0.f, 0.f, 0.f};
  // 8 entries per round (indices clamped, out-of-piece entries add 0): two
  // dependent load rounds per 8 entries instead of per 2
  for (int e = beg; e < end; e += 8) {
    int pi[8], ri[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int eu = min(e + u, end - 1);
      pi[u] = perm[eu];
      ri[u] = row_of[eu];
    }
    float gv[8];
    float4 pr[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      gv[u] = Gr[pi[u]];
      pr[u] = ld4(P + (size_t)ri[u] * R + c);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const float g = e + u < end ? gv[u] : 0.f;
      if (pr[u].x + qb[0] > 0.f) dq[0] += g;
      if (pr[u].y + qb[1] > 0.f) dq[1] += g;
      if (pr[u].z + qb[2] > 0.f) dq[2] += g;
      if (pr[u].w + qb[3] > 0.f) dq[3] += g;
    }
  }
  if (single) {
    const float4 w = ld4(w2 + c);
    *reinterpret_cast<float4*>(dQ + (size_t)j * R + c) =
        make_float4(-dq[0] * w.x, -dq[1] * w.y, -dq[2] * w.z, -dq[3] * w.w);
  } else {
    *reinterpret_cast<float4*>(part + (size_t)v * R + c) =
        make_float4(dq[0], dq[1], dq[2], dq[3]);
  }
}

void spmm_piece_fold_f32(const at::Tensor& pptr, const at::Tensor& part,
                         int R, int C, const float* colscale, float sign,
                         float* out);

// Lanes per candidate for the group kernels (0: not eligible).
static int group_lanes(int64_t C, std::initializer_list<const void*> ptrs) {
  if (C % 4 != 0 || C > 256 || C == 0) return 0;
  for (const void* p : ptrs)
    if (!aligned16(p)) return 0;
  int G = 1;
  while (G * 4 < C) G <<= 1;
  return G;
}

#define DGMC_GROUP_DISPATCH(G, ...)                             \
  switch (G) {                                                  \
    case 1: { constexpr int GG = 1; __VA_ARGS__; } break;       \
    case 2: { constexpr int GG = 2; __VA_ARGS__; } break;       \
    case 4: { constexpr int GG = 4; __VA_ARGS__; } break;       \
    case 8: { constexpr int GG = 8; __VA_ARGS__; } break;       \
    case 16: { constexpr int GG = 16; __VA_ARGS__; } break;     \
    case 32: { constexpr int GG = 32; __VA_ARGS__; } break;     \
    default: { constexpr int GG = 64; __VA_ARGS__; } break;     \
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
  const int G = group_lanes(A.size(1), {A.data_ptr(), B.data_ptr()});
  if (G > 0) {
    DGMC_GROUP_DISPATCH(G, hipLaunchKernelGGL(
        sddmm_g_kernel<GG>, dim3(sp_blocks(rows)), dim3(256), 0, stream(),
        rowptr.data_ptr<int>(), col.data_ptr<int>(), A.data_ptr<float>(),
        B.data_ptr<float>(), val.data_ptr<float>(), (int)rows,
        (int)A.size(1)));
    DGMC_CHECK_LAUNCH();
    return val;
  }
  hipLaunchKernelGGL(sddmm_kernel, dim3(sp_blocks(rows)), dim3(256), 0,
                     stream(), rowptr.data_ptr<int>(), col.data_ptr<int>(),
                     A.data_ptr<float>(), B.data_ptr<float>(),
                     val.data_ptr<float>(), (int)rows, (int)A.size(1));
  DGMC_CHECK_LAUNCH();
  return val;
}

// Max candidates per row of the fused-softmax variants (forward: 4
// iterations x 2 batches x 64 / G; backward: one candidate per lane).
static int64_t soft_max_k(int G) { return std::min<int64_t>(64, 8 * (kWave / G)); }

std::tuple<at::Tensor, at::Tensor> sparse_consensus_fwd_impl(
    const at::Tensor& rowptr, const at::Tensor& col, const at::Tensor& S_hat,
    const at::Tensor& P, const at::Tensor& Q, const at::Tensor& b1,
    const at::Tensor& w2, const at::Tensor& b2, int64_t k_soft) {
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
  at::Tensor prob;
  if (rows == 0) return {out, k_soft > 0 ? at::empty_like(S_hat) : prob};
  const int G = group_lanes(R, {P.data_ptr(), Q.data_ptr(), b1.data_ptr(),
                                w2.data_ptr()});
  if (k_soft > 0) {
    // uniform rows of k_soft candidates (the top-k candidate CSR)
    TORCH_CHECK(G > 0 && k_soft <= soft_max_k(G) &&
                    col.numel() == rows * k_soft,
                "sparse_consensus_fwd_prob: needs C % 4 == 0, C <= 256 and "
                "uniform rows of <= ", G > 0 ? soft_max_k(G) : 0,
                " candidates");
    prob = at::empty_like(S_hat);
    DGMC_GROUP_DISPATCH(G, hipLaunchKernelGGL(
        (sparse_consensus_fwd_g_kernel<GG, true>), dim3(sp_blocks(rows)),
        dim3(256), 0, stream(), rowptr.data_ptr<int>(), col.data_ptr<int>(),
        S_hat.data_ptr<float>(), P.data_ptr<float>(), Q.data_ptr<float>(),
        b1.data_ptr<float>(), w2.data_ptr<float>(), b2.data_ptr<float>(),
        out.data_ptr<float>(), prob.data_ptr<float>(), (int)rows, R));
    DGMC_CHECK_LAUNCH();
    return {out, prob};
  }
  if (G > 0) {
    DGMC_GROUP_DISPATCH(G, hipLaunchKernelGGL(
        (sparse_consensus_fwd_g_kernel<GG, false>), dim3(sp_blocks(rows)),
        dim3(256), 0, stream(), rowptr.data_ptr<int>(), col.data_ptr<int>(),
        S_hat.data_ptr<float>(), P.data_ptr<float>(), Q.data_ptr<float>(),
        b1.data_ptr<float>(), w2.data_ptr<float>(), b2.data_ptr<float>(),
        out.data_ptr<float>(), (float*)nullptr, (int)rows, R));
    DGMC_CHECK_LAUNCH();
    return {out, prob};
  }
  hipLaunchKernelGGL(sparse_consensus_fwd_kernel, dim3(sp_blocks(rows)),
                     dim3(256), 0, stream(), rowptr.data_ptr<int>(),
                     col.data_ptr<int>(), S_hat.data_ptr<float>(),
                     P.data_ptr<float>(), Q.data_ptr<float>(),
                     b1.data_ptr<float>(), w2.data_ptr<float>(),
                     b2.data_ptr<float>(), out.data_ptr<float>(), (int)rows,
                     R);
  DGMC_CHECK_LAUNCH();
  return {out, prob};
}

at::Tensor sparse_consensus_fwd(const at::Tensor& rowptr, const at::Tensor& col,
                                const at::Tensor& S_hat, const at::Tensor& P,
                                const at::Tensor& Q, const at::Tensor& b1,
                                const at::Tensor& w2, const at::Tensor& b2) {
  return std::get<0>(
      sparse_consensus_fwd_impl(rowptr, col, S_hat, P, Q, b1, w2, b2, 0));
}

// The update and the row softmax of its result (uniform rows of k).
std::tuple<at::Tensor, at::Tensor> sparse_consensus_fwd_prob(
    const at::Tensor& rowptr, const at::Tensor& col, const at::Tensor& S_hat,
    const at::Tensor& P, const at::Tensor& Q, const at::Tensor& b1,
    const at::Tensor& w2, const at::Tensor& b2, int64_t k) {
  TORCH_CHECK(k >= 1, "sparse_consensus_fwd_prob: k >= 1");
  return sparse_consensus_fwd_impl(rowptr, col, S_hat, P, Q, b1, w2, b2, k);
}

std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor>
sparse_consensus_bwd(
    const at::Tensor& rowptr, const at::Tensor& col, const at::Tensor& colptr,
    const at::Tensor& row_of, const at::Tensor& perm, const at::Tensor& G,
    const at::Tensor& P, const at::Tensor& Q, const at::Tensor& b1,
    const at::Tensor& w2, const c10::optional<at::Tensor>& pptr,
    const c10::optional<at::Tensor>& prow,
    const c10::optional<at::Tensor>& pbeg,
    const c10::optional<at::Tensor>& pend,
    const c10::optional<at::Tensor>& prob,
    const c10::optional<at::Tensor>& gS,
    const c10::optional<at::Tensor>& dpq) {
  check_f32_2d(P, "P");
  check_f32_2d(Q, "Q");
  const bool pieces = pptr.has_value() && pptr->defined() &&
                      prow.has_value() && prow->defined() &&
                      pbeg.has_value() && pbeg->defined() &&
                      pend.has_value() && pend->defined();
  TORCH_CHECK(pieces ? perm.scalar_type() == at::kInt
                     : perm.scalar_type() == at::kLong,
              "perm must be int32 with a piece plan, int64 otherwise");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(P.device());
  const int64_t rows = rowptr.numel() - 1, cols = colptr.numel() - 1;
  const int R = P.size(1);
  TORCH_CHECK(rows == P.size(0) && cols == Q.size(0), "shape mismatch");
  TORCH_CHECK(G.numel() == col.numel() && perm.numel() == col.numel() &&
                  row_of.numel() == col.numel(),
              "sparse_consensus_bwd: entry arrays");
  at::Tensor dP, dQ;
  if (dpq.has_value() && dpq->defined()) {   // [dP; dQ] in one buffer
    TORCH_CHECK(dpq->scalar_type() == at::kFloat && dpq->is_contiguous() &&
                    dpq->dim() == 2 && dpq->size(0) == rows + cols &&
                    dpq->size(1) == R,
                "sparse_consensus_bwd: dpq fp32 contiguous [rows + cols, R]");
    dP = dpq->narrow(0, 0, rows);
    dQ = dpq->narrow(0, rows, cols);
  } else {
    dP = at::empty_like(P);
    dQ = at::empty_like(Q);
  }
  const int nb = std::max(1, std::min(sp_blocks(rows), 1024));
  // per-block partials [dw2 (R) | db1 (R) | db2, 0, 0, 0]
  const int ldp = 2 * R + 4;
  at::Tensor dw2 = at::empty({nb, ldp}, P.options());
  const int Gl = group_lanes(R, {P.data_ptr(), Q.data_ptr(), b1.data_ptr(),
                                 w2.data_ptr()});
  const bool soft = prob.has_value() && prob->defined() && gS.has_value() &&
                    gS->defined();
  at::Tensor Gt = G;   // total score gradient (read by the column walk)
  if (soft) {
    TORCH_CHECK(Gl > 0 && rows > 0 && col.numel() % rows == 0 &&
                    col.numel() / rows <= 64 &&
                    prob->numel() == col.numel() &&
                    gS->numel() == col.numel() && prob->is_contiguous() &&
                    gS->is_contiguous(),
                "sparse_consensus_bwd: softmax-fused backward needs uniform "
                "rows of <= 64 candidates");
    Gt = at::empty_like(G);
    DGMC_GROUP_DISPATCH(Gl, hipLaunchKernelGGL(
        (sparse_consensus_bwd_rows_g_kernel<GG, true>), dim3(nb), dim3(256), 0,
        stream(), rowptr.data_ptr<int>(), col.data_ptr<int>(),
        G.data_ptr<float>(), prob->data_ptr<float>(), gS->data_ptr<float>(),
        Gt.data_ptr<float>(), P.data_ptr<float>(), Q.data_ptr<float>(),
        b1.data_ptr<float>(), w2.data_ptr<float>(), dP.data_ptr<float>(),
        dw2.data_ptr<float>(), ldp, (int)rows, R));
    DGMC_CHECK_LAUNCH();
  } else if (rows > 0 && Gl > 0) {
    DGMC_GROUP_DISPATCH(Gl, hipLaunchKernelGGL(
        (sparse_consensus_bwd_rows_g_kernel<GG, false>), dim3(nb), dim3(256),
        0, stream(), rowptr.data_ptr<int>(), col.data_ptr<int>(),
        G.data_ptr<float>(), (const float*)nullptr, (const float*)nullptr,
        (float*)nullptr, P.data_ptr<float>(), Q.data_ptr<float>(),
        b1.data_ptr<float>(), w2.data_ptr<float>(), dP.data_ptr<float>(),
        dw2.data_ptr<float>(), ldp, (int)rows, R));
    DGMC_CHECK_LAUNCH();
  } else if (rows > 0) {
    hipLaunchKernelGGL(sparse_consensus_bwd_rows_kernel, dim3(nb), dim3(256),
                       0, stream(), rowptr.data_ptr<int>(),
                       col.data_ptr<int>(), G.data_ptr<float>(),
                       P.data_ptr<float>(), Q.data_ptr<float>(),
                       b1.data_ptr<float>(), w2.data_ptr<float>(),
                       dP.data_ptr<float>(), dw2.data_ptr<float>(), (int)rows,
                       R, ldp);
    DGMC_CHECK_LAUNCH();
    // (wide-R fallback: the bias partials by library reductions, block 0)
    dw2.narrow(1, R, R + 4).zero_();
    dw2.select(0, 0).narrow(0, R, R).copy_(dP.sum(0));
    dw2.select(0, 0).narrow(0, 2 * R, 1).copy_(G.sum().view({1}));
  } else {
    dw2.zero_();
  }
  if (cols > 0 && pieces && Gl > 0) {
    TORCH_CHECK(pptr->scalar_type() == at::kInt &&
                    prow->scalar_type() == at::kInt &&
                    pbeg->scalar_type() == at::kInt &&
                    pend->scalar_type() == at::kInt &&
                    pptr->numel() == cols + 1 &&
                    prow->numel() == pbeg->numel() &&
                    prow->numel() == pend->numel(),
                "sparse_consensus_bwd: piece plan");
    const int npieces = (int)prow->numel();
    at::Tensor part = at::empty({(int64_t)npieces, R}, P.options());
    DGMC_GROUP_DISPATCH(Gl, hipLaunchKernelGGL(
        sparse_consensus_bwd_cols_piece_kernel<GG>,
        dim3((npieces + 256 / GG - 1) / (256 / GG)), dim3(256), 0, stream(),
        row_of.data_ptr<int>(), perm.data_ptr<int>(), prow->data_ptr<int>(),
        pbeg->data_ptr<int>(), pend->data_ptr<int>(), npieces,
        Gt.data_ptr<float>(), P.data_ptr<float>(), Q.data_ptr<float>(),
        b1.data_ptr<float>(), w2.data_ptr<float>(), dQ.data_ptr<float>(),
        part.data_ptr<float>(), (int)cols, R));
    DGMC_CHECK_LAUNCH();
    spmm_piece_fold_f32(*pptr, part, (int)cols, R, w2.data_ptr<float>(), -1.f,
                        dQ.data_ptr<float>());
  } else if (cols > 0) {
    at::Tensor perm64 = perm.to(at::kLong);
    hipLaunchKernelGGL(sparse_consensus_bwd_cols_kernel, dim3(sp_blocks(cols)),
                       dim3(256), 0, stream(), colptr.data_ptr<int>(),
                       row_of.data_ptr<int>(), perm64.data_ptr<int64_t>(),
                       Gt.data_ptr<float>(), P.data_ptr<float>(),
                       Q.data_ptr<float>(), b1.data_ptr<float>(),
                       w2.data_ptr<float>(), dQ.data_ptr<float>(), (int)cols,
                       R);
    DGMC_CHECK_LAUNCH();
  }
  return {dP, dQ, dw2, Gt};
}

}  // namespace dgmc
