// Fused RelConv (psi_2 of the DBP15K config) on exact-f32 MFMA.
//
// Reference: /root/reference/dgmc/models/rel.py:25-31 -
//   out_i = root(x)_i + mean_{j->i} lin1(x)_j + mean_{i->j} lin2(x)_j
// (PyG MessagePassing, flows source_to_target / target_to_source, mean
// aggregation = sum / max(count, 1)), used with 32 channels in DBP15K's
// consensus network (examples/dbp15k.py:29-33: RelCNN(32, 32, 3, cat=True,
// lin=True)).  Per layer and consensus step the reference runs three Linear
// GEMMs and two scatter-means; here ONE kernel per layer and direction:
//
//   forward   A_i = [ mean_in(x)_i | mean_out(x)_i | x_i ]        (gathered)
//             out = act(A W_cat^T + b),  W_cat = [W1 | W2 | Wr]  [C, 3K]
//   backward  G_j = [ sum_{i in out(j)} g'_i / deg_in(i) |
//                     sum_{i in in(j)}  g'_i / deg_out(i) | g'_j ]
//             dx  = G W_stack,  W_stack = [W1; W2; Wr]           [3C, K]
//             dW_stack += G^T x (per-tile partials, loop-accumulated),
//             db += sum_j g'_j
//
// (aggregate-then-multiply: the same linear map as multiply-then-aggregate,
// rounded differently.)  Lists: one joint CSR per direction (forward: row i =
// in-neighbours then out-neighbours; backward: out-list then in-list with the
// per-entry weights), so a tile's entries are one contiguous range, staged
// into LDS in one coalesced round.  A workgroup owns a 64-row tile; the
// tile's contiguous entry range is cut into 32 equal chunks gathered by
// 8-lane groups (one 16-byte vector per lane and entry, 16 loads in flight
// per lane), partial sums of segments crossing chunk borders completed in
// chunk order (merge-path balance: knowledge-graph hub rows are spread over
// several groups, no group walks more than ceil(entries / 32)).  All loads
// that do not depend on the lists are issued in one round at kernel start,
// so a tile costs ~2 + entries / 512 memory round trips.  Then the
// tile is multiplied on v_mfma_f32_16x16x4_f32 (exact fp32 products) and the
// epilogue adds the bias / ReLU, the fused consensus projection, or the
// masked gradient adds.  Deterministic: fixed summation orders, no atomics;
// weight-gradient partials per tile are folded by rel_fold (two stages).
#include "common.h"

namespace dgmc {

namespace {

constexpr int kRcK = 32;          // input channels (rnd_dim of the config)
constexpr int kRcC = 32;          // output channels
constexpr int kRcRows = 64;       // rows per tile
constexpr int kRcP = 98;          // LDS pitch of [row][96] tiles (98 % 32 == 2)
constexpr int kRcXP = 48;         // pitch of the [row][32] x tile (48 % 32 == 16)
constexpr int kRcFP = 130;        // pitch of [row][128] projection tiles
constexpr int kRcDP = 34;         // pitch of [row][32] dPQ tiles
constexpr int kRcFT = 144;        // pitch of the [row][128] feat tile (bwd)
constexpr int kRcCap = 1024;      // tile entries staged in LDS (rest: global)
constexpr int kRcU = 16;          // gather loads in flight per lane (max)
constexpr int kRcPart = 3 * kRcC * kRcK + kRcC;   // dW_stack + db per tile
constexpr int kRcPartPer = (kRcPart + 255) / 256; // per thread

typedef float rc_f32x4 __attribute__((ext_vector_type(4)));
typedef float rc_f32x2 __attribute__((ext_vector_type(2)));

// Joint lists of one direction: row i's entries [ptr[i], ptr[i+1]), the
// second list starting at split[i]; w: per-entry weights (backward only).
struct RcPlan {
  const int* ptr;
  const int* col;     // packed: column | (2 (row % 64) + list) << 24
  const int* split;
  const float* w;
  const unsigned char* hub;   // 1: gathered by the whole wave
  int N;
};

// Row j of a layer input: j < split ? a[j] : b[j - split] (the first
// layer's input [r_s; r_t] is read from the two separate buffers).
struct RcRows {
  const float* a;
  const float* b;
  int split, lda, ldb;
  // (32-bit offsets: the host checks rows * ld < 2^31)
  __device__ __forceinline__ const float* row(int j) const {
    const bool first = j < split;
    return (first ? a : b) + (first ? j * lda : (j - split) * ldb);
  }
};

struct RcFwd {
  RcRows x;
  const float* w[3];    // lin1, lin2, root weights [C][K]
  const float* bias;    // root bias [C]
  float* out;           // [N][ldo] (a column slice of the feature buffer)
  int ldo;
  float* xcopy;         // optional: own input rows copied here (feat slice 0)
  int ldxc;
  int relu;
  // fused consensus projection (last layer): pq_i = [feat_i[0:96] | out_i]
  // fold^T, fold [32][128]
  const float* feat;
  int ldf;
  const float* fold;
  float* pq;
};

struct RcBwd {
  const float* g;       // g' of this layer (already masked), [N][ldg]
  int ldg;
  RcRows x;             // this layer's input rows
  const float* w[3];
  const float* dadd;    // addend of dx (the input slice's own gradient)
  int ldadd;
  float* dout;          // dx rows j >= row0 at dout[(j - row0) * lddo]
  int lddo, row0;
  int mask;             // multiply (dadd + dx) by (x > 0)
  float* part;          // [n_tiles][kRcPart]
  int part_acc;
};

__device__ __forceinline__ float4 f4_ld(const float* p) {
  return *reinterpret_cast<const float4*>(p);
}
__device__ __forceinline__ void f4_add(float4& a, const float4& b) {
  a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
}
__device__ __forceinline__ void f4_fma(float4& a, float s, const float4& b) {
  a.x = fmaf(s, b.x, a.x); a.y = fmaf(s, b.y, a.y);
  a.z = fmaf(s, b.z, a.z); a.w = fmaf(s, b.w, a.w);
}
__device__ __forceinline__ float4 f4_zero() { return make_float4(0, 0, 0, 0); }
// Loads are issued unconditionally (from clamped, in-bounds addresses) and
// zeroed afterwards by a select: `cond ? load : 0` compiles to a divergent
// branch whose other side writes the load's registers, which forces a wait
// for that load on the spot - one memory round trip per load instead of one
// per round of independent loads.
__device__ __forceinline__ float4 f4_keep(bool keep, const float4& v) {
  return keep ? v : f4_zero();
}
__device__ __forceinline__ float4 f4_scale(const float4& a, float s) {
  return make_float4(a.x * s, a.y * s, a.z * s, a.w * s);
}
__device__ __forceinline__ float4 f4_xor(const float4& a, int m) {
  return make_float4(__shfl_xor(a.x, m), __shfl_xor(a.y, m),
                     __shfl_xor(a.z, m), __shfl_xor(a.w, m));
}

__device__ __forceinline__ void lds_put4(DGMC_LDS float* p, const float4& v) {
  // (8-byte aligned rows: pitch 98)
  reinterpret_cast<DGMC_LDS rc_f32x2*>(p)[0] = rc_f32x2{v.x, v.y};
  reinterpret_cast<DGMC_LDS rc_f32x2*>(p)[1] = rc_f32x2{v.z, v.w};
}
__device__ __forceinline__ void lds_put4a(DGMC_LDS float* p,
                                          const float4& v) {   // 16-byte
  *reinterpret_cast<DGMC_LDS rc_f32x4*>(p) = rc_f32x4{v.x, v.y, v.z, v.w};
}
__device__ __forceinline__ float4 lds_get4(const DGMC_LDS float* p) {
  const rc_f32x2 a = reinterpret_cast<const DGMC_LDS rc_f32x2*>(p)[0];
  const rc_f32x2 b = reinterpret_cast<const DGMC_LDS rc_f32x2*>(p)[1];
  return make_float4(a.x, a.y, b.x, b.y);
}

// Per-tile list staging: row pointers / splits of the tile's 64 rows and
// its entries (up to kRcCap) in LDS.  Every stage issues all of its global
// loads before its first LDS store (constant, unrolled trip counts), so a
// stage costs one memory round trip rather than one per loop iteration: the
// row heads are loaded with the kernel's other independent loads
// (rc_load_heads), the entries in one unrolled round after them.
struct RcTileLists {
  DGMC_LDS int* ptr;     // [65] absolute entry indices
  DGMC_LDS int* split;   // [64] (padding rows: ptr[N], so segment ends stay sorted)
  DGMC_LDS float* inv;   // [128] 1 / max(segment entries, 1)
  DGMC_LDS int* col;     // [kRcCap] packed entries: column | tile segment << 24
  DGMC_LDS float* w;     // [kRcCap] (weighted plans)
};
constexpr int kRcListInts =    // (padded to 16 bytes: the partials follow)
    (kRcRows + 1 + kRcRows + 2 * kRcRows + kRcCap + 3) & ~3;
constexpr int kRcColMask = (1 << 24) - 1;

__device__ __forceinline__ RcTileLists rc_lists(DGMC_LDS int* l, DGMC_LDS float* w) {
  return RcTileLists{l, l + kRcRows + 1, reinterpret_cast<DGMC_LDS float*>(l) +
                     2 * kRcRows + 1, l + 4 * kRcRows + 1, w};
}

__device__ __forceinline__ void rc_load_heads(const RcPlan& pl, int r0,
                                              int& hp, int& hs) {
  const int tid = threadIdx.x;
  hp = pl.ptr[min(r0 + min(tid, kRcRows), pl.N)];
  hs = pl.split[min(r0 + min(tid, kRcRows - 1), pl.N - 1)];
}

template <bool WEIGHTED>
__device__ __forceinline__ void rc_stage_lists(const RcPlan& pl, int r0,
                                               const RcTileLists& s, int hp,
                                               int hs) {
  static_assert(kRcCap == 4 * 256, "four entries per thread");
  const int tid = threadIdx.x;
  if (tid <= kRcRows) s.ptr[tid] = hp;
  if (tid < kRcRows) s.split[tid] = r0 + tid < pl.N ? hs : hp;
  __syncthreads();
  if (tid < 2 * kRcRows) {
    const int lr = tid >> 1;
    const int b = (tid & 1) ? s.split[lr] : s.ptr[lr];
    const int e = (tid & 1) ? s.ptr[lr + 1] : s.split[lr];
    s.inv[tid] = 1.f / (float)max(e - b, 1);
  }
  const int e0 = s.ptr[0], n = min(s.ptr[kRcRows] - e0, kRcCap);
  int cv[4];
  float wv[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {      // (the lists end with a dummy entry)
    const int t = e0 + max(min(tid + 256 * u, n - 1), 0);
    cv[u] = pl.col[t];
    wv[u] = WEIGHTED ? pl.w[t] : 0.f;
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int t = tid + 256 * u;
    if (t < n) {
      s.col[t] = cv[u];
      if (WEIGHTED) s.w[t] = wv[u];
    }
  }
  __syncthreads();
}

// Balanced (merge-path) gather of the tile's 128 segments (row lr, list
// l: segment 2 lr + l): the tile's contiguous entry range is cut into 32
// equal chunks, one per lane group (8 lanes, lane q holds channels
// 4q..4q+3); a group walks its chunk in order with kRcU loads in flight per
// lane and writes every segment that starts and ends inside it straight
// to sA (MEAN: divided by the segment's entry count), while the partial
// sums of segments crossing a chunk border go to LDS and are added in
// chunk order by the group where the segment starts.  Long rows (hub
// entities) are spread over several groups; no group walks more than
// ceil(n / 32) entries.  Empty segments keep the zeros written up front.
struct RcFlat {
  DGMC_LDS float* P;    // [32][2][32] border partials: slot 0 head, slot 1 tail
  DGMC_LDS int* PS;     // [32][2] their segments (-1: none)
  DGMC_LDS int* PO;     // [32] 1: the tail segment started in this chunk (owner)
};

__device__ __forceinline__ int rc_seg_end(const RcTileLists& s, int seg) {
  return (seg & 1) ? s.ptr[(seg >> 1) + 1] : s.split[seg >> 1];
}
__device__ __forceinline__ int rc_seg_begin(const RcTileLists& s, int seg) {
  return (seg & 1) ? s.split[seg >> 1] : s.ptr[seg >> 1];
}

// First segment whose end is past e (segment ends are non-decreasing):
// the non-empty segment holding entry e; 7 unrolled, branch-free steps.
__device__ __forceinline__ int rc_seg_of(const RcTileLists& s, int e) {
  int lo = 0;
#pragma unroll
  for (int st = kRcRows; st > 0; st >>= 1)
    lo += rc_seg_end(s, lo + st - 1) <= e ? st : 0;
  return lo;
}

// One 8-lane group's walk over its chunk [c0, c1): running segment `seg`
// (started inside the chunk or not), its partial sum `acc`.
template <bool WEIGHTED, bool MEAN, bool TWO>
struct RcWalk {
  const RcPlan& pl;
  const RcTileLists& s;
  const RcRows& src;
  DGMC_LDS float* sA;
  int pitch;
  const RcFlat& fl;
  int q, g, E0, c1;
  bool fits;
  int seg;
  bool started;
  float4 acc;

  __device__ __forceinline__ const float* row(int j) const {
    return TWO ? src.row(j) : src.a + (unsigned)(j * src.lda);
  }
  // The finished segment: its sum (MEAN: scaled by 1 / count) into the
  // tile, or - it began in an earlier chunk - the head partial.  (One code
  // path; divergent groups of a wave flush in the same instructions.)
  __device__ __forceinline__ void flush() {
    const float sc = (MEAN && started) ? s.inv[seg] : 1.f;
    DGMC_LDS float* p = started ? sA + (seg >> 1) * pitch + (seg & 1) * kRcK + 4 * q
                       : fl.P + (2 * g) * kRcK + 4 * q;
    lds_put4(p, f4_scale(acc, sc));
    if (!started && q == 0) fl.PS[2 * g] = seg;
  }
  // U entries from e0 (FULL: all before c1), U loads in flight per lane.
  template <int U, bool FULL>
  __device__ __forceinline__ void batch(int e0) {
    int pk[U];
    float wt[U];
    if (fits) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = (FULL ? e0 + u : min(e0 + u, c1 - 1)) - E0;
        pk[u] = s.col[e];
        wt[u] = WEIGHTED ? s.w[e] : 1.f;
      }
    } else {                         // > kRcCap entries: lists from global
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = FULL ? e0 + u : min(e0 + u, c1 - 1);
        pk[u] = pl.col[e];
        wt[u] = WEIGHTED ? pl.w[e] : 1.f;
      }
    }
    float4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = f4_ld(row(pk[u] & kRcColMask) + 4 * q);
    // Entries past c1 (clamped duplicates) add 0 and keep the segment; a
    // segment change (the packed tile segment of the entry - empty segments
    // never appear and keep their zeros) flushes the running sum.
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool live = FULL || e0 + u < c1;
      const int sg = live ? (pk[u] >> 24) : seg;
      if (sg != seg) {
        flush();
        acc = f4_zero();
        seg = sg;
        started = true;
      }
      f4_fma(acc, live ? wt[u] : 0.f, v[u]);     // (fma by 1: exact add)
    }
  }
};

template <bool WEIGHTED, bool MEAN, bool TWO, int U>
__device__ __forceinline__ void rc_gather_flat(const RcPlan& pl,
                                               const RcTileLists& s,
                                               const RcRows& src, DGMC_LDS float* sA,
                                               int pitch, const RcFlat& fl) {
  const int tid = threadIdx.x, q = tid & 7, g = tid >> 3;   // 32 groups
  const int E0 = s.ptr[0], E1 = s.ptr[kRcRows];
  const int n = E1 - E0;
  const int L = (n + 31) >> 5;
  const int c0 = E0 + min(n, g * L), c1 = E0 + min(n, (g + 1) * L);
  if (q == 0) {
    fl.PS[2 * g] = -1;
    fl.PS[2 * g + 1] = -1;
    fl.PO[g] = 0;
  }
  if (c0 < c1) {
    const int seg = rc_seg_of(s, c0);
    RcWalk<WEIGHTED, MEAN, TWO> w{pl, s, src, sA, pitch, fl, q, g, E0, c1,
                                  n <= kRcCap, seg,
                                  rc_seg_begin(s, seg) >= c0, f4_zero()};
    int e0 = c0;
    for (; e0 + U <= c1; e0 += U) w.template batch<U, true>(e0);
    for (; e0 < c1; e0 += U / 2) w.template batch<U / 2, false>(e0);
    // the segment current at c1
    if (rc_seg_end(s, w.seg) <= c1) {
      w.flush();
    } else {
      DGMC_LDS float* p = fl.P + (2 * g + 1) * kRcK + 4 * q;     // tail partial
      lds_put4(p, w.acc);
      if (q == 0) {
        fl.PS[2 * g + 1] = w.seg;
        fl.PO[g] = w.started ? 1 : 0;
      }
    }
  }
  __syncthreads();
  // owners complete their border segments in chunk order
  if (fl.PO[g]) {
    const int seg = fl.PS[2 * g + 1];
    float4 acc = lds_get4(fl.P + (2 * g + 1) * kRcK + 4 * q);
    int h = g + 1;
    for (; h < 32 && fl.PS[2 * h + 1] == seg && fl.PO[h] == 0; ++h)
      f4_add(acc, lds_get4(fl.P + (2 * h + 1) * kRcK + 4 * q));
    if (h < 32 && fl.PS[2 * h] == seg)
      f4_add(acc, lds_get4(fl.P + (2 * h) * kRcK + 4 * q));
    const float4 v = MEAN ? f4_scale(acc, s.inv[seg]) : acc;
    lds_put4(sA + (seg >> 1) * pitch + (seg & 1) * kRcK + 4 * q, v);
  }
}

// The three [C][K] weights: loaded into registers with the other
// independent loads (rc_load_w), stored afterwards (rc_store_w).  FWD:
// sW[c][s * K + k] = W_s[c][k] (pitch kRcP); else (backward)
// sW[k][s * C + c] = W_s[c][k].
__device__ __forceinline__ void rc_load_w(const float* const w[3],
                                          float4 (&v)[3]) {
  static_assert(kRcC * kRcK == 4 * 256, "one vector per thread and weight");
#pragma unroll
  for (int u = 0; u < 3; ++u) v[u] = f4_ld(w[u] + 4 * threadIdx.x);
}

template <bool FWD>
__device__ __forceinline__ void rc_store_w(const float4 (&v)[3], DGMC_LDS float* sW) {
  const int r = 4 * threadIdx.x, c = r / kRcK, k = r % kRcK;
#pragma unroll
  for (int u = 0; u < 3; ++u) {
    if (FWD) {
      lds_put4(sW + c * kRcP + u * kRcK + k, v[u]);
    } else {
      DGMC_LDS float* p = sW + k * kRcP + u * kRcC + c;
      p[0] = v[u].x;
      p[kRcP] = v[u].y;
      p[2 * kRcP] = v[u].z;
      p[3 * kRcP] = v[u].w;
    }
  }
}

// zero the first `vecs` 4-float vectors of each of the 64 rows of an LDS tile
template <int VECS>
__device__ __forceinline__ void rc_zero_rows(DGMC_LDS float* sA, int pitch) {
#pragma unroll
  for (int u = 0; u < kRcRows * VECS / 256; ++u) {
    const int t = threadIdx.x + 256 * u;
    lds_put4(sA + (t / VECS) * pitch + (t % VECS) * 4, f4_zero());
  }
}

// ---------------------------------------------------------------------------
// Forward.  LDS: sA [64][kRcP] (PROJ: sF [64][kRcFP]), sW [32][kRcP] (PROJ:
// then the fold [32][kRcFP]), lists.
// ---------------------------------------------------------------------------
constexpr int kRcListLds = kRcListInts * 4 +
                           (64 * kRcK + 64 + 32) * 4;   // + RcFlat
constexpr int kRcFwdLds = (kRcRows * kRcP + kRcC * kRcP) * 4 + kRcListLds;
constexpr int kRcFwdProjLds =
    (kRcRows * kRcFP + 32 * kRcFP) * 4 + kRcListLds;

template <bool PROJ, bool TWO>
__global__ __launch_bounds__(256) void relconv_fwd_kernel(RcPlan pl,
                                                          RcFwd a) {
  extern __shared__ __attribute__((aligned(16))) float rc_smem[];
  // sA [64][kRcP] / [64][kRcFP]
  DGMC_LDS float* sA = (DGMC_LDS float*)rc_smem;
  DGMC_LDS float* sW = sA + kRcRows * (PROJ ? kRcFP : kRcP);
  DGMC_LDS int* lists = reinterpret_cast<DGMC_LDS int*>(
      sW + (PROJ ? 32 * kRcFP : kRcC * kRcP));
  const RcTileLists s = rc_lists(lists, nullptr);
  DGMC_LDS float* flp = reinterpret_cast<DGMC_LDS float*>(lists + kRcListInts);
  const RcFlat fl{flp, reinterpret_cast<DGMC_LDS int*>(flp + 64 * kRcK),
                  reinterpret_cast<DGMC_LDS int*>(flp + 64 * kRcK) + 64};
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r0 = blockIdx.x * kRcRows;
  const int q = lane & 7, grp = lane >> 3;
  const int la = wave * 16 + grp, lb = la + 8;
  const int ra = r0 + la, rb = r0 + lb;
  // round 1: every load that does not depend on the lists
  const int rl = pl.N - 1;
  const float4 xa = f4_keep(ra < pl.N, f4_ld(a.x.row(min(ra, rl)) + 4 * q));
  const float4 xb = f4_keep(rb < pl.N, f4_ld(a.x.row(min(rb, rl)) + 4 * q));
  float4 wv[3];
  rc_load_w(a.w, wv);
  int hp, hs;
  rc_load_heads(pl, r0, hp, hs);
  float4 fr[6], fo[4];     // PROJ: this lane's share of feat[:, 0:96], fold
  if (PROJ) {
#pragma unroll
    for (int u = 0; u < 6; ++u) {
      const int t = lane + 64 * u;            // 16 rows x 24 vectors
      const int r = r0 + wave * 16 + t / 24;
      fr[u] = f4_keep(r < pl.N, f4_ld(a.feat + (size_t)min(r, rl) * a.ldf +
                                      (t % 24) * 4));
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) fo[u] = f4_ld(a.fold + 4 * (tid + 256 * u));
  }
  rc_store_w<true>(wv, sW);
  rc_zero_rows<16>(sA, PROJ ? kRcFP : kRcP);       // mean parts := 0
  rc_stage_lists<false>(pl, r0, s, hp, hs);
  {
    const int P = PROJ ? kRcFP : kRcP;
    rc_gather_flat<false, true, TWO, PROJ ? 8 : kRcU>(pl, s, a.x, sA, P,
                                                            fl);
    lds_put4(sA + la * P + 2 * kRcK + 4 * q, xa);
    lds_put4(sA + lb * P + 2 * kRcK + 4 * q, xb);
    if (a.xcopy) {
      if (ra < pl.N)
        *reinterpret_cast<float4*>(a.xcopy + (size_t)ra * a.ldxc + 4 * q) = xa;
      if (rb < pl.N)
        *reinterpret_cast<float4*>(a.xcopy + (size_t)rb * a.ldxc + 4 * q) = xb;
    }
  }
  __syncthreads();
  // out[16 rows of this wave][32] = A W_cat^T on 16x16x4 f32 MFMA.
  const int i = lane & 15, kk = lane >> 4;
  const int P = PROJ ? kRcFP : kRcP;
  rc_f32x4 o0 = {0.f, 0.f, 0.f, 0.f}, o1 = {0.f, 0.f, 0.f, 0.f};
  const DGMC_LDS float* arow = sA + (wave * 16 + i) * P + kk;
#pragma unroll 8
  for (int k0 = 0; k0 < 3 * kRcK; k0 += 4) {
    const float av = arow[k0];
    o0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av, sW[i * kRcP + k0 + kk], o0,
                                              0, 0, 0);
    o1 = __builtin_amdgcn_mfma_f32_16x16x4f32(
        av, sW[(16 + i) * kRcP + k0 + kk], o1, 0, 0, 0);
  }
  if (PROJ) {
    __syncthreads();        // sA / sW are reused below
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int t = 4 * (tid + 256 * u);
      lds_put4(sW + (t >> 7) * kRcFP + (t & 127), fo[u]);
    }
  }
  DGMC_LDS float* sF = sA;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int c = 16 * h + i;
    const float bc = a.bias[c];
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int lr = wave * 16 + kk * 4 + rr;
      const int r = r0 + lr;
      float v = (h ? o1[rr] : o0[rr]) + bc;
      if (a.relu) v = fmaxf(v, 0.f);
      if (r < pl.N) a.out[(size_t)r * a.ldo + c] = v;
      if (PROJ) sF[lr * kRcFP + 96 + c] = v;
    }
  }
  if (!PROJ) return;
#pragma unroll
  for (int u = 0; u < 6; ++u) {
    const int t = lane + 64 * u;
    DGMC_LDS float* p = sF + (wave * 16 + t / 24) * kRcFP + (t % 24) * 4;
    p[0] = fr[u].x; p[1] = fr[u].y; p[2] = fr[u].z; p[3] = fr[u].w;
  }
  __syncthreads();
  // pq[16 rows][32] = [feat[:, 0:96] | out] fold^T
  rc_f32x4 p0 = {0.f, 0.f, 0.f, 0.f}, p1 = {0.f, 0.f, 0.f, 0.f};
  const DGMC_LDS float* frow = sF + (wave * 16 + i) * kRcFP + kk;
#pragma unroll 8
  for (int k0 = 0; k0 < 128; k0 += 4) {
    const float av = frow[k0];
    p0 = __builtin_amdgcn_mfma_f32_16x16x4f32(
        av, sW[i * kRcFP + k0 + kk], p0, 0, 0, 0);
    p1 = __builtin_amdgcn_mfma_f32_16x16x4f32(
        av, sW[(16 + i) * kRcFP + k0 + kk], p1, 0, 0, 0);
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int r = r0 + wave * 16 + kk * 4 + rr;
      if (r < pl.N) a.pq[(size_t)r * 32 + 16 * h + i] = h ? p1[rr] : p0[rr];
    }
  }
}

// ---------------------------------------------------------------------------
// Backward.  LDS: sG [64][kRcP], sW [32 (k)][kRcP], sX [64][kRcXP], lists.
// ---------------------------------------------------------------------------
constexpr int kRcBwdLds =
    (kRcRows * kRcP + kRcK * kRcP + kRcRows * kRcXP + kRcCap) * 4 +
    kRcListLds;

__global__ __launch_bounds__(256) void relconv_bwd_kernel(RcPlan pl,
                                                          RcBwd a) {
  extern __shared__ __attribute__((aligned(16))) float rc_smem[];
  DGMC_LDS float* sG = (DGMC_LDS float*)rc_smem;   // [64][kRcP]
  DGMC_LDS float* sW = sG + kRcRows * kRcP;           // [32 k][kRcP] (3C wide)
  DGMC_LDS float* sX = sW + kRcK * kRcP;              // [64][kRcXP]
  DGMC_LDS float* sWt = sX + kRcRows * kRcXP;         // [kRcCap] entry weights
  DGMC_LDS int* lists = reinterpret_cast<DGMC_LDS int*>(sWt + kRcCap);
  const RcTileLists s = rc_lists(lists, sWt);
  DGMC_LDS float* flp = reinterpret_cast<DGMC_LDS float*>(lists + kRcListInts);
  const RcFlat fl{flp, reinterpret_cast<DGMC_LDS int*>(flp + 64 * kRcK),
                  reinterpret_cast<DGMC_LDS int*>(flp + 64 * kRcK) + 64};
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bool pacc = a.part_acc != 0;
  const int r0 = blockIdx.x * kRcRows;
  float* part = a.part + (size_t)blockIdx.x * kRcPart;
  // earlier uses' partials, loaded now (added after the MFMAs)
  float old[kRcPartPer];
#pragma unroll
  for (int u = 0; u < kRcPartPer; ++u) {
    const int t = tid + 256 * u;
    const float v = part[min(t, kRcPart - 1)];
    old[u] = (pacc && t < kRcPart) ? v : 0.f;
  }
  const int q = lane & 7, grp = lane >> 3;
  const int la = wave * 16 + grp, lb = la + 8;
  const int ra = r0 + la, rb = r0 + lb;
  const int rl = pl.N - 1;
  const float4 ga = f4_keep(
      ra < pl.N, f4_ld(a.g + (size_t)min(ra, rl) * a.ldg + 4 * q));
  const float4 gb = f4_keep(
      rb < pl.N, f4_ld(a.g + (size_t)min(rb, rl) * a.ldg + 4 * q));
  const float4 xa = f4_keep(ra < pl.N, f4_ld(a.x.row(min(ra, rl)) + 4 * q));
  const float4 xb = f4_keep(rb < pl.N, f4_ld(a.x.row(min(rb, rl)) + 4 * q));
  float4 wv[3];
  rc_load_w(a.w, wv);
  int hp, hs;
  rc_load_heads(pl, r0, hp, hs);
  rc_store_w<false>(wv, sW);
  rc_zero_rows<16>(sG, kRcP);                            // t_in / t_out := 0
  rc_stage_lists<true>(pl, r0, s, hp, hs);
  const RcRows gsrc{a.g, a.g, 0, a.ldg, a.ldg};
  rc_gather_flat<true, false, false, 12>(pl, s, gsrc, sG, kRcP, fl);
  lds_put4(sG + la * kRcP + 2 * kRcC + 4 * q, ga);
  lds_put4(sG + lb * kRcP + 2 * kRcC + 4 * q, gb);
  lds_put4a(sX + la * kRcXP + 4 * q, xa);
  lds_put4a(sX + lb * kRcXP + 4 * q, xb);
  __syncthreads();
  const int i = lane & 15, kk = lane >> 4;
  // dx[16 rows][32] = G W_stack
  {
    rc_f32x4 o0 = {0.f, 0.f, 0.f, 0.f}, o1 = {0.f, 0.f, 0.f, 0.f};
    const DGMC_LDS float* grow = sG + (wave * 16 + i) * kRcP + kk;
#pragma unroll 8
    for (int k0 = 0; k0 < 3 * kRcC; k0 += 4) {
      const float av = grow[k0];
      o0 = __builtin_amdgcn_mfma_f32_16x16x4f32(
          av, sW[i * kRcP + k0 + kk], o0, 0, 0, 0);
      o1 = __builtin_amdgcn_mfma_f32_16x16x4f32(
          av, sW[(16 + i) * kRcP + k0 + kk], o1, 0, 0, 0);
    }
    float dv[2][4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    if (a.dadd) {                                  // (uniform)
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int r = min(r0 + wave * 16 + kk * 4 + rr, rl);
          dv[h][rr] = a.dadd[(size_t)r * a.ldadd + 16 * h + i];
        }
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int k = 16 * h + i;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int lr = wave * 16 + kk * 4 + rr;
        const int r = r0 + lr;
        if (r < pl.N && r >= a.row0) {
          float v = (h ? o1[rr] : o0[rr]) + dv[h][rr];
          if (a.mask && !(sX[lr * kRcXP + k] > 0.f)) v = 0.f;
          a.dout[(size_t)(r - a.row0) * a.lddo + k] = v;
        }
      }
    }
  }
  // dW_stack partial [96][32] = G^T X over the tile's rows; wave w: output
  // blocks 3w .. 3w + 2 of the 6 x 2 grid.  Results go through LDS (sG's
  // space is free once every wave passed the barrier) so the partial is
  // written (and added to the earlier uses' values) by linear threads.
  rc_f32x4 d[3];
#pragma unroll
  for (int bb = 0; bb < 3; ++bb) {
    const int blk = 3 * wave + bb, mb = blk >> 1, nb = blk & 1;
    d[bb] = rc_f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
    for (int j0 = 0; j0 < kRcRows; j0 += 4) {
      const float av = sG[(j0 + kk) * kRcP + mb * 16 + i];
      const float bv = sX[(j0 + kk) * kRcXP + nb * 16 + i];
      d[bb] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, d[bb], 0, 0, 0);
    }
  }
  float dbias = 0.f;
  if (tid < kRcC)
    for (int j = 0; j < kRcRows; ++j) dbias += sG[j * kRcP + 2 * kRcC + tid];
  __syncthreads();
  DGMC_LDS float* sP = sG;                           // [kRcPart] staging
#pragma unroll
  for (int bb = 0; bb < 3; ++bb) {
    const int blk = 3 * wave + bb, mb = blk >> 1, nb = blk & 1;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr)
      sP[(mb * 16 + kk * 4 + rr) * kRcK + nb * 16 + i] = d[bb][rr];
  }
  if (tid < kRcC) sP[3 * kRcC * kRcK + tid] = dbias;
  __syncthreads();
#pragma unroll
  for (int u = 0; u < kRcPartPer; ++u) {
    const int t = tid + 256 * u;
    if (t < kRcPart) part[t] = old[u] + sP[t];
  }
}

// ---------------------------------------------------------------------------
// Projection backward: dfeat = dPQ fold (the last 32 columns masked by
// feat > 0: they are the last layer's g'), dfold partial += dPQ^T feat.
// LDS: sD [64][kRcDP], sFo [32][kRcFT] (fold), sF [64][kRcFT].
// ---------------------------------------------------------------------------
constexpr int kRcPbLds =
    (kRcRows * kRcDP + 32 * kRcFT + kRcRows * kRcFT) * 4;

__global__ __launch_bounds__(256) void rel_proj_bwd_kernel(
    const float* __restrict__ dpq, const float* __restrict__ feat, int ldf,
    const float* __restrict__ fold, float* __restrict__ dfeat, int lddf,
    float* __restrict__ part, int part_acc, int N) {
  extern __shared__ __attribute__((aligned(16))) float rc_smem[];
  DGMC_LDS float* sD = (DGMC_LDS float*)rc_smem;
  DGMC_LDS float* sFo = sD + kRcRows * kRcDP;
  DGMC_LDS float* sF = sFo + 32 * kRcFT;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r0 = blockIdx.x * kRcRows;
  float* pp = part + (size_t)blockIdx.x * (32 * 128);
  float old[16];
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    const float v = pp[tid + 256 * u];
    old[u] = part_acc ? v : 0.f;
  }
  float4 dv[2], fv[8], wv[4];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int t = tid + 256 * u, r = r0 + (t >> 3);
    dv[u] = f4_keep(r < N,
                    f4_ld(dpq + (size_t)min(r, N - 1) * 32 + (t & 7) * 4));
  }
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int t = tid + 256 * u, r = r0 + (t >> 5);
    fv[u] = f4_keep(r < N,
                    f4_ld(feat + (size_t)min(r, N - 1) * ldf + (t & 31) * 4));
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) wv[u] = f4_ld(fold + 4 * (tid + 256 * u));
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int t = tid + 256 * u;
    DGMC_LDS float* p = sD + (t >> 3) * kRcDP + (t & 7) * 4;
    p[0] = dv[u].x; p[1] = dv[u].y; p[2] = dv[u].z; p[3] = dv[u].w;
  }
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int t = tid + 256 * u;
    lds_put4a(sF + (t >> 5) * kRcFT + (t & 31) * 4, fv[u]);
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int t = 4 * (tid + 256 * u);       // fold[c'][k .. k + 3]
    lds_put4a(sFo + (t >> 7) * kRcFT + (t & 127), wv[u]);
  }
  __syncthreads();
  const int i = lane & 15, kk = lane >> 4;
  // dfeat[16 rows of wave][128] = dPQ fold: 8 column blocks, K = 32
  {
    const DGMC_LDS float* drow = sD + (wave * 16 + i) * kRcDP + kk;
    float a8[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) a8[s] = drow[4 * s];
#pragma unroll
    for (int nb = 0; nb < 8; ++nb) {
      rc_f32x4 o = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 8; ++s)
        o = __builtin_amdgcn_mfma_f32_16x16x4f32(
            a8[s], sFo[(4 * s + kk) * kRcFT + nb * 16 + i], o, 0, 0, 0);
      const int c = nb * 16 + i;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int lr = wave * 16 + kk * 4 + rr, r = r0 + lr;
        float v = o[rr];
        if (c >= 96 && !(sF[lr * kRcFT + c] > 0.f)) v = 0.f;
        if (r < N) dfeat[(size_t)r * lddf + c] = v;
      }
    }
  }
  // dfold partial [32][128] = dPQ^T feat: 2 x 8 blocks, 4 per wave
  rc_f32x4 d[4];
#pragma unroll
  for (int bb = 0; bb < 4; ++bb) {
    const int blk = 4 * wave + bb, mb = blk >> 3, nb = blk & 7;
    d[bb] = rc_f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
    for (int j0 = 0; j0 < kRcRows; j0 += 4)
      d[bb] = __builtin_amdgcn_mfma_f32_16x16x4f32(
          sD[(j0 + kk) * kRcDP + mb * 16 + i],
          sF[(j0 + kk) * kRcFT + nb * 16 + i], d[bb], 0, 0, 0);
  }
  __syncthreads();
  DGMC_LDS float* sP = sF;                           // [32][128] staging
#pragma unroll
  for (int bb = 0; bb < 4; ++bb) {
    const int blk = 4 * wave + bb, mb = blk >> 3, nb = blk & 7;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr)
      sP[(mb * 16 + kk * 4 + rr) * 128 + nb * 16 + i] = d[bb][rr];
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    const int t = tid + 256 * u;
    pp[t] = old[u] + sP[t];
  }
}

// Fold of per-tile partials: dst[z][c] = sum_{r in block rows} src[z][r][c]
// for up to 4 buffers (blockIdx.z); rows summed in order, 8 loads in flight.
struct RcFold {
  const float* src[4];
  float* dst[4];
  int cols[4];
};

__global__ __launch_bounds__(256) void rel_fold_kernel(RcFold f, int rows,
                                                       int rows_per_block) {
  const int z = blockIdx.z;
  const int c = blockIdx.x * 256 + threadIdx.x;
  const int C = f.cols[z];
  if (c >= C) return;
  const int r0 = blockIdx.y * rows_per_block;
  const int r1 = min(rows, r0 + rows_per_block);
  const float* src = f.src[z] + c;
  float acc = 0.f;
  int r = r0;
  for (; r + 8 <= r1; r += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = src[(size_t)(r + u) * C];
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += v[u];
  }
  for (; r < r1; ++r) acc += src[(size_t)r * C];
  f.dst[z][(size_t)blockIdx.y * C + c] = acc;
}

// Backward of the folded projection fold = W1 W_f (models/dgmc.py): from
// its gradient g [R, K]: gw1 = g W_f^T [R, Kin], gwf = W1^T g [Kin, K].
// One output per thread over the staged (L1 / L2-resident) operands, four
// interleaved fmaf chains (k mod 4) summed in a fixed order: four times
// the latency-bound chain's throughput at R = 128, K = 384 (PascalVOC).
__global__ __launch_bounds__(256) void fold_weights_bwd_kernel(
    const float* __restrict__ w1, const float* __restrict__ wf,
    const float* __restrict__ g, float* __restrict__ gw1,
    float* __restrict__ gwf, int R, int Kin, int K, int nb1) {
  if ((int)blockIdx.x < nb1) {
    const int t = blockIdx.x * 256 + threadIdx.x;
    if (t >= R * Kin) return;
    const int r = t / Kin, m = t % Kin;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
#pragma unroll 8
    for (int k = 0; k < K; k += 4) {
      const float4 a = f4_ld(g + (size_t)r * K + k);
      const float4 b = f4_ld(wf + (size_t)m * K + k);
      s0 = fmaf(a.x, b.x, s0); s1 = fmaf(a.y, b.y, s1);
      s2 = fmaf(a.z, b.z, s2); s3 = fmaf(a.w, b.w, s3);
    }
    gw1[t] = (s0 + s1) + (s2 + s3);
    return;
  }
  const int t = (blockIdx.x - nb1) * 256 + threadIdx.x;
  if (t >= Kin * K) return;
  const int m = t / K, k = t % K;
  float s[4] = {0.f, 0.f, 0.f, 0.f};
  int r = 0;
#pragma unroll 4
  for (; r + 4 <= R; r += 4)
#pragma unroll
    for (int u = 0; u < 4; ++u)
      s[u] = fmaf(w1[(r + u) * Kin + m], g[(size_t)(r + u) * K + k], s[u]);
  for (; r < R; ++r) s[0] = fmaf(w1[r * Kin + m], g[(size_t)r * K + k], s[0]);
  gwf[t] = (s[0] + s[1]) + (s[2] + s[3]);
}

RcPlan make_plan(const at::Tensor& ptr, const at::Tensor& col,
                 const at::Tensor& split, const c10::optional<at::Tensor>& w,
                 const at::Tensor& hub) {
  const int64_t N = ptr.numel() - 1;
  TORCH_CHECK(ptr.scalar_type() == at::kInt && col.scalar_type() == at::kInt &&
                  split.scalar_type() == at::kInt,
              "rel plan: int32 CSR arrays");
  TORCH_CHECK(hub.scalar_type() == at::kByte && hub.numel() == N &&
                  split.numel() == N,
              "rel plan: uint8 hub flags / int32 splits [N]");
  for (const at::Tensor* t : {&ptr, &col, &split, &hub})
    TORCH_CHECK(t->is_cuda() && t->is_contiguous(), "rel plan: contiguous "
                "device tensors");
  TORCH_CHECK(N > 0 && N < (1 << 24) && col.numel() > 0,
              "rel plan: 1 .. 2^24 - 1 rows and a trailing dummy list entry "
              "(ops/relconv.py RelPlan)");
  const float* wp = nullptr;
  if (w.has_value() && w->defined()) {
    TORCH_CHECK(w->scalar_type() == at::kFloat && w->is_contiguous() &&
                    w->numel() == col.numel(),
                "rel plan: fp32 entry weights [nnz]");
    wp = w->data_ptr<float>();
  }
  return RcPlan{ptr.data_ptr<int>(), col.data_ptr<int>(),
                split.data_ptr<int>(), wp, hub.data_ptr<unsigned char>(),
                (int)N};
}

void check_rows(const at::Tensor& t, int64_t rows, int64_t cols,
                const char* what) {
  TORCH_CHECK(rows * std::max<int64_t>(t.stride(0), cols) < (int64_t(1) << 31),
              what, ": rows * row stride must stay below 2^31");
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.dim() == 2 &&
                  t.size(0) == rows && t.size(1) == cols && t.stride(1) == 1 &&
                  t.stride(0) % 4 == 0 && aligned16(t.data_ptr()),
              what, ": fp32 [", rows, ", ", cols,
              "] rows with unit column stride and 16-byte aligned rows");
}

RcRows make_rows(const at::Tensor& xa, const c10::optional<at::Tensor>& xb,
                 int64_t N) {
  if (xb.has_value() && xb->defined()) {
    const int64_t split = xa.size(0);
    check_rows(xa, split, kRcK, "relconv x (first part)");
    check_rows(*xb, N - split, kRcK, "relconv x (second part)");
    return RcRows{xa.data_ptr<float>(), xb->data_ptr<float>(), (int)split,
                  (int)xa.stride(0), (int)xb->stride(0)};
  }
  check_rows(xa, N, kRcK, "relconv x");
  return RcRows{xa.data_ptr<float>(), xa.data_ptr<float>(), (int)N,
                (int)xa.stride(0), (int)xa.stride(0)};
}

void check_w(const at::Tensor& w, int64_t rows, int64_t cols) {
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kFloat &&
                  w.is_contiguous() && w.dim() == 2 && w.size(0) == rows &&
                  w.size(1) == cols,
              "relconv: contiguous fp32 weight [", rows, ", ", cols, "]");
}

}  // namespace

constexpr int64_t kRcPartSize = kRcPart;

// out = act([mean_in x | mean_out x | x] [W1 | W2 | Wr]^T + b) into `out`
// (a [N, 32] view with 16-byte rows); optional copy of the input rows into
// `xcopy` and, with `fold`, the fused consensus projection
// pq = [feat[:, 0:96] | out] fold^T.  (ptr, col, split): the forward joint
// lists (row i: in-neighbours, then out-neighbours from split[i]).
void relconv_fwd(const at::Tensor& ptr, const at::Tensor& col,
                 const at::Tensor& split, const at::Tensor& hub,
                 const at::Tensor& xa, const c10::optional<at::Tensor>& xb,
                 const at::Tensor& w1, const at::Tensor& w2,
                 const at::Tensor& wr, const at::Tensor& bias, bool relu,
                 at::Tensor out, const c10::optional<at::Tensor>& xcopy,
                 const c10::optional<at::Tensor>& feat,
                 const c10::optional<at::Tensor>& fold,
                 const c10::optional<at::Tensor>& pq) {
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(xa.device());
  RcPlan pl = make_plan(ptr, col, split, c10::nullopt, hub);
  const int64_t N = pl.N;
  RcFwd a{};
  a.x = make_rows(xa, xb, N);
  check_w(w1, kRcC, kRcK);
  check_w(w2, kRcC, kRcK);
  check_w(wr, kRcC, kRcK);
  TORCH_CHECK(bias.is_cuda() && bias.scalar_type() == at::kFloat &&
                  bias.is_contiguous() && bias.numel() == kRcC,
              "relconv: fp32 bias [32]");
  a.w[0] = w1.data_ptr<float>();
  a.w[1] = w2.data_ptr<float>();
  a.w[2] = wr.data_ptr<float>();
  a.bias = bias.data_ptr<float>();
  check_rows(out, N, kRcC, "relconv out");
  a.out = out.data_ptr<float>();
  a.ldo = (int)out.stride(0);
  if (xcopy.has_value() && xcopy->defined()) {
    check_rows(*xcopy, N, kRcK, "relconv xcopy");
    a.xcopy = xcopy->data_ptr<float>();
    a.ldxc = (int)xcopy->stride(0);
  }
  a.relu = relu ? 1 : 0;
  const bool proj = fold.has_value() && fold->defined();
  if (proj) {
    TORCH_CHECK(feat.has_value() && feat->defined() && pq.has_value() &&
                    pq->defined(),
                "relconv: the projection needs feat, fold and pq");
    check_rows(*feat, N, 96, "relconv feat[:, 0:96]");
    check_w(*fold, 32, 128);
    check_rows(*pq, N, 32, "relconv pq");
    TORCH_CHECK(pq->is_contiguous(), "relconv: contiguous pq");
    a.feat = feat->data_ptr<float>();
    a.ldf = (int)feat->stride(0);
    a.fold = fold->data_ptr<float>();
    a.pq = pq->data_ptr<float>();
  }
  const int n_tiles = (int)((N + kRcRows - 1) / kRcRows);
  if (n_tiles == 0) return;
  const bool two = xb.has_value() && xb->defined();   // [x_s; x_t] split
  auto kern = proj ? (two ? relconv_fwd_kernel<true, true>
                          : relconv_fwd_kernel<true, false>)
                   : (two ? relconv_fwd_kernel<false, true>
                          : relconv_fwd_kernel<false, false>);
  const int lds = proj ? kRcFwdProjLds : kRcFwdLds;
  DGMC_CHECK_HIP(hipFuncSetAttribute(
      reinterpret_cast<const void*>(kern),
      hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  hipLaunchKernelGGL(kern, dim3(n_tiles), dim3(256), lds, stream(), pl, a);
  DGMC_CHECK_LAUNCH();
}

// Backward of one layer: dout[j - row0] = mask(dadd_j + (G W_stack)_j) for
// j >= row0; part[tile] (+)= [G^T x | sum g'] per 64-row tile.  (ptr, col,
// w, split): the backward joint lists (row j: out-neighbours weighted
// 1 / deg_in, then in-neighbours weighted 1 / deg_out from split[j]).
void relconv_bwd(const at::Tensor& ptr, const at::Tensor& col,
                 const at::Tensor& w, const at::Tensor& split,
                 const at::Tensor& hub, const at::Tensor& g,
                 const at::Tensor& xa, const c10::optional<at::Tensor>& xb,
                 const at::Tensor& w1, const at::Tensor& w2,
                 const at::Tensor& wr, const c10::optional<at::Tensor>& dadd,
                 at::Tensor dout, int64_t row0, bool mask, at::Tensor part,
                 bool part_acc) {
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(g.device());
  RcPlan pl = make_plan(ptr, col, split, w, hub);
  const int64_t N = pl.N;
  RcBwd a{};
  check_rows(g, N, kRcC, "relconv g");
  a.g = g.data_ptr<float>();
  a.ldg = (int)g.stride(0);
  a.x = make_rows(xa, xb, N);
  check_w(w1, kRcC, kRcK);
  check_w(w2, kRcC, kRcK);
  check_w(wr, kRcC, kRcK);
  a.w[0] = w1.data_ptr<float>();
  a.w[1] = w2.data_ptr<float>();
  a.w[2] = wr.data_ptr<float>();
  if (dadd.has_value() && dadd->defined()) {
    check_rows(*dadd, N, kRcK, "relconv dadd");
    a.dadd = dadd->data_ptr<float>();
    a.ldadd = (int)dadd->stride(0);
  }
  TORCH_CHECK(row0 >= 0 && row0 <= N, "relconv: 0 <= row0 <= N");
  check_rows(dout, N - row0, kRcK, "relconv dout");
  a.dout = dout.data_ptr<float>();
  a.lddo = (int)dout.stride(0);
  a.row0 = (int)row0;
  a.mask = mask ? 1 : 0;
  const int n_tiles = (int)((N + kRcRows - 1) / kRcRows);
  TORCH_CHECK(part.is_cuda() && part.scalar_type() == at::kFloat &&
                  part.is_contiguous() &&
                  part.numel() == (int64_t)n_tiles * kRcPart,
              "relconv: part [n_tiles, ", kRcPartSize, "]");
  a.part = part.data_ptr<float>();
  a.part_acc = part_acc ? 1 : 0;
  if (n_tiles == 0) return;
  DGMC_CHECK_HIP(hipFuncSetAttribute(
      reinterpret_cast<const void*>(relconv_bwd_kernel),
      hipFuncAttributeMaxDynamicSharedMemorySize, kRcBwdLds));
  hipLaunchKernelGGL(relconv_bwd_kernel, dim3(n_tiles), dim3(256), kRcBwdLds,
                     stream(), pl, a);
  DGMC_CHECK_LAUNCH();
}

void rel_proj_bwd(const at::Tensor& dpq, const at::Tensor& feat,
                  const at::Tensor& fold, at::Tensor dfeat, at::Tensor part,
                  bool part_acc) {
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(dpq.device());
  const int64_t N = dpq.size(0);
  check_rows(dpq, N, 32, "rel_proj_bwd dpq");
  TORCH_CHECK(dpq.is_contiguous(), "rel_proj_bwd: contiguous dpq");
  check_rows(feat, N, 128, "rel_proj_bwd feat");
  check_rows(dfeat, N, 128, "rel_proj_bwd dfeat");
  check_w(fold, 32, 128);
  const int n_tiles = (int)((N + kRcRows - 1) / kRcRows);
  TORCH_CHECK(part.is_cuda() && part.scalar_type() == at::kFloat &&
                  part.is_contiguous() &&
                  part.numel() == (int64_t)n_tiles * 32 * 128,
              "rel_proj_bwd: part [n_tiles, 4096]");
  if (n_tiles == 0) return;
  DGMC_CHECK_HIP(hipFuncSetAttribute(
      reinterpret_cast<const void*>(rel_proj_bwd_kernel),
      hipFuncAttributeMaxDynamicSharedMemorySize, kRcPbLds));
  hipLaunchKernelGGL(rel_proj_bwd_kernel, dim3(n_tiles), dim3(256), kRcPbLds,
                     stream(), dpq.data_ptr<float>(), feat.data_ptr<float>(),
                     (int)feat.stride(0), fold.data_ptr<float>(),
                     dfeat.data_ptr<float>(), (int)dfeat.stride(0),
                     part.data_ptr<float>(), part_acc ? 1 : 0, (int)N);
  DGMC_CHECK_LAUNCH();
}

// outs[z] = column sums of parts[z] ([rows, cols_z], all with the same row
// count): two fixed-order stages (blocks of 16 rows, then their sums).
void rel_fold(at::TensorList parts, at::TensorList outs) {
  const int64_t nb = (int64_t)parts.size();
  TORCH_CHECK(nb >= 1 && nb <= 4 && (int64_t)outs.size() == nb,
              "rel_fold: 1..4 buffers");
  const int64_t rows = parts[0].size(0);
  int64_t maxc = 0;
  for (int64_t z = 0; z < nb; ++z) {
    TORCH_CHECK(parts[z].is_cuda() && parts[z].scalar_type() == at::kFloat &&
                    parts[z].is_contiguous() && parts[z].dim() == 2 &&
                    parts[z].size(0) == rows,
                "rel_fold: contiguous fp32 [rows, cols] partials");
    TORCH_CHECK(outs[z].scalar_type() == at::kFloat &&
                    outs[z].is_contiguous() &&
                    outs[z].numel() == parts[z].size(1),
                "rel_fold: contiguous fp32 [cols] outputs");
    maxc = std::max<int64_t>(maxc, parts[z].size(1));
  }
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(parts[0].device());
  if (rows == 0 || maxc == 0) {
    for (int64_t z = 0; z < nb; ++z) at::Tensor(outs[z]).zero_();
    return;
  }
  constexpr int kRpb = 16;
  const int64_t nby = (rows + kRpb - 1) / kRpb;
  std::vector<at::Tensor> tmp;
  RcFold f1{}, f2{};
  for (int64_t z = 0; z < nb; ++z) {
    tmp.push_back(at::empty({nby, parts[z].size(1)}, parts[z].options()));
    f1.src[z] = parts[z].data_ptr<float>();
    f1.dst[z] = tmp[z].data_ptr<float>();
    f1.cols[z] = (int)parts[z].size(1);
    f2.src[z] = tmp[z].data_ptr<float>();
    f2.dst[z] = outs[z].data_ptr<float>();
    f2.cols[z] = f1.cols[z];
  }
  const unsigned gx = (unsigned)((maxc + 255) / 256);
  hipLaunchKernelGGL(rel_fold_kernel, dim3(gx, (unsigned)nby, (unsigned)nb),
                     dim3(256), 0, stream(), f1, (int)rows, kRpb);
  DGMC_CHECK_LAUNCH();
  hipLaunchKernelGGL(rel_fold_kernel, dim3(gx, 1, (unsigned)nb), dim3(256), 0,
                     stream(), f2, (int)nby, (int)nby);
  DGMC_CHECK_LAUNCH();
}

std::tuple<at::Tensor, at::Tensor> fold_weights_bwd(const at::Tensor& w1,
                                                    const at::Tensor& wf,
                                                    const at::Tensor& g) {
  TORCH_CHECK(w1.is_cuda() && w1.scalar_type() == at::kFloat &&
                  wf.scalar_type() == at::kFloat &&
                  g.scalar_type() == at::kFloat && w1.is_contiguous() &&
                  wf.is_contiguous() && g.is_contiguous() && w1.dim() == 2 &&
                  wf.dim() == 2 && g.dim() == 2 && w1.size(1) == wf.size(0) &&
                  g.size(0) == w1.size(0) && g.size(1) == wf.size(1) &&
                  wf.size(1) % 4 == 0 && aligned16(g.data_ptr()) &&
                  aligned16(wf.data_ptr()),
              "fold_weights_bwd: fp32 W1 [R, Kin], W_f [Kin, K % 4], "
              "g [R, K]");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(w1.device());
  at::Tensor gw1 = at::empty_like(w1), gwf = at::empty_like(wf);
  const int64_t n1 = w1.numel(), n2 = wf.numel();
  if (n1 + n2 == 0) return {gw1, gwf};
  const int nb1 = (int)((n1 + 255) / 256), nb2 = (int)((n2 + 255) / 256);
  hipLaunchKernelGGL(fold_weights_bwd_kernel, dim3(nb1 + nb2), dim3(256), 0,
                     stream(), w1.data_ptr<float>(), wf.data_ptr<float>(),
                     g.data_ptr<float>(), gw1.data_ptr<float>(),
                     gwf.data_ptr<float>(), (int)w1.size(0), (int)w1.size(1),
                     (int)wf.size(1), nb1);
  DGMC_CHECK_LAUNCH();
  return {gw1, gwf};
}

}  // namespace dgmc
