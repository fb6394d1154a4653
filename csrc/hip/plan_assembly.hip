// Per-step assembly of a static pair batch's slot-structured sparse operator
// (SplineConv's A and A^T, ops/plans.py::spline_plan) from per-graph pieces.
//
// Every graph of a GraphStore has fixed edges and pseudo-coordinates, so its
// spline operator (basis / in-degree per (edge, slot), root diagonal) never
// changes.  It is built ONCE for the whole store (block-diagonal CSR, rows of
// graph g contiguous, entries of graph g contiguous, both for A and A^T).  A
// batch's operator is the block-diagonal concatenation of its graphs' blocks
// with renumbered rows/columns, so instead of rebuilding it per step (basis,
// degree, two stable sorts and scans: ~100 small launches per step in the
// reference-style path) one launch copies the pieces:
//
//   segment k < B          source graph gid[k]  at node offset ptr_s[k]
//   segment B              source padding rows  [ptr_s[B], cap_s)
//   segment B + 1 + b      target graph gid[B+b] at cap_s + ptr_t[b]
//   segment 2B + 1         target padding rows  [cap_s + ptr_t[B], cap_s+cap_t)
//
// One workgroup per segment: it derives its entry offset from the segment
// sizes (a block reduction over the preceding segments - no separate scan
// launch), then copies row pointers, columns (renumbered) and values of A and
// A^T.  Padding rows get only their root entry (their outputs are never read
// by valid rows: no entry of a valid row points at a padding node).
// Identical entry order to spline_plan (edge order, slot, then root) => the
// SpMM results on valid rows are bitwise identical to the per-step build.
#include "common.h"

namespace dgmc {

constexpr int kAsmThreads = 256;

struct SegInfo {
  int64_t gid;    // store graph id, -1 = padding
  int64_t off;    // first batch node
  int64_t n;      // nodes
};

__device__ __forceinline__ SegInfo segment(int k, const int64_t* gid,
                                           const int64_t* ptr_s,
                                           const int64_t* ptr_t, int B,
                                           int64_t cap_s, int64_t cap_t) {
  SegInfo s;
  if (k < B) {
    s.gid = gid[k]; s.off = ptr_s[k]; s.n = ptr_s[k + 1] - ptr_s[k];
  } else if (k == B) {
    s.gid = -1; s.off = ptr_s[B]; s.n = cap_s - ptr_s[B];
  } else if (k < 2 * B + 1) {
    const int b = k - B - 1;
    s.gid = gid[B + b]; s.off = cap_s + ptr_t[b]; s.n = ptr_t[b + 1] - ptr_t[b];
  } else {
    s.gid = -1; s.off = cap_s + ptr_t[B]; s.n = cap_t - ptr_t[B];
  }
  return s;
}

__global__ __launch_bounds__(kAsmThreads) void assemble_slot_plan_kernel(
    const int* __restrict__ st_rowptr, const int* __restrict__ st_col,
    const float* __restrict__ st_val, const int* __restrict__ st_trowptr,
    const int* __restrict__ st_tcol, const float* __restrict__ st_tval,
    const int64_t* __restrict__ node_ptr, const int64_t* __restrict__ gid,
    const int64_t* __restrict__ ptr_s, const int64_t* __restrict__ ptr_t,
    int B, int64_t cap_s, int64_t cap_t, int S, int root_slot, int64_t cap,
    int* __restrict__ rowptr, int* __restrict__ col, float* __restrict__ val,
    int* __restrict__ trowptr, int* __restrict__ tcol,
    float* __restrict__ tval, uint8_t* __restrict__ gflag,
    const int64_t* __restrict__ st_row, int64_t* __restrict__ row_out) {
  __shared__ int64_t red[kAsmThreads / kWave];
  const int k = blockIdx.x;
  const int tid = threadIdx.x;
  const bool root = root_slot >= 0;
  auto seg_nnz = [&](int kk) -> int64_t {
    const SegInfo s = segment(kk, gid, ptr_s, ptr_t, B, cap_s, cap_t);
    if (s.gid < 0) return root ? s.n : 0;
    return (int64_t)st_rowptr[node_ptr[s.gid + 1]] - st_rowptr[node_ptr[s.gid]];
  };
  // Entry offset of this segment = sum of the preceding segments' sizes.
  int64_t part = 0;
  for (int kk = tid; kk < k; kk += kAsmThreads) part += seg_nnz(kk);
#pragma unroll
  for (int o = kWave / 2; o > 0; o >>= 1) part += __shfl_xor(part, o);
  if (tid % kWave == 0) red[tid / kWave] = part;
  __syncthreads();
  int64_t eo = 0;
#pragma unroll
  for (int w = 0; w < kAsmThreads / kWave; ++w) eo += red[w];

  const SegInfo s = segment(k, gid, ptr_s, ptr_t, B, cap_s, cap_t);
  if (gflag) {
    // Graph-start flags (the tiling of csrc/hip/slot_conv.hip): a graph's
    // first row, and every padding row (padding rows form 1-node graphs).
    for (int64_t r = tid; r < s.n; r += kAsmThreads)
      gflag[s.off + r] = (s.gid < 0 || r == 0) ? 1 : 0;
  }
  if (s.gid >= 0) {
    const int64_t n0 = node_ptr[s.gid];
    const int r0 = st_rowptr[n0];
    const int nnz = st_rowptr[n0 + s.n] - r0;
    const int t0 = st_trowptr[n0 * S];
    for (int64_t r = tid; r < s.n; r += kAsmThreads)
      rowptr[s.off + r] = (int)(eo + st_rowptr[n0 + r] - r0);
    for (int64_t q = tid; q < s.n * S; q += kAsmThreads)
      trowptr[s.off * S + q] = (int)(eo + st_trowptr[n0 * S + q] - t0);
    const int64_t dcol = (s.off - n0) * S, dt = s.off - n0;
    for (int e = tid; e < nnz; e += kAsmThreads) {
      col[eo + e] = (int)(st_col[r0 + e] + dcol);
      val[eo + e] = st_val[r0 + e];
      tcol[eo + e] = (int)(st_tcol[t0 + e] + dt);
      tval[eo + e] = st_tval[t0 + e];
      // Row of every entry (the slot weight gradient's pair lists need it;
      // otherwise a searchsorted over rowptr per step).
      if (row_out) row_out[eo + e] = st_row[r0 + e] + dt;
    }
  } else {
    // Padding rows: root entry only (or nothing without a root weight).
    for (int64_t r = tid; r < s.n; r += kAsmThreads) {
      const int64_t node = s.off + r;
      rowptr[node] = (int)(eo + (root ? r : 0));
      if (root) {
        col[eo + r] = (int)(node * S + root_slot);
        val[eo + r] = 1.f;
        tcol[eo + r] = (int)node;
        tval[eo + r] = 1.f;
        if (row_out) row_out[eo + r] = node;
      }
    }
    for (int64_t q = tid; q < s.n * S; q += kAsmThreads) {
      const int64_t r = q / S, slot = q - r * S;
      trowptr[s.off * S + q] =
          (int)(eo + (root ? r + (slot > root_slot ? 1 : 0) : 0));
    }
  }
  if (k == gridDim.x - 1) {
    // Totals, and an inert tail: entries past the total (left over from a
    // larger batch) become (col 0, val 0) so the fixed-capacity entry arrays
    // stay a valid operator for consumers that read all of them.
    const int64_t total = eo + seg_nnz(k);
    if (tid == 0) {
      rowptr[cap_s + cap_t] = (int)total;
      trowptr[(cap_s + cap_t) * S] = (int)total;
    }
    for (int64_t e = total + tid; e < cap; e += kAsmThreads) {
      col[e] = 0;
      val[e] = 0.f;
      tcol[e] = 0;
      tval[e] = 0.f;
    }
  }
}

// buf: the static batch's int64 index buffer views (gid [2B], ptr_s/ptr_t
// [B+1]); store operator (A, A^T) in int32/fp32 CSR; outputs preallocated
// (rowptr [N+1], col/val [cap], trowptr [N*S+1], tcol/tval [cap]).
void assemble_slot_plan(const at::Tensor& st_rowptr, const at::Tensor& st_col,
                        const at::Tensor& st_val, const at::Tensor& st_trowptr,
                        const at::Tensor& st_tcol, const at::Tensor& st_tval,
                        const at::Tensor& node_ptr, const at::Tensor& gid,
                        const at::Tensor& ptr_s, const at::Tensor& ptr_t,
                        int64_t cap_s, int64_t cap_t, int64_t S,
                        int64_t root_slot, at::Tensor rowptr, at::Tensor col,
                        at::Tensor val, at::Tensor trowptr, at::Tensor tcol,
                        at::Tensor tval,
                        const c10::optional<at::Tensor>& gflag,
                        const c10::optional<at::Tensor>& st_row,
                        const c10::optional<at::Tensor>& row_out) {
  for (const at::Tensor* t : std::initializer_list<const at::Tensor*>{
           &st_rowptr, &st_col, &st_trowptr, &st_tcol, &rowptr, &col,
           &trowptr, &tcol})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kInt &&
                    t->is_contiguous(),
                "assemble_slot_plan: int32 contiguous CUDA index tensors");
  for (const at::Tensor* t :
       std::initializer_list<const at::Tensor*>{&st_val, &st_tval, &val, &tval})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat &&
                    t->is_contiguous(),
                "assemble_slot_plan: fp32 contiguous CUDA value tensors");
  for (const at::Tensor* t : {&node_ptr, &gid, &ptr_s, &ptr_t})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kLong &&
                    t->is_contiguous(),
                "assemble_slot_plan: int64 contiguous CUDA batch tensors");
  const int64_t B = ptr_s.numel() - 1;
  TORCH_CHECK(B >= 1 && ptr_t.numel() == B + 1 && gid.numel() == 2 * B,
              "assemble_slot_plan: gid [2B], ptr_s/ptr_t [B+1]");
  const int64_t N = cap_s + cap_t;
  TORCH_CHECK(rowptr.numel() == N + 1 && trowptr.numel() == N * S + 1,
              "assemble_slot_plan: row pointer sizes");
  TORCH_CHECK(col.numel() == val.numel() && tcol.numel() == col.numel() &&
                  tval.numel() == col.numel(),
              "assemble_slot_plan: entry buffer sizes");
  TORCH_CHECK(st_trowptr.numel() == (st_rowptr.numel() - 1) * S + 1,
              "assemble_slot_plan: store operator shape");
  TORCH_CHECK(root_slot < S && N * S < INT32_MAX,
              "assemble_slot_plan: slot / size range");
  uint8_t* fp = nullptr;
  if (gflag.has_value() && gflag->defined()) {
    TORCH_CHECK(gflag->is_cuda() && gflag->scalar_type() == at::kByte &&
                    gflag->is_contiguous() && gflag->numel() >= N,
                "assemble_slot_plan: gflag uint8 [N]");
    fp = gflag->data_ptr<uint8_t>();
  }
  const int64_t* srp = nullptr;
  int64_t* rop = nullptr;
  if (row_out.has_value() && row_out->defined()) {
    TORCH_CHECK(st_row.has_value() && st_row->defined() &&
                    st_row->scalar_type() == at::kLong &&
                    st_row->is_contiguous() &&
                    st_row->numel() == st_col.numel() &&
                    row_out->scalar_type() == at::kLong &&
                    row_out->is_contiguous() &&
                    row_out->numel() == col.numel(),
                "assemble_slot_plan: int64 st_row [store nnz], row_out [cap]");
    srp = st_row->data_ptr<int64_t>();
    rop = row_out->data_ptr<int64_t>();
  }
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(col.device());
  hipLaunchKernelGGL(assemble_slot_plan_kernel, dim3(2 * B + 2),
                     dim3(kAsmThreads), 0, stream(), st_rowptr.data_ptr<int>(),
                     st_col.data_ptr<int>(), st_val.data_ptr<float>(),
                     st_trowptr.data_ptr<int>(), st_tcol.data_ptr<int>(),
                     st_tval.data_ptr<float>(), node_ptr.data_ptr<int64_t>(),
                     gid.data_ptr<int64_t>(), ptr_s.data_ptr<int64_t>(),
                     ptr_t.data_ptr<int64_t>(), (int)B, cap_s, cap_t, (int)S,
                     (int)root_slot, col.numel(), rowptr.data_ptr<int>(),
                     col.data_ptr<int>(), val.data_ptr<float>(),
                     trowptr.data_ptr<int>(), tcol.data_ptr<int>(),
                     tval.data_ptr<float>(), fp, srp, rop);
  DGMC_CHECK_LAUNCH();
}

}  // namespace dgmc
