// Fused column reductions and backward helpers.
//
// relu_bias_bwd: for an aggregation output `out = relu(A x + bias)` the
// backward needs g' = grad * (out > 0) for the transposed aggregation and
// dbias = sum_rows g'.  Eager PyTorch spends four kernels (compare, mul,
// column reduction, cast) plus one gradient-accumulation add per reuse of
// the bias; here: one pass writing g' and per-block fp32 column partials,
// then a small fold kernel into `dbias`, optionally accumulating into an
// existing fp32 buffer (the consensus loop reuses psi_2's biases ten times -
// see runtime/loopgrad.py).  Deterministic (fixed fold order).
//
// col_sum: the same machinery without the g' output (dst (+)= sum_rows src).
//
// reduce_add_rows: dst[n] (+)= sum_s src[s, n] - the split-K combine of the
// weight-gradient GEMMs, accumulating straight into the fp32 gradient.
#include "common.h"

namespace dgmc {

namespace {
// Partial rows folded by the 2nd kernel (keep in sync with
// ops/gemm.py::col_partial_rows, which sizes the callers' partial buffers).
// 1024: a [11k, 128] gradient gets one 16-row pass per block instead of ~6
// sequential passes at 1 wave per SIMD.
constexpr int kMaxColBlocks = 1024;
int max_col_blocks() { return kMaxColBlocks; }
}  // namespace

// NOTE (MI355X): a single-kernel "last block folds" reduction needs a
// device-scope release fence per block, which gfx950 lowers to
// `buffer_wbl2 sc1` - a write-back of the XCD's whole L2.  Measured: 76 us
// for a [9216, 128] column sum.  Two launches (partials, then a fold) cost
// ~2 us of extra launch latency inside a hipGraph instead.

// Stage 1.  LPR lanes own one row (VEC channels per pass); a block holds
// RPB = 256/LPR row slots and walks its row range, keeping channel partials
// in registers; the block partial goes through LDS to `part[block]`.
template <typename TG, typename TO, typename TR, int VEC, int LPR, bool WRITE_G>
__global__ __launch_bounds__(256) void colsum_kernel(
    const TG* __restrict__ grad, const TO* __restrict__ out,
    TR* __restrict__ g_out, float* __restrict__ part, int rows, int C,
    int64_t ldg, int relu) {
  constexpr int RPB = 256 / LPR;
  extern __shared__ __attribute__((aligned(16))) float lds[];  // [RPB][C]
  const int slot = threadIdx.x / LPR, lane = threadIdx.x % LPR;
  const int per = (rows + gridDim.x - 1) / gridDim.x;
  const int r0 = blockIdx.x * per, r1 = min(rows, r0 + per);
  for (int c0 = lane * VEC; c0 < C; c0 += LPR * VEC) {
    float acc[VEC];
#pragma unroll
    for (int k = 0; k < VEC; ++k) acc[k] = 0.f;
#pragma unroll 2
    for (int r = r0 + slot; r < r1; r += RPB) {
      const size_t o = (size_t)r * C + c0;
      float g[VEC], m[VEC];
      load_vec<TG, VEC>(grad + (size_t)r * ldg + c0, g);   // row stride ldg
      if (relu) {
        load_vec<TO, VEC>(out + o, m);
#pragma unroll
        for (int k = 0; k < VEC; ++k) g[k] = m[k] > 0.f ? g[k] : 0.f;
      }
#pragma unroll
      for (int k = 0; k < VEC; ++k) acc[k] += g[k];
      if constexpr (WRITE_G) {
        if constexpr (VEC * sizeof(TR) == 16) {
          store_vec<TR, VEC>(g_out + o, g);
        } else {
#pragma unroll
          for (int k = 0; k < VEC; ++k) g_out[o + k] = Cvt<TR>::from_f(g[k]);
        }
      }
    }
#pragma unroll
    for (int k = 0; k < VEC; ++k) lds[slot * C + c0 + k] = acc[k];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float s = 0.f;
    for (int q = 0; q < RPB; ++q) s += lds[q * C + c];
    part[(size_t)blockIdx.x * C + c] = s;
  }
}

// Stage 2.  dst[c] (+)= sum_r part[r, c]: block = 32 columns x 8 row groups,
// each thread keeps 8 loads in flight; LDS fold in fixed order
// (deterministic).
__global__ __launch_bounds__(256) void fold_rows_kernel(
    const float* __restrict__ part, float* __restrict__ dst, int nrows, int C,
    int accumulate) {
  __shared__ float lds[8][33];
  const int cl = threadIdx.x % 32, rg = threadIdx.x / 32;
  const int c = blockIdx.x * 32 + cl;
  float s = 0.f;
  if (c < C) {
#pragma unroll 8
    for (int r = rg; r < nrows; r += 8) s += part[(size_t)r * C + c];
  }
  lds[rg][cl] = s;
  __syncthreads();
  if (rg == 0 && c < C) {
    float t = accumulate ? dst[c] : 0.f;
#pragma unroll
    for (int g = 0; g < 8; ++g) t += lds[g][cl];
    dst[c] = t;
  }
}

template <typename TG, typename TO, typename TR, int VEC, int LPR, bool WRITE_G>
void launch_colsum(const at::Tensor& grad, const void* out, void* g,
                   at::Tensor& part, float* dst, int blocks, int rows, int C,
                   bool relu, bool accumulate) {
  constexpr int RPB = 256 / LPR;
  const size_t lds = (size_t)RPB * C * sizeof(float);
  hipLaunchKernelGGL((colsum_kernel<TG, TO, TR, VEC, LPR, WRITE_G>),
                     dim3(blocks), dim3(256), lds, stream(),
                     reinterpret_cast<const TG*>(grad.data_ptr()),
                     reinterpret_cast<const TO*>(out),
                     reinterpret_cast<TR*>(g), part.data_ptr<float>(), rows, C,
                     grad.stride(0), relu ? 1 : 0);
  if (dst)  // dst == nullptr: the caller keeps the per-block partials
    hipLaunchKernelGGL(fold_rows_kernel, dim3((C + 31) / 32), dim3(256), 0,
                       stream(), part.data_ptr<float>(), dst, blocks, C,
                       accumulate ? 1 : 0);
}

template <typename T, typename TR, bool WRITE_G>
void dispatch_colsum(const at::Tensor& grad, const void* out, void* g,
                     at::Tensor& part, float* dst, int blocks, int rows,
                     int C, bool relu, bool accumulate, bool vec) {
  constexpr int V = Vec16<T>::N;
  if (vec && C % V == 0) {
    const int lanes = C / V;
    if (lanes <= 8)
      launch_colsum<T, T, TR, V, 8, WRITE_G>(grad, out, g, part, dst, blocks,
                                             rows, C, relu, accumulate);
    else if (lanes <= 16)
      launch_colsum<T, T, TR, V, 16, WRITE_G>(grad, out, g, part, dst, blocks,
                                              rows, C, relu, accumulate);
    else if (lanes <= 32)
      launch_colsum<T, T, TR, V, 32, WRITE_G>(grad, out, g, part, dst, blocks,
                                              rows, C, relu, accumulate);
    else
      launch_colsum<T, T, TR, V, 64, WRITE_G>(grad, out, g, part, dst, blocks,
                                              rows, C, relu, accumulate);
  } else {
    launch_colsum<T, T, TR, 1, 64, WRITE_G>(grad, out, g, part, dst, blocks,
                                            rows, C, relu, accumulate);
  }
}

// Keep in sync with ops/gemm.py::col_partial_rows.
static int colsum_blocks(int rows) {
  return std::max(1, std::min((rows + 15) / 16, max_col_blocks()));
}

// Optional caller-owned partial buffer [blocks, C] fp32 (a loop-gradient
// stack slot): then only the partials are written and the fold is skipped.
static at::Tensor partials_or_new(const c10::optional<at::Tensor>& part_out,
                                  int blocks, int C, const at::Tensor& like,
                                  bool& keep) {
  keep = part_out.has_value() && part_out->defined();
  if (keep) {
    TORCH_CHECK(part_out->scalar_type() == at::kFloat &&
                    part_out->is_contiguous() &&
                    part_out->numel() == (int64_t)blocks * C,
                "colsum: part_out must be contiguous fp32 [", blocks, ", ", C,
                "]");
    return *part_out;
  }
  return at::empty({blocks, C}, like.options().dtype(at::kFloat));
}

static at::Tensor dst_or_new(const c10::optional<at::Tensor>& dst, int64_t C,
                             const at::Tensor& like, bool& accumulate) {
  if (dst.has_value() && dst->defined()) {
    TORCH_CHECK(dst->scalar_type() == at::kFloat && dst->is_contiguous() &&
                    dst->numel() == C && dst->device() == like.device(),
                "colsum: dst must be a contiguous fp32 [C] tensor");
    return *dst;
  }
  accumulate = false;
  return at::empty({C}, like.options().dtype(at::kFloat));
}

std::tuple<at::Tensor, at::Tensor> relu_bias_bwd(
    const at::Tensor& grad, const at::Tensor& out, bool relu,
    at::ScalarType g_dtype, const c10::optional<at::Tensor>& dbias,
    bool accumulate, const c10::optional<at::Tensor>& part_out) {
  // grad may be a column slice (unit column stride, any row stride), e.g. the
  // gradient of one block of a concatenation.
  TORCH_CHECK(grad.is_cuda() && grad.dim() == 2 && grad.stride(1) == 1 &&
                  grad.stride(0) >= grad.size(1) &&
                  (!relu || (out.is_contiguous() && out.sizes() == grad.sizes())),
              "relu_bias_bwd: grad [rows, C] with unit column stride, out "
              "contiguous");
  TORCH_CHECK(grad.scalar_type() == out.scalar_type(),
              "relu_bias_bwd: grad/out dtype mismatch");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(grad.device());
  const int rows = grad.size(0), C = grad.size(1);
  TORCH_CHECK(C <= 2048, "relu_bias_bwd: C <= 2048");
  at::Tensor g = at::empty({rows, C}, grad.options().dtype(g_dtype));
  at::Tensor db = dst_or_new(dbias, C, grad, accumulate);
  if (C == 0) return {g, db};
  if (rows == 0) {
    if (!accumulate) db.zero_();
    return {g, db};
  }
  const int blocks = colsum_blocks(rows);
  bool keep;
  at::Tensor part = partials_or_new(part_out, blocks, C, grad, keep);
  const bool vec = aligned16(grad.data_ptr()) && aligned16(out.data_ptr()) &&
                   aligned16(g.data_ptr()) &&
                   (grad.stride(0) * grad.element_size()) % 16 == 0;
  DGMC_DISPATCH_FLOAT(grad.scalar_type(), T, [&] {
    DGMC_DISPATCH_FLOAT(g_dtype, TR, [&] {
      dispatch_colsum<T, TR, true>(grad, out.data_ptr(), g.data_ptr(), part,
                                   keep ? nullptr : db.data_ptr<float>(),
                                   blocks, rows, C, relu, accumulate, vec);
    });
  });
  DGMC_CHECK_LAUNCH();
  return {g, keep ? part : db};
}

at::Tensor col_sum(const at::Tensor& src, const c10::optional<at::Tensor>& dst,
                   bool accumulate, const c10::optional<at::Tensor>& part_out) {
  TORCH_CHECK(src.is_cuda() && src.dim() == 2 && src.is_contiguous(),
              "col_sum: contiguous [rows, C] expected");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(src.device());
  const int rows = src.size(0), C = src.size(1);
  TORCH_CHECK(C <= 2048, "col_sum: C <= 2048");
  at::Tensor out = dst_or_new(dst, C, src, accumulate);
  if (C == 0) return out;
  if (rows == 0) {
    if (!accumulate) out.zero_();
    return out;
  }
  const int blocks = colsum_blocks(rows);
  bool keep;
  at::Tensor part = partials_or_new(part_out, blocks, C, src, keep);
  const bool vec = aligned16(src.data_ptr());
  DGMC_DISPATCH_FLOAT(src.scalar_type(), T, [&] {
    dispatch_colsum<T, float, false>(src, src.data_ptr(), nullptr, part,
                                     keep ? nullptr : out.data_ptr<float>(),
                                     blocks, rows, C, false, accumulate, vec);
  });
  DGMC_CHECK_LAUNCH();
  return keep ? part : out;
}

// dst (+)= sum over the leading dim of src [S, n] (fp32), float4 vectorised.
__global__ __launch_bounds__(256) void reduce_add_rows_kernel(
    const float* __restrict__ src, float* __restrict__ dst, int S, int64_t n,
    int accumulate) {
  const int64_t n4 = n / 4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
       i += stride) {
    float4 acc = accumulate ? reinterpret_cast<const float4*>(dst)[i]
                            : make_float4(0.f, 0.f, 0.f, 0.f);
    for (int s = 0; s < S; ++s) {
      const float4 v = reinterpret_cast<const float4*>(src + s * n)[i];
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    reinterpret_cast<float4*>(dst)[i] = acc;
  }
  for (int64_t i = n4 * 4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
       i < n; i += stride) {
    float acc = accumulate ? dst[i] : 0.f;
    for (int s = 0; s < S; ++s) acc += src[s * n + i];
    dst[i] = acc;
  }
}

void reduce_add_rows(const at::Tensor& src, at::Tensor dst, bool accumulate) {
  TORCH_CHECK(src.is_cuda() && src.scalar_type() == at::kFloat &&
                  src.is_contiguous() && dst.scalar_type() == at::kFloat &&
                  dst.is_contiguous(),
              "reduce_add_rows: contiguous fp32 tensors expected");
  const int S = src.size(0);
  const int64_t n = dst.numel();
  TORCH_CHECK(src.numel() == S * n, "reduce_add_rows: size mismatch");
  TORCH_CHECK(aligned16(src.data_ptr()) && aligned16(dst.data_ptr()),
              "reduce_add_rows: 16-byte alignment required");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(src.device());
  if (n == 0) return;
  const int blocks = (int)std::min<int64_t>((n / 4 + 255) / 256 + 1, 2048);
  hipLaunchKernelGGL(reduce_add_rows_kernel, dim3(blocks), dim3(256), 0,
                     stream(), src.data_ptr<float>(), dst.data_ptr<float>(), S,
                     n, accumulate ? 1 : 0);
  DGMC_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------
// Row concatenation of up to kCatMax 2-D blocks in ONE launch (loop-gradient
// operand stacks, runtime/loopgrad.py).  torch.cat splits such a list over
// several batched launches at ~0.7 TB/s; here every source is a 2-D grid of
// 16-byte chunks (rows may be strided - column-slice views are copied without
// a contiguous() pass) and blockIdx.y selects the source.
// ---------------------------------------------------------------------------
constexpr int kCatMax = 32;

struct CatArgs {
  const char* src[kCatMax];
  int64_t ld_bytes[kCatMax];    // source row stride
  int64_t rows[kCatMax];
  int64_t dst_row0[kCatMax];    // first output row of the block
};

__global__ __launch_bounds__(256) void cat_rows_kernel(CatArgs args,
                                                       char* __restrict__ dst,
                                                       int64_t row_bytes) {
  const int s = blockIdx.y;
  const int64_t cpr = row_bytes / 16;             // 16-byte chunks per row
  const int64_t total = args.rows[s] * cpr;
  const char* __restrict__ src = args.src[s];
  const int64_t ld = args.ld_bytes[s];
  char* __restrict__ out = dst + args.dst_row0[s] * row_bytes;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < total;
       c += stride) {
    const int64_t r = c / cpr, q = c - r * cpr;
    *reinterpret_cast<uint4*>(out + r * row_bytes + q * 16) =
        *reinterpret_cast<const uint4*>(src + r * ld + q * 16);
  }
}

at::Tensor cat_rows(at::TensorList srcs, const c10::optional<at::Tensor>& out) {
  TORCH_CHECK(!srcs.empty() && (int64_t)srcs.size() <= kCatMax,
              "cat_rows: 1..", kCatMax, " tensors");
  const at::Tensor& first = srcs[0];
  TORCH_CHECK(first.is_cuda() && first.dim() == 2, "cat_rows: 2-D CUDA tensors");
  const int64_t C = first.size(1);
  const int64_t es = first.element_size();
  const int64_t row_bytes = C * es;
  TORCH_CHECK(row_bytes % 16 == 0,
              "cat_rows: row bytes must be a multiple of 16");
  CatArgs args;
  int64_t rows = 0, max_rows = 0;
  for (size_t i = 0; i < srcs.size(); ++i) {
    const at::Tensor& t = srcs[i];
    TORCH_CHECK(t.dim() == 2 && t.size(1) == C &&
                    t.scalar_type() == first.scalar_type() &&
                    t.device() == first.device() && t.stride(1) == 1,
                "cat_rows: tensors must share dtype/device/columns and have "
                "unit column stride");
    const int64_t ld = (t.size(0) > 1 ? t.stride(0) : C) * es;
    TORCH_CHECK(aligned16(t.data_ptr()) && ld % 16 == 0,
                "cat_rows: 16-byte aligned rows required");
    args.src[i] = reinterpret_cast<const char*>(t.data_ptr());
    args.ld_bytes[i] = ld;
    args.rows[i] = t.size(0);
    args.dst_row0[i] = rows;
    rows += t.size(0);
    max_rows = std::max(max_rows, t.size(0));
  }
  at::Tensor dst;
  if (out.has_value() && out->defined()) {
    dst = *out;
    TORCH_CHECK(dst.is_contiguous() && dst.numel() == rows * C &&
                    dst.scalar_type() == first.scalar_type() &&
                    dst.device() == first.device() && aligned16(dst.data_ptr()),
                "cat_rows: out must be contiguous [sum rows, C], same dtype");
  } else {
    dst = at::empty({rows, C}, first.options());
  }
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(first.device());
  if (rows == 0 || C == 0) return dst;
  const int64_t chunks = max_rows * (row_bytes / 16);
  const int64_t want = (chunks + 255) / 256;
  const int64_t cap = std::max<int64_t>(1, 4096 / (int64_t)srcs.size());
  const int bx = (int)std::max<int64_t>(1, std::min<int64_t>(want, cap));
  hipLaunchKernelGGL(cat_rows_kernel, dim3(bx, (unsigned)srcs.size()),
                     dim3(256), 0, stream(), args,
                     reinterpret_cast<char*>(dst.data_ptr()), row_bytes);
  DGMC_CHECK_LAUNCH();
  return dst;
}

}  // namespace dgmc
