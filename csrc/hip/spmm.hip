// Deterministic CSR gather-reduce ("SpMM") - the one message-passing kernel.
//
//   out[r, :] = act( sum_{p in [rowptr[r], rowptr[r+1])} val[p] * x[col[p], :]
//                    + self_scale * self_x[r, :] + bias )
//
// Every aggregation of the reference's encoders maps onto it (see
// deep_graph_matching_consensus_amd/ops/sparse.py): SplineConv
// (torch_spline_conv weighting + PyG mean, reference spline.py:49), GIN sum
// (gin.py:49) and RelConv's two-flow mean (rel.py:26-31); the backward is the
// same kernel on the transposed operator, so there are no float atomics and
// results are bitwise reproducible.
//
// Mapping (CDNA4): a row is owned by LPR lanes of one wave64; each lane moves
// one 16-byte vector (8 bf16 / 4 f32 channels) per gathered row, so a bf16
// 256-channel row is one 512-byte coalesced read by 32 lanes.  UNROLL gathers
// are issued back-to-back for memory-level parallelism.  Blocks are remapped
// XCD-contiguously so the rows of one graph (adjacent ids) hit one L2.
#include "common.h"

namespace dgmc {

template <typename TOut, int VEC>
__device__ __forceinline__ void store_row(TOut* __restrict__ p,
                                          const float* v) {
  if constexpr (VEC * sizeof(TOut) % 16 == 0) {
    constexpr int N = 16 / sizeof(TOut);
#pragma unroll
    for (int k = 0; k < VEC; k += N) store_vec<TOut, N>(p + k, v + k);
  } else {
#pragma unroll
    for (int k = 0; k < VEC; ++k) p[k] = Cvt<TOut>::from_f(v[k]);
  }
}

template <typename TIn, typename TOut, int VEC, int LPR, int UNROLL>
__global__ __launch_bounds__(256) void spmm_csr_kernel(
    const int* __restrict__ rowptr, const int* __restrict__ col,
    const float* __restrict__ val, const TIn* __restrict__ x,
    const TIn* __restrict__ self_x, const float* __restrict__ self_scale,
    const float* __restrict__ bias, TOut* __restrict__ out, int R, int C,
    int relu) {
  constexpr int RPB = 256 / LPR;
  const int blk = xcd_remap(blockIdx.x, gridDim.x);
  const int r = blk * RPB + threadIdx.x / LPR;
  const int lane = threadIdx.x % LPR;
  if (r >= R) return;
  const int p0 = rowptr[r], p1 = rowptr[r + 1];
  const float scale = self_x != nullptr ? self_scale[0] : 0.f;

  for (int c0 = lane * VEC; c0 < C; c0 += LPR * VEC) {
    float acc[VEC];
#pragma unroll
    for (int k = 0; k < VEC; ++k) acc[k] = 0.f;

    int p = p0;
    for (; p + UNROLL <= p1; p += UNROLL) {
      float v[UNROLL][VEC];
      float w[UNROLL];
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) {
        const int j = col[p + u];
        w[u] = val[p + u];
        load_vec<TIn, VEC>(x + (size_t)j * C + c0, v[u]);
      }
#pragma unroll
      for (int u = 0; u < UNROLL; ++u)
#pragma unroll
        for (int k = 0; k < VEC; ++k) acc[k] = fmaf(w[u], v[u][k], acc[k]);
    }
    for (; p < p1; ++p) {
      float v[VEC];
      const float w = val[p];
      load_vec<TIn, VEC>(x + (size_t)col[p] * C + c0, v);
#pragma unroll
      for (int k = 0; k < VEC; ++k) acc[k] = fmaf(w, v[k], acc[k]);
    }
    if (self_x != nullptr) {
      float v[VEC];
      load_vec<TIn, VEC>(self_x + (size_t)r * C + c0, v);
#pragma unroll
      for (int k = 0; k < VEC; ++k) acc[k] = fmaf(scale, v[k], acc[k]);
    }
    if (bias != nullptr) {
#pragma unroll
      for (int k = 0; k < VEC; ++k) acc[k] += bias[c0 + k];
    }
    if (relu) {
#pragma unroll
      for (int k = 0; k < VEC; ++k) acc[k] = fmaxf(acc[k], 0.f);
    }
    store_row<TOut, VEC>(out + (size_t)r * C + c0, acc);
  }
}

template <typename TIn, typename TOut, int VEC, int LPR>
void launch_spmm(const int* rowptr, const int* col, const float* val,
                 const TIn* x, const TIn* self_x, const float* self_scale,
                 const float* bias, TOut* out, int R, int C, bool relu) {
  constexpr int RPB = 256 / LPR;
  const int blocks = (R + RPB - 1) / RPB;
  if (blocks == 0) return;
  hipLaunchKernelGGL((spmm_csr_kernel<TIn, TOut, VEC, LPR, 4>), dim3(blocks),
                     dim3(256), 0, stream(), rowptr, col, val, x, self_x,
                     self_scale, bias, out, R, C, relu ? 1 : 0);
  DGMC_CHECK_LAUNCH();
}

template <typename TIn, typename TOut>
void spmm_dispatch(const int* rowptr, const int* col, const float* val,
                   const TIn* x, const TIn* self_x, const float* self_scale,
                   const float* bias, TOut* out, int R, int C, bool relu,
                   bool vec_ok) {
  constexpr int V = Vec16<TIn>::N;
  if (vec_ok && C % V == 0) {
    const int lanes = C / V;
    if (lanes <= 4)
      return launch_spmm<TIn, TOut, V, 4>(rowptr, col, val, x, self_x,
                                          self_scale, bias, out, R, C, relu);
    if (lanes <= 8)
      return launch_spmm<TIn, TOut, V, 8>(rowptr, col, val, x, self_x,
                                          self_scale, bias, out, R, C, relu);
    if (lanes <= 16)
      return launch_spmm<TIn, TOut, V, 16>(rowptr, col, val, x, self_x,
                                           self_scale, bias, out, R, C, relu);
    if (lanes <= 32)
      return launch_spmm<TIn, TOut, V, 32>(rowptr, col, val, x, self_x,
                                           self_scale, bias, out, R, C, relu);
    return launch_spmm<TIn, TOut, V, 64>(rowptr, col, val, x, self_x,
                                         self_scale, bias, out, R, C, relu);
  }
  launch_spmm<TIn, TOut, 1, 64>(rowptr, col, val, x, self_x, self_scale, bias,
                                out, R, C, relu);
}

static void spmm_into(const at::Tensor& rowptr, const at::Tensor& col,
                      const at::Tensor& val, const at::Tensor& x,
                      const c10::optional<at::Tensor>& self_x,
                      const c10::optional<at::Tensor>& self_scale,
                      const c10::optional<at::Tensor>& bias, bool relu,
                      at::Tensor& out) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 2 && x.is_contiguous(), "spmm: x");
  TORCH_CHECK(rowptr.scalar_type() == at::kInt && col.scalar_type() == at::kInt,
              "spmm: int32 index expected");
  TORCH_CHECK(val.scalar_type() == at::kFloat, "spmm: fp32 values expected");
  TORCH_CHECK(col.numel() == val.numel(), "spmm: col/val size mismatch");
  const int64_t R = rowptr.numel() - 1;
  const int64_t C = x.size(1);
  TORCH_CHECK(R >= 0 && R < INT32_MAX && C < INT32_MAX, "spmm: size");
  TORCH_CHECK(out.is_contiguous() && out.numel() == R * C &&
                  out.device() == x.device(),
              "spmm: out must be a contiguous tensor with R*C elements");
  const at::ScalarType out_dtype = out.scalar_type();
  if (R == 0 || C == 0) return;

  const at::Tensor* sx = nullptr;
  at::Tensor sx_c, ss_c, b_c;
  if (self_x.has_value() && self_x->defined()) {
    sx_c = self_x->contiguous();
    TORCH_CHECK(sx_c.scalar_type() == x.scalar_type() && sx_c.size(0) == R &&
                    sx_c.size(1) == C,
                "spmm: self_x must match x dtype and [R, C]");
    TORCH_CHECK(self_scale.has_value() && self_scale->defined(),
                "spmm: self_scale required with self_x");
    ss_c = self_scale->to(at::kFloat).contiguous();
    sx = &sx_c;
  }
  if (bias.has_value() && bias->defined()) {
    b_c = bias->to(at::kFloat).contiguous();
    TORCH_CHECK(b_c.numel() == C, "spmm: bias size");
  }
  const bool vec_ok = aligned16(x.data_ptr()) &&
                      (sx == nullptr || aligned16(sx->data_ptr())) &&
                      aligned16(out.data_ptr());

  DGMC_DISPATCH_FLOAT(x.scalar_type(), TIn, [&] {
    const TIn* xp = reinterpret_cast<const TIn*>(x.data_ptr());
    const TIn* sp = sx ? reinterpret_cast<const TIn*>(sx->data_ptr()) : nullptr;
    const float* ssp = sx ? ss_c.data_ptr<float>() : nullptr;
    const float* bp = b_c.defined() ? b_c.data_ptr<float>() : nullptr;
    DGMC_DISPATCH_FLOAT(out_dtype, TOut, [&] {
      spmm_dispatch<TIn, TOut>(rowptr.data_ptr<int>(), col.data_ptr<int>(),
                               val.data_ptr<float>(), xp, sp, ssp, bp,
                               reinterpret_cast<TOut*>(out.data_ptr()), (int)R,
                               (int)C, relu, vec_ok);
    });
  });
  DGMC_CHECK_LAUNCH();
}

at::Tensor spmm_csr(const at::Tensor& rowptr, const at::Tensor& col,
                    const at::Tensor& val, const at::Tensor& x,
                    const c10::optional<at::Tensor>& self_x,
                    const c10::optional<at::Tensor>& self_scale,
                    const c10::optional<at::Tensor>& bias, bool relu,
                    at::ScalarType out_dtype) {
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  at::Tensor out =
      at::empty({rowptr.numel() - 1, x.size(1)}, x.options().dtype(out_dtype));
  spmm_into(rowptr, col, val, x, self_x, self_scale, bias, relu, out);
  return out;
}

// Writes into a caller-owned buffer (e.g. a slot of a loop-gradient stack,
// runtime/loopgrad.py), so the consumer needs no copy.
void spmm_csr_out(const at::Tensor& rowptr, const at::Tensor& col,
                  const at::Tensor& val, const at::Tensor& x,
                  const c10::optional<at::Tensor>& self_x,
                  const c10::optional<at::Tensor>& self_scale,
                  const c10::optional<at::Tensor>& bias, bool relu,
                  at::Tensor out) {
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  spmm_into(rowptr, col, val, x, self_x, self_scale, bias, relu, out);
}

}  // namespace dgmc
