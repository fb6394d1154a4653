// Fused element-wise backward helpers.
//
// relu_bias_bwd: for an aggregation output `out = relu(A x + bias)` the
// backward needs g' = grad * (out > 0) for the transposed aggregation and
// dbias = sum_rows g'.  Eager PyTorch spends three kernels (compare, mul,
// column reduction); this kernel does both in one pass: each workgroup owns a
// row range, writes g' (in the activation dtype) and one fp32 partial column
// sum per block; the tiny [blocks, C] partial is summed by the caller.
//
// reduce_add_rows: dst[n] (+)= sum_s src[s, n] - the split-K combine of the
// weight-gradient GEMMs, accumulating straight into the fp32 gradient.
#include "common.h"

namespace dgmc {

// LPR lanes own one row (VEC channels each per pass); a block holds
// RPB = 256 / LPR row slots and walks rows grid-stride, keeping per-thread
// channel partials in registers; the block's column partial is reduced
// through LDS once at the end.
template <typename TG, typename TO, typename TR, int VEC, int LPR>
__global__ __launch_bounds__(256) void relu_bias_bwd_kernel(
    const TG* __restrict__ grad, const TO* __restrict__ out,
    TR* __restrict__ g_out, float* __restrict__ dbias_part, int rows, int C,
    int relu) {
  constexpr int RPB = 256 / LPR;
  extern __shared__ __attribute__((aligned(16))) float part[];  // [RPB][C]
  const int slot = threadIdx.x / LPR, lane = threadIdx.x % LPR;
  for (int c0 = lane * VEC; c0 < C; c0 += LPR * VEC) {
    float acc[VEC];
#pragma unroll
    for (int k = 0; k < VEC; ++k) acc[k] = 0.f;
    for (int r = blockIdx.x * RPB + slot; r < rows; r += gridDim.x * RPB) {
      const size_t o = (size_t)r * C + c0;
      float g[VEC], m[VEC];
      load_vec<TG, VEC>(grad + o, g);
      if (relu) {
        load_vec<TO, VEC>(out + o, m);
#pragma unroll
        for (int k = 0; k < VEC; ++k) g[k] = m[k] > 0.f ? g[k] : 0.f;
      }
#pragma unroll
      for (int k = 0; k < VEC; ++k) acc[k] += g[k];
      if constexpr (VEC * sizeof(TR) == 16) {
        store_vec<TR, VEC>(g_out + o, g);
      } else {
#pragma unroll
        for (int k = 0; k < VEC; ++k) g_out[o + k] = Cvt<TR>::from_f(g[k]);
      }
    }
#pragma unroll
    for (int k = 0; k < VEC; ++k) part[slot * C + c0 + k] = acc[k];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float s = 0.f;
    for (int q = 0; q < RPB; ++q) s += part[q * C + c];
    dbias_part[(size_t)blockIdx.x * C + c] = s;
  }
}

template <typename TG, typename TO, typename TR, int VEC, int LPR>
void launch_relu_bias(const at::Tensor& grad, const at::Tensor& out,
                      at::Tensor& g, at::Tensor& part, int blocks, int rows,
                      int C, bool relu) {
  constexpr int RPB = 256 / LPR;
  hipLaunchKernelGGL((relu_bias_bwd_kernel<TG, TO, TR, VEC, LPR>),
                     dim3(blocks), dim3(256), RPB * C * sizeof(float),
                     stream(), reinterpret_cast<const TG*>(grad.data_ptr()),
                     reinterpret_cast<const TO*>(out.data_ptr()),
                     reinterpret_cast<TR*>(g.data_ptr()),
                     part.data_ptr<float>(), rows, C, relu ? 1 : 0);
}

std::tuple<at::Tensor, at::Tensor> relu_bias_bwd(const at::Tensor& grad,
                                                 const at::Tensor& out,
                                                 bool relu,
                                                 at::ScalarType g_dtype) {
  TORCH_CHECK(grad.is_cuda() && grad.dim() == 2 && grad.is_contiguous() &&
                  out.is_contiguous() && out.sizes() == grad.sizes(),
              "relu_bias_bwd: grad/out must be contiguous [rows, C]");
  TORCH_CHECK(grad.scalar_type() == out.scalar_type(),
              "relu_bias_bwd: grad/out dtype mismatch");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(grad.device());
  const int rows = grad.size(0), C = grad.size(1);
  TORCH_CHECK(C <= 2048, "relu_bias_bwd: C <= 2048");
  at::Tensor g = at::empty({rows, C}, grad.options().dtype(g_dtype));
  const int blocks = std::max(1, std::min((rows + 7) / 8, 1024));
  at::Tensor part = at::empty({blocks, C}, grad.options().dtype(at::kFloat));
  if (rows == 0 || C == 0) return {g, part.zero_()};
  const bool vec = aligned16(grad.data_ptr()) && aligned16(out.data_ptr()) &&
                   aligned16(g.data_ptr());
  DGMC_DISPATCH_FLOAT(grad.scalar_type(), T, [&] {
    DGMC_DISPATCH_FLOAT(g_dtype, TR, [&] {
      constexpr int V = Vec16<T>::N;
      if (vec && C % V == 0) {
        const int lanes = C / V;
        if (lanes <= 8)
          launch_relu_bias<T, T, TR, V, 8>(grad, out, g, part, blocks, rows,
                                           C, relu);
        else if (lanes <= 16)
          launch_relu_bias<T, T, TR, V, 16>(grad, out, g, part, blocks, rows,
                                            C, relu);
        else if (lanes <= 32)
          launch_relu_bias<T, T, TR, V, 32>(grad, out, g, part, blocks, rows,
                                            C, relu);
        else
          launch_relu_bias<T, T, TR, V, 64>(grad, out, g, part, blocks, rows,
                                            C, relu);
      } else {
        launch_relu_bias<T, T, TR, 1, 64>(grad, out, g, part, blocks, rows, C,
                                          relu);
      }
    });
  });
  DGMC_CHECK_LAUNCH();
  return {g, part};
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

}  // namespace dgmc
