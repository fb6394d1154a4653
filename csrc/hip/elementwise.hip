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

constexpr int kRowsPerBlock = 64;

template <typename TG, typename TO, typename TR>
__global__ __launch_bounds__(256) void relu_bias_bwd_kernel(
    const TG* __restrict__ grad, const TO* __restrict__ out,
    TR* __restrict__ g_out, float* __restrict__ dbias_part, int rows, int C,
    int relu) {
  extern __shared__ __attribute__((aligned(16))) float part[];  // [4][C]
  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  const int r0 = blockIdx.x * kRowsPerBlock;
  const int r1 = min(r0 + kRowsPerBlock, rows);
  for (int c0 = 0; c0 < C; c0 += kWave) {
    const int c = c0 + lane;
    float acc = 0.f;
    if (c < C) {
      for (int r = r0 + wave; r < r1; r += 4) {
        const size_t o = (size_t)r * C + c;
        float g = Cvt<TG>::to_f(grad[o]);
        if (relu && !(Cvt<TO>::to_f(out[o]) > 0.f)) g = 0.f;
        g_out[o] = Cvt<TR>::from_f(g);
        acc += g;
      }
    }
    if (c < C) part[wave * C + c] = acc;
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += blockDim.x)
    dbias_part[(size_t)blockIdx.x * C + c] =
        part[c] + part[C + c] + part[2 * C + c] + part[3 * C + c];
}

std::tuple<at::Tensor, at::Tensor> relu_bias_bwd(const at::Tensor& grad,
                                                 const at::Tensor& out,
                                                 bool relu,
                                                 at::ScalarType g_dtype) {
  TORCH_CHECK(grad.is_cuda() && grad.dim() == 2 && grad.is_contiguous() &&
                  out.is_contiguous() && out.sizes() == grad.sizes(),
              "relu_bias_bwd: grad/out must be contiguous [rows, C]");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(grad.device());
  const int rows = grad.size(0), C = grad.size(1);
  at::Tensor g = at::empty({rows, C}, grad.options().dtype(g_dtype));
  const int blocks = std::max(1, (rows + kRowsPerBlock - 1) / kRowsPerBlock);
  at::Tensor part = at::empty({blocks, C}, grad.options().dtype(at::kFloat));
  if (rows == 0 || C == 0) return {g, part.zero_()};
  const size_t lds = 4 * (size_t)C * sizeof(float);
  TORCH_CHECK(lds <= 64 * 1024, "relu_bias_bwd: C too large");
  DGMC_DISPATCH_FLOAT(grad.scalar_type(), TG, [&] {
    DGMC_DISPATCH_FLOAT(out.scalar_type(), TO, [&] {
      DGMC_DISPATCH_FLOAT(g_dtype, TR, [&] {
        hipLaunchKernelGGL((relu_bias_bwd_kernel<TG, TO, TR>), dim3(blocks),
                           dim3(256), lds, stream(),
                           reinterpret_cast<const TG*>(grad.data_ptr()),
                           reinterpret_cast<const TO*>(out.data_ptr()),
                           reinterpret_cast<TR*>(g.data_ptr()),
                           part.data_ptr<float>(), rows, C, relu ? 1 : 0);
      });
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
