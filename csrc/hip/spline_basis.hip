// B-spline basis + weight index (torch_spline_conv ``spline_basis`` semantics,
// used by PyG SplineConv at reference spline.py:49).
//
// For edge e and slot s in [0, (degree+1)^D):
//   wi(e,s) = sum_d ((floor(v_d) + k_d) mod K_d) * prod_{d'<d} K_d'
//   b(e,s)  = prod_d N_{degree,k_d}(frac(v_d)),  v_d = pseudo[e,d]*(K_d - deg*open_d)
// with k_d the d-th base-(degree+1) digit of s.  One thread per (edge, slot);
// computed once per batch and folded into the spline sparse operator.
#include "common.h"

namespace dgmc {

template <int DEG>
__device__ __forceinline__ float basis_fn(float v, int k) {
  if constexpr (DEG == 1) {
    return k == 0 ? 1.f - v : v;
  } else if constexpr (DEG == 2) {
    if (k == 0) return 0.5f * v * v - v + 0.5f;
    if (k == 1) return -v * v + v + 0.5f;
    return 0.5f * v * v;
  } else {
    if (k == 0) return (1.f - v) * (1.f - v) * (1.f - v) / 6.f;
    if (k == 1) return (3.f * v * v * v - 6.f * v * v + 4.f) / 6.f;
    if (k == 2) return (-3.f * v * v * v + 3.f * v * v + 3.f * v + 1.f) / 6.f;
    return v * v * v / 6.f;
  }
}

template <int DEG>
__global__ __launch_bounds__(256) void spline_basis_kernel(
    const float* __restrict__ pseudo, const int* __restrict__ kernel_size,
    const int* __restrict__ is_open, float* __restrict__ basis,
    int64_t* __restrict__ wi, int64_t E, int D, int S) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= E * S) return;
  const int64_t e = t / S;
  const int s = (int)(t % S);
  float b = 1.f;
  int64_t index = 0, offset = 1;
  int rem = s;
  for (int d = 0; d < D; ++d) {
    const int k = rem % (DEG + 1);
    rem /= (DEG + 1);
    const int ks = kernel_size[d];
    float v = pseudo[e * D + d] * (float)(ks - DEG * is_open[d]);
    const float fl = floorf(v);
    int idx = ((int)fl + k) % ks;
    if (idx < 0) idx += ks;
    index += (int64_t)idx * offset;
    offset *= ks;
    b *= basis_fn<DEG>(v - fl, k);
  }
  basis[t] = b;
  wi[t] = index;
}

std::tuple<at::Tensor, at::Tensor> spline_basis(const at::Tensor& pseudo,
                                                const at::Tensor& kernel_size,
                                                const at::Tensor& is_open,
                                                int64_t degree) {
  TORCH_CHECK(pseudo.is_cuda() && pseudo.dim() == 2 &&
                  pseudo.scalar_type() == at::kFloat && pseudo.is_contiguous(),
              "spline_basis: pseudo must be contiguous fp32 [E, D]");
  TORCH_CHECK(degree >= 1 && degree <= 3, "spline_basis: degree 1..3");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(pseudo.device());
  const int64_t E = pseudo.size(0);
  const int D = (int)pseudo.size(1);
  TORCH_CHECK(kernel_size.numel() == D && is_open.numel() == D,
              "spline_basis: kernel_size/is_open must have D entries");
  int S = 1;
  for (int d = 0; d < D; ++d) S *= (int)(degree + 1);
  auto ks = kernel_size.to(at::kInt).contiguous();
  auto op = is_open.to(at::kInt).contiguous();
  at::Tensor basis = at::empty({E, S}, pseudo.options());
  at::Tensor wi = at::empty({E, S}, pseudo.options().dtype(at::kLong));
  const int64_t total = E * S;
  if (total == 0) return {basis, wi};
  const int blocks = (int)((total + 255) / 256);
  auto launch = [&](auto kernel) {
    hipLaunchKernelGGL(kernel, dim3(blocks), dim3(256), 0, stream(),
                       pseudo.data_ptr<float>(), ks.data_ptr<int>(),
                       op.data_ptr<int>(), basis.data_ptr<float>(),
                       wi.data_ptr<int64_t>(), E, D, S);
  };
  if (degree == 1) launch(spline_basis_kernel<1>);
  else if (degree == 2) launch(spline_basis_kernel<2>);
  else launch(spline_basis_kernel<3>);
  DGMC_CHECK_LAUNCH();
  return {basis, wi};
}

}  // namespace dgmc
