// SplineConv weight layouts (per training step, once per forward scope).
//
// The reference keeps PyG's parameter layout (``weight [K, in, out]``,
// ``root [in, out]``; /root/reference/dgmc/models/spline.py:21 via
// SplineConv) and torch_spline_conv indexes it per edge.  Here a SplineConv
// is ONE GEMM ``x @ [W_0 | .. | W_{K-1} | root]`` followed by the sparse
// slot aggregation, so every forward needs the stacked low-precision operand
//
//   w_lp[i, s * O + o] = s < K ? weight[s, i, o] : root[i, o]     (bf16)
//
// and every backward maps the stacked fp32 gradient back:
//
//   gweight[s, i, o] = g[i, s * O + o],   groot[i, o] = g[i, K * O + o].
//
// Eager PyTorch spends a permute copy + a concatenation + a cast in the
// forward (3 kernels, 2 fp32 intermediates: ~32 us for psi_1's first layer
// [1024, 26 x 256]) and slice / permute-backward copies in the backward.
// Both directions are single bandwidth-bound passes here: 16-byte fp32
// loads, contiguous along ``o`` on both sides.
#include "common.h"

namespace dgmc {

namespace {

// One thread per 4 consecutive ``o`` of one (i, s) row segment; thread ids
// run o-fastest, then s, then i, so the stacked side is written (or read)
// contiguously and the parameter side in O-long contiguous runs.
template <typename TOUT>
__global__ __launch_bounds__(256) void spline_weight_pack_kernel(
    const float* __restrict__ weight, const float* __restrict__ root,
    TOUT* __restrict__ out, int in, int K, int S, int O) {
  const int O4 = O / 4;
  const int64_t total = (int64_t)in * S * O4;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int o = (int)(t % O4) * 4;
    const int64_t rs = t / O4;
    const int s = (int)(rs % S);
    const int i = (int)(rs / S);
    const float* src = s < K ? weight + ((int64_t)s * in + i) * O + o
                             : root + (int64_t)i * O + o;
    const float4 v = *reinterpret_cast<const float4*>(src);
    TOUT* dst = out + (int64_t)i * S * O + (int64_t)s * O + o;
    if constexpr (sizeof(TOUT) == 2) {
      typedef TOUT v4 __attribute__((ext_vector_type(4)));
      const v4 w = {(TOUT)v.x, (TOUT)v.y, (TOUT)v.z, (TOUT)v.w};
      *reinterpret_cast<v4*>(dst) = w;
    } else {
      *reinterpret_cast<float4*>(dst) = v;
    }
  }
}

__global__ __launch_bounds__(256) void spline_weight_unpack_kernel(
    const float* __restrict__ g, float* __restrict__ gweight,
    float* __restrict__ groot, int in, int K, int S, int O) {
  const int O4 = O / 4;
  const int64_t total = (int64_t)in * S * O4;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int o = (int)(t % O4) * 4;
    const int64_t rs = t / O4;
    const int s = (int)(rs % S);
    const int i = (int)(rs / S);
    const float4 v = *reinterpret_cast<const float4*>(
        g + (int64_t)i * S * O + (int64_t)s * O + o);
    float* dst = s < K ? gweight + ((int64_t)s * in + i) * O + o
                       : groot + (int64_t)i * O + o;
    *reinterpret_cast<float4*>(dst) = v;
  }
}

int grid_for(int64_t work) {
  return (int)std::min<int64_t>((work + 255) / 256, 4096);
}

void check_params(const at::Tensor& weight,
                  const c10::optional<at::Tensor>& root) {
  TORCH_CHECK(weight.is_cuda() && weight.scalar_type() == at::kFloat &&
                  weight.dim() == 3 && weight.is_contiguous() &&
                  aligned16(weight.data_ptr()),
              "spline_weight: fp32 contiguous weight [K, in, out] expected");
  TORCH_CHECK(weight.size(2) % 4 == 0, "spline_weight: out % 4 != 0");
  if (root.has_value() && root->defined())
    TORCH_CHECK(root->is_cuda() && root->scalar_type() == at::kFloat &&
                    root->is_contiguous() && aligned16(root->data_ptr()) &&
                    root->dim() == 2 && root->size(0) == weight.size(1) &&
                    root->size(1) == weight.size(2),
                "spline_weight: fp32 contiguous root [in, out] expected");
}

}  // namespace

at::Tensor spline_weight_pack(const at::Tensor& weight,
                              const c10::optional<at::Tensor>& root,
                              at::ScalarType dtype) {
  check_params(weight, root);
  const bool has_root = root.has_value() && root->defined();
  const int K = weight.size(0), in = weight.size(1), O = weight.size(2);
  const int S = K + (has_root ? 1 : 0);
  TORCH_CHECK(dtype == at::kBFloat16 || dtype == at::kFloat,
              "spline_weight_pack: bf16 or fp32 output");
  at::Tensor out = at::empty({in, (int64_t)S * O}, weight.options().dtype(dtype));
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(weight.device());
  const int64_t work = (int64_t)in * S * (O / 4);
  if (work == 0) return out;
  const float* rp = has_root ? root->data_ptr<float>() : nullptr;
  if (dtype == at::kBFloat16)
    hipLaunchKernelGGL(spline_weight_pack_kernel<__bf16>, dim3(grid_for(work)),
                       dim3(256), 0, stream(), weight.data_ptr<float>(), rp,
                       reinterpret_cast<__bf16*>(out.data_ptr()), in, K, S, O);
  else
    hipLaunchKernelGGL(spline_weight_pack_kernel<float>, dim3(grid_for(work)),
                       dim3(256), 0, stream(), weight.data_ptr<float>(), rp,
                       out.data_ptr<float>(), in, K, S, O);
  DGMC_CHECK_LAUNCH();
  return out;
}

std::tuple<at::Tensor, at::Tensor> spline_weight_unpack(const at::Tensor& g,
                                                        int64_t K,
                                                        bool has_root) {
  TORCH_CHECK(g.is_cuda() && g.scalar_type() == at::kFloat && g.dim() == 2 &&
                  g.is_contiguous() && aligned16(g.data_ptr()),
              "spline_weight_unpack: fp32 contiguous [in, S * out] expected");
  const int S = (int)K + (has_root ? 1 : 0);
  TORCH_CHECK(K >= 1 && g.size(1) % S == 0, "spline_weight_unpack: shape");
  const int in = g.size(0), O = g.size(1) / S;
  TORCH_CHECK(O % 4 == 0, "spline_weight_unpack: out % 4 != 0");
  at::Tensor gw = at::empty({K, in, O}, g.options());
  at::Tensor gr = has_root ? at::empty({in, O}, g.options()) : at::Tensor();
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(g.device());
  const int64_t work = (int64_t)in * S * (O / 4);
  if (work > 0) {
    hipLaunchKernelGGL(spline_weight_unpack_kernel, dim3(grid_for(work)),
                       dim3(256), 0, stream(), g.data_ptr<float>(),
                       gw.data_ptr<float>(),
                       has_root ? gr.data_ptr<float>() : nullptr, in, (int)K,
                       S, O);
    DGMC_CHECK_LAUNCH();
  }
  return {gw, gr};
}

// ---------------------------------------------------------------------------
// spline_slot_images: the two weight images of the fused slot conv
// (csrc/hip/slot_conv.hip) straight from the parameters, for 128 -> 128
// SplineConvs (psi_2):
//   fwd  [S, out, in]:  img[s, o, p] = W_s[perm[p], o]
//   trans[S, in, out]:  img[s, i, p] = W_s[i, perm[p]]
// with W_s = weight[s] (s < K) or root, perm the kernel's K order
// (ops/sparse.py::slot_k_order).  One launch instead of a bf16 pack plus
// two permute-gather kernels (ops/sparse.py::slot_conv_image).
namespace {
__global__ __launch_bounds__(256) void spline_slot_images_kernel(
    const float* __restrict__ weight, const float* __restrict__ root,
    const int64_t* __restrict__ perm, __bf16* __restrict__ img_f,
    __bf16* __restrict__ img_t, int K, int S) {
  constexpr int C = 128;
  const int64_t total = (int64_t)2 * S * C * (C / 8);
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int p8 = (int)(t % (C / 8)) * 8;
    const int64_t rest = t / (C / 8);
    const int r = (int)(rest % C);
    const int64_t rest2 = rest / C;
    const int s = (int)(rest2 % S);
    const bool trans = rest2 >= S;
    const float* W = s < K ? weight + (int64_t)s * C * C : root;
    typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
    bf16x8 v;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int q = (int)perm[p8 + e];
      v[e] = (__bf16)(trans ? W[r * C + q] : W[q * C + r]);
    }
    __bf16* dst = (trans ? img_t : img_f) + ((int64_t)s * C + r) * C + p8;
    *reinterpret_cast<bf16x8*>(dst) = v;
  }
}
}  // namespace

std::tuple<at::Tensor, at::Tensor> spline_slot_images(
    const at::Tensor& weight, const c10::optional<at::Tensor>& root,
    const at::Tensor& perm) {
  check_params(weight, root);
  TORCH_CHECK(weight.size(1) == 128 && weight.size(2) == 128,
              "spline_slot_images: 128 -> 128 SplineConv only");
  TORCH_CHECK(perm.is_cuda() && perm.scalar_type() == at::kLong &&
                  perm.numel() == 128 && perm.is_contiguous(),
              "spline_slot_images: int64 perm [128]");
  const bool has_root = root.has_value() && root->defined();
  const int K = weight.size(0), S = K + (has_root ? 1 : 0);
  auto opt = weight.options().dtype(at::kBFloat16);
  at::Tensor img_f = at::empty({S, 128, 128}, opt);
  at::Tensor img_t = at::empty({S, 128, 128}, opt);
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(weight.device());
  const int64_t work = (int64_t)2 * S * 128 * 16;
  hipLaunchKernelGGL(spline_slot_images_kernel, dim3(grid_for(work)),
                     dim3(256), 0, stream(), weight.data_ptr<float>(),
                     has_root ? root->data_ptr<float>() : nullptr,
                     perm.data_ptr<int64_t>(),
                     reinterpret_cast<__bf16*>(img_f.data_ptr()),
                     reinterpret_cast<__bf16*>(img_t.data_ptr()), K, S);
  DGMC_CHECK_LAUNCH();
  return {img_f, img_t};
}

// ---------------------------------------------------------------------------
// fold_weights: the folded consensus projection W = W1 @ W_f (fp32, once per
// training step; models/dgmc.py::_FoldProduct) together with the two bf16
// operand images the projection kernels read - W (ops/dense.py::cat_gemm
// forward) and W^T (its backward) - in ONE launch instead of an fp32 GEMM
// plus a cast and a transposed cast.  Block = one output row r, one thread
// per output column (coalesced W_f reads, W1[r, :] broadcast from LDS).
namespace {
__global__ __launch_bounds__(512) void fold_weights_kernel(
    const float* __restrict__ w1, const float* __restrict__ wf,
    float* __restrict__ w, __bf16* __restrict__ wn, __bf16* __restrict__ wnt,
    int R, int Kin, int K) {
  extern __shared__ float w1r[];                  // [Kin]
  const int r = blockIdx.x;
  for (int q = threadIdx.x; q < Kin; q += blockDim.x)
    w1r[q] = w1[(size_t)r * Kin + q];
  __syncthreads();
  for (int c = threadIdx.x; c < K; c += blockDim.x) {
    float a0 = 0.f, a1 = 0.f;
    int q = 0;
    for (; q + 1 < Kin; q += 2) {
      a0 = fmaf(w1r[q], wf[(size_t)q * K + c], a0);
      a1 = fmaf(w1r[q + 1], wf[(size_t)(q + 1) * K + c], a1);
    }
    if (q < Kin) a0 = fmaf(w1r[q], wf[(size_t)q * K + c], a0);
    const float v = a0 + a1;
    w[(size_t)r * K + c] = v;
    wn[(size_t)r * K + c] = (__bf16)v;
    wnt[(size_t)c * R + r] = (__bf16)v;
  }
}
}  // namespace

std::tuple<at::Tensor, at::Tensor, at::Tensor> fold_weights(
    const at::Tensor& w1, const at::Tensor& wf) {
  TORCH_CHECK(w1.is_cuda() && wf.is_cuda() &&
                  w1.scalar_type() == at::kFloat &&
                  wf.scalar_type() == at::kFloat && w1.dim() == 2 &&
                  wf.dim() == 2 && w1.size(1) == wf.size(0) &&
                  w1.is_contiguous() && wf.is_contiguous(),
              "fold_weights: fp32 contiguous W1 [R, Kin], W_f [Kin, K]");
  const int R = (int)w1.size(0), Kin = (int)w1.size(1), K = (int)wf.size(1);
  at::Tensor w = at::empty({R, K}, w1.options());
  at::Tensor wn = at::empty({R, K}, w1.options().dtype(at::kBFloat16));
  at::Tensor wnt = at::empty({K, R}, w1.options().dtype(at::kBFloat16));
  if (R == 0 || K == 0) return {w, wn, wnt};
  TORCH_CHECK(Kin <= 8192, "fold_weights: inner size");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(w1.device());
  hipLaunchKernelGGL(fold_weights_kernel, dim3(R),
                     dim3(std::min(512, std::max(64, (K + 63) / 64 * 64))),
                     (size_t)Kin * sizeof(float), stream(),
                     w1.data_ptr<float>(), wf.data_ptr<float>(),
                     w.data_ptr<float>(),
                     reinterpret_cast<__bf16*>(wn.data_ptr()),
                     reinterpret_cast<__bf16*>(wnt.data_ptr()), R, Kin, K);
  DGMC_CHECK_LAUNCH();
  return {w, wn, wnt};
}

}  // namespace dgmc
