// Multi-tensor Adam for the training step (torch.optim.Adam semantics,
// amsgrad=False, L2 weight decay folded into the gradient):
//
//   g' = g + wd p;  m = b1 m + (1 - b1) g';  v = b2 v + (1 - b2) g'^2
//   p -= lr / (1 - b1^t) * m / (sqrt(v) / sqrt(1 - b2^t) + eps)
//
// Replaces the fused torch Adam (multi_tensor_apply: ~122 us for the 9.5 M
// fp32 parameters of the PascalVOC flagship, ~2.2 TB/s): ONE launch over a
// pointer table of every parameter, float4 loads/stores, 4 float4 per
// thread in flight.  Every parameter keeps its own fp32 device step counter
// (torch's per-parameter ``state['step']``, incremented by adam_step_inc -
// one thread per counter - unless found_inf is set), and the non-finite flag
// is read on the device, so the whole update is capturable in a hipGraph
// and skips itself on the device.
#include "common.h"

namespace dgmc {

namespace {

constexpr int kAdamMax = 64;          // parameters per launch
constexpr int kAdamThreads = 256;
constexpr int kAdamVec = 4;           // float4 per thread per block
constexpr int kAdamBlock = kAdamThreads * kAdamVec * 4;   // floats per block

struct AdamTable {
  float* p[kAdamMax];
  const float* g[kAdamMax];
  float* m[kAdamMax];
  float* v[kAdamMax];
  const float* s[kAdamMax];           // per-parameter step (already bumped)
  int n[kAdamMax];
  int first_block[kAdamMax + 1];
  int count;
};

}  // namespace

struct StepTable {
  float* s[kAdamMax];
  int count;
};

// With ``flags`` (per-block non-finite flags written by pack_grads): fold
// them first - found_inf = any, skip counter += any - then bump the step
// counters of a finite step (one launch instead of two check kernels).
__global__ void adam_step_inc_kernel(const StepTable T, float* found_inf,
                                     const int* __restrict__ flags,
                                     int nflags, double* __restrict__ skips) {
  const int i = threadIdx.x;
  bool bad;
  if (flags) {
    __shared__ int any;
    if (i == 0) any = 0;
    __syncthreads();
    int b = 0;
    for (int j = i; j < nflags; j += blockDim.x) b |= flags[j];
    if (b) any = 1;        // benign race: every writer stores 1
    __syncthreads();
    bad = any != 0;
    if (i == 0) {
      if (found_inf) *found_inf = bad ? 1.f : 0.f;
      if (skips) *skips += bad ? 1.0 : 0.0;
    }
  } else {
    bad = found_inf && *found_inf != 0.f;
  }
  if (i < T.count && !bad) *T.s[i] += 1.f;
}

__global__ __launch_bounds__(kAdamThreads) void adam_multi_kernel(
    const AdamTable T, const float* __restrict__ found_inf, float lr, float b1, float b2,
    float eps, float wd) {
  if (found_inf && *found_inf != 0.f) return;   // non-finite step: skip
  const int b = blockIdx.x;
  int ti = 0;
  while (ti + 1 < T.count && T.first_block[ti + 1] <= b) ++ti;
  const int n = T.n[ti];
  const int base = (b - T.first_block[ti]) * kAdamBlock;
  const float t = *T.s[ti];
  const float bc1 = 1.f - powf(b1, t), bc2 = 1.f - powf(b2, t);
  const float step_size = lr / bc1, rs2 = 1.f / sqrtf(bc2);
  float* __restrict__ P = T.p[ti];
  const float* __restrict__ G = T.g[ti];
  float* __restrict__ M = T.m[ti];
  float* __restrict__ V = T.v[ti];
  auto upd = [&](float& p, float g, float& m, float& v) {
    g += wd * p;
    m = b1 * m + (1.f - b1) * g;
    v = b2 * v + (1.f - b2) * g * g;
    p -= step_size * m / (sqrtf(v) * rs2 + eps);
  };
  if (base + kAdamBlock <= n) {
    float4 pv[kAdamVec], gv[kAdamVec], mv[kAdamVec], vv[kAdamVec];
#pragma unroll
    for (int u = 0; u < kAdamVec; ++u) {
      const int i = base + 4 * (u * kAdamThreads + threadIdx.x);
      pv[u] = *reinterpret_cast<const float4*>(P + i);
      gv[u] = *reinterpret_cast<const float4*>(G + i);
      mv[u] = *reinterpret_cast<const float4*>(M + i);
      vv[u] = *reinterpret_cast<const float4*>(V + i);
    }
#pragma unroll
    for (int u = 0; u < kAdamVec; ++u) {
      upd(pv[u].x, gv[u].x, mv[u].x, vv[u].x);
      upd(pv[u].y, gv[u].y, mv[u].y, vv[u].y);
      upd(pv[u].z, gv[u].z, mv[u].z, vv[u].z);
      upd(pv[u].w, gv[u].w, mv[u].w, vv[u].w);
      const int i = base + 4 * (u * kAdamThreads + threadIdx.x);
      *reinterpret_cast<float4*>(P + i) = pv[u];
      *reinterpret_cast<float4*>(M + i) = mv[u];
      *reinterpret_cast<float4*>(V + i) = vv[u];
    }
  } else {
    for (int i = base + threadIdx.x; i < min(n, base + kAdamBlock);
         i += kAdamThreads) {
      float p = P[i], m = M[i], v = V[i];
      upd(p, G[i], m, v);
      P[i] = p;
      M[i] = m;
      V[i] = v;
    }
  }
}

// params / grads / exp_avg / exp_avg_sq: fp32 contiguous, 16-byte aligned,
// pairwise equal sizes; steps: one fp32 1-element device counter per param
// (already incremented for this step); found_inf: optional fp32 0-dim flag.
namespace {
void check_step(const at::Tensor& s, const at::Tensor& like) {
  TORCH_CHECK(s.is_cuda() && s.scalar_type() == at::kFloat &&
                  s.numel() == 1 && s.device() == like.device(),
              "adam: fp32 1-element step counter on the parameter's device");
}
}  // namespace

void adam_multi(at::TensorList params, at::TensorList grads,
                at::TensorList exp_avg, at::TensorList exp_avg_sq,
                at::TensorList steps,
                const c10::optional<at::Tensor>& found_inf, double lr,
                double beta1, double beta2, double eps, double weight_decay) {
  const int64_t count = (int64_t)params.size();
  TORCH_CHECK(count >= 1 && (int64_t)grads.size() == count &&
                  (int64_t)exp_avg.size() == count &&
                  (int64_t)exp_avg_sq.size() == count &&
                  (int64_t)steps.size() == count,
              "adam_multi: one grad / exp_avg / exp_avg_sq / step per param");
  const float* fi = nullptr;
  if (found_inf.has_value() && found_inf->defined()) {
    TORCH_CHECK(found_inf->is_cuda() &&
                    found_inf->scalar_type() == at::kFloat &&
                    found_inf->numel() == 1,
                "adam_multi: fp32 found_inf flag");
    fi = found_inf->data_ptr<float>();
  }
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(params[0].device());
  for (int64_t c0 = 0; c0 < count; c0 += kAdamMax) {
    AdamTable T{};
    T.count = (int)std::min<int64_t>(kAdamMax, count - c0);
    int blocks = 0;
    for (int j = 0; j < T.count; ++j) {
      const at::Tensor* ts[4] = {&params[c0 + j], &grads[c0 + j],
                                 &exp_avg[c0 + j], &exp_avg_sq[c0 + j]};
      for (const at::Tensor* x : ts)
        TORCH_CHECK(x->is_cuda() && x->scalar_type() == at::kFloat &&
                        x->is_contiguous() && aligned16(x->data_ptr()) &&
                        x->numel() == params[c0 + j].numel(),
                    "adam_multi: fp32 contiguous 16-B aligned tensors of "
                    "equal size");
      TORCH_CHECK(params[c0 + j].numel() < INT32_MAX, "adam_multi: size");
      check_step(steps[c0 + j], params[c0 + j]);
      T.s[j] = steps[c0 + j].data_ptr<float>();
      T.p[j] = params[c0 + j].data_ptr<float>();
      T.g[j] = grads[c0 + j].data_ptr<float>();
      T.m[j] = exp_avg[c0 + j].data_ptr<float>();
      T.v[j] = exp_avg_sq[c0 + j].data_ptr<float>();
      T.n[j] = (int)params[c0 + j].numel();
      T.first_block[j] = blocks;
      blocks += (T.n[j] + kAdamBlock - 1) / kAdamBlock;
    }
    T.first_block[T.count] = blocks;
    if (blocks == 0) continue;
    hipLaunchKernelGGL(adam_multi_kernel, dim3(blocks), dim3(kAdamThreads), 0,
                       stream(), T, fi, (float)lr,
                       (float)beta1, (float)beta2, (float)eps,
                       (float)weight_decay);
    DGMC_CHECK_LAUNCH();
  }
}

void adam_step_inc(at::TensorList steps,
                   const c10::optional<at::Tensor>& found_inf,
                   const c10::optional<at::Tensor>& flags,
                   const c10::optional<at::Tensor>& skips) {
  const int64_t count = (int64_t)steps.size();
  if (count == 0) return;
  float* fi = nullptr;
  if (found_inf.has_value() && found_inf->defined())
    fi = found_inf->data_ptr<float>();
  const int* fl = nullptr;
  int nflags = 0;
  if (flags.has_value() && flags->defined()) {
    // Only the first 64-parameter chunk folds the flags; later chunks read
    // found_inf, so it must be given.
    TORCH_CHECK(fi != nullptr, "adam_step_inc: flags need found_inf");
    TORCH_CHECK(flags->scalar_type() == at::kInt && flags->is_contiguous() &&
                    flags->device() == steps[0].device(),
                "adam_step_inc: int32 flags on the device");
    fl = flags->data_ptr<int>();
    nflags = (int)flags->numel();
  }
  double* sk = nullptr;
  if (skips.has_value() && skips->defined()) {
    TORCH_CHECK(skips->scalar_type() == at::kDouble && skips->numel() == 1,
                "adam_step_inc: fp64 [1] skip counter");
    sk = skips->data_ptr<double>();
  }
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(steps[0].device());
  for (int64_t c0 = 0; c0 < count; c0 += kAdamMax) {
    StepTable T{};
    T.count = (int)std::min<int64_t>(kAdamMax, count - c0);
    for (int j = 0; j < T.count; ++j) {
      check_step(steps[c0 + j], steps[0]);
      T.s[j] = steps[c0 + j].data_ptr<float>();
    }
    // The flag fold runs once (first launch); later launches read found_inf.
    hipLaunchKernelGGL(adam_step_inc_kernel, dim3(1), dim3(kAdamMax), 0,
                       stream(), T, fi, c0 == 0 ? fl : nullptr, nflags,
                       c0 == 0 ? sk : nullptr);
    DGMC_CHECK_LAUNCH();
  }
}

// ---------------------------------------------------------------------------
// pack_grads: flat[off_i : off_i + n_i] = grads[i] (or 0 for an undefined
// gradient) for every parameter, in ONE launch over a pointer table.
//
// The trainer lets autograd's AccumulateGrad *steal* each parameter's
// freshly computed gradient (p.grad = None before backward) and then packs
// them into the flat all-reduce / optimizer buffer here - instead of keeping
// p.grad as views of a zeroed flat buffer, which costs one zero-fill of the
// whole buffer plus one read-modify-write add kernel per parameter
// (~20 adds of ~5 us each per PascalVOC step).
namespace {
struct PackTable {
  const float* g[kAdamMax];
  float* dst[kAdamMax];
  int n[kAdamMax];
  int first_block[kAdamMax + 1];
  int count;
};
}  // namespace

__global__ __launch_bounds__(kAdamThreads) void pack_grads_kernel(
    const PackTable T, int* __restrict__ flags) {
  const int b = blockIdx.x;
  __shared__ int any;
  if (flags && threadIdx.x == 0) any = 0;
  int bad = 0;
  int ti = 0;
  while (ti + 1 < T.count && T.first_block[ti + 1] <= b) ++ti;
  const int n = T.n[ti];
  const int base = (b - T.first_block[ti]) * kAdamBlock;
  const float* __restrict__ G = T.g[ti];
  float* __restrict__ D = T.dst[ti];
  if (base + kAdamBlock <= n) {
    float4 v[kAdamVec];
#pragma unroll
    for (int u = 0; u < kAdamVec; ++u) {
      const int i = base + 4 * (u * kAdamThreads + threadIdx.x);
      v[u] = G ? *reinterpret_cast<const float4*>(G + i)
               : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < kAdamVec; ++u) {
      const int i = base + 4 * (u * kAdamThreads + threadIdx.x);
      *reinterpret_cast<float4*>(D + i) = v[u];
      bad |= !isfinite(v[u].x) | !isfinite(v[u].y) | !isfinite(v[u].z) |
             !isfinite(v[u].w);
    }
  } else {
    for (int i = base + threadIdx.x; i < min(n, base + kAdamBlock);
         i += kAdamThreads) {
      const float x = G ? G[i] : 0.f;
      D[i] = x;
      bad |= !isfinite(x);
    }
  }
  if (flags) {
    // Per-block non-finite flag (folded by adam_step_inc).
    __syncthreads();
    if (bad) any = 1;      // benign race: every writer stores 1
    __syncthreads();
    if (threadIdx.x == 0) flags[b] = any;
  }
}

// grads[i]: fp32 contiguous 16-B aligned gradient of numel n_i (or None);
// views[i]: the destination fp32 contiguous 16-B aligned view (numel n_i).
// with_flags: also returns int32 per-block non-finite flags of the packed
// gradients (for adam_step_inc's fold; undefined otherwise).
at::Tensor pack_grads(const c10::List<c10::optional<at::Tensor>>& grads,
                      at::TensorList views, bool with_flags) {
  const int64_t count = (int64_t)views.size();
  TORCH_CHECK((int64_t)grads.size() == count,
              "pack_grads: one gradient slot per destination view");
  if (count == 0) return at::Tensor();
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(views[0].device());
  at::Tensor flags;
  if (with_flags) {
    int64_t total = 0;
    for (int64_t j = 0; j < count; ++j)
      total += (views[j].numel() + kAdamBlock - 1) / kAdamBlock;
    // Every block writes its flag: no zero-fill.
    flags = at::empty({total}, views[0].options().dtype(at::kInt));
  }
  int64_t flag_off = 0;
  for (int64_t c0 = 0; c0 < count; c0 += kAdamMax) {
    PackTable T{};
    T.count = (int)std::min<int64_t>(kAdamMax, count - c0);
    int blocks = 0;
    for (int j = 0; j < T.count; ++j) {
      const at::Tensor& d = views[c0 + j];
      TORCH_CHECK(d.is_cuda() && d.scalar_type() == at::kFloat &&
                      d.is_contiguous() && aligned16(d.data_ptr()) &&
                      d.numel() < INT32_MAX,
                  "pack_grads: fp32 contiguous 16-B aligned destination");
      const c10::optional<at::Tensor> g = grads.get(c0 + j);
      const float* gp = nullptr;
      if (g.has_value() && g->defined()) {
        TORCH_CHECK(g->is_cuda() && g->scalar_type() == at::kFloat &&
                        g->is_contiguous() && aligned16(g->data_ptr()) &&
                        g->numel() == d.numel(),
                    "pack_grads: fp32 contiguous 16-B aligned gradient of "
                    "the destination's size");
        gp = g->data_ptr<float>();
      }
      T.g[j] = gp;
      T.dst[j] = d.data_ptr<float>();
      T.n[j] = (int)d.numel();
      T.first_block[j] = blocks;
      blocks += (T.n[j] + kAdamBlock - 1) / kAdamBlock;
    }
    T.first_block[T.count] = blocks;
    if (blocks == 0) continue;
    hipLaunchKernelGGL(pack_grads_kernel, dim3(blocks), dim3(kAdamThreads), 0,
                       stream(), T,
                       with_flags ? flags.data_ptr<int>() + flag_off : nullptr);
    DGMC_CHECK_LAUNCH();
    flag_off += blocks;
  }
  return flags;
}

}  // namespace dgmc
