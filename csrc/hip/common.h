// Shared device helpers for the gfx950 (MI355X, CDNA4) kernels.
//
// * wave64 reductions via __shfl_xor (CDNA wavefront = 64 lanes);
// * bf16/f16/f32 <-> f32 vector load helpers (16-byte per lane loads);
// * bijective XCD-aware block remap: consecutive *logical* blocks land on the
//   same XCD so neighbouring rows (nodes of one graph) share that XCD's L2.
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>
#include <stdint.h>

#include <ATen/ATen.h>
#include <ATen/hip/HIPContext.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>

#define DGMC_CHECK_HIP(expr)                                                   \
  do {                                                                         \
    hipError_t _e = (expr);                                                    \
    TORCH_CHECK(_e == hipSuccess, "HIP error: ", hipGetErrorString(_e));       \
  } while (0)

#define DGMC_CHECK_LAUNCH() DGMC_CHECK_HIP(hipGetLastError())

namespace dgmc {

constexpr int kWave = 64;

// LDS-typed pointers: generic pointers into shared memory compile to flat_*
// accesses (vmcnt + lgkmcnt waits); address_space(3) gives ds_* ops.
#define DGMC_LDS __attribute__((address_space(3)))
constexpr int kNumXcd = 8;

inline hipStream_t stream() { return at::hip::getCurrentHIPStream().stream(); }

// Bijective remap of a linear block id so that blocks b and b+1 share an XCD
// (hardware dispatches block ids round-robin over the 8 XCDs).
__device__ __forceinline__ int xcd_remap(int bid, int nblocks) {
  if (nblocks <= kNumXcd) return bid;
  const int q = nblocks / kNumXcd, r = nblocks % kNumXcd;
  const int xcd = bid % kNumXcd, slot = bid / kNumXcd;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + slot;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}

// DPP lane exchanges (VALU modifiers, no LDS round trip unlike __shfl_xor's
// ds_bpermute).  CTRL: 0xB1 / 0x4E quad_perm xor 1 / xor 2, 0x141
// row_half_mirror, 0x140 row_mirror.  Callers keep EXEC full.
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __builtin_bit_cast(
      float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL,
                                         0xF, 0xF, false));
}
__device__ __forceinline__ float lane_of(float v, int l) {
  return __builtin_bit_cast(
      float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}
// Sum over each aligned group of 4 lanes (every lane gets its group's sum).
__device__ __forceinline__ float quad_sum(float v) {
  v += dpp_mov<0xB1>(v);
  return v + dpp_mov<0x4E>(v);
}
// Whole-wave sum / max: DPP within rows of 16, then the 4 row results by
// readlane (wave-uniform result).
__device__ __forceinline__ float wave_sum_dpp(float v) {
  v = quad_sum(v);
  v += dpp_mov<0x141>(v);
  v += dpp_mov<0x140>(v);
  return (lane_of(v, 0) + lane_of(v, 16)) + (lane_of(v, 32) + lane_of(v, 48));
}
__device__ __forceinline__ float wave_max_dpp(float v) {
  v = fmaxf(v, dpp_mov<0xB1>(v));
  v = fmaxf(v, dpp_mov<0x4E>(v));
  v = fmaxf(v, dpp_mov<0x141>(v));
  v = fmaxf(v, dpp_mov<0x140>(v));
  return fmaxf(fmaxf(lane_of(v, 0), lane_of(v, 16)),
               fmaxf(lane_of(v, 32), lane_of(v, 48)));
}

// ---------------------------------------------------------------------------
// Scalar conversions
// ---------------------------------------------------------------------------
template <typename T> struct Cvt;
template <> struct Cvt<float> {
  __device__ __forceinline__ static float to_f(float v) { return v; }
  __device__ __forceinline__ static float from_f(float v) { return v; }
};
template <> struct Cvt<__hip_bfloat16> {
  __device__ __forceinline__ static float to_f(__hip_bfloat16 v) {
    return __bfloat162float(v);
  }
  __device__ __forceinline__ static __hip_bfloat16 from_f(float v) {
    return __float2bfloat16(v);
  }
};
template <> struct Cvt<__half> {
  __device__ __forceinline__ static float to_f(__half v) {
    return __half2float(v);
  }
  __device__ __forceinline__ static __half from_f(float v) {
    return __float2half(v);
  }
};

// Elements per 16-byte vector access.
template <typename T> struct Vec16 {
  static constexpr int N = 16 / sizeof(T);
};

// Load N consecutive elements (16-byte aligned) into floats.
template <typename T, int N>
__device__ __forceinline__ void load_vec(const T* __restrict__ p, float* out) {
  static_assert(N * sizeof(T) == 16 || N == 1, "vector width");
  if constexpr (N == 1) {
    out[0] = Cvt<T>::to_f(p[0]);
  } else {
    const uint4 raw = *reinterpret_cast<const uint4*>(p);
    const T* e = reinterpret_cast<const T*>(&raw);
#pragma unroll
    for (int k = 0; k < N; ++k) out[k] = Cvt<T>::to_f(e[k]);
  }
}

template <typename T, int N>
__device__ __forceinline__ void store_vec(T* __restrict__ p, const float* v) {
  static_assert(N * sizeof(T) == 16 || N == 1, "vector width");
  if constexpr (N == 1) {
    p[0] = Cvt<T>::from_f(v[0]);
  } else {
    uint4 raw;
    T* e = reinterpret_cast<T*>(&raw);
#pragma unroll
    for (int k = 0; k < N; ++k) e[k] = Cvt<T>::from_f(v[k]);
    *reinterpret_cast<uint4*>(p) = raw;
  }
}

// fp32 -> three bf16 terms x = hi + mid + lo (round-to-nearest per stage;
// the bf16x6 operand planes of slot_gemm_x6.hip).
__device__ __forceinline__ void split3_bf16(float x, __bf16& h, __bf16& m,
                                            __bf16& l) {
  h = (__bf16)x;
  const float r1 = x - (float)h;      // exact
  m = (__bf16)r1;
  l = (__bf16)(r1 - (float)m);        // exact residual, rounded
}

__host__ __device__ inline bool aligned16(const void* p) {
  return (reinterpret_cast<uintptr_t>(p) & 15u) == 0;
}

// CUs left out of the persistent / CU-sized grids (x6 GEMMs, weight
// gradients): under data parallelism RCCL's channel kernels run concurrently
// with the backward and hold CUs; a persistent grid sized to every CU then
// waits on its busiest one.  Set from Python (DGMC_AMD_RESERVE_CUS,
// ops/_backend.py -> set_cu_reserve); 0 by default.
inline int& cu_reserve() {
  static int v = 0;
  return v;
}
// `total` CUs minus the reserve (at least 1).
inline int usable_cus(int total) {
  const int r = cu_reserve();
  return total - r >= 1 ? total - r : 1;
}
// The device's CU count, reserve ignored.  Work DECOMPOSITIONS that fix a
// summation order (split-K chunks, weight-gradient items) are sized from
// this, so results never depend on the reserve; only persistent grid sizes
// use usable_cus().
inline int device_cus(int dev) {
  static int cached[64] = {0};
  if (dev < 0 || dev >= 64) dev = 0;
  if (cached[dev] == 0) {
    hipDeviceProp_t prop;
    DGMC_CHECK_HIP(hipGetDeviceProperties(&prop, dev));
    cached[dev] = prop.multiProcessorCount;
  }
  return cached[dev];
}

// Diagnostic knobs (kernel ablations, relaxed top-k margins, forced split
// counts) exist only in the diagnostic library (`tools/build_native.py
// --diag` -> _C_hip_diag.so, compiled with -DDGMC_DIAG, loaded when
// DGMC_AMD_DIAG=1).  The production library never reads the environment
// for them: it always uses `dflt`, so no stray variable can skip MFMAs or
// shrink a proven error margin.
#ifdef DGMC_DIAG
constexpr bool kDiagBuild = true;
#else
constexpr bool kDiagBuild = false;
#endif
inline int diag_env_int(const char* name, int dflt) {
#ifdef DGMC_DIAG
  const char* e = getenv(name);
  return e ? atoi(e) : dflt;
#else
  (void)name;
  return dflt;
#endif
}

}  // namespace dgmc

// Dispatch over the floating types our kernels accept (f32, bf16, f16).
#define DGMC_DISPATCH_FLOAT(ST, T, ...)                                        \
  [&] {                                                                        \
    switch (ST) {                                                              \
      case at::kFloat: { using T = float; return __VA_ARGS__(); }              \
      case at::kBFloat16: { using T = __hip_bfloat16; return __VA_ARGS__(); }  \
      case at::kHalf: { using T = __half; return __VA_ARGS__(); }              \
      default: TORCH_CHECK(false, "dgmc_amd: unsupported dtype ", ST);         \
    }                                                                          \
  }()
