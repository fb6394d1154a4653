// Runtime controls and the CU-contention micro-benchmark kernel.
//
// * set_cu_reserve(n): CUs the persistent / CU-sized grids leave free
//   (common.h::cu_reserve), so concurrently running RCCL channel kernels do
//   not stretch a grid that expects every CU.
// * cu_hog(blocks, usec): occupies `blocks` CUs for `usec` microseconds -
//   one workgroup per CU (its dynamic LDS exceeds half of a CU's 160 KB),
//   spinning on the constant-rate wall clock and exiting on its own.  Run on
//   a side stream it emulates RCCL channels holding CUs during the backward
//   (tools/bench_cu_reserve.py).
#include "common.h"

namespace dgmc {

namespace {
constexpr int kHogLds = 96 * 1024;   // > 80 KB: one workgroup per CU

__global__ __launch_bounds__(64) void cu_hog_kernel(long long ticks,
                                                    int* __restrict__ done) {
  extern __shared__ int hog_lds[];
  const long long t0 = wall_clock64();
  int spins = 0;
  while (wall_clock64() - t0 < ticks) {
    __builtin_amdgcn_s_sleep(2);
    ++spins;
  }
  hog_lds[threadIdx.x] = spins;
  __syncthreads();
  if (threadIdx.x == 0) done[blockIdx.x] = hog_lds[0] > 0 ? 1 : 2;
}
}  // namespace

int64_t set_cu_reserve(int64_t n) {
  TORCH_CHECK(n >= 0 && n < 1024, "set_cu_reserve: 0 <= n < 1024");
  const int prev = cu_reserve();
  cu_reserve() = (int)n;
  return prev;
}

at::Tensor cu_hog(const at::Tensor& like, int64_t blocks, double usec) {
  TORCH_CHECK(like.is_cuda(), "cu_hog: device tensor for the device");
  TORCH_CHECK(blocks >= 1 && blocks <= 4096 && usec > 0 && usec <= 1e6,
              "cu_hog: 1..4096 blocks, 0 < usec <= 1e6");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(like.device());
  at::Tensor done = at::zeros({blocks}, like.options().dtype(at::kInt));
  int dev = like.device().index();
  int rate_khz = 0;
  DGMC_CHECK_HIP(hipDeviceGetAttribute(
      &rate_khz, hipDeviceAttributeWallClockRate, dev));
  const long long ticks =
      (long long)(usec * 1e-3 * (double)(rate_khz > 0 ? rate_khz : 100000));
  DGMC_CHECK_HIP(hipFuncSetAttribute(
      reinterpret_cast<const void*>(cu_hog_kernel),
      hipFuncAttributeMaxDynamicSharedMemorySize, kHogLds));
  hipLaunchKernelGGL(cu_hog_kernel, dim3((unsigned)blocks), dim3(64), kHogLds,
                     stream(), ticks, done.data_ptr<int>());
  DGMC_CHECK_LAUNCH();
  return done;
}

}  // namespace dgmc
