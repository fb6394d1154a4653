// Micro-benchmark: issue rate of v_mfma_f32_32x32x2_f32 on gfx950.
//   mode 0: 4 independent accumulators, operands in registers
//   mode 1: + one ds_read_b32 per operand per k-step (LDS fragments)
//   mode 2: + a block barrier every 16 k-steps (GEMM chunk structure)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int MODE>
__global__ __launch_bounds__(256) void k(float* out, int iters) {
  __shared__ float lds[4096 + 64];
  const int lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < 4096 + 64; i += 256) lds[i] = 0.001f * i;
  __syncthreads();
  f32x16 acc[4] = {};
  float a0 = lane * 1e-3f, a1 = a0 + 1, b0 = a0 + 2, b1 = a0 + 3;
  for (int it = 0; it < iters; ++it) {
    if (MODE >= 1) {
      const int o = (it * 64 + lane) & 4095;
      a0 = lds[o]; a1 = lds[o + 32]; b0 = lds[o + 1]; b1 = lds[o + 33];
    }
    acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0], 0, 0, 0);
    acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[1], 0, 0, 0);
    acc[2] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[2], 0, 0, 0);
    acc[3] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[3], 0, 0, 0);
    if (MODE >= 2 && (it & 15) == 15) __syncthreads();
  }
  float s = 0;
  for (int j = 0; j < 4; ++j)
    for (int r = 0; r < 16; ++r) s += acc[j][r];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int MODE>
void run(int blocks, int iters) {
  float* out;
  hipMalloc(&out, blocks * 256 * 4);
  hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(256), 0, 0, out, iters);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(256), 0, 0, out, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double flop = 2.0 * 32 * 32 * 2 * 4 * (double)iters * blocks * 4;
  printf("mode %d blocks %5d iters %6d: %8.3f ms  %7.1f TF/s\n", MODE, blocks,
         iters, ms, flop / ms / 1e9);
  hipFree(out);
}

int main() {
  for (int b : {256, 512, 768, 1024}) run<0>(b, 4096);
  for (int b : {256, 512, 768, 1024}) run<1>(b, 4096);
  for (int b : {256, 512, 768, 1024}) run<2>(b, 4096);
  return 0;
}
