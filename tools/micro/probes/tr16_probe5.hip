// ds_read_b64_tr_b16 on DYNAMIC LDS: allocation 32 KB vs 80 KB, image at
// offset 0 and at 40 KB.  Prints lane 0's 4 elements (want rows 0..3).
#include <hip/hip_runtime.h>

#include <cstdio>

typedef short i16x4 __attribute__((ext_vector_type(4)));
#define LDS __attribute__((address_space(3)))

__global__ void probe(short* out, int base) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  short* img = (short*)(smem + base);
  for (int e = threadIdx.x; e < 16 * 128; e += blockDim.x)
    img[e] = (short)((e / 128) * 1000 + e % 128);
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int q = (lane & 15) >> 2, p = lane & 3;
  const int o0 = q * 128 + 4 * p;
  const i16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (LDS i16x4*)((LDS short*)img + o0));
  if (threadIdx.x < 64)
    for (int e = 0; e < 4; ++e) out[lane * 4 + e] = a[e];
}

int main() {
  short* d;
  if (hipMalloc(&d, 512) != hipSuccess) return 1;
  if (hipFuncSetAttribute((const void*)probe,
                          hipFuncAttributeMaxDynamicSharedMemorySize,
                          80 * 1024) != hipSuccess)
    return 2;
  const int cfg[4][3] = {{32 * 1024, 0, 64}, {80 * 1024, 0, 64},
                         {80 * 1024, 40 * 1024, 64}, {80 * 1024, 0, 256}};
  for (auto& c : cfg) {
    hipLaunchKernelGGL(probe, dim3(1), dim3(c[2]), c[0], 0, d, c[1]);
    short h[256];
    if (hipMemcpy(h, d, 512, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    printf("lds %d base %d threads %d: lane0 %d %d %d %d  lane4 %d %d %d %d\n",
           c[0], c[1], c[2], h[0], h[1], h[2], h[3], h[16], h[17], h[18], h[19]);
  }
  return 0;
}
