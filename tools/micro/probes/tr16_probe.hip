// Probe of ds_read_b64_tr_b16 (__builtin_amdgcn_ds_read_tr16_b64_v4i16):
// LDS holds a [16 rows][128 cols] 16-bit image with value r * 256 + c; every
// lane supplies the address of row q = (lane & 15) >> 2, columns
// 4 (lane & 3) .. + 3 of a 4 x 16 block (block column base 16 * (lane >> 4)).
// Prints what each lane receives.
//   hipcc --offload-arch=gfx950 -O2 -o tr16_probe tr16_probe.hip && ./tr16_probe
#include <hip/hip_runtime.h>

#include <cstdio>

typedef short i16x4 __attribute__((ext_vector_type(4)));

__global__ void probe(short* out) {
  __shared__ __attribute__((aligned(16))) short img[16 * 128];
  for (int e = threadIdx.x; e < 16 * 128; e += 64)
    img[e] = (short)((e / 128) * 256 + (e % 128));
  __syncthreads();
  const int lane = threadIdx.x;
  const int q = (lane & 15) >> 2, p = lane & 3, g = lane >> 4;
  const int off = q * 128 + 16 * g + 4 * p;
  const i16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) i16x4*)(img + off));
  for (int e = 0; e < 4; ++e) out[lane * 4 + e] = v[e];
}

int main() {
  short* d;
  if (hipMalloc(&d, 256 * 2) != hipSuccess) return 1;
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
  short h[256];
  if (hipMemcpy(h, d, 512, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  for (int l = 0; l < 64; ++l) {
    printf("lane %2d:", l);
    for (int e = 0; e < 4; ++e)
      printf(" (r%d,c%d)", h[l * 4 + e] / 256, h[l * 4 + e] % 256);
    printf("\n");
  }
  return 0;
}
