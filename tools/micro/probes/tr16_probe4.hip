// Two / four back-to-back ds_read_b64_tr_b16 (rows 0-3 and 4-7 of a
// [16][128] 16-bit image holding row index * 1000 + col), lane 0/4 results.
#include <hip/hip_runtime.h>

#include <cstdio>

typedef short i16x4 __attribute__((ext_vector_type(4)));
#define LDS __attribute__((address_space(3)))

__global__ void probe(short* out, int mode) {
  __shared__ __attribute__((aligned(16))) short img[16 * 128];
  for (int e = threadIdx.x; e < 16 * 128; e += 64)
    img[e] = (short)((e / 128) * 1000 + e % 128);
  __syncthreads();
  const int lane = threadIdx.x;
  const int q = (lane & 15) >> 2, p = lane & 3;
  const int o0 = q * 128 + 4 * p, o1 = (4 + q) * 128 + 4 * p;
  i16x4 a, b;
  if (mode == 0) {
    a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS i16x4*)(img + o0));
    b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS i16x4*)(img + o1));
  } else {
    a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS i16x4*)(img + o0));
    __builtin_amdgcn_s_waitcnt(0xc07f);
    b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS i16x4*)(img + o1));
  }
  for (int e = 0; e < 4; ++e) {
    out[lane * 8 + e] = a[e];
    out[lane * 8 + 4 + e] = b[e];
  }
}

int main() {
  short* d;
  if (hipMalloc(&d, 1024) != hipSuccess) return 1;
  for (int mode = 0; mode < 2; ++mode) {
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, mode);
    short h[512];
    if (hipMemcpy(h, d, 1024, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    for (int l : {0, 4}) {
      printf("mode %d lane %d:", mode, l);
      for (int e = 0; e < 8; ++e) printf(" %d", h[l * 8 + e]);
      printf("\n");
    }
  }
  return 0;
}
