// ds_read_b64_tr_b16 with arbitrary per-lane addresses: LDS[e] = e; lane l
// supplies element address a[l] (multiple of 4); prints, for lanes 0..15,
// the element indices received - i.e. which lane's address fed each
// element.
#include <hip/hip_runtime.h>

#include <cstdio>

typedef short i16x4 __attribute__((ext_vector_type(4)));

__global__ void probe(const int* addr, short* out) {
  __shared__ __attribute__((aligned(16))) short img[4096];
  for (int e = threadIdx.x; e < 4096; e += 64) img[e] = (short)e;
  __syncthreads();
  const int lane = threadIdx.x;
  const i16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) i16x4*)(img + addr[lane]));
  for (int e = 0; e < 4; ++e) out[lane * 4 + e] = v[e];
}

int main() {
  int ha[64];
  for (int l = 0; l < 64; ++l) ha[l] = 4 * ((l * 37 + 11) % 512);   // distinct
  int* da;
  short* d;
  if (hipMalloc(&da, 256) != hipSuccess || hipMalloc(&d, 512) != hipSuccess)
    return 1;
  if (hipMemcpy(da, ha, 256, hipMemcpyHostToDevice) != hipSuccess) return 1;
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, da, d);
  short h[256];
  if (hipMemcpy(h, d, 512, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  for (int l = 0; l < 16; ++l) {
    printf("lane %2d (addr %4d):", l, ha[l]);
    for (int e = 0; e < 4; ++e) {
      const int v = h[l * 4 + e];
      int src = -1;
      for (int k = 0; k < 64; ++k)
        if (v >= ha[k] && v < ha[k] + 4) src = k;
      printf(" [elem %4d = lane %2d word %d]", v, src, src >= 0 ? v - ha[src] : -1);
    }
    printf("\n");
  }
  return 0;
}
