// ds_read_b64_tr_b16 with the bf16x6 weight-gradient kernel's addresses
// (lane 4q + p -> row q, 16-B chunk (p >> 1) ^ swz(q), +8 B for odd p; rows
// of 256 B) on an image whose element e holds e.  Variants: (a) one wave,
// image written by ds_write; (b) four waves; (c) image filled by
// global_load_lds_dwordx4.  Prints lane 0 / 1 / 4 received elements.
#include <hip/hip_runtime.h>

#include <cstdio>

typedef short i16x4 __attribute__((ext_vector_type(4)));

__device__ int swz(int r) { return ((r & 3) << 2) | ((r >> 2) & 3); }

__global__ void probe(const short* gsrc, short* out, int mode) {
  __shared__ __attribute__((aligned(16))) short img[16 * 128];
  const int tid = threadIdx.x, lane = tid & 63;
  if (mode == 2) {
    if (tid < 64) {
      // 4 DMAs of 1 KB: lane L -> row 4 d + L / 16, 16 B at chunk L % 16
      for (int d = 0; d < 4; ++d) {
        const short* g = gsrc + (4 * d + lane / 16) * 128 + 8 * (lane % 16);
        const unsigned m0 = __builtin_amdgcn_readfirstlane(
            (unsigned)(uintptr_t)(img + 4 * d * 128));
        asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off"
                     :: "v"(g), "s"(m0) : "memory", "m0");
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  } else {
    for (int e = tid; e < 16 * 128; e += blockDim.x) img[e] = (short)e;
  }
  __syncthreads();
  const int q = (lane & 15) >> 2, p = lane & 3;
  const int chunk = (p >> 1) ^ swz(q);
  const int off = q * 128 + 8 * chunk + 4 * (p & 1);
  const i16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) i16x4*)(img + off));
  if (tid < 64)
    for (int e = 0; e < 4; ++e) out[lane * 4 + e] = v[e];
}

int main() {
  short hs[16 * 128];
  for (int e = 0; e < 16 * 128; ++e) hs[e] = (short)e;
  short *gs, *d;
  if (hipMalloc(&gs, sizeof(hs)) != hipSuccess || hipMalloc(&d, 512) != hipSuccess)
    return 1;
  if (hipMemcpy(gs, hs, sizeof(hs), hipMemcpyHostToDevice) != hipSuccess) return 1;
  const char* names[3] = {"(a) 1 wave ds_write", "(b) 4 waves ds_write",
                          "(c) 1 wave LDS-DMA"};
  for (int mode = 0; mode < 3; ++mode) {
    hipLaunchKernelGGL(probe, dim3(1), dim3(mode == 1 ? 256 : 64), 0, 0, gs, d,
                       mode);
    short h[256];
    if (hipMemcpy(h, d, 512, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    printf("%s\n", names[mode]);
    for (int l : {0, 1, 4, 5}) {
      printf("  lane %d:", l);
      for (int e = 0; e < 4; ++e) {
        const int v = h[l * 4 + e];
        printf(" (row %d, phys col %d)", v / 128, v % 128);
      }
      printf("\n");
    }
  }
  return 0;
}
