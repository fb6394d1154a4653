// Numerics probe: fp32 GEMM emulated on bf16 MFMA ("bf16x6": every fp32
// operand split into three bf16 terms hi + mid + lo, the six products whose
// order is >= 2^-16 accumulated in fp32) against the exact f32-input MFMA
// (v_mfma_f32_32x32x2_f32, a k-ordered fmaf chain) and an fp64 host oracle.
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/split_probe split_bf16_numerics.hip
//   ./split_probe            (prints one JSON line per K)
//
// One wave computes one 32 x 32 block C = A[32, K] B[K, 32]; 64 blocks of
// independent random N(0, 1) data per K.  Variants:
//   f32   : 32x32x2 f32 MFMA chain over k (the current exact kernels);
//   x6    : bf16 32x32x16 MFMA, one accumulator, per k16 step the five small
//           products first, then hi*hi;
//   x6d   : two accumulators (hi*hi | the five small products), summed at
//           the end;
//   x6p   : one accumulator, but each k-chunk of 64 is first summed in a
//           fresh accumulator before being added (pairwise-style blocking).
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

#define CHECK(x)                                                         \
  do {                                                                   \
    hipError_t e = (x);                                                  \
    if (e != hipSuccess) {                                               \
      fprintf(stderr, "HIP %s at %d\n", hipGetErrorString(e), __LINE__); \
      exit(1);                                                           \
    }                                                                    \
  } while (0)

// A: [nb][32][K] row-major, B: [nb][K][32] (k-major rows).  Split planes
// Ah/Am/Al [nb][32][K] bf16, Bh/Bm/Bl [nb][32][K] bf16 (stored B^T so both
// operands read 8 consecutive k).
__global__ void f32_kernel(const float* A, const float* B, int K, float* C) {
  const int b = blockIdx.x, lane = threadIdx.x;
  const float* a = A + (size_t)b * 32 * K;
  const float* bb = B + (size_t)b * K * 32;
  f32x16 acc = {};
  const int i = lane & 31, h = lane >> 5;
  for (int k = 0; k < K; k += 2)
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i * K + k + h],
                                               bb[(k + h) * 32 + i], acc, 0, 0,
                                               0);
  for (int r = 0; r < 16; ++r) {
    const int row = (r & 3) + 8 * (r >> 2) + 4 * h, col = i;
    C[(size_t)b * 1024 + row * 32 + col] = acc[r];
  }
}

__device__ inline bf16x8 ld8(const __bf16* p) {
  return *reinterpret_cast<const bf16x8*>(p);
}

template <int MODE>
__global__ void x6_kernel(const __bf16* Ah, const __bf16* Am,
                          const __bf16* Al, const __bf16* Bh,
                          const __bf16* Bm, const __bf16* Bl, int K,
                          float* C) {
  const int b = blockIdx.x, lane = threadIdx.x;
  const int i = lane & 31, h = lane >> 5;
  const size_t off = (size_t)b * 32 * K + (size_t)i * K + 8 * h;
  f32x16 acc = {}, acc2 = {}, part = {};
  for (int k = 0; k < K; k += 16) {
    const bf16x8 ah = ld8(Ah + off + k), am = ld8(Am + off + k),
                 al = ld8(Al + off + k);
    const bf16x8 bh = ld8(Bh + off + k), bm = ld8(Bm + off + k),
                 bl = ld8(Bl + off + k);
    f32x16& s = MODE == 1 ? acc2 : (MODE == 2 ? part : acc);
    s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, s, 0, 0, 0);
    s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, s, 0, 0, 0);
    s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bm, s, 0, 0, 0);
    s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bh, s, 0, 0, 0);
    s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bm, s, 0, 0, 0);
    if (MODE == 1) {
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc, 0, 0, 0);
    } else {
      s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, s, 0, 0, 0);
    }
    if (MODE == 2 && ((k + 16) % 64 == 0 || k + 16 >= K)) {
      for (int r = 0; r < 16; ++r) {
        acc[r] += part[r];
        part[r] = 0.f;
      }
    }
  }
  for (int r = 0; r < 16; ++r) {
    const int row = (r & 3) + 8 * (r >> 2) + 4 * h, col = i;
    const float v = MODE == 1 ? acc[r] + acc2[r] : acc[r];
    C[(size_t)b * 1024 + row * 32 + col] = v;
  }
}

static __bf16 to_bf16(float x) {
  // round to nearest even
  uint32_t u;
  memcpy(&u, &x, 4);
  const uint32_t lsb = (u >> 16) & 1u;
  u += 0x7fffu + lsb;
  const uint16_t hbits = (uint16_t)(u >> 16);
  __bf16 r;
  memcpy(&r, &hbits, 2);
  return r;
}
static float from_bf16(__bf16 v) {
  uint16_t hbits;
  memcpy(&hbits, &v, 2);
  const uint32_t u = (uint32_t)hbits << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}
static void split3(float x, __bf16* h, __bf16* m, __bf16* l) {
  *h = to_bf16(x);
  const float r1 = x - from_bf16(*h);
  *m = to_bf16(r1);
  const float r2 = r1 - from_bf16(*m);
  *l = to_bf16(r2);
}

int main(int argc, char** argv) {
  const int nb = 64;
  const int Ks[] = {128, 256, 1024, 4096, 16384};
  for (int K : Ks) {
    std::mt19937 gen(1234 + K);
    std::normal_distribution<float> nd(0.f, 1.f);
    std::vector<float> A((size_t)nb * 32 * K), B((size_t)nb * K * 32);
    for (auto& v : A) v = nd(gen);
    for (auto& v : B) v = nd(gen);
    // Split planes (B stored transposed [32][K]).
    std::vector<__bf16> ah(A.size()), am(A.size()), al(A.size()),
        bh(B.size()), bm(B.size()), bl(B.size());
    for (size_t t = 0; t < A.size(); ++t) split3(A[t], &ah[t], &am[t], &al[t]);
    for (int b = 0; b < nb; ++b)
      for (int k = 0; k < K; ++k)
        for (int j = 0; j < 32; ++j) {
          const size_t src = (size_t)b * K * 32 + (size_t)k * 32 + j;
          const size_t dst = (size_t)b * 32 * K + (size_t)j * K + k;
          split3(B[src], &bh[dst], &bm[dst], &bl[dst]);
        }
    // fp64 oracle + sum |a||b|.
    std::vector<double> ref((size_t)nb * 1024), mag((size_t)nb * 1024);
    for (int b = 0; b < nb; ++b)
      for (int r = 0; r < 32; ++r)
        for (int c = 0; c < 32; ++c) {
          double s = 0, m = 0;
          for (int k = 0; k < K; ++k) {
            const double p = (double)A[(size_t)b * 32 * K + r * K + k] *
                             (double)B[(size_t)b * K * 32 + k * 32 + c];
            s += p;
            m += fabs(p);
          }
          ref[(size_t)b * 1024 + r * 32 + c] = s;
          mag[(size_t)b * 1024 + r * 32 + c] = m;
        }
    float *dA, *dB, *dC;
    __bf16* d[6];
    CHECK(hipMalloc(&dA, A.size() * 4));
    CHECK(hipMalloc(&dB, B.size() * 4));
    CHECK(hipMalloc(&dC, (size_t)nb * 1024 * 4));
    const std::vector<__bf16>* planes[6] = {&ah, &am, &al, &bh, &bm, &bl};
    for (int p = 0; p < 6; ++p) {
      CHECK(hipMalloc(&d[p], planes[p]->size() * 2));
      CHECK(hipMemcpy(d[p], planes[p]->data(), planes[p]->size() * 2,
                      hipMemcpyHostToDevice));
    }
    CHECK(hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice));
    std::vector<float> C((size_t)nb * 1024);
    printf("{\"K\": %d", K);
    for (int v = 0; v < 4; ++v) {
      if (v == 0)
        hipLaunchKernelGGL(f32_kernel, dim3(nb), dim3(64), 0, 0, dA, dB, K,
                           dC);
      else if (v == 1)
        hipLaunchKernelGGL(x6_kernel<0>, dim3(nb), dim3(64), 0, 0, d[0], d[1],
                           d[2], d[3], d[4], d[5], K, dC);
      else if (v == 2)
        hipLaunchKernelGGL(x6_kernel<1>, dim3(nb), dim3(64), 0, 0, d[0], d[1],
                           d[2], d[3], d[4], d[5], K, dC);
      else
        hipLaunchKernelGGL(x6_kernel<2>, dim3(nb), dim3(64), 0, 0, d[0], d[1],
                           d[2], d[3], d[4], d[5], K, dC);
      CHECK(hipGetLastError());
      CHECK(hipMemcpy(C.data(), dC, C.size() * 4, hipMemcpyDeviceToHost));
      double maxabs = 0, maxrel = 0, rms = 0;
      for (size_t t = 0; t < C.size(); ++t) {
        const double e = fabs((double)C[t] - ref[t]);
        maxabs = fmax(maxabs, e);
        maxrel = fmax(maxrel, e / mag[t]);
        rms += e * e;
      }
      rms = sqrt(rms / C.size());
      const char* name[] = {"f32", "x6", "x6d", "x6p"};
      printf(", \"%s\": {\"max_abs\": %.3e, \"max_rel_mag\": %.3e, "
             "\"rms\": %.3e}",
             name[v], maxabs, maxrel, rms);
    }
    printf("}\n");
    fflush(stdout);
    hipFree(dA);
    hipFree(dB);
    hipFree(dC);
    for (int p = 0; p < 6; ++p) hipFree(d[p]);
  }
  return 0;
}
