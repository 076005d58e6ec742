// Diagnostic: does v_mfma_f32_16x16x16_bf16 / 16x16x32_bf16 sum its K
// products (+ C) exactly before one rounding, or in fp32 steps?  Row 0 x col 0
// gets products {1, 2^-30, -1} placed at different K slots; exact = 2^-30.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

static unsigned short bf(float v) { unsigned u; memcpy(&u, &v, 4); return (unsigned short)(u >> 16); }

__global__ void k16(const unsigned short *A, const unsigned short *B, float c0, float *out) {
  const int l = threadIdx.x;
  s16x4 a, b;
  for (int j = 0; j < 4; ++j) { a[j] = A[(l & 15) * 16 + 4 * (l >> 4) + j]; b[j] = B[(4 * (l >> 4) + j) * 16 + (l & 15)]; }
  f32x4 c = {0, 0, 0, 0};
  if (l == 0) c[0] = c0;
  f32x4 d = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0);
  if (l == 0) out[0] = d[0];
}
__global__ void k32(const unsigned short *A, const unsigned short *B, float c0, float *out) {
  const int l = threadIdx.x;
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) {
    unsigned short ua = A[(l & 15) * 32 + 8 * (l >> 4) + j], ub = B[(8 * (l >> 4) + j) * 16 + (l & 15)];
    a[j] = __builtin_bit_cast(__bf16, ua); b[j] = __builtin_bit_cast(__bf16, ub);
  }
  f32x4 c = {0, 0, 0, 0};
  if (l == 0) c[0] = c0;
  f32x4 d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  if (l == 0) out[0] = d[0];
}

int main() {
  unsigned short *A, *B; float *out;
  hipMalloc(&A, 16 * 32 * 2); hipMalloc(&B, 32 * 16 * 2); hipMalloc(&out, 4);
  const float vals[3] = {1.0f, 0x1p-30f, -1.0f};
  const int K[2] = {16, 32};
  for (int which = 0; which < 2; ++which) {
    const int KK = K[which];
    int slots[][3] = {{0, 1, 2}, {2, 1, 0}, {0, 5, 11}, {0, 15, 7}, {3, 8, 13}, {0, 20, 31}, {31, 0, 17}};
    for (auto &s : slots) {
      if (s[0] >= KK || s[1] >= KK || s[2] >= KK) continue;
      unsigned short hA[16 * 32] = {0}, hB[32 * 16] = {0};
      for (int t = 0; t < 3; ++t) { hA[0 * KK + s[t]] = bf(vals[t]); hB[s[t] * 16 + 0] = bf(1.0f); }
      hipMemcpy(A, hA, sizeof(hA), hipMemcpyHostToDevice); hipMemcpy(B, hB, sizeof(hB), hipMemcpyHostToDevice);
      float r;
      if (which == 0) hipLaunchKernelGGL(k16, dim3(1), dim3(64), 0, 0, A, B, 0.f, out);
      else hipLaunchKernelGGL(k32, dim3(1), dim3(64), 0, 0, A, B, 0.f, out);
      hipMemcpy(&r, out, 4, hipMemcpyDeviceToHost);
      printf("K=%d slots(1,2^-30,-1)=(%d,%d,%d) C=0: %g  (exact 9.31e-10)\n", KK, s[0], s[1], s[2], r);
    }
    // C participates: products {2^-30 at slot 0, -1 at slot 1}, C = 1
    unsigned short hA[16 * 32] = {0}, hB[32 * 16] = {0};
    hA[0] = bf(0x1p-30f); hA[1] = bf(-1.0f); hB[0] = bf(1.0f); hB[16] = bf(1.0f);
    hipMemcpy(A, hA, sizeof(hA), hipMemcpyHostToDevice); hipMemcpy(B, hB, sizeof(hB), hipMemcpyHostToDevice);
    float r;
    if (which == 0) hipLaunchKernelGGL(k16, dim3(1), dim3(64), 0, 0, A, B, 1.f, out);
    else hipLaunchKernelGGL(k32, dim3(1), dim3(64), 0, 0, A, B, 1.f, out);
    hipMemcpy(&r, out, 4, hipMemcpyDeviceToHost);
    printf("K=%d products(2^-30,-1) + C=1: %g (exact 9.31e-10)\n", KK, r);
    // C small: products {1, -1}, C = 2^-30
    memset(hA, 0, sizeof(hA)); memset(hB, 0, sizeof(hB));
    hA[0] = bf(1.0f); hA[1] = bf(-1.0f); hB[0] = bf(1.0f); hB[16] = bf(1.0f);
    hipMemcpy(A, hA, sizeof(hA), hipMemcpyHostToDevice); hipMemcpy(B, hB, sizeof(hB), hipMemcpyHostToDevice);
    if (which == 0) hipLaunchKernelGGL(k16, dim3(1), dim3(64), 0, 0, A, B, 0x1p-30f, out);
    else hipLaunchKernelGGL(k32, dim3(1), dim3(64), 0, 0, A, B, 0x1p-30f, out);
    hipMemcpy(&r, out, 4, hipMemcpyDeviceToHost);
    printf("K=%d products(1,-1) + C=2^-30: %g (exact 9.31e-10)\n", KK, r);
    // C = 1 + 2^-23 (1 ulp), products -1: exact 2^-23; and C=1, products (-1, 2^-24, 2^-24)
    memset(hA, 0, sizeof(hA)); memset(hB, 0, sizeof(hB));
    hA[0] = bf(-1.0f); hA[1] = bf(0x1p-24f); hA[2] = bf(0x1p-24f); hB[0] = hB[16] = hB[32] = bf(1.0f);
    hipMemcpy(A, hA, sizeof(hA), hipMemcpyHostToDevice); hipMemcpy(B, hB, sizeof(hB), hipMemcpyHostToDevice);
    if (which == 0) hipLaunchKernelGGL(k16, dim3(1), dim3(64), 0, 0, A, B, 1.0f, out);
    else hipLaunchKernelGGL(k32, dim3(1), dim3(64), 0, 0, A, B, 1.0f, out);
    hipMemcpy(&r, out, 4, hipMemcpyDeviceToHost);
    printf("K=%d C=1 + products(-1, 2^-24, 2^-24): %g (exact 1.19e-07)\n", KK, r);
  }
  return 0;
}
