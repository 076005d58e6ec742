// Microbenchmark (diagnostic): per-instruction throughput of the ops the
// RotatE kernel is built from, measured with every CU busy, and the in-kernel
// shader clock (s_memtime against the 100 MHz s_memrealtime).
// Build: hipcc --offload-arch=gfx950 -O3 -mllvm -amdgpu-mfma-vgpr-form valu_rates.hip -o valu_rates
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int ITERS = 4096;

__device__ __forceinline__ void stamp(unsigned long long *clk, int slot) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    clk[2 * slot] = __builtin_amdgcn_s_memtime();
    clk[2 * slot + 1] = __builtin_amdgcn_s_memrealtime();
  }
}

__global__ void k_fma(float *out, unsigned long long *clk, float x) {
  stamp(clk, 0);
  float a[8];
  for (int j = 0; j < 8; ++j) a[j] = x + threadIdx.x + j;
  for (int i = 0; i < ITERS; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = fmaf(a[j], 0.999f, 0.001f);
  float s = 0; for (int j = 0; j < 8; ++j) s += a[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  stamp(clk, 1);
}
__global__ void k_sqrt(float *out, unsigned long long *clk, float x) {
  stamp(clk, 0);
  float a[8];
  for (int j = 0; j < 8; ++j) a[j] = x + threadIdx.x + j;
  for (int i = 0; i < ITERS; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = __builtin_amdgcn_sqrtf(a[j]);
  float s = 0; for (int j = 0; j < 8; ++j) s += a[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  stamp(clk, 1);
}
__global__ void k_sqrt_add(float *out, unsigned long long *clk, float x) {
  stamp(clk, 0);
  float a[8], acc[8];
  for (int j = 0; j < 8; ++j) { a[j] = x + threadIdx.x + j; acc[j] = 0; }
  for (int i = 0; i < ITERS; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) { acc[j] += __builtin_amdgcn_sqrtf(a[j]); a[j] += 1.0f; }
  float s = 0; for (int j = 0; j < 8; ++j) s += acc[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  stamp(clk, 1);
}
__global__ void k_mfma(float *out, unsigned long long *clk, float x) {
  stamp(clk, 0);
  f32x4 c[4];
  for (int j = 0; j < 4; ++j) c[j] = (f32x4){0, 0, 0, 0};
  float a = x + threadIdx.x, b = x - threadIdx.x;
  for (int i = 0; i < ITERS; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) c[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c[j], 0, 0, 0);
  float s = 0; for (int j = 0; j < 4; ++j) s += c[j][0] + c[j][1] + c[j][2] + c[j][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  stamp(clk, 1);
}
// the RotatE inner pattern: per tile one MFMA (fresh accumulator) then
// sqrt(|s|) + add of its 4 results; NT independent tiles per iteration
template <int NT, bool ADD>
__global__ void k_mfma_sqrt(float *out, unsigned long long *clk, float x) {
  stamp(clk, 0);
  f32x4 acc[NT];
  for (int j = 0; j < NT; ++j) acc[j] = (f32x4){0, 0, 0, 0};
  float a = x + threadIdx.x, b[NT];
  for (int j = 0; j < NT; ++j) b[j] = x - threadIdx.x + j;
  for (int i = 0; i < ITERS / 4; ++i) {
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const f32x4 s = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b[j], (f32x4){0, 0, 0, 0}, 0, 0, 0);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (ADD) acc[j][q] += __builtin_amdgcn_sqrtf(__builtin_fabsf(s[q]));
        else acc[j][q] = __builtin_amdgcn_sqrtf(__builtin_fabsf(s[q] + acc[j][q]));
      }
    }
    a += 1.0f;
  }
  float s = 0; for (int j = 0; j < NT; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  stamp(clk, 1);
}

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
// same pattern on the bf16 matrix pipe (16x16x32: one MFMA per 4 wave-terms)
template <int NT>
__global__ void k_bf16_sqrt(float *out, unsigned long long *clk, float x) {
  stamp(clk, 0);
  f32x4 acc[NT];
  for (int j = 0; j < NT; ++j) acc[j] = (f32x4){0, 0, 0, 0};
  bf16x8 a, b[NT];
  for (int q = 0; q < 8; ++q) a[q] = (__bf16)(x + threadIdx.x + q);
  for (int j = 0; j < NT; ++j)
    for (int q = 0; q < 8; ++q) b[j][q] = (__bf16)(x - threadIdx.x + j + q);
  for (int i = 0; i < ITERS / 4; ++i) {
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const f32x4 s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b[j], (f32x4){0, 0, 0, 0}, 0, 0, 0);
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[j][q] += __builtin_amdgcn_sqrtf(__builtin_fabsf(s[q]));
    }
    a[0] = a[0] + (__bf16)1.0f;
  }
  float s = 0; for (int j = 0; j < NT; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  stamp(clk, 1);
}
typedef short s16x4 __attribute__((ext_vector_type(4)));
// 16x16x16 bf16 (K = 16, 2 VGPRs per operand)
template <int NT>
__global__ void k_bf16k16_sqrt(float *out, unsigned long long *clk, float x) {
  stamp(clk, 0);
  f32x4 acc[NT];
  for (int j = 0; j < NT; ++j) acc[j] = (f32x4){0, 0, 0, 0};
  s16x4 a, b[NT];
  for (int q = 0; q < 4; ++q) a[q] = (short)(0x3f80 + threadIdx.x + q);
  for (int j = 0; j < NT; ++j)
    for (int q = 0; q < 4; ++q) b[j][q] = (short)(0x3f80 + j + q);
  for (int i = 0; i < ITERS / 4; ++i) {
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const f32x4 s = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b[j], (f32x4){0, 0, 0, 0}, 0, 0, 0);
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[j][q] += __builtin_amdgcn_sqrtf(__builtin_fabsf(s[q]));
    }
    a[0] += 1;
  }
  float s = 0; for (int j = 0; j < NT; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  stamp(clk, 1);
}
__global__ void k_bf16k16(float *out, unsigned long long *clk, float x) {
  stamp(clk, 0);
  f32x4 c[4];
  for (int j = 0; j < 4; ++j) c[j] = (f32x4){0, 0, 0, 0};
  s16x4 a, b;
  for (int q = 0; q < 4; ++q) { a[q] = (short)(0x3f80 + threadIdx.x + q); b[q] = (short)(0x3f80 + q); }
  for (int i = 0; i < ITERS; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) c[j] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c[j], 0, 0, 0);
  float s = 0; for (int j = 0; j < 4; ++j) s += c[j][0] + c[j][1] + c[j][2] + c[j][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  stamp(clk, 1);
}
// 32x32x16 bf16: two MFMAs (K = 32) per 32x32 tile = 16 wave-terms
template <int NT>
__global__ void k_bf16_32_sqrt(float *out, unsigned long long *clk, float x) {
  stamp(clk, 0);
  f32x16 acc[NT];
  for (int j = 0; j < NT; ++j) for (int q = 0; q < 16; ++q) acc[j][q] = 0;
  bf16x8 a, b[NT];
  for (int q = 0; q < 8; ++q) a[q] = (__bf16)(x + threadIdx.x + q);
  for (int j = 0; j < NT; ++j)
    for (int q = 0; q < 8; ++q) b[j][q] = (__bf16)(x - threadIdx.x + j + q);
  for (int i = 0; i < ITERS / 16; ++i) {
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      f32x16 z;
      for (int q = 0; q < 16; ++q) z[q] = 0;
      f32x16 s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b[j], z, 0, 0, 0);
      s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[j], a, s, 0, 0, 0);
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[j][q] += __builtin_amdgcn_sqrtf(__builtin_fabsf(s[q]));
    }
    a[0] = a[0] + (__bf16)1.0f;
  }
  float s = 0; for (int j = 0; j < NT; ++j) for (int q = 0; q < 16; ++q) s += acc[j][q];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  stamp(clk, 1);
}

typedef float f32x2 __attribute__((ext_vector_type(2)));
__global__ void k_pkfma(float *out, unsigned long long *clk, float x) {
  stamp(clk, 0);
  f32x2 a[8];
  for (int j = 0; j < 8; ++j) a[j] = (f32x2){x + threadIdx.x + j, x - j};
  const f32x2 m = {0.999f, 0.998f}, c = {0.001f, 0.002f};
  for (int i = 0; i < ITERS; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = __builtin_elementwise_fma(a[j], m, c);
  float s = 0; for (int j = 0; j < 8; ++j) s += a[j][0] + a[j][1];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  stamp(clk, 1);
}
// the direct RotatE term: sub, sub, mul, fma, [sqrt], add per term; the query
// side in SGPRs (kernel argument array) or VGPRs
template <bool SQRT, bool SGPR>
__global__ void k_direct(float *out, unsigned long long *clk, float x) {
  stamp(clk, 0);
  float acc[16], a = x + threadIdx.x, b = x - threadIdx.x;
  float qx[16], qy[16];
  for (int j = 0; j < 16; ++j) {
    acc[j] = 0;
    qx[j] = SGPR ? x * j : x * j + threadIdx.x;
    qy[j] = SGPR ? x + j : x + j - threadIdx.x;
  }
  for (int i = 0; i < ITERS / 2; ++i) {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const float dx = qx[j] - a;
      const float dy = qy[j] - b;
      const float s = fmaf(dx, dx, dy * dy);
      acc[j] += SQRT ? __builtin_amdgcn_sqrtf(s) : s;
    }
    a += 1.0f;
    b -= 1.0f;
  }
  float s = 0; for (int j = 0; j < 16; ++j) s += acc[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  stamp(clk, 1);
}

// (e) sqrt on last iteration's value (no same-iteration dependency): software pipelined
__global__ void k_direct_pipe(float *out, unsigned long long *clk, float x) {
  stamp(clk, 0);
  float acc[16], sp[16], a = x + threadIdx.x, b = x - threadIdx.x;
  float qx[16], qy[16];
  for (int j = 0; j < 16; ++j) { acc[j] = 0; sp[j] = 1.f + j; qx[j] = x * j + threadIdx.x; qy[j] = x + j - threadIdx.x; }
  for (int i = 0; i < ITERS / 2; ++i) {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      acc[j] += __builtin_amdgcn_sqrtf(sp[j]);
      const float dx = qx[j] - a;
      const float dy = qy[j] - b;
      sp[j] = fmaf(dx, dx, dy * dy);
    }
    a += 1.0f;
    b -= 1.0f;
  }
  float s = 0; for (int j = 0; j < 16; ++j) s += acc[j] + sp[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  stamp(clk, 1);
}
// (f) 4 plain ops + sqrt, all independent of each other across terms
__global__ void k_mix(float *out, unsigned long long *clk, float x) {
  stamp(clk, 0);
  float acc[16], v[16];
  for (int j = 0; j < 16; ++j) { acc[j] = x + j + threadIdx.x; v[j] = x * j; }
  for (int i = 0; i < ITERS / 2; ++i) {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      v[j] = fmaf(v[j], 0.999f, 0.001f);
      acc[j] = __builtin_amdgcn_sqrtf(acc[j]);
    }
  }
  float s = 0; for (int j = 0; j < 16; ++j) s += acc[j] + v[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  stamp(clk, 1);
}

// the direct term with the query side from s_load (wave-uniform buffer reads,
// as rotate_direct_kernel), entity values from VGPRs
__constant__ float c_h[64 * 32];
__global__ void k_direct_sgpr(float *out, unsigned long long *clk, float x) {
  stamp(clk, 0);
  const float *hq = c_h;  // 32 floats per iteration, uniform (s_load)
  float acc[16], sq[16], a = x + threadIdx.x, b = x - threadIdx.x;
  for (int j = 0; j < 16; ++j) acc[j] = sq[j] = 0;
  for (int i = 0; i < ITERS / 2; ++i) {
    const float *h = hq + (i & 63) * 32;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      acc[j] += __builtin_amdgcn_sqrtf(sq[j]);
      const float dx = h[j] - a;
      const float dy = h[16 + j] - b;
      sq[j] = fmaf(dx, dx, dy * dy);
    }
    a += 1.0f;
    b -= 1.0f;
  }
  float s = 0; for (int j = 0; j < 16; ++j) s += acc[j] + sq[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  stamp(clk, 1);
}

// the SUM scoring gather's per-element arithmetic: fp64 FMA chains, the
// int32 -> fp64 conversion + FMA pair, and the int64 multiply-add form
__global__ void k_f64fma(float *out, unsigned long long *clk, float x) {
  stamp(clk, 0);
  double a[8];
  for (int j = 0; j < 8; ++j) a[j] = x + threadIdx.x + j;
  for (int i = 0; i < ITERS; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = fma(a[j], 0.999, 0.001);
  double s = 0; for (int j = 0; j < 8; ++j) s += a[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (float)s;
  stamp(clk, 1);
}
__global__ void k_cvt_fma(float *out, unsigned long long *clk, float x) {
  stamp(clk, 0);
  double a[8];
  int v[8];
  for (int j = 0; j < 8; ++j) { a[j] = 0; v[j] = (int)x + threadIdx.x + j; }
  const double c = x;
  for (int i = 0; i < ITERS; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) { a[j] = fma(c, (double)v[j], a[j]); v[j] += 3; }
  double s = 0; for (int j = 0; j < 8; ++j) s += a[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (float)s;
  stamp(clk, 1);
}
__global__ void k_mad64(float *out, unsigned long long *clk, float x) {
  stamp(clk, 0);
  long long a[8];
  int v[8];
  for (int j = 0; j < 8; ++j) { a[j] = 0; v[j] = (int)x + threadIdx.x + j; }
  const long long c = (long long)x + threadIdx.x;
  for (int i = 0; i < ITERS; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) { a[j] += c * v[j]; v[j] += 3; }
  long long s = 0; for (int j = 0; j < 8; ++j) s += a[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (float)s;
  stamp(clk, 1);
}
__global__ void k_madi64(float *out, unsigned long long *clk, float x) {
  stamp(clk, 0);
  long long a[8];
  int v[8];
  for (int j = 0; j < 8; ++j) { a[j] = 0; v[j] = (int)x + threadIdx.x + j; }
  const int c = (int)x + threadIdx.x;
  for (int i = 0; i < ITERS; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      unsigned long long carry;
      asm volatile("v_mad_i64_i32 %0, %1, %2, %3, %0" : "+v"(a[j]), "=s"(carry) : "v"(c), "v"(v[j]));
      v[j] += 3;
    }
  long long s = 0; for (int j = 0; j < 8; ++j) s += a[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (float)s;
  stamp(clk, 1);
}
__global__ void k_add32(float *out, unsigned long long *clk, float x) {
  stamp(clk, 0);
  int v[8];
  for (int j = 0; j < 8; ++j) v[j] = (int)x + threadIdx.x + j;
  for (int i = 0; i < ITERS; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] += 3;
  int s = 0; for (int j = 0; j < 8; ++j) s += v[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (float)s;
  stamp(clk, 1);
}

template <typename K>
double run(K kern, float *out, unsigned long long *clk, int blocks, int threads, double *ghz) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, out, clk, 1.0f);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, out, clk, 1.0f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  unsigned long long h[4];
  hipMemcpy(h, clk, sizeof(h), hipMemcpyDeviceToHost);
  *ghz = (double)(h[2] - h[0]) / (double)(h[3] - h[1]) * 0.1;
  return ms / 5;
}

int main() {
  float *out;
  unsigned long long *clk;
  hipMalloc(&out, 256 * 8 * 256 * sizeof(float) * 4);
  hipMalloc(&clk, 64);
  const int blocks = 256 * 8, threads = 256;
  const double waves = blocks * threads / 64.0;
  double t, g;
  auto cyc = [&](double t, double g, double per_wave) { return t * 1e-3 * g * 1e9 * 1024 / (waves * per_wave); };
  t = run(k_fma, out, clk, blocks, threads, &g);
  printf("fma:            %.3f ms %.2f GHz -> %.2f cyc/wave-instr/SIMD\n", t, g, cyc(t, g, ITERS * 8.0));
  t = run(k_pkfma, out, clk, blocks, threads, &g);
  printf("pk_fma:         %.3f ms %.2f GHz -> %.2f cyc/wave-instr/SIMD\n", t, g, cyc(t, g, ITERS * 8.0));
  t = run(k_direct<true, true>, out, clk, blocks, threads, &g);
  printf("direct sgpr:    %.3f ms %.2f GHz -> %.2f cyc/wave-term/SIMD\n", t, g, cyc(t, g, ITERS / 2 * 16.0));
  t = run(k_direct<true, false>, out, clk, blocks, threads, &g);
  printf("direct vgpr:    %.3f ms %.2f GHz -> %.2f cyc/wave-term/SIMD\n", t, g, cyc(t, g, ITERS / 2 * 16.0));
  t = run(k_direct<false, true>, out, clk, blocks, threads, &g);
  printf("direct nosqrt:  %.3f ms %.2f GHz -> %.2f cyc/wave-term/SIMD\n", t, g, cyc(t, g, ITERS / 2 * 16.0));
  t = run(k_direct_pipe, out, clk, blocks, threads, &g);
  printf("direct pipelined: %.3f ms %.2f GHz -> %.2f cyc/wave-term/SIMD\n", t, g, cyc(t, g, ITERS / 2 * 16.0));
  t = run(k_direct_sgpr, out, clk, blocks, threads, &g);
  printf("direct sgpr-load pipelined: %.3f ms %.2f GHz -> %.2f cyc/wave-term/SIMD\n", t, g, cyc(t, g, ITERS / 2 * 16.0));
  t = run(k_mix, out, clk, blocks, threads, &g);
  printf("fma+sqrt mix:   %.3f ms %.2f GHz -> %.2f cyc/(fma+sqrt)/SIMD\n", t, g, cyc(t, g, ITERS / 2 * 16.0));
  t = run(k_sqrt, out, clk, blocks, threads, &g);
  printf("sqrt:           %.3f ms %.2f GHz -> %.2f cyc/wave-instr/SIMD\n", t, g, cyc(t, g, ITERS * 8.0));
  t = run(k_sqrt_add, out, clk, blocks, threads, &g);
  printf("sqrt+add+add:   %.3f ms %.2f GHz -> %.2f cyc/wave-term/SIMD\n", t, g, cyc(t, g, ITERS * 8.0));
  t = run(k_mfma, out, clk, blocks, threads, &g);
  printf("mfma16x16x4f32: %.3f ms %.2f GHz -> %.2f cyc/mfma/SIMD\n", t, g, cyc(t, g, ITERS * 4.0));
  t = run(k_mfma_sqrt<4, true>, out, clk, blocks, threads, &g);
  printf("mfma+4(sqrt+add) NT4:  %.3f ms %.2f GHz -> %.2f cyc/wave-term\n", t, g, cyc(t, g, ITERS / 4 * 4 * 4.0));
  t = run(k_mfma_sqrt<8, true>, out, clk, blocks, threads, &g);
  printf("mfma+4(sqrt+add) NT8:  %.3f ms %.2f GHz -> %.2f cyc/wave-term\n", t, g, cyc(t, g, ITERS / 4 * 8 * 4.0));
  t = run(k_mfma_sqrt<8, false>, out, clk, blocks, threads, &g);
  printf("mfma+4(add->sqrt) NT8: %.3f ms %.2f GHz -> %.2f cyc/wave-term\n", t, g, cyc(t, g, ITERS / 4 * 8 * 4.0));
  t = run(k_bf16_sqrt<4>, out, clk, blocks, threads, &g);
  printf("bf16 16x16x32+4(sqrt+add) NT4: %.3f ms %.2f GHz -> %.2f cyc/wave-term\n", t, g, cyc(t, g, ITERS / 4 * 4 * 4.0));
  t = run(k_bf16_sqrt<8>, out, clk, blocks, threads, &g);
  printf("bf16 16x16x32+4(sqrt+add) NT8: %.3f ms %.2f GHz -> %.2f cyc/wave-term\n", t, g, cyc(t, g, ITERS / 4 * 8 * 4.0));
  t = run(k_bf16_32_sqrt<2>, out, clk, blocks, threads, &g);
  printf("bf16 2x32x32x16+16(sqrt+add) NT2: %.3f ms %.2f GHz -> %.2f cyc/wave-term\n", t, g, cyc(t, g, ITERS / 16 * 2 * 16.0));
  t = run(k_bf16k16, out, clk, blocks, threads, &g);
  printf("mfma16x16x16bf16: %.3f ms %.2f GHz -> %.2f cyc/mfma/SIMD\n", t, g, cyc(t, g, ITERS * 4.0));
  t = run(k_bf16k16_sqrt<4>, out, clk, blocks, threads, &g);
  printf("bf16 16x16x16+4(sqrt+add) NT4: %.3f ms %.2f GHz -> %.2f cyc/wave-term\n", t, g, cyc(t, g, ITERS / 4 * 4 * 4.0));
  t = run(k_bf16k16_sqrt<8>, out, clk, blocks, threads, &g);
  printf("bf16 16x16x16+4(sqrt+add) NT8: %.3f ms %.2f GHz -> %.2f cyc/wave-term\n", t, g, cyc(t, g, ITERS / 4 * 8 * 4.0));
  t = run(k_f64fma, out, clk, blocks, threads, &g);
  printf("fma_f64:        %.3f ms %.2f GHz -> %.2f cyc/wave-instr/SIMD\n", t, g, cyc(t, g, ITERS * 8.0));
  t = run(k_cvt_fma, out, clk, blocks, threads, &g);
  printf("cvt_f64_i32+fma_f64+add: %.3f ms %.2f GHz -> %.2f cyc/element/SIMD\n", t, g, cyc(t, g, ITERS * 8.0));
  t = run(k_mad64, out, clk, blocks, threads, &g);
  printf("int64 += i64*i32 +add: %.3f ms %.2f GHz -> %.2f cyc/element/SIMD\n", t, g, cyc(t, g, ITERS * 8.0));
  t = run(k_madi64, out, clk, blocks, threads, &g);
  printf("v_mad_i64_i32+add: %.3f ms %.2f GHz -> %.2f cyc/element/SIMD\n", t, g, cyc(t, g, ITERS * 8.0));
  t = run(k_add32, out, clk, blocks, threads, &g);
  printf("add_u32:        %.3f ms %.2f GHz -> %.2f cyc/wave-instr/SIMD\n", t, g, cyc(t, g, ITERS * 8.0));
  hipLaunchKernelGGL((k_mfma_sqrt<8, true>), dim3(blocks / 2), dim3(threads), 0, 0, out, clk, 1.0f);
  t = run(k_mfma_sqrt<8, true>, out, clk, blocks / 4, threads, &g);
  printf("mfma+4(sqrt+add) NT8 1 block/CU: %.3f ms %.2f GHz -> %.2f cyc/wave-term\n", t, g,
         t * 1e-3 * g * 1e9 * 1024 / (waves / 4 * ITERS / 4 * 8 * 4.0));
  return 0;
}
