// Microbenchmark (diagnostic): the RotatE direct term in packed fp32
// (v_pk_add/v_pk_mul/v_pk_fma on two dims at once) vs scalar fp32, with the
// query side as wave-uniform s_load pairs. Cycles per wave-term per SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 pk_direct.hip -o pk_direct
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f32x2 __attribute__((ext_vector_type(2)));
constexpr int ITERS = 4096;
__constant__ float c_h[64 * 64];

__device__ __forceinline__ void stamp(unsigned long long *clk, int slot) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    clk[2 * slot] = __builtin_amdgcn_s_memtime();
    clk[2 * slot + 1] = __builtin_amdgcn_s_memrealtime();
  }
}

// scalar: sub, sub, mul, fma, sqrt (pipelined), add per term; 16 queries x 1 dim per iteration
__global__ void k_scalar(float *out, unsigned long long *clk, float x) {
  stamp(clk, 0);
  float acc[16], sq[16], a = x + threadIdx.x, b = x - threadIdx.x;
  for (int j = 0; j < 16; ++j) acc[j] = sq[j] = 0;
  for (int i = 0; i < ITERS; ++i) {
    const float *h = c_h + (i & 63) * 64;
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

// packed: 2 dims per op: pk_add(-), pk_add(-), pk_mul, pk_fma, 2 sqrt, pk_add per 2 terms
template <int NQ>
__global__ void k_packed(float *out, unsigned long long *clk, float x) {
  stamp(clk, 0);
  f32x2 acc[NQ], sq[NQ];
  f32x2 a = {x + threadIdx.x, x + threadIdx.x + 1}, b = {x - threadIdx.x, x - threadIdx.x - 2};
  for (int j = 0; j < NQ; ++j) acc[j] = sq[j] = (f32x2){0, 0};
  const f32x2 one = {1.0f, 1.0f};
  for (int i = 0; i < ITERS / 2; ++i) {
    const f32x2 *h = (const f32x2 *)c_h + (i & 63) * 32;
#pragma unroll
    for (int j = 0; j < NQ; ++j) {
      acc[j] += (f32x2){__builtin_amdgcn_sqrtf(sq[j].x), __builtin_amdgcn_sqrtf(sq[j].y)};
      const f32x2 dx = h[j] - a;
      const f32x2 dy = h[NQ + j] - b;
      sq[j] = __builtin_elementwise_fma(dx, dx, dy * dy);
    }
    a += one;
    b -= one;
  }
  float s = 0; for (int j = 0; j < NQ; ++j) s += acc[j].x + acc[j].y + sq[j].x + sq[j].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
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
  float hh[64 * 64];
  for (int i = 0; i < 64 * 64; ++i) hh[i] = 0.01f * (i % 97);
  hipMemcpyToSymbol(HIP_SYMBOL(c_h), hh, sizeof(hh));
  const int blocks = 256 * 8, threads = 256;
  const double waves = blocks * threads / 64.0;
  double t, g;
  auto cyc = [&](double t, double g, double per_wave) { return t * 1e-3 * g * 1e9 * 1024 / (waves * per_wave); };
  t = run(k_scalar, out, clk, blocks, threads, &g);
  printf("scalar direct:  %.3f ms %.2f GHz -> %.2f cyc/64 wave-terms/SIMD\n", t, g, 64 * cyc(t, g, ITERS * 16.0));
  t = run(k_packed<16>, out, clk, blocks, threads, &g);
  printf("packed16:       %.3f ms %.2f GHz -> %.2f cyc/64 wave-terms/SIMD\n", t, g, 64 * cyc(t, g, ITERS * 16.0));
  t = run(k_packed<10>, out, clk, blocks, threads, &g);
  printf("packed10:       %.3f ms %.2f GHz -> %.2f cyc/64 wave-terms/SIMD\n", t, g, 64 * cyc(t, g, ITERS * 10.0));
  return 0;
}
