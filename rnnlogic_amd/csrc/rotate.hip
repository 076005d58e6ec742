// RotatE entity feature + base-score fills for gfx950.
//
// rotate_score: score[q][e] (+)= gamma - sum_d sqrt(dre^2 + dim^2) with
//   (h o r)_d = (re_h re_r - im_h im_r, re_h im_r + im_h re_r),
//   (re_r, im_r) = (cos, sin)(remb[r][d] / ((gamma + 2) / D / pi))
// (reference src/embedding.py:28-70, forward at :64-70).
//
// Shape of the work: B queries x |E| entities x D complex dims, every term a
// sqrt — VALU/transcendental-bound (about 5 FMA-class ops + 1 sqrt per term),
// not a GEMM (the sqrt sits inside the reduction).  Each lane owns one entity
// and QB = 32 query rows; the entity table is read transposed (2D x E) so a
// wave's loads are 256 contiguous bytes, and h o r of the 32 rows sits in LDS
// (uniform broadcast reads).  One pass over the table serves 32 rows, so the
// table traffic is |E| * 8D bytes per 32 queries (L2/MALL resident).
#include <hip/hip_runtime.h>

#include <stdlib.h>

#include "internal.h"

namespace rnnl {

constexpr int RB = 256;  // entities per block (one per lane)
constexpr int QB = 32;   // query rows per block
constexpr int DC = 64;   // dims per LDS chunk

__global__ __launch_bounds__(RB) void rotate_kernel(const float *__restrict__ eemb, const float *__restrict__ eemb_t,
                                                    const float *__restrict__ remb, int D, float gamma,
                                                    const int64_t *__restrict__ all_h,
                                                    const int64_t *__restrict__ all_r, int nq, int E,
                                                    float *__restrict__ score, int accumulate) {
  __shared__ float s_re[DC][QB];
  __shared__ float s_im[DC][QB];
  const int tid = threadIdx.x;
  const int e = blockIdx.x * RB + tid;
  const int q0 = blockIdx.y * QB;
  const int nrow = min(QB, nq - q0);
  // torch computes vec / (range / pi) in fp32 with the divisor rounded to fp32
  const float div = (float)(((double)gamma + 2.0) / (double)D / 3.141592653589793238462643383279);
  float acc[QB];
#pragma unroll
  for (int k = 0; k < QB; ++k) acc[k] = 0.f;
  for (int d0 = 0; d0 < D; d0 += DC) {
    const int nd = min(DC, D - d0);
    __syncthreads();
    // h o r for QB rows x nd dims (RB lanes cover QB * DC = 2048 terms)
    for (int i = tid; i < QB * DC; i += RB) {
      const int k = i / DC, dd = i % DC;
      float re = 0.f, im = 0.f;
      if (k < nrow && dd < nd) {
        const int q = q0 + k;
        const int64_t h = all_h[q], r = all_r[q];
        const int d = d0 + dd;
        const float ph = remb[r * D + d] / div;
        const float cr = cosf(ph), sr = sinf(ph);
        const float rh = eemb[h * 2 * D + d], ih = eemb[h * 2 * D + D + d];
        re = rh * cr - ih * sr;
        im = rh * sr + ih * cr;
      }
      s_re[dd][k] = re;
      s_im[dd][k] = im;
    }
    __syncthreads();
    if (e < E) {
      float part[QB];
#pragma unroll
      for (int k = 0; k < QB; ++k) part[k] = 0.f;
      for (int dd = 0; dd < nd; ++dd) {
        const float a = eemb_t[(int64_t)(d0 + dd) * E + e];
        const float b = eemb_t[(int64_t)(D + d0 + dd) * E + e];
#pragma unroll
        for (int k = 0; k < QB; ++k) {
          const float x = s_re[dd][k] - a;
          const float y = s_im[dd][k] - b;
          part[k] += __builtin_amdgcn_sqrtf(fmaf(x, x, y * y));  // v_sqrt_f32 (1 ulp)
        }
      }
#pragma unroll
      for (int k = 0; k < QB; ++k) acc[k] += part[k];
    }
  }
  if (e < E) {
    for (int k = 0; k < nrow; ++k) {
      const int64_t idx = (int64_t)(q0 + k) * E + e;
      const float v = gamma - acc[k];
      score[idx] = accumulate ? score[idx] + v : v;
    }
  }
}

// ---------------------------------------------------------------------------
// MFMA formulation.  For one dimension d the squared distance of every
// (query q, entity e) pair is a K = 4 contraction:
//   s = (hr_re - a)^2 + (hr_im - b)^2
//     = [-2 hr_re, -2 hr_im, |hr|^2, 1] . [a, b, 1, a^2 + b^2]
// so one v_mfma_f32_16x16x4_f32 yields s for a 16 x 16 tile (exact fp32
// fmaf chain), and the VALU is left with sqrt(|s|) + accumulate per term
// (|s| absorbs a rounding-negative s at a near-zero distance; abs is a free
// source modifier).  Block = 64 queries x 256 entities, wave = 64 x 64
// (16 tiles, 64 accumulator VGPRs); A fragments (per query) come from LDS,
// B fragments (per entity) from the transposed table, one dword per lane.
constexpr int MQ = 64;   // queries per block
constexpr int ME = 256;  // entities per block (64 per wave)
constexpr int MDC = 32;  // dims per LDS chunk
constexpr int MQP = MQ + 16;  // padded row (bank spread of the 4 k-groups)

typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void rotate_mfma_kernel(const float *__restrict__ eemb,
                                                          const float *__restrict__ eemb_t,
                                                          const float *__restrict__ remb, int D, float gamma,
                                                          const int64_t *__restrict__ all_h,
                                                          const int64_t *__restrict__ all_r, int nq, int E,
                                                          float *__restrict__ score, int accumulate) {
  __shared__ __attribute__((aligned(16))) float sA[MDC][4][MQP];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int k = lane >> 4, i16 = lane & 15;
  const int q0 = blockIdx.y * MQ;
  const int e_base = blockIdx.x * ME + wave * 64;
  const float div = (float)(((double)gamma + 2.0) / (double)D / 3.141592653589793238462643383279);
  // entity of this lane in each of the 4 entity groups; loads are clamped in-range
  int ecol[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) ecol[g] = min(e_base + g * 16 + i16, E - 1);
  const int plane = (k & 1) ? D : 0;  // k = 0, 2: real plane; k = 1, 3: imaginary plane
  f32x4 acc[4][4];
#pragma unroll
  for (int qg = 0; qg < 4; ++qg)
#pragma unroll
    for (int g = 0; g < 4; ++g) acc[qg][g] = (f32x4){0.f, 0.f, 0.f, 0.f};
  for (int d0 = 0; d0 < D; d0 += MDC) {
    const int nd = min(MDC, D - d0);
    __syncthreads();
    // A fragments for MQ queries x nd dims: [-2 re, -2 im, |hr|^2, 1] of h o r
    for (int idx = tid; idx < MQ * MDC; idx += 256) {
      const int qq = idx / MDC, dd = idx % MDC;
      float re = 0.f, im = 0.f;
      if (q0 + qq < nq && dd < nd) {
        const int64_t h = all_h[q0 + qq], r = all_r[q0 + qq];
        const int d = d0 + dd;
        const float ph = remb[r * D + d] / div;
        const float cr = cosf(ph), sr = sinf(ph);
        const float rh = eemb[h * 2 * D + d], ih = eemb[h * 2 * D + D + d];
        re = rh * cr - ih * sr;
        im = rh * sr + ih * cr;
      }
      sA[dd][0][qq] = -2.f * re;
      sA[dd][1][qq] = -2.f * im;
      sA[dd][2][qq] = fmaf(re, re, im * im);
      sA[dd][3][qq] = (dd < nd) ? 1.f : 0.f;
    }
    __syncthreads();
    float v[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) v[g] = eemb_t[(int64_t)(plane + d0) * E + ecol[g]];
    for (int dd = 0; dd < nd; ++dd) {
      // prefetch the next dimension's table values
      float vn[4];
      const int dn = min(dd + 1, nd - 1);
#pragma unroll
      for (int g = 0; g < 4; ++g) vn[g] = eemb_t[(int64_t)(plane + d0 + dn) * E + ecol[g]];
      float b[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float o = __shfl_xor(v[g], 16, 64);  // k = 3 lanes: real part from their k = 2 partner
        b[g] = k == 0 || k == 1 ? v[g] : (k == 2 ? 1.f : fmaf(o, o, v[g] * v[g]));
      }
      float a[4];
#pragma unroll
      for (int qg = 0; qg < 4; ++qg) a[qg] = sA[dd][k][qg * 16 + i16];
#pragma unroll
      for (int qg = 0; qg < 4; ++qg) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const f32x4 s = __builtin_amdgcn_mfma_f32_16x16x4f32(a[qg], b[g], (f32x4){0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[qg][g][j] += __builtin_amdgcn_sqrtf(__builtin_fabsf(s[j]));
        }
      }
#pragma unroll
      for (int g = 0; g < 4; ++g) v[g] = vn[g];
    }
  }
  // D layout: lane holds entity column i16 of group g, query rows 4k + j of group qg
#pragma unroll
  for (int qg = 0; qg < 4; ++qg)
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int q = q0 + qg * 16 + k * 4 + j;
        const int e = e_base + g * 16 + i16;
        if (q < nq && e < E) {
          const int64_t idx = (int64_t)q * E + e;
          const float val = gamma - acc[qg][g][j];
          score[idx] = accumulate ? score[idx] + val : val;
        }
      }
}

__global__ void transpose_kernel(const float *__restrict__ in, int rows, int cols, float *__restrict__ out) {
  __shared__ float tile[32][33];
  const int c0 = blockIdx.x * 32, r0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 256 threads: 32 x 8
  for (int j = ty; j < 32; j += 8) {
    const int r = r0 + j, c = c0 + tx;
    tile[j][tx] = (r < rows && c < cols) ? in[(int64_t)r * cols + c] : 0.f;
  }
  __syncthreads();
  for (int j = ty; j < 32; j += 8) {
    const int c = c0 + j, r = r0 + tx;
    if (c < cols && r < rows) out[(int64_t)c * rows + r] = tile[tx][j];
  }
}

__global__ void fill_rows_kernel(const float *__restrict__ row, int nq, int E, float *__restrict__ out) {
  const int64_t n = (int64_t)nq * E;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = row[i % E];
}

__global__ void fill_value_kernel(float v, int64_t n, float *__restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = v;
}

static unsigned grid_for(int64_t n) { return (unsigned)std::min<int64_t>((n + 255) / 256, 256 * 16); }

}  // namespace rnnl

using namespace rnnl;

extern "C" {

int rnnl_fill_rows(const float *row, int32_t nq, int32_t E, float *score, void *stream) {
  if (!row || !score || nq < 0 || E <= 0) {
    set_error("rnnl_fill_rows: bad arguments");
    return RNNL_ERR_INVALID;
  }
  const int64_t n = (int64_t)nq * E;
  if (n == 0) return RNNL_OK;
  hipLaunchKernelGGL(fill_rows_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, row, nq, E, score);
  RNNL_HIP_CHECK(hipGetLastError());
  return RNNL_OK;
}

int rnnl_fill_value(float v, int64_t n, float *score, void *stream) {
  if (!score || n < 0) {
    set_error("rnnl_fill_value: bad arguments");
    return RNNL_ERR_INVALID;
  }
  if (n == 0) return RNNL_OK;
  hipLaunchKernelGGL(fill_value_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, v, n, score);
  RNNL_HIP_CHECK(hipGetLastError());
  return RNNL_OK;
}

int rnnl_rotate_transpose(const float *eemb, int32_t E, int32_t dim2, float *eemb_t, void *stream) {
  if (!eemb || !eemb_t || E <= 0 || dim2 <= 0) {
    set_error("rnnl_rotate_transpose: bad arguments");
    return RNNL_ERR_INVALID;
  }
  hipLaunchKernelGGL(transpose_kernel, dim3((dim2 + 31) / 32, (E + 31) / 32), dim3(256), 0, (hipStream_t)stream,
                     eemb, E, dim2, eemb_t);
  RNNL_HIP_CHECK(hipGetLastError());
  return RNNL_OK;
}

int rnnl_rotate_score(const float *eemb, const float *eemb_t, const float *remb, int32_t D, float gamma,
                      const int64_t *all_h, const int64_t *all_r, int32_t nq, int32_t E, float *score,
                      int32_t accumulate, void *stream) {
  if (!eemb || !eemb_t || !remb || !all_h || !all_r || !score || D <= 0 || E <= 0 || nq < 0) {
    set_error("rnnl_rotate_score: bad arguments");
    return RNNL_ERR_INVALID;
  }
  if (nq == 0) return RNNL_OK;
  static const bool valu = getenv("RNNL_ROTATE_VALU") != nullptr;  // diagnostic: VALU-only variant
  if (valu)
    hipLaunchKernelGGL(rotate_kernel, dim3((E + RB - 1) / RB, (nq + QB - 1) / QB), dim3(RB), 0,
                       (hipStream_t)stream, eemb, eemb_t, remb, D, gamma, all_h, all_r, nq, E, score, accumulate);
  else
    hipLaunchKernelGGL(rotate_mfma_kernel, dim3((E + ME - 1) / ME, (nq + MQ - 1) / MQ), dim3(256), 0,
                       (hipStream_t)stream, eemb, eemb_t, remb, D, gamma, all_h, all_r, nq, E, score, accumulate);
  RNNL_HIP_CHECK(hipGetLastError());
  return RNNL_OK;
}

}  // extern "C"
