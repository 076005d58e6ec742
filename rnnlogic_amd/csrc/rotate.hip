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
  hipLaunchKernelGGL(rotate_kernel, dim3((E + RB - 1) / RB, (nq + QB - 1) / QB), dim3(RB), 0,
                     (hipStream_t)stream, eemb, eemb_t, remb, D, gamma, all_h, all_r, nq, E, score, accumulate);
  RNNL_HIP_CHECK(hipGetLastError());
  return RNNL_OK;
}

}  // extern "C"
