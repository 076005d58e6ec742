// Device-side training batches (reference src/data.py:201-219).
//
// TrainDataset.__getitem__ builds, per batch row (h, r, t), the dense
// multi-hot target over hr2o[(h, r)] (|E| floats) and the relation-local id of
// the row's own edge.  rnnl_multi_hot builds the target rows on the device
// from a CSR of the key -> value lists (keys = r * |E| + h, ascending): one
// workgroup per row zero-fills its row with coalesced stores, one lane
// binary-searches the row's key, and the workgroup scatters the ones.
// rnnl_filter_flags is the same walk for the evaluation filters
// (ValidDataset / TestDataset.__getitem__, src/data.py:250-255, 287-291): a
// bool row that is 1 everywhere except at the known answers hr2oo / hr2ooo.
#include <hip/hip_runtime.h>

#include <string>

#include "internal.h"

namespace rnnl {

template <typename T>
__global__ __launch_bounds__(256) void multi_hot_kernel(const int64_t *__restrict__ keys,
                                                        const int64_t *__restrict__ offs,
                                                        const int32_t *__restrict__ vals, int64_t n_keys,
                                                        const int64_t *__restrict__ qkeys, int32_t width,
                                                        T *__restrict__ out, T fill, T hit_value) {
  __shared__ int64_t s_beg, s_end;
  const int row = blockIdx.x;
  T *o = out + (int64_t)row * width;
  for (int i = threadIdx.x; i < width; i += blockDim.x) o[i] = fill;
  if (threadIdx.x == 0) {
    const int64_t k = qkeys[row];
    int64_t lo = 0, hi = n_keys;  // first index with keys[i] >= k
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (keys[mid] < k)
        lo = mid + 1;
      else
        hi = mid;
    }
    const bool hit = lo < n_keys && keys[lo] == k;
    s_beg = hit ? offs[lo] : 0;
    s_end = hit ? offs[lo + 1] : 0;
  }
  // the fill must land before another wave's store to the same address:
  // drain this wave's stores, then the barrier
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int64_t i = s_beg + threadIdx.x; i < s_end; i += blockDim.x) {
    const int v = vals[i];
    if (v >= 0 && v < width) o[v] = hit_value;
  }
}

static int check_lists(const char *fn, const int64_t *keys, const int64_t *offs, const int32_t *vals, int64_t n_keys,
                       const int64_t *row_keys, int32_t n_rows, int32_t width, const void *out) {
  if (n_rows < 0 || width <= 0 || n_keys < 0 || !out || (n_rows > 0 && !row_keys) ||
      (n_keys > 0 && (!keys || !offs || !vals))) {
    set_error(std::string(fn) + ": bad arguments");
    return RNNL_ERR_INVALID;
  }
  return RNNL_OK;
}

}  // namespace rnnl

using namespace rnnl;

// Filtered rank bounds of evaluate() (trainer.py:191-203) for one row per
// workgroup, in one pass over the row: L = #(flagged scores > s_t) + 1,
// H = #(flagged scores >= s_t) + 2, or (1, E + 1) when t is not a candidate.
__global__ __launch_bounds__(256) void filtered_ranks_kernel(const float *__restrict__ score,
                                                             const uint8_t *__restrict__ mask,
                                                             const uint8_t *__restrict__ flag,
                                                             const int64_t *__restrict__ all_t, int E,
                                                             int64_t *__restrict__ L, int64_t *__restrict__ H) {
  __shared__ int s_gt[4], s_ge[4];
  const int64_t row = blockIdx.x;
  const float *sr = score + row * E;
  const uint8_t *fr = flag + row * E;
  const int t = (int)all_t[row];
  const float val = sr[t];
  int gt = 0, ge = 0;
  for (int e = threadIdx.x; e < E; e += 256) {
    const float v = sr[e];
    const int f = fr[e] != 0;
    gt += f & (v > val);
    ge += f & (v >= val);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    gt += __shfl_xor(gt, o, 64);
    ge += __shfl_xor(ge, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    s_gt[threadIdx.x >> 6] = gt;
    s_ge[threadIdx.x >> 6] = ge;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const bool hit = mask[row * E + t] != 0;
    L[row] = hit ? (int64_t)(s_gt[0] + s_gt[1] + s_gt[2] + s_gt[3]) + 1 : 1;
    H[row] = hit ? (int64_t)(s_ge[0] + s_ge[1] + s_ge[2] + s_ge[3]) + 2 : (int64_t)E + 1;
  }
}

// First index in [0, n) with a[i] >= k (n if none).
__device__ __forceinline__ int64_t lower_bound64(const int64_t *__restrict__ a, int64_t n, int64_t k) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (a[mid] < k)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo;
}

// One TrainDataset batch (data.py:201-219) from the device row table in one
// launch: row i of the batch is table[row0 + i] = (h, r, t); out_h / out_r /
// out_t receive it, out_etr the relation-local id of its own edge (key
// (r |E| + t) |E| + h in the sorted edge-key table, as torch.searchsorted
// with the index clamped), and out_target row i the multi-hot row of hr2o.
__global__ __launch_bounds__(256) void train_batch_kernel(const int64_t *__restrict__ table, int64_t row0,
                                                          const int64_t *__restrict__ keys,
                                                          const int64_t *__restrict__ offs,
                                                          const int32_t *__restrict__ vals, int64_t n_keys,
                                                          const int64_t *__restrict__ edge_keys,
                                                          const int64_t *__restrict__ edge_ids, int64_t n_edges,
                                                          int32_t E, int64_t *__restrict__ out_h,
                                                          int64_t *__restrict__ out_r, int64_t *__restrict__ out_t,
                                                          int64_t *__restrict__ out_etr,
                                                          float *__restrict__ out_target) {
  __shared__ int64_t s_beg, s_end;
  const int row = blockIdx.x;
  float *o = out_target + (int64_t)row * E;
  for (int i = threadIdx.x; i < E; i += blockDim.x) o[i] = 0.f;
  if (threadIdx.x == 0) {
    const int64_t *hrt = table + 3 * (row0 + row);
    const int64_t h = hrt[0], r = hrt[1], t = hrt[2];
    out_h[row] = h;
    out_r[row] = r;
    out_t[row] = t;
    const int64_t k = r * E + h;
    const int64_t lo = lower_bound64(keys, n_keys, k);
    const bool hit = lo < n_keys && keys[lo] == k;
    s_beg = hit ? offs[lo] : 0;
    s_end = hit ? offs[lo + 1] : 0;
    const int64_t pos = min(lower_bound64(edge_keys, n_edges, (r * E + t) * E + h), max(n_edges - 1, (int64_t)0));
    out_etr[row] = n_edges > 0 ? edge_ids[pos] : 0;
  }
  // the fill must land before another wave's store to the same address
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int64_t i = s_beg + threadIdx.x; i < s_end; i += blockDim.x) {
    const int v = vals[i];
    if (v >= 0 && v < E) o[v] = 1.f;
  }
}

extern "C" {

int rnnl_train_batch(const int64_t *table, int64_t row0, int32_t n_rows, const int64_t *keys, const int64_t *offs,
                     const int32_t *vals, int64_t n_keys, const int64_t *edge_keys, const int64_t *edge_ids,
                     int64_t n_edges, int32_t n_entities, int64_t *out_h, int64_t *out_r, int64_t *out_t,
                     int64_t *out_etr, float *out_target, void *stream) {
  if (!table || row0 < 0 || n_rows < 0 || n_entities <= 0 || n_keys < 0 || n_edges < 0 ||
      (n_keys > 0 && (!keys || !offs || !vals)) || (n_edges > 0 && (!edge_keys || !edge_ids)) ||
      (n_rows > 0 && (!out_h || !out_r || !out_t || !out_etr || !out_target))) {
    set_error("rnnl_train_batch: bad arguments");
    return RNNL_ERR_INVALID;
  }
  if (n_rows == 0) return RNNL_OK;
  hipLaunchKernelGGL(train_batch_kernel, dim3(n_rows), dim3(256), 0, (hipStream_t)stream, table, row0, keys, offs,
                     vals, n_keys, edge_keys, edge_ids, n_edges, n_entities, out_h, out_r, out_t, out_etr,
                     out_target);
  RNNL_HIP_CHECK(hipGetLastError());
  return RNNL_OK;
}

int rnnl_multi_hot(const int64_t *keys, const int64_t *offs, const int32_t *vals, int64_t n_keys,
                   const int64_t *row_keys, int32_t n_rows, int32_t width, float *out, void *stream) {
  const int rc = check_lists("rnnl_multi_hot", keys, offs, vals, n_keys, row_keys, n_rows, width, out);
  if (rc != RNNL_OK || n_rows == 0) return rc;
  hipLaunchKernelGGL(multi_hot_kernel<float>, dim3(n_rows), dim3(256), 0, (hipStream_t)stream, keys, offs, vals,
                     n_keys, row_keys, width, out, 0.f, 1.f);
  RNNL_HIP_CHECK(hipGetLastError());
  return RNNL_OK;
}

int rnnl_filter_flags(const int64_t *keys, const int64_t *offs, const int32_t *vals, int64_t n_keys,
                      const int64_t *row_keys, int32_t n_rows, int32_t width, uint8_t *out, void *stream) {
  const int rc = check_lists("rnnl_filter_flags", keys, offs, vals, n_keys, row_keys, n_rows, width, out);
  if (rc != RNNL_OK || n_rows == 0) return rc;
  hipLaunchKernelGGL(multi_hot_kernel<uint8_t>, dim3(n_rows), dim3(256), 0, (hipStream_t)stream, keys, offs, vals,
                     n_keys, row_keys, width, out, (uint8_t)1, (uint8_t)0);
  RNNL_HIP_CHECK(hipGetLastError());
  return RNNL_OK;
}

int rnnl_filtered_ranks(const float *score, const uint8_t *mask, const uint8_t *flag, const int64_t *all_t,
                        int32_t n_rows, int32_t n_entities, int64_t *L, int64_t *H, void *stream) {
  if (!score || !mask || !flag || !all_t || !L || !H || n_rows < 0 || n_entities <= 0) {
    set_error("rnnl_filtered_ranks: bad arguments");
    return RNNL_ERR_INVALID;
  }
  if (n_rows == 0) return RNNL_OK;
  hipLaunchKernelGGL(filtered_ranks_kernel, dim3(n_rows), dim3(256), 0, (hipStream_t)stream, score, mask, flag, all_t,
                     n_entities, L, H);
  RNNL_HIP_CHECK(hipGetLastError());
  return RNNL_OK;
}

}  // extern "C"
