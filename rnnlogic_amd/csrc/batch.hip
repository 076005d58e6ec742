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

extern "C" {

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

}  // extern "C"
