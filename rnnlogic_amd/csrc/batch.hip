// Device-side training batches (reference src/data.py:201-219).
//
// TrainDataset.__getitem__ builds, per batch row (h, r, t), the dense
// multi-hot target over hr2o[(h, r)] (|E| floats) and the relation-local id of
// the row's own edge.  rnnl_multi_hot builds the target rows on the device
// from a CSR of the key -> value lists (keys = r * |E| + h, ascending): one
// workgroup per row zero-fills its row with coalesced stores, one lane
// binary-searches the row's key, and the workgroup scatters the ones.
#include <hip/hip_runtime.h>

#include "internal.h"

namespace rnnl {

__global__ __launch_bounds__(256) void multi_hot_kernel(const int64_t *__restrict__ keys,
                                                        const int64_t *__restrict__ offs,
                                                        const int32_t *__restrict__ vals, int64_t n_keys,
                                                        const int64_t *__restrict__ qkeys, int32_t width,
                                                        float *__restrict__ out) {
  __shared__ int64_t s_beg, s_end;
  const int row = blockIdx.x;
  float *o = out + (int64_t)row * width;
  for (int i = threadIdx.x; i < width; i += blockDim.x) o[i] = 0.f;
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
  __syncthreads();  // the zero fill is ordered before the ones (same workgroup, barrier drains stores)
  for (int64_t i = s_beg + threadIdx.x; i < s_end; i += blockDim.x) {
    const int v = vals[i];
    if (v >= 0 && v < width) o[v] = 1.f;
  }
}

}  // namespace rnnl

using namespace rnnl;

extern "C" {

int rnnl_multi_hot(const int64_t *keys, const int64_t *offs, const int32_t *vals, int64_t n_keys,
                   const int64_t *row_keys, int32_t n_rows, int32_t width, float *out, void *stream) {
  if (n_rows < 0 || width <= 0 || n_keys < 0 || !out || (n_rows > 0 && !row_keys) ||
      (n_keys > 0 && (!keys || !offs || !vals))) {
    set_error("rnnl_multi_hot: bad arguments");
    return RNNL_ERR_INVALID;
  }
  if (n_rows == 0) return RNNL_OK;
  hipLaunchKernelGGL(multi_hot_kernel, dim3(n_rows), dim3(256), 0, (hipStream_t)stream, keys, offs, vals, n_keys,
                     row_keys, width, out);
  RNNL_HIP_CHECK(hipGetLastError());
  return RNNL_OK;
}

}  // extern "C"
