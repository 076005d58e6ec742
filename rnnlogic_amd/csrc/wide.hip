// Exact 64-bit path counts for the rows the grounding kernel flags
// (ERR_COUNT_WIDTH: a path count or PNA degree reached 2^32 in its u32 LDS
// sums).  The reference counts in int64 (src/data.py:139-171: one_hot, then
// per body relation a gather and a scatter-sum), so such rows are grounded
// again here, rule-end node by rule-end node, with u64 sums:
//
//   wide_ground_kernel — one workgroup per flagged row.  For every trie node
//   of the row's head relation at which rules end (a leaf of head_leaf_node),
//   the node's body is recovered by walking parents up the breadth-first
//   trie, then applied hop by hop to a dense u64 vector over the entities
//   (global scratch, two per workgroup): every entity with a non-zero count
//   expands over its CSR range of the hop's relation with 64-bit atomic adds
//   (exact, order-free), skipping the row's own edge on hops of the query
//   relation (data.py:164-169).  The non-zero entries of the last vector are
//   appended as (row, entity, node, count) to the output with one atomic
//   cursor; the host sorts them into the reference's order.
//
// O(|E|) per hop and no prefix sharing: a rare exactness path, not the
// forward's (the forward's u32 kernel covers every count below 2^32).
#include <hip/hip_runtime.h>

#include "fwd.h"

namespace rnnl {

constexpr int WGB = 256;

__global__ __launch_bounds__(WGB) void wide_ground_kernel(GraphDev g, RulesDev rl, const int64_t *__restrict__ all_h,
                                                          const int64_t *__restrict__ all_r,
                                                          const int64_t *__restrict__ etr,
                                                          const int32_t *__restrict__ rows, int n_rows,
                                                          unsigned long long *__restrict__ scratch,
                                                          int32_t *__restrict__ out_row, int32_t *__restrict__ out_ent,
                                                          int32_t *__restrict__ out_node,
                                                          unsigned long long *__restrict__ out_count, int64_t cap,
                                                          unsigned long long *__restrict__ cursor) {
  __shared__ int s_body[64];
  __shared__ int s_len;
  const int tid = threadIdx.x;
  const int E = g.E;
  unsigned long long *x = scratch + (int64_t)blockIdx.x * 2 * E;
  unsigned long long *y = x + E;
  for (int k = blockIdx.x; k < n_rows; k += gridDim.x) {
    const int q = rows[k];
    const int h = (int)all_h[q], r = (int)all_r[q];
    const int root = rl.head_root[r];
    if (root < 0) continue;
    int rm_src = -1, rm_dst = -1;
    if (etr && etr[q] >= 0) {
      const int base = g.edge_base[r];
      rm_src = g.edge_src[base + (int)etr[q]];
      rm_dst = g.edge_dst[base + (int)etr[q]];
    }
    const int lb = rl.head_leaf_ptr[r], le = rl.head_leaf_ptr[r + 1];
    for (int li = lb; li < le; ++li) {
      const int leaf = rl.head_leaf_node[li];
      if (tid == 0) {  // the leaf's body: parents up to the root (breadth-first trie)
        int n = leaf, len = 0;
        int stack[64];
        while (n != root && len < 64) {
          stack[len++] = rl.node_rel[n];
          int par = root;
          for (int c = root; c < n; ++c)
            if (rl.node_nchild[c] > 0 && rl.node_child[c] <= n && n < rl.node_child[c] + rl.node_nchild[c]) {
              par = c;
              break;
            }
          n = par;
        }
        for (int i = 0; i < len; ++i) s_body[i] = stack[len - 1 - i];
        s_len = len;
      }
      for (int v = tid; v < E; v += WGB) x[v] = v == h ? 1ull : 0ull;
      wg_sync_global();  // stores drained and L1 dropped: the vectors are handed between waves
      const int len = s_len;
      for (int hop = 0; hop < len; ++hop) {
        const int rel = s_body[hop];
        for (int v = tid; v < E; v += WGB) y[v] = 0ull;
        wg_sync_global();
        for (int v = tid; v < E; v += WGB) {
          const unsigned long long c = x[v];
          if (!c) continue;
          const uint2 vb = g.vbits[(int64_t)v * g.W + (rel >> 5)];
          const uint32_t bit = 1u << (rel & 31);
          if (!(vb.x & bit)) continue;
          const int pos = (int)vb.y + __popc(vb.x & (bit - 1u));
          for (int e = g.dvoff[pos]; e < g.dvoff[pos + 1]; ++e) {
            const int t = g.col[e];
            if (rel == r && v == rm_src && t == rm_dst) continue;  // the row's own edge (data.py:164-169)
            atomicAdd(y + t, c);
          }
        }
        wg_sync_global();
        unsigned long long *tmp = x;
        x = y;
        y = tmp;
      }
      for (int v = tid; v < E; v += WGB) {
        const unsigned long long c = x[v];
        if (!c) continue;
        const unsigned long long at = atomicAdd(cursor, 1ull);
        if ((int64_t)at < cap) {
          out_row[at] = q;
          out_ent[at] = v;
          out_node[at] = leaf;
          out_count[at] = c;
        }
      }
      __syncthreads();  // (x is rewritten by the next leaf)
    }
  }
}

}  // namespace rnnl

using namespace rnnl;

extern "C" {

int rnnl_ground_wide_scratch_bytes(rnnl_graph g, int32_t n_rows, size_t *bytes) {
  if (!g || n_rows < 0 || !bytes) {
    set_error("rnnl_ground_wide_scratch_bytes: bad arguments");
    return RNNL_ERR_INVALID;
  }
  const int64_t wg = std::max<int64_t>(1, std::min<int64_t>(n_rows, NUM_CU));
  *bytes = (size_t)(wg * 2 * (int64_t)g->d.E * 8);
  return RNNL_OK;
}

int rnnl_ground_wide(rnnl_graph g, rnnl_rules r, const int64_t *all_h, const int64_t *all_r, const int64_t *etr,
                     const int32_t *rows, int32_t n_rows, void *scratch, size_t scratch_bytes, int32_t *out_row,
                     int32_t *out_ent, int32_t *out_node, uint64_t *out_count, int64_t cap, uint64_t *cursor,
                     void *stream) {
  if (!g || !r || !all_h || !all_r || !rows || n_rows < 0 || !scratch || cap < 0 || !cursor ||
      (cap > 0 && (!out_row || !out_ent || !out_node || !out_count))) {
    set_error("rnnl_ground_wide: bad arguments");
    return RNNL_ERR_INVALID;
  }
  const int64_t wg = std::max<int64_t>(1, std::min<int64_t>(n_rows, NUM_CU));
  if ((int64_t)scratch_bytes < wg * 2 * (int64_t)g->d.E * 8) {
    set_error("rnnl_ground_wide: scratch too small");
    return RNNL_ERR_INVALID;
  }
  hipStream_t st = (hipStream_t)stream;
  RNNL_HIP_CHECK(hipMemsetAsync(cursor, 0, sizeof(uint64_t), st));
  if (n_rows == 0) return RNNL_OK;
  hipLaunchKernelGGL(wide_ground_kernel, dim3((unsigned)wg), dim3(WGB), 0, st, g->d, r->d, all_h, all_r, etr, rows,
                     n_rows, static_cast<unsigned long long *>(scratch), out_row, out_ent, out_node,
                     reinterpret_cast<unsigned long long *>(out_count), cap,
                     reinterpret_cast<unsigned long long *>(cursor));
  RNNL_HIP_CHECK(hipGetLastError());
  return RNNL_OK;
}

int rnnl_forward_error_bits(void *ws, void *stream, uint32_t *bits) {
  if (!ws || !bits) {
    set_error("rnnl_forward_error_bits: bad arguments");
    return RNNL_ERR_INVALID;
  }
  uint32_t h[8];
  RNNL_HIP_CHECK(hipMemcpyAsync(h, ws, sizeof(h), hipMemcpyDeviceToHost, (hipStream_t)stream));
  RNNL_HIP_CHECK(hipStreamSynchronize((hipStream_t)stream));
  *bits = h[H_ERRBITS];
  return RNNL_OK;
}

}  // extern "C"
