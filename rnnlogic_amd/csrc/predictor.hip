// The EM loop's rule-weight Predictor (reference src/predictors.py:17-119) on
// the grounding of ground.hip: per-node rule-weight sums in int32 fixed
// point, the exact per-candidate score (score_linear_kernel), compute_H's
// per-node path statistics (rule_stats_kernel) and the backward
// (predictor_backward_kernel).  C-ABI: rnnl_linear_node_weights*,
// rnnl_predictor_*.
#include <hip/hip_runtime.h>

#include <string>

#include "fwd.h"

namespace rnnl {

// ---------------------------------------------------------------- EM Predictor (a12)
// Predictor.forward (reference src/predictors.py:53-80): score = sum over the
// relation's rules of path count x rule weight.  Rules ending at the same trie
// node have identical counts, so the grounding COO's (node, count) entries
// need one scalar per node: the sum of its rules' weights.  As for the SUM
// records, that is int32 fixed point with one shift for the table, so the
// per-candidate int64 sum of count x fix is exact and independent of the
// order of the entries.  Layout: int32 fix[n_nodes], then (at
// lin_trailer_off) u32 max|sum| bits, i32 shift.
__host__ __device__ inline int64_t lin_trailer_off(int n_nodes) { return ((int64_t)n_nodes * 4 + 15) & ~int64_t(15); }

__global__ void lin_node_kernel(RulesDev rl, const float *__restrict__ w, unsigned char *__restrict__ out) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  const bool valid = n < rl.n_nodes;
  double s = 0.0;
  const int k0 = valid ? rl.node_rule_ptr[n] : 0, k1 = valid ? rl.node_rule_ptr[n + 1] : 0;
  for (int k = k0; k < k1; ++k) s += (double)w[rl.node_rules[k]];
  const float f = (float)s;
  if (valid) reinterpret_cast<float *>(out)[n] = f;
  unsigned int m = __float_as_uint(fabsf(f));  // wave max, then one atomic per wave
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = max(m, (unsigned int)__shfl_xor((int)m, o, 64));
  if ((threadIdx.x & 63) == 0 && m) atomicMax(reinterpret_cast<unsigned int *>(out + lin_trailer_off(rl.n_nodes)), m);
}

__global__ void lin_fix_kernel(int n_nodes, unsigned char *__restrict__ out) {
  unsigned int *trailer = reinterpret_cast<unsigned int *>(out + lin_trailer_off(n_nodes));
  bool bad;
  const int shift = fix_shift(trailer, bad);
  const float sc = ldexpf(1.f, shift);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n_nodes; i += gridDim.x * blockDim.x) {
    const float f = reinterpret_cast<float *>(out)[i];
    reinterpret_cast<int *>(out)[i] = bad ? 0 : (int)rintf(f * sc);
  }
}


// One workgroup per query (grid-stride), one lane per candidate: the
// candidate's exact sum, added into the pre-filled bias row (entity_feature
// 'bias') or written (otherwise; the rows were pre-filled with -inf).
__global__ __launch_bounds__(BS) void score_linear_kernel(KParams p, const int *__restrict__ fix) {
  const int shift = (int)reinterpret_cast<const unsigned int *>(reinterpret_cast<const unsigned char *>(fix) +
                                                                lin_trailer_off(p.rl.n_nodes))[1];
  const double inv = ldexp(1.0, -shift);
  check_node_table(p, reinterpret_cast<const unsigned int *>(reinterpret_cast<const unsigned char *>(fix) +
                                                             lin_trailer_off(p.rl.n_nodes)));
  // one wave per 64-candidate chunk of the grounding's chunk list (grid-stride)
  const long long nchunks = (long long)*reinterpret_cast<const unsigned long long *>(
      reinterpret_cast<const unsigned int *>(p.ws) + H_CHUNKS);
  const long long nw = (long long)gridDim.x * (BS / 64);
  for (long long c = blockIdx.x * (BS / 64) + (threadIdx.x >> 6); c < nchunks; c += nw) {
    const int2 ck = p.chunks[c];
    const int q = ck.x;
    const int nc = p.n_cand[q];
    const int64_t qb = p.q_base[q];
    {
      const int s = ck.y + (int)(threadIdx.x & 63);
      if (s >= nc) continue;
      const int4 cr = p.cand[qb + s];
      const int t = cr.x;
      long long acc = 0;
      uint64_t csum = 0;
      for (int e = cr.y; e < cr.y + cr.z; ++e) {
        const int2 be = p.bent[e];
        csum += (uint32_t)be.y;
        acc += (long long)(uint32_t)be.y * fix[be.x];
      }
      if (csum >> 33) flag_acc_range(p);  // |int32 fix| < 2^30
      const float out = (float)((double)acc * inv);
      const int64_t idx = (int64_t)q * p.g.E + t;
      if (p.feature == RNNL_FEATURE_NONE)
        p.score[idx] = out;
      else
        p.score[idx] = out + p.score[idx];
      if (p.mask) p.mask[idx] = 1;
    }
  }
}

// Predictor.compute_H (src/predictors.py:82-119) needs, per (row, rule):
// the path count at the row's true tail and the total over all candidates.
// Both only depend on the rule's trie node: per row, for every node of the
// head's trie (local index node - root < ld), pos = count at all_t[q] and
// tot = sum over candidates.  One workgroup per row; tot is summed in LDS.
__global__ __launch_bounds__(BS) void rule_stats_kernel(KParams p, const int64_t *__restrict__ all_t, int ld,
                                                        long long *__restrict__ pos, long long *__restrict__ tot) {
  extern __shared__ unsigned long long s_tot[];
  for (int q = blockIdx.x; q < p.nq; q += gridDim.x) {
    const int nc = p.n_cand[q];
    if (nc <= 0) continue;
    const int r = (int)p.all_r[q];
    const int root = p.rl.head_root[r], nh = min(p.rl.head_nodes[r], ld);
    for (int i = threadIdx.x; i < nh; i += BS) s_tot[i] = 0ull;
    __syncthreads();
    const int64_t qb = p.q_base[q];
    const int tq = (int)all_t[q];
    for (int s = threadIdx.x; s < nc; s += BS) {
      const int4 cr = p.cand[qb + s];
      const int t = cr.x;
      for (int e = cr.y; e < cr.y + cr.z; ++e) {
        const int2 be = p.bent[e];
        const int k = be.x - root;
        const unsigned long long c = (uint32_t)be.y;
        atomicAdd(&s_tot[k], c);
        if (t == tq) pos[(int64_t)q * ld + k] += (long long)c;  // one lane owns the true tail
      }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < nh; i += BS) tot[(int64_t)q * ld + i] = (long long)s_tot[i];
    __syncthreads();
  }
}

// Predictor.forward's gradient (the backward of predictors.py:62-66 under
// trainer.py:86-90): d score[q, t] / d rule_weights[rho] = count_rho(q, t), and
// rules ending at one trie node share the count, so per node
// grad_node[n] = sum over (q, t) of count_n(q, t) x grad_score[q, t].  One
// workgroup per row (grid-stride): the row's contributions are summed in LDS
// (one slot per node of the head's trie), then one global atomic per (row,
// touched node), both int64 fixed point (order-independent).  The caller
// zero-fills grad_node.
//
// The launch's max |grad| at candidates and sum of their entries' path counts
// (a max and an integer sum: order-independent), for the fixed-point scale.
__global__ __launch_bounds__(BS) void predictor_bw_stats_kernel(KParams p, const float *__restrict__ grad) {
  unsigned int m = 0u;
  unsigned long long k = 0ull;
  for (int q = blockIdx.x; q < p.nq; q += gridDim.x) {
    const int nc = p.n_cand[q];
    const int64_t qb = p.q_base[q];
    for (int s = threadIdx.x; s < nc; s += BS) {
      const int4 cr = p.cand[qb + s];
      const float g = grad[(int64_t)q * p.g.E + cr.x];
      if (g == 0.f) continue;
      m = max(m, __float_as_uint(fabsf(g)));
      for (int e = cr.y; e < cr.y + cr.z; ++e) k += (uint32_t)p.bent[e].y;
    }
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    m = max(m, (unsigned int)__shfl_xor((int)m, o, 64));
    k += __shfl_xor(k, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    unsigned int *hdr = reinterpret_cast<unsigned int *>(p.ws);
    if (m) atomicMax(&hdr[H_BW_MAXG], m);
    if (k) atomicAdd(reinterpret_cast<unsigned long long *>(hdr + H_BW_SUMK), k);
  }
}

// 2^s with sum k x max |grad| x 2^s < 2^62 (bad: a non-finite gradient)
__device__ __forceinline__ int pred_bw_scale(const KParams &p, bool &bad) {
  const unsigned int *hdr = reinterpret_cast<const unsigned int *>(p.ws);
  const unsigned int mb = hdr[H_BW_MAXG];
  const unsigned long long k = *reinterpret_cast<const unsigned long long *>(hdr + H_BW_SUMK);
  bad = mb >= 0x7f800000u;
  const double total = (double)k * (double)__uint_as_float(mb);
  return (bad || !(total > 0.0)) ? 0 : 61 - ilogb(total);
}

// Per row (one workgroup per query, grid-stride): G_n += count x grad at
// (row, candidate) for the row's head trie in LDS, then added per node into
// grad_node — as int64 fixed point at the launch's scale, so the sums do not
// depend on the order of the adds (run-to-run bitwise); predictor_bw_fix_kernel
// turns them into fp64.  A non-finite gradient takes fp64 sums instead (NaN /
// inf reach the nodes the reference's would).
__global__ __launch_bounds__(BS) void predictor_backward_kernel(KParams p, const float *__restrict__ grad, int ld,
                                                                unsigned long long *__restrict__ grad_node) {
  extern __shared__ unsigned long long s_g[];
  bool bad;
  const int sc = pred_bw_scale(p, bad);
  for (int q = blockIdx.x; q < p.nq; q += gridDim.x) {
    const int nc = p.n_cand[q];
    if (nc <= 0) continue;
    const int r = (int)p.all_r[q];
    const int root = p.rl.head_root[r], nh = min(p.rl.head_nodes[r], ld);
    for (int i = threadIdx.x; i < nh; i += BS) s_g[i] = 0ull;
    __syncthreads();
    const int64_t qb = p.q_base[q];
    const float *__restrict__ gq = grad + (int64_t)q * p.g.E;
    for (int s = threadIdx.x; s < nc; s += BS) {
      const int4 cr = p.cand[qb + s];
      const double g = (double)gq[cr.x];
      if (g == 0.0) continue;
      // the gradient on the fixed-point grid once, times each entry's integer
      // count: split and merged (node, candidate) entries sum alike
      const long long gf = bad ? 0 : llrint(ldexp(g, sc));
      for (int e = cr.y; e < cr.y + cr.z; ++e) {
        const int2 be = p.bent[e];
        if (bad)
          atomicAdd(reinterpret_cast<double *>(&s_g[be.x - root]), (double)(uint32_t)be.y * g);
        else
          atomicAdd(&s_g[be.x - root], (unsigned long long)((long long)(uint32_t)be.y * gf));
      }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < nh; i += BS) {
      if (s_g[i] == 0ull) continue;
      if (bad)
        atomicAdd(reinterpret_cast<double *>(&grad_node[root + i]), __longlong_as_double((long long)s_g[i]));
      else
        atomicAdd(&grad_node[root + i], s_g[i]);
    }
    __syncthreads();
  }
}

// grad_node's int64 fixed-point sums -> fp64 in place (the zero fill is 0 in both)
__global__ void predictor_bw_fix_kernel(KParams p, int n_nodes, unsigned long long *__restrict__ grad_node) {
  bool bad;
  const int sc = pred_bw_scale(p, bad);
  if (bad) return;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n_nodes; i += gridDim.x * blockDim.x) {
    const long long v = (long long)grad_node[i];
    if (v) reinterpret_cast<double *>(grad_node)[i] = ldexp((double)v, -sc);
  }
}

}  // namespace rnnl

using namespace rnnl;

extern "C" {

int rnnl_linear_node_weights_size(rnnl_rules r, size_t *bytes) {
  if (!r || !bytes) {
    set_error("rnnl_linear_node_weights_size: bad arguments");
    return RNNL_ERR_INVALID;
  }
  *bytes = (size_t)(lin_trailer_off(r->d.n_nodes) + 64);
  return RNNL_OK;
}

int rnnl_linear_node_weights(rnnl_rules r, const float *rule_weights, int32_t n_rules, void *node_w, void *stream) {
  if (!r || !rule_weights || !node_w || n_rules != r->d.n_rules) {
    set_error("rnnl_linear_node_weights: bad arguments (rule_weights must hold n_rules floats)");
    return RNNL_ERR_INVALID;
  }
  unsigned char *out = static_cast<unsigned char *>(node_w);
  hipStream_t st = (hipStream_t)stream;
  RNNL_HIP_CHECK(hipMemsetAsync(out + lin_trailer_off(r->d.n_nodes), 0, 16, st));
  const int n = r->d.n_nodes;
  if (n == 0) return RNNL_OK;
  hipLaunchKernelGGL(lin_node_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, r->d, rule_weights, out);
  hipLaunchKernelGGL(lin_fix_kernel, dim3((unsigned)std::min((n + 255) / 256, 1024)), dim3(256), 0, st, n, out);
  RNNL_HIP_CHECK(hipGetLastError());
  return RNNL_OK;
}

int rnnl_predictor_forward(rnnl_graph g, rnnl_rules r, const void *node_w, int32_t feature, const int64_t *all_h,
                           const int64_t *all_r, const int64_t *etr, int32_t nq, float *score, uint8_t *mask,
                           int32_t *n_cand, void *ws, size_t ws_bytes, int32_t scale, void *stream) {
  if (!node_w || !score || (feature != RNNL_FEATURE_ADD && feature != RNNL_FEATURE_NONE)) {
    set_error("rnnl_predictor_forward: bad arguments");
    return RNNL_ERR_INVALID;
  }
  KParams p;
  if (int rc = setup_params("rnnl_predictor_forward", g, r, all_h, all_r, etr, nq, n_cand, ws, ws_bytes, scale, p))
    return rc;
  hipStream_t st = (hipStream_t)stream;
  RNNL_HIP_CHECK(hipMemsetAsync(ws, 0, HDR_WORDS_BYTES, st));
  if (nq == 0) return RNNL_OK;
  p.agg = RNNL_AGG_SUM;
  p.feature = feature;
  p.score = score;
  p.mask = mask;
  launch_ground(p, RNNL_AGG_SUM, st);
  launch_chunk_list(p, st);
  hipLaunchKernelGGL(score_linear_kernel, dim3((unsigned)std::min<int64_t>(nq, (int64_t)NUM_CU * 8)), dim3(BS), 0, st,
                     p, static_cast<const int *>(node_w));
  RNNL_HIP_CHECK(hipGetLastError());
  return RNNL_OK;
}

int rnnl_predictor_ground(rnnl_graph g, rnnl_rules r, const int64_t *all_h, const int64_t *all_r, const int64_t *etr,
                          int32_t nq, int32_t *n_cand, void *ws, size_t ws_bytes, int32_t scale, void *stream) {
  KParams p;
  if (int rc = setup_params("rnnl_predictor_ground", g, r, all_h, all_r, etr, nq, n_cand, ws, ws_bytes, scale, p))
    return rc;
  hipStream_t st = (hipStream_t)stream;
  RNNL_HIP_CHECK(hipMemsetAsync(ws, 0, HDR_WORDS_BYTES, st));
  if (nq == 0) return RNNL_OK;
  p.agg = RNNL_AGG_SUM;
  launch_ground(p, RNNL_AGG_SUM, st);
  launch_chunk_list(p, st);
  RNNL_HIP_CHECK(hipGetLastError());
  return RNNL_OK;
}

int rnnl_predictor_score(rnnl_graph g, rnnl_rules r, const void *node_w, int32_t feature, const int64_t *all_h,
                         const int64_t *all_r, int32_t nq, float *score, uint8_t *mask, int32_t *n_cand, void *ws,
                         size_t ws_bytes, int32_t scale, void *stream) {
  if (!node_w || !score || (feature != RNNL_FEATURE_ADD && feature != RNNL_FEATURE_NONE)) {
    set_error("rnnl_predictor_score: bad arguments");
    return RNNL_ERR_INVALID;
  }
  KParams p;
  if (int rc = setup_params("rnnl_predictor_score", g, r, all_h, all_r, nullptr, nq, n_cand, ws, ws_bytes, scale, p))
    return rc;
  if (nq == 0) return RNNL_OK;
  p.agg = RNNL_AGG_SUM;
  p.feature = feature;
  p.score = score;
  p.mask = mask;
  hipLaunchKernelGGL(score_linear_kernel, dim3((unsigned)std::min<int64_t>(nq, (int64_t)NUM_CU * 8)), dim3(BS), 0,
                     (hipStream_t)stream, p, static_cast<const int *>(node_w));
  RNNL_HIP_CHECK(hipGetLastError());
  return RNNL_OK;
}

int rnnl_predictor_rule_stats(void *ws, int32_t nq, int32_t scale, const int32_t *n_cand, rnnl_rules r,
                              const int64_t *all_r, const int64_t *all_t, int32_t ld, int64_t *pos, int64_t *tot,
                              void *stream) {
  if (!ws || nq < 0 || scale < 1 || !n_cand || !r || !all_r || !all_t || !pos || !tot ||
      ld < r->d.max_head_nodes || ld < 1) {
    set_error("rnnl_predictor_rule_stats: bad arguments (ld >= max_head_nodes)");
    return RNNL_ERR_INVALID;
  }
  if (nq == 0) return RNNL_OK;
  if ((int64_t)ld * 8 > 64 * 1024) {
    set_error("rnnl_predictor_rule_stats: head trie too large for the LDS table");
    return RNNL_ERR_INVALID;
  }
  KParams p = export_params(ws, nq, scale, n_cand);
  p.rl = r->d;
  p.all_r = all_r;
  hipLaunchKernelGGL(rule_stats_kernel, dim3((unsigned)std::min<int64_t>(nq, 4096)), dim3(BS), (size_t)ld * 8,
                     (hipStream_t)stream, p, all_t, ld, reinterpret_cast<long long *>(pos),
                     reinterpret_cast<long long *>(tot));
  RNNL_HIP_CHECK(hipGetLastError());
  return RNNL_OK;
}

int rnnl_predictor_backward(void *ws, int32_t nq, int32_t scale, const int32_t *n_cand, rnnl_rules r,
                            const int64_t *all_r, int32_t n_entities, const float *grad_score, int32_t ld,
                            double *grad_node, void *stream) {
  if (!ws || nq < 0 || scale < 1 || !n_cand || !r || !all_r || !grad_score || !grad_node || n_entities <= 0 ||
      ld < r->d.max_head_nodes || ld < 1) {
    set_error("rnnl_predictor_backward: bad arguments (ld >= max_head_nodes)");
    return RNNL_ERR_INVALID;
  }
  if (nq == 0) return RNNL_OK;
  if ((int64_t)ld * 8 > 64 * 1024) {
    set_error("rnnl_predictor_backward: head trie too large for the LDS table");
    return RNNL_ERR_INVALID;
  }
  KParams p = export_params(ws, nq, scale, n_cand);
  p.rl = r->d;
  p.all_r = all_r;
  p.g.E = n_entities;
  hipStream_t st = (hipStream_t)stream;
  const unsigned nb = (unsigned)std::min<int64_t>(nq, 4096);
  RNNL_HIP_CHECK(hipMemsetAsync(static_cast<unsigned char *>(ws) + 4 * H_BW_MAXG, 0, 16, st));
  hipLaunchKernelGGL(predictor_bw_stats_kernel, dim3(nb), dim3(BS), 0, st, p, grad_score);
  hipLaunchKernelGGL(predictor_backward_kernel, dim3(nb), dim3(BS), (size_t)ld * 8, st, p, grad_score, ld,
                     reinterpret_cast<unsigned long long *>(grad_node));
  hipLaunchKernelGGL(predictor_bw_fix_kernel, dim3((unsigned)std::min<int64_t>((r->d.n_nodes + 255) / 256, 1024)),
                     dim3(256), 0, st, p, r->d.n_nodes, reinterpret_cast<unsigned long long *>(grad_node));
  RNNL_HIP_CHECK(hipGetLastError());
  return RNNL_OK;
}

}  // extern "C"
