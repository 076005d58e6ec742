// PNA (FuncToNode) training path for gfx950 (MI355X): the aggregation over
// the grounding COO and its backward.
//
// Reference: src/layers.py:89-101 (degree, sum / sq_sum of count x rule
// embedding, min / max over the rules reaching a candidate) under the
// autograd of src/trainer.py:84-93.  The dense rest of FuncToNode (mean,
// std, degree scalers, Linear(192, 16), LayerNorm, ReLU) and score_model stay
// torch layers on these per-candidate statistics (layers.FuncToNode.finish:
// plain GEMMs and elementwise ops); what was ~15 torch ops on the exported
// COO — node tables by index_add / scatter_reduce, then per-candidate
// index_add / scatter_reduce — is one kernel each way:
//
//   pna_features_kernel   one workgroup per row (grid-stride), one lane per
//       candidate: the walk over its (trie node, path count) entries of the
//       node records (rnnl_node_weights, aggregator PNA: int32 fixed-point
//       sums of x and x^2, f32 min / max per node) — exact int64 sums, then
//       one rounding; deg = 1 + sum of count x rules at the node.
//   pna_grad_stats_kernel / pna_grad_nodes_kernel / pna_grad_rules_kernel
//       the backward: per node G1 = sum count x dL/dwsum, G2 likewise for
//       wsq, and each candidate's min / max gradient to one node tied at the
//       min / max (the smallest; the reference's dense .min(1) / .max(1)
//       route it to one index), split evenly among that node's tied rules —
//       all int64 fixed point at one scale per launch, each gradient rounded
//       to it once per candidate, so the sums depend neither on the order of
//       the adds nor on how a (node, candidate) pair is split over bucket
//       entries; then per rule dL/dx = G1 + 2 x G2 + its min / max shares.
#include <hip/hip_runtime.h>

#include <climits>
#include <string>

#include "fwd.h"

namespace rnnl {

constexpr int PG_BS = 256;
constexpr int PG_LDS_NODES = 96;  // the head's first nodes summed in LDS (4 tables: 48 KB)
constexpr int PG_GRID = 240;      // accumulation workgroups (one partial row block each)

struct PnaGradStats {
  unsigned int maxg, pad;
  unsigned long long sumk, ncand;
};

__device__ __forceinline__ const unsigned int *pna_trailer(const KParams &p, const unsigned char *node_w) {
  return reinterpret_cast<const unsigned int *>(node_w + (int64_t)p.rl.n_nodes * kStridePna);
}

// The row of candidate c (cand_off: exclusive prefix of n_cand, nq + 1
// entries): the largest q with cand_off[q] <= c.
__device__ __forceinline__ int cand_row(const int64_t *__restrict__ cand_off, int nq, int64_t c) {
  int lo = 0, hi = nq;  // cand_off[lo] <= c < cand_off[hi]
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (cand_off[mid] <= c) lo = mid; else hi = mid;
  }
  return lo;
}

// One wave per candidate (grid-stride over the launch's C candidates,
// row-major order), lane = (entry slot j = lane >> 4, dim d = lane & 15): the
// wave takes the candidate's bucket entries four at a time, each lane one
// (entry, dim) pair of the node records — no per-lane entry loops, so a few
// registers and every wave busy whatever the lists' lengths — then sums /
// min / max over the four slots by two xor shuffles.
__global__ __launch_bounds__(PG_BS) void pna_features_kernel(KParams p, const unsigned char *__restrict__ node_w,
                                                              const int64_t *__restrict__ cand_off, int64_t C,
                                                              float *__restrict__ wsum, float *__restrict__ wsq,
                                                              float *__restrict__ mn, float *__restrict__ mx,
                                                              float *__restrict__ deg, int64_t *__restrict__ row,
                                                              int64_t *__restrict__ ent,
                                                              unsigned long long *__restrict__ lsum) {
  const unsigned int *tr = pna_trailer(p, node_w);
  unsigned int *hdr = reinterpret_cast<unsigned int *>(p.ws);
  if (blockIdx.x == 0 && threadIdx.x == 0 && tr[2]) {  // the table cannot hold the aggregates
    atomicOr(&hdr[H_ERRBITS], (unsigned)ERR_NODE_RANGE);
    atomicOr(&hdr[H_STATUS], 2u);
  }
  const double inv1 = ldexp(1.0, -(int)tr[1]), inv2 = ldexp(1.0, -(int)tr[4]);
  const int lane = threadIdx.x & 63, d = lane & 15, j = lane >> 4;
  const int64_t nw = (int64_t)gridDim.x * (PG_BS / 64);
  for (int64_t c = (int64_t)blockIdx.x * (PG_BS / 64) + (threadIdx.x >> 6); c < C; c += nw) {
    const int q = cand_row(cand_off, p.nq, c);
    const int4 cr = p.cand[p.q_base[q] + (c - cand_off[q])];
    long long a1 = 0, a2 = 0;
    float m1 = __builtin_huge_valf(), m2 = -__builtin_huge_valf();
    unsigned long long dsum = 0, csum = 0;
#pragma unroll 1
    for (int e = cr.y + j; e < cr.y + cr.z; e += 4) {
      const int2 be = p.bent[e];
      const long long k = (uint32_t)be.y;
      const int *rec = reinterpret_cast<const int *>(node_w + (uint32_t)be.x * (uint32_t)kStridePna);
      a1 += k * rec[d];
      a2 += k * rec[16 + d];
      m1 = fminf(m1, __int_as_float(rec[32 + d]));
      m2 = fmaxf(m2, __int_as_float(rec[48 + d]));
      if (d == 0) {
        dsum += (unsigned long long)k * (unsigned)p.rl.node_nrules[be.x];
        csum += (unsigned long long)k;
      }
    }
#pragma unroll
    for (int o = 16; o <= 32; o <<= 1) {  // over the four entry slots
      a1 += __shfl_xor(a1, o, 64);
      a2 += __shfl_xor(a2, o, 64);
      m1 = fminf(m1, __shfl_xor(m1, o, 64));
      m2 = fmaxf(m2, __shfl_xor(m2, o, 64));
      dsum += __shfl_xor(dsum, o, 64);
      csum += __shfl_xor(csum, o, 64);
    }
    if (lane < 16) {
      wsum[c * 16 + d] = (float)((double)a1 * inv1);
      wsq[c * 16 + d] = (float)((double)a2 * inv2);
      mn[c * 16 + d] = m1;
      mx[c * 16 + d] = m2;
    }
    if (lane == 0) {
      if (csum >> 33) flag_acc_range(p);  // |record| < 2^30: the int64 sums are exact below 2^33 paths
      const float degf = (float)(dsum + 1);
      deg[c] = degf;  // layers.py:92: A_fn.sum(0) + 1
      row[c] = q;
      ent[c] = cr.x;
      // the row's sum of log(degree) in 2^32 fixed point (integer adds: order-free)
      atomicAdd(&lsum[q], (unsigned long long)(long long)llrint((double)logf(degf) * 4294967296.0));
    }
  }
}

// The rows' mean log-degree (layers.py:108-114), as the eval kernel's
// q_scale: from the order-free fixed-point sums, so the scalers are run-to-run
// bitwise; 0 for a row without candidates.
__global__ void pna_rowscale_kernel(const int32_t *__restrict__ n_cand, int nq,
                                    const unsigned long long *__restrict__ lsum, float *__restrict__ rscale) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= nq) return;
  const int nc = n_cand[q];
  const double sum = (double)(long long)lsum[q] / 4294967296.0;
  rscale[q] = nc > 0 ? (float)((float)sum / fmaxf((float)nc, 1e-6f)) : 0.f;
}

// The launch's max |incoming gradient| over the four statistics and its
// path-count and candidate totals (a max and integer sums: order-free).
__global__ __launch_bounds__(PG_BS) void pna_grad_stats_kernel(KParams p, const int64_t *__restrict__ cand_off,
                                                                int64_t C, const float *__restrict__ g0,
                                                                const float *__restrict__ g1,
                                                                const float *__restrict__ g2,
                                                                const float *__restrict__ g3,
                                                                PnaGradStats *__restrict__ st) {
  unsigned int m = 0u;
  unsigned long long k = 0ull, n = 0ull;
  for (int64_t c = (int64_t)blockIdx.x * PG_BS + threadIdx.x; c < C; c += (int64_t)gridDim.x * PG_BS) {
#pragma unroll
    for (int d = 0; d < 16; ++d) {
      m = max(m, __float_as_uint(fabsf(g0[c * 16 + d])));
      m = max(m, __float_as_uint(fabsf(g1[c * 16 + d])));
      m = max(m, __float_as_uint(fabsf(g2[c * 16 + d])));
      m = max(m, __float_as_uint(fabsf(g3[c * 16 + d])));
    }
    const int q = cand_row(cand_off, p.nq, c);
    const int4 cr = p.cand[p.q_base[q] + (c - cand_off[q])];
    for (int e = cr.y; e < cr.y + cr.z; ++e) k += (uint32_t)p.bent[e].y;
    ++n;
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    m = max(m, (unsigned int)__shfl_xor((int)m, o, 64));
    k += __shfl_xor(k, o, 64);
    n += __shfl_xor(n, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    if (m) atomicMax(&st->maxg, m);
    if (k) atomicAdd(&st->sumk, k);
    if (n) atomicAdd(&st->ncand, n);
  }
}

// 2^s with (sum count + candidates) x max |gradient| x 2^s < 2^62: every
// accumulator's total (count x dL/dwsum over entries, or a candidate's whole
// min / max gradient) fits int64.  bad: a non-finite gradient.
__device__ __forceinline__ int pna_grad_scale(const PnaGradStats *st, bool &bad) {
  bad = st->maxg >= 0x7f800000u;
  const double total = ((double)st->sumk + (double)st->ncand) * (double)__uint_as_float(st->maxg);
  return (bad || !(total > 0.0)) ? 0 : 61 - ilogb(total);
}

__device__ __forceinline__ unsigned long long pg_fix(double v, int sc) {
  return (unsigned long long)llrint(ldexp(v, sc));
}

// One wave per candidate (grid-stride over the C candidates), lane = (entry
// slot j, dim d) as pna_features_kernel: per bucket entry (node n, count k)
// G1[n] += k fix(dL/dwsum), G2[n] += k fix(dL/dwsq) — each gradient on the
// fixed-point grid once, times the integer count, so a (node, candidate) pair
// split over several bucket entries (phase A's raw duplicates, which vary
// with its LDS hash's insertion order) sums exactly as its merged entry — and
// the candidate's min / max gradient whole to the smallest trie node among
// its entries tied at the min / max (the reference's dense .min(1) / .max(1)
// route it to one index, layers.py:100-101; a node's duplicate entries tie
// with each other, so it gets the gradient once whatever the split).  A
// wave's adds go to 64 distinct (entry, dim) words (a lane per candidate had
// every lane of a wave add into the same few shared nodes: 2.2 ms per WN18RR
// batch).  Four int64 tables at the launch's scale; the first nl nodes from
// `lo` (a one-relation launch's head trie) summed in LDS and written as this
// workgroup's partial rows (summed by pna_grad_rules_kernel), the rest by
// int64 HBM atomics.
__global__ __launch_bounds__(PG_BS) void pna_grad_nodes_kernel(
    KParams p, const unsigned char *__restrict__ node_w, const int64_t *__restrict__ cand_off, int64_t C,
    const float *__restrict__ mn, const float *__restrict__ mx, const float *__restrict__ d_wsum,
    const float *__restrict__ d_wsq, const float *__restrict__ d_mn, const float *__restrict__ d_mx,
    const PnaGradStats *__restrict__ st, int lo, int nl, unsigned long long *__restrict__ G,
    long long *__restrict__ gpart, int64_t tab) {
  __shared__ unsigned long long s[4][PG_LDS_NODES * 16];  // G1 | G2 | Gmin | Gmax of nodes lo .. lo + nl
  bool bad;
  const int sc = pna_grad_scale(st, bad);
  for (int i = threadIdx.x; i < nl * 16; i += PG_BS) s[0][i] = s[1][i] = s[2][i] = s[3][i] = 0ull;
  __syncthreads();
  auto add = [&](int k, int n, int d, unsigned long long v) {
    const unsigned ln = (unsigned)(n - lo);
    if (ln < (unsigned)nl)
      atomicAdd(&s[k][ln * 16 + d], v);
    else
      atomicAdd(&G[k * tab + (int64_t)n * 16 + d], v);
  };
  const int lane = threadIdx.x & 63, d = lane & 15, j = lane >> 4;
  const int64_t nw = (int64_t)gridDim.x * (PG_BS / 64);
  if (!bad)  // (a non-finite gradient: pna_grad_rules_kernel writes NaN)
    for (int64_t c = (int64_t)blockIdx.x * (PG_BS / 64) + (threadIdx.x >> 6); c < C; c += nw) {
      const int q = cand_row(cand_off, p.nq, c);
      const int4 cr = p.cand[p.q_base[q] + (c - cand_off[q])];
      const long long f1 = (long long)pg_fix((double)d_wsum[c * 16 + d], sc);
      const long long f2 = (long long)pg_fix((double)d_wsq[c * 16 + d], sc);
      const float vmn = mn[c * 16 + d], vmx = mx[c * 16 + d];
      int nmn = INT_MAX, nmx = INT_MAX;  // the smallest node tied at the candidate's min / max (dim d)
#pragma unroll 1
      for (int e = cr.y + j; e < cr.y + cr.z; e += 4) {
        const int2 be = p.bent[e];
        const float *fr = reinterpret_cast<const float *>(node_w + (uint32_t)be.x * (uint32_t)kStridePna) + 32;
        const long long k = (long long)(uint32_t)be.y;
        if (fr[d] == vmn) nmn = min(nmn, be.x);
        if (fr[16 + d] == vmx) nmx = min(nmx, be.x);
        if (f1) add(0, be.x, d, (unsigned long long)(k * f1));
        if (f2) add(1, be.x, d, (unsigned long long)(k * f2));
      }
      nmn = min(nmn, __shfl_xor(nmn, 16, 64));
      nmn = min(nmn, __shfl_xor(nmn, 32, 64));
      nmx = min(nmx, __shfl_xor(nmx, 16, 64));
      nmx = min(nmx, __shfl_xor(nmx, 32, 64));
      if (j == 0) {
        const float gmn = d_mn[c * 16 + d], gmx = d_mx[c * 16 + d];
        if (gmn != 0.f && nmn != INT_MAX) add(2, nmn, d, pg_fix((double)gmn, sc));
        if (gmx != 0.f && nmx != INT_MAX) add(3, nmx, d, pg_fix((double)gmx, sc));
      }
    }
  __syncthreads();
  long long *row = gpart + (int64_t)blockIdx.x * 4 * nl * 16;
  for (int i = threadIdx.x; i < nl * 16; i += PG_BS)
#pragma unroll
    for (int k = 0; k < 4; ++k) row[k * nl * 16 + i] = (long long)s[k][i];
}

// Per (node, dim) of nodes [lo, hi): the node's four sums (its HBM table word
// plus, for the first nl nodes, the accumulation workgroups' partial rows —
// integer sums), then its member rules' gradient rows:
//   dL/dx_r[d] = G1 + 2 x_r[d] G2 (node_sum / node_sq are sums over the
//   members) + Gmin / (members tied at the node's min) if x_r[d] is the min,
//   + the same for the max.
__global__ __launch_bounds__(PG_BS) void pna_grad_rules_kernel(RulesDev rl, int lo, int hi,
                                                                const unsigned char *__restrict__ node_w,
                                                                const float *__restrict__ x, int ld,
                                                                const PnaGradStats *__restrict__ st,
                                                                const long long *__restrict__ G, int64_t tab,
                                                                const long long *__restrict__ gpart, int nrow,
                                                                int nl, float *__restrict__ d_x) {
  bool bad;
  const int sc = pna_grad_scale(st, bad);
  const int64_t total = (int64_t)(hi - lo) * 16;
  for (int64_t gid = (int64_t)blockIdx.x * PG_BS + threadIdx.x; gid < total; gid += (int64_t)gridDim.x * PG_BS) {
    const int n = lo + (int)(gid >> 4), d = (int)(gid & 15);
    const int kb = rl.node_rule_ptr[n], ke = rl.node_rule_ptr[n + 1];
    if (kb == ke) continue;
    long long g[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) g[k] = G[k * tab + (int64_t)n * 16 + d];
    if (gid < (int64_t)nl * 16)
      for (int b = 0; b < nrow; ++b)
#pragma unroll
        for (int k = 0; k < 4; ++k) g[k] += gpart[((int64_t)b * 4 + k) * nl * 16 + gid];
    const float *fr = reinterpret_cast<const float *>(node_w + (int64_t)n * kStridePna) + 32;
    const float vmn = fr[d], vmx = fr[16 + d];
    int tmn = 0, tmx = 0;
    for (int k = kb; k < ke; ++k) {
      const float v = x[(int64_t)rl.node_rules[k] * ld + d];
      tmn += v == vmn;
      tmx += v == vmx;
    }
    const float f1 = (float)ldexp((double)g[0], -sc), f2 = (float)ldexp((double)g[1], -sc);
    const float fmn = (float)ldexp((double)g[2], -sc), fmx = (float)ldexp((double)g[3], -sc);
    for (int k = kb; k < ke; ++k) {
      const int r = rl.node_rules[k];
      const float v = x[(int64_t)r * ld + d];
      float gr = f1 + 2.f * v * f2;
      if (v == vmn) gr += fmn / (float)tmn;
      if (v == vmx) gr += fmx / (float)tmx;
      d_x[(int64_t)r * 16 + d] = bad ? __builtin_nanf("") : gr;
    }
  }
}

// Scratch: four int64 node tables [n_nodes][16] | the accumulation
// workgroups' LDS partial rows [PG_GRID][4][PG_LDS_NODES][16] | stats
struct PgLayout {
  int64_t tab, gpart, stats, total;
};

static PgLayout pg_layout(int64_t n_nodes) {
  PgLayout L;
  L.tab = 16 * std::max<int64_t>(n_nodes, 1);  // int64 words per table
  L.gpart = align256(8 * 4 * L.tab);
  L.stats = align256(L.gpart + 8 * (int64_t)PG_GRID * 4 * PG_LDS_NODES * 16);
  L.total = L.stats + 256;
  return L;
}

}  // namespace rnnl

using namespace rnnl;

extern "C" {

int rnnl_pna_features(rnnl_rules r, const void *node_w, void *ws, int32_t nq, int32_t scale, const int32_t *n_cand,
                      const int64_t *cand_off, int64_t n_cand_total, float *wsum, float *wsq, float *mn, float *mx,
                      float *deg, int64_t *row, int64_t *ent, float *row_scale, void *row_scratch, void *stream) {
  if (!r || !node_w || !ws || nq < 0 || scale < 1 || !n_cand || !cand_off || n_cand_total < 0 || !wsum || !wsq ||
      !mn || !mx || !deg || !row || !ent || !row_scale || !row_scratch) {
    set_error("rnnl_pna_features: bad arguments");
    return RNNL_ERR_INVALID;
  }
  if (nq == 0) return RNNL_OK;
  hipStream_t st = (hipStream_t)stream;
  auto *lsum = static_cast<unsigned long long *>(row_scratch);
  RNNL_HIP_CHECK(hipMemsetAsync(lsum, 0, sizeof(unsigned long long) * (size_t)nq, st));
  KParams p = export_params(ws, nq, scale, n_cand);
  p.rl = r->d;
  if (n_cand_total > 0)
    hipLaunchKernelGGL(pna_features_kernel, dim3((unsigned)std::min<int64_t>((n_cand_total + 3) / 4, 8192)),
                       dim3(PG_BS), 0, st, p, static_cast<const unsigned char *>(node_w), cand_off, n_cand_total, wsum,
                       wsq, mn, mx, deg, row, ent, lsum);
  hipLaunchKernelGGL(pna_rowscale_kernel, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, st, n_cand, nq,
                     (const unsigned long long *)lsum, row_scale);
  RNNL_HIP_CHECK(hipGetLastError());
  return RNNL_OK;
}

int rnnl_pna_features_backward_scratch(rnnl_rules r, size_t *bytes) {
  if (!r || !bytes) {
    set_error("rnnl_pna_features_backward_scratch: bad arguments");
    return RNNL_ERR_INVALID;
  }
  *bytes = (size_t)pg_layout(r->d.n_nodes).total;
  return RNNL_OK;
}

int rnnl_pna_features_backward(rnnl_rules r, const void *node_w, const float *x, int32_t ld, void *ws, int32_t nq,
                               int32_t scale, const int64_t *all_r, const int32_t *n_cand, const int64_t *cand_off,
                               int64_t n_cand_total, const float *mn, const float *mx, const float *d_wsum,
                               const float *d_wsq, const float *d_mn, const float *d_mx, int32_t head, void *scratch,
                               size_t scratch_bytes, float *d_x, void *stream) {
  const PgLayout L = r ? pg_layout(r->d.n_nodes) : PgLayout{};
  if (!r || !node_w || !x || ld < 16 || !ws || nq < 0 || scale < 1 || !all_r || !n_cand || !cand_off ||
      n_cand_total < 0 || !mn || !mx || !d_wsum || !d_wsq || !d_mn || !d_mx || !scratch ||
      scratch_bytes < (size_t)L.total || !d_x || head >= (int)r->head_root.size()) {
    set_error("rnnl_pna_features_backward: bad arguments");
    return RNNL_ERR_INVALID;
  }
  hipStream_t st = (hipStream_t)stream;
  RNNL_HIP_CHECK(hipMemsetAsync(d_x, 0, sizeof(float) * 16 * (size_t)r->d.n_rules, st));
  if (nq == 0 || n_cand_total == 0) return RNNL_OK;
  // the nodes whose gradient can be non-zero: the head's trie (a training
  // batch is one relation; its first nodes summed in LDS), else every node
  int lo = 0, hi = r->d.n_nodes, nl = 0;
  if (head >= 0) {
    lo = std::max(r->head_root[head], 0);
    hi = r->head_root[head] < 0 ? lo : lo + r->head_nodes[head];
    nl = std::min(hi - lo, PG_LDS_NODES);
  }
  unsigned char *sb = static_cast<unsigned char *>(scratch);
  auto *G = reinterpret_cast<unsigned long long *>(sb);
  for (int k = 0; k < 4; ++k)
    if (hi > lo) RNNL_HIP_CHECK(hipMemsetAsync(G + k * L.tab + (int64_t)lo * 16, 0, (size_t)(hi - lo) * 16 * 8, st));
  auto *stats = reinterpret_cast<PnaGradStats *>(sb + L.stats);
  RNNL_HIP_CHECK(hipMemsetAsync(stats, 0, sizeof(PnaGradStats), st));
  KParams p = export_params(ws, nq, scale, n_cand);
  p.rl = r->d;
  p.all_r = all_r;
  const unsigned nb = (unsigned)std::min<int64_t>((n_cand_total + PG_BS - 1) / PG_BS, 4096);
  const unsigned na = (unsigned)std::min<int64_t>((n_cand_total + 3) / 4, PG_GRID);
  const auto *nw = static_cast<const unsigned char *>(node_w);
  hipLaunchKernelGGL(pna_grad_stats_kernel, dim3(nb), dim3(PG_BS), 0, st, p, cand_off, n_cand_total, d_wsum, d_wsq,
                     d_mn, d_mx, stats);
  hipLaunchKernelGGL(pna_grad_nodes_kernel, dim3(na), dim3(PG_BS), 0, st, p, nw, cand_off, n_cand_total, mn, mx, d_wsum,
                     d_wsq, d_mn, d_mx, (const PnaGradStats *)stats, lo, nl, G,
                     reinterpret_cast<long long *>(sb + L.gpart), L.tab);
  const int64_t nthreads = (int64_t)std::max(hi - lo, 0) * 16;
  if (nthreads > 0)
    hipLaunchKernelGGL(pna_grad_rules_kernel, dim3((unsigned)std::min<int64_t>((nthreads + PG_BS - 1) / PG_BS, 4096)),
                       dim3(PG_BS), 0, st, r->d, lo, hi, nw, x, ld, (const PnaGradStats *)stats,
                       reinterpret_cast<const long long *>(G), L.tab, reinterpret_cast<const long long *>(sb + L.gpart),
                       (int)na, nl, d_x);
  RNNL_HIP_CHECK(hipGetLastError());
  return RNNL_OK;
}

}  // extern "C"
