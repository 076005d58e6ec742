// PredictorPlus training backward for gfx950 (MI355X), K2^T: the gradient of
// FuncToNodeSum + score_model on the grounding COO.
//
// Reference: src/predictors.py:238-271 (rule_to_entity, cat with
// relation_emb, score_model, scatter into the score rows) and
// src/layers.py:9-77 (MLP, FuncToNodeSum), differentiated by torch autograd
// in the reference's training step (src/trainer.py:84-93).  Here, after the
// fused forward (rnnl_predictorplus_forward, whose workspace keeps the
// grounding COO and the scoring chunk list), three launches:
//
//   sum_backward_kernel   one wave x one chunk of <= 64 candidates at a time
//       (static chunk -> wave assignment: deterministic partial sums).  Per
//       candidate (lane) the forward is recomputed from the same folded node
//       records (y = W_add . feat + b_add, LayerNorm, ReLU, score_model) and
//       differentiated: dL/dy_c from the score gradient at (row, entity).
//       Then, lane-owned: lane l owns score_model.layers.0 rows 2l, 2l + 1 and
//       walks the chunk's 64 staged candidates (z_c, g_c) — weight gradients
//       as register sums, no atomics.  Each candidate's dL/dy_c goes to a
//       per-chunk slot, with the launch's max |dL/dy| and its sum of path
//       counts (order-independent: a max and an integer sum).
//   node_accum_kernel     per bucket entry (node n, count k) of a candidate:
//       G_n += k dL/dy_c, as int64 fixed point at one scale for the launch
//       (2^s with sum k x max |dL/dy| x 2^s < 2^62): integer sums, so the
//       result does not depend on the order of the adds — run-to-run bitwise
//       (G_n is the gradient of the node's un-folded rule-embedding sum
//       before the Linear).
//   node_grad_kernel      per trie node: dL/dx_rule = W_add^T G_n for each
//       member rule (the reference's index_select / matmul backward), and
//       dL/dW_add = sum_n G_n (x) s_n with s_n the node's embedding sum.
//   grad_reduce_kernel    the per-block partials summed in a fixed order into
//       the parameter gradients; rel_grad_kernel: relation_emb's gradient of a
//       one-relation launch (a training batch) as W0[:, 16:]^T dL/db0, in a
//       fixed order (mixed-relation launches: fp64 atomics per relation run).
//
// Not differentiated here: the grounding (integer, no gradient: data.py:138
// torch.no_grad), the entity feature (bias: column sums; RotatE: its own HIP
// backward in rotate.hip) — the caller adds those.
#include <hip/hip_runtime.h>

#include "fwd.h"

namespace rnnl {

constexpr int BWB = 256;        // threads per workgroup
constexpr int BW_WAVES = BWB / 64;
// per-block partial row (floats): fields in the order grad_reduce_kernel maps them
enum : int {
  PB_W0 = 0,                  // score_model.layers.0.weight (128 x 32, row-major)
  PB_B0 = PB_W0 + 128 * 32,   // score_model.layers.0.bias (128)
  PB_W1 = PB_B0 + 128,        // score_model.layers.1.weight (128)
  PB_LNW = PB_W1 + 128,       // layer_norm.weight (16)
  PB_LNB = PB_LNW + 16,       // layer_norm.bias (16)
  PB_ADDB = PB_LNB + 16,      // add_model bias (16)
  PB_B1 = PB_ADDB + 16,       // score_model.layers.1.bias (1, padded to 4)
  PB_N = PB_B1 + 4
};
constexpr int BW_GRID = 256;    // sum_backward_kernel workgroups (max)
constexpr int BW_BIG = 24;      // bucket lists longer than this are walked by the whole wave
// Per-workgroup LDS sums of G_n for the first BW_LDS_NODES trie nodes of the
// batch's head relation.  Many candidates of a batch share a node (a short
// rule reaches most of them), so per-entry global atomics serialise on a few
// addresses (2.4 ms per FB15k-237 batch); summed in LDS first, each
// workgroup writes one partial row.  int64 fixed point (node_accum_kernel):
// exact integer sums in any order; the trie's breadth-first numbering puts
// the short (most shared) rule prefixes first, and nodes past the LDS range
// take int64 HBM atomics.
constexpr int BW_LDS_NODES = 768;
// stats words (scratch): u32 max |dL/dy| bits, pad, u64 sum of the path counts
// of the entries of candidates with a non-zero score gradient
struct BwStats {
  unsigned int maxgy, pad;
  unsigned long long sumk;
};

// The launch's fixed-point scale: 2^s with sum k x max|dL/dy| x 2^s < 2^62, so
// every term and every partial sum of count x dL/dy fits int64.  `bad`: a
// non-finite dL/dy (the gradients are then NaN, as the reference's would be).
__device__ __forceinline__ int bw_scale(const BwStats *st, bool &bad) {
  const float mg = __uint_as_float(st->maxgy);
  bad = st->maxgy >= 0x7f800000u;
  const double total = (double)st->sumk * (double)mg;
  return (bad || !(total > 0.0)) ? 0 : 61 - ilogb(total);
}
constexpr int NG_GRID = 128;    // node_grad_kernel workgroups (max)

struct BwdLds {
  float w0[128][32];            // score_model.layers.0.weight
  float w1[128], b0[128];
  float addb[16], lnw[16], lnb[16];
  float relb[BW_WAVES][128];    // per wave: b0 + W0[:, 16:] . rel_emb[r]
  float stage[BW_WAVES][64][20];  // per wave: candidate c's z[16] | g | pad
  float red[BWB];               // block reduction
};

__device__ __forceinline__ float relu_f(float x) { return x > 0.f ? x : 0.f; }

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Sum a per-lane value over the block's waves into lane-independent totals:
// every wave adds its lane values of one field into red[] (BWB floats), the
// caller reads red[field index] after the barrier.  Used for the lane-owned
// accumulators (lane l of every wave owns the same rows).
__device__ __forceinline__ float block_sum_lane(BwdLds &S, float v) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  __syncthreads();
  S.red[wv * 64 + lane] = v;
  __syncthreads();
  float t = 0.f;
  if (wv == 0)
#pragma unroll
    for (int w = 0; w < BW_WAVES; ++w) t += S.red[w * 64 + lane];
  return t;  // valid in wave 0
}

// gy: per chunk c of the chunk list, lane l: dL/dy of candidate s0 + l at
// gy[(c * 16 + d) * 64 + l] (chunk capacity gy_cap).  single: every row is of
// one relation (relation_emb's gradient is then rel_grad_kernel's).
__global__ __launch_bounds__(BWB) void sum_backward_kernel(KParams p, const float *__restrict__ grad,
                                                            double *__restrict__ grel, float *__restrict__ part,
                                                            float *__restrict__ gy_out, int64_t gy_cap,
                                                            BwStats *__restrict__ stats, int single) {
  __shared__ BwdLds S;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  for (int i = tid; i < 128 * 32; i += BWB) S.w0[i >> 5][i & 31] = p.s0_w[i];
  for (int i = tid; i < 128; i += BWB) {
    S.w1[i] = p.s1_w[i];
    S.b0[i] = p.s0_b[i];
  }
  if (tid < 16) {
    S.addb[tid] = p.add_b[tid];
    S.lnw[tid] = p.ln_w[tid];
    S.lnb[tid] = p.ln_b[tid];
  }
  __syncthreads();
  const unsigned int *hdr = reinterpret_cast<const unsigned int *>(p.ws);
  const long long nchunks = (long long)*reinterpret_cast<const unsigned long long *>(hdr + H_CHUNKS);
  const int shift = (int)reinterpret_cast<const unsigned int *>(p.node_w + (int64_t)p.rl.n_nodes * kStrideSum)[1];
  const double inv_scale = ldexp(1.0, -shift);
  const int E = p.g.E;
  // lane-owned rows of score_model.layers.0: o = 2 lane + j
  float w0r[2][16];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int i = 0; i < 16; ++i) w0r[j][i] = S.w0[2 * lane + j][i];
  float a_w0[2][16], a_w1[2], a_b0[2], a_rel[2][16], run_s[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    a_w1[j] = a_b0[j] = run_s[j] = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) a_w0[j][i] = a_rel[j][i] = 0.f;
  }
  // lane-local sums over the candidates this lane differentiated
  float a_lnw[16], a_lnb[16], a_addb[16], a_b1 = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) a_lnw[i] = a_lnb[i] = a_addb[i] = 0.f;
  float *relb = S.relb[wv];
  float(*stage)[20] = S.stage[wv];
  int cur_r = -1;
  // the relation run's lane-owned sums of dL/dh (for the relation half of
  // layers.0 and relation_emb) flushed when the relation changes / at the end
  auto flush_rel = [&](int r) {
    if (r < 0) return;
    if (single) {  // relation_emb's gradient from dL/db0 (rel_grad_kernel)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int i = 0; i < 16; ++i) a_rel[j][i] = fmaf(run_s[j], p.rel_emb[r * 16 + i], a_rel[j][i]);
      run_s[0] = run_s[1] = 0.f;
      return;
    }
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int i = 0; i < 16; ++i) a_rel[j][i] = fmaf(run_s[j], p.rel_emb[r * 16 + i], a_rel[j][i]);
    // relation_emb[r][i] gradient: sum_o S_o W0[o][16 + i]
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      float v = run_s[0] * S.w0[2 * lane][16 + i] + run_s[1] * S.w0[2 * lane + 1][16 + i];
      v = wave_sum(v);
      if (lane == i) unsafeAtomicAdd(grel + r * 16 + i, (double)v);
    }
    run_s[0] = run_s[1] = 0.f;
  };
  const long long nw = (long long)gridDim.x * BW_WAVES;
  unsigned int my_max = 0u;         // lane max |dL/dy| bits
  unsigned long long my_k = 0ull;   // lane sum of the path counts
#pragma unroll 1
  for (long long c = (long long)blockIdx.x * BW_WAVES + wv; c < nchunks && c < gy_cap; c += nw) {
    const int2 ck = p.chunks[c];
    const int q = __builtin_amdgcn_readfirstlane(ck.x);
    const int s0 = __builtin_amdgcn_readfirstlane(ck.y);
    const int r = __builtin_amdgcn_readfirstlane((int)p.all_r[q]);
    if (r != cur_r) {
      flush_rel(cur_r);
      wave_lds_sync();
      for (int o = lane; o < 128; o += 64) {
        float acc = S.b0[o];
        for (int i = 0; i < 16; ++i) acc = fmaf(S.w0[o][16 + i], p.rel_emb[r * 16 + i], acc);
        relb[o] = acc;
      }
      wave_lds_sync();
      cur_r = r;
    }
    const int nc = p.n_cand[q];
    const int64_t qb = p.q_base[q];
    const int s = s0 + lane;
    const bool live = s < nc;
    int4 cr = make_int4(0, 0, 0, 0);
    float g = 0.f;
    double acc[16];
#pragma unroll
    for (int d = 0; d < 16; ++d) acc[d] = 0.0;
    unsigned long long ksum = 0ull;  // the candidate's sum of path counts
    if (live) {
      cr = p.cand[qb + s];
      g = grad[(int64_t)q * E + cr.x];
      if (cr.z <= BW_BIG)  // short lists: the lane's own walk
#pragma unroll 1
        for (int e = cr.y; e < cr.y + cr.z; ++e) {
          const int2 be = p.bent[e];
          ksum += (uint32_t)be.y;
          const double k = (double)(uint32_t)be.y;
          const int *x = reinterpret_cast<const int *>(p.node_w + (uint32_t)be.x * (uint32_t)kStrideSum);
#pragma unroll
          for (int d = 0; d < 16; ++d) acc[d] = fma(k, (double)x[d], acc[d]);
        }
    }
    // long lists (> BW_BIG entries) gathered by the whole wave: a lane's own
    // walk would set the chunk's time (two dependent loads per entry)
#pragma unroll 1
    for (uint64_t big = __ballot(live && cr.z > BW_BIG); big; big &= big - 1) {
      const int owner = __builtin_ctzll(big);
      const int beg = __builtin_amdgcn_readlane(cr.y, owner), cnt = __builtin_amdgcn_readlane(cr.z, owner);
      double a[16];
#pragma unroll
      for (int d = 0; d < 16; ++d) a[d] = 0.0;
      unsigned long long kk = 0ull;
#pragma unroll 1
      for (int e = beg + lane; e < beg + cnt; e += 64) {
        const int2 be = p.bent[e];
        kk += (uint32_t)be.y;
        const double k = (double)(uint32_t)be.y;
        const int *x = reinterpret_cast<const int *>(p.node_w + (uint32_t)be.x * (uint32_t)kStrideSum);
#pragma unroll
        for (int d = 0; d < 16; ++d) a[d] = fma(k, (double)x[d], a[d]);
      }
      kk = wave_sum(kk);
      if (lane == owner) ksum = kk;
#pragma unroll
      for (int d = 0; d < 16; ++d) {
        const double t = wave_sum(a[d]);
        if (lane == owner) acc[d] = t;
      }
    }
    // FuncToNodeSum tail: y = feat + b, LayerNorm, ReLU (as the forward's sum_hidden)
    float y[16], xh[16], z[16];
#pragma unroll
    for (int d = 0; d < 16; ++d) y[d] = (float)(acc[d] * inv_scale) + S.addb[d];
    float mu = 0.f;
#pragma unroll
    for (int d = 0; d < 16; ++d) mu += y[d];
    mu = mu / 16.0f;
    float var = 0.f;
#pragma unroll
    for (int d = 0; d < 16; ++d) var = fmaf(y[d] - mu, y[d] - mu, var);
    var = var / 16.0f;
    const float rstd = 1.0f / sqrtf(var + 1e-5f);
#pragma unroll
    for (int d = 0; d < 16; ++d) {
      xh[d] = (y[d] - mu) * rstd;
      z[d] = relu_f(xh[d] * S.lnw[d] + S.lnb[d]);
    }
    // score_model backward to z: dL/dz = W0[:, :16]^T (g W1 [h > 0])
    float gz[16];
#pragma unroll
    for (int d = 0; d < 16; ++d) gz[d] = 0.f;
#pragma unroll 2
    for (int o = 0; o < 128; ++o) {
      float h = relb[o];
#pragma unroll
      for (int i = 0; i < 16; ++i) h = fmaf(S.w0[o][i], z[i], h);
      const float gh = h > 0.f ? g * S.w1[o] : 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) gz[i] = fmaf(gh, S.w0[o][i], gz[i]);
    }
    // ReLU, LayerNorm backward: dL/dy = rstd (gxh - mean(gxh) - xh mean(gxh xh))
    float gxh[16], m1 = 0.f, m2 = 0.f;
#pragma unroll
    for (int d = 0; d < 16; ++d) {
      const float gx1 = z[d] > 0.f ? gz[d] : 0.f;
      a_lnw[d] = fmaf(gx1, xh[d], a_lnw[d]);
      a_lnb[d] += gx1;
      gxh[d] = gx1 * S.lnw[d];
      m1 += gxh[d];
      m2 = fmaf(gxh[d], xh[d], m2);
    }
    m1 = m1 / 16.0f;
    m2 = m2 / 16.0f;
    float gy[16];
#pragma unroll
    for (int d = 0; d < 16; ++d) {
      gy[d] = rstd * (gxh[d] - m1 - xh[d] * m2);  // NaN-preserving |.| max below
      a_addb[d] += gy[d];
    }
    a_b1 += g;
    // the candidate's dL/dy for node_accum_kernel (0 where there is no score
    // gradient: those candidates add nothing to G_n)
    const bool adds = live && g != 0.f;
#pragma unroll
    for (int d = 0; d < 16; ++d) {
      const float v = adds ? gy[d] : 0.f;
      gy_out[((int64_t)c * 16 + d) * 64 + lane] = v;
      my_max = max(my_max, __float_as_uint(fabsf(v)));
    }
    if (adds) my_k += ksum;
    // stage (z, g) for the lane-owned weight sums
#pragma unroll
    for (int d = 0; d < 16; ++d) stage[lane][d] = z[d];
    stage[lane][16] = live ? g : 0.f;
    wave_lds_sync();
#pragma unroll 1
    for (int cc = 0; cc < 64; ++cc) {
      const float gc = stage[cc][16];
      if (gc == 0.f) continue;  // wave-uniform (one LDS word)
      float zc[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) zc[i] = stage[cc][i];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        float h = relb[2 * lane + j];
#pragma unroll
        for (int i = 0; i < 16; ++i) h = fmaf(w0r[j][i], zc[i], h);
        if (h > 0.f) {
          a_w1[j] = fmaf(gc, h, a_w1[j]);
          const float gh = gc * S.w1[2 * lane + j];
          a_b0[j] += gh;
          run_s[j] += gh;
#pragma unroll
          for (int i = 0; i < 16; ++i) a_w0[j][i] = fmaf(gh, zc[i], a_w0[j][i]);
        }
      }
    }
    wave_lds_sync();  // the next chunk rewrites the stage
  }
  flush_rel(cur_r);
  // the launch's max |dL/dy| and sum of path counts: one atomic per wave
  // (a max and an integer sum: order-independent)
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    my_max = max(my_max, (unsigned int)__shfl_xor((int)my_max, o, 64));
    my_k += __shfl_xor(my_k, o, 64);
  }
  if (lane == 0) {
    if (my_max) atomicMax(&stats->maxgy, my_max);
    if (my_k) atomicAdd(&stats->sumk, my_k);
  }
  // block partial row: lane-owned fields summed over the waves (fixed order),
  // lane-local fields summed over the lanes, then over the waves
  // field-major partials: field f of this workgroup at part[f * BW_GRID + block]
  float *row = part + blockIdx.x;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int o = 2 * lane + j;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float t1 = block_sum_lane(S, a_w0[j][i]);
      if (wv == 0) row[(PB_W0 + o * 32 + i) * BW_GRID] = t1;
      const float t2 = block_sum_lane(S, a_rel[j][i]);
      if (wv == 0) row[(PB_W0 + o * 32 + 16 + i) * BW_GRID] = t2;
    }
    const float t3 = block_sum_lane(S, a_b0[j]);
    if (wv == 0) row[(PB_B0 + o) * BW_GRID] = t3;
    const float t4 = block_sum_lane(S, a_w1[j]);
    if (wv == 0) row[(PB_W1 + o) * BW_GRID] = t4;
  }
#pragma unroll
  for (int d = 0; d < 16; ++d) {
    const float v1 = block_sum_lane(S, wave_sum(a_lnw[d]));
    const float v2 = block_sum_lane(S, wave_sum(a_lnb[d]));
    const float v3 = block_sum_lane(S, wave_sum(a_addb[d]));
    if (tid == 0) {
      row[(PB_LNW + d) * BW_GRID] = v1;
      row[(PB_LNB + d) * BW_GRID] = v2;
      row[(PB_ADDB + d) * BW_GRID] = v3;
    }
  }
  const float vb = block_sum_lane(S, wave_sum(a_b1));
  if (tid == 0) {
    row[PB_B1 * BW_GRID] = vb;
  }
}

// G_n += k dL/dy_c per bucket entry (node n, count k) of the candidates of
// the chunk list, as int64 fixed point at the launch's scale (bw_scale):
// LDS sums for the head's first nl nodes (one int64 partial row per
// workgroup, summed by node_grad_kernel), int64 HBM atomics past them.
// Integer adds: the sums do not depend on their order.
__global__ __launch_bounds__(BWB) void node_accum_kernel(KParams p, const float *__restrict__ gy, int64_t gy_cap,
                                                          const BwStats *__restrict__ stats,
                                                          unsigned long long *__restrict__ gnode,
                                                          long long *__restrict__ gpart, int lo, int nl) {
  __shared__ unsigned long long gacc[BW_LDS_NODES * 16];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  for (int i = tid; i < nl * 16; i += BWB) gacc[i] = 0ull;
  __syncthreads();
  bool bad;
  const int sc = bw_scale(stats, bad);
  const unsigned int *hdr = reinterpret_cast<const unsigned int *>(p.ws);
  const long long nchunks = (long long)*reinterpret_cast<const unsigned long long *>(hdr + H_CHUNKS);
  // bad (a non-finite dL/dy): fp64 sums in the same words instead, so that
  // NaN / inf reach exactly the nodes the reference's would
  // each dL/dy is rounded to the fixed-point grid once and multiplied by the
  // integer count: a (node, candidate) pair split over several bucket entries
  // (phase A's raw duplicates, which vary with the LDS hash's insertion order)
  // then sums to exactly its merged entry's k x fix(dL/dy)
  auto add = [&](const int2 be, const float (&g)[16]) {
    const double k = (double)(uint32_t)be.y;
    const long long ki = (long long)(uint32_t)be.y;
    const unsigned ln = (unsigned)(be.x - lo);
#pragma unroll
    for (int d = 0; d < 16; ++d) {
      if (g[d] == 0.f) continue;
      unsigned long long *w = ln < (unsigned)nl ? &gacc[ln * 16 + d] : &gnode[(int64_t)be.x * 16 + d];
      if (bad)
        atomicAdd(reinterpret_cast<double *>(w), k * (double)g[d]);
      else
        atomicAdd(w, (unsigned long long)(ki * llrint(ldexp((double)g[d], sc))));
    }
  };
  const long long nw = (long long)gridDim.x * BW_WAVES;
#pragma unroll 1
    for (long long c = (long long)blockIdx.x * BW_WAVES + wv; c < nchunks && c < gy_cap; c += nw) {
      const int2 ck = p.chunks[c];
      const int q = __builtin_amdgcn_readfirstlane(ck.x);
      const int s0 = __builtin_amdgcn_readfirstlane(ck.y);
      const int nc = p.n_cand[q];
      const bool live = s0 + lane < nc;
      float g[16];
      bool any = false;
#pragma unroll
      for (int d = 0; d < 16; ++d) {
        g[d] = gy[((int64_t)c * 16 + d) * 64 + lane];
        any = any || g[d] != 0.f;
      }
      int4 cr = make_int4(0, 0, 0, 0);
      if (live && any) cr = p.cand[p.q_base[q] + s0 + lane];
      if (live && any && cr.z <= BW_BIG)
#pragma unroll 1
        for (int e = cr.y; e < cr.y + cr.z; ++e) add(p.bent[e], g);
      // long lists: the whole wave adds the owner's dL/dy into its entries
#pragma unroll 1
      for (uint64_t big = __ballot(live && any && cr.z > BW_BIG); big; big &= big - 1) {
        const int owner = __builtin_ctzll(big);
        const int beg = __builtin_amdgcn_readlane(cr.y, owner), cnt = __builtin_amdgcn_readlane(cr.z, owner);
        float go[16];
#pragma unroll
        for (int d = 0; d < 16; ++d)
          go[d] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, g[d]), owner));
#pragma unroll 1
        for (int e = beg + lane; e < beg + cnt; e += 64) add(p.bent[e], go);
      }
    }
  __syncthreads();
  // this workgroup's G_n of the head's first nl nodes: one partial row
  // (summed per node by node_grad_kernel; atomics from every workgroup to
  // the same node words serialised at ~0.3 ms per FB15k-237 batch)
  long long *grow = gpart + (int64_t)blockIdx.x * nl * 16;
  for (int i = tid; i < nl * 16; i += BWB) grow[i] = (long long)gacc[i];
}

// Per trie node n of [lo, hi) (16 lanes per node, lane d = dimension d):
// member rules' gradient rows W_add^T G_n, and the block's partial of
// dL/dW_add = sum_n G_n (x) s_n (s_n: the members' embedding sum, f32 in
// rule order as node_weights_kernel forms it).  part: 256 floats per block.
// G_n = (the int64 HBM sums (nodes past the LDS range) + the accumulation
// workgroups' int64 partial rows gpart[b][n - lo] (b < nrow, n < lo + nl))
// x 2^-s: exact integer sums, then one rounding.
__global__ __launch_bounds__(BWB) void node_grad_kernel(RulesDev rl, int lo, int hi,
                                                         const long long *__restrict__ gnode,
                                                         const long long *__restrict__ gpart, int nrow, int nl,
                                                         const BwStats *__restrict__ stats,
                                                         const float *__restrict__ emb, int ld,
                                                         const float *__restrict__ add_w, float *__restrict__ gemb,
                                                         int gld, float *__restrict__ part) {
  __shared__ float s_w[256];
  __shared__ float s_red[BW_WAVES][256];
  const int tid = threadIdx.x, d = tid & 15;
  bool bad;
  const int sc = bw_scale(stats, bad);
  s_w[tid] = add_w[tid];  // (16 x 16) row-major: y[i] = sum_j W[i][j] f[j]
  __syncthreads();
  float acc[16];  // lane d: sum_n G_n[d] s_n[j]
#pragma unroll
  for (int j = 0; j < 16; ++j) acc[j] = 0.f;
  const int64_t total = (int64_t)(hi - lo) * 16;
  // (total is a multiple of 16 and the stride too: a node's 16 lanes enter
  // and leave the loop together, as the width-16 shuffles need)
  for (int64_t gid = (int64_t)blockIdx.x * BWB + tid; gid < total; gid += (int64_t)gridDim.x * BWB) {
    const int n = lo + (int)(gid >> 4);
    float gn;
    if (!bad) {
      long long gi = gnode[(int64_t)n * 16 + d];
      if (gid < (int64_t)nl * 16) {
        long long a[4] = {0, 0, 0, 0};
        int b = 0;
        for (; b + 4 <= nrow; b += 4)
#pragma unroll
          for (int u = 0; u < 4; ++u) a[u] += gpart[(int64_t)(b + u) * nl * 16 + gid];
        for (; b < nrow; ++b) a[0] += gpart[(int64_t)b * nl * 16 + gid];
        gi += (a[0] + a[1]) + (a[2] + a[3]);
      }
      gn = (float)ldexp((double)gi, -sc);
    } else {  // non-finite dL/dy: the fp64 sums of node_accum_kernel's fallback
      double gd = __longlong_as_double(gnode[(int64_t)n * 16 + d]);
      if (gid < (int64_t)nl * 16)
        for (int b = 0; b < nrow; ++b) gd += __longlong_as_double(gpart[(int64_t)b * nl * 16 + gid]);
      gn = (float)gd;
    }
    float s = 0.f;
    const int kb = rl.node_rule_ptr[n], ke = rl.node_rule_ptr[n + 1];
    for (int k = kb; k < ke; ++k) s += emb[(int64_t)rl.node_rules[k] * ld + d];
    // dL/dx[d] = sum_i W[i][d] G[i]
    float gx = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) gx = fmaf(s_w[i * 16 + d], __shfl(gn, i, 16), gx);
    for (int k = kb; k < ke; ++k) gemb[(int64_t)rl.node_rules[k] * gld + d] = gx;
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[j] = fmaf(gn, __shfl(s, j, 16), acc[j]);
  }
  // lanes d, d + 16, d + 32, d + 48 of a wave hold the same row: fold, then over the waves
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    acc[j] += __shfl_xor(acc[j], 16, 64);
    acc[j] += __shfl_xor(acc[j], 32, 64);
  }
  if ((tid & 63) < 16)
#pragma unroll
    for (int j = 0; j < 16; ++j) s_red[tid >> 6][d * 16 + j] = acc[j];
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int w = 0; w < BW_WAVES; ++w) t += s_red[w][tid];
  part[(int64_t)tid * NG_GRID + blockIdx.x] = t;  // field-major
}

// Fixed-order sums of the partials into the gradient tensors: one wave per
// field, lanes over the workgroups' partials (field-major: coalesced), a
// butterfly (fixed order) over the lanes.
__global__ __launch_bounds__(BWB) void grad_reduce_kernel(const float *__restrict__ part, int nrow,
                                                           const float *__restrict__ npart, int nnrow,
                                                           const double *__restrict__ grel, int R,
                                                           rnnl_sum_grads gr) {
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * BW_WAVES + (threadIdx.x >> 6);
  if (i < PB_N) {
    float t = 0.f;
    for (int k = lane; k < nrow; k += 64) t += part[(int64_t)i * BW_GRID + k];
    t = wave_sum(t);
    if (lane != 0) return;
    if (i < PB_B0) gr.s0_w[i] = t;
    else if (i < PB_W1) gr.s0_b[i - PB_B0] = t;
    else if (i < PB_LNW) gr.s1_w[i - PB_W1] = t;
    else if (i < PB_LNB) gr.ln_w[i - PB_LNW] = t;
    else if (i < PB_ADDB) gr.ln_b[i - PB_LNB] = t;
    else if (i < PB_B1) gr.add_b[i - PB_ADDB] = t;
    else if (i == PB_B1) gr.s1_b[0] = t;
    return;
  }
  const int j = i - PB_N;
  if (j < 256) {
    float t = 0.f;
    for (int k = lane; k < nnrow; k += 64) t += npart[(int64_t)j * NG_GRID + k];
    t = wave_sum(t);
    if (lane == 0) gr.add_w[j] = t;
    return;
  }
  const int k = (j - 256) * 64 + lane;  // relation_emb: a wave per 64 entries
  if (k < R * 16) gr.rel_emb[k] = (float)grel[k];
}

// relation_emb's gradient of a one-relation launch: the relation half of
// score_model.layers.0 sees rel_emb[head] in every candidate, so
// dL/drel_emb[head][i] = sum_o W0[o][16 + i] dL/db0[o] (dL/db0 from
// grad_reduce_kernel; o ascending), every other relation 0.
__global__ void rel_grad_kernel(const float *__restrict__ s0_w, int head, rnnl_sum_grads gr) {
  const int i = threadIdx.x;
  if (i >= 16) return;
  float t = 0.f;
  for (int o = 0; o < 128; ++o) t = fmaf(s0_w[o * 32 + 16 + i], gr.s0_b[o], t);
  gr.rel_emb[head * 16 + i] = t;
}

// Scratch carve-up (bytes): gnode i64 [n_nodes x 16] | grel f64 [R x 16] |
// partial rows f32 [BW_GRID x PB_N] | node partials f32 [NG_GRID x 256] |
// LDS-node partial rows i64 [BW_GRID x BW_LDS_NODES x 16] | stats
struct BwdLayout {
  int64_t gnode, grel, part, npart, gpart, stats, total;
};

static BwdLayout bwd_layout(int64_t n_nodes, int64_t R) {
  BwdLayout L;
  int64_t o = 0;
  L.gnode = o;
  o = align256(o + 8 * 16 * std::max<int64_t>(n_nodes, 1));
  L.grel = o;
  o = align256(o + 8 * 16 * std::max<int64_t>(R, 1));
  L.part = o;
  o = align256(o + 4 * (int64_t)BW_GRID * PB_N);
  L.npart = o;
  o = align256(o + 4 * (int64_t)NG_GRID * 256);
  L.gpart = o;
  o = align256(o + 8 * (int64_t)BW_GRID * BW_LDS_NODES * 16);
  L.stats = o;
  o = align256(o + (int64_t)sizeof(BwStats));
  L.total = o;
  return L;
}

}  // namespace rnnl

using namespace rnnl;

extern "C" {

int rnnl_predictorplus_backward_size(rnnl_rules r, int32_t n_relations, size_t *bytes) {
  if (!r || !bytes || n_relations <= 0) {
    set_error("rnnl_predictorplus_backward_size: bad arguments");
    return RNNL_ERR_INVALID;
  }
  *bytes = (size_t)bwd_layout(r->d.n_nodes, n_relations).total;
  return RNNL_OK;
}

// per-call scratch: one dL/dy slot of 16 x 64 floats per scoring chunk
// (<= n_cand_total / 64 + one per row)
static int64_t gy_chunks(int64_t nq, int64_t n_cand_total) { return n_cand_total / 64 + nq + 1; }

int rnnl_predictorplus_backward_rows_size(int32_t nq, int64_t n_cand_total, size_t *bytes) {
  if (!bytes || nq < 0 || n_cand_total < 0) {
    set_error("rnnl_predictorplus_backward_rows_size: bad arguments");
    return RNNL_ERR_INVALID;
  }
  *bytes = (size_t)gy_chunks(nq, n_cand_total) * 16 * 64 * sizeof(float);
  return RNNL_OK;
}

int rnnl_predictorplus_backward(rnnl_graph g, rnnl_rules r, const rnnl_predictor_params *pp, const float *emb,
                                int32_t ld, const int64_t *all_r, int32_t nq, const float *grad_score,
                                const int32_t *n_cand, int64_t n_cand_total, void *ws, size_t ws_bytes,
                                int32_t scale, int32_t head, void *scratch, size_t scratch_bytes,
                                void *rows_scratch, size_t rows_bytes, const rnnl_sum_grads *gr, void *stream) {
  if (!g || !r || !pp || !emb || ld < 16 || !all_r || nq < 0 || !grad_score || !n_cand || !ws || scale < 1 ||
      !scratch || !gr || !gr->emb || gr->emb_ld < 16 || !gr->add_w || !gr->add_b || !gr->ln_w || !gr->ln_b ||
      !gr->s0_w || !gr->s0_b || !gr->s1_w || !gr->s1_b || !gr->rel_emb || pp->aggregator != RNNL_AGG_SUM ||
      !pp->node_w || !pp->add_w || !pp->add_b || !pp->ln_w || !pp->ln_b || !pp->s0_w || !pp->s0_b || !pp->s1_w ||
      !pp->rel_emb || head >= g->d.R || n_cand_total < 0 || !rows_scratch) {
    set_error("rnnl_predictorplus_backward: bad arguments");
    return RNNL_ERR_INVALID;
  }
  const int R = g->d.R;
  const BwdLayout B = bwd_layout(r->d.n_nodes, R);
  const Layout Ly = make_layout(nq, scale, r->d.n_nodes);
  const int64_t gy_cap = gy_chunks(nq, n_cand_total);
  if (scratch_bytes < (size_t)B.total || ws_bytes < (size_t)Ly.total ||
      rows_bytes < (size_t)gy_cap * 16 * 64 * sizeof(float)) {
    set_error("rnnl_predictorplus_backward: scratch or workspace too small");
    return RNNL_ERR_INVALID;
  }
  hipStream_t st = (hipStream_t)stream;
  unsigned char *sb = static_cast<unsigned char *>(scratch);
  unsigned long long *gnode = reinterpret_cast<unsigned long long *>(sb + B.gnode);
  double *grel = reinterpret_cast<double *>(sb + B.grel);
  float *part = reinterpret_cast<float *>(sb + B.part);
  float *npart = reinterpret_cast<float *>(sb + B.npart);
  long long *gpart = reinterpret_cast<long long *>(sb + B.gpart);
  BwStats *stats = reinterpret_cast<BwStats *>(sb + B.stats);
  float *gy = static_cast<float *>(rows_scratch);
  // the nodes whose gradient can be non-zero: the head's trie (training
  // batches are one relation), else every node
  int lo = 0, hi = r->d.n_nodes;
  if (head >= 0) {
    lo = r->head_root[head];
    hi = lo < 0 ? 0 : lo + r->head_nodes[head];
    if (lo < 0) lo = 0;
  }
  RNNL_HIP_CHECK(hipMemsetAsync(gr->emb, 0, sizeof(float) * (size_t)gr->emb_ld * (size_t)r->d.n_rules, st));
  if (hi > lo) RNNL_HIP_CHECK(hipMemsetAsync(gnode + (int64_t)lo * 16, 0, sizeof(long long) * 16 * (size_t)(hi - lo), st));
  RNNL_HIP_CHECK(hipMemsetAsync(grel, 0, sizeof(double) * 16 * (size_t)R, st));
  RNNL_HIP_CHECK(hipMemsetAsync(stats, 0, sizeof(BwStats), st));
  KParams p{};
  p.g = g->d;
  p.rl = r->d;
  p.agg = RNNL_AGG_SUM;
  p.node_w = static_cast<const unsigned char *>(pp->node_w);
  p.add_w = pp->add_w;
  p.add_b = pp->add_b;
  p.ln_w = pp->ln_w;
  p.ln_b = pp->ln_b;
  p.s0_w = pp->s0_w;
  p.s0_b = pp->s0_b;
  p.s1_w = pp->s1_w;
  p.s1_b = pp->s1_b;
  p.rel_emb = pp->rel_emb;
  p.all_r = all_r;
  p.nq = nq;
  p.n_cand = const_cast<int32_t *>(n_cand);
  p.ws = static_cast<unsigned char *>(ws);
  unsigned char *base = static_cast<unsigned char *>(ws);
  p.q_base = reinterpret_cast<int64_t *>(base + Ly.off_qbase);
  p.cand = reinterpret_cast<int4 *>(base + Ly.off_cand);
  p.bent = reinterpret_cast<int2 *>(base + Ly.off_bent);
  p.chunks = reinterpret_cast<int2 *>(base + Ly.off_chunk);
  // grid: about one chunk per wave (the chunks: <= n_cand_total / 64 + one
  // per row), at most BW_GRID workgroups
  const int64_t nchunk = n_cand_total / 64 + nq;
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(BW_GRID, (nchunk + BW_WAVES - 1) / BW_WAVES));
  const int nl = head >= 0 ? std::min(std::max(hi - lo, 0), BW_LDS_NODES) : 0;
  hipLaunchKernelGGL(sum_backward_kernel, dim3(grid), dim3(BWB), 0, st, p, grad_score, grel, part, gy, gy_cap, stats,
                     head >= 0 ? 1 : 0);
  hipLaunchKernelGGL(node_accum_kernel, dim3(grid), dim3(BWB), 0, st, p, (const float *)gy, gy_cap,
                     (const BwStats *)stats, gnode, gpart, lo, nl);
  const int64_t nthreads = (int64_t)std::max(hi - lo, 0) * 16;
  const int ngrid = (int)std::max<int64_t>(1, std::min<int64_t>(NG_GRID, (nthreads + BWB - 1) / BWB));
  hipLaunchKernelGGL(node_grad_kernel, dim3(ngrid), dim3(BWB), 0, st, r->d, lo, std::max(hi, lo),
                     (const long long *)gnode, (const long long *)gpart, grid, nl, (const BwStats *)stats, emb, ld,
                     pp->add_w, gr->emb, gr->emb_ld, npart);
  const int nwaves = PB_N + 256 + (R * 16 + 63) / 64;  // one wave per field (relation_emb: per 64 entries)
  hipLaunchKernelGGL(grad_reduce_kernel, dim3((nwaves + BW_WAVES - 1) / BW_WAVES), dim3(BWB), 0, st, part, grid,
                     npart, ngrid, grel, R, *gr);
  if (head >= 0) hipLaunchKernelGGL(rel_grad_kernel, dim3(1), dim3(64), 0, st, pp->s0_w, head, *gr);
  RNNL_HIP_CHECK(hipGetLastError());
  return RNNL_OK;
}

}  // extern "C"
