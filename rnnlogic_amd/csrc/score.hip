// PredictorPlus forward for gfx950 (MI355X), K2: rule_to_entity + score_model.
//
// After the grounding (ground.hip) every candidate of a query has a bucket of
// (trie node, path count) entries.  Its score (ref src/predictors.py:238-271):
//   rule_to_entity (layers.py:53-126): FuncToNodeSum — the exact sum of
//       count x node record (the node's rule-embedding sum times the
//       Linear(16, 16) weight, int32 fixed point with one shift per table;
//       summed in fp64, which is exact below 2^23 total count, else int64),
//       then the Linear's bias, LayerNorm, ReLU; FuncToNode (pna) — sums of x and x^2,
//       min and max per node, degree scalers, Linear(192, 16), LayerNorm, ReLU
//   score_model (layers.py:9-51): Linear(32, 128) (the relation half folded
//       into a per-relation bias), ReLU, Linear(128, 1)
// added into the base score (bias / RotatE) or written (entity_feature none).
// The unit of work is one wave x one chunk of <= 64 candidates of a query
// (the chunk list in row order, see ground.hip).
#include <hip/hip_runtime.h>

#include "fwd.h"

namespace rnnl {

// Byte offset of node n's record: 32-bit (rnnl_rules_create bounds the node
// count), so the loads take the scalar-base + 32-bit-offset form
__device__ __forceinline__ uint32_t rec_off(int n, int stride) { return (uint32_t)n * (uint32_t)stride; }

// score_model's weights as the scoring kernels keep them in LDS: layer 0's
// candidate half (128 x 16) as the A fragments of v_mfma_f32_16x16x16_f16,
// each weight split into two fp16 parts, and the last layer as floats.
struct Mlp0Lds {
  uint2 a0[8][2][64];  // [output tile][part][lane]: lane (k, i16) holds W0[16 ot + i16][4k .. 4k + 3]
  float s1w[128], s1b[4];
};

typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// ReLU as one v_med3_f32 (fmaxf(x, 0) compiles to a canonicalize + max pair);
// the same value for every non-NaN x
__device__ __forceinline__ float relu(float x) { return __builtin_amdgcn_fmed3f(x, 0.f, __builtin_huge_valf()); }

// v = hi + lo + r with hi, lo fp16 (RNE) and |r| <= 2^-22 |v| for normal
// parts (a subnormal lo part keeps an absolute error below 2^-25)
__device__ __forceinline__ void split_f16(float v, _Float16 &hi, _Float16 &lo) {
  hi = (_Float16)v;
  lo = (_Float16)(v - (float)hi);
}

__device__ __forceinline__ void load_mlp0(Mlp0Lds &m, const float *__restrict__ W) {
  for (int i = threadIdx.x; i < 128; i += blockDim.x) m.s1w[i] = W[W_S1W + i];
  if (threadIdx.x < 4) m.s1b[threadIdx.x] = threadIdx.x == 0 ? W[W_S1B] : 0.f;
  for (int i = threadIdx.x; i < 8 * 64; i += blockDim.x) {
    const int ot = i >> 6, l = i & 63, o = ot * 16 + (l & 15), k0 = (l >> 4) * 4;
    f16x4 hi, lo;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      _Float16 h, q;
      split_f16(W[W_S0X + o * 16 + k0 + j], h, q);
      hi[j] = h;
      lo[j] = q;
    }
    m.a0[ot][0][l] = __builtin_bit_cast(uint2, hi);
    m.a0[ot][1][l] = __builtin_bit_cast(uint2, lo);
  }
}

// score_model (layers.py:9-51) for the wave's 64 candidates (lane = candidate,
// x1 its FuncToNodeSum output; whole wave, dead lanes pass anything finite):
// Linear(32, 128) with the relation half folded into relb, ReLU,
// Linear(128, 1).  Layer 0 runs on the matrix cores as D = W0 . X1^T, 16
// candidates x 128 outputs per round (8 output tiles of
// v_mfma_f32_16x16x16_f16; x1 and W0 split into two fp16 parts, the three
// part products hi.hi, hi.lo, lo.hi accumulated in fp32 onto C = relb, the
// dropped lo.lo below 2^-22 of |w x|; x1 >= 0 is post-LayerNorm, so fp16's
// range holds it).  D lane (k, i16) holds outputs 4k .. 4k + 3 of candidate
// i16: ReLU and the 128 -> 1 dot stay on the VALU per lane, summed over the
// four k-lanes of a candidate by two xor shuffles.  A candidate's output
// depends on its own x1 only (its own D column), in a fixed order, so equal
// inputs give bit-identical outputs whatever the other lanes hold.  On the
// VALU this layer was 2,048 FMAs + 256 max/fma per candidate, the bulk of the
// SUM pass's VALU instructions, which take RotatE's issue slots beside it.
// stage: the wave's 16 x 16 floats; relb: the wave's 128 folded biases.
__device__ __forceinline__ void split4(const float4 v, f16x4 &hi, f16x4 &lo) {
  const float xs[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    _Float16 h, q;
    split_f16(xs[j], h, q);
    hi[j] = h;
    lo[j] = q;
  }
}

// score_model on one 16-candidate tile whose x1 is in B layout (lane (k, i16):
// hidden 4k .. 4k + 3 of candidate i16, as fp16 parts): the candidate's
// output, summed over its four k-lanes (every k-lane holds it).
__device__ __forceinline__ float mlp0_tile(const f16x4 bh, const f16x4 bl, const Mlp0Lds &w, const float *relb) {
  const int lane = threadIdx.x & 63, k = lane >> 4;
  float acc = 0.f;
#pragma unroll 1
  for (int ot = 0; ot < 8; ++ot) {
    const f16x4 ah = __builtin_bit_cast(f16x4, w.a0[ot][0][lane]);
    const f16x4 al = __builtin_bit_cast(f16x4, w.a0[ot][1][lane]);
    const float4 rb = reinterpret_cast<const float4 *>(relb)[ot * 4 + k];
    f32x4 d = {rb.x, rb.y, rb.z, rb.w};
    d = __builtin_amdgcn_mfma_f32_16x16x16f16(al, bh, d, 0, 0, 0);  // smallest products first
    d = __builtin_amdgcn_mfma_f32_16x16x16f16(ah, bl, d, 0, 0, 0);
    d = __builtin_amdgcn_mfma_f32_16x16x16f16(ah, bh, d, 0, 0, 0);
    const float4 w1 = reinterpret_cast<const float4 *>(w.s1w)[ot * 4 + k];
    acc = fmaf(relu(d[0]), w1.x, acc);
    acc = fmaf(relu(d[1]), w1.y, acc);
    acc = fmaf(relu(d[2]), w1.z, acc);
    acc = fmaf(relu(d[3]), w1.w, acc);
  }
  acc += __shfl_xor(acc, 16, 64);
  acc += __shfl_xor(acc, 32, 64);
  return acc + w.s1b[0];
}

__device__ __forceinline__ float score_mlp_f16(const float (&x1)[16], const Mlp0Lds &w, float *stage,
                                               const float *relb) {
  const int lane = threadIdx.x & 63, k = lane >> 4, i16 = lane & 15;
  float out = 0.f;
#pragma unroll 1
  for (int t = 0; t < 4; ++t) {
    if (k == t) {
      float4 *dst = reinterpret_cast<float4 *>(stage + i16 * 16);
#pragma unroll
      for (int j = 0; j < 4; ++j) dst[j] = make_float4(x1[4 * j], x1[4 * j + 1], x1[4 * j + 2], x1[4 * j + 3]);
    }
    wave_lds_sync();
    const float4 xv = reinterpret_cast<const float4 *>(stage)[i16 * 4 + k];  // candidate 16 t + i16, K 4k..4k+3
    wave_lds_sync();  // the next round rewrites the stage
    f16x4 bh, bl;
    split4(xv, bh, bl);
    const float o = mlp0_tile(bh, bl, w, relb);
    if (k == t) out = o;  // lane 16 t + i16 is candidate i16 of this round
  }
  return out;
}

// relation half of score_model.layers.0 folded into a per-relation bias (128 lanes)
__device__ __forceinline__ float relation_bias(const KParams &p, int r, int o) {
  float acc = p.s0_b[o];
  for (int i = 0; i < 16; ++i) acc = fmaf(p.s0_w[o * 32 + 16 + i], p.rel_emb[r * 16 + i], acc);
  return acc;
}

// ---------------------------------------------------------------- PNA scoring over chunks
// FuncToNode (pna, layers.py:79-126) + score_model for one wave x one chunk of
// <= 64 consecutive candidates of one query, p.chunks[0 .. hdr[H_CHUNKS]).
// Waves dequeue chunks independently, so a query with 17k candidates (WN18RR)
// is spread over ~280 waves instead of holding one workgroup while the rest
// of the grid drains; no workgroup barrier per query.
//
// Per 16-candidate tile, one walk over each candidate's bucket entries (four
// lanes per candidate, below) gives the 64 features [mean, min, max, std]
// (16 dims each); the degree scalers {1, s, 1/s} make 192 inputs of
// add_model, Linear(192, 16).  That layer runs on the matrix cores as
// D1 = W . U^T for the tile: U[c][(f, s3)] = feature f x scaler s3, the
// features split into two fp16 parts (means, minima, maxima and standard
// deviations of rule embeddings: bounded), W (16 x 192) the A fragments per
// (feature block, scaler), three part products per 16-wide K step; the
// scalers are per candidate, so they factor out of the Linear (D_s
// accumulates W_s . x and the output is D_1 + s D_s + D_{1/s} / s: one split
// per feature block instead of one per (block, scaler)).  D1's lane (k, i16)
// holds outputs 4k .. 4k + 3 of candidate i16, so LayerNorm's mean and
// variance are two xor shuffles away, and after ReLU the lane holds exactly
// score_model's B fragment (hidden 4k .. 4k + 3 of candidate i16): mlp0_tile
// runs on it with no second staging.  On the VALU the Linear was 3,072 FMAs
// per candidate, most of the pass's VALU instructions — which take RotatE's
// issue slots beside it.

// LDS image of the PNA weights: add_model as A fragments per (feature block
// b, scaler s3): lane (k, i16) holds W[i16][(16 b + 4k + j) 3 + s3], j < 4;
// its bias, LayerNorm and score_model (Mlp0Lds).
struct PnaLds {
  uint2 aa[4][3][2][64];  // [block][scaler][part][lane]
  float addb[16], lnw[16], lnb[16], pad[16];
  Mlp0Lds m;
};

__device__ __forceinline__ void load_pna_weights(PnaLds &w, const float *__restrict__ W) {
  for (int i = threadIdx.x; i < 4 * 3 * 64; i += blockDim.x) {
    const int b = i / 192, s3 = (i / 64) % 3, l = i & 63, o = l & 15, k0 = (l >> 4) * 4;
    f16x4 hi, lo;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      _Float16 h, q;
      split_f16(W[W_ADDW + o * 192 + (b * 16 + k0 + j) * 3 + s3], h, q);
      hi[j] = h;
      lo[j] = q;
    }
    w.aa[b][s3][0][l] = __builtin_bit_cast(uint2, hi);
    w.aa[b][s3][1][l] = __builtin_bit_cast(uint2, lo);
  }
  if (threadIdx.x < 16) {
    w.addb[threadIdx.x] = W[W_ADDB + threadIdx.x];
    w.lnw[threadIdx.x] = W[W_LNW + threadIdx.x];
    w.lnb[threadIdx.x] = W[W_LNB + threadIdx.x];
  }
  load_mlp0(w.m, W);
}

// ---- lane = (candidate, dim quad) walks
// The features are walked with four lanes per candidate: a round takes the 16
// candidates of a tile (lane 4 c + dq: candidate c, dims 4 dq .. 4 dq + 3,
// 16-byte record loads), each lane accumulating its dims' sums and sums of
// squares (exact fp64, int64 past a total count of 2^23), minima and maxima
// over the candidate's entries in ONE walk.  A per-candidate lane walk
// carries 16 dims x 4 statistics in registers (233 VGPRs + AGPRs: two waves
// per SIMD, holding RotatE to three beside it) and its wave waits for the
// longest of 64 lists, twice; here a round waits for the longest of 16, a
// lane holds 4 dims, and the features go straight into the tile's LDS stage
// for add_model's MFMA steps (WN18RR ground + PNA alone 5.05-5.2 -> 4.73-4.8
// ms).  Every sum is exact and min / max are order-free: the walk order does
// not change a feature.
struct PnaAcc {
  double s[4], q[4];  // sum of count x record (sums half, squares half), this lane's dims
  float mn[4], mx[4];
  uint64_t csum;      // count total
  long long deg;      // degree term: sum of count x rules at the node
  uint64_t fp;        // digest fingerprint term
};

__device__ __forceinline__ void pna_acc_init(PnaAcc &A) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    A.s[j] = 0;
    A.q[j] = 0;
    A.mn[j] = __builtin_huge_valf();
    A.mx[j] = -__builtin_huge_valf();
  }
  A.csum = 0;
  A.deg = 0;
  A.fp = 0;
}

// entries e0, e0 + step, ... < e1, dims 4 dq .. 4 dq + 3, into A
__device__ __forceinline__ void pna_lane_walk(const KParams &p, int e0, int e1, int step, int dq, bool want_fp,
                                              PnaAcc &A) {
  int2 nx = e0 < e1 ? p.bent[e0] : make_int2(0, 0);
#pragma unroll 1
  for (int e = e0; e < e1; e += step) {
    const int2 be = nx;
    if (e + step < e1) nx = p.bent[e + step];
    const uint32_t c = (uint32_t)be.y;
    A.csum += c;
    A.deg += (long long)c * p.rl.node_nrules[be.x];
    if (want_fp) A.fp += (uint64_t)c * p.rl.node_fp[be.x];
    const int4 *rec = reinterpret_cast<const int4 *>(p.node_w + rec_off(be.x, kStridePna));
    const int4 rs = rec[dq], rq = rec[4 + dq];
    const float4 fmn = reinterpret_cast<const float4 *>(rec)[8 + dq], fmx = reinterpret_cast<const float4 *>(rec)[12 + dq];
    const int xs[4] = {rs.x, rs.y, rs.z, rs.w}, xq[4] = {rq.x, rq.y, rq.z, rq.w};
    const float vn[4] = {fmn.x, fmn.y, fmn.z, fmn.w}, vx[4] = {fmx.x, fmx.y, fmx.z, fmx.w};
    const double cd = (double)c;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      A.s[j] = fma(cd, (double)xs[j], A.s[j]);
      A.q[j] = fma(cd, (double)xq[j], A.q[j]);
      A.mn[j] = __builtin_amdgcn_fmed3f(A.mn[j], vn[j], -__builtin_huge_valf());
      A.mx[j] = __builtin_amdgcn_fmed3f(A.mx[j], vx[j], __builtin_huge_valf());
    }
  }
}

// the same entries' int64 sums (totals past the exact fp64 range)
__device__ __forceinline__ void pna_lane_exact(const KParams &p, int e0, int e1, int step, int dq, long long (&s)[4],
                                               long long (&q)[4]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) s[j] = q[j] = 0;
#pragma unroll 1
  for (int e = e0; e < e1; e += step) {
    const int2 be = p.bent[e];
    const long long c = (uint32_t)be.y;
    const int *rec = reinterpret_cast<const int *>(p.node_w + rec_off(be.x, kStridePna));
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      s[j] += c * rec[4 * dq + j];
      q[j] += c * rec[16 + 4 * dq + j];
    }
  }
}

// The four features of dims 4 dq .. 4 dq + 3 of tile candidate c16 into the
// stage (block b: stage[(16 b + c16) 16 + dim], one 16-byte store each); lane
// dq == 0 also writes the scalers and the digest term.  inv0 / inv1: the
// sums' / squares' fixed-point scales.  mean = sum / degree and
// std = sqrt(max(sum x^2 / degree - mean^2, 1e-6)) in the reference's
// separately rounded fp32 operations (layers.py:103-110).
__device__ __forceinline__ void pna_features_out(const KParams &p, const PnaAcc &A, int dq, int c16, bool live,
                                                 int q, int ent, double inv0, double inv1, float *stage, float2 *sc) {
  const float degf = (float)(A.deg + 1);
  const float idcl = 1.0f / fmaxf(degf, 1e-6f);
  float mean[4], sd[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float sum = (float)(A.s[j] * inv0), sq = (float)(A.q[j] * inv1);
    mean[j] = __fmul_rn(sum, idcl);
    sd[j] = sqrtf(fmaxf(__fsub_rn(__fmul_rn(sq, idcl), __fmul_rn(mean[j], mean[j])), 1e-6f));
  }
  float4 *st = reinterpret_cast<float4 *>(stage);
  st[(0 * 16 + c16) * 4 + dq] = make_float4(mean[0], mean[1], mean[2], mean[3]);
  st[(1 * 16 + c16) * 4 + dq] = live ? make_float4(A.mn[0], A.mn[1], A.mn[2], A.mn[3]) : make_float4(0.f, 0.f, 0.f, 0.f);
  st[(2 * 16 + c16) * 4 + dq] = live ? make_float4(A.mx[0], A.mx[1], A.mx[2], A.mx[3]) : make_float4(0.f, 0.f, 0.f, 0.f);
  st[(3 * 16 + c16) * 4 + dq] = make_float4(sd[0], sd[1], sd[2], sd[3]);
  if (dq == 0) {
    // degree scalers (layers.py:92, 103-116): degree = sum of A_fn + 1
    const float sc1 = live ? logf(degf) / fmaxf(p.q_scale[q], 1e-6f) : 1.0f;
    sc[c16] = make_float2(sc1, 1.0f / fmaxf(sc1, 1e-6f));
    if (live) {
      if (p.digest)
        atomicAdd(reinterpret_cast<unsigned long long *>(p.digest + q),
                  (unsigned long long)mix64((uint64_t)ent ^ mix64((uint64_t)A.deg ^ mix64(A.fp))));
      if (A.csum >> 33) flag_acc_range(p);  // |int32 record| < 2^30: int64 sums exact below 2^33
    }
  }
}

// Lists longer than this are walked by the whole wave (16 entry slots x 4
// dim quads, then a reduction over the slots) instead of the candidate's
// four lanes.
constexpr int PNA_BIG = 16;

__global__ __launch_bounds__(BS, 4) void score_pna_chunk_kernel(KParams p, const float *__restrict__ W) {
  __shared__ PnaLds s_w;
  __shared__ __attribute__((aligned(16))) float s_relb[BS / 64][128];
  __shared__ __attribute__((aligned(16))) float s_stage[BS / 64][4 * 16 * 16];  // a tile's 16 x 64 features
  __shared__ float2 s_sc[BS / 64][16];                                         // their scalers (s, 1 / s)
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, k = lane >> 4, i16 = lane & 15;
  const int c4 = lane >> 2, dq = lane & 3;  // the walks' lane roles: candidate of the tile, dim quad
  unsigned int *hdr = reinterpret_cast<unsigned int *>(p.ws);
  const unsigned int *trailer = reinterpret_cast<const unsigned int *>(p.node_w + (int64_t)p.rl.n_nodes * kStridePna);
  check_node_table(p, trailer);
  load_pna_weights(s_w, W);
  __syncthreads();  // the only workgroup barrier: waves run independently from here
  const double inv0 = ldexp(1.0, -(int)trailer[1]), inv1 = ldexp(1.0, -(int)trailer[4]);
  const bool want_fp = p.digest != nullptr;
  const long long nchunks = (long long)*reinterpret_cast<const unsigned long long *>(hdr + H_CHUNKS);
  float *relb = s_relb[wv], *stage = s_stage[wv];
  float2 *sc = s_sc[wv];
  int cur_r = -1;
  unsigned c = 0, cend = 0;  // wave-uniform: the dequeued chunk range
#pragma unroll 1
  for (;; ++c) {
    if (c == cend) next_chunks(&hdr[H_DEQUEUE2], nchunks, 1, c, cend);
    if ((long long)c >= nchunks) break;
    const int2 ck = p.chunks[c];
    const int q = __builtin_amdgcn_readfirstlane(ck.x);
    const int s0 = __builtin_amdgcn_readfirstlane(ck.y);
    const int r = __builtin_amdgcn_readfirstlane((int)p.all_r[q]);
    if (r != cur_r) {
      wave_lds_sync();  // the previous chunk's reads of the slice are done
      relb[lane] = relation_bias(p, r, lane);
      relb[lane + 64] = relation_bias(p, r, lane + 64);
      wave_lds_sync();
      cur_r = r;
    }
    const int nc = __builtin_amdgcn_readfirstlane(p.n_cand[q]);
    const int64_t qb = p.q_base[q];
    // lane = candidate s0 + lane for the loads and the final store; lanes past
    // the chunk's candidates carry zero features and store nothing
    const int s = s0 + lane;
    const bool live = s < nc;
    int4 cr = make_int4(0, 0, 0, 0);
    if (live) cr = p.cand[qb + s];
    float out = 0.f;
#pragma unroll 1
    for (int t = 0; t < 4 && s0 + 16 * t < nc; ++t) {
      // the tile's long lists: the whole wave, entry slot c4, dim quad dq
      uint64_t big = __ballot(live && cr.z > PNA_BIG && (lane >> 4) == t);
#pragma unroll 1
      while (big) {
        const int owner = __builtin_ctzll(big);
        big &= big - 1;
        const int beg = __builtin_amdgcn_readlane(cr.y, owner), cnt = __builtin_amdgcn_readlane(cr.z, owner);
        PnaAcc A;
        pna_acc_init(A);
        pna_lane_walk(p, beg + c4, beg + cnt, 16, dq, want_fp, A);
#pragma unroll
        for (int off = 4; off < 64; off <<= 1) {
          A.csum += __shfl_xor(A.csum, off, 64);
          A.deg += __shfl_xor(A.deg, off, 64);
          A.fp += __shfl_xor(A.fp, off, 64);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            A.mn[j] = __builtin_amdgcn_fmed3f(A.mn[j], __shfl_xor(A.mn[j], off, 64), -__builtin_huge_valf());
            A.mx[j] = __builtin_amdgcn_fmed3f(A.mx[j], __shfl_xor(A.mx[j], off, 64), __builtin_huge_valf());
          }
        }
        if (A.csum >> 23) {  // wave-uniform: the slots' exact int64 sums
          long long es[4], eq[4];
          pna_lane_exact(p, beg + c4, beg + cnt, 16, dq, es, eq);
#pragma unroll
          for (int off = 4; off < 64; off <<= 1)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              es[j] += __shfl_xor(es[j], off, 64);
              eq[j] += __shfl_xor(eq[j], off, 64);
            }
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            A.s[j] = (double)es[j];
            A.q[j] = (double)eq[j];
          }
        } else {  // exact integers in fp64: any order
#pragma unroll
          for (int off = 4; off < 64; off <<= 1)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              A.s[j] += __shfl_xor(A.s[j], off, 64);
              A.q[j] += __shfl_xor(A.q[j], off, 64);
            }
        }
        if (c4 == 0)
          pna_features_out(p, A, dq, owner - 16 * t, true, q, __builtin_amdgcn_readlane(cr.x, owner), inv0, inv1,
                           stage, sc);
      }
      // the other 16: candidate 16 t + c4 on lanes 4 c4 .. 4 c4 + 3
      {
        const int src = 16 * t + c4;
        const int beg = __shfl(cr.y, src, 64), cnt = __shfl(cr.z, src, 64), ent = __shfl(cr.x, src, 64);
        const bool liv = s0 + src < nc;
        if (!(liv && cnt > PNA_BIG)) {  // (long lists: written by the wave walk above)
          const int n = liv ? cnt : 0;
          PnaAcc A;
          pna_acc_init(A);
          pna_lane_walk(p, beg, beg + n, 1, dq, want_fp, A);
          if (A.csum >> 23) {
            long long es[4], eq[4];
            pna_lane_exact(p, beg, beg + n, 1, dq, es, eq);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              A.s[j] = (double)es[j];
              A.q[j] = (double)eq[j];
            }
          }
          pna_features_out(p, A, dq, c4, liv, q, ent, inv0, inv1, stage, sc);
        }
      }
      wave_lds_sync();
      // add_model on the matrix cores: per feature block one fp16 split, per
      // scaler one 16-wide K step (three part products)
      f32x4 D[3];
      {
        const float4 ab = reinterpret_cast<const float4 *>(s_w.addb)[k];
        D[0] = (f32x4){ab.x, ab.y, ab.z, ab.w};
        D[1] = (f32x4){0.f, 0.f, 0.f, 0.f};
        D[2] = (f32x4){0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const float4 x = reinterpret_cast<const float4 *>(stage)[(b * 16 + i16) * 4 + k];
        f16x4 bh, bl;
        split4(x, bh, bl);
#pragma unroll
        for (int s3 = 0; s3 < 3; ++s3) {
          const f16x4 ah = __builtin_bit_cast(f16x4, s_w.aa[b][s3][0][lane]);
          const f16x4 al = __builtin_bit_cast(f16x4, s_w.aa[b][s3][1][lane]);
          D[s3] = __builtin_amdgcn_mfma_f32_16x16x16f16(al, bh, D[s3], 0, 0, 0);
          D[s3] = __builtin_amdgcn_mfma_f32_16x16x16f16(ah, bl, D[s3], 0, 0, 0);
          D[s3] = __builtin_amdgcn_mfma_f32_16x16x16f16(ah, bh, D[s3], 0, 0, 0);
        }
      }
      // LayerNorm over each candidate's 16 outputs (four k-lanes), ReLU, score_model
      const float2 scl = sc[i16];
      wave_lds_sync();  // the next tile rewrites the stage and the scalers
      f32x4 o4;
#pragma unroll
      for (int j = 0; j < 4; ++j) o4[j] = fmaf(scl.y, D[2][j], fmaf(scl.x, D[1][j], D[0][j]));
      float s4 = (o4[0] + o4[1]) + (o4[2] + o4[3]);
      s4 += __shfl_xor(s4, 16, 64);
      s4 += __shfl_xor(s4, 32, 64);
      const float mu = s4 / 16.0f;
      float z[4], v4 = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        z[j] = o4[j] - mu;
        v4 = fmaf(z[j], z[j], v4);
      }
      v4 += __shfl_xor(v4, 16, 64);
      v4 += __shfl_xor(v4, 32, 64);
      const float rstd = 1.0f / sqrtf(v4 / 16.0f + 1e-5f);
      const float4 lw = reinterpret_cast<const float4 *>(s_w.lnw)[k];
      const float4 lb = reinterpret_cast<const float4 *>(s_w.lnb)[k];
      const float4 x1 = make_float4(relu(z[0] * rstd * lw.x + lb.x), relu(z[1] * rstd * lw.y + lb.y),
                                    relu(z[2] * rstd * lw.z + lb.z), relu(z[3] * rstd * lw.w + lb.w));
      f16x4 bh, bl;
      split4(x1, bh, bl);
      const float o = mlp0_tile(bh, bl, s_w.m, relb);
      if (k == t) out = o;  // lane 16 t + i16 is candidate i16 of tile t
    }
    if (!live) continue;
    const int te = cr.x;
    const int64_t idx = (int64_t)q * p.g.E + te;
    if (p.atomic_out) {  // deferred beside RotatE: added into the zeroed row (see sum_write_out)
      unsafeAtomicAdd(p.score + idx, out);
      continue;
    }
    if (p.feature == RNNL_FEATURE_NONE)
      p.score[idx] = out;
    else
      p.score[idx] = out + (p.base_row ? p.base_row[te] : p.score[idx]);
    if (p.mask) p.mask[idx] = 1;
  }
}

// ---------------------------------------------------------------- SUM aggregator (FuncToNodeSum)
// A candidate's feature is the exact sum over its bucket entries (trie node
// n, path count c) of c x record[n], the record being the int32 fixed-point
// sum of the rule embeddings ending at n (one shift for the table, every
// value < 2^30).  The sums are accumulated in fp64: below a total count of
// 2^23 every product and partial sum is an integer under 2^53, so the fp64
// sum IS the int64 sum (one v_cvt_f64_i32 + one v_fma_f64 per element instead
// of two 64-bit integer multiply-adds and their fix-ups) and does not depend
// on the entry order; past it the int64 walk below.

// The exact int64 walk (counts past the fp64 range; also the digest's
// degree / fingerprint terms).
template <bool DIGEST>
__device__ __forceinline__ void gather_sum_int64(const KParams &p, int beg, int cnt, float inv_scale, float f[16],
                                              long long &deg, uint64_t &fp) {
  long long acc[16];
#pragma unroll
  for (int d = 0; d < 16; ++d) acc[d] = 0;
  deg = 0;
  fp = 0;
  uint64_t csum = 0;
  for (int e = beg; e < beg + cnt; ++e) {
    const int2 be = p.bent[e];
    const int n = be.x;
    const uint32_t cu = (uint32_t)be.y;
    const long long c = cu;
    csum += cu;
    const int *x = reinterpret_cast<const int *>(p.node_w + rec_off(n, kStrideSum));
#pragma unroll
    for (int d = 0; d < 16; ++d) acc[d] += c * x[d];
    if constexpr (DIGEST) {
      deg += c * p.rl.node_nrules[n];
      fp += (uint64_t)c * p.rl.node_fp[n];
    }
  }
  if (csum >> 33) flag_acc_range(p);  // |int32 record| < 2^30: int64 sums exact below 2^33 total count
#pragma unroll
  for (int d = 0; d < 16; ++d) f[d] = (float)((double)acc[d] * (double)inv_scale);
}

template <bool DIGEST>
__device__ __forceinline__ void gather_sum(const KParams &p, int beg, int cnt, float inv_scale, float f[16],
                                           long long &deg, uint64_t &fp) {
  double accd[16];
#pragma unroll
  for (int d = 0; d < 16; ++d) accd[d] = 0.0;
  deg = 0;
  fp = 0;
  uint64_t csum = 0;
  // the next entry's (node, count) loaded beside this entry's record: one
  // dependent load per entry on the walk's critical path instead of two
  // (FB15k-237 bias step 9.47 -> 9.24 ms)
  int2 nx = cnt > 0 ? p.bent[beg] : make_int2(0, 0);
  for (int e = beg; e < beg + cnt; ++e) {
    const int2 be = nx;
    if (e + 1 < beg + cnt) nx = p.bent[e + 1];
    const int n = be.x;
    const uint32_t cu = (uint32_t)be.y;
    csum += cu;
    const int *x = reinterpret_cast<const int *>(p.node_w + rec_off(n, kStrideSum));
    const double cd = (double)cu;
#pragma unroll
    for (int d = 0; d < 16; ++d) accd[d] = fma(cd, (double)x[d], accd[d]);
    if constexpr (DIGEST) {
      deg += (long long)cu * p.rl.node_nrules[n];
      fp += (uint64_t)cu * p.rl.node_fp[n];
    }
  }
  if (csum >= (1ull << 23)) {  // rare: the exact int64 walk
    gather_sum_int64<DIGEST>(p, beg, cnt, inv_scale, f, deg, fp);
    return;
  }
#pragma unroll
  for (int d = 0; d < 16; ++d) f[d] = (float)(accd[d] * (double)inv_scale);
}

// LDS image of the SUM scoring weights: FuncToNodeSum's Linear bias and
// LayerNorm as floats (VALU) and score_model (Mlp0Lds).
struct SumLds {
  float addb[16], lnw[16], lnb[16];
  Mlp0Lds m;
};

__device__ __forceinline__ void load_sum_weights(SumLds &w, const float *__restrict__ W) {
  if (threadIdx.x < 16) {
    w.addb[threadIdx.x] = W[W_ADDB + threadIdx.x];
    w.lnw[threadIdx.x] = W[W_LNW + threadIdx.x];
    w.lnb[threadIdx.x] = W[W_LNB + threadIdx.x];
  }
  load_mlp0(w.m, W);
}

// FuncToNodeSum tail: x1 = ReLU(LayerNorm(Linear(16, 16)(f)))   (layers.py:53-77);
// the node records carry the Linear's weight already (node_weights_kernel), so
// f is W . (sum of count x node sum) and only the bias is added here
__device__ __forceinline__ void sum_hidden(const SumLds &w, const float f[16], float (&x1)[16]) {
#pragma unroll
  for (int o = 0; o < 16; ++o) x1[o] = f[o] + w.addb[o];
  float mu = 0.f;
#pragma unroll
  for (int d = 0; d < 16; ++d) mu += x1[d];
  mu = mu / 16.0f;
  float var = 0.f;
#pragma unroll
  for (int d = 0; d < 16; ++d) {
    const float z = x1[d] - mu;
    var = fmaf(z, z, var);
  }
  var = var / 16.0f;
  const float rstd = 1.0f / sqrtf(var + 1e-5f);
#pragma unroll
  for (int d = 0; d < 16; ++d) x1[d] = relu((x1[d] - mu) * rstd * w.lnw[d] + w.lnb[d]);
}


// ---------------------------------------------------------------- single-path memo
// 38 % of the FB15k-237 test candidates are reached by exactly one path of
// one rule-end node n (one bucket entry of count 1).  Their feature is n's
// record itself, so their score_model output depends on (head relation, n)
// only: memo_sum_kernel computes it once per launch for every leaf node of
// every head (131,883 MLPs instead of ~22 M), with the full path's own
// arithmetic (the single entry's gather, then sum_hidden and score_mlp_f16).
// Launches with at most this many rows skip it (pair-memo keys instead).
constexpr int MEMO_SCAN_ROWS = 2048;

// One workgroup per head relation with rules: memo[n] for its leaf nodes
// (whole waves: score_model runs on the matrix cores, score_mlp_f16).
__global__ __launch_bounds__(BS) void memo_sum_kernel(KParams p, const float *__restrict__ W) {
  __shared__ SumLds s_w;
  __shared__ __attribute__((aligned(16))) float s_relb[128];
  __shared__ __attribute__((aligned(16))) float s_stage[BS / 64][256];
  const int r = blockIdx.x;
  const int lp = p.rl.head_leaf_ptr[r], nl = p.rl.head_leaf_ptr[r + 1] - lp;
  if (nl <= 0) return;  // uniform
  load_sum_weights(s_w, W);
  if (threadIdx.x < 128) s_relb[threadIdx.x] = relation_bias(p, r, threadIdx.x);
  __syncthreads();
  const int shift = (int)reinterpret_cast<const unsigned int *>(p.node_w + (int64_t)p.rl.n_nodes * kStrideSum)[1];
  const float inv_scale = ldexpf(1.f, -shift);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int b0 = wv * 64; b0 < nl; b0 += BS) {  // wave-uniform
    const int i = b0 + lane;
    const int n = i < nl ? p.rl.head_leaf_node[lp + i] : -1;
    float f[16];
#pragma unroll
    for (int d = 0; d < 16; ++d) f[d] = 0.f;
    if (n >= 0) {
      const int *x = reinterpret_cast<const int *>(p.node_w + rec_off(n, kStrideSum));
#pragma unroll
      for (int d = 0; d < 16; ++d) f[d] = (float)((double)x[d] * (double)inv_scale);  // gather_sum of (n, 1)
    }
    float x1[16];
    sum_hidden(s_w, f, x1);
    const float out = score_mlp_f16(x1, s_w.m, s_stage[wv], s_relb);
    if (n >= 0) p.memo[n] = out;
  }
}

__device__ __forceinline__ void sum_write_out(const KParams &p, int q, int t, float out, float base) {
  const int64_t idx = (int64_t)q * p.g.E + t;
  if (p.atomic_out) {
    // deferred beside RotatE: the row starts at zero and RotatE adds its score
    // atomically too — two addends on an exact zero give fl(base + out) in
    // either order, the one-stream path's bit for bit
    unsafeAtomicAdd(p.score + idx, out);
    return;
  }
  p.score[idx] = p.feature == RNNL_FEATURE_NONE ? out : out + base;
  if (p.mask) p.mask[idx] = 1;
}

__device__ __forceinline__ float sum_base(const KParams &p, int q, int t) {
  if (p.feature == RNNL_FEATURE_NONE || p.atomic_out) return 0.f;
  return p.base_row ? p.base_row[t] : p.score[(int64_t)q * p.g.E + t];
}

// ---------------------------------------------------------------- pair memo
// A candidate's feature is the exact sum of count x record over its bucket
// entries, so candidates whose entries are equal get bit-identical
// score_model outputs.  On an FB15k-237 test sample 57 % of the candidates
// past the single-path memo hold one or two entries and 19 % three, and
// within a 32-row relation batch only 7 % / 27 % of those entry lists are
// distinct.  The key packs (relation, each entry's node offset and count, in
// canonical order) exactly into K = 31 + psbits bits and is mixed by a
// bijection of [0, 2^K): the low psbits bits pick the slot, the high 31 bits
// are the tag, so (slot, tag) identifies the entries exactly.  A slot is one
// 8-B word (tag + 1) << 32 | output bits, written and read whole: any word a
// lane reads is some key's true output, and a lost or overwritten insert
// only costs a recomputation.
constexpr unsigned long long PAIR_NOKEY = ~0ull;

__device__ __forceinline__ void entry_cswap(unsigned &oa, unsigned &ca, unsigned &ob, unsigned &cb) {
  if (ob < oa || (ob == oa && cb < ca)) {
    const unsigned to = oa, tc = ca;
    oa = ob;
    ca = cb;
    ob = to;
    cb = tc;
  }
}

// z = 1..3 bucket entries (absent ones (0, 0): a node offset is never 0, the
// root ends no rule).  Format bit 0: one or two entries, pbc-bit counts; 1:
// three entries, pbc3-bit counts.
__device__ __forceinline__ unsigned long long pair_key(const KParams &p, int r, int root, int z, int2 b0, int2 b1,
                                                       int2 b2) {
  unsigned o0 = (unsigned)(b0.x - root), c0 = (unsigned)b0.y;
  unsigned o1 = z >= 2 ? (unsigned)(b1.x - root) : 0u, c1 = z >= 2 ? (unsigned)b1.y : 0u;
  unsigned o2 = z >= 3 ? (unsigned)(b2.x - root) : 0u, c2 = z >= 3 ? (unsigned)b2.y : 0u;
  if (z >= 2) entry_cswap(o0, c0, o1, c1);  // canonical order
  if (z == 3) {
    entry_cswap(o1, c1, o2, c2);
    entry_cswap(o0, c0, o1, c1);
  }
  const int bc = z == 3 ? p.pbc3 : p.pbc;
  if (bc <= 0 || ((c0 | c1 | c2) >> bc)) return PAIR_NOKEY;  // a count past the key's field
  unsigned long long k = z == 3 ? 1ull : 0ull;
  int sh = 1;
  k |= (unsigned long long)r << sh;
  sh += p.pbr;
  k |= (unsigned long long)o0 << sh;
  sh += p.pbo;
  k |= (unsigned long long)o1 << sh;
  sh += p.pbo;
  if (z == 3) {
    k |= (unsigned long long)o2 << sh;
    sh += p.pbo;
  }
  k |= (unsigned long long)c0 << sh;
  sh += bc;
  k |= (unsigned long long)c1 << sh;
  sh += bc;
  if (z == 3) k |= (unsigned long long)c2 << sh;
  const int K = 31 + p.psbits;
  const unsigned long long mk = (1ull << K) - 1ull;
  k = (k * 0x9E3779B97F4A7C15ull) & mk;  // odd multiplier mod 2^K, xor-shifts: a bijection of [0, 2^K)
  k ^= k >> (K / 2);
  k = (k * 0xBF58476D1CE4E5B9ull) & mk;
  k ^= k >> (K / 2 + 1);
  return k;
}

__device__ __forceinline__ bool pair_lookup(const KParams &p, unsigned long long m, float &out) {
  const unsigned long long w = p.ptab[m & ((1ull << p.psbits) - 1ull)];
  out = __uint_as_float((unsigned)w);
  return (unsigned)(w >> 32) == (unsigned)(m >> p.psbits) + 1u;
}

__device__ __forceinline__ void pair_insert(const KParams &p, unsigned long long m, float out) {
  p.ptab[m & ((1ull << p.psbits) - 1ull)] =
      ((unsigned long long)((unsigned)(m >> p.psbits) + 1u) << 32) | (unsigned long long)__float_as_uint(out);
}

// ---------------------------------------------------------------- SUM scoring over chunks
// One wave x one 64-candidate chunk of one query at a time (p.chunks, in row
// order), no workgroup barrier after the weight load.  Single-path
// candidates take the memo and candidates whose entries are in the pair memo
// take it (three loads and the store); the others are compacted (ballot +
// prefix) into the wave's LDS queue of (query, pool index) and scored 64 at a
// time by the full gather + MLP, so the MLP runs on full waves; the queue is
// flushed early only when the next chunk's relation differs (the folded
// relation bias is per wave) and at the end.
//
// A candidate with more than BIG_ENTRIES bucket entries is gathered by the
// whole wave (COOP builds; lane i takes entries i, i + 64, ...; a
// butterfly sums the 16 fp64 partials): its lane would otherwise walk the
// list alone, two dependent loads per entry, while the wave waits — on a
// one-batch launch the scoring time is the longest such walk.  The fp64 sums
// of exact count x record products are exact in any order, so the feature is
// the per-lane walk's bit for bit.  Up to BIG_SLOTS per round, their features
// staged in LDS.  A lane-per-candidate walk costs the wave its longest list:
// on the FB15k-237 split the chunks' longest lists sum to 9.5x the entries /
// 64 (tools/entry_stats.py); past 24 entries the whole wave takes the list.
#ifndef RNNL_BIG_ENTRIES
#define RNNL_BIG_ENTRIES 24
#endif
constexpr int BIG_ENTRIES = RNNL_BIG_ENTRIES;
constexpr int BIG_SLOTS = 16;
static_assert(BIG_SLOTS * 16 <= 256, "the long-list features share a wave's 256-float score_model stage");

template <bool DIGEST>
__device__ __forceinline__ void coop_gather(const KParams &p, int beg, int cnt, float inv_scale, float *fslot,
                                            uint64_t &csum, long long &deg, uint64_t &fp) {
  const int lane = threadIdx.x & 63;
  double acc[16];
#pragma unroll
  for (int d = 0; d < 16; ++d) acc[d] = 0.0;
  csum = 0;
  deg = 0;
  fp = 0;
  for (int e = beg + lane; e < beg + cnt; e += 64) {
    const int2 be = p.bent[e];
    const int n = be.x;
    const uint32_t cu = (uint32_t)be.y;
    csum += cu;
    const int *x = reinterpret_cast<const int *>(p.node_w + rec_off(n, kStrideSum));
    const double cd = (double)cu;
#pragma unroll
    for (int d = 0; d < 16; ++d) acc[d] = fma(cd, (double)x[d], acc[d]);
    if constexpr (DIGEST) {
      deg += (long long)cu * p.rl.node_nrules[n];
      fp += (uint64_t)cu * p.rl.node_fp[n];
    }
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
#pragma unroll
    for (int d = 0; d < 16; ++d) acc[d] += __shfl_xor(acc[d], off, 64);
    csum += __shfl_xor(csum, off, 64);
    if constexpr (DIGEST) {
      deg += __shfl_xor(deg, off, 64);
      fp += __shfl_xor(fp, off, 64);
    }
  }
  float v = 0.f;
#pragma unroll
  for (int d = 0; d < 16; ++d)
    if (lane == d) v = (float)(acc[d] * (double)inv_scale);
  if (lane < 16) fslot[lane] = v;
}

// Score m <= 64 queued candidates of relation r (lane i: queue[i]); the
// whole wave calls it (score_model on the matrix cores needs every lane).
// COOP = false (the 8-waves/SIMD builds): each lane walks its own list — the
// cooperative rounds' registers spill at the 64-VGPR cap.
template <bool DIGEST>
__device__ __forceinline__ void sum_score_lane(const KParams &p, const SumLds &w, const float *relb, float *stage,
                                               bool live, const int2 it, const int4 cr, const float (&f)[16],
                                               long long deg, uint64_t fp, float base, int r, int root) {
  if constexpr (DIGEST)
    if (live)
      atomicAdd(reinterpret_cast<unsigned long long *>(p.digest + it.x),
                (unsigned long long)mix64((uint64_t)cr.x ^ mix64((uint64_t)deg ^ mix64(fp))));
  asm volatile("" ::: "memory");  // keep the LDS weight reads inside (hoisted they pin ~200 VGPRs)
  float x1[16];
  sum_hidden(w, f, x1);
  const float out = score_mlp_f16(x1, w.m, stage, relb);
  if (!live) return;
  sum_write_out(p, it.x, cr.x, out, base);
  if (!DIGEST && p.ptab && cr.z <= 3) {
    const int2 z0 = make_int2(0, 0);
    const unsigned long long key = pair_key(p, r, root, cr.z, p.bent[cr.y], cr.z >= 2 ? p.bent[cr.y + 1] : z0,
                                            cr.z >= 3 ? p.bent[cr.y + 2] : z0);
    if (key != PAIR_NOKEY) pair_insert(p, key, out);
  }
}

template <bool DIGEST, bool COOP>
__device__ __forceinline__ void sum_chunk_flush(const KParams &p, const SumLds &w, const float *relb, float *stage,
                                                const int2 *queue, int m, float inv_scale, int r, int root,
                                                float *fbig) {
  const int lane = threadIdx.x & 63;
  if constexpr (!COOP) {
    const bool live = lane < m;
    int2 it = make_int2(0, 0);
    int4 cr = make_int4(0, 0, 0, 0);
    float base = 0.f;
    float f[16];
    long long deg = 0;
    uint64_t fp = 0;
#pragma unroll
    for (int d = 0; d < 16; ++d) f[d] = 0.f;
    if (live) {
      it = queue[lane];
      cr = p.cand[it.y];
      base = sum_base(p, it.x, cr.x);  // issued before the gather: its latency hides under it
      gather_sum<DIGEST>(p, cr.y, cr.z, inv_scale, f, deg, fp);
    }
    sum_score_lane<DIGEST>(p, w, relb, stage, live, it, cr, f, deg, fp, base, r, root);
    return;
  }
  int2 it = make_int2(0, 0);
  int4 cr = make_int4(0, 0, 0, 0);
  if (lane < m) {
    it = queue[lane];
    cr = p.cand[it.y];
  }
  bool todo = lane < m;
#pragma unroll 1
  while (true) {
    // this round's long-list candidates, gathered by the whole wave
    uint64_t big = __ballot(todo && cr.z > BIG_ENTRIES);
    int slot = -1;  // >= 0: this lane's feature is in fbig[slot]; -2: walk it here (int64 range)
    long long bdeg = 0;
    uint64_t bfp = 0;
#pragma unroll 1
    for (int nb = 0; big && nb < BIG_SLOTS; ++nb) {
      const int owner = __builtin_ctzll(big);
      big &= big - 1;
      const int beg = __builtin_amdgcn_readlane(cr.y, owner), cnt = __builtin_amdgcn_readlane(cr.z, owner);
      uint64_t csum;
      long long deg;
      uint64_t fp;
      coop_gather<DIGEST>(p, beg, cnt, inv_scale, fbig + nb * 16, csum, deg, fp);
      if (lane == owner) {
        slot = csum >= (1ull << 23) ? -2 : nb;  // past the exact fp64 range: the lane's int64 walk
        bdeg = deg;
        bfp = fp;
      }
    }
    wave_lds_sync();
    const bool go = todo && (cr.z <= BIG_ENTRIES || slot != -1);
    float base = 0.f;
    float f[16];
    long long deg = 0;
    uint64_t fp = 0;
#pragma unroll
    for (int d = 0; d < 16; ++d) f[d] = 0.f;
    if (go) {
      base = sum_base(p, it.x, cr.x);  // issued before the gather: its latency hides under it
      if (slot >= 0) {
#pragma unroll
        for (int d = 0; d < 16; ++d) f[d] = fbig[slot * 16 + d];
        deg = bdeg;
        fp = bfp;
      } else {
        gather_sum<DIGEST>(p, cr.y, cr.z, inv_scale, f, deg, fp);
      }
    }
    sum_score_lane<DIGEST>(p, w, relb, stage, go, it, cr, f, deg, fp, base, r, root);
    if (go) todo = false;
    wave_lds_sync();  // fbig is reused by the next round
    if (__ballot(todo) == 0ull) break;
  }
}

constexpr int SUM_CK = 8;  // chunks per dequeue on large launches
// Register budget (waves per SIMD) of the scoring pass that runs beside RotatE
// (atomic_out); a compile-time knob for A/B builds (tools/build_variants.sh).
// 5 (96 VGPRs, 120 B of spills): the pass is launched when the grounding ends,
// into a chip RotatE keeps full, and its workgroups must fit the space a
// grounding workgroup (106 -> 112 VGPRs per wave) frees.  At 4 (127 VGPRs)
// they did not, and trickled in as RotatE's waves retired: the scoring chain
// took 79 ms instead of 34 and often ended after RotatE (FB15k-237 step 82.0 /
// 82.4 ms vs 80.2 / 80.1 at 5, tools/interference.py).
#ifndef RNNL_OVERLAP_WPE
#define RNNL_OVERLAP_WPE 5
#endif
#ifndef RNNL_OVERLAP_COOP
#define RNNL_OVERLAP_COOP true
#endif
// One-stream launches (the chip to itself): up to SOLO_FEW_ROWS rows (e.g.
// the kinship split, 5,343 rows, ~10k chunks for the 8,192 waves of the grid)
// the 8-waves/SIMD build, whose whole grid is resident; larger ones (the
// FB15k-237 split: 0.9M chunks) the spill-free 4-waves/SIMD build with the
// cooperative long-list gather (ground + score alone 12.9 -> 10.4 ms).
constexpr int SOLO_FEW_ROWS = 8192;
// Launches with about one chunk per wave or fewer (up to SOLO_FEW_ROWS rows;
// one reference batch per call) keep a wave per chunk, so occupancy buys
// nothing there and the register budget goes to the entry walk: the
// 8-waves/SIMD build spilled ~90 VGPRs to scratch inside it (kinship step
// 0.570 -> 0.515 ms at 4 waves / 128 VGPRs, no spills; 0.531 at 5).  A/B knobs.
#ifndef RNNL_FEW_WPE
#define RNNL_FEW_WPE 4
#endif
#ifndef RNNL_SMALL_WPE
#define RNNL_SMALL_WPE 4
#endif
#ifndef RNNL_SMALL_OVERLAP_WPE
#define RNNL_SMALL_OVERLAP_WPE 4
#endif
#ifndef RNNL_SOLO_WPE
#define RNNL_SOLO_WPE 4
#endif
#ifndef RNNL_SOLO_COOP
#define RNNL_SOLO_COOP true
#endif

// WPE: waves per SIMD the register budget is sized for — 8 (64 VGPRs) when
// the pass has the chip to itself, RNNL_OVERLAP_WPE beside RotatE (above)
template <bool DIGEST, bool COOP, int WPE>
__global__ __launch_bounds__(BS) __attribute__((amdgpu_waves_per_eu(WPE, WPE))) void score_sum_chunk_kernel(
    KParams p, const float *__restrict__ W) {
  __shared__ SumLds s_w;
  __shared__ __attribute__((aligned(16))) float s_relb[BS / 64][128];
  __shared__ __attribute__((aligned(16))) float s_stage[BS / 64][256];  // score_mlp_f16's x1 staging
  __shared__ int2 s_queue[BS / 64][128];
  // the COOP flush's long-list features (BIG_SLOTS x 16 floats) share the
  // stage: they are read into registers before score_model stages x1
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  unsigned int *hdr = reinterpret_cast<unsigned int *>(p.ws);
  load_sum_weights(s_w, W);
  check_node_table(p, reinterpret_cast<const unsigned int *>(p.node_w + (int64_t)p.rl.n_nodes * kStrideSum));
  const int shift = (int)reinterpret_cast<const unsigned int *>(p.node_w + (int64_t)p.rl.n_nodes * kStrideSum)[1];
  const float inv_scale = ldexpf(1.f, -shift);
  __syncthreads();  // the only workgroup barrier: waves run independently from here
  const long long nchunks = (long long)*reinterpret_cast<const unsigned long long *>(hdr + H_CHUNKS);
  float *relb = s_relb[wv];
  int2 *queue = s_queue[wv];
  int cur_r = -1, cur_root = 0, n = 0;  // wave-uniform: the queue's relation, its trie root, the queue length
  unsigned c = 0, cend = 0;  // wave-uniform: the dequeued chunk range
  // chunks per dequeue: SUM_CK on large launches, fewer where that would leave
  // waves idle (at least 8 dequeues per wave)
  const int ck = (int)max(1ll, min((long long)SUM_CK, nchunks / ((long long)gridDim.x * (BS / 64) * 8)));
#pragma unroll 1
  while (true) {
    // up to SUM_CK chunks per atomic: one counter word serialises ~10^6 single dequeues per launch
    if (c == cend) next_chunks(&hdr[H_DEQUEUE2], nchunks, ck, c, cend);
    const bool done = (long long)c >= nchunks;
    int q = 0, s0 = 0, r = cur_r;
    if (!done) {
      const int2 ck2 = p.chunks[c];
      q = __builtin_amdgcn_readfirstlane(ck2.x);
      s0 = __builtin_amdgcn_readfirstlane(ck2.y);
      r = __builtin_amdgcn_readfirstlane((int)p.all_r[q]);
    }
    const bool drain = done || r != cur_r;
    // score full waves of queued candidates (all of them before a relation change / the exit)
#pragma unroll 1
    while (true) {
      const int m = drain ? min(n, 64) : (n >= 64 ? 64 : 0);
      if (m == 0) break;
      wave_lds_sync();
      sum_chunk_flush<DIGEST, COOP>(p, s_w, relb, s_stage[wv], queue, m, inv_scale, cur_r, cur_root, s_stage[wv]);
      n -= m;
      const int2 v = lane < n ? queue[m + lane] : make_int2(0, 0);
      wave_lds_sync();
      if (lane < n) queue[lane] = v;
    }
    if (done) break;
    if (r != cur_r) {
      wave_lds_sync();  // every lane is done with the previous relation's bias
      relb[lane] = relation_bias(p, r, lane);
      relb[lane + 64] = relation_bias(p, r, lane + 64);
      cur_r = r;
      cur_root = __builtin_amdgcn_readfirstlane(p.rl.head_root[r]);
    }
    const int nc = p.n_cand[q];
    const int64_t qb = p.q_base[q];
    const int s = s0 + lane;
    bool queued = false;
    if (s < nc) {
      const int4 cr = p.cand[qb + s];
      queued = true;
      unsigned long long key = PAIR_NOKEY;
      if (cr.z == 1) {
        const int2 be = p.bent[cr.y];
        if (be.y == 1 && p.memo) {  // one path of one leaf node: the memo
          queued = false;
          const float base = sum_base(p, q, cr.x);
          if constexpr (DIGEST)
            atomicAdd(reinterpret_cast<unsigned long long *>(p.digest + q),
                      (unsigned long long)mix64((uint64_t)cr.x ^ mix64((uint64_t)p.rl.node_nrules[be.x] ^
                                                                        mix64(p.rl.node_fp[be.x]))));
          sum_write_out(p, q, cr.x, p.memo[be.x], base);
        } else if (!DIGEST && p.ptab) {
          key = pair_key(p, r, cur_root, 1, be, make_int2(0, 0), make_int2(0, 0));
        }
      } else if (!DIGEST && p.ptab && cr.z <= 3) {
        key = pair_key(p, r, cur_root, cr.z, p.bent[cr.y], p.bent[cr.y + 1],
                       cr.z == 3 ? p.bent[cr.y + 2] : make_int2(0, 0));
      }
      float out;
      if (key != PAIR_NOKEY && pair_lookup(p, key, out)) {  // the pair memo holds these entries' output
        queued = false;
        sum_write_out(p, q, cr.x, out, sum_base(p, q, cr.x));
      }
    }
    const uint64_t bal = __ballot(queued);
    const int pos = n + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                       __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
    wave_lds_sync();
    if (queued) queue[pos] = make_int2(q, (int)(qb + s));
    n += (int)__popcll(bal);  // < 128: the queue held < 64 before this chunk
    ++c;
  }
}

// ---------------------------------------------------------------- launch
bool g_pair_memo = true;  // rnnl_debug_pair_memo (tests compare the outputs with the table off)

// Packs the MLP weights behind the workspace header (layout W_* in fwd.h).
__global__ void pack_weights_kernel(KParams p, float *__restrict__ W) {
  const int kin = p.agg == RNNL_AGG_SUM ? 16 : 192;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < W_FLOATS; i += gridDim.x * blockDim.x) {
    float v = 0.f;
    if (i < W_ADDB) {
      if (i < 16 * kin) v = p.add_w[i];
    } else if (i < W_LNW) {
      v = p.add_b[i - W_ADDB];
    } else if (i < W_LNB) {
      v = p.ln_w[i - W_LNW];
    } else if (i < W_S0X) {
      v = p.ln_b[i - W_LNB];
    } else if (i < W_S1W) {
      const int k = i - W_S0X;
      v = p.s0_w[(k / 16) * 32 + (k % 16)];
    } else if (i < W_S1B) {
      v = p.s1_w[i - W_S1W];
    } else if (i == W_S1B) {
      v = p.s1_b[0];
    }
    W[i] = v;
  }
}

extern "C" int rnnl_pack_weights_floats(size_t *n_floats) {
  if (!n_floats) {
    set_error("rnnl_pack_weights_floats: bad arguments");
    return RNNL_ERR_INVALID;
  }
  *n_floats = W_FLOATS;
  return RNNL_OK;
}

extern "C" int rnnl_pack_weights(const rnnl_predictor_params *pp, float *out, void *stream) {
  if (!pp || !out || (pp->aggregator != RNNL_AGG_SUM && pp->aggregator != RNNL_AGG_PNA)) {
    set_error("rnnl_pack_weights: bad arguments");
    return RNNL_ERR_INVALID;
  }
  KParams p{};
  set_score_params(p, pp, nullptr, nullptr, nullptr);
  hipLaunchKernelGGL(pack_weights_kernel, dim3((W_FLOATS + 255) / 256), dim3(256), 0, (hipStream_t)stream, p, out);
  RNNL_HIP_CHECK(hipGetLastError());
  return RNNL_OK;
}

// The scoring pass after a grounding (K2): packs the weights (unless the
// caller passes them packed), builds the
// chunk list and launches the aggregator's chunk kernel.  `grid` caps its
// persistent workgroups (0: the full grid); a smaller grid leaves CUs to a
// concurrent kernel (RotatE).
void launch_score(const KParams &p0, const RulesDev &rl, hipStream_t st, int grid) {
  KParams p = p0;
  const int nq = p.nq;
  const float *W = p.packed;
  if (!W) {
    float *Wp = reinterpret_cast<float *>(p.ws + HDR_WORDS_BYTES);
    hipLaunchKernelGGL(pack_weights_kernel, dim3((W_FLOATS + 255) / 256), dim3(256), 0, st, p, Wp);
    W = Wp;
  }
  // the pair memo (SUM; not with the test digest, which needs every
  // candidate's entries); a key needs >= 2 count bits per entry.  Its table
  // is zeroed by the chunk-list kernel.
  const bool pair = p.agg == RNNL_AGG_SUM && !p.digest && g_pair_memo && p.pbc >= 2;
  p.ptab = pair ? p.ptab_region : nullptr;
  launch_chunk_list(p, st);
  if (p.digest) (void)hipMemsetAsync(p.digest, 0, sizeof(uint64_t) * (size_t)nq, st);  // sums over chunks
  const unsigned cgrid = (unsigned)(grid > 0 ? grid : NUM_CU * SCORE_WG_PER_CU);
  if (p.agg != RNNL_AGG_SUM) {
    hipLaunchKernelGGL(score_pna_chunk_kernel, dim3(cgrid), dim3(BS), 0, st, p, W);
    return;
  }
  // few rows (e.g. one reference batch per call) with the pair memo on: no
  // memo pass (one workgroup per relation, on the call's critical path); the
  // single-path candidates take pair-memo keys instead — the same outputs
  const bool small = nq <= MEMO_SCAN_ROWS;
  if (small && pair)
    p.memo = nullptr;
  else
    hipLaunchKernelGGL(memo_sum_kernel, dim3((unsigned)std::max(p.g.R, 1)), dim3(BS), 0, st, p, W);
  // one reference batch per call: the wave-cooperative walk of long entry lists
  // (bit-identical features); large launches keep the per-lane walk
  if (p.digest && small)
    hipLaunchKernelGGL((score_sum_chunk_kernel<true, true, 8>), dim3(cgrid), dim3(BS), 0, st, p, W);
  else if (p.digest)
    hipLaunchKernelGGL((score_sum_chunk_kernel<true, false, 8>), dim3(cgrid), dim3(BS), 0, st, p, W);
  else if (p.atomic_out && small)
    hipLaunchKernelGGL((score_sum_chunk_kernel<false, true, RNNL_SMALL_OVERLAP_WPE>), dim3(cgrid), dim3(BS), 0, st, p,
                       W);
  else if (p.atomic_out)
    hipLaunchKernelGGL((score_sum_chunk_kernel<false, RNNL_OVERLAP_COOP, RNNL_OVERLAP_WPE>), dim3(cgrid), dim3(BS), 0, st, p, W);
  else if (small)
    hipLaunchKernelGGL((score_sum_chunk_kernel<false, true, RNNL_SMALL_WPE>), dim3(cgrid), dim3(BS), 0, st, p, W);
  else if (nq <= SOLO_FEW_ROWS)  // about one chunk per wave: occupancy (8 waves/SIMD) over spill-free waves
    hipLaunchKernelGGL((score_sum_chunk_kernel<false, false, RNNL_FEW_WPE>), dim3(cgrid), dim3(BS), 0, st, p, W);
  else
    hipLaunchKernelGGL((score_sum_chunk_kernel<false, RNNL_SOLO_COOP, RNNL_SOLO_WPE>), dim3(cgrid), dim3(BS), 0, st, p, W);
}

}  // namespace rnnl
