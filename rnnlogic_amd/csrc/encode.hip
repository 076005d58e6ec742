// Rule encoder for gfx950: PredictorPlus.encode_rules (reference
// src/predictors.py:201-208) for type == 'lstm' in one kernel.
//
// Every rule is a short token sequence [head, body..., pad...] (length <= 6);
// the reference runs torch.nn.LSTM(16, 16, num_layers) over the padded batch
// and gathers the top layer's output at the last non-pad position.  The LSTM
// is causal, so that output only depends on the first `len` tokens: one lane
// per rule walks its own `len` steps through all layers, with the 16-wide
// states in registers and the gate weights (layers x 4 gates x 16 x 32) in LDS
// (wave-uniform broadcast reads).  131,883 FB15k-237 rules: ~3 GFLOP, one
// launch instead of the per-layer/per-step library kernels.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "internal.h"

namespace rnnl {

constexpr int LH = 16;       // hidden size (the kernels' specialisation)
constexpr int LMAXL = 3;     // layers supported
constexpr int LG = 4 * LH;   // gates per layer (i, f, g, o: torch order)
constexpr int LMAXT = 8;     // tokens per rule (head + body <= 7)
#ifndef LSTM_BLOCKS_PER_CU
#define LSTM_BLOCKS_PER_CU 4
#endif

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + expf(-x)); }

// LDS image per layer: w[gate][k] (k < 16: input, 16 <= k < 32: hidden),
// rows padded to 33 floats so the 16 lanes of a rule (16 different gate rows)
// hit 16 different banks; bias = b_ih + b_hh.
constexpr int LROW = 2 * LH + 1;
struct LstmLds {
  float w[LMAXL][LG][LROW];
  float b[LMAXL][LG];
};

// Element K of a 16-lane row (a rule's group) broadcast to the row: one DPP
// row_newbcast operand, no LDS traffic (ds_bpermute was 32 LDS ops per step).
template <int K>
__device__ __forceinline__ float row_bcast(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x150 + K, 0xF, 0xF,
                                                               false));
}

// The gate pre-activations of one step, k ascending (the order of the
// shuffle form it replaces): a[q] += w[q][k] x_k + w[q][16 + k] h_k.
template <int K>
__device__ __forceinline__ void gate_terms(const float (&w)[4][2 * LH], float x, float h, float (&a)[4]) {
  const float xk = row_bcast<K>(x), hk = row_bcast<K>(h);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    a[q] = fmaf(w[q][K], xk, a[q]);
    a[q] = fmaf(w[q][LH + K], hk, a[q]);
  }
  if constexpr (K + 1 < LH) gate_terms<K + 1>(w, x, h, a);
}

// 16 lanes per rule, lane j owns hidden unit j: its 4 gate rows (in registers
// for the layer's steps: the LDS image is read once per layer and rule
// group, not once per step), c_j, h_j and its element of every step's layer
// output.  The step input and the previous hidden state are broadcast within
// the rule's 16-lane DPP row.
__global__ __launch_bounds__(256) void lstm_encode_kernel(const float *__restrict__ vocab, const float *__restrict__ w_ih,
                                                          const float *__restrict__ w_hh,
                                                          const float *__restrict__ b_ih,
                                                          const float *__restrict__ b_hh,
                                                          const int32_t *__restrict__ tokens, int T, int pad,
                                                          int n_rules, int layers, float *__restrict__ out,
                                                          int ld_out) {
  __shared__ LstmLds S;
  for (int i = threadIdx.x; i < layers * LG * 2 * LH; i += blockDim.x) {
    const int l = i / (LG * 2 * LH), g = (i / (2 * LH)) % LG, k = i % (2 * LH);
    S.w[l][g][k] = k < LH ? w_ih[(l * LG + g) * LH + k] : w_hh[(l * LG + g) * LH + (k - LH)];
  }
  for (int i = threadIdx.x; i < layers * LG; i += blockDim.x) S.b[i / LG][i % LG] = b_ih[i] + b_hh[i];
  __syncthreads();
  const int j = threadIdx.x & (LH - 1);
  // grid-stride over 16-rule groups: the weight image is loaded once per block
  for (int64_t g0 = (int64_t)blockIdx.x * blockDim.x; g0 < (int64_t)n_rules * LH;
       g0 += (int64_t)gridDim.x * blockDim.x) {
    const int rule = (int)((g0 + threadIdx.x) / LH);
    const bool valid = rule < n_rules;  // whole 16-lane groups agree
    const int32_t *tok = tokens + (int64_t)(valid ? rule : 0) * T;
    int len = 0;
    while (len < T && tok[len] != pad) ++len;
    float seq[LMAXT];  // element j of the current layer's input (then output) at each step
#pragma unroll
    for (int t = 0; t < LMAXT; ++t) seq[t] = vocab[(int64_t)tok[t < len ? t : 0] * LH + j];
#pragma unroll 1
    for (int l = 0; l < layers; ++l) {
      float w[4][2 * LH], bias[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        bias[q] = S.b[l][q * LH + j];
#pragma unroll
        for (int k = 0; k < 2 * LH; ++k) w[q][k] = S.w[l][q * LH + j][k];
      }
      float h = 0.f, c = 0.f;
#pragma unroll
      for (int t = 0; t < LMAXT; ++t) {
        if (t < len) {  // uniform over the rule's row (DPP reads of inactive lanes would return 0)
          float a[4] = {bias[0], bias[1], bias[2], bias[3]};
          gate_terms<0>(w, seq[t], h, a);
          c = fmaf(sigm(a[1]), c, sigm(a[0]) * tanhf(a[2]));
          h = sigm(a[3]) * tanhf(c);
          seq[t] = h;
        }
      }
    }
    // top layer's output at the last non-pad position (len >= 1: the head token)
    if (valid) {
      float v = 0.f;
#pragma unroll
      for (int t = 0; t < LMAXT; ++t)
        if (t == len - 1) v = seq[t];
      out[(int64_t)rule * ld_out + j] = v;
    }
  }
}

// ---------------------------------------------------------------------------
// The same encoder over the rule trie (rnnl_lstm_encode_trie).  The LSTM is
// causal and a rule's tokens are [head, body...], so every prefix a trie node
// stands for (the root: [head]) has one state, shared by all rules through
// it: one step per trie node (FB15k-237: 183,810 nodes instead of 473,782
// rule steps), one launch per depth.  A 16-lane row owns TK nodes of a level
// (TK_WIDE; one on small levels) and runs them layer by layer, so each
// layer's gate rows are read from LDS once per TK nodes; the step reads the parent's (h, c) of every layer from
// `state` [node][layer][h | c][16] and writes the node's.  The arithmetic of
// a step is lstm_encode_kernel's, on the same inputs: the outputs are
// bitwise those of rnnl_lstm_encode.  A node's top-layer h goes to every
// rule ending there.
// Levels of fewer than TK1_NODES nodes (kinship's whole trie; the top
// levels of larger ones) take one node per row instead: the grid is far
// below the chip there, and a row's TK steps per layer are a serial chain.
constexpr int TK_WIDE = 4;
constexpr int TK1_NODES = 8192;  // 4,096 / 32,768 / all levels: no better (kinship 0.60 / 0.60 / 0.60 ms)

// per-layer parameter pointers (torch's weight_ih_l{k} ... used in place)
struct LstmLayerPtrs {
  const float *w_ih[LMAXL], *w_hh[LMAXL], *b_ih[LMAXL], *b_hh[LMAXL];
};


template <int TK>
__global__ __launch_bounds__(256) void lstm_trie_level_kernel(const float *__restrict__ vocab, LstmLayerPtrs P,
                                                              RulesDev rl, int lv0, int n_level, int layers,
                                                              float *__restrict__ state, float *__restrict__ out,
                                                              int ld_out, const float *__restrict__ add_w,
                                                              unsigned char *__restrict__ rec) {
  __shared__ LstmLds S;
  for (int i = threadIdx.x; i < layers * LG * 2 * LH; i += blockDim.x) {
    const int l = i / (LG * 2 * LH), g = (i / (2 * LH)) % LG, k = i % (2 * LH);
    S.w[l][g][k] = k < LH ? P.w_ih[l][g * LH + k] : P.w_hh[l][g * LH + (k - LH)];
  }
  for (int i = threadIdx.x; i < layers * LG; i += blockDim.x)
    S.b[i / LG][i % LG] = P.b_ih[i / LG][i % LG] + P.b_hh[i / LG][i % LG];
  __syncthreads();
  const int j = threadIdx.x & (LH - 1);
  unsigned int rm = 0, rm2 = 0;  // max |record|, max |node sum| bits (rec)
  const int64_t n_groups = ((int64_t)n_level + TK - 1) / TK;
  for (int64_t g0 = (int64_t)blockIdx.x * blockDim.x; g0 < n_groups * LH; g0 += (int64_t)gridDim.x * blockDim.x) {
    const int64_t grp = (g0 + threadIdx.x) / LH;  // uniform over the 16-lane row
    int node[TK], par[TK];
    float x[TK];
#pragma unroll
    for (int k = 0; k < TK; ++k) {
      const int64_t i = grp * TK + k;
      node[k] = i < n_level ? rl.level_nodes[lv0 + i] : -1;
      par[k] = node[k] >= 0 ? rl.node_parent[node[k]] : -1;
      x[k] = node[k] >= 0 ? vocab[(int64_t)rl.node_tok[node[k]] * LH + j] : 0.f;
    }
    // the parents' (h, c) of every layer, loaded before this group's first
    // store: the stores below may alias `state` as far as the compiler knows,
    // so a load issued after one waits for it — one memory latency per
    // (node, layer) step instead of one per group
    static_assert(LMAXL == 3, "the layer select below");
    float ph[TK][LMAXL], pc[TK][LMAXL];
#pragma unroll
    for (int k = 0; k < TK; ++k)
#pragma unroll
      for (int l = 0; l < LMAXL; ++l) {
        const bool ld = par[k] >= 0 && l < layers;
        const float *ps = state + ((int64_t)(ld ? par[k] : 0) * layers + l) * 2 * LH;
        ph[k][l] = ld ? ps[j] : 0.f;
        pc[k][l] = ld ? ps[LH + j] : 0.f;
      }
#pragma unroll 1
    for (int l = 0; l < layers; ++l) {
      float w[4][2 * LH], bias[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        bias[q] = S.b[l][q * LH + j];
#pragma unroll
        for (int k = 0; k < 2 * LH; ++k) w[q][k] = S.w[l][q * LH + j][k];
      }
#pragma unroll
      for (int k = 0; k < TK; ++k) {
        if (node[k] >= 0) {  // uniform over the row
          const float h = l == 0 ? ph[k][0] : l == 1 ? ph[k][1] : ph[k][2];
          const float c0 = l == 0 ? pc[k][0] : l == 1 ? pc[k][1] : pc[k][2];
          float a[4] = {bias[0], bias[1], bias[2], bias[3]};
          gate_terms<0>(w, x[k], h, a);
          const float c = fmaf(sigm(a[1]), c0, sigm(a[0]) * tanhf(a[2]));
          const float hn = sigm(a[3]) * tanhf(c);
          float *st = state + ((int64_t)node[k] * layers + l) * 2 * LH;
          st[j] = hn;
          st[LH + j] = c;
          x[k] = hn;
        }
      }
    }
#pragma unroll
    for (int k = 0; k < TK; ++k)
      if (node[k] >= 0) {  // uniform over the row
        float s1 = 0.f;
        for (int m = rl.node_rule_ptr[node[k]]; m < rl.node_rule_ptr[node[k] + 1]; ++m) {
          out[(int64_t)rl.node_rules[m] * ld_out + j] = x[k];
          s1 += x[k];
        }
        if (rec) {  // the SUM record: node_weights_kernel's arithmetic on the rows just written
          float y = 0.f;
#pragma unroll
          for (int i = 0; i < 16; ++i) y = fmaf(__shfl(s1, i, 16), add_w[j * 16 + i], y);
          reinterpret_cast<float *>(rec + (int64_t)node[k] * kStrideSum)[j] = y;
          rm = max(rm, __float_as_uint(fabsf(y)));
          rm2 = max(rm2, __float_as_uint(fabsf(s1)));
        }
      }
  }
  if (rec) {  // table maxima into the trailer (node_fix_kernel's shift), as node_weights_kernel
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      rm = max(rm, (unsigned int)__shfl_xor((int)rm, o, 64));
      rm2 = max(rm2, (unsigned int)__shfl_xor((int)rm2, o, 64));
    }
    __shared__ unsigned int s_m[4], s_m2[4];
    if ((threadIdx.x & 63) == 0) {
      s_m[threadIdx.x >> 6] = rm;
      s_m2[threadIdx.x >> 6] = rm2;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned int *trailer = reinterpret_cast<unsigned int *>(rec + (int64_t)rl.n_nodes * kStrideSum);
      rm = max(max(s_m[0], s_m[1]), max(s_m[2], s_m[3]));
      rm2 = max(max(s_m2[0], s_m2[1]), max(s_m2[2], s_m2[3]));
      if (rm) atomicMax(trailer, rm);
      if (rm2) atomicMax(trailer + 3, rm2);
    }
  }
}

// ---------------------------------------------------------------------------
// Training (autograd through the rule encoder): the same recurrence over the
// rules ridx[0..n) of one batch, saving each step's activations, and the
// backward through time.  Activation / gradient rows are (row, t) = row T + t.
//
//   act  [L][T][6][n 16]: i, f, g, o, c_t, h_t (lane-contiguous per field)
//   da   [L][n T][64]  : dL/d(gate pre-activations) (zero for pad steps)
//   xh   [L][n T][32]  : the step's input x_t | h_(t-1) (zero for pad steps)
//   dvx  [n T][16]     : dL/d(layer-0 input) = the vocab rows' gradient
// The weight gradients are then dW_l = da_l^T xh_l and db_l = sum of da_l's
// rows (a batched GEMM over the n T rows, host side), the vocab gradient a
// per-token sum of dvx rows (vocab_grad_kernel).

__global__ __launch_bounds__(256) void lstm_train_fwd_kernel(const float *__restrict__ vocab, LstmLayerPtrs P,
                                                             const int32_t *__restrict__ tokens, int T, int pad,
                                                             const int64_t *__restrict__ ridx, int n, int layers,
                                                             float *__restrict__ out, float *__restrict__ act) {
  __shared__ LstmLds S;
  for (int i = threadIdx.x; i < layers * LG * 2 * LH; i += blockDim.x) {
    const int l = i / (LG * 2 * LH), g = (i / (2 * LH)) % LG, k = i % (2 * LH);
    S.w[l][g][k] = k < LH ? P.w_ih[l][g * LH + k] : P.w_hh[l][g * LH + (k - LH)];
  }
  for (int i = threadIdx.x; i < layers * LG; i += blockDim.x) S.b[i / LG][i % LG] = P.b_ih[i / LG][i % LG] + P.b_hh[i / LG][i % LG];
  __syncthreads();
  const int j = threadIdx.x & (LH - 1);
  const int64_t N16 = (int64_t)n * LH;
  for (int64_t g0 = (int64_t)blockIdx.x * blockDim.x; g0 < N16; g0 += (int64_t)gridDim.x * blockDim.x) {
    const int row = (int)((g0 + threadIdx.x) / LH);
    const bool valid = row < n;
    const int32_t *tok = tokens + (valid ? ridx[row] : ridx[0]) * (int64_t)T;
    int len = 0;
    while (len < T && tok[len] != pad) ++len;
    float seq[LMAXT];
#pragma unroll
    for (int t = 0; t < LMAXT; ++t) seq[t] = vocab[(int64_t)tok[t < len ? t : 0] * LH + j];
#pragma unroll 1
    for (int l = 0; l < layers; ++l) {
      float w[4][2 * LH], bias[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        bias[q] = S.b[l][q * LH + j];
#pragma unroll
        for (int k = 0; k < 2 * LH; ++k) w[q][k] = S.w[l][q * LH + j][k];
      }
      float h = 0.f, c = 0.f;
#pragma unroll
      for (int t = 0; t < LMAXT; ++t) {
        if (t < len) {
          float a[4] = {bias[0], bias[1], bias[2], bias[3]};
          gate_terms<0>(w, seq[t], h, a);
          const float gi = sigm(a[0]), gf = sigm(a[1]), gg = tanhf(a[2]), go = sigm(a[3]);
          c = fmaf(gf, c, gi * gg);
          h = go * tanhf(c);
          seq[t] = h;
          if (valid) {
            float *o = act + ((int64_t)(l * T + t) * 6) * N16 + (int64_t)row * LH + j;
            o[0] = gi;
            o[N16] = gf;
            o[2 * N16] = gg;
            o[3 * N16] = go;
            o[4 * N16] = c;
            o[5 * N16] = h;
          }
        }
      }
    }
    if (valid) {
      float v = 0.f;
#pragma unroll
      for (int t = 0; t < LMAXT; ++t)
        if (t == len - 1) v = seq[t];
      out[(int64_t)row * LH + j] = v;
    }
  }
}

// dst[k] = sum over the rule row's 16 lanes jj and the 4 gates q of
// wt[q][jj] a_q(lane jj): the lane's column of W times the row's gate grads
template <int JJ>
__device__ __forceinline__ void col_terms(const float (&wi)[4][LH], const float (&wh)[4][LH], const float (&a)[4],
                                          float &dx, float &dh) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float aq = row_bcast<JJ>(a[q]);
    dx = fmaf(wi[q][JJ], aq, dx);
    dh = fmaf(wh[q][JJ], aq, dh);
  }
  if constexpr (JJ + 1 < LH) col_terms<JJ + 1>(wi, wh, a, dx, dh);
}

__global__ __launch_bounds__(256) void lstm_train_bwd_kernel(const float *__restrict__ vocab, LstmLayerPtrs P,
                                                             const int32_t *__restrict__ tokens, int T, int pad,
                                                             const int64_t *__restrict__ ridx, int n, int layers,
                                                             const float *__restrict__ act,
                                                             const float *__restrict__ d_out, float *__restrict__ da,
                                                             float *__restrict__ xh, float *__restrict__ dvx) {
  // W^T images: s_wt[l][k][gate] (k < 16: w_ih column k, else w_hh column k - 16)
  __shared__ float s_wt[LMAXL][2 * LH][LG + 1];
  for (int i = threadIdx.x; i < layers * LG * 2 * LH; i += blockDim.x) {
    const int l = i / (LG * 2 * LH), g = (i / (2 * LH)) % LG, k = i % (2 * LH);
    s_wt[l][k][g] = k < LH ? P.w_ih[l][g * LH + k] : P.w_hh[l][g * LH + (k - LH)];
  }
  __syncthreads();
  const int j = threadIdx.x & (LH - 1);
  const int64_t N16 = (int64_t)n * LH;
  const int64_t NT = (int64_t)n * T;
  for (int64_t g0 = (int64_t)blockIdx.x * blockDim.x; g0 < N16; g0 += (int64_t)gridDim.x * blockDim.x) {
    const int row = (int)((g0 + threadIdx.x) / LH);
    const bool valid = row < n;  // whole 16-lane rows agree
    const int32_t *tok = tokens + (valid ? ridx[row] : ridx[0]) * (int64_t)T;
    int len = 0;
    while (len < T && tok[len] != pad) ++len;
    if (!valid) len = 0;
    float dseq[LMAXT];  // dL/d(this layer's output h_t), element j
#pragma unroll
    for (int t = 0; t < LMAXT; ++t) dseq[t] = (valid && t == len - 1) ? d_out[(int64_t)row * LH + j] : 0.f;
#pragma unroll 1
    for (int l = layers - 1; l >= 0; --l) {
      float wi[4][LH], wh[4][LH];
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int jj = 0; jj < LH; ++jj) {
          wi[q][jj] = s_wt[l][j][q * LH + jj];
          wh[q][jj] = s_wt[l][LH + j][q * LH + jj];
        }
      const float *A = act + (int64_t)l * T * 6 * N16 + (int64_t)row * LH + j;
      float dh_next = 0.f, dc_next = 0.f;
#pragma unroll
      for (int t = LMAXT - 1; t >= 0; --t) {
        if (t >= T) continue;
        float *dar = da + ((int64_t)l * NT + (int64_t)row * T + t) * LG;
        float *xr = xh + ((int64_t)l * NT + (int64_t)row * T + t) * 2 * LH;
        if (t < len) {  // uniform over the row
          const float *at = A + (int64_t)t * 6 * N16;
          const float gi = at[0], gf = at[N16], gg = at[2 * N16], go = at[3 * N16], c = at[4 * N16];
          const float cp = t > 0 ? at[4 * N16 - 6 * N16] : 0.f;
          const float hp = t > 0 ? at[5 * N16 - 6 * N16] : 0.f;
          const float x = l == 0 ? vocab[(int64_t)tok[t] * LH + j] : act[((int64_t)((l - 1) * T + t) * 6 + 5) * N16 +
                                                                           (int64_t)row * LH + j];
          const float dh = dseq[t] + dh_next;
          const float tc = tanhf(c);
          const float dc = fmaf(dh * go, 1.f - tc * tc, dc_next);
          float a[4];
          a[0] = dc * gg * gi * (1.f - gi);
          a[1] = dc * cp * gf * (1.f - gf);
          a[2] = dc * gi * (1.f - gg * gg);
          a[3] = dh * tc * go * (1.f - go);
          dc_next = dc * gf;
#pragma unroll
          for (int q = 0; q < 4; ++q) dar[q * LH + j] = a[q];
          xr[j] = x;
          xr[LH + j] = hp;
          float dx = 0.f, dhp = 0.f;
          col_terms<0>(wi, wh, a, dx, dhp);
          dh_next = dhp;
          dseq[t] = dx;  // this step's gradient to the layer below (or to the vocab row)
        } else if (valid) {
#pragma unroll
          for (int q = 0; q < 4; ++q) dar[q * LH + j] = 0.f;
          xr[j] = 0.f;
          xr[LH + j] = 0.f;
        }
      }
    }
    if (valid) {
#pragma unroll
      for (int t = 0; t < LMAXT; ++t)
        if (t < T) dvx[((int64_t)row * T + t) * LH + j] = t < len ? dseq[t] : 0.f;
    }
  }
}

// d_vocab[tok_id[u]][k] = sum of dvx rows pos[ptr[u] .. ptr[u + 1]) (in list
// order: deterministic), one thread per (token, k); the other vocab rows are
// zeroed by the caller.
__global__ void vocab_grad_kernel(const float *__restrict__ dvx, const int32_t *__restrict__ tok_id,
                                  const int32_t *__restrict__ ptr, const int32_t *__restrict__ pos, int n_tok,
                                  float *__restrict__ d_vocab) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_tok * LH) return;
  const int u = i / LH, k = i % LH;
  float s = 0.f;
  for (int p = ptr[u]; p < ptr[u + 1]; ++p) s += dvx[(int64_t)pos[p] * LH + k];
  d_vocab[(int64_t)tok_id[u] * LH + k] = s;
}

// Weight gradients dW_l = da_l^T [x | h_prev], db_l = column sums of da_l
// (torch.nn.LSTM's, summed over every rule and step) in a fixed order: block
// (segment, layer) sums its WG_SEG rows in row order into part, then
// lstm_wgrad_fold_kernel sums the segments in segment order.  Column
// WG_COLS - 1 is the bias (an all-ones input column).
constexpr int WG_SEG = 128;
constexpr int WG_COLS = 2 * LH + 1;
constexpr int WG_PER = (WG_COLS + 3) / 4;  // columns per thread (4 column groups)

static inline int64_t wg_segments(int64_t rows) { return (rows + WG_SEG - 1) / WG_SEG; }

__global__ void __launch_bounds__(256) lstm_wgrad_part_kernel(const float *__restrict__ da,
                                                              const float *__restrict__ xh, int64_t rows,
                                                              float *__restrict__ part) {
  const int g = threadIdx.x & (LG - 1), cg = threadIdx.x >> 6;
  const int l = blockIdx.y, L = gridDim.y;
  const int64_t seg = blockIdx.x, r0 = seg * WG_SEG, r1 = r0 + WG_SEG < rows ? r0 + WG_SEG : rows;
  float acc[WG_PER];
#pragma unroll
  for (int j = 0; j < WG_PER; ++j) acc[j] = 0.f;
  const float *dal = da + (int64_t)l * rows * LG;
  const float *xhl = xh + (int64_t)l * rows * 2 * LH;
  for (int64_t r = r0; r < r1; ++r) {
    const float a = dal[r * LG + g];
    const float *x = xhl + r * 2 * LH;
#pragma unroll
    for (int j = 0; j < WG_PER; ++j) {
      const int c = cg + 4 * j;
      if (c < 2 * LH)
        acc[j] = fmaf(a, x[c], acc[j]);
      else if (c == 2 * LH)
        acc[j] += a;
    }
  }
#pragma unroll
  for (int j = 0; j < WG_PER; ++j) {
    const int c = cg + 4 * j;
    if (c < WG_COLS) part[((seg * L + l) * WG_COLS + c) * LG + g] = acc[j];
  }
}

__global__ void lstm_wgrad_fold_kernel(const float *__restrict__ part, int L, int64_t nseg, float *__restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= L * WG_COLS * LG) return;
  const int g = i % LG, c = (i / LG) % WG_COLS, l = i / (LG * WG_COLS);
  float s = 0.f;
  for (int64_t seg = 0; seg < nseg; ++seg) s += part[((seg * L + l) * WG_COLS + c) * LG + g];
  const int64_t wsz = (int64_t)L * LG * LH;
  if (c < LH)
    out[((int64_t)l * LG + g) * LH + c] = s;
  else if (c < 2 * LH)
    out[wsz + ((int64_t)l * LG + g) * LH + (c - LH)] = s;
  else
    out[2 * wsz + (int64_t)l * LG + g] = s;
}

}  // namespace rnnl

using namespace rnnl;

extern "C" {

int rnnl_lstm_encode(const float *vocab, const float *w_ih, const float *w_hh, const float *b_ih, const float *b_hh,
                     int32_t layers, int32_t hidden, const int32_t *tokens, int32_t n_rules, int32_t seq_len,
                     int32_t pad, float *out, int32_t ld_out, void *stream) {
  if (!vocab || !w_ih || !w_hh || !b_ih || !b_hh || !tokens || !out || n_rules < 0 || seq_len <= 0 ||
      seq_len > LMAXT || layers < 1 || layers > LMAXL || hidden != LH || ld_out < LH) {
    set_error("rnnl_lstm_encode: bad arguments (hidden 16, 1 <= layers <= 3, rules of <= 7 tokens)");
    return RNNL_ERR_INVALID;
  }
  if (n_rules == 0) return RNNL_OK;
  // at most LSTM_BLOCKS_PER_CU blocks per CU, each looping over rule groups
  const int64_t blocks = std::min<int64_t>(((int64_t)n_rules * LH + 255) / 256, 256 * LSTM_BLOCKS_PER_CU);
  hipLaunchKernelGGL(lstm_encode_kernel, dim3((unsigned)blocks), dim3(256), 0,
                     (hipStream_t)stream, vocab, w_ih,
                     w_hh, b_ih, b_hh, tokens, seq_len, pad, n_rules, layers, out, ld_out);
  RNNL_HIP_CHECK(hipGetLastError());
  return RNNL_OK;
}

int rnnl_lstm_encode_trie_scratch(rnnl_rules r, int32_t layers, size_t *bytes) {
  if (!r || layers < 1 || layers > LMAXL || !bytes) {
    set_error("rnnl_lstm_encode_trie_scratch: bad arguments");
    return RNNL_ERR_INVALID;
  }
  *bytes = (size_t)std::max(r->d.n_nodes, 1) * layers * 2 * LH * sizeof(float);
  return RNNL_OK;
}

static int encode_trie(const char *who, rnnl_rules r, const float *vocab, const float *const *w_ih,
                       const float *const *w_hh, const float *const *b_ih, const float *const *b_hh, int32_t layers,
                       int32_t hidden, float *out, int32_t ld_out, void *scratch, size_t scratch_bytes,
                       const float *add_w, unsigned char *rec, void *stream) {
  size_t need = 0;
  LstmLayerPtrs P{};
  bool ok = r && vocab && w_ih && w_hh && b_ih && b_hh && out && hidden == LH && ld_out >= LH &&
            rnnl_lstm_encode_trie_scratch(r, layers, &need) == RNNL_OK && scratch && scratch_bytes >= need;
  for (int l = 0; ok && l < layers; ++l) {
    ok = w_ih[l] && w_hh[l] && b_ih[l] && b_hh[l];
    P.w_ih[l] = w_ih[l];
    P.w_hh[l] = w_hh[l];
    P.b_ih[l] = b_ih[l];
    P.b_hh[l] = b_hh[l];
  }
  if (!ok) {
    set_error(std::string(who) + ": bad arguments (hidden 16, 1 <= layers <= 3, scratch: "
              "rnnl_lstm_encode_trie_scratch)");
    return RNNL_ERR_INVALID;
  }
  if (rec)  // the trailer's maxima (node_fix_kernel's shift) start from zero
    RNNL_HIP_CHECK(hipMemsetAsync(rec + (int64_t)r->d.n_nodes * kStrideSum, 0, 32, (hipStream_t)stream));
  for (size_t d = 0; d + 1 < r->level_ptr.size(); ++d) {
    const int lv0 = r->level_ptr[d], n = r->level_ptr[d + 1] - lv0;
    if (n <= 0) continue;
    const int tk = n < TK1_NODES ? 1 : TK_WIDE;
    const int64_t lanes = ((int64_t)n + tk - 1) / tk * LH;
    const unsigned blocks = (unsigned)std::min<int64_t>((lanes + 255) / 256, 256 * LSTM_BLOCKS_PER_CU);
    if (tk == 1)
      hipLaunchKernelGGL(lstm_trie_level_kernel<1>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, vocab, P, r->d,
                         lv0, n, layers, static_cast<float *>(scratch), out, ld_out, add_w, rec);
    else
      hipLaunchKernelGGL(lstm_trie_level_kernel<TK_WIDE>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, vocab, P,
                         r->d, lv0, n, layers, static_cast<float *>(scratch), out, ld_out, add_w, rec);
  }
  RNNL_HIP_CHECK(hipGetLastError());
  return RNNL_OK;
}

int rnnl_lstm_encode_trie(rnnl_rules r, const float *vocab, const float *const *w_ih, const float *const *w_hh,
                          const float *const *b_ih, const float *const *b_hh, int32_t layers, int32_t hidden,
                          float *out, int32_t ld_out, void *scratch, size_t scratch_bytes, void *stream) {
  return encode_trie("rnnl_lstm_encode_trie", r, vocab, w_ih, w_hh, b_ih, b_hh, layers, hidden, out, ld_out, scratch,
                     scratch_bytes, nullptr, nullptr, stream);
}

int rnnl_lstm_encode_trie_sum(rnnl_rules r, const float *vocab, const float *const *w_ih, const float *const *w_hh,
                              const float *const *b_ih, const float *const *b_hh, int32_t layers, int32_t hidden,
                              float *out, int32_t ld_out, void *scratch, size_t scratch_bytes, const float *add_w,
                              void *node_w, void *stream) {
  if (!add_w || !node_w) {
    set_error("rnnl_lstm_encode_trie_sum: bad arguments");
    return RNNL_ERR_INVALID;
  }
  if (int rc = encode_trie("rnnl_lstm_encode_trie_sum", r, vocab, w_ih, w_hh, b_ih, b_hh, layers, hidden, out, ld_out,
                           scratch, scratch_bytes, add_w, static_cast<unsigned char *>(node_w), stream))
    return rc;
  return node_fix_enqueue(r, node_w, stream);
}

static bool lstm_train_args(const float *vocab, const float *const *w_ih, const float *const *w_hh,
                            const float *const *b_ih, const float *const *b_hh, int32_t layers, const int32_t *tokens,
                            int32_t seq_len, const int64_t *ridx, int32_t n, LstmLayerPtrs &P) {
  if (!vocab || !w_ih || !w_hh || !b_ih || !b_hh || !tokens || !ridx || n <= 0 || seq_len <= 0 ||
      seq_len > LMAXT || layers < 1 || layers > LMAXL)
    return false;
  for (int l = 0; l < layers; ++l) {
    if (!w_ih[l] || !w_hh[l] || !b_ih[l] || !b_hh[l]) return false;
    P.w_ih[l] = w_ih[l];
    P.w_hh[l] = w_hh[l];
    P.b_ih[l] = b_ih[l];
    P.b_hh[l] = b_hh[l];
  }
  return true;
}

static unsigned lstm_blocks(int32_t n) {
  return (unsigned)std::min<int64_t>(((int64_t)n * LH + 255) / 256, 256 * LSTM_BLOCKS_PER_CU);
}

int rnnl_lstm_train_sizes(int32_t layers, int32_t hidden, int32_t seq_len, int32_t n, size_t *act_floats,
                          size_t *da_floats, size_t *xh_floats, size_t *dvx_floats) {
  if (hidden != LH || layers < 1 || layers > LMAXL || seq_len <= 0 || seq_len > LMAXT || n < 0 || !act_floats ||
      !da_floats || !xh_floats || !dvx_floats) {
    set_error("rnnl_lstm_train_sizes: bad arguments (hidden 16, 1 <= layers <= 3, rules of <= 7 tokens)");
    return RNNL_ERR_INVALID;
  }
  *act_floats = (size_t)layers * seq_len * 6 * n * LH;
  *da_floats = (size_t)layers * n * seq_len * LG;
  *xh_floats = (size_t)layers * n * seq_len * 2 * LH;
  *dvx_floats = (size_t)n * seq_len * LH;
  return RNNL_OK;
}

int rnnl_lstm_train_forward(const float *vocab, const float *const *w_ih, const float *const *w_hh,
                            const float *const *b_ih, const float *const *b_hh, int32_t layers, int32_t hidden,
                            const int32_t *tokens, int32_t seq_len, int32_t pad, const int64_t *ridx, int32_t n,
                            float *out, float *act, void *stream) {
  LstmLayerPtrs P{};
  if (hidden != LH || !out || !act || !lstm_train_args(vocab, w_ih, w_hh, b_ih, b_hh, layers, tokens, seq_len, ridx, n, P)) {
    set_error("rnnl_lstm_train_forward: bad arguments (hidden 16, 1 <= layers <= 3, rules of <= 7 tokens, n >= 1)");
    return RNNL_ERR_INVALID;
  }
  hipLaunchKernelGGL(lstm_train_fwd_kernel, dim3(lstm_blocks(n)), dim3(256), 0, (hipStream_t)stream, vocab, P, tokens,
                     seq_len, pad, ridx, n, layers, out, act);
  RNNL_HIP_CHECK(hipGetLastError());
  return RNNL_OK;
}

int rnnl_lstm_train_backward(const float *vocab, const float *const *w_ih, const float *const *w_hh,
                             const float *const *b_ih, const float *const *b_hh, int32_t layers, int32_t hidden,
                             const int32_t *tokens, int32_t seq_len, int32_t pad, const int64_t *ridx, int32_t n,
                             const float *act, const float *d_out, float *da, float *xh, float *dvx,
                             const int32_t *tok_id, const int32_t *tok_ptr, const int32_t *tok_pos, int32_t n_tok,
                             float *d_vocab, int32_t vocab_rows, void *stream) {
  LstmLayerPtrs P{};
  if (hidden != LH || !act || !d_out || !da || !xh || !dvx || !d_vocab || n_tok < 0 || vocab_rows <= 0 ||
      (n_tok > 0 && (!tok_id || !tok_ptr || !tok_pos)) ||
      !lstm_train_args(vocab, w_ih, w_hh, b_ih, b_hh, layers, tokens, seq_len, ridx, n, P)) {
    set_error("rnnl_lstm_train_backward: bad arguments");
    return RNNL_ERR_INVALID;
  }
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(lstm_train_bwd_kernel, dim3(lstm_blocks(n)), dim3(256), 0, st, vocab, P, tokens, seq_len, pad,
                     ridx, n, layers, act, d_out, da, xh, dvx);
  RNNL_HIP_CHECK(hipMemsetAsync(d_vocab, 0, (size_t)vocab_rows * LH * sizeof(float), st));
  if (n_tok > 0)
    hipLaunchKernelGGL(vocab_grad_kernel, dim3((unsigned)((n_tok * LH + 255) / 256)), dim3(256), 0, st, dvx, tok_id,
                       tok_ptr, tok_pos, n_tok, d_vocab);
  RNNL_HIP_CHECK(hipGetLastError());
  return RNNL_OK;
}

int rnnl_lstm_weight_grads_scratch(int32_t layers, int64_t rows, size_t *part_floats) {
  if (layers < 1 || layers > LMAXL || rows < 0 || !part_floats) {
    set_error("rnnl_lstm_weight_grads_scratch: bad arguments");
    return RNNL_ERR_INVALID;
  }
  *part_floats = (size_t)wg_segments(rows) * layers * WG_COLS * LG;
  return RNNL_OK;
}

int rnnl_lstm_weight_grads(const float *da, const float *xh, int32_t layers, int64_t rows, float *part,
                           size_t part_floats, float *out, void *stream) {
  size_t need = 0;
  if (!da || !xh || !part || !out || rnnl_lstm_weight_grads_scratch(layers, rows, &need) != RNNL_OK ||
      part_floats < need || rows <= 0) {
    set_error("rnnl_lstm_weight_grads: bad arguments (rows >= 1, part: rnnl_lstm_weight_grads_scratch floats)");
    return RNNL_ERR_INVALID;
  }
  hipStream_t st = (hipStream_t)stream;
  const int64_t nseg = wg_segments(rows);
  hipLaunchKernelGGL(lstm_wgrad_part_kernel, dim3((unsigned)nseg, (unsigned)layers), dim3(256), 0, st, da, xh, rows,
                     part);
  const int total = layers * WG_COLS * LG;
  hipLaunchKernelGGL(lstm_wgrad_fold_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, part, layers,
                     nseg, out);
  RNNL_HIP_CHECK(hipGetLastError());
  return RNNL_OK;
}

}  // extern "C"
