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

}  // extern "C"
