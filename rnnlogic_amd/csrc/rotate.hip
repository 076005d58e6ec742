// RotatE entity feature + base-score fills for gfx950.
//
// rotate_score: score[q][e] (+)= gamma - sum_d sqrt(dre^2 + dim^2) with
//   (h o r)_d = (re_h re_r - im_h im_r, re_h im_r + im_h re_r),
//   (re_r, im_r) = (cos, sin)(remb[r][d] / ((gamma + 2) / D / pi))
// (reference src/embedding.py:28-70, forward at :64-70).
//
// Shape of the work: B queries x |E| entities x D complex dims, one sqrt per
// term inside the reduction.  The sqrt is a quarter-rate transcendental
// (8 issue cycles per wave64 instruction vs 2 for an FMA, measured with
// tools/micro/valu_rates.hip), so the VALU issue port is the bound: the
// kernel's job is to leave the VALU nothing but sqrt + accumulate.
//
// Weight-derived tables (built once per weight version, see RotatE in
// rnnlogic_amd/embedding.py):
//   etab [D][4][Ep]   per dim d and K group kg: the 4 bf16 B-operand slots
//                     (8 bytes) of every entity for the MFMA contraction
//                     below, built from the exact 3-part bf16 split of
//                     a = re, b = im and m = a^2 + b^2; Ep = |E| rounded up to
//                     256 and zero padded, so 16 lanes read 128 contiguous
//                     bytes and never need clamping;
//   rtab [R2][D][2]   (cos, sin) of every relation phase (R2 = 2 |R|, the
//                     second half negated, embedding.py:26).
#include <hip/hip_runtime.h>

#include "internal.h"

namespace rnnl {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// Diagnostic clock (rnnl_debug_clock): when set, thread 0 of every RotatE
// block adds its (shader-clock ticks, 100 MHz real-time ticks) into
// clk[0..1]; their ratio x 0.1 GHz is the effective clock under this load.
static unsigned long long *g_clk = nullptr;
struct ClockStamp {
  unsigned long long t0, r0;
  __device__ __forceinline__ void begin(const unsigned long long *clk) {
    if (clk && threadIdx.x == 0) {
      t0 = __builtin_amdgcn_s_memtime();
      r0 = __builtin_amdgcn_s_memrealtime();
    }
  }
  __device__ __forceinline__ void end(unsigned long long *clk) {
    if (clk && threadIdx.x == 0) {
      atomicAdd(&clk[0], __builtin_amdgcn_s_memtime() - t0);
      atomicAdd(&clk[1], __builtin_amdgcn_s_memrealtime() - r0);
    }
  }
};

__host__ __device__ constexpr int64_t ent_pad(int64_t E) { return (E + 255) / 256 * 256; }

// torch computes vec / (range / pi) in fp32 with the python-float divisor
// rounded to fp32 (embedding.py:57-58)
__device__ __forceinline__ float phase_div(float gamma, int D) {
  return (float)(((double)gamma + 2.0) / (double)D / 3.141592653589793238462643383279);
}

// (h o r)_d for one query row, rounded as torch evaluates it: two products
// then one difference/sum, no contraction (embedding.py:60-61)
__device__ __forceinline__ void rotate_head(const float *hrow, const float2 *rrow, int D, int d, float &re,
                                            float &im) {
  const float rh = hrow[d], ih = hrow[D + d];
  const float2 cs = rrow[d];
  re = __fsub_rn(__fmul_rn(rh, cs.x), __fmul_rn(ih, cs.y));
  im = __fadd_rn(__fmul_rn(rh, cs.y), __fmul_rn(ih, cs.x));
}

// XCD-aware tile order.  Blocks are dealt to the 8 XCDs round-robin by
// linear id; remap so each XCD walks its own contiguous slab of tiles, swept
// in super-rows of G query tiles x all entity tiles: the blocks resident on
// one XCD at a time then cover ~G query tiles x (resident / G) entity tiles,
// and both the entity table slices and the query rows are re-read from that
// XCD's L2 instead of MALL/HBM.  Only the speed depends on the placement.
constexpr int XCDS = 8;
constexpr int TILE_G = 16;
__device__ __forceinline__ bool xcd_tile(int nE, int nQ, int &et, int &qt, int64_t blk0 = 0) {
  const int64_t n = (int64_t)nE * nQ;
  const int64_t per = (n + XCDS - 1) / XCDS;
  const int64_t b = blk0 + blockIdx.x;  // blk0: a multiple of XCDS (one piece of a split launch)
  const int64_t v = (b % XCDS) * per + b / XCDS;
  if (v >= n) return false;
  const int64_t super = v / ((int64_t)TILE_G * nE);
  const int64_t w = v % ((int64_t)TILE_G * nE);
  const int g = (int)min<int64_t>(TILE_G, nQ - super * TILE_G);
  et = (int)(w / g);
  qt = (int)(super * TILE_G + w % g);
  return true;
}
static unsigned xcd_grid(int64_t nE, int64_t nQ) { return (unsigned)((nE * nQ + XCDS - 1) / XCDS * XCDS); }

// ---------------------------------------------------------------------------
// MFMA formulation (default).  For one dimension d the squared distance of
// every (query q, entity e) pair is a short contraction:
//   s = (hr_re - a)^2 + (hr_im - b)^2 = |hr|^2 + x a + y b + |t|^2,
//   x = -2 hr_re, y = -2 hr_im, |t|^2 = a^2 + b^2,
// evaluated by one v_mfma_f32_16x16x16_bf16 per 16 x 16 tile: every fp32
// operand is split exactly into three bf16 parts (v = v0 + v1 + v2, 8 + 8 + 8
// mantissa bits), the cross products keep the six part pairs i + j <= 2 (the
// dropped ones are below 2^-23 |x a|), |t|^2 rides on constant-1 slots and
// |hr|^2 is the fp32 accumulator input C.  16 K slots:
//   k  0..3   x0 a0 | x0 a1 | x0 a2 | x1 a0
//   k  4..7   x1 a1 | x2 a0 | y0 b0 | y0 b1
//   k  8..11  y0 b2 | y1 b0 | y1 b1 | y2 b0
//   k 12..15  1 m0  | 1 m1  | 1 m2  | 0
// The bf16 matrix pipe runs beside the VALU (the f32 MFMA shares the VALU's
// issue; tools/micro/valu_rates.hip: 13.1 vs 21.3 cycles per 64 terms), so
// the VALU keeps only sqrt(|s|) + accumulate per term (|s| absorbs a
// rounding-negative s at a near-zero distance; abs is a free modifier).
// Rounding: s carries the fp32 cancellation of the expanded form,
// ~2^-24 (|hr|^2 + |t|^2); DESIGN.md "RotatE numerics".
//
// Block = 64 queries x 256 entities (4 waves of 64 x 64: 16 tiles, 64
// accumulator VGPRs).  A fragments (8 B per lane) and C = |hr|^2 (4 rows per
// lane) are built per MDC-dim chunk in a double-buffered LDS image; B
// fragments (8 B per lane) come straight from the entity table, two dims
// ahead.
typedef short s16x4 __attribute__((ext_vector_type(4)));

constexpr int WQ = 4;    // 16-query tile rows per wave
constexpr int WE = 4;    // 16-entity tile columns per wave
constexpr int MQ = 16 * WQ;    // queries per block
constexpr int ME = 64 * WE;    // entities per block (4 waves side by side; divides 256)
constexpr int MDC = 8;  // dims per LDS chunk (unrolled; even)
constexpr int AST = 256 / MQ;  // A side: dims built per pass of the block
static_assert(MDC % 2 == 0 && MDC % AST == 0, "chunk shape");

__device__ __forceinline__ unsigned short bf16_bits(float v) {
  return __builtin_bit_cast(unsigned short, (__bf16)v);  // v_cvt_pk_bf16_f32 (RNE)
}
__device__ __forceinline__ float bf16_val(unsigned short h) { return __uint_as_float((unsigned)h << 16); }
// v = p0 + p1 + p2 exactly (each residual is exact by Sterbenz)
__device__ __forceinline__ void split3(float v, unsigned short p[3]) {
  p[0] = bf16_bits(v);
  const float r1 = v - bf16_val(p[0]);
  p[1] = bf16_bits(r1);
  p[2] = bf16_bits(r1 - bf16_val(p[1]));
}
__device__ __forceinline__ uint2 pack4(unsigned short a, unsigned short b, unsigned short c, unsigned short d) {
  return make_uint2(a | ((unsigned)b << 16), c | ((unsigned)d << 16));
}

__global__ __launch_bounds__(256, 1) void rotate_mfma_kernel(const float *__restrict__ eemb,
                                                          const uint2 *__restrict__ etab,
                                                          const float2 *__restrict__ rtab, int D, float gamma,
                                                          const int64_t *__restrict__ all_h,
                                                          const int64_t *__restrict__ all_r, int nq, int E,
                                                          float *__restrict__ score, int accumulate,
                                                          unsigned long long *clk) {
  __shared__ __attribute__((aligned(16))) uint2 sA[2][MDC][4][MQ];
  __shared__ __attribute__((aligned(16))) float sN[2][MDC][MQ];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int k = lane >> 4, i16 = lane & 15;
  const int64_t Ep = ent_pad(E);
  int et, qt;
  if (!xcd_tile((int)(Ep / ME), (nq + MQ - 1) / MQ, et, qt)) return;
  ClockStamp cs;
  cs.begin(clk);
  const int q0 = qt * MQ;
  const int e_base = et * ME + wave * 16 * WE;
  const int nchunk = (D + MDC - 1) / MDC;

  // ---- A side: this thread builds query row q0 + tid % MQ, dims tid / MQ + AST i of each chunk
  const int aq = tid % MQ, adw = tid / MQ;
  const bool avalid = q0 + aq < nq;
  const float *hrow = eemb;
  const float2 *rrow = rtab;
  if (avalid) {
    hrow = eemb + all_h[q0 + aq] * 2 * (int64_t)D;
    rrow = rtab + all_r[q0 + aq] * (int64_t)D;
  }
  float pre[MDC / AST], pim[MDC / AST];
  auto load_chunk = [&](int c) {
#pragma unroll
    for (int i = 0; i < MDC / AST; ++i) {
      const int d = c * MDC + adw + AST * i;
      pre[i] = pim[i] = 0.f;
      if (avalid && d < D) rotate_head(hrow, rrow, D, d, pre[i], pim[i]);
    }
  };
  auto store_chunk = [&](int c, int buf) {
#pragma unroll
    for (int i = 0; i < MDC / AST; ++i) {
      const int dd = adw + AST * i;
      const bool live = avalid && c * MDC + dd < D;
      unsigned short x[3], y[3];
      split3(-2.f * pre[i], x);
      split3(-2.f * pim[i], y);
      const unsigned short one = live ? 0x3f80 : 0;  // dead rows / dims: A = 0, C = 0, s = 0
      sA[buf][dd][0][aq] = pack4(x[0], x[0], x[0], x[1]);
      sA[buf][dd][1][aq] = pack4(x[1], x[2], y[0], y[0]);
      sA[buf][dd][2][aq] = pack4(y[0], y[1], y[1], y[2]);
      sA[buf][dd][3][aq] = pack4(one, one, one, 0);
      sN[buf][dd][aq] = fmaf(pre[i], pre[i], pim[i] * pim[i]);
    }
  };

  // ---- B side: lane (k, i16) loads k-group k of entity e_base + 16 g + i16, dim d
  const uint2 *bp = etab + k * Ep + e_base + i16;
  const int64_t dstride = 4 * Ep;
  uint2 vb[2][WE];  // ring: dim d lives in slot d & 1, reloaded with d + 2 once consumed
#pragma unroll
  for (int p = 0; p < 2; ++p)
#pragma unroll
    for (int g = 0; g < WE; ++g) vb[p][g] = bp[min(p, D - 1) * dstride + g * 16];

  f32x4 acc[WQ][WE];
#pragma unroll
  for (int qg = 0; qg < WQ; ++qg)
#pragma unroll
    for (int g = 0; g < WE; ++g) acc[qg][g] = (f32x4){0.f, 0.f, 0.f, 0.f};

  load_chunk(0);
  store_chunk(0, 0);
  for (int c = 0; c < nchunk; ++c) {
    __syncthreads();  // chunk c's image is complete; chunk c-1's buffer is free
    const int buf = c & 1;
    if (c + 1 < nchunk) load_chunk(c + 1);  // global loads in flight under the compute
    // dims past D in the last chunk: A and C are zero there, so s = 0 adds sqrt(0)
#pragma unroll
    for (int dd = 0; dd < MDC; ++dd) {
      const int slot = dd & 1;  // MDC is even: slot of dim c*MDC + dd
      s16x4 b[WE];
#pragma unroll
      for (int g = 0; g < WE; ++g) b[g] = __builtin_bit_cast(s16x4, vb[slot][g]);
      const int dn = min(c * MDC + dd + 2, D - 1);
#pragma unroll
      for (int g = 0; g < WE; ++g) vb[slot][g] = bp[dn * dstride + g * 16];
#pragma unroll
      for (int qg = 0; qg < WQ; ++qg) {
        const s16x4 a = __builtin_bit_cast(s16x4, sA[buf][dd][k][qg * 16 + i16]);
        const f32x4 cn = *reinterpret_cast<const f32x4 *>(&sN[buf][dd][qg * 16 + k * 4]);
#pragma unroll
        for (int g = 0; g < WE; ++g) {
          const f32x4 s = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b[g], cn, 0, 0, 0);
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[qg][g][j] += __builtin_amdgcn_sqrtf(__builtin_fabsf(s[j]));
        }
      }
      // keep the unrolled dims apart: the accumulators are complete here and
      // the next dim's LDS/global reads stay below (memory clobber), so its
      // MFMAs cannot be hoisted — hoisting every MFMA of the chunk first
      // needs MDC x the result registers and spills
#pragma unroll
      for (int qg = 0; qg < WQ; ++qg)
#pragma unroll
        for (int g = 0; g < WE; ++g) asm volatile("" ::"v"(acc[qg][g]) : "memory");
    }
    if (c + 1 < nchunk) store_chunk(c + 1, buf ^ 1);
  }
  cs.end(clk);
  // D layout: lane holds entity column i16 of group g, query rows 4k + j of group qg
#pragma unroll
  for (int qg = 0; qg < WQ; ++qg)
#pragma unroll
    for (int g = 0; g < WE; ++g)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int q = q0 + qg * 16 + k * 4 + j;
        const int e = e_base + g * 16 + i16;
        if (q < nq && e < E) {
          const int64_t idx = (int64_t)q * E + e;
          const float val = gamma - acc[qg][g][j];
          if (accumulate == 2)
            unsafeAtomicAdd(score + idx, val);
          else
            score[idx] = accumulate ? score[idx] + val : val;
        }
      }
}

// ---------------------------------------------------------------------------
// Direct formulation (mode RNNL_ROTATE_DIRECT, the default): the reference's
// arithmetic term by term — (hr_re - a), (hr_im - b), sqrt of the sum of
// squares — on the VALU, so no cancellation beyond the reference's own
// rounding.  Each lane owns one entity; a wave owns DQ = 20 queries whose
// h o r values for the current dim are wave-uniform and come in as SGPR
// operands (s_load from the per-call hr workspace, built by rotate_hr_kernel)
// — per term the VALU issues exactly sub, sub, mul, fma, sqrt, add.
// Sums are kept per DCH-dim chunk and folded into the row total, which keeps
// the fp32 summation error of a 1000-term row near the reference's.  Entity
// values come LCH = 2 dims at a time into fixed register slots, one block
// ahead.  DQ = 20 / LCH = 2 measured best (75 ms vs 88 ms for 16 / 1 on the
// FB15k-237 bench shape): more terms per dim amortise the per-dim loads and
// address work, at 5 waves per SIMD.
constexpr int RB = 256;   // entities per block (one per lane)
constexpr int DQ = 20;  // queries per block (SGPR-resident)
constexpr int DCH = 32;   // dims per partial sum
constexpr int LCH = 2;  // dims per entity-value prefetch block (divides DCH)

// hr[g][d][0..DQ-1 | DQ..2DQ-1] = (re | im) of (h o r)_d for queries DQ g + k.
// One block per (query group, 64 dims): entity rows read coalesced along d,
// the group's 64 x 2DQ slab transposed in LDS and written contiguously.
__global__ __launch_bounds__(256) void rotate_hr_kernel(const float *__restrict__ eemb,
                                                        const float2 *__restrict__ rtab, int D,
                                                        const int64_t *__restrict__ all_h,
                                                        const int64_t *__restrict__ all_r, int nq,
                                                        float *__restrict__ hr) {
  __shared__ float s_re[64][DQ + 1], s_im[64][DQ + 1];
  const int g = blockIdx.x, d0 = blockIdx.y * 64;
  const int dl = threadIdx.x & 63, nd = min(64, D - d0);
  for (int k = threadIdx.x >> 6; k < DQ; k += 4) {
    const int q = g * DQ + k;
    float re = 0.f, im = 0.f;
    if (q < nq && dl < nd)
      rotate_head(eemb + all_h[q] * 2 * (int64_t)D, rtab + all_r[q] * (int64_t)D, D, d0 + dl, re, im);
    s_re[dl][k] = re;
    s_im[dl][k] = im;
  }
  __syncthreads();
  float *out = hr + ((int64_t)g * D + d0) * 2 * DQ;
  for (int j = threadIdx.x; j < nd * 2 * DQ; j += 256) {
    const int d = j / (2 * DQ), w = j % (2 * DQ);
    out[j] = w < DQ ? s_re[d][w] : s_im[d][w - DQ];
  }
}

constexpr int ROT_QW = 1;              // query groups per block (divides RB / 64)
constexpr int ROT_RE = RB / ROT_QW;    // entities per block
static_assert(ROT_RE % 64 == 0 && 256 % ROT_RE == 0, "whole waves per query group; ent_pad divisible");
__global__ __launch_bounds__(RB) void rotate_direct_kernel(const float *__restrict__ ptab,
                                                           const float *__restrict__ hr, int D, float gamma,
                                                           int nq, int E, float *__restrict__ score,
                                                           int accumulate, unsigned long long *clk, int64_t blk0) {
  const int64_t Ep = ent_pad(E);
  int et, qt;
  const int ngroups = (nq + DQ - 1) / DQ;
  if (!xcd_tile((int)(Ep / ROT_RE), (ngroups + ROT_QW - 1) / ROT_QW, et, qt, blk0)) return;
  // ROT_QW query groups per block, one per wave row, over the same ROT_RE
  // entities (their entity-plane loads meet in L1)
  qt = __builtin_amdgcn_readfirstlane(qt * ROT_QW + (int)threadIdx.x / ROT_RE);  // wave-uniform: SGPR h o r operands
  if (qt >= ngroups) return;  // wave-uniform; the kernel has no barrier
  ClockStamp cs;
  cs.begin(clk);
  const int e = et * ROT_RE + (int)threadIdx.x % ROT_RE;  // < Ep: the table is padded
  const int q0 = qt * DQ;
  const float *hp = hr + (int64_t)qt * D * 2 * DQ;
  const float *ap = ptab + e;
  // software pipeline: the sqrt of dim d runs one dim later than its
  // squared distance (a VALU result feeding v_sqrt directly costs ~6 more
  // cycles per term; tools/micro/valu_rates.hip "direct pipelined")
  float acc[DQ], sq[DQ];
#pragma unroll
  for (int k = 0; k < DQ; ++k) acc[k] = sq[k] = 0.f;
  // entity values: LCH dims at a time, loaded one LCH-block ahead (fixed
  // register slots per dim, so the prefetch never waits on a rotation)
  float va[LCH], vb[LCH], na[LCH], nb[LCH];
#pragma unroll
  for (int j = 0; j < LCH; ++j) {
    const int64_t d = min(j, D - 1);
    va[j] = ap[d * 2 * Ep];
    vb[j] = ap[d * 2 * Ep + Ep];
  }
  for (int d0 = 0; d0 < D; d0 += DCH) {
    float part[DQ];
#pragma unroll
    for (int k = 0; k < DQ; ++k) part[k] = 0.f;
    for (int d1 = d0; d1 < min(d0 + DCH, D); d1 += LCH) {
#pragma unroll
      for (int j = 0; j < LCH; ++j) {
        const int64_t d = min(d1 + LCH + j, D - 1);
        na[j] = ap[d * 2 * Ep];
        nb[j] = ap[d * 2 * Ep + Ep];
      }
#pragma unroll
      for (int j = 0; j < LCH; ++j) {
        const int d = d1 + j;
        if (d < D) {  // wave-uniform
          const float a = va[j], b = vb[j];
          const float *h = hp + (int64_t)d * 2 * DQ;  // wave-uniform: s_load
#pragma unroll
          for (int k = 0; k < DQ; ++k) {
            part[k] += __builtin_amdgcn_sqrtf(sq[k]);  // dim d - 1 (sqrt(0) = 0 before the first)
            const float x = h[k] - a;
            const float y = h[DQ + k] - b;
            sq[k] = fmaf(x, x, y * y);
          }
        }
      }
#pragma unroll
      for (int j = 0; j < LCH; ++j) {
        va[j] = na[j];
        vb[j] = nb[j];
      }
    }
#pragma unroll
    for (int k = 0; k < DQ; ++k) acc[k] += part[k];
  }
#pragma unroll
  for (int k = 0; k < DQ; ++k) acc[k] += __builtin_amdgcn_sqrtf(sq[k]);  // v_sqrt_f32 (1 ulp)
  cs.end(clk);
  if (e < E) {
#pragma unroll
    for (int k = 0; k < DQ; ++k) {
      if (q0 + k < nq) {
        const int64_t idx = (int64_t)(q0 + k) * E + e;
        const float v = gamma - acc[k];
        if (accumulate == 2)  // into a zeroed matrix beside deferred scoring adds (rnnl_rotate_score)
          unsafeAtomicAdd(score + idx, v);
        else
          score[idx] = accumulate ? score[idx] + v : v;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Split-dimension form of rotate_direct_kernel for launches with few rows
// (e.g. one 32-row reference batch per call, trainer.py:150-173): there the
// (query group x entity tile) grid has ~100 blocks and each wave walks all D
// dims alone — latency-bound (525 us for 32 rows x 14,541 entities x 1000
// dims on FB15k-237, vs 64 us at the full-split rate).  Here the DCH-dim
// chunks are dealt to `groups` blocks per tile: each wave computes, for its
// DQ queries and 64 entities, every chunk sum of its chunk range exactly as
// rotate_direct_kernel does (the same sub, sub, mul, fma, sqrt per term, the
// same sequential adds within a chunk, the sqrt of a dim added in the next
// dim's step) and stores it; rotate_combine_kernel then folds the chunk sums
// into the row total in chunk order and adds the last dim's sqrt — the same
// fp32 operations in the same order, so the scores are bitwise those of
// rotate_direct_kernel.  parts layout: [nchunks + 1][nq][E].
__global__ __launch_bounds__(RB) void rotate_split_kernel(const float *__restrict__ ptab,
                                                          const float *__restrict__ hr, int D, int nq, int E,
                                                          int chunks_per_group, float *__restrict__ parts) {
  const int64_t Ep = ent_pad(E);
  const int n_et = (int)(Ep / RB);
  const int ngroups_q = (nq + DQ - 1) / DQ;
  const int nchunks = (D + DCH - 1) / DCH;
  // block -> (chunk group, query group, entity tile): entity tiles fastest,
  // so the blocks of one dim range share their slice of the entity planes
  int b = blockIdx.x;
  const int et = b % n_et;
  b /= n_et;
  const int qt = __builtin_amdgcn_readfirstlane(b % ngroups_q);
  const int cg = __builtin_amdgcn_readfirstlane(b / ngroups_q);
  const int c0 = cg * chunks_per_group, c1 = min(nchunks, c0 + chunks_per_group);
  if (c0 >= nchunks) return;  // block-uniform; no barrier in the kernel
  const int e = et * RB + (int)threadIdx.x;  // < Ep: the table is padded
  const int q0 = qt * DQ;
  const float *hp = hr + (int64_t)qt * D * 2 * DQ;
  const float *ap = ptab + e;
  float sq[DQ];
#pragma unroll
  for (int k = 0; k < DQ; ++k) sq[k] = 0.f;
  if (c0 > 0) {  // the pipeline's carried value: the previous chunk's last dim
    const int d = c0 * DCH - 1;
    const float a = ap[(int64_t)d * 2 * Ep], bb = ap[(int64_t)d * 2 * Ep + Ep];
    const float *h = hp + (int64_t)d * 2 * DQ;
#pragma unroll
    for (int k = 0; k < DQ; ++k) {
      const float x = h[k] - a;
      const float y = h[DQ + k] - bb;
      sq[k] = fmaf(x, x, y * y);
    }
  }
  const int64_t plane = (int64_t)nq * E;
  for (int c = c0; c < c1; ++c) {
    float part[DQ];
#pragma unroll
    for (int k = 0; k < DQ; ++k) part[k] = 0.f;
    for (int d = c * DCH; d < min(c * DCH + DCH, D); ++d) {
      const float a = ap[(int64_t)d * 2 * Ep], bb = ap[(int64_t)d * 2 * Ep + Ep];
      const float *h = hp + (int64_t)d * 2 * DQ;  // wave-uniform: s_load
#pragma unroll
      for (int k = 0; k < DQ; ++k) {
        part[k] += __builtin_amdgcn_sqrtf(sq[k]);
        const float x = h[k] - a;
        const float y = h[DQ + k] - bb;
        sq[k] = fmaf(x, x, y * y);
      }
    }
    if (e < E) {
#pragma unroll
      for (int k = 0; k < DQ; ++k)
        if (q0 + k < nq) parts[(int64_t)c * plane + (int64_t)(q0 + k) * E + e] = part[k];
    }
  }
  if (c1 == nchunks && e < E) {  // the last dim's sqrt, added after the chunk sums
#pragma unroll
    for (int k = 0; k < DQ; ++k)
      if (q0 + k < nq) parts[(int64_t)nchunks * plane + (int64_t)(q0 + k) * E + e] = __builtin_amdgcn_sqrtf(sq[k]);
  }
}

__global__ __launch_bounds__(256) void rotate_combine_kernel(const float *__restrict__ parts, int nchunks, int nq,
                                                             int E, float gamma, float *__restrict__ score,
                                                             int accumulate) {
  const int64_t n = (int64_t)nq * E;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float acc = 0.f;
    for (int c = 0; c < nchunks; ++c) acc += parts[(int64_t)c * n + i];
    acc += parts[(int64_t)nchunks * n + i];
    const float v = gamma - acc;
    if (accumulate == 2)
      unsafeAtomicAdd(score + i, v);
    else
      score[i] = accumulate ? score[i] + v : v;
  }
}

// Chunk groups of the split form for a launch (1: the one-pass direct kernel):
// when the (query group x entity tile) grid is below ~1,024 blocks, deal the
// chunks to enough groups for ~2,048 blocks, capped so the chunk sums stay
// within 512 MB.
static int split_groups(int64_t nq, int64_t E, int D) {
  const int64_t base = (ent_pad(E) / RB) * ((nq + DQ - 1) / DQ);
  const int nchunks = (D + DCH - 1) / DCH;
  if (base >= 1024 || nchunks < 2) return 1;
  if ((int64_t)(nchunks + 1) * nq * E * 4 > (int64_t)512 << 20) return 1;
  int groups = (int)std::min<int64_t>(nchunks, (2048 + base - 1) / base);
  const int cpg = (nchunks + groups - 1) / groups;
  return (nchunks + cpg - 1) / cpg;
}

// ---------------------------------------------------------------------------
// Table builders (once per weight version)

// etab[d][kg][e] from eemb[e][2D]: 32 entities x 32 dims per tile through
// LDS, so both the row reads and the table writes are coalesced.
__global__ void entity_table_kernel(const float *__restrict__ eemb, int E, int D, uint2 *__restrict__ etab) {
  __shared__ float ta[32][33], tb[32][33];
  const int d0 = blockIdx.x * 32, e0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 256 threads: 32 x 8
  const int64_t Ep = ent_pad(E);
  for (int j = ty; j < 32; j += 8) {
    const int e = e0 + j, d = d0 + tx;
    const bool in = e < E && d < D;
    ta[j][tx] = in ? eemb[(int64_t)e * 2 * D + d] : 0.f;
    tb[j][tx] = in ? eemb[(int64_t)e * 2 * D + D + d] : 0.f;
  }
  __syncthreads();
  for (int j = ty; j < 32; j += 8) {
    const int d = d0 + j, e = e0 + tx;
    if (d < D && e < Ep) {
      const float a = ta[tx][j], b = tb[tx][j];
      unsigned short pa[3], pb[3], pm[3];
      split3(a, pa);
      split3(b, pb);
      split3(fmaf(a, a, b * b), pm);
      uint2 *col = etab + (int64_t)d * 4 * Ep + e;
      col[0] = pack4(pa[0], pa[1], pa[2], pa[0]);
      col[Ep] = pack4(pa[1], pa[0], pb[0], pb[1]);
      col[2 * Ep] = pack4(pb[2], pb[0], pb[1], pb[0]);
      col[3 * Ep] = pack4(pm[0], pm[1], pm[2], 0);
    }
  }
}

// ptab[d][0 | 1][e] = re | im of every entity (direct mode), same tiling
__global__ void plane_table_kernel(const float *__restrict__ eemb, int E, int D, float *__restrict__ ptab) {
  __shared__ float ta[32][33], tb[32][33];
  const int d0 = blockIdx.x * 32, e0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const int64_t Ep = ent_pad(E);
  for (int j = ty; j < 32; j += 8) {
    const int e = e0 + j, d = d0 + tx;
    const bool in = e < E && d < D;
    ta[j][tx] = in ? eemb[(int64_t)e * 2 * D + d] : 0.f;
    tb[j][tx] = in ? eemb[(int64_t)e * 2 * D + D + d] : 0.f;
  }
  __syncthreads();
  for (int j = ty; j < 32; j += 8) {
    const int d = d0 + j, e = e0 + tx;
    if (d < D && e < Ep) {
      ptab[(int64_t)d * 2 * Ep + e] = ta[tx][j];
      ptab[(int64_t)d * 2 * Ep + Ep + e] = tb[tx][j];
    }
  }
}

__global__ void relation_table_kernel(const float *__restrict__ remb, int64_t n, int D, float gamma,
                                      float2 *__restrict__ rtab) {
  const float div = phase_div(gamma, D);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float ph = remb[i] / div;
    rtab[i] = make_float2(cosf(ph), sinf(ph));
  }
}

__global__ void fill_rows_kernel(const float *__restrict__ row, int nq, int E, float *__restrict__ out) {
  const int64_t n = (int64_t)nq * E;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = row[i % E];
}

__global__ void fill_value_kernel(float v, int64_t n, float *__restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = v;
}

static unsigned grid_for(int64_t n) { return (unsigned)std::min<int64_t>((n + 255) / 256, 256 * 16); }

}  // namespace rnnl

using namespace rnnl;

// ------------------------------------------------------------ backward (training)
// Gradient of score[q][e] = gamma - sum_d |hr[q][d] - t[e][d]| (complex
// entries; embedding.py:45-70, torch.norm's backward with grad 0 at a zero
// norm) for the incoming grad g (B x E):
//   d_tail[e][d] = sum_q g[q][e] (hr - t) / |hr - t|   (both parts)
//   d_hr[q][d]  -= sum_e g[q][e] (hr - t) / |hr - t|
// One thread per (entity, dim) for BW_EPT entities (stride 256, coalesced over
// the transposed entity planes [D][2][ld]); the per-query sums over entities
// are reduce-scattered over the wave (63 shuffles for 32 queries x 2 parts),
// then over the block's waves in LDS, then per (block, q, part) one value:
// into d_hr_part[block][q][part D + d] (rnnl_rotate_param_grads: summed over
// the blocks in block order by head_grad_kernel — deterministic) or, without
// a partial buffer (rnnl_rotate_backward), one atomicAdd into d_hr.
constexpr int BW_EPT = 4;
constexpr int BW_BS = 256;

__global__ __launch_bounds__(BW_BS) void rotate_backward_kernel(const float *__restrict__ planes, int ld,
                                                                const float *__restrict__ hr,
                                                                const float *__restrict__ g, int B, int E, int D,
                                                                float *__restrict__ d_hr,
                                                                float *__restrict__ d_hr_part,
                                                                float *__restrict__ d_tail) {
  __shared__ float s_red[BW_BS / 64][64];
  const int d = blockIdx.y;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int e0 = blockIdx.x * (BW_BS * BW_EPT) + threadIdx.x;
  float a[BW_EPT], b[BW_EPT], ta[BW_EPT], tb[BW_EPT];
#pragma unroll
  for (int k = 0; k < BW_EPT; ++k) {
    const int e = e0 + k * BW_BS;
    a[k] = e < E ? planes[(int64_t)(2 * d) * ld + e] : 0.f;
    b[k] = e < E ? planes[(int64_t)(2 * d + 1) * ld + e] : 0.f;
    ta[k] = tb[k] = 0.f;
  }
  for (int q0 = 0; q0 < B; q0 += 32) {
    float v[64];  // v[j] = sum over this thread's entities of w x (query q0 + j), v[32 + j] = w y
#pragma unroll
    for (int j = 0; j < 32; ++j) {
      float sx = 0.f, sy = 0.f;
      const int q = q0 + j;
      if (q < B) {  // uniform
        const float hre = hr[(int64_t)q * 2 * D + d], him = hr[(int64_t)q * 2 * D + D + d];
#pragma unroll
        for (int k = 0; k < BW_EPT; ++k) {
          const int e = e0 + k * BW_BS;
          if (e < E) {
            const float x = hre - a[k], y = him - b[k];
            const float s = fmaf(x, x, y * y);
            // g / |hr - t| as g x rsq(s) (v_rsq_f32, 1 ulp): the correctly
            // rounded sqrt + divide sequence was ~60 % of the kernel's VALU
            const float w = s > 0.f ? g[(int64_t)q * E + e] * __builtin_amdgcn_rsqf(s) : 0.f;
            sx = fmaf(w, x, sx);
            sy = fmaf(w, y, sy);
            ta[k] = fmaf(w, x, ta[k]);
            tb[k] = fmaf(w, y, tb[k]);
          }
        }
      }
      v[j] = sx;
      v[32 + j] = sy;
    }
    // reduce-scatter over the wave: lane L ends with the wave's total of v[L]
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
      const bool up = (lane & m) != 0;
#pragma unroll
      for (int o = 0; o < m; ++o) {
        const float keep = up ? v[o + m] : v[o];
        const float give = up ? v[o] : v[o + m];
        v[o] = keep + __shfl_xor(give, m, 64);
      }
    }
    s_red[wave][lane] = v[0];
    __syncthreads();
    if (wave == 0) {
      float t = 0.f;
#pragma unroll
      for (int w2 = 0; w2 < BW_BS / 64; ++w2) t += s_red[w2][lane];
      const int q = q0 + (lane & 31);
      const int64_t j = (int64_t)q * 2 * D + (lane < 32 ? d : D + d);
      if (q < B) {
        if (d_hr_part)
          d_hr_part[(int64_t)blockIdx.x * B * 2 * D + j] = -t;
        else
          atomicAdd(&d_hr[j], -t);
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int k = 0; k < BW_EPT; ++k) {
    const int e = e0 + k * BW_BS;
    if (d_tail && e < E) {  // d_tail == nullptr: the entity table is frozen
      d_tail[(int64_t)(2 * d) * E + e] = ta[k];
      d_tail[(int64_t)(2 * d + 1) * E + e] = tb[k];
    }
  }
}

namespace rnnl {

// hr[q][d | D + d] = re | im of (h o r)_d (rotate_head: the forward's rounding)
__global__ void hr_rows_kernel(const float *__restrict__ eemb, const float2 *__restrict__ rtab, int D,
                               const int64_t *__restrict__ all_h, const int64_t *__restrict__ all_r,
                               float *__restrict__ hr) {
  const int q = blockIdx.y, d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= D) return;
  float re, im;
  rotate_head(eemb + all_h[q] * 2 * (int64_t)D, rtab + all_r[q] * (int64_t)D, D, d, re, im);
  hr[(int64_t)q * 2 * D + d] = re;
  hr[(int64_t)q * 2 * D + D + d] = im;
}

// d(h o r) = the sum of rotate_backward_kernel's per-entity-block partials,
// in block order (one thread per (row, part, dim); the partial rows are
// coalesced along the dims)
__global__ void hr_fold_kernel(const float *__restrict__ parts, int nparts, int64_t n, float *__restrict__ d_hr) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float t = 0.f;
    for (int b = 0; b < nparts; ++b) t += parts[(int64_t)b * n + i];
    d_hr[i] = t;
  }
}

// d_eemb[e][part D + d] = d_tail[2 d + part][e]: 32 x 32 tiles through LDS
// (the transposing copy torch's permute().reshape() made at ~1 TB/s)
__global__ void tail_rows_kernel(const float *__restrict__ d_tail, int E, int D, float *__restrict__ d_eemb) {
  __shared__ float ta[32][33], tb[32][33];
  const int d0 = blockIdx.x * 32, e0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int j = ty; j < 32; j += 8) {
    const int d = d0 + j, e = e0 + tx;
    const bool in = d < D && e < E;
    ta[j][tx] = in ? d_tail[(int64_t)(2 * d) * E + e] : 0.f;
    tb[j][tx] = in ? d_tail[(int64_t)(2 * d + 1) * E + e] : 0.f;
  }
  __syncthreads();
  for (int j = ty; j < 32; j += 8) {
    const int e = e0 + j, d = d0 + tx;
    if (e < E && d < D) {
      d_eemb[(int64_t)e * 2 * D + d] = ta[tx][j];
      d_eemb[(int64_t)e * 2 * D + D + d] = tb[tx][j];
    }
  }
}

// The chain rule from d(h o r) to the head rows of eemb and to remb
// (embedding.py:55-61: phase = remb[r] / div, (cos, sin) of the phase, the
// complex product), one thread per dim, the rows in order (deterministic
// sums where a head entity or relation repeats in the batch):
//   d re_h = g_re c + g_im s          d im_h = g_im c - g_re s
//   d c = g_re re_h + g_im im_h       d s = g_im re_h - g_re im_h
//   d remb[r][d] += (d s c - d c s) / div
__global__ void head_grad_kernel(const float *__restrict__ eemb, const float2 *__restrict__ rtab, int D, float gamma,
                                 const int64_t *__restrict__ all_h, const int64_t *__restrict__ all_r, int nq,
                                 const float *__restrict__ d_hr, float *__restrict__ d_eemb,
                                 float *__restrict__ d_remb) {
  const int d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= D) return;
  const float div = phase_div(gamma, D);
  for (int q = 0; q < nq; ++q) {
    const int64_t h = all_h[q], r = all_r[q];
    const float rh = eemb[h * 2 * D + d], ih = eemb[h * 2 * D + D + d];
    const float2 cs = rtab[r * D + d];
    const float gre = d_hr[(int64_t)q * 2 * D + d], gim = d_hr[(int64_t)q * 2 * D + D + d];
    if (d_eemb) {
      d_eemb[h * 2 * D + d] += gre * cs.x + gim * cs.y;
      d_eemb[h * 2 * D + D + d] += gim * cs.x - gre * cs.y;
    }
    if (d_remb) {
      const float dc = gre * rh + gim * ih, ds = gim * rh - gre * ih;
      d_remb[r * D + d] += (ds * cs.x - dc * cs.y) / div;
    }
  }
}

}  // namespace rnnl

extern "C" {

int rnnl_fill_rows(const float *row, int32_t nq, int32_t E, float *score, void *stream) {
  if (!row || !score || nq < 0 || E <= 0) {
    set_error("rnnl_fill_rows: bad arguments");
    return RNNL_ERR_INVALID;
  }
  const int64_t n = (int64_t)nq * E;
  if (n == 0) return RNNL_OK;
  hipLaunchKernelGGL(fill_rows_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, row, nq, E, score);
  RNNL_HIP_CHECK(hipGetLastError());
  return RNNL_OK;
}

int rnnl_fill_value(float v, int64_t n, float *score, void *stream) {
  if (!score || n < 0) {
    set_error("rnnl_fill_value: bad arguments");
    return RNNL_ERR_INVALID;
  }
  if (n == 0) return RNNL_OK;
  hipLaunchKernelGGL(fill_value_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, v, n, score);
  RNNL_HIP_CHECK(hipGetLastError());
  return RNNL_OK;
}

int rnnl_debug_clock(void *dev_counters) {
  g_clk = static_cast<unsigned long long *>(dev_counters);
  return RNNL_OK;
}

static bool valid_mode(int32_t mode) { return mode == RNNL_ROTATE_DIRECT || mode == RNNL_ROTATE_MFMA; }

int rnnl_rotate_table_sizes(int32_t E, int32_t D, int32_t n_rel_total, int32_t mode, size_t *entity_bytes,
                            size_t *relation_bytes) {
  if (E <= 0 || D <= 0 || n_rel_total <= 0 || !valid_mode(mode) || !entity_bytes || !relation_bytes) {
    set_error("rnnl_rotate_table_sizes: bad arguments");
    return RNNL_ERR_INVALID;
  }
  *entity_bytes = mode == RNNL_ROTATE_MFMA ? (size_t)4 * D * ent_pad(E) * sizeof(uint2)
                                           : (size_t)2 * D * ent_pad(E) * sizeof(float);
  *relation_bytes = (size_t)n_rel_total * D * 2 * sizeof(float);
  return RNNL_OK;
}

int rnnl_rotate_entity_table(const float *eemb, int32_t E, int32_t D, int32_t mode, void *etab, void *stream) {
  if (!eemb || !etab || E <= 0 || D <= 0 || !valid_mode(mode)) {
    set_error("rnnl_rotate_entity_table: bad arguments");
    return RNNL_ERR_INVALID;
  }
  const dim3 grid((D + 31) / 32, (unsigned)(ent_pad(E) / 32));
  if (mode == RNNL_ROTATE_MFMA)
    hipLaunchKernelGGL(entity_table_kernel, grid, dim3(256), 0, (hipStream_t)stream, eemb, E, D, (uint2 *)etab);
  else
    hipLaunchKernelGGL(plane_table_kernel, grid, dim3(256), 0, (hipStream_t)stream, eemb, E, D, (float *)etab);
  RNNL_HIP_CHECK(hipGetLastError());
  return RNNL_OK;
}

int rnnl_rotate_relation_table(const float *remb, int32_t n_rel_total, int32_t D, float gamma, float *rtab,
                               void *stream) {
  if (!remb || !rtab || n_rel_total <= 0 || D <= 0) {
    set_error("rnnl_rotate_relation_table: bad arguments");
    return RNNL_ERR_INVALID;
  }
  const int64_t n = (int64_t)n_rel_total * D;
  hipLaunchKernelGGL(relation_table_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, remb, n, D,
                     gamma, (float2 *)rtab);
  RNNL_HIP_CHECK(hipGetLastError());
  return RNNL_OK;
}

// hr slabs, then (split form only) the chunk sums, 256-byte aligned
static size_t hr_bytes(int64_t nq, int D) { return (size_t)((nq + DQ - 1) / DQ) * D * 2 * DQ * sizeof(float); }

int rnnl_rotate_workspace_size(int32_t nq, int32_t E, int32_t D, int32_t mode, size_t *bytes) {
  if (nq < 0 || E <= 0 || D <= 0 || !valid_mode(mode) || !bytes) {
    set_error("rnnl_rotate_workspace_size: bad arguments");
    return RNNL_ERR_INVALID;
  }
  if (mode != RNNL_ROTATE_DIRECT) {
    *bytes = 0;
    return RNNL_OK;
  }
  size_t b = (hr_bytes(nq, D) + 255) / 256 * 256;
  if (split_groups(nq, E, D) > 1) b += (size_t)((D + DCH - 1) / DCH + 1) * nq * E * sizeof(float);
  *bytes = b;
  return RNNL_OK;
}

int rnnl_rotate_score(const float *eemb, const void *etab, const float *rtab, int32_t D, float gamma,
                      const int64_t *all_h, const int64_t *all_r, int32_t nq, int32_t E, float *score,
                      int32_t accumulate, int32_t mode, void *workspace, size_t ws_bytes, void *stream) {
  return rnnl_rotate_score_pieces(eemb, etab, rtab, D, gamma, all_h, all_r, nq, E, score, accumulate, mode, workspace,
                                  ws_bytes, 1, 0.f, stream);
}

int rnnl_rotate_score_pieces(const float *eemb, const void *etab, const float *rtab, int32_t D, float gamma,
                             const int64_t *all_h, const int64_t *all_r, int32_t nq, int32_t E, float *score,
                             int32_t accumulate, int32_t mode, void *workspace, size_t ws_bytes, int32_t pieces_req,
                             float first_share, void *stream) {
  if (!eemb || !etab || !rtab || !all_h || !all_r || !score || D <= 0 || E <= 0 || nq < 0 || !valid_mode(mode) ||
      accumulate < 0 || accumulate > 2 || pieces_req < 1 || !(first_share >= 0.f && first_share < 1.f)) {
    set_error("rnnl_rotate_score: bad arguments");
    return RNNL_ERR_INVALID;
  }
  if (nq == 0) return RNNL_OK;
  if (mode == RNNL_ROTATE_DIRECT) {
    size_t need = 0;
    rnnl_rotate_workspace_size(nq, E, D, mode, &need);
    if (!workspace || ws_bytes < need) {
      set_error("rnnl_rotate_score: workspace too small (see rnnl_rotate_workspace_size)");
      return RNNL_ERR_INVALID;
    }
    hipLaunchKernelGGL(rotate_hr_kernel, dim3((unsigned)((nq + DQ - 1) / DQ), (unsigned)((D + 63) / 64)), dim3(256), 0,
                       (hipStream_t)stream, eemb,
                       (const float2 *)rtab, D, all_h, all_r, nq, (float *)workspace);
    RNNL_HIP_CHECK(hipGetLastError());
    const int groups = split_groups(nq, E, D);
    if (groups > 1) {  // few rows: chunk sums over more blocks, then the in-order fold
      const int nchunks = (D + DCH - 1) / DCH, cpg = (nchunks + groups - 1) / groups;
      float *parts = reinterpret_cast<float *>(static_cast<unsigned char *>(workspace) +
                                               (hr_bytes(nq, D) + 255) / 256 * 256);
      const int64_t nblk = (ent_pad(E) / RB) * ((nq + DQ - 1) / DQ) * groups;
      hipLaunchKernelGGL(rotate_split_kernel, dim3((unsigned)nblk), dim3(RB), 0, (hipStream_t)stream,
                         (const float *)etab, (const float *)workspace, D, nq, E, cpg, parts);
      hipLaunchKernelGGL(rotate_combine_kernel, dim3(grid_for((int64_t)nq * E)), dim3(256), 0, (hipStream_t)stream,
                         (const float *)parts, nchunks, nq, E, gamma, score, accumulate);
      RNNL_HIP_CHECK(hipGetLastError());
      return RNNL_OK;
    }
    // pieces > 1: the grid in back-to-back launches over consecutive block
    // ranges (the first one `first_share` of the blocks, 0 = equal pieces) —
    // the same blocks and the same per-element arithmetic, so the scores are
    // bitwise those of one launch.  Each launch boundary drains RotatE's
    // waves once: side-stream workgroups that wait for registers RotatE's
    // waves hold (the 168-VGPR PNA scoring pass) become resident there
    // (DESIGN §3.7).
    const int64_t total = xcd_grid(ent_pad(E) / ROT_RE, ((nq + DQ - 1) / DQ + ROT_QW - 1) / ROT_QW);
    const float share = first_share;
    const int pieces = (int)std::max<int64_t>(1, std::min<int64_t>(pieces_req, total / (64 * XCDS)));
    int64_t step = (total / pieces + XCDS - 1) / XCDS * XCDS;
    int64_t first = pieces > 1 ? (int64_t)(share * total) / XCDS * XCDS : step;
    if (first <= 0 || first >= total) first = step;
    if (pieces > 1 && first != step) step = ((total - first) / (pieces - 1) + XCDS - 1) / XCDS * XCDS;
    for (int64_t b0 = 0; b0 < total; b0 += (b0 == 0 ? first : step))
      hipLaunchKernelGGL(rotate_direct_kernel, dim3((unsigned)std::min(b0 == 0 ? first : step, total - b0)), dim3(RB),
                         0, (hipStream_t)stream, (const float *)etab, (const float *)workspace, D, gamma, nq, E,
                         score, accumulate, g_clk, b0);
  } else {
    hipLaunchKernelGGL(rotate_mfma_kernel, dim3(xcd_grid(ent_pad(E) / ME, (nq + MQ - 1) / MQ)), dim3(256), 0,
                       (hipStream_t)stream, eemb, (const uint2 *)etab, (const float2 *)rtab, D, gamma, all_h, all_r,
                       nq, E, score, accumulate, g_clk);
  }
  RNNL_HIP_CHECK(hipGetLastError());
  return RNNL_OK;
}

int rnnl_rotate_backward(const float *planes, int32_t ld, const float *hr, const float *grad, int32_t nq,
                         int32_t E, int32_t D, float *d_hr, float *d_tail, void *stream) {
  if (!planes || !hr || !grad || !d_hr || nq < 0 || E <= 0 || D <= 0 || ld < E) {
    set_error("rnnl_rotate_backward: bad arguments");
    return RNNL_ERR_INVALID;
  }
  if (nq == 0) return RNNL_OK;
  const unsigned bx = (unsigned)((E + BW_BS * BW_EPT - 1) / (BW_BS * BW_EPT));
  hipLaunchKernelGGL(rotate_backward_kernel, dim3(bx, (unsigned)D), dim3(BW_BS), 0, (hipStream_t)stream, planes, ld,
                     hr, grad, nq, E, D, d_hr, (float *)nullptr, d_tail);
  RNNL_HIP_CHECK(hipGetLastError());
  return RNNL_OK;
}

static size_t grads_hr_bytes(int64_t nq, int D) { return ((size_t)nq * 2 * D * sizeof(float) + 255) / 256 * 256; }
static unsigned bw_blocks(int E) { return (unsigned)((E + BW_BS * BW_EPT - 1) / (BW_BS * BW_EPT)); }

int rnnl_rotate_param_grads_scratch(int32_t nq, int32_t E, int32_t D, int32_t with_eemb, size_t *bytes) {
  if (nq < 0 || E <= 0 || D <= 0 || !bytes) {
    set_error("rnnl_rotate_param_grads_scratch: bad arguments");
    return RNNL_ERR_INVALID;
  }
  // hr | d(h o r) | the entity blocks' d(h o r) partials | d_tail
  *bytes = (2 + bw_blocks(E)) * grads_hr_bytes(nq, D) + (with_eemb ? (size_t)2 * D * E * sizeof(float) : 0);
  return RNNL_OK;
}

int rnnl_rotate_param_grads(const float *eemb, const float *planes, int32_t ld, const float *rtab, float gamma,
                            const int64_t *all_h, const int64_t *all_r, int32_t nq, int32_t E, int32_t D,
                            int32_t n_rel_total, const float *grad, void *scratch, size_t scratch_bytes,
                            float *d_eemb, float *d_remb, void *stream) {
  size_t need = 0;
  if (!eemb || !planes || !rtab || !all_h || !all_r || !grad || nq < 0 || E <= 0 || D <= 0 || ld < E ||
      n_rel_total <= 0 || (!d_eemb && !d_remb) ||
      rnnl_rotate_param_grads_scratch(nq, E, D, d_eemb != nullptr, &need) != RNNL_OK || !scratch ||
      scratch_bytes < need) {
    set_error("rnnl_rotate_param_grads: bad arguments (see rnnl_rotate_param_grads_scratch)");
    return RNNL_ERR_INVALID;
  }
  hipStream_t st = (hipStream_t)stream;
  if (d_remb) RNNL_HIP_CHECK(hipMemsetAsync(d_remb, 0, (size_t)n_rel_total * D * sizeof(float), st));
  if (nq == 0) {
    if (d_eemb) RNNL_HIP_CHECK(hipMemsetAsync(d_eemb, 0, (size_t)E * 2 * D * sizeof(float), st));
    return RNNL_OK;
  }
  unsigned char *ws = static_cast<unsigned char *>(scratch);
  const unsigned bx = bw_blocks(E);
  float *hr = reinterpret_cast<float *>(ws);
  // per entity block a partial d(h o r) (every entry written: no fill), summed
  // in block order by head_grad_kernel — no atomics, run-to-run bitwise
  float *d_hr = reinterpret_cast<float *>(ws + grads_hr_bytes(nq, D));
  float *d_hr_part = reinterpret_cast<float *>(ws + 2 * grads_hr_bytes(nq, D));
  float *d_tail = d_eemb ? reinterpret_cast<float *>(ws + (2 + bx) * grads_hr_bytes(nq, D)) : nullptr;
  hipLaunchKernelGGL(hr_rows_kernel, dim3((unsigned)((D + 255) / 256), (unsigned)nq), dim3(256), 0, st, eemb,
                     (const float2 *)rtab, D, all_h, all_r, hr);
  hipLaunchKernelGGL(rotate_backward_kernel, dim3(bx, (unsigned)D), dim3(BW_BS), 0, st, planes, ld, hr, grad, nq, E, D,
                     (float *)nullptr, d_hr_part, d_tail);
  const int64_t nhr = (int64_t)nq * 2 * D;
  hipLaunchKernelGGL(hr_fold_kernel, dim3(grid_for(nhr)), dim3(256), 0, st, (const float *)d_hr_part, (int)bx, nhr,
                     d_hr);
  if (d_eemb)
    hipLaunchKernelGGL(tail_rows_kernel, dim3((unsigned)((D + 31) / 32), (unsigned)((E + 31) / 32)), dim3(256), 0, st,
                       d_tail, E, D, d_eemb);
  hipLaunchKernelGGL(head_grad_kernel, dim3((unsigned)((D + 255) / 256)), dim3(256), 0, st, eemb,
                     (const float2 *)rtab, D, gamma, all_h, all_r, nq, (const float *)d_hr, d_eemb, d_remb);
  RNNL_HIP_CHECK(hipGetLastError());
  return RNNL_OK;
}

}  // extern "C"
