// Shared internals of the PredictorPlus / Predictor forward kernels for
// gfx950 (MI355X): launch parameters, the workspace carve-up and small
// device helpers.  Included by ground.hip (grounding, K1), score.hip
// (rule-to-entity aggregation + score_model, K2) and predictor.hip (the EM
// loop's rule-weight Predictor).  Not part of the C-ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "internal.h"

namespace rnnl {

constexpr int BS = 256;        // threads per workgroup (scoring kernels)
// Grounding workgroups: 512 lanes, two per CU (LDS-bound) with the chip to
// itself — 256 lanes at three per CU measured 12 % slower on the FB15k-237
// split (ground + score 10.2 vs 9.0 ms), 128 at five 40 % — and 256 lanes,
// one per CU, beside RotatE (a 512-lane workgroup would hold two of RotatE's
// six waves per SIMD); launches of <= WIDE_ROWS rows use 1,024 lanes.
constexpr int GBS = 256;       // threads per grounding workgroup beside another kernel (capped grid)
constexpr int SOLO_GBS = 512;  // threads per grounding workgroup with the chip to itself
constexpr int HBITS = 12;
constexpr int HCAP = 1 << HBITS;  // phase-A hash slots ((node, entity) -> count)
constexpr int OCC_CAP = 1024;     // phase-A occupied-slot list (fuller levels scan all HCAP slots)
constexpr int WBITS = 11;         // phase-B entity window: WIN entities
constexpr int WIN = 1 << WBITS;
constexpr int MAXE_BITS = 19;   // |E| <= 2^MAXE_BITS
// Phase B's counting sort of a large query's contributions: by sort window of
// 2^sbits entities, sbits the smallest with at most SORT_WINS windows
// (FB15k-237: 16 entities, WN18RR: 64, kinship / UMLS: 1), so that
// consecutive windows fill LDS hash passes (which merge a candidate's
// duplicate (node, entity) entries) and only a window of more than HB_LOAD
// contributions takes the dense direct-mapped pass.
constexpr int SORT_WINS = 256;
constexpr int MAX_SBITS = MAXE_BITS - 10;  // 2^MAXE_BITS / SORT_WINS entities per window at most
static_assert((1 << MAX_SBITS) <= WIN, "a sort window must fit the dense pass's direct map");
constexpr int HB = WIN;                // phase-B candidate hash slots
constexpr int HB_LOAD = HB * 3 / 4;    // max contributions per hash pass
constexpr int WG_PER_CU = 2;           // grounding workgroups per CU at SOLO_GBS lanes (LDS-bound)
constexpr int NUM_CU = 256;
constexpr int SCORE_WG_PER_CU = 8;     // scoring workgroups per CU (full grid)
constexpr int EMPTY = -1;
constexpr int WIDE_ROWS = 256;  // launches of at most this many rows ground with 1024-lane workgroups
// Phase-B hash passes rank their candidates by entity through an LDS bitmap
// over the pass's entity range (it shares phase A's per-thread arrays, 36 B
// per thread): ranges up to sort_words(G) x 32 entities (49,152 at G = 256).
constexpr int sort_words(int G) { return (9 * G * 4 / 6) & ~(G - 1); }

// Workspace header words (uint32), then a 64-bit pool counter at byte 64.
enum {
  H_STATUS = 0, H_DEQUEUE = 1, H_FLAGS = 2, H_ERRBITS = 3, H_ERRQ = 4, H_DEQUEUE2 = 5, H_CHUNKS = 6, H_NCAND = 8,
  H_NENT = 10,  // 64-bit: bucket entries written (<= the pool reserved: duplicates merge in phase B)
  H_BW_MAXG = 20, H_BW_SUMK = 22  // EM Predictor backward's fixed-point stats (past the status read-back)
};
// H_FLAGS bit 0: the launch's rows hold more than one relation (the
// reference forward's one-relation-per-batch check, predictors.py:54-55 /
// 211-212, read back with the status instead of a separate reduction)
enum { FLAG_MIXED = 1 };
// (64-bit words: H_CHUNKS the scoring chunk total, H_NCAND the candidate total of the grounding)
// H_ERRBITS: 4 watchdog, 8 a path count or PNA degree reached 2^32 (the u32
// sums would wrap), 16 the node-weight table is out of its fixed-point range
// (a non-finite aggregate, or |sum| >= 2^30), 32 a candidate's counts sum past
// the exact int64 feature sums.  8, 16 and 32 -> RNNL_ERR_RANGE.
enum { ERR_WATCHDOG = 4, ERR_COUNT_WIDTH = 8, ERR_NODE_RANGE = 16, ERR_ACC_RANGE = 32 };
constexpr int HDR_WORDS_BYTES = 256;

// Packed MLP weights (written by pack_weights_kernel behind the header).
constexpr int W_ADDW = 0;                 // add_model weight (16 x 16 | 16 x 192)
constexpr int W_ADDB = W_ADDW + 16 * 192; // add_model bias (16)
constexpr int W_LNW = W_ADDB + 16;        // layer_norm weight (16)
constexpr int W_LNB = W_LNW + 16;         // layer_norm bias (16)
constexpr int W_S0X = W_LNB + 16;         // score_model.layers.0.weight[:, :16] (128 x 16)
constexpr int W_S1W = W_S0X + 128 * 16;   // score_model.layers.1.weight (128)
constexpr int W_S1B = W_S1W + 128;        // score_model.layers.1.bias (1)
constexpr int W_FLOATS = 5376;            // padded
constexpr int HDR_BYTES = HDR_WORDS_BYTES + W_FLOATS * 4;

// LDS copy of the weights used by K2: [add_w 16*KIN | add_b | ln_w | ln_b | s0x 128x16 | s1w 128 | s1b]
template <int AGG>
struct WL {
  static constexpr int KIN = AGG == RNNL_AGG_SUM ? 16 : 192;
  static constexpr int ADDW = 0, ADDB = 16 * KIN, LNW = ADDB + 16, LNB = LNW + 16, S0X = LNB + 16,
                       S1W = S0X + 128 * 16, S1B = S1W + 128, N = S1B + 4;
};

// Per-slot scratch (entries), scaled by capacity_scale.
constexpr int64_t FCAP_BASE = 1 << 16;  // frontier list (and window-sorted contributions)
constexpr int64_t PCAP_BASE = 1 << 16;  // contributions of one query
static_assert(FCAP_BASE >= PCAP_BASE, "phase B sorts contributions into the frontier buffer");
constexpr int64_t POOL_PER_QUERY = 8192;  // global bucket pool entries per query (x scale)

struct KParams {
  GraphDev g;
  RulesDev rl;
  int32_t agg, feature;
  const unsigned char *node_w;
  const float *add_w, *add_b, *ln_w, *ln_b, *s0_w, *s0_b, *s1_w, *s1_b, *rel_emb;
  const float *base_row;  // nullable: every row's base score (bias), read instead of score[q][t]
  const float *packed;    // nullable: the weights packed by rnnl_pack_weights (else packed per launch)
  const int64_t *all_h, *all_r, *etr;
  int32_t nq;
  int32_t ebits;     // entity bits of the packed (trie node, entity) keys
  uint32_t emask;    // (1 << ebits) - 1
  int32_t sbits;     // phase B's sort windows: 2^sbits entities (SORT_WINS)
  float *score;
  uint8_t *mask;
  int32_t *n_cand;
  uint64_t *digest;
  unsigned char *ws;
  // workspace carve-up
  int64_t fcap, pcap, pool_cap;
  int32_t nslots;
  unsigned char *slots;
  int64_t *q_base;   // per query: first pool index of its run
  float *q_scale;    // per query: PNA mean log-degree
  const int32_t *order;  // nullable: the grounding's dequeue order (heaviest estimated queries first)
  int32_t atomic_out;  // deferred scoring into a zeroed score matrix: atomic adds
  int4 *cand;        // per pool index: candidate record (entity, bucket start, bucket length, 0)
                     // (the first n_cand entries of a query's run)
  int2 *bent;        // bucket entries: (trie node, path count bits)
  float *memo;       // SUM: score_model output of a candidate reached by one path of one leaf node
  // SUM: score_model outputs keyed by a candidate's bucket entries when it has
  // one to three (pair memo, score_sum_chunk_kernel); nullptr = off
  unsigned long long *ptab, *ptab_region;
  int32_t psbits, pbr, pbo, pbc, pbc3;  // slots 2^psbits; key field bits: relation, node offset, count (pair,
                                       // triple; 0: no triple keys)
  int2 *chunks;      // scoring work units (query, first candidate) of <= 64 candidates each
  int64_t chunk_cap;
  unsigned long long *prof;  // diagnostic phase cycle counters (nullable)
};

extern unsigned long long *g_prof;  // rnnl_debug_profile (ground.hip)

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ULL;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
  return x ^ (x >> 31);
}

__device__ __forceinline__ uint32_t hash32(uint32_t k) { return k * 2654435761u; }

// Per-slot scratch: two frontier buffers and the contribution list, each an
// array of 8-B entries (key, count) — one contiguous run per list, so a query
// touches a few compact address ranges.  key = (trie node - head root) <<
// ebits | entity, the phase-A hash key (ebits = bits of |E|; the host checks
// that a head's trie nodes fit the remaining 31 - ebits bits).
struct Ent {
  uint32_t k, c;
};

struct Slot {
  Ent *f0;
  int64_t fcap;
  Ent *ct;
  __device__ __forceinline__ Ent *f(int k) const { return f0 + (int64_t)k * fcap; }
};

__host__ __device__ inline int64_t slot_bytes(int64_t fcap, int64_t pcap) {
  return 2 * fcap * (int64_t)sizeof(Ent) + pcap * (int64_t)sizeof(Ent);
}

__device__ inline Slot make_slot(unsigned char *base, int slot, int64_t fcap, int64_t pcap) {
  unsigned char *b = base + (int64_t)slot * slot_bytes(fcap, pcap);
  Slot s;
  s.f0 = reinterpret_cast<Ent *>(b);
  s.fcap = fcap;
  s.ct = reinterpret_cast<Ent *>(b + 2 * fcap * (int64_t)sizeof(Ent));
  return s;
}

#ifndef RNNL_PTAB_MIN_BITS  // compile-time knob for A/B builds (tools/build_variants.sh)
#define RNNL_PTAB_MIN_BITS 12
#endif
constexpr int PTAB_MIN_BITS = RNNL_PTAB_MIN_BITS;

// Workspace layout, shared by host sizing and the launch.
struct Layout {
  int64_t nslots, fcap, pcap, pool_cap;
  int64_t off_qbase, off_qscale, off_order, off_cand, off_bent, off_slots, off_chunk, chunk_cap, off_memo, off_ptab, ptab_bits,
      total;
};

inline int64_t align256(int64_t x) { return (x + 255) & ~int64_t(255); }

// Base capacities (entries at capacity_scale 1); rnnl_debug_capacity lowers
// them so tests can force the overflow -> retry path (ground.hip).
extern int64_t g_fcap_base, g_pcap_base, g_pool_per_query;

// n_nodes: the rules' trie nodes, for the SUM scoring memo at the end of the
// workspace (0 where only the offsets before it are needed)
inline Layout make_layout(int64_t nq, int64_t scale, int64_t n_nodes = 0) {
  Layout L;
  L.nslots = std::max<int64_t>(1, std::min<int64_t>(nq, (int64_t)NUM_CU * WG_PER_CU));
  L.fcap = g_fcap_base * scale;
  L.pcap = g_pcap_base * scale;
  L.pool_cap = std::max<int64_t>(g_pool_per_query * scale * std::max<int64_t>(nq, 1), L.pcap);
  int64_t o = HDR_BYTES;
  L.off_qbase = o = align256(o);
  o += 8 * std::max<int64_t>(nq, 1);
  L.off_qscale = o = align256(o);
  o += 4 * std::max<int64_t>(nq, 1);
  L.off_order = o = align256(o);
  o += 4 * std::max<int64_t>(nq, 1);
  L.off_cand = o = align256(o);
  o += 16 * L.pool_cap;
  L.off_bent = o = align256(o);
  o += 8 * L.pool_cap;
  L.off_slots = o = align256(o);
  o += L.nslots * slot_bytes(L.fcap, L.pcap);
  // scoring chunks: sum over queries of ceil(candidates / 64) <= nq + pool_cap / 64
  L.chunk_cap = std::max<int64_t>(nq, 1) + L.pool_cap / 64 + 1;
  L.off_chunk = o = align256(o);
  o += 8 * L.chunk_cap + 4 * (std::max<int64_t>(nq, 1) / 256 + 1);  // list | per-block chunk totals
  L.off_memo = o = align256(o);
  o += 4 * n_nodes;
  // pair memo (SUM): 2^ptab_bits 8-B slots, ~128 per row, 2^PTAB_MIN_BITS .. 2^23
  // (a 32-row reference batch: 2^12, 32 KB, zeroed by one block of the
  // chunk-list kernel on the call's critical path)
  L.ptab_bits = PTAB_MIN_BITS;
  while (L.ptab_bits < 23 && (1ll << L.ptab_bits) < 128 * std::max<int64_t>(nq, 1)) ++L.ptab_bits;
  L.off_ptab = o = align256(o);
  if (n_nodes > 0) o += 8ll << L.ptab_bits;
  L.total = o;
  return L;
}

// Exclusive block scan of one int per thread (G threads); `total` gets the block sum.
template <int G>
__device__ __forceinline__ int block_scan(int x, int *s_ws, int &total) {
  constexpr int GNW = G / 64;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int v = x;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    int y = __shfl_up(v, o, 64);
    if (lane >= o) v += y;
  }
  if (lane == 63) s_ws[wid] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int w = 0; w < GNW; ++w) {
      int t = s_ws[w];
      s_ws[w] = acc;
      acc += t;
    }
    s_ws[GNW] = acc;
  }
  __syncthreads();
  const int res = v - x + s_ws[wid];
  total = s_ws[GNW];
  __syncthreads();
  return res;
}

// Largest i in [0, n) with a[i] <= k, n <= G, for a non-decreasing a of
// G entries (the workgroup's lanes) with a[0] <= k and a[i] > k for every i >= n — the block
// scans' exclusive prefixes: threads past n add nothing, so their prefix is
// the total, > k.  Branch-free: ceil(log2 n) steps of one LDS read, a
// compare and a select (the bisection's bounds bookkeeping cost ~7 VALU
// instructions a step; this is the grounding's per-edge / per-item search).
__device__ __forceinline__ int upper_idx(const int *a, int n, int k) {
  int lo = 0;
  for (int step = n > 1 ? 1 << (31 - __clz(n - 1)) : 0; step > 0; step >>= 1) {
    const int c = lo + step;
    lo = a[c] <= k ? c : lo;
  }
  return lo;
}

// Workgroup barrier for data handed between waves through GLOBAL scratch:
// __syncthreads() alone lowers to s_barrier without waiting for this wave's
// outstanding stores, so a store could still be in flight when another wave
// of the workgroup loads the address.  Drain the stores, barrier, and drop
// this CU's L1 lines (stale copies from the previous query in the slot).
__device__ __forceinline__ void wg_sync_global() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  asm volatile("buffer_inv sc0" ::: "memory");
}

// LDS hand-off between the lanes of one wave (no workgroup barrier).
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Scoring kernels: a node table flagged by fix_shift / node_weights_kernel
// fails the launch (ERR_NODE_RANGE) instead of scoring with it.
__device__ __forceinline__ void check_node_table(const KParams &p, const unsigned int *trailer) {
  if (blockIdx.x == 0 && threadIdx.x == 0 && trailer[2]) {
    unsigned int *hdr = reinterpret_cast<unsigned int *>(p.ws);
    atomicOr(&hdr[H_ERRBITS], (unsigned)ERR_NODE_RANGE);
    atomicOr(&hdr[H_STATUS], 2u);
  }
}

// A candidate whose path counts sum to more than the exact int64 feature
// sums can hold (sum of counts x max |record| >= 2^63) fails the launch
// (ERR_ACC_RANGE) instead of wrapping: the reference sums int64 counts in
// fp32 (predictors.py:224) and never wraps.
__device__ __forceinline__ void flag_acc_range(const KParams &p) {
  unsigned int *hdr = reinterpret_cast<unsigned int *>(p.ws);
  atomicOr(&hdr[H_ERRBITS], (unsigned)ERR_ACC_RANGE);
  atomicOr(&hdr[H_STATUS], 2u);
}

// Table-wide fixed-point shift from the max |sum| bits in trailer[0]
// (node_fix_kernel, lin_fix_kernel); trailer[2] = 1 when the table cannot be
// represented (a non-finite sum — its |x| bits are >= those of +inf — or
// |sum| >= 2^30, which would need a negative shift): the records are zeroed
// and the scoring kernels report ERR_NODE_RANGE.
// `pre_bits`: the max |x| bits of values the records were derived from (the
// SUM table's member sums before the folded Linear), held to the same 2^30.
__device__ __forceinline__ int fix_shift(unsigned int *trailer, bool &bad, unsigned int pre_bits = 0u) {
  const unsigned int bits = trailer[0];
  int e = 0;
  bad = bits >= 0x7f800000u || pre_bits >= 0x4e800000u;  // 0x4e800000 = 2^30 as f32
  if (!bad && bits) frexpf(__uint_as_float(bits), &e);  // max < 2^e
  bad = bad || e > 30;
  const int shift = bad ? 0 : min(30 - e, 60);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    trailer[1] = (unsigned)shift;
    trailer[2] = bad ? 1u : 0u;
  }
  return shift;
}

// A wave's next range of k chunks: its first range is static (its grid-wide
// wave index), later ones come from the dequeue counter past the static part,
// which is never touched when the static ranges cover the list.  Wave-uniform.
__device__ __forceinline__ void next_chunks(unsigned int *ctr, long long nchunks, int k, unsigned &c, unsigned &cend) {
  const unsigned long long stat = (unsigned long long)gridDim.x * (BS / 64) * k;
  if (cend == 0u) {
    c = (blockIdx.x * (BS / 64) + (threadIdx.x >> 6)) * (unsigned)k;
  } else if ((long long)stat >= nchunks) {
    c = (unsigned)nchunks;
  } else {
    if ((threadIdx.x & 63) == 0) c = (unsigned)stat + atomicAdd(ctr, (unsigned)k);
    c = __builtin_amdgcn_readfirstlane(c);
  }
  cend = c + (unsigned)k;
}

// Host-side launch sequences and parameter set-up shared across the
// translation units.
extern bool g_pair_memo;                                                          // score.hip
void launch_chunk_list(const KParams &p, hipStream_t st);                         // ground.hip
void launch_ground(const KParams &p, int agg, hipStream_t st, int grid = 0);     // ground.hip
void launch_score(const KParams &p, const RulesDev &rl, hipStream_t st, int grid);  // score.hip
int setup_params(const char *who, rnnl_graph g, rnnl_rules r, const int64_t *all_h, const int64_t *all_r,
                 const int64_t *etr, int32_t nq, int32_t *n_cand, void *ws, size_t ws_bytes, int32_t scale,
                 KParams &p);                                                     // ground.hip
void set_score_params(KParams &p, const rnnl_predictor_params *pp, float *score, uint8_t *mask, uint64_t *digest);
bool bad_params(const rnnl_predictor_params *pp, const float *score);
KParams export_params(void *ws, int32_t nq, int32_t scale, const int32_t *n_cand);  // the pool's carve-up only

}  // namespace rnnl
