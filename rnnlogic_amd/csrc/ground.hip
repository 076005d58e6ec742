// PredictorPlus forward for gfx950 (MI355X): two kernels per launch.
//
// K1 ground_kernel — one persistent workgroup (256 lanes) per query at a
// time, dequeued from a device counter:
//   grounding / propagate (ref src/data.py:136-173, torch_scatter scatter-sum)
//       -> level-synchronous walk of the head relation's rule-prefix trie over
//          the vertex-major CSR; every (trie node, entity) path count lives in
//          an LDS hash (integer, exact); the query's own edge is skipped on
//          hops of the query relation (data.py:164-169).
//   candidate set + rule_count stack (ref src/predictors.py:221-244)
//       -> leaf contributions (entity, node, count) are counting-sorted by
//          entity window and bucketed per candidate through a direct-mapped
//          LDS table into a global pool: per query a contiguous run of
//          candidate records (entity, bucket) and (node, count) entries —
//          the COO of the reference's stacked rule_count matrix.
// K2 score_kernel — one workgroup per query (grid-stride), one lane per
// candidate:
//   rule_to_entity (ref src/layers.py:53-126) + score_model (layers.py:9-51)
//       -> node sums in exact fixed point (order-independent, deterministic),
//          Linear/LayerNorm/ReLU, then the 32->128->1 MLP with the weights in
//          LDS and the relation half folded into a per-query bias; the result
//          is added into the pre-filled base score (bias/RotatE) or written
//          (entity_feature none).
// Splitting the MLP out of K1 keeps K1's registers low (it is latency-bound:
// dependent CSR reads and barriers) and gives K2 a simple, fully occupied
// streaming shape.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <string>

#include "internal.h"

namespace rnnl {

constexpr int BS = 256;      // threads per workgroup (scoring kernels)
#ifndef RNNL_GBS
#define RNNL_GBS 256
#endif
constexpr int GBS = RNNL_GBS;  // threads per grounding workgroup
constexpr int GNW = GBS / 64;  // its waves
#ifndef RNNL_EPT
#define RNNL_EPT 1
#endif
constexpr int EPT = RNNL_EPT;  // phase-A edges per lane per pass
#ifndef RNNL_HBITS
#define RNNL_HBITS 12
#endif
#ifndef RNNL_WBITS
#define RNNL_WBITS 11
#endif
#ifndef RNNL_WG_PER_CU
#define RNNL_WG_PER_CU 3
#endif
#ifndef RNNL_CSR_COMPACT
#define RNNL_CSR_COMPACT 1  // (v, rel) edge ranges from the compact per-vertex view (0: the E x R offsets)
#endif
constexpr int HBITS = RNNL_HBITS;
constexpr int HCAP = 1 << HBITS;  // phase-A hash slots ((node, entity) -> count)
constexpr int WBITS = RNNL_WBITS;  // phase-B entity window: WIN entities
constexpr int WIN = 1 << WBITS;
#ifndef RNNL_MAXE_BITS
#define RNNL_MAXE_BITS 19
#endif
constexpr int MAXWIN = (1 << RNNL_MAXE_BITS) >> WBITS;  // windows per graph (|E| <= 2^RNNL_MAXE_BITS)
constexpr int HB = WIN;            // phase-B candidate hash slots (one window at <= 0.75 load... or less)
constexpr int HB_LOAD = HB * 3 / 4;  // max contributions per hash pass
constexpr int WG_PER_CU = RNNL_WG_PER_CU;
constexpr int NUM_CU = 256;
constexpr int EMPTY = -1;
// Phase-B hash passes rank their candidates by entity through an LDS bitmap
// over the pass's entity range (it shares phase A's per-thread arrays, 36 B
// per thread): ranges up to SORT_WORDS x 32 entities (49,152 at GBS = 256).
constexpr int SORT_WORDS = (9 * GBS * 4 / 6) & ~(GBS - 1);

// Workspace header words (uint32), then a 64-bit pool counter at byte 64.
enum { H_STATUS = 0, H_DEQUEUE = 1, H_ERRBITS = 3, H_ERRQ = 4, H_DEQUEUE2 = 5, H_CHUNKS = 6, H_NCAND = 8 };
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
#ifndef RNNL_FCAP_BITS
#define RNNL_FCAP_BITS 16
#endif
constexpr int64_t FCAP_BASE = 1 << RNNL_FCAP_BITS;  // frontier list (and window-sorted contributions)
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
  const int64_t *all_h, *all_r, *etr;
  int32_t nq;
  int32_t ebits;     // entity bits of the packed (trie node, entity) keys
  uint32_t emask;    // (1 << ebits) - 1
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
  float *cand_out;   // deferred scoring: score_model output per candidate record (nullable)
  int32_t atomic_out;  // deferred scoring into a zeroed score matrix: atomic adds (no cand_out stores)
  int4 *cand;        // per pool index: candidate record (entity, bucket start, bucket length, 0)
                     // (the first n_cand entries of a query's run)
  int2 *bent;        // bucket entries: (trie node, path count bits)
  float *memo;       // SUM: score_model output of a candidate reached by one path of one leaf node
  // SUM: score_model outputs keyed by a candidate's bucket entries when it has
  // one or two (pair memo, score_sum_chunk_kernel); nullptr = off
  unsigned long long *ptab, *ptab_region;
  int32_t psbits, pbr, pbo, pbc, pbc3;  // slots 2^psbits; key field bits: relation, node offset, count (pair,
                                       // triple; 0: no triple keys)
  int2 *chunks;      // PNA: scoring work units (query, first candidate) of <= 64 candidates each
  int64_t chunk_cap;
  unsigned long long *prof;  // diagnostic phase cycle counters (nullable)
};

static unsigned long long *g_prof = nullptr;

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ULL;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
  return x ^ (x >> 31);
}

__device__ __forceinline__ uint32_t hash32(uint32_t k) { return k * 2654435761u; }

// Deferred scoring output of candidate record ci (entity t of row q): stored
// for rnnl_predictorplus_apply, or (atomic_out) added into a score matrix that
// starts at zero and receives the base score by atomic adds too — two addends
// on an exact zero give fl(base + out) in either order, so the result is the
// one-stream path's bit for bit.
__device__ __forceinline__ void deferred_store(const KParams &p, int q, int64_t ci, int t, float out) {
  if (p.atomic_out)
    unsafeAtomicAdd(p.score + (int64_t)q * p.g.E + t, out);
  else
    p.cand_out[ci] = out;
}


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

// Workspace layout, shared by host sizing and the launch.
struct Layout {
  int64_t nslots, fcap, pcap, pool_cap;
  int64_t off_qbase, off_qscale, off_cand, off_bent, off_cout, off_slots, off_chunk, chunk_cap, off_memo, off_ptab,
      ptab_bits, total;
};

static inline int64_t align256(int64_t x) { return (x + 255) & ~int64_t(255); }

// Base capacities (entries at capacity_scale 1); rnnl_debug_capacity lowers
// them so tests can force the overflow -> retry path.
static int64_t g_fcap_base = FCAP_BASE, g_pcap_base = PCAP_BASE, g_pool_per_query = POOL_PER_QUERY;

// n_nodes: the rules' trie nodes, for the SUM scoring memo at the end of the
// workspace (0 where only the offsets before it are needed)
static Layout make_layout(int64_t nq, int64_t scale, int64_t n_nodes = 0) {
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
  L.off_cand = o = align256(o);
  o += 16 * L.pool_cap;
  L.off_bent = o = align256(o);
  o += 8 * L.pool_cap;
  L.off_cout = o = align256(o);
  o += 4 * L.pool_cap;
  L.off_slots = o = align256(o);
  o += L.nslots * slot_bytes(L.fcap, L.pcap);
  // PNA scoring chunks: sum over queries of ceil(candidates / 64) <= nq + pool_cap / 64
  L.chunk_cap = std::max<int64_t>(nq, 1) + L.pool_cap / 64 + 1;
  L.off_chunk = o = align256(o);
  o += 8 * L.chunk_cap + 4 * (std::max<int64_t>(nq, 1) / 256 + 1);  // list | per-block chunk totals
  L.off_memo = o = align256(o);
  o += 4 * n_nodes;
  // pair memo (SUM): 2^ptab_bits 8-B slots, ~128 per row, 2^16 .. 2^23
  L.ptab_bits = 16;
  while (L.ptab_bits < 23 && (1ll << L.ptab_bits) < 128 * std::max<int64_t>(nq, 1)) ++L.ptab_bits;
  L.off_ptab = o = align256(o);
  if (n_nodes > 0) o += 8ll << L.ptab_bits;
  L.total = o;
  return L;
}

// Exclusive block scan of one int per thread; `total` gets the block sum.
__device__ __forceinline__ int block_scan(int x, int *s_ws, int &total) {
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

// Largest i in [0, n) with a[i] <= k (a non-decreasing, a[0] == 0 <= k).
__device__ __forceinline__ int upper_idx(const int *a, int n, int k) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (a[mid] <= k)
      lo = mid;
    else
      hi = mid - 1;
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

struct __align__(16) Smem {
  union {
    struct {
      int key[HCAP];
      uint32_t val[HCAP];
    } a;
    struct {
      int map[WIN];  // entity offset -> candidate slot
      int cnt[WIN];
      int off[WIN];
      int st[WIN];   // slot -> entity
    } b;
    struct {
      int key[HB];   // entity (EMPTY: free)
      int cnt[HB];   // bucket size, then the scatter fill counter / degree
      int off[HB];   // bucket start within the pass
      int cid[HB];   // candidate index within the pass
    } c;
  } u;
  union {
    struct {  // phase A: per-thread frontier items and edge batches
      int ent_v[GBS], ent_fch[GBS], item_off[GBS];
      uint32_t ent_c[GBS];
      int it_child[GBS], it_beg[GBS], it_flags[GBS], edge_off[GBS];
      uint32_t it_c[GBS];
    };
    struct {  // phase B: entity bitmap of one hash pass and its popcount prefix (candidate ranks)
      uint32_t sbits[SORT_WORDS];
      unsigned short spre[SORT_WORDS];
    };
  };
  int ws[GNW + 1];
  int q, nd, np, ovf, err, root;
  long long qbase;
  unsigned long long t0;
  int whist[MAXWIN], wbeg[MAXWIN + 1], wfill[MAXWIN];
  unsigned long long sumlog;
  unsigned long long tp[8];  // diagnostic sub-phase cycles (thread 0)
};

__device__ __forceinline__ void emit_contrib(Smem &S, const Slot &sl, int64_t pcap, uint32_t key, uint32_t c) {
  const int pos = atomicAdd(&S.np, 1);
  if (pos < pcap) {
    sl.ct[pos] = Ent{key, c};
  } else {
    S.ovf = 1;
  }
}

__device__ __forceinline__ void emit_frontier(Smem &S, const Slot &sl, int buf, int64_t fcap, uint32_t key,
                                              uint32_t c) {
  const int pos = atomicAdd(&S.nd, 1);
  if (pos < fcap) {
    sl.f(buf)[pos] = Ent{key, c};
  } else {
    S.ovf = 1;
  }
}

// (node, entity) += c in the phase-A hash; false if the table is full.
__device__ __forceinline__ bool hash_add(Smem &S, int key, uint32_t c) {
  uint32_t h = hash32((uint32_t)key) >> (32 - HBITS);
#pragma unroll 1
  for (int probe = 0; probe < 64; ++probe) {
    const int k = atomicCAS(&S.u.a.key[h], EMPTY, key);
    if (k == EMPTY || k == key) {
      const uint32_t old = atomicAdd(&S.u.a.val[h], c);
      if (old + c < old) atomicOr(&S.err, ERR_COUNT_WIDTH);  // carry out of the u32 path count
      return true;
    }
    h = (h + 1) & (HCAP - 1);
  }
  return false;
}

// Watchdog: true (uniformly, after the barrier) once the current query has
// run longer than kWatchdogTicks of the 100 MHz real-time clock; thread 0
// then flags S.err.  Guarantees every wave reaches the kernel exit.
constexpr unsigned long long kWatchdogTicks = 200000000ull;  // 2 s
__device__ __forceinline__ bool watchdog(Smem &S) {
  if (threadIdx.x == 0 && __builtin_amdgcn_s_memrealtime() - S.t0 > kWatchdogTicks) atomicOr(&S.err, ERR_WATCHDOG);
  __syncthreads();
  return S.err != 0;
}

#define PSTAMP(k)                                                     \
  do {                                                                \
    if (p.prof && tid == 0) {                                         \
      const unsigned long long _t = __builtin_amdgcn_s_memtime();     \
      S.tp[k] += _t - S.tp[7];                                        \
      S.tp[7] = _t;                                                   \
    }                                                                 \
  } while (0)

// ---------------------------------------------------------------- phase A
__device__ void ground_query(const KParams &p, Smem &S, const Slot &sl, int h, int r, int root, int rm_src,
                             int rm_dst) {
  const int tid = threadIdx.x;
  const int E = p.g.E, R = p.g.R;
  const int depth = p.rl.head_depth[r];
  if (tid == 0) {
    sl.f(0)[0] = Ent{(uint32_t)h, 1u};
    if (p.rl.node_info[root].w > 0) emit_contrib(S, sl, p.pcap, (uint32_t)h, 1u);
  }
  wg_sync_global();
  if (p.prof && tid == 0) S.tp[7] = __builtin_amdgcn_s_memtime();
  int cur = 0, n_prev = 1;
  for (int d = 1; d <= depth; ++d) {
    const int nxt = cur ^ 1;
    for (int cb = 0; cb < n_prev; cb += GBS) {
      if (watchdog(S)) break;
      const int ne = min(GBS, n_prev - cb);
      int nch = 0;
      if (tid < ne) {
        const Ent fe = sl.f(cur)[cb + tid];
        const int node = root + (int)(fe.k >> p.ebits);
        S.ent_v[tid] = (int)(fe.k & p.emask);
        S.ent_c[tid] = fe.c;
        const int4 ni = p.rl.node_info[node];
        S.ent_fch[tid] = ni.y;
        nch = ni.z;
      }
      int NI;
      const int ioff = block_scan(nch, S.ws, NI);
      S.item_off[tid] = ioff;
      __syncthreads();
      PSTAMP(3);
      for (int ib = 0; ib < NI; ib += GBS) {
        const int k = ib + tid;
        int deg = 0;
        if (k < NI) {
          const int ent = upper_idx(S.item_off, ne, k);
          const int child = S.ent_fch[ent] + (k - S.item_off[ent]);
          const int4 ci = p.rl.node_info[child];
          const int rel = ci.x;
          const int v = S.ent_v[ent];
#if RNNL_CSR_COMPACT
          // the (v, rel) edge range from v's relation bitmap word + the dense offsets (L2-sized)
          const uint2 vb = p.g.vbits[(int64_t)v * p.g.W + (rel >> 5)];
          const uint32_t bit = 1u << (rel & 31);
          int beg = 0;
          if (vb.x & bit) {
            const int pos = (int)vb.y + __popc(vb.x & (bit - 1u));
            beg = p.g.dvoff[pos];
            deg = p.g.dvoff[pos + 1] - beg;
          }
#else
          const int64_t o = (int64_t)v * R + rel;
          const int beg = p.g.off[o];
          deg = p.g.off[o + 1] - beg;
#endif
          S.it_child[tid] = child;
          S.it_beg[tid] = beg;
          S.it_c[tid] = S.ent_c[ent];
          // bit 0: leaf (rules end here), bit 1: inner (has children),
          // bit 2: this hop may traverse the query's own edge (data.py:143-146)
          S.it_flags[tid] = (ci.w > 0 ? 1 : 0) | (ci.z > 0 ? 2 : 0) |
                            (rel == r && v == rm_src ? 4 : 0);
        }
        int NE;
        const int eoff = block_scan(deg, S.ws, NE);
        S.edge_off[tid] = eoff;
        __syncthreads();
        PSTAMP(4);
        const int nit = min(GBS, NI - ib);
        // EPT edges per lane per pass: their binary searches and col loads are
        // independent, so EPT loads are in flight before the first is used
        for (int eb = 0; eb < NE; eb += GBS * EPT) {
          int ev_it[EPT], ev_t[EPT];
#pragma unroll
          for (int k = 0; k < EPT; ++k) {
            const int j = eb + k * GBS + tid;
            ev_it[k] = -1;
            if (j < NE) {
              const int it = upper_idx(S.edge_off, nit, j);
              ev_it[k] = it;
              ev_t[k] = p.g.col[S.it_beg[it] + (j - S.edge_off[it])];
            }
          }
#pragma unroll
          for (int k = 0; k < EPT; ++k) {
            const int it = ev_it[k];
            if (it >= 0) {
              const int tt = ev_t[k];
              const int fl = S.it_flags[it];
              if (!((fl & 4) && tt == rm_dst)) {
                const uint32_t key = ((uint32_t)(S.it_child[it] - root) << p.ebits) | (uint32_t)tt;
                const uint32_t c = S.it_c[it];
                if (fl & 1) emit_contrib(S, sl, p.pcap, key, c);
                if (fl & 2) {
                  if (!hash_add(S, (int)key, c)) emit_frontier(S, sl, nxt, p.fcap, key, c);
                }
              }
            }
          }
        }
        __syncthreads();
        PSTAMP(5);
      }
    }
    // compact the hash into the next frontier and clear it
    for (int s = tid; s < HCAP; s += GBS) {
      const int k = S.u.a.key[s];
      if (k != EMPTY) {
        emit_frontier(S, sl, nxt, p.fcap, (uint32_t)k, S.u.a.val[s]);
        S.u.a.key[s] = EMPTY;
        S.u.a.val[s] = 0u;
      }
    }
    wg_sync_global();
    PSTAMP(6);
    n_prev = min((int64_t)S.nd, p.fcap);
    __syncthreads();
    if (tid == 0) S.nd = 0;
    cur = nxt;
    __syncthreads();
  }
}

// ---------------------------------------------------------------- phase B
// PNA degree += count x rules at the node (u32 in LDS), carry-checked.
__device__ __forceinline__ void degree_add(Smem &S, uint32_t *cell, uint32_t c, int nrules) {
  const uint64_t v = (uint64_t)c * (uint32_t)nrules;
  const uint32_t old = atomicAdd(cell, (uint32_t)v);
  if ((v >> 32) || old + (uint32_t)v < old) atomicOr(&S.err, ERR_COUNT_WIDTH);
}

// Exclusive scan of WIN ints in place (PER consecutive per thread); returns the total.
__device__ __forceinline__ int scan_win(int *a, int *s_ws) {
  constexpr int PER = WIN / GBS;
  const int tid = threadIdx.x;
  int loc[PER];
  int sum = 0;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    loc[j] = a[tid * PER + j];
    sum += loc[j];
  }
  int total;
  int base = block_scan(sum, s_ws, total);
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    a[tid * PER + j] = base;
    base += loc[j];
  }
  __syncthreads();
  return total;
}

// One entity window [lo, lo + WIN) whose contributions are w[beg, end):
// candidate records for it are written at pool indices cbase + [0, nc) and
// its buckets at pool indices qbase + beg + [0, end - beg).  degree_only (PNA
// sweep 1) accumulates sum log(degree) instead.  Returns nc.
__device__ int window_pass(const KParams &p, Smem &S, const Slot &sl, int lo, int beg, int end, int64_t cbase,
                           bool degree_only) {
  const int tid = threadIdx.x;
  const Ent *w = sl.f(0);  // window-sorted contributions: a = entity, b = node, c = count
  if (p.prof && tid == 0) S.tp[7] = __builtin_amdgcn_s_memtime();
  for (int i = tid; i < WIN; i += GBS) S.u.b.map[i] = 0;
  __syncthreads();
  for (int i = beg + tid; i < end; i += GBS) S.u.b.map[(int)(w[i].k & p.emask) - lo] = 1;  // mark present entities
  __syncthreads();
  for (int i = tid; i < WIN; i += GBS) S.u.b.cnt[i] = S.u.b.map[i];
  __syncthreads();
  const int nc = scan_win(S.u.b.cnt, S.ws);  // slots in ascending entity order
  for (int i = tid; i < WIN; i += GBS) {
    if (S.u.b.map[i]) {
      const int slot = S.u.b.cnt[i];
      S.u.b.map[i] = slot;
      S.u.b.st[slot] = lo + i;
    }
  }
  __syncthreads();
  for (int i = tid; i < WIN; i += GBS) S.u.b.cnt[i] = 0;
  __syncthreads();
  PSTAMP(0);
  if (degree_only) {
    // PNA sweep 1: degree = 1 + sum_rho count (layers.py:99) per candidate
    for (int i = beg + tid; i < end; i += GBS)
      degree_add(S, reinterpret_cast<uint32_t *>(&S.u.b.cnt[S.u.b.map[(int)(w[i].k & p.emask) - lo]]), w[i].c,
                 p.rl.node_nrules[S.root + (int)(w[i].k >> p.ebits)]);
    __syncthreads();
    for (int s2 = tid; s2 < nc; s2 += GBS) {
      const float degf = (float)((double)(uint32_t)S.u.b.cnt[s2] + 1.0);
      atomicAdd(&S.sumlog, (unsigned long long)(long long)llrint((double)logf(degf) * 4294967296.0));
    }
    __syncthreads();
    return nc;
  }
  for (int i = beg + tid; i < end; i += GBS) atomicAdd(&S.u.b.cnt[S.u.b.map[(int)(w[i].k & p.emask) - lo]], 1);  // bucket sizes
  __syncthreads();
  for (int i = tid; i < WIN; i += GBS) S.u.b.off[i] = S.u.b.cnt[i];
  __syncthreads();
  scan_win(S.u.b.off, S.ws);
  // candidate records
  const int64_t qb = S.qbase;
  for (int s2 = tid; s2 < nc; s2 += GBS) {
    p.cand[cbase + s2] = make_int4(S.u.b.st[s2], (int32_t)(qb + beg + S.u.b.off[s2]), S.u.b.cnt[s2], 0);
  }
  __syncthreads();
  for (int i = tid; i < WIN; i += GBS) S.u.b.cnt[i] = 0;
  __syncthreads();
  PSTAMP(1);
  for (int i = beg + tid; i < end; i += GBS) {  // scatter (node, count) into the buckets
    const int s2 = S.u.b.map[(int)(w[i].k & p.emask) - lo];
    const int64_t pos = qb + beg + S.u.b.off[s2] + atomicAdd(&S.u.b.cnt[s2], 1);
    p.bent[pos] = make_int2(S.root + (int)(w[i].k >> p.ebits), (int)w[i].c);
  }
  __syncthreads();
  PSTAMP(2);
  return nc;
}

// Sparse windows: contributions [beg, end) of consecutive entity windows
// (end - beg <= HB_LOAD) bucketed through an LDS hash keyed by entity —
// O(contributions) work and six barriers, against the dense window_pass's
// O(WIN) passes.  Candidates are emitted in ascending entity order (ranked
// through an LDS bitmap of the pass's entity range, as window_pass's slots
// are), so a query's candidate records — and the scoring pass's score
// accesses, one lane per candidate — run along the score row; a range wider
// than SORT_WORDS x 32 entities keeps the hash order (nothing downstream
// depends on the order for correctness: scores scatter by entity, PNA's mean
// and the digests are order-independent sums).
__device__ __forceinline__ int hb_slot(Smem &S, int t, bool insert) {
  uint32_t h = hash32((uint32_t)t) >> (32 - WBITS);
#pragma unroll 1
  for (int probe = 0; probe < HB; ++probe) {
    const int k = insert ? atomicCAS(&S.u.c.key[h], EMPTY, t) : S.u.c.key[h];
    if (k == t || (insert && k == EMPTY)) return (int)h;
    h = (h + 1) & (HB - 1);
  }
  return -1;  // unreachable: at most HB_LOAD < HB distinct keys
}

__device__ int hash_pass(const KParams &p, Smem &S, const Ent *w, int beg, int end, int64_t cbase,
                         bool degree_only, int lo, int hi) {
  // w: contributions (a = entity, b = node, c = count), window-sorted or raw;
  // every entity lies in [lo, hi)
  const int tid = threadIdx.x;
  const int w0 = lo >> 5, nw = ((hi - 1) >> 5) - w0 + 1;
  // candidates in ascending entity order (the reference's nonzero order, and
  // neighbouring lanes of the scoring pass then touch neighbouring score entries)
  const bool by_rank = !degree_only && nw <= SORT_WORDS;
  for (int i = tid; i < HB; i += GBS) {
    S.u.c.key[i] = EMPTY;
    S.u.c.cnt[i] = 0;
    S.u.c.off[i] = 0;
  }
  if (by_rank)
    for (int i = tid; i < nw; i += GBS) S.sbits[i] = 0u;
  __syncthreads();
  for (int i = beg + tid; i < end; i += GBS) atomicAdd(&S.u.c.cnt[hb_slot(S, (int)(w[i].k & p.emask), true)], 1);
  __syncthreads();
  constexpr int PER = HB / GBS;
  int loc[PER];
  int nc;
  if (by_rank) {
    for (int i = tid; i < HB; i += GBS) {
      const int k = S.u.c.key[i];
      if (k != EMPTY) atomicOr(&S.sbits[(k >> 5) - w0], 1u << (k & 31));
    }
    __syncthreads();
    // rank of a bit = popcounts of the words before it + of its word below it
    const int per = (nw + GBS - 1) / GBS;
    int sum = 0;
    for (int j = 0; j < per; ++j) {
      const int i = tid * per + j;
      if (i < nw) sum += __popc(S.sbits[i]);
    }
    int base = block_scan(sum, S.ws, nc);
    for (int j = 0; j < per; ++j) {
      const int i = tid * per + j;
      if (i < nw) {
        S.spre[i] = (unsigned short)base;
        base += __popc(S.sbits[i]);
      }
    }
    __syncthreads();
    for (int i = tid; i < HB; i += GBS) {
      const int k = S.u.c.key[i];
      if (k != EMPTY) {
        const int kk = k - (w0 << 5), wd = kk >> 5;
        const int rank = S.spre[wd] + __popc(S.sbits[wd] & ((1u << (kk & 31)) - 1u));
        S.u.c.cid[i] = rank;
        S.u.c.off[rank] = S.u.c.cnt[i];  // bucket sizes in rank order
      }
    }
    __syncthreads();
    // exclusive scan of the bucket sizes (rank order): off[rank] = bucket start
    int s2 = 0;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      loc[j] = S.u.c.off[tid * PER + j];
      s2 += loc[j];
    }
    int tot;
    int run = block_scan(s2, S.ws, tot);
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      S.u.c.off[tid * PER + j] = run;
      run += loc[j];
    }
    __syncthreads();
  } else {
    // one scan of (bucket size << 12 | occupied): bucket offsets and candidate ids (hash order)
    int sum = 0;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int sidx = tid * PER + j;
      loc[j] = (S.u.c.cnt[sidx] << 12) | (S.u.c.key[sidx] != EMPTY ? 1 : 0);
      sum += loc[j];
    }
    int total;
    int run = block_scan(sum, S.ws, total);
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int sidx = tid * PER + j;
      S.u.c.off[sidx] = run >> 12;
      S.u.c.cid[sidx] = run & 4095;
      run += loc[j];
    }
    nc = total & 4095;
    __syncthreads();
  }
  if (degree_only) {
    // PNA sweep 1: degree = 1 + sum_rho count (layers.py:99) per candidate
    for (int i = tid; i < HB; i += GBS) S.u.c.cnt[i] = 0;
    __syncthreads();
    for (int i = beg + tid; i < end; i += GBS)
      degree_add(S, reinterpret_cast<uint32_t *>(&S.u.c.cnt[hb_slot(S, (int)(w[i].k & p.emask), false)]), w[i].c,
                 p.rl.node_nrules[S.root + (int)(w[i].k >> p.ebits)]);
    __syncthreads();
    for (int i = tid; i < HB; i += GBS) {
      if (S.u.c.key[i] != EMPTY) {
        const float degf = (float)((double)(uint32_t)S.u.c.cnt[i] + 1.0);
        atomicAdd(&S.sumlog, (unsigned long long)(long long)llrint((double)logf(degf) * 4294967296.0));
      }
    }
    __syncthreads();
    return nc;
  }
  // bucket start of hash slot i: off is indexed by rank (by_rank) or by slot
  const int64_t qb = S.qbase;
  for (int i = tid; i < HB; i += GBS) {
    if (S.u.c.key[i] != EMPTY) {
      const int cid = S.u.c.cid[i];
      const int64_t c = cbase + cid;
      p.cand[c] = make_int4(S.u.c.key[i], (int32_t)(qb + beg + S.u.c.off[by_rank ? cid : i]), S.u.c.cnt[i], 0);
    }
  }
  __syncthreads();
  for (int i = tid; i < HB; i += GBS) S.u.c.cnt[i] = 0;
  __syncthreads();
  for (int i = beg + tid; i < end; i += GBS) {  // scatter (node, count) into the buckets
    const int sl2 = hb_slot(S, (int)(w[i].k & p.emask), false);
    const int64_t pos = qb + beg + S.u.c.off[by_rank ? S.u.c.cid[sl2] : sl2] + atomicAdd(&S.u.c.cnt[sl2], 1);
    p.bent[pos] = make_int2(S.root + (int)(w[i].k >> p.ebits), (int)w[i].c);
  }
  __syncthreads();
  return nc;
}

// Counting sort of the contributions by entity window into fn/fv/fc[0]
// (free during phase B), then window_pass over every non-empty window.
__device__ int candidates_phase(const KParams &p, Smem &S, const Slot &sl, int P, bool degree_only, bool sorted) {
  const int tid = threadIdx.x;
  // all contributions fit one hash pass: no window sort (it exists only to
  // bound the hash load) — one read of the raw list instead of a sorted copy
  if (P <= HB_LOAD) return P > 0 ? hash_pass(p, S, sl.ct, 0, P, S.qbase, degree_only, 0, p.g.E) : 0;
  const int nwin = (p.g.E + WIN - 1) >> WBITS;
  if (!sorted) {
    for (int i = tid; i < nwin; i += GBS) S.whist[i] = 0;
    __syncthreads();
    for (int i = tid; i < P; i += GBS) atomicAdd(&S.whist[(int)(sl.ct[i].k & p.emask) >> WBITS], 1);
    __syncthreads();
    if (tid == 0) {
      int acc = 0;
      for (int w = 0; w < nwin; ++w) {
        const int c = S.whist[w];
        S.wbeg[w] = acc;
        S.wfill[w] = acc;
        acc += c;
      }
      S.wbeg[nwin] = acc;
    }
    __syncthreads();
    for (int i = tid; i < P; i += GBS) {
      const Ent ce = sl.ct[i];
      const int t = (int)(ce.k & p.emask);
      const int pos = atomicAdd(&S.wfill[t >> WBITS], 1);
      sl.f(0)[pos] = ce;
    }
    wg_sync_global();
  }
  // consecutive windows are merged while their contributions fit one hash
  // pass; a window heavier than that takes the dense direct-mapped pass
  int ncand = 0;
  for (int w = 0; w < nwin;) {
    const int beg = S.wbeg[w];
    if (S.wbeg[w + 1] - beg > HB_LOAD) {
      ncand += window_pass(p, S, sl, w << WBITS, beg, S.wbeg[w + 1], S.qbase + ncand, degree_only);
      ++w;
      continue;
    }
    int w2 = w + 1;
    while (w2 < nwin && S.wbeg[w2 + 1] - beg <= HB_LOAD) ++w2;
    if (S.wbeg[w2] > beg)
      ncand += hash_pass(p, S, sl.f(0), beg, S.wbeg[w2], S.qbase + ncand, degree_only, w << WBITS,
                         min(w2 << WBITS, p.g.E));
    w = w2;
  }
  return ncand;
}

__device__ __forceinline__ void flag_error(const KParams &p, unsigned int *hdr, Smem &S, int q) {
  atomicOr(&hdr[H_STATUS], S.err ? 2u : 1u);
  if (S.err) {
    atomicOr(&hdr[H_ERRBITS], (unsigned)S.err);
    atomicExch(&hdr[H_ERRQ], (unsigned)q);
  }
  if (p.n_cand) p.n_cand[q] = S.err ? -2 : -1;
}

#ifndef RNNL_GROUND_MINB
#define RNNL_GROUND_MINB 1
#endif
template <int AGG>
__global__ __launch_bounds__(GBS, RNNL_GROUND_MINB) void ground_kernel(KParams p) {
  __shared__ Smem S;
  const int tid = threadIdx.x;
  unsigned int *hdr = reinterpret_cast<unsigned int *>(p.ws);
  unsigned long long *pool_ctr = reinterpret_cast<unsigned long long *>(p.ws + 64);
  const Slot sl = make_slot(p.slots, blockIdx.x, p.fcap, p.pcap);
  for (int s = tid; s < HCAP; s += GBS) {
    S.u.a.key[s] = EMPTY;
    S.u.a.val[s] = 0u;
  }
  unsigned long long pr[6] = {0, 0, 0, 0, 0, 0};
  if (tid < 8) S.tp[tid] = 0ull;
  unsigned long long t_q = 0, t_a = 0;
  __syncthreads();
#pragma unroll 1
  while (true) {
    if (tid == 0) S.q = (int)atomicAdd(&hdr[H_DEQUEUE], 1u);
    __syncthreads();
    const int q = S.q;
    if (q >= p.nq) break;
    if (p.prof && tid == 0) t_q = __builtin_amdgcn_s_memtime();
    const int h = (int)p.all_h[q];
    const int r = (int)p.all_r[q];
    const int root = p.rl.head_root[r];
    if (root < 0) {
      if (tid == 0) {
        p.n_cand[q] = 0;
        p.q_base[q] = 0;
      }
      __syncthreads();
      continue;
    }
    int rm_src = -1, rm_dst = -1;
    if (p.etr) {
      const int64_t e = p.etr[q];
      if (e >= 0) {
        const int base = p.g.edge_base[r];
        rm_src = p.g.edge_src[base + e];
        rm_dst = p.g.edge_dst[base + e];
      }
    }
    if (tid == 0) {
      S.t0 = __builtin_amdgcn_s_memrealtime();
      S.err = 0;
      S.root = root;
      S.np = 0;
      S.nd = 0;
      S.ovf = 0;
      S.sumlog = 0ull;
    }
    __syncthreads();
    if (p.prof && tid == 0) t_a = __builtin_amdgcn_s_memtime();
    ground_query(p, S, sl, h, r, root, rm_src, rm_dst);
    wg_sync_global();
    if (p.prof && tid == 0) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      pr[1] += t - t_a;
      pr[0] += t_a - t_q;
      t_a = t;
    }
    const int P = S.np;
    if (tid == 0 && !S.ovf && !S.err && P <= p.pcap) {
      // reserve the query's pool run: P bucket entries and <= P candidate records
      const unsigned long long b = atomicAdd(pool_ctr, (unsigned long long)P);
      if (b + P > (unsigned long long)p.pool_cap) S.ovf = 1;
      S.qbase = (long long)b;
    }
    __syncthreads();
    if (S.ovf || P > p.pcap || S.err) {
      for (int s = tid; s < HCAP; s += GBS) {  // leave the LDS hash clean for the next query
        S.u.a.key[s] = EMPTY;
        S.u.a.val[s] = 0u;
      }
      if (tid == 0) flag_error(p, hdr, S, q);
      __syncthreads();
      continue;
    }
    bool sorted = false;
    if constexpr (AGG == RNNL_AGG_PNA) {
      // sweep 1: per-query mean of log(degree) over candidates (layers.py:109-116)
      const int nc1 = candidates_phase(p, S, sl, P, true, false);
      sorted = true;
      if (tid == 0) {
        const double sum = (double)(long long)S.sumlog / 4294967296.0;
        p.q_scale[q] = (float)((float)sum / fmaxf((float)nc1, 1e-6f));
      }
    }
    const int ncand = candidates_phase(p, S, sl, P, false, sorted);
    __syncthreads();  // S.err: a PNA degree may have hit 2^32 in phase B
    if (tid == 0 && S.err) {
      flag_error(p, hdr, S, q);
    } else if (tid == 0) {
      p.n_cand[q] = ncand;
      atomicAdd(reinterpret_cast<unsigned long long *>(hdr + H_NCAND), (unsigned long long)ncand);
      p.q_base[q] = S.qbase;
      if (p.prof) {
        pr[2] += __builtin_amdgcn_s_memtime() - t_a;
        pr[3] += 1;
        pr[4] += P;
        pr[5] += ncand;
      }
    }
    for (int s = tid; s < HCAP; s += GBS) {  // restore the phase-A hash (phase B reused its LDS)
      S.u.a.key[s] = EMPTY;
      S.u.a.val[s] = 0u;
    }
    __syncthreads();
  }
  if (p.prof && tid == 0) {
#pragma unroll
    for (int k = 0; k < 6; ++k) atomicAdd(&p.prof[k], pr[k]);
#pragma unroll
    for (int k = 0; k < 6; ++k) atomicAdd(&p.prof[6 + k], S.tp[k]);
  }
}

// ---------------------------------------------------------------- K2: scoring
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

template <int AGG>
__device__ __forceinline__ float score_one(const KParams &p, const float *__restrict__ wl, const float *relb,
                                           int beg, int cnt, float mean_scale, uint64_t *dig_out, int t) {
  static_assert(AGG == RNNL_AGG_PNA, "the SUM aggregator scores in score_sum_kernel / score_sum_memo_kernel");
  using L = WL<AGG>;
  long long a1[16], a2[16];
  float mn[16], mx[16];
#pragma unroll
  for (int d = 0; d < 16; ++d) {
    a1[d] = 0;
    a2[d] = 0;
    mn[d] = __builtin_huge_valf();
    mx[d] = -__builtin_huge_valf();
  }
  long long deg = 0;
  uint64_t fp = 0, csum = 0;
  for (int e = beg; e < beg + cnt; ++e) {
    const int2 be = p.bent[e];
    const int n = be.x;
    const long long c = (uint32_t)be.y;
    csum += (uint64_t)c;
    const int *rec = reinterpret_cast<const int *>(p.node_w + (int64_t)n * kStridePna);
#pragma unroll
    for (int d = 0; d < 16; ++d) a1[d] += c * rec[d];
#pragma unroll
    for (int d = 0; d < 16; ++d) a2[d] += c * rec[16 + d];
#if !RNNL_PNA_SPLIT
    const float *fr = reinterpret_cast<const float *>(rec + 32);
#pragma unroll
    for (int d = 0; d < 16; ++d) {
      mn[d] = fminf(mn[d], fr[d]);
      mx[d] = fmaxf(mx[d], fr[16 + d]);
    }
#endif
    deg += c * p.rl.node_nrules[n];
    if (dig_out) fp += (uint64_t)c * p.rl.node_fp[n];
  }
#if RNNL_PNA_SPLIT
  // min / max in a second walk over the entries (fewer registers live in either walk)
  asm volatile("" ::: "memory");
  for (int e = beg; e < beg + cnt; ++e) {
    const float *fr = reinterpret_cast<const float *>(p.node_w + (int64_t)p.bent[e].x * kStridePna) + 32;
#pragma unroll
    for (int d = 0; d < 16; ++d) {
      mn[d] = fminf(mn[d], fr[d]);
      mx[d] = fmaxf(mx[d], fr[16 + d]);
    }
  }
#endif
  if (dig_out) *dig_out = mix64((uint64_t)t ^ mix64((uint64_t)deg ^ mix64(fp)));
  if (csum >> 33) flag_acc_range(p);  // |int32 record| < 2^30: int64 sums exact below 2^33 total count
#ifdef RNNL_SCORE_NOMLP  // diagnostic build: the node-sum gather alone
  return (float)a1[0] + (float)a1[15];
#endif
  const unsigned int *trailer = reinterpret_cast<const unsigned int *>(p.node_w + (int64_t)p.rl.n_nodes * kStridePna);
  const double inv1 = ldexp(1.0, -(int)trailer[1]), inv2 = ldexp(1.0, -(int)trailer[4]);
  // FuncToNode (pna): mean/min/max/std x {1, s, 1/s} -> Linear(192,16) (layers.py:93-123).
  // Each dim's four features are folded into the 16 outputs as soon as they
  // exist (input j = (block * 16 + d) * 3 + s3; weights in LDS as [j][o]).
  const float degf = (float)(deg + 1);
  const float dcl = fmaxf(degf, 1e-6f);
  const float scale = logf(degf) / fmaxf(mean_scale, 1e-6f);
  const float sc[3] = {1.0f, scale, 1.0f / fmaxf(scale, 1e-6f)};
  float x1[16];
#pragma unroll
  for (int o = 0; o < 16; ++o) x1[o] = 0.f;
#pragma unroll
  for (int d = 0; d < 16; ++d) {
    const float s = (float)((double)a1[d] * inv1);
    const float sq = (float)((double)a2[d] * inv2);
    const float mean = s / dcl;
    const float sqm = sq / dcl;
    const float fv[4] = {mean, mn[d], mx[d], sqrtf(fmaxf(sqm - mean * mean, 1e-6f))};
#pragma unroll
    for (int b = 0; b < 4; ++b) {
#pragma unroll
      for (int s3 = 0; s3 < 3; ++s3) {
        asm volatile("" ::: "memory");  // one input's 16 weights live at a time
        const float v = fv[b] * sc[s3];
        const float *w = wl + L::ADDW + ((b * 16 + d) * 3 + s3) * 16;
#pragma unroll
        for (int o = 0; o < 16; ++o) x1[o] = fmaf(v, w[o], x1[o]);
      }
    }
  }
#pragma unroll
  for (int o = 0; o < 16; ++o) x1[o] += wl[L::ADDB + o];
  // LayerNorm(16) + ReLU (layers.py:74-75 / 124-125)
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
  for (int d = 0; d < 16; ++d) x1[d] = fmaxf((x1[d] - mu) * rstd * wl[L::LNW + d] + wl[L::LNB + d], 0.f);
  // score_model: Linear(32,128) [relation half folded into relb], ReLU, Linear(128,1)
  float out = 0.f;
#pragma unroll 2
  for (int o = 0; o < 128; ++o) {
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc = fmaf(x1[i], wl[L::S0X + o * 16 + i], acc);
    acc = fmaxf(acc + relb[o], 0.f);
    out = fmaf(acc, wl[L::S1W + o], out);
  }
  return out + wl[L::S1B];
}

// Exact int64 sums of count x record word (off + d) over a candidate's bucket
// entries, one dim at a time (few registers), as the double the one-walk
// score_one converts them to: the fallback of score_one_2walk's fp64 sums.
__device__ __forceinline__ void exact_sums(const KParams &p, int beg, int cnt, int off, double (&a)[16]) {
#pragma unroll
  for (int d = 0; d < 16; ++d) {
    long long acc = 0;
#pragma unroll 1
    for (int e = beg; e < beg + cnt; ++e) {
      const int2 be = p.bent[e];
      acc += (long long)(uint32_t)be.y * reinterpret_cast<const int *>(p.node_w + (int64_t)be.x * kStridePna)[off + d];
    }
    a[d] = (double)acc;
  }
}

// Two walks over the candidate's bucket entries, one per half of the node
// record, each folding its features into the Linear(192, 16) sums as soon
// as it ends: walk 1 the mean and min features (Σ c·x, min), walk 2 the max
// and std ones (Σ c·x², max; std from walk 1's means).  Only one half's
// accumulators (16 int64 + 16 float) and the 16 sums and 16 means are live
// in either walk instead of both halves' (the one-walk score_one holds ~250
// VGPRs, 2 waves/SIMD); the entries are read twice (the second walk's loads
// hit L2).  Same arithmetic per feature as score_one; only the order in
// which the 192 inputs are summed into the 16 outputs differs.
// Materialise the 16 sums here, and keep later loads below: the FMAs of one
// Linear input complete before the next input's weights are read (a plain
// memory clobber orders the loads but lets the scheduler hoist all of them
// ahead of the FMAs, which spills).
__device__ __forceinline__ void pin16(float (&x)[16]) {
  asm volatile("" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]),
               "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]), "+v"(x[14]), "+v"(x[15])
               :
               : "memory");
}

// score_one_2walk up to score_model: x1 = ReLU(LayerNorm(Linear(192, 16)(features)))
// (returns false in the diagnostic RNNL_SCORE_NOMLP build, `diag` then holds the output).
template <int AGG>
__device__ __forceinline__ bool pna_hidden_2walk(const KParams &p, const float *wl, int beg, int cnt,
                                                 float mean_scale, uint64_t *dig_out, int t, float (&x1)[16],
                                                 float &diag) {
  static_assert(AGG == RNNL_AGG_PNA, "the SUM aggregator scores in score_sum_kernel / score_sum_memo_kernel");
  using L = WL<AGG>;
  const unsigned int *trailer = reinterpret_cast<const unsigned int *>(p.node_w + (int64_t)p.rl.n_nodes * kStridePna);
  double a[16];  // exact: see the walk
  float m[16];
#pragma unroll
  for (int d = 0; d < 16; ++d) {
    a[d] = 0;
    m[d] = __builtin_huge_valf();
  }
  long long deg = 0;
  uint64_t fp = 0, csum = 0;
#pragma unroll 1
  for (int e = beg; e < beg + cnt; ++e) {
    const int2 be = p.bent[e];
    const int n = be.x;
    const long long c = (uint32_t)be.y;
    const double cd = (double)(uint32_t)be.y;
    csum += (uint64_t)c;
    const int *rec = reinterpret_cast<const int *>(p.node_w + (int64_t)n * kStridePna);
    const float *fr = reinterpret_cast<const float *>(rec + 32);
#pragma unroll
    for (int d = 0; d < 16; ++d) {
      a[d] = fma(cd, (double)rec[d], a[d]);
      m[d] = fminf(m[d], fr[d]);
    }
    deg += c * p.rl.node_nrules[n];
    if (dig_out) fp += (uint64_t)c * p.rl.node_fp[n];
  }
  if (dig_out) *dig_out = mix64((uint64_t)t ^ mix64((uint64_t)deg ^ mix64(fp)));
  if (csum >> 33) flag_acc_range(p);  // |int32 record| < 2^30: int64 sums exact below 2^33 total count
  // |record| < 2^30, so below a total count of 2^23 every product and partial
  // sum is an integer under 2^53 and the fp64 FMAs are exact: a[d] is the
  // int64 sum itself.  Past it (rare), exact int64 sums one dim at a time.
  if (csum >> 23) exact_sums(p, beg, cnt, 0, a);
  const double inv1 = ldexp(1.0, -(int)trailer[1]);
#ifdef RNNL_SCORE_NOMLP  // diagnostic build: the two walks without the Linear / MLP
  {
    float z = (float)deg;
#pragma unroll
    for (int d = 0; d < 16; ++d) z += (float)(a[d] * inv1) + m[d];
#pragma unroll
    for (int d = 0; d < 16; ++d) {
      a[d] = 0;
      m[d] = -__builtin_huge_valf();
    }
    for (int e = beg; e < beg + cnt; ++e) {
      const int2 be = p.bent[e];
      const double cd = (double)(uint32_t)be.y;
      const int *rec = reinterpret_cast<const int *>(p.node_w + (int64_t)be.x * kStridePna);
#pragma unroll
      for (int d = 0; d < 16; ++d) {
        a[d] = fma(cd, (double)rec[16 + d], a[d]);
        m[d] = fmaxf(m[d], reinterpret_cast<const float *>(rec + 48)[d]);
      }
    }
#pragma unroll
    for (int d = 0; d < 16; ++d) z += (float)a[d] + m[d];
    diag = z * wl[L::S1B];
    return false;
  }
#endif
  // FuncToNode (pna): mean/min/max/std x {1, s, 1/s} -> Linear(192,16) (layers.py:93-123);
  // input j = (block * 16 + d) * 3 + s3, weights in LDS as [j][o]
  const float degf = (float)(deg + 1);
  const float dcl = fmaxf(degf, 1e-6f);
  const float scale = logf(degf) / fmaxf(mean_scale, 1e-6f);
  const float sc[3] = {1.0f, scale, 1.0f / fmaxf(scale, 1e-6f)};
  float mean[16];
#pragma unroll
  for (int o = 0; o < 16; ++o) x1[o] = 0.f;
#pragma unroll
  for (int d = 0; d < 16; ++d) {
    const float s = (float)(a[d] * inv1);
    mean[d] = s / dcl;
    const float fv[2] = {mean[d], m[d]};
#pragma unroll
    for (int b = 0; b < 2; ++b) {
#pragma unroll
      for (int s3 = 0; s3 < 3; ++s3) {
        pin16(x1);  // one input's 16 weights live at a time: its FMAs end before the next loads
        const float v = fv[b] * sc[s3];
        const float *w = wl + L::ADDW + ((b * 16 + d) * 3 + s3) * 16;
#pragma unroll
        for (int o = 0; o < 16; ++o) x1[o] = fmaf(v, w[o], x1[o]);
      }
    }
  }
  // walk 2: the squared half of the records and the max
#pragma unroll
  for (int d = 0; d < 16; ++d) {
    a[d] = 0;
    m[d] = -__builtin_huge_valf();
  }
  asm volatile("" ::: "memory");
#pragma unroll 1
  for (int e = beg; e < beg + cnt; ++e) {
    const int2 be = p.bent[e];
    const double cd = (double)(uint32_t)be.y;
    const int *rec = reinterpret_cast<const int *>(p.node_w + (int64_t)be.x * kStridePna);
    const float *fr = reinterpret_cast<const float *>(rec + 48);
#pragma unroll
    for (int d = 0; d < 16; ++d) {
      a[d] = fma(cd, (double)rec[16 + d], a[d]);
      m[d] = fmaxf(m[d], fr[d]);
    }
  }
  if (csum >> 23) exact_sums(p, beg, cnt, 16, a);
  const double inv2 = ldexp(1.0, -(int)trailer[4]);
#pragma unroll
  for (int d = 0; d < 16; ++d) {
    const float sq = (float)(a[d] * inv2);
    const float sqm = sq / dcl;
    const float fv[2] = {m[d], sqrtf(fmaxf(sqm - mean[d] * mean[d], 1e-6f))};
#pragma unroll
    for (int b = 0; b < 2; ++b) {
#pragma unroll
      for (int s3 = 0; s3 < 3; ++s3) {
        pin16(x1);  // one input's 16 weights live at a time: its FMAs end before the next loads
        const float v = fv[b] * sc[s3];
        const float *w = wl + L::ADDW + (((b + 2) * 16 + d) * 3 + s3) * 16;
#pragma unroll
        for (int o = 0; o < 16; ++o) x1[o] = fmaf(v, w[o], x1[o]);
      }
    }
  }
#pragma unroll
  for (int o = 0; o < 16; ++o) x1[o] += wl[L::ADDB + o];
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
  for (int d = 0; d < 16; ++d) x1[d] = fmaxf((x1[d] - mu) * rstd * wl[L::LNW + d] + wl[L::LNB + d], 0.f);
  return true;
}

template <int AGG>
__device__ __forceinline__ float score_one_2walk(const KParams &p, const float *wl, const float *relb,
                                                 int beg, int cnt, float mean_scale, uint64_t *dig_out, int t) {
  using L = WL<AGG>;
  float x1[16], diag = 0.f;
  if (!pna_hidden_2walk<AGG>(p, wl, beg, cnt, mean_scale, dig_out, t, x1, diag)) return diag;
  float out = 0.f;
#pragma unroll 2
  for (int o = 0; o < 128; ++o) {
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc = fmaf(x1[i], wl[L::S0X + o * 16 + i], acc);
    acc = fmaxf(acc + relb[o], 0.f);
    out = fmaf(acc, wl[L::S1W + o], out);
  }
  return out + wl[L::S1B];
}

// score_model (Linear(32, 128) with the relation half folded into relb, ReLU,
// Linear(128, 1)) for the wave's 64 candidates at once on the bf16 matrix
// cores: 64 x 16 hidden inputs times the 16 x 128 layer-0 weights as
// v_mfma_f32_16x16x16_bf16 tiles, every fp32 operand split exactly into three
// bf16 parts (v = v0 + v1 + v2) and the six part products with i + j <= 2 kept
// (the dropped ones are below 2^-24 of |x w|), accumulated in fp32.  On the
// VALU this layer is 2,048 FMAs per candidate — a third of the PNA pass's
// VALU instructions, and those take RotatE's issue slots when the pass runs
// beside it; the matrix pipe runs beside the VALU.  Tile layout
// (lane = 16 k + i16): A row i16 (candidate rt * 16 + i16), K 4k .. 4k + 3;
// B K 4k .. 4k + 3, column i16 (output ct * 16 + i16); D rows 4k + j, column
// i16.  Whole-wave (EXEC full): dead lanes pass x1 = 0 and ignore the result.
// sb: [8 column tiles][3 parts][64 lanes] B fragments (built once per block);
// sx: the wave's [3 parts][64 candidates][4 K-groups] staging; so: [64].
typedef short pna_s16x4 __attribute__((ext_vector_type(4)));
typedef float pna_f32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ unsigned short pna_bf16(float v) { return __builtin_bit_cast(unsigned short, (__bf16)v); }
__device__ __forceinline__ void pna_split3(float v, unsigned short (&q)[3]) {
  q[0] = pna_bf16(v);
  const float r1 = v - __uint_as_float((unsigned)q[0] << 16);
  q[1] = pna_bf16(r1);
  q[2] = pna_bf16(r1 - __uint_as_float((unsigned)q[1] << 16));
}
__device__ __forceinline__ uint2 pna_pack4(const unsigned short (&q)[4][3], int part) {
  return make_uint2(q[0][part] | ((unsigned)q[1][part] << 16), q[2][part] | ((unsigned)q[3][part] << 16));
}
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// score_mlp_mfma's B fragments from the packed weights: column tile ct, lane
// (k, i16) holds W[ct * 16 + i16][4k .. 4k + 3] as 3 bf16 parts
__device__ __forceinline__ void build_mlp_b(const float *__restrict__ W, uint2 *sb, int tid) {
  for (int i = tid; i < 8 * 64; i += BS) {
    const int ct = i >> 6, l = i & 63, o = ct * 16 + (l & 15), k0 = (l >> 4) * 4;
    unsigned short q[4][3];
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) pna_split3(W[W_S0X + o * 16 + k0 + kk], q[kk]);
#pragma unroll
    for (int part = 0; part < 3; ++part) sb[(ct * 3 + part) * 64 + l] = pna_pack4(q, part);
  }
}
template <int AGG>
__device__ __forceinline__ float score_mlp_mfma(const float (&x1)[16], const uint2 *__restrict__ sb, uint2 *sx,
                                                float *so, const float *relb, const float *wl, int lane) {
  using L = WL<AGG>;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    unsigned short q[4][3];
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) pna_split3(x1[4 * g + kk], q[kk]);
#pragma unroll
    for (int part = 0; part < 3; ++part) sx[(part * 64 + lane) * 4 + g] = pna_pack4(q, part);
  }
  wave_lds_sync();
  const int k = lane >> 4, i16 = lane & 15;
#pragma unroll 1
  for (int rt = 0; rt < 4; ++rt) {
    pna_s16x4 a[3];
#pragma unroll
    for (int part = 0; part < 3; ++part)
      a[part] = __builtin_bit_cast(pna_s16x4, sx[(part * 64 + rt * 16 + i16) * 4 + k]);
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
    for (int ct = 0; ct < 8; ++ct) {
      pna_s16x4 b[3];
#pragma unroll
      for (int part = 0; part < 3; ++part) b[part] = __builtin_bit_cast(pna_s16x4, sb[(ct * 3 + part) * 64 + lane]);
      const float rb = relb[ct * 16 + i16], w1 = wl[L::S1W + ct * 16 + i16];
      pna_f32x4 d = {0.f, 0.f, 0.f, 0.f};
      d = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a[2], b[0], d, 0, 0, 0);  // smallest parts first
      d = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a[1], b[1], d, 0, 0, 0);
      d = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a[0], b[2], d, 0, 0, 0);
      d = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a[1], b[0], d, 0, 0, 0);
      d = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a[0], b[1], d, 0, 0, 0);
      d = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a[0], b[0], d, 0, 0, 0);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] = fmaf(fmaxf(d[j] + rb, 0.f), w1, acc[j]);
    }
    // each lane holds 8 of the 128 output terms of rows 4k + j: sum over the
    // 16 lanes of its K-group (xor 1, 2, 4, 8 stays inside the group)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float v = acc[j];
      v += __shfl_xor(v, 1);
      v += __shfl_xor(v, 2);
      v += __shfl_xor(v, 4);
      v += __shfl_xor(v, 8);
      if (i16 == 0) so[rt * 16 + 4 * k + j] = v;
    }
  }
  wave_lds_sync();
  const float out = so[lane] + wl[L::S1B];
  wave_lds_sync();  // sx / so are rewritten by the next call
  return out;
}

// One walk over a candidate's bucket entries for 8 dims (d0 .. d0 + 7) of
// one half of the node records: the exact sums of count x record word
// (fp64, exact below a total count of 2^23, else the int64 fallback) and the
// min (half 0) / max (half 1) of the float words.
// STATS (the first walk): also the degree sum, the digest fingerprint and
// the count total.
template <int HALF, bool STATS>
__device__ __forceinline__ void pna_walk8(const KParams &p, int beg, int cnt, int d0, uint64_t &csum, long long &deg,
                                          uint64_t &fp, bool want_fp, double (&a)[8], float (&m)[8]) {
#pragma unroll
  for (int d = 0; d < 8; ++d) {
    a[d] = 0;
    m[d] = HALF == 0 ? __builtin_huge_valf() : -__builtin_huge_valf();
  }
#pragma unroll 1
  for (int e = beg; e < beg + cnt; ++e) {
    const int2 be = p.bent[e];
    const double cd = (double)(uint32_t)be.y;
    if constexpr (STATS) {
      const long long c = (uint32_t)be.y;
      csum += (uint64_t)c;
      deg += c * p.rl.node_nrules[be.x];
      if (want_fp) fp += (uint64_t)c * p.rl.node_fp[be.x];
    }
    const int *rec = reinterpret_cast<const int *>(p.node_w + (int64_t)be.x * kStridePna) + HALF * 16 + d0;
    const float *fr = reinterpret_cast<const float *>(rec + 32);
#pragma unroll
    for (int d = 0; d < 8; ++d) {
      a[d] = fma(cd, (double)rec[d], a[d]);
      m[d] = HALF == 0 ? fminf(m[d], fr[d]) : fmaxf(m[d], fr[d]);
    }
  }
  if (csum >> 23) {  // exact int64 sums one dim at a time (rare)
#pragma unroll
    for (int d = 0; d < 8; ++d) {
      long long acc = 0;
#pragma unroll 1
      for (int e = beg; e < beg + cnt; ++e) {
        const int2 be = p.bent[e];
        acc += (long long)(uint32_t)be.y *
               reinterpret_cast<const int *>(p.node_w + (int64_t)be.x * kStridePna)[HALF * 16 + d0 + d];
      }
      a[d] = (double)acc;
    }
  }
}

__device__ __forceinline__ void pin8(float (&x)[8]) {
  asm volatile("" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7])
               :
               : "memory");
}

// score_one_2walk with each walk split in two 8-dim walks (four walks over
// the entries): only 8 fp64 sums and 8 min / max are live at a time, which
// takes the PNA scoring pass from 168 to ~100 VGPRs (more waves beside
// RotatE).  The 192 Linear inputs are folded into the 16 outputs in the
// same order as score_one_2walk (mean, min of dims 0..15, then max, std of
// dims 0..15), so the scores are bitwise the same.
__device__ __forceinline__ float score_one_4walk(const KParams &p, const float *wl, const float *relb, int beg,
                                                 int cnt, float mean_scale, uint64_t *dig_out, int t) {
  using L = WL<RNNL_AGG_PNA>;
  const unsigned int *trailer = reinterpret_cast<const unsigned int *>(p.node_w + (int64_t)p.rl.n_nodes * kStridePna);
  long long deg = 0;
  uint64_t fp = 0, csum = 0;
  double a[8];
  float m[8];
  // walk 1 also sums the degree, the digest fingerprint and the count total
  pna_walk8<0, true>(p, beg, cnt, 0, csum, deg, fp, dig_out != nullptr, a, m);
  if (dig_out) *dig_out = mix64((uint64_t)t ^ mix64((uint64_t)deg ^ mix64(fp)));
  if (csum >> 33) flag_acc_range(p);
  const double inv1 = ldexp(1.0, -(int)trailer[1]), inv2 = ldexp(1.0, -(int)trailer[4]);
  const float degf = (float)(deg + 1);
  const float dcl = fmaxf(degf, 1e-6f);
  const float scale = logf(degf) / fmaxf(mean_scale, 1e-6f);
  const float sc[3] = {1.0f, scale, 1.0f / fmaxf(scale, 1e-6f)};
  float x1[16], mean[16];
#pragma unroll
  for (int o = 0; o < 16; ++o) x1[o] = 0.f;
  // walks 1-2: sums of x (means) and min, dims 0..7 then 8..15
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    if (h) pna_walk8<0, false>(p, beg, cnt, 8, csum, deg, fp, false, a, m);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int d = h * 8 + j;
      mean[d] = (float)(a[j] * inv1) / dcl;
      const float fv[2] = {mean[d], m[j]};
#pragma unroll
      for (int b = 0; b < 2; ++b) {
#pragma unroll
        for (int s3 = 0; s3 < 3; ++s3) {
          pin16(x1);
          const float v = fv[b] * sc[s3];
          const float *w = wl + L::ADDW + ((b * 16 + d) * 3 + s3) * 16;
#pragma unroll
          for (int o = 0; o < 16; ++o) x1[o] = fmaf(v, w[o], x1[o]);
        }
      }
    }
  }
  // walks 3-4: sums of x^2 (std) and max, dims 0..7 then 8..15
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    pna_walk8<1, false>(p, beg, cnt, h * 8, csum, deg, fp, false, a, m);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int d = h * 8 + j;
      const float sqm = (float)(a[j] * inv2) / dcl;
      const float fv[2] = {m[j], sqrtf(fmaxf(sqm - mean[d] * mean[d], 1e-6f))};
#pragma unroll
      for (int b = 0; b < 2; ++b) {
#pragma unroll
        for (int s3 = 0; s3 < 3; ++s3) {
          pin16(x1);
          const float v = fv[b] * sc[s3];
          const float *w = wl + L::ADDW + (((b + 2) * 16 + d) * 3 + s3) * 16;
#pragma unroll
          for (int o = 0; o < 16; ++o) x1[o] = fmaf(v, w[o], x1[o]);
        }
      }
    }
  }
#pragma unroll
  for (int o = 0; o < 16; ++o) x1[o] += wl[L::ADDB + o];
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
  for (int d = 0; d < 16; ++d) x1[d] = fmaxf((x1[d] - mu) * rstd * wl[L::LNW + d] + wl[L::LNB + d], 0.f);
  float out = 0.f;
#pragma unroll 2
  for (int o = 0; o < 128; ++o) {
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc = fmaf(x1[i], wl[L::S0X + o * 16 + i], acc);
    acc = fmaxf(acc + relb[o], 0.f);
    out = fmaf(acc, wl[L::S1W + o], out);
  }
  return out + wl[L::S1B];
}

// Measured on WN18RR (config 3, round 3): the four-walk form at 4 waves/SIMD
// 22.4 ms/step, at 3 waves 22.0, the two-walk form (190 VGPRs, 2 waves) 21.1
// — the extra entry walks cost more than the occupancy gains beside RotatE.
// Kept for A/B (RNNL_PNA_4WALK=1); bitwise the same scores.
#ifndef RNNL_PNA_4WALK
#define RNNL_PNA_4WALK 0
#endif

#ifndef RNNL_PNA_SPLIT
#define RNNL_PNA_SPLIT 0
#endif
#ifndef RNNL_PNA_2WALK
#define RNNL_PNA_2WALK 1
#endif
#ifndef RNNL_PNA_WAVES
#define RNNL_PNA_WAVES 1
#endif
template <int AGG>
__global__ __launch_bounds__(BS) __attribute__((amdgpu_waves_per_eu(RNNL_PNA_WAVES, 8))) void score_kernel(
    KParams p, const float *__restrict__ W) {
  using L = WL<AGG>;
  __shared__ __attribute__((aligned(16))) float s_w[L::N];
  __shared__ float s_relb[128];
  __shared__ int s_q;
  __shared__ unsigned long long s_dig;
  const int tid = threadIdx.x;
  unsigned int *hdr = reinterpret_cast<unsigned int *>(p.ws);
  check_node_table(p, reinterpret_cast<const unsigned int *>(
                          p.node_w + (int64_t)p.rl.n_nodes * (AGG == RNNL_AGG_SUM ? kStrideSum : kStridePna)));
  for (int i = tid; i < L::N; i += BS) {
    float v = 0.f;
    if (i < L::ADDB) v = W[W_ADDW + (i % 16) * L::KIN + i / 16];  // add_w transposed: [input j][output o]
    else if (i < L::LNW) v = W[W_ADDB + i - L::ADDB];
    else if (i < L::LNB) v = W[W_LNW + i - L::LNW];
    else if (i < L::S0X) v = W[W_LNB + i - L::LNB];
    else if (i < L::S1W) v = W[W_S0X + i - L::S0X];
    else if (i < L::S1B) v = W[W_S1W + i - L::S1W];
    else if (i == L::S1B) v = W[W_S1B];
    s_w[i] = v;
  }
#pragma unroll 1
  while (true) {
    __syncthreads();
    if (tid == 0) {
      s_q = (int)atomicAdd(&hdr[H_DEQUEUE2], 1u);
      s_dig = 0ull;
    }
    __syncthreads();
    const int q = s_q;
    if (q >= p.nq) break;
    const int nc = p.n_cand[q];
    if (nc <= 0) {
      if (tid == 0 && p.digest && nc == 0) p.digest[q] = 0;
      continue;
    }
    const int r = (int)p.all_r[q];
    if (tid < 128) {
      // relation half of score_model.layers.0 folded into a per-query bias
      float acc = p.s0_b[tid];
      for (int i = 0; i < 16; ++i) acc = fmaf(p.s0_w[tid * 32 + 16 + i], p.rel_emb[r * 16 + i], acc);
      s_relb[tid] = acc;
    }
    __syncthreads();
    const int64_t qb = p.q_base[q];
    const float ms = AGG == RNNL_AGG_PNA ? p.q_scale[q] : 0.f;
    for (int s = tid; s < nc; s += BS) {
      const int4 cr = p.cand[qb + s];
      const int t = cr.x;
      uint64_t dg = 0;
      // keep the loop-invariant LDS weight reads inside the loop (hoisted,
      // they would pin ~200 VGPRs and starve occupancy)
      asm volatile("" ::: "memory");
#if RNNL_PNA_2WALK
      const float out = score_one_2walk<AGG>(p, s_w, s_relb, cr.y, cr.z, ms, p.digest ? &dg : nullptr, t);
#else
      const float out = score_one<AGG>(p, s_w, s_relb, cr.y, cr.z, ms,
                                       p.digest ? &dg : nullptr, t);
#endif
      if (p.digest) atomicAdd(&s_dig, (unsigned long long)dg);
      if (p.cand_out) {  // deferred: added once the base score exists (deferred_store)
        deferred_store(p, q, qb + s, t, out);
        continue;
      }
      const int64_t idx = (int64_t)q * p.g.E + t;
      if (p.feature == RNNL_FEATURE_NONE)
        p.score[idx] = out;
      else
        p.score[idx] = out + (p.base_row ? p.base_row[t] : p.score[idx]);
      if (p.mask) p.mask[idx] = 1;
    }
    __syncthreads();
    if (tid == 0 && p.digest) p.digest[q] = s_dig;
  }
}

// ---------------------------------------------------------------- scoring chunks
// The scoring passes' unit of work: one wave x one chunk of <= 64 consecutive
// candidates of one query.  The chunk list p.chunks (query, first candidate) is
// in ROW order — eval and train rows come in same-relation batches, so waves
// walking the list rarely change relation — and is built after the grounding
// by two small kernels: per 256-row block the chunk total (chunk_sum_kernel),
// then per block its prefix, a block scan and the entries (chunk_fill_kernel).
// The total goes to hdr[H_CHUNKS].
constexpr int CHB = 256;  // rows per chunk-list block (small blocks: they launch beside RotatE)

__device__ __forceinline__ int row_chunks(const KParams &p, int q) {
  const int nc = q < p.nq ? p.n_cand[q] : 0;
  return nc > 0 ? (nc + 63) >> 6 : 0;
}

__global__ __launch_bounds__(CHB) void chunk_sum_kernel(KParams p, int *__restrict__ bsum) {
  __shared__ int s_ws[CHB / 64];
  int v = row_chunks(p, blockIdx.x * CHB + threadIdx.x);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if ((threadIdx.x & 63) == 0) s_ws[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    int t = 0;
    for (int w = 0; w < CHB / 64; ++w) t += s_ws[w];
    bsum[blockIdx.x] = t;
  }
}

__global__ __launch_bounds__(CHB) void chunk_fill_kernel(KParams p, const int *__restrict__ bsum) {
  __shared__ int s_ws[CHB / 64];
  __shared__ long long s_pb[CHB / 64], s_pt[CHB / 64];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  // this block's prefix and the list total from the per-block totals
  long long pb = 0, pt = 0;
  for (int k = tid; k < (int)gridDim.x; k += CHB) {
    const int v = bsum[k];
    pt += v;
    if (k < (int)blockIdx.x) pb += v;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    pb += __shfl_xor(pb, o, 64);
    pt += __shfl_xor(pt, o, 64);
  }
  if (lane == 0) {
    s_pb[wid] = pb;
    s_pt[wid] = pt;
  }
  const int q = blockIdx.x * CHB + tid;
  const int n = row_chunks(p, q);
  int v = n;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(v, o, 64);
    if (lane >= o) v += y;
  }
  if (lane == 63) s_ws[wid] = v;
  __syncthreads();
  if (tid == 0) {
    int acc = 0;
    for (int w = 0; w < CHB / 64; ++w) {
      const int t = s_ws[w];
      s_ws[w] = acc;
      acc += t;
    }
    long long base = 0, total = 0;
    for (int w = 0; w < CHB / 64; ++w) {
      base += s_pb[w];
      total += s_pt[w];
    }
    s_pb[0] = base;
    if (blockIdx.x == 0)
      *reinterpret_cast<unsigned long long *>(reinterpret_cast<unsigned int *>(p.ws) + H_CHUNKS) = total;
  }
  __syncthreads();
  const long long off = s_pb[0] + s_ws[wid] + v - n;
  for (int k = 0; k < n; ++k) p.chunks[off + k] = make_int2(q, k << 6);
}

static void launch_chunk_list(const KParams &p, hipStream_t st) {
  const unsigned nb = (unsigned)((p.nq + CHB - 1) / CHB);
  int *bsum = reinterpret_cast<int *>(p.chunks + p.chunk_cap);  // nb ints after the list (layout)
  hipLaunchKernelGGL(chunk_sum_kernel, dim3(nb), dim3(CHB), 0, st, p, bsum);
  hipLaunchKernelGGL(chunk_fill_kernel, dim3(nb), dim3(CHB), 0, st, p, (const int *)bsum);
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

// PNA scoring over chunks (default; RNNL_PNA_CHUNKED=0 keeps score_kernel<PNA>).
// The unit of work is one wave x one chunk of <= 64 consecutive candidates of
// one query (lane = candidate), p.chunks[0 .. hdr[H_CHUNKS]).  Waves dequeue chunks independently, so a
// query with 17k candidates (WN18RR) is spread over ~280 waves instead of
// holding one workgroup while the rest of the grid drains; no workgroup
// barrier per query.  Each wave folds its relation's half of
// score_model.layers.0 into its own LDS slice when the relation changes.
// Same arithmetic per candidate as score_kernel<PNA> (score_one_2walk).
#ifndef RNNL_PNA_CK
#define RNNL_PNA_CK 1
#endif
// score_model on the matrix cores in the chunked PNA pass (score_mlp_mfma);
// -DRNNL_PNA_MFMA=0 builds the VALU form
#ifndef RNNL_PNA_MFMA
#define RNNL_PNA_MFMA 1
#endif
constexpr int PNA_CK = RNNL_PNA_CK;  // chunks per dequeue

// 4 waves/SIMD for the four-walk scoring (128 VGPRs, no spills; 138 unforced
// = 3 waves)
#ifndef RNNL_PNA_CHUNK_WAVES
#define RNNL_PNA_CHUNK_WAVES (RNNL_PNA_4WALK ? 4 : RNNL_PNA_WAVES)
#endif
__global__ __launch_bounds__(BS) __attribute__((amdgpu_waves_per_eu(RNNL_PNA_CHUNK_WAVES, 8))) void score_pna_chunk_kernel(
    KParams p, const float *__restrict__ W) {
  using L = WL<RNNL_AGG_PNA>;
  __shared__ __attribute__((aligned(16))) float s_w[L::N];
  __shared__ float s_relb[BS / 64][128];
#if RNNL_PNA_MFMA
  __shared__ uint2 s_b[8 * 3 * 64];           // score_model layer-0 B fragments (score_mlp_mfma)
  __shared__ uint2 s_x[BS / 64][3 * 64 * 4];  // per wave: hidden inputs, 3 bf16 parts
  __shared__ float s_o[BS / 64][64];
#endif
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  unsigned int *hdr = reinterpret_cast<unsigned int *>(p.ws);
  check_node_table(p, reinterpret_cast<const unsigned int *>(p.node_w + (int64_t)p.rl.n_nodes * kStridePna));
  for (int i = tid; i < L::N; i += BS) {
    float v = 0.f;
    if (i < L::ADDB) v = W[W_ADDW + (i % 16) * L::KIN + i / 16];  // add_w transposed: [input j][output o]
    else if (i < L::LNW) v = W[W_ADDB + i - L::ADDB];
    else if (i < L::LNB) v = W[W_LNW + i - L::LNW];
    else if (i < L::S0X) v = W[W_LNB + i - L::LNB];
    else if (i < L::S1W) v = W[W_S0X + i - L::S0X];
    else if (i < L::S1B) v = W[W_S1W + i - L::S1W];
    else if (i == L::S1B) v = W[W_S1B];
    s_w[i] = v;
  }
#if RNNL_PNA_MFMA
  build_mlp_b(W, s_b, tid);
#endif
  __syncthreads();  // the only workgroup barrier: waves run independently from here
  const long long nchunks = (long long)*reinterpret_cast<const unsigned long long *>(hdr + H_CHUNKS);
  float *relb = s_relb[wv];
  int cur_r = -1;
  unsigned c = 0, cend = 0;  // wave-uniform: the dequeued chunk range
#pragma unroll 1
  for (;; ++c) {
    if (c == cend) next_chunks(&hdr[H_DEQUEUE2], nchunks, PNA_CK, c, cend);
    if ((long long)c >= nchunks) break;
    const int2 ck = p.chunks[c];
    const int q = __builtin_amdgcn_readfirstlane(ck.x);
    const int s0 = __builtin_amdgcn_readfirstlane(ck.y);
    const int r = __builtin_amdgcn_readfirstlane((int)p.all_r[q]);
    if (r != cur_r) {
      // relation half of score_model.layers.0 folded into a per-wave bias
      __builtin_amdgcn_wave_barrier();  // the previous chunk's reads of the slice are done
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int o = lane + 64 * j;
        float acc = p.s0_b[o];
        for (int i = 0; i < 16; ++i) acc = fmaf(p.s0_w[o * 32 + 16 + i], p.rel_emb[r * 16 + i], acc);
        relb[o] = acc;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      cur_r = r;
    }
    const int nc = p.n_cand[q];
    const int s = s0 + lane;
#if RNNL_PNA_MFMA && !RNNL_PNA_4WALK && !defined(RNNL_SCORE_NOMLP)
    // every lane reaches the whole-wave score_model; lanes past the chunk's
    // candidates carry x1 = 0 and store nothing
    const bool live = s < nc;
    int64_t qb = 0;
    int t = 0;
    float x1[16], diag;
#pragma unroll
    for (int d = 0; d < 16; ++d) x1[d] = 0.f;
    if (live) {
      qb = p.q_base[q];
      const float ms = p.q_scale[q];
      const int4 cr = p.cand[qb + s];
      t = cr.x;
      uint64_t dg = 0;
      asm volatile("" ::: "memory");  // keep the LDS weight reads inside the loop (see score_kernel)
      pna_hidden_2walk<RNNL_AGG_PNA>(p, s_w, cr.y, cr.z, ms, p.digest ? &dg : nullptr, t, x1, diag);
      if (p.digest) atomicAdd(reinterpret_cast<unsigned long long *>(p.digest + q), (unsigned long long)dg);
    }
    const float out = score_mlp_mfma<RNNL_AGG_PNA>(x1, s_b, s_x[wv], s_o[wv], relb, s_w, lane);
    if (!live) continue;
#else
    if (s >= nc) continue;
    const int64_t qb = p.q_base[q];
    const float ms = p.q_scale[q];
    const int4 cr = p.cand[qb + s];
    const int t = cr.x;
    uint64_t dg = 0;
    asm volatile("" ::: "memory");  // keep the LDS weight reads inside the loop (see score_kernel)
#if RNNL_PNA_4WALK
    const float out = score_one_4walk(p, s_w, relb, cr.y, cr.z, ms, p.digest ? &dg : nullptr, t);
#else
    const float out = score_one_2walk<RNNL_AGG_PNA>(p, s_w, relb, cr.y, cr.z, ms, p.digest ? &dg : nullptr, t);
#endif
    if (p.digest) atomicAdd(reinterpret_cast<unsigned long long *>(p.digest + q), (unsigned long long)dg);
#endif
    if (p.cand_out) {  // deferred: added once the base score exists (deferred_store)
      deferred_store(p, q, qb + s, t, out);
      continue;
    }
    const int64_t idx = (int64_t)q * p.g.E + t;
    if (p.feature == RNNL_FEATURE_NONE)
      p.score[idx] = out;
    else
      p.score[idx] = out + (p.base_row ? p.base_row[t] : p.score[idx]);
    if (p.mask) p.mask[idx] = 1;
  }
}

// ---------------------------------------------------------------- K2 (sum): staged scoring
// FuncToNodeSum path.  The node records of a query's head relation (only its
// leaves: <= a few hundred, f32 x 16 each) are staged into LDS once per run of
// same-relation queries, so the per-entry gather reads LDS instead of ~128 B
// of L2/MALL per (candidate, node) entry.  Sums are accumulated in fp64 from
// the exact products count x f32: the result is independent of the entry
// order (which comes from LDS atomics) short of a double rounding.
#ifndef RNNL_QCHUNK
#define RNNL_QCHUNK 1
#endif
#ifndef RNNL_SCORE_WG_PER_CU
#define RNNL_SCORE_WG_PER_CU 8
#endif
constexpr int QCHUNK = RNNL_QCHUNK;  // consecutive queries dequeued together (same relation in batch order)

struct SumStage {
  float *rec;      // [max_leaves][16]
  int *nr;         // [max_leaves] rules ending at the leaf
  uint2 *fp;       // [max_leaves] node fingerprint (digest)
  short *map;      // [max_head_nodes] node - root -> leaf index
};

__host__ __device__ inline int64_t sum_stage_bytes(int max_leaves, int max_head_nodes) {
  return (int64_t)max_leaves * (64 + 4 + 8) + (int64_t)max_head_nodes * 2 + 64;
}

#ifndef RNNL_MAC
#define RNNL_MAC 2  // count x record MAC: 0 C++ int64, 1 v_mad_i64_i32, 2 exact fp64 (default; measured fastest)
#endif
#if RNNL_MAC == 2
// The candidate's exact feature sums in fp64: with |record| < 2^30 every
// count x record product below 2^53 is an exact double and so is every
// partial sum while sum(count) < 2^23, so accd equals the int64 sum bit for
// bit (one v_cvt_f64_i32 + one v_fma_f64 per element instead of two 64-bit
// integer multiply-adds and their fix-ups); a candidate whose counts sum
// past that takes the int64 walk below.
template <bool STAGED, bool DIGEST>
__device__ __forceinline__ void gather_sum_int64(const KParams &p, const SumStage &st, int root, int beg, int cnt,
                                                 float inv_scale, float f[16], long long &deg, uint64_t &fp);
template <bool STAGED, bool DIGEST>
__device__ __forceinline__ void gather_sum(const KParams &p, const SumStage &st, int root, int beg, int cnt,
                                           float inv_scale, float f[16], long long &deg, uint64_t &fp) {
  if constexpr (STAGED) {  // the LDS-staged variant keeps the int64 walk
    gather_sum_int64<STAGED, DIGEST>(p, st, root, beg, cnt, inv_scale, f, deg, fp);
    return;
  }
  double accd[16];
#pragma unroll
  for (int d = 0; d < 16; ++d) accd[d] = 0.0;
  deg = 0;
  fp = 0;
  uint64_t csum = 0;
  for (int e = beg; e < beg + cnt; ++e) {
    const int2 be = p.bent[e];
    const int n = be.x;
    const uint32_t cu = (uint32_t)be.y;
    csum += cu;
    const int *x = reinterpret_cast<const int *>(p.node_w + (int64_t)n * kStrideSum);
    const double cd = (double)cu;
#pragma unroll
    for (int d = 0; d < 16; ++d) accd[d] = fma(cd, (double)x[d], accd[d]);
    if constexpr (DIGEST) {
      deg += (long long)cu * p.rl.node_nrules[n];
      fp += (uint64_t)cu * p.rl.node_fp[n];
    }
  }
  if (csum >= (1ull << 23)) {  // rare: the exact int64 walk
    gather_sum_int64<STAGED, DIGEST>(p, st, root, beg, cnt, inv_scale, f, deg, fp);
    return;
  }
#pragma unroll
  for (int d = 0; d < 16; ++d) f[d] = (float)(accd[d] * (double)inv_scale);
}
#define gather_sum gather_sum_int64
#endif
template <bool STAGED, bool DIGEST>
__device__ __forceinline__ void gather_sum(const KParams &p, const SumStage &st, int root, int beg, int cnt,
                                           float inv_scale, float f[16], long long &deg, uint64_t &fp) {
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
    const int *x;
    int nr;
    uint64_t nf;
    nr = 0;
    nf = 0;
    if constexpr (STAGED) {
      const int li = st.map[n - root];
      x = reinterpret_cast<const int *>(st.rec) + li * 16;
      if constexpr (DIGEST) {
        nr = st.nr[li];
        nf = ((uint64_t)st.fp[li].y << 32) | st.fp[li].x;
      }
    } else {
      x = reinterpret_cast<const int *>(p.node_w + (int64_t)n * kStrideSum);
#ifdef RNNL_DIAG_NOGATHER  // diagnostic build: one shared record instead of the per-node gather
      x = reinterpret_cast<const int *>(p.node_w);
#endif
      if constexpr (DIGEST) {  // the digest's degree / fingerprint terms only
        nr = p.rl.node_nrules[n];
        nf = p.rl.node_fp[n];
      }
    }
    // (the compiler folds the two forms into the uint32 one: two v_mad_u64_u32
    // per element; an explicit v_mad_i64_i32 measured slower, 16.2 -> 16.6 ms)
#if RNNL_MAC == 1
    if (cu < 0x80000000u) {
#pragma unroll
      for (int d = 0; d < 16; ++d) {
        long long r;
        unsigned long long carry;
        asm("v_mad_i64_i32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(carry) : "v"((int)cu), "v"(x[d]), "v"(acc[d]));
        acc[d] = r;
      }
    } else {
#pragma unroll
      for (int d = 0; d < 16; ++d) acc[d] += c * x[d];
    }
#else
    if (cu < 0x80000000u) {
      const int ci = (int)cu;
#pragma unroll
      for (int d = 0; d < 16; ++d) acc[d] += (long long)ci * x[d];
    } else {
#pragma unroll
      for (int d = 0; d < 16; ++d) acc[d] += c * x[d];
    }
#endif
    deg += c * nr;
    fp += (uint64_t)c * nf;
  }
  if (csum >> 33) flag_acc_range(p);  // |int32 record| < 2^30: int64 sums exact below 2^33 total count
#pragma unroll
  for (int d = 0; d < 16; ++d) f[d] = (float)((double)acc[d] * (double)inv_scale);
}
#if RNNL_MAC == 2
#undef gather_sum
#endif

// The feature of a candidate whose only bucket entry is (n, c): gather_sum's
// arithmetic for that single entry (the memo of score_sum_memo_kernel).
template <bool DIGEST>
__device__ __forceinline__ void gather_sum_entry(const KParams &p, int n, uint32_t cu, float inv_scale, float f[16],
                                                 long long &deg, uint64_t &fp) {
  const int *x = reinterpret_cast<const int *>(p.node_w + (int64_t)n * kStrideSum);
  const long long c = cu;
#pragma unroll
  for (int d = 0; d < 16; ++d) f[d] = (float)((double)(0ll + c * x[d]) * (double)inv_scale);
  deg = DIGEST ? c * p.rl.node_nrules[n] : 0;
  fp = DIGEST ? (uint64_t)c * p.rl.node_fp[n] : 0;
}

// FuncToNodeSum tail: x1 = ReLU(LayerNorm(Linear(16, 16)(f)))
__device__ __forceinline__ void sum_hidden(const float *__restrict__ wl, const float f[16], float (&x1)[16]) {
  using L = WL<RNNL_AGG_SUM>;
#pragma unroll
  for (int o = 0; o < 16; ++o) {
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc = fmaf(f[i], wl[L::ADDW + o * 16 + i], acc);
    x1[o] = acc + wl[L::ADDB + o];
  }
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
  for (int d = 0; d < 16; ++d) x1[d] = fmaxf((x1[d] - mu) * rstd * wl[L::LNW + d] + wl[L::LNB + d], 0.f);
}

// FuncToNodeSum tail + score_model on the candidate's feature sums
__device__ __forceinline__ float mlp_sum(const float *__restrict__ wl, const float *relb, const float f[16]) {
  using L = WL<RNNL_AGG_SUM>;
#ifdef RNNL_DIAG_NOMLP  // diagnostic build: the MLP's cost bounded (every caller)
  return f[0] + f[15];
#endif
  float x1[16];
  sum_hidden(wl, f, x1);
  float out = 0.f;
#pragma unroll 2
  for (int o = 0; o < 128; ++o) {
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc = fmaf(x1[i], wl[L::S0X + o * 16 + i], acc);
    acc = fmaxf(acc + relb[o], 0.f);
    out = fmaf(acc, wl[L::S1W + o], out);
  }
  return out + wl[L::S1B];
}

#ifndef RNNL_SCORE_WAVES
#define RNNL_SCORE_WAVES 8
#endif
template <bool STAGED, bool DIGEST>
__global__ __launch_bounds__(BS) __attribute__((amdgpu_waves_per_eu(RNNL_SCORE_WAVES, 8))) void score_sum_kernel(
    KParams p, const float *__restrict__ W) {
  using L = WL<RNNL_AGG_SUM>;
  extern __shared__ __attribute__((aligned(16))) unsigned char dyn[];
  float *s_w = reinterpret_cast<float *>(dyn);
  float *s_relb = s_w + L::N;
  SumStage st{};
  if constexpr (STAGED) {
    unsigned char *b = dyn + (L::N + 128) * 4;
    st.fp = reinterpret_cast<uint2 *>(b);
    b += (int64_t)p.rl.max_leaves * 8;
    st.rec = reinterpret_cast<float *>(b);
    b += (int64_t)p.rl.max_leaves * 64;
    st.nr = reinterpret_cast<int *>(b);
    b += (int64_t)p.rl.max_leaves * 4;
    st.map = reinterpret_cast<short *>(b);
  }
  __shared__ int s_q0, s_r;
  __shared__ unsigned long long s_dig;
  const int tid = threadIdx.x;
  unsigned int *hdr = reinterpret_cast<unsigned int *>(p.ws);
  for (int i = tid; i < L::N; i += BS) {
    float v = 0.f;
    if (i < L::ADDB) v = W[W_ADDW + i];
    else if (i < L::LNW) v = W[W_ADDB + i - L::ADDB];
    else if (i < L::LNB) v = W[W_LNW + i - L::LNW];
    else if (i < L::S0X) v = W[W_LNB + i - L::LNB];
    else if (i < L::S1W) v = W[W_S0X + i - L::S0X];
    else if (i < L::S1B) v = W[W_S1W + i - L::S1W];
    else if (i == L::S1B) v = W[W_S1B];
    s_w[i] = v;
  }
  if (tid == 0) s_r = -1;
  check_node_table(p, reinterpret_cast<const unsigned int *>(p.node_w + (int64_t)p.rl.n_nodes * kStrideSum));
  const int shift = (int)reinterpret_cast<const unsigned int *>(p.node_w + (int64_t)p.rl.n_nodes * kStrideSum)[1];
  const float inv_scale = ldexpf(1.f, -shift);
#pragma unroll 1
  while (true) {
    __syncthreads();
    if (tid == 0) s_q0 = (int)atomicAdd(&hdr[H_DEQUEUE2], (unsigned)QCHUNK);
    __syncthreads();
    const int q0 = s_q0;
    if (q0 >= p.nq) break;
    for (int q = q0; q < min(q0 + QCHUNK, p.nq); ++q) {
      const int nc = p.n_cand[q];
      if (nc <= 0) {
        if (tid == 0 && p.digest && nc == 0) p.digest[q] = 0;
        continue;
      }
      const int r = (int)p.all_r[q];
      const int root = p.rl.head_root[r];
      if (r != s_r) {
        __syncthreads();  // every lane is done with the previous relation's stage and bias
        if (tid < 128) {
          // relation half of score_model.layers.0 folded into a per-query bias
          float acc = p.s0_b[tid];
          for (int i = 0; i < 16; ++i) acc = fmaf(p.s0_w[tid * 32 + 16 + i], p.rel_emb[r * 16 + i], acc);
          s_relb[tid] = acc;
        }
        if constexpr (STAGED) {
          const int lp = p.rl.head_leaf_ptr[r], nl = p.rl.head_leaf_ptr[r + 1] - lp;
          for (int i = tid; i < p.rl.head_nodes[r]; i += BS) st.map[i] = (short)p.rl.node_leaf[root + i];
          for (int i = tid; i < nl * 16; i += BS) {
            const int n = p.rl.head_leaf_node[lp + i / 16];
            st.rec[i] = reinterpret_cast<const float *>(p.node_w + (int64_t)n * kStrideSum)[i % 16];  // int32 bits
          }
          for (int i = tid; i < nl; i += BS) {
            const int n = p.rl.head_leaf_node[lp + i];
            st.nr[i] = p.rl.node_nrules[n];
            const uint64_t f = p.rl.node_fp[n];
            st.fp[i] = make_uint2((unsigned)f, (unsigned)(f >> 32));
          }
        }
        if (tid == 0) {
          s_r = r;
          s_dig = 0ull;
        }
        __syncthreads();
      } else if (p.digest) {
        __syncthreads();
        if (tid == 0) s_dig = 0ull;
        __syncthreads();
      }
      const int64_t qb = p.q_base[q];
      for (int s2 = tid; s2 < nc; s2 += BS) {
        const int4 cr = p.cand[qb + s2];
        const int t = cr.x;
        float f[16];
        long long deg;
        uint64_t fp;
        const int64_t idx = (int64_t)q * p.g.E + t;
        // the base score's load is issued before the gather (its latency hides under it)
#ifdef RNNL_DIAG_NOSCORE
        const float base = 0.f;
#else
        const float base = (p.feature == RNNL_FEATURE_NONE || p.cand_out) ? 0.f
                           : p.base_row                                    ? p.base_row[t]
                                                                           : p.score[idx];
#endif
#ifdef RNNL_DIAG_NOENTRIES  // diagnostic build: no bucket-entry walk
        for (int d = 0; d < 16; ++d) f[d] = (float)(cr.z * d);
        deg = 0;
        fp = 0;
#else
        gather_sum<STAGED, DIGEST>(p, st, root, cr.y, cr.z, inv_scale, f, deg, fp);
#endif
        if constexpr (DIGEST)
          atomicAdd(&s_dig, (unsigned long long)mix64((uint64_t)t ^ mix64((uint64_t)deg ^ mix64(fp))));
        // keep the loop-invariant LDS weight reads inside the loop (hoisted,
        // they would pin ~200 VGPRs and starve occupancy)
        asm volatile("" ::: "memory");
        const float out = mlp_sum(s_w, s_relb, f);
#ifdef RNNL_DIAG_NOSCORE  // diagnostic build: no score/mask traffic
        if (out == 1234.5f) p.score[idx] = base;
        continue;
#endif
        if (p.cand_out) {  // deferred: added once the base score exists (deferred_store)
          deferred_store(p, q, qb + s2, t, out);
          continue;
        }
        p.score[idx] = p.feature == RNNL_FEATURE_NONE ? out : out + base;
        if (p.mask) p.mask[idx] = 1;
      }
      if (DIGEST) {
        __syncthreads();
        if (tid == 0) p.digest[q] = s_dig;
      }
    }
  }
}


// ---------------------------------------------------------------- K2 (sum): single-path memo
// Most candidates are reached by few paths; 38 % of the FB15k-237 test
// candidates by exactly one path of one rule-end node n (one bucket entry of
// count 1).  Their feature is n's record itself, so their score_model output
// depends on (head relation, n) only: memo_sum_kernel computes it once per
// launch for every leaf node of every head (131,883 MLPs instead of ~22 M).
// score_sum_memo_kernel sends those candidates down a short path (candidate
// record, one bucket entry, the memo: three loads and the store) and queues
// the others in LDS, running the full gather + MLP over full tiles of queued
// candidates — the MLP tiles are full, and a query needs ~62 % as many.  The
// memo entry is computed by the same code from the same integer record as
// the full path (gather_sum with one entry of count 1, mlp_sum), so the two
// paths give the same output for such a candidate.
__device__ __forceinline__ void load_sum_weights(float *s_w, const float *__restrict__ W) {
  using L = WL<RNNL_AGG_SUM>;
  for (int i = threadIdx.x; i < L::N; i += blockDim.x) {
    float v = 0.f;
    if (i < L::ADDB) v = W[W_ADDW + i];
    else if (i < L::LNW) v = W[W_ADDB + i - L::ADDB];
    else if (i < L::LNB) v = W[W_LNW + i - L::LNW];
    else if (i < L::S0X) v = W[W_LNB + i - L::LNB];
    else if (i < L::S1W) v = W[W_S0X + i - L::S0X];
    else if (i < L::S1B) v = W[W_S1W + i - L::S1W];
    else if (i == L::S1B) v = W[W_S1B];
    s_w[i] = v;
  }
}

__device__ __forceinline__ void fold_relation_bias(const KParams &p, float *s_relb, int r) {
  if (threadIdx.x < 128) {
    // relation half of score_model.layers.0 folded into a per-query bias
    float acc = p.s0_b[threadIdx.x];
    for (int i = 0; i < 16; ++i) acc = fmaf(p.s0_w[threadIdx.x * 32 + 16 + i], p.rel_emb[r * 16 + i], acc);
    s_relb[threadIdx.x] = acc;
  }
}

// Launches with at most this many rows compute the memo only for the
// relations their rows hold (a scan of all_r per workgroup).
constexpr int MEMO_SCAN_ROWS = 2048;

// One workgroup per head relation with rules: memo[n] for its leaf nodes.
__global__ __launch_bounds__(BS) void memo_sum_kernel(KParams p, const float *__restrict__ W) {
  using L = WL<RNNL_AGG_SUM>;
  __shared__ __attribute__((aligned(16))) float s_w[L::N];
  __shared__ float s_relb[128];
  const int r = blockIdx.x;
  const int lp = p.rl.head_leaf_ptr[r], nl = p.rl.head_leaf_ptr[r + 1] - lp;
  if (nl <= 0) return;  // uniform
  if (p.nq <= MEMO_SCAN_ROWS) {
    // few rows (e.g. one reference batch): only the relations present need a memo
    bool any = false;
    for (int q = threadIdx.x; q < p.nq; q += BS) any |= (int)p.all_r[q] == r;
    if (!__syncthreads_or(any)) return;  // block-uniform
  }
  load_sum_weights(s_w, W);
  fold_relation_bias(p, s_relb, r);
  __syncthreads();
  const int shift = (int)reinterpret_cast<const unsigned int *>(p.node_w + (int64_t)p.rl.n_nodes * kStrideSum)[1];
  const float inv_scale = ldexpf(1.f, -shift);
  SumStage st{};
  for (int i = threadIdx.x; i < nl; i += BS) {
    const int n = p.rl.head_leaf_node[lp + i];
    float f[16];
    long long deg;
    uint64_t fp;
    // the full path's feature for a candidate with the single entry (n, 1)
    gather_sum_entry<false>(p, n, 1u, inv_scale, f, deg, fp);
    asm volatile("" ::: "memory");
    p.memo[n] = mlp_sum(s_w, s_relb, f);
  }
}

__device__ __forceinline__ void sum_write_out(const KParams &p, int q, int64_t ci, int t, float out, float base) {
  if (p.cand_out) {  // deferred: added once the base score exists (deferred_store)
    deferred_store(p, q, ci, t, out);
    return;
  }
  const int64_t idx = (int64_t)q * p.g.E + t;
  p.score[idx] = p.feature == RNNL_FEATURE_NONE ? out : out + base;
  if (p.mask) p.mask[idx] = 1;
}

__device__ __forceinline__ float sum_base(const KParams &p, int q, int t) {
  if (p.feature == RNNL_FEATURE_NONE || p.cand_out) return 0.f;
  return p.base_row ? p.base_row[t] : p.score[(int64_t)q * p.g.E + t];
}

template <bool DIGEST>
__global__ __launch_bounds__(BS) __attribute__((amdgpu_waves_per_eu(RNNL_SCORE_WAVES, 8))) void score_sum_memo_kernel(
    KParams p, const float *__restrict__ W) {
  using L = WL<RNNL_AGG_SUM>;
  __shared__ __attribute__((aligned(16))) float s_w[L::N];
  __shared__ float s_relb[128];
  __shared__ int s_queue[2 * BS];
  __shared__ int s_q, s_r, s_n;
  __shared__ unsigned long long s_dig;
  const int tid = threadIdx.x;
  unsigned int *hdr = reinterpret_cast<unsigned int *>(p.ws);
  load_sum_weights(s_w, W);
  if (tid == 0) s_r = -1;
  check_node_table(p, reinterpret_cast<const unsigned int *>(p.node_w + (int64_t)p.rl.n_nodes * kStrideSum));
  const int shift = (int)reinterpret_cast<const unsigned int *>(p.node_w + (int64_t)p.rl.n_nodes * kStrideSum)[1];
  const float inv_scale = ldexpf(1.f, -shift);
  SumStage st{};
#pragma unroll 1
  while (true) {
    __syncthreads();
    if (tid == 0) {
      s_q = (int)atomicAdd(&hdr[H_DEQUEUE2], 1u);
      s_dig = 0ull;
      s_n = 0;
    }
    __syncthreads();
    const int q = s_q;
    if (q >= p.nq) break;
    const int nc = p.n_cand[q];
    if (nc <= 0) {
      if (tid == 0 && DIGEST && nc == 0) p.digest[q] = 0;
      continue;
    }
    const int r = (int)p.all_r[q];
    const int root = p.rl.head_root[r];
    if (r != s_r) {
      fold_relation_bias(p, s_relb, r);
      __syncthreads();
      if (tid == 0) s_r = r;
    }
    const int64_t qb = p.q_base[q];
    for (int s0 = 0; s0 < nc; s0 += BS) {
      const int s2 = s0 + tid;
      if (s2 < nc) {
        const int4 cr = p.cand[qb + s2];
        bool queued = true;
        if (cr.z == 1) {
          const int2 be = p.bent[cr.y];
          if (be.y == 1) {  // one path of one leaf node: the memo
            queued = false;
            const float base = sum_base(p, q, cr.x);
            if constexpr (DIGEST)
              atomicAdd(&s_dig, (unsigned long long)mix64((uint64_t)cr.x ^
                                                          mix64((uint64_t)p.rl.node_nrules[be.x] ^
                                                                mix64(p.rl.node_fp[be.x]))));
            sum_write_out(p, q, qb + s2, cr.x, p.memo[be.x], base);
          }
        }
        if (queued) s_queue[atomicAdd(&s_n, 1)] = s2;
      }
      __syncthreads();
      const bool last = s0 + BS >= nc;
#pragma unroll 1
      while (true) {
        const int n = s_n;  // uniform (read after a barrier)
        if (!(n >= BS || (last && n > 0))) break;
        const int take = min(n, BS);
        if (tid < take) {
          const int c2 = s_queue[tid];
          const int4 cr = p.cand[qb + c2];
          const float base = sum_base(p, q, cr.x);  // issued before the gather: its latency hides under it
          float f[16];
          long long deg;
          uint64_t fp;
          gather_sum<false, DIGEST>(p, st, root, cr.y, cr.z, inv_scale, f, deg, fp);
          if constexpr (DIGEST)
            atomicAdd(&s_dig, (unsigned long long)mix64((uint64_t)cr.x ^ mix64((uint64_t)deg ^ mix64(fp))));
          // keep the loop-invariant LDS weight reads inside the loop (hoisted,
          // they would pin ~200 VGPRs and starve occupancy)
          asm volatile("" ::: "memory");
          sum_write_out(p, q, qb + c2, cr.x, mlp_sum(s_w, s_relb, f), base);
        }
        __syncthreads();  // every lane has read its queue entry
        const int rest = n - take;
        const int v = tid < rest ? s_queue[take + tid] : 0;
        __syncthreads();
        if (tid < rest) s_queue[tid] = v;
        if (tid == 0) s_n = rest;
        __syncthreads();
      }
    }
    if (DIGEST) {
      __syncthreads();
      if (tid == 0) p.digest[q] = s_dig;
    }
  }
}

// Pair memo.  A candidate's feature is the exact sum of count x record over
// its bucket entries, so candidates whose entries are equal get bit-identical
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

// SUM scoring over chunks (default; RNNL_SUM_CHUNKED=0 keeps
// score_sum_memo_kernel): one wave x one 64-candidate chunk of one query at a
// time (p.chunks, in row order), no
// workgroup barrier after the weight load.  Single-path candidates take the
// memo (three loads and the store); the others are compacted (ballot + prefix)
// into the wave's LDS queue of (query, pool index) and scored 64 at a time by
// the full gather + MLP, so the MLP runs on full waves; the queue is flushed
// early only when the next chunk's relation differs (the folded relation bias
// is per wave) and at the end.  Same arithmetic per candidate as
// score_sum_memo_kernel (wave_lds_sync: above, score_mlp_mfma).

// A candidate with more than BIG_ENTRIES bucket entries is gathered by the
// whole wave (lane i takes entries i, i + 64, ...; a butterfly sums the 16
// fp64 partials): its lane would otherwise walk the list alone, two dependent
// loads per entry, while the wave waits — on a one-batch launch the scoring
// time is the longest such walk.  The fp64 sums of exact count x record
// products are exact in any order, so the feature is the per-lane walk's bit
// for bit.  Up to BIG_SLOTS per round, their features staged in LDS.
#ifndef RNNL_BIG_ENTRIES
#define RNNL_BIG_ENTRIES 16
#endif
constexpr int BIG_ENTRIES = RNNL_BIG_ENTRIES;
constexpr int BIG_SLOTS = 16;

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
    const int *x = reinterpret_cast<const int *>(p.node_w + (int64_t)n * kStrideSum);
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

// COOP = false (large launches): each lane walks its own list — the
// cooperative rounds' registers spill at the 64-VGPR cap, which costs the
// throughput-bound launches more (RotatE step +0.8 ms) than the long walks.
template <bool DIGEST, bool COOP>
__device__ __forceinline__ void sum_chunk_flush(const KParams &p, const float *s_w, const float *relb,
                                                const int2 *queue, int m, float inv_scale, int r, int root,
                                                float *fbig) {
  const int lane = threadIdx.x & 63;
  if constexpr (!COOP) {
    if (lane < m) {
      const int2 it = queue[lane];
      const int4 cr = p.cand[it.y];
      const float base = sum_base(p, it.x, cr.x);  // issued before the gather: its latency hides under it
      float f[16];
      long long deg;
      uint64_t fp;
      SumStage st{};
      gather_sum<false, DIGEST>(p, st, 0, cr.y, cr.z, inv_scale, f, deg, fp);
      if constexpr (DIGEST)
        atomicAdd(reinterpret_cast<unsigned long long *>(p.digest + it.x),
                  (unsigned long long)mix64((uint64_t)cr.x ^ mix64((uint64_t)deg ^ mix64(fp))));
      asm volatile("" ::: "memory");  // keep the LDS weight reads inside (see score_sum_kernel)
      const float out = mlp_sum(s_w, relb, f);
      sum_write_out(p, it.x, it.y, cr.x, out, base);
      if (!DIGEST && p.ptab && cr.z <= 3) {
        const int2 z0 = make_int2(0, 0);
        const unsigned long long key = pair_key(p, r, root, cr.z, p.bent[cr.y], cr.z >= 2 ? p.bent[cr.y + 1] : z0,
                                                cr.z >= 3 ? p.bent[cr.y + 2] : z0);
        if (key != PAIR_NOKEY) pair_insert(p, key, out);
      }
    }
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
    if (go) {
      const float base = sum_base(p, it.x, cr.x);  // issued before the gather: its latency hides under it
      float f[16];
      long long deg;
      uint64_t fp;
      if (slot >= 0) {
#pragma unroll
        for (int d = 0; d < 16; ++d) f[d] = fbig[slot * 16 + d];
        deg = bdeg;
        fp = bfp;
      } else {
        SumStage st{};
        gather_sum<false, DIGEST>(p, st, 0, cr.y, cr.z, inv_scale, f, deg, fp);
      }
      if constexpr (DIGEST)
        atomicAdd(reinterpret_cast<unsigned long long *>(p.digest + it.x),
                  (unsigned long long)mix64((uint64_t)cr.x ^ mix64((uint64_t)deg ^ mix64(fp))));
      asm volatile("" ::: "memory");  // keep the LDS weight reads inside (see score_sum_kernel)
      const float out = mlp_sum(s_w, relb, f);
      sum_write_out(p, it.x, it.y, cr.x, out, base);
      if (!DIGEST && p.ptab && cr.z <= 3) {
        const int2 z0 = make_int2(0, 0);
        const unsigned long long key = pair_key(p, r, root, cr.z, p.bent[cr.y], cr.z >= 2 ? p.bent[cr.y + 1] : z0,
                                                cr.z >= 3 ? p.bent[cr.y + 2] : z0);
        if (key != PAIR_NOKEY) pair_insert(p, key, out);
      }
      todo = false;
    }
    wave_lds_sync();  // fbig is reused by the next round
    if (__ballot(todo) == 0ull) break;
  }
}


#ifndef RNNL_SUM_CK
#define RNNL_SUM_CK 8
#endif
constexpr int SUM_CK = RNNL_SUM_CK;  // chunks per dequeue

#ifndef RNNL_SCORE_PROF
#define RNNL_SCORE_PROF 0  // 1: phase clocks in score_sum_chunk_kernel (tools/score_phases.py)
#endif
constexpr bool kScoreProf = RNNL_SCORE_PROF;

template <bool DIGEST, bool COOP>
__global__ __launch_bounds__(BS) __attribute__((amdgpu_waves_per_eu(RNNL_SCORE_WAVES, 8))) void score_sum_chunk_kernel(
    KParams p, const float *__restrict__ W) {
  using L = WL<RNNL_AGG_SUM>;
  __shared__ __attribute__((aligned(16))) float s_w[L::N];
  __shared__ float s_relb[BS / 64][128];
  __shared__ int2 s_queue[BS / 64][128];
  __shared__ float s_fbig[BS / 64][COOP ? BIG_SLOTS * 16 : 1];  // long-list candidates' features (COOP flush)
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  unsigned int *hdr = reinterpret_cast<unsigned int *>(p.ws);
  // diagnostic phase clocks (-DRNNL_SCORE_PROF=1 builds, rnnl_debug_profile; prof[16..24]): per wave,
  // setup / classify / flush / total cycles, the chunks taken and the max total
  const unsigned long long t_start = kScoreProf && p.prof ? __builtin_amdgcn_s_memtime() : 0ull;
  const unsigned long long rt_start = kScoreProf && p.prof ? __builtin_amdgcn_s_memrealtime() : 0ull;
  unsigned long long t_cls = 0, t_fl = 0, n_ck = 0, t_ready = 0;
  load_sum_weights(s_w, W);
  check_node_table(p, reinterpret_cast<const unsigned int *>(p.node_w + (int64_t)p.rl.n_nodes * kStrideSum));
  const int shift = (int)reinterpret_cast<const unsigned int *>(p.node_w + (int64_t)p.rl.n_nodes * kStrideSum)[1];
  const float inv_scale = ldexpf(1.f, -shift);
  __syncthreads();  // the only workgroup barrier: waves run independently from here
  if (kScoreProf && p.prof) t_ready = __builtin_amdgcn_s_memtime();
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
      const int2 ck = p.chunks[c];
      q = __builtin_amdgcn_readfirstlane(ck.x);
      s0 = __builtin_amdgcn_readfirstlane(ck.y);
      r = __builtin_amdgcn_readfirstlane((int)p.all_r[q]);
    }
    const bool drain = done || r != cur_r;
    // score full waves of queued candidates (all of them before a relation change / the exit)
#pragma unroll 1
    while (true) {
      const int m = drain ? min(n, 64) : (n >= 64 ? 64 : 0);
      if (m == 0) break;
      wave_lds_sync();
      const unsigned long long tf = kScoreProf && p.prof ? __builtin_amdgcn_s_memtime() : 0ull;
      sum_chunk_flush<DIGEST, COOP>(p, s_w, relb, queue, m, inv_scale, cur_r, cur_root, s_fbig[wv]);
      if (kScoreProf && p.prof) {
        __builtin_amdgcn_s_waitcnt(0);
        t_fl += __builtin_amdgcn_s_memtime() - tf;
      }
      n -= m;
      const int2 v = lane < n ? queue[m + lane] : make_int2(0, 0);
      wave_lds_sync();
      if (lane < n) queue[lane] = v;
    }
    if (done) break;
    const unsigned long long tc = kScoreProf && p.prof ? __builtin_amdgcn_s_memtime() : 0ull;
    if (r != cur_r) {
      wave_lds_sync();  // every lane is done with the previous relation's bias
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int o = lane + 64 * j;
        float acc = p.s0_b[o];
        for (int i = 0; i < 16; ++i) acc = fmaf(p.s0_w[o * 32 + 16 + i], p.rel_emb[r * 16 + i], acc);
        relb[o] = acc;
      }
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
          sum_write_out(p, q, qb + s, cr.x, p.memo[be.x], base);
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
        sum_write_out(p, q, qb + s, cr.x, out, sum_base(p, q, cr.x));
      }
    }
    const uint64_t bal = __ballot(queued);
    const int pos = n + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                       __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
    wave_lds_sync();
    if (queued) queue[pos] = make_int2(q, (int)(qb + s));
    n += (int)__popcll(bal);  // < 128: the queue held < 64 before this chunk
    ++c;
    if (kScoreProf && p.prof) {
      __builtin_amdgcn_s_waitcnt(0);
      t_cls += __builtin_amdgcn_s_memtime() - tc;
      ++n_ck;
    }
  }
  if (kScoreProf && p.prof && lane == 0 && n_ck) {  // waves that took a chunk
    const unsigned long long tot = __builtin_amdgcn_s_memtime() - t_start;
    atomicAdd(&p.prof[16], t_ready - t_start);
    atomicAdd(&p.prof[17], t_cls);
    atomicAdd(&p.prof[18], t_fl);
    atomicAdd(&p.prof[19], tot);
    atomicAdd(&p.prof[20], n_ck);
    atomicAdd(&p.prof[21], n_ck ? 1ull : 0ull);
    atomicMax(&p.prof[22], tot);
    atomicMax(&p.prof[23], t_fl);
    atomicAdd(&p.prof[24], __builtin_amdgcn_s_memrealtime() - rt_start);
  }
}

// Deferred scoring, second half: score[q][t] = out + score[q][t] (the same
// fp32 sum as the direct path, operands commuted) and mask[q][t] = 1 for every
// candidate record, once the base score (RotatE) is in place.  One workgroup
// per query (grid-stride).
__global__ __launch_bounds__(BS) void apply_kernel(KParams p) {
  for (int q = blockIdx.x; q < p.nq; q += gridDim.x) {
    const int nc = p.n_cand[q];
    if (nc <= 0) continue;
    const int64_t qb = p.q_base[q];
    for (int s = threadIdx.x; s < nc; s += BS) {
      const int64_t idx = (int64_t)q * p.g.E + p.cand[qb + s].x;
      const float out = p.cand_out[qb + s];
      p.score[idx] = p.feature == RNNL_FEATURE_NONE ? out : out + p.score[idx];
      if (p.mask) p.mask[idx] = 1;
    }
  }
}

// Packs the MLP weights behind the workspace header (layout W_* above).
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

// ---------------------------------------------------------------- node weights
// Grid-stride over (node, dim) pairs; the table-wide max |s1| (the SUM table's
// shift) is reduced per thread, per wave and per block before one atomic per
// block (one atomic per lane on a single word serialised at ~0.5 ms).
__global__ __launch_bounds__(256) void node_weights_kernel(RulesDev rl, const float *__restrict__ emb, int ld,
                                                          int agg, unsigned char *__restrict__ out) {
  const int64_t total = (int64_t)rl.n_nodes * 16;
  unsigned int m = 0, m2 = 0;
  for (int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; gid < total;
       gid += (int64_t)gridDim.x * blockDim.x) {
    const int n = (int)(gid >> 4), d = (int)(gid & 15);
    float s1 = 0.f, s2 = 0.f, mn = __builtin_huge_valf(), mx = -__builtin_huge_valf();
    for (int k = rl.node_rule_ptr[n]; k < rl.node_rule_ptr[n + 1]; ++k) {
      const float x = emb[(int64_t)rl.node_rules[k] * ld + d];
      s1 += x;
      s2 += x * x;
      mn = fminf(mn, x);
      mx = fmaxf(mx, x);
    }
    if (agg == RNNL_AGG_SUM) {
      // f32 sum for now; node_fix_kernel turns it into int32 fixed point
      reinterpret_cast<float *>(out + (int64_t)n * kStrideSum)[d] = s1;
      m = max(m, __float_as_uint(fabsf(s1)));
    } else {
      // f32 sums for now; pna_fix_kernel turns them into int32 fixed point with
      // one shift per column (max |sum x| bits -> trailer[0], max |sum x^2| -> trailer[3])
      float *rec = reinterpret_cast<float *>(out + (int64_t)n * kStridePna);
      if (isnan(mn) || isnan(mx)) atomicOr(reinterpret_cast<unsigned int *>(out + (int64_t)rl.n_nodes * kStridePna) + 2, 1u);
      m = max(m, __float_as_uint(fabsf(s1)));
      m2 = max(m2, __float_as_uint(fabsf(s2)));
      rec[d] = s1;
      rec[16 + d] = s2;
      rec[32 + d] = mn;
      rec[48 + d] = mx;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    m = max(m, (unsigned int)__shfl_xor((int)m, o, 64));
    m2 = max(m2, (unsigned int)__shfl_xor((int)m2, o, 64));
  }
  __shared__ unsigned int s_m[4], s_m2[4];
  if ((threadIdx.x & 63) == 0) {
    s_m[threadIdx.x >> 6] = m;
    s_m2[threadIdx.x >> 6] = m2;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned int *trailer =
        reinterpret_cast<unsigned int *>(out + (int64_t)rl.n_nodes * (agg == RNNL_AGG_SUM ? kStrideSum : kStridePna));
    m = max(max(s_m[0], s_m[1]), max(s_m[2], s_m[3]));
    m2 = max(max(s_m2[0], s_m2[1]), max(s_m2[2], s_m2[3]));
    if (m) atomicMax(trailer, m);
    if (m2 && agg != RNNL_AGG_SUM) atomicMax(trailer + 3, m2);
  }
}

// PNA records: sum x and sum x^2 to int32 fixed point, each column with its
// own table-wide shift (as the SUM table: every value fits 2^30, so count x
// record is exact in int64); shifts in trailer[1] / trailer[4], trailer[2]
// flags a table that cannot be represented (or held a NaN min / max).
__global__ void pna_fix_kernel(int n_nodes, unsigned char *__restrict__ out) {
  unsigned int *trailer = reinterpret_cast<unsigned int *>(out + (int64_t)n_nodes * kStridePna);
  const unsigned int b1 = trailer[0], b2 = trailer[3];
  int e1 = 0, e2 = 0;
  bool bad = b1 >= 0x7f800000u || b2 >= 0x7f800000u || trailer[2] != 0;
  if (!bad && b1) frexpf(__uint_as_float(b1), &e1);
  if (!bad && b2) frexpf(__uint_as_float(b2), &e2);
  bad = bad || e1 > 30 || e2 > 30;
  const int sh1 = bad ? 0 : min(30 - e1, 60), sh2 = bad ? 0 : min(30 - e2, 60);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    trailer[1] = (unsigned)sh1;
    trailer[4] = (unsigned)sh2;
    trailer[2] = bad ? 1u : 0u;
  }
  const float sc1 = ldexpf(1.f, sh1), sc2 = ldexpf(1.f, sh2);
  const int64_t n = (int64_t)n_nodes * 32;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t node = i >> 5;
    const int w = (int)(i & 31);
    float *rec = reinterpret_cast<float *>(out + node * kStridePna);
    const float f = rec[w];
    reinterpret_cast<int *>(rec)[w] = bad ? 0 : (int)rintf(f * (w < 16 ? sc1 : sc2));
  }
}

// ---------------------------------------------------------------- COO export
// The grounding COO of one launch in reference order: per query its
// candidates in ascending entity order (= row-major nonzero, predictors.py:239)
// and, per candidate, its (trie node, path count) bucket entries.  A query's
// bucket entries are contiguous in the pool in candidate order, so the entry
// export is one copy per query.
__global__ void export_candidates_kernel(KParams p, const int64_t *__restrict__ cand_off, int32_t *__restrict__ out_t,
                                         int32_t *__restrict__ out_nent) {
  for (int q = blockIdx.x; q < p.nq; q += gridDim.x) {
    const int nc = p.n_cand[q];
    if (nc <= 0) continue;
    const int64_t qb = p.q_base[q], o = cand_off[q];
    for (int s = threadIdx.x; s < nc; s += blockDim.x) {
      const int4 cr = p.cand[qb + s];
      out_t[o + s] = cr.x;
      out_nent[o + s] = cr.z;
    }
  }
}

__global__ void export_entries_kernel(KParams p, const int64_t *__restrict__ ent_off, int32_t *__restrict__ out_node,
                                      int32_t *__restrict__ out_count) {
  for (int q = blockIdx.x; q < p.nq; q += gridDim.x) {
    if (p.n_cand[q] <= 0) continue;
    const int64_t qb = p.q_base[q], o = ent_off[q], n = ent_off[q + 1] - o;
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
      const int2 be = p.bent[qb + i];
      out_node[o + i] = be.x;
      out_count[o + i] = be.y;
    }
  }
}

// SUM records -> int32 fixed point with one shift for the whole table:
// |fix| < 2^30 for the largest |sum|, so a candidate's int64 sum of
// count x fix is exact (deterministic in any entry order) with ~2^-30
// relative resolution.  Trailer: u32 max|x| bits, i32 shift.
// Table-wide shift from the max |sum| bits in trailer[0]; trailer[2] = 1 when
// the table cannot be represented (a non-finite sum — its |x| bits are >=
// those of +inf — or |sum| >= 2^30, which would need a negative shift): the
// records are zeroed and the scoring kernels report ERR_NODE_RANGE.
__device__ __forceinline__ int fix_shift(unsigned int *trailer, bool &bad) {
  const unsigned int bits = trailer[0];
  int e = 0;
  bad = bits >= 0x7f800000u;
  if (!bad && bits) frexpf(__uint_as_float(bits), &e);  // max < 2^e
  bad = bad || e > 30;
  const int shift = bad ? 0 : min(30 - e, 60);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    trailer[1] = (unsigned)shift;
    trailer[2] = bad ? 1u : 0u;
  }
  return shift;
}

__global__ void node_fix_kernel(int n_nodes, unsigned char *__restrict__ out) {
  unsigned int *trailer = reinterpret_cast<unsigned int *>(out + (int64_t)n_nodes * kStrideSum);
  bool bad;
  const int shift = fix_shift(trailer, bad);
  const float sc = ldexpf(1.f, shift);
  const int64_t n = (int64_t)n_nodes * 16;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float *f = reinterpret_cast<float *>(out) + i;
    reinterpret_cast<int *>(out)[i] = bad ? 0 : (int)rintf(*f * sc);
  }
}

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
// (fp64, one slot per node of the head's trie), then one global fp64 atomic
// per (row, touched node).  The caller zero-fills grad_node.
__global__ __launch_bounds__(BS) void predictor_backward_kernel(KParams p, const float *__restrict__ grad, int ld,
                                                                double *__restrict__ grad_node) {
  extern __shared__ double s_g[];
  for (int q = blockIdx.x; q < p.nq; q += gridDim.x) {
    const int nc = p.n_cand[q];
    if (nc <= 0) continue;
    const int r = (int)p.all_r[q];
    const int root = p.rl.head_root[r], nh = min(p.rl.head_nodes[r], ld);
    for (int i = threadIdx.x; i < nh; i += BS) s_g[i] = 0.0;
    __syncthreads();
    const int64_t qb = p.q_base[q];
    const float *__restrict__ gq = grad + (int64_t)q * p.g.E;
    for (int s = threadIdx.x; s < nc; s += BS) {
      const int4 cr = p.cand[qb + s];
      const double g = (double)gq[cr.x];
      if (g == 0.0) continue;
      for (int e = cr.y; e < cr.y + cr.z; ++e) {
        const int2 be = p.bent[e];
        atomicAdd(&s_g[be.x - root], (double)(uint32_t)be.y * g);
      }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < nh; i += BS)
      if (s_g[i] != 0.0) atomicAdd(&grad_node[root + i], s_g[i]);
    __syncthreads();
  }
}

}  // namespace rnnl

using namespace rnnl;

extern "C" {

int rnnl_node_weights(rnnl_rules r, const float *emb, int32_t ld, int32_t agg, void *node_w, void *stream) {
  if (!r || !emb || !node_w || (agg != RNNL_AGG_SUM && agg != RNNL_AGG_PNA) || ld < 16) {
    set_error("rnnl_node_weights: bad arguments");
    return RNNL_ERR_INVALID;
  }
  const int64_t n = (int64_t)r->d.n_nodes * 16;
  unsigned char *out = static_cast<unsigned char *>(node_w);
  RNNL_HIP_CHECK(hipMemsetAsync(out + (int64_t)r->d.n_nodes * (agg == RNNL_AGG_SUM ? kStrideSum : kStridePna), 0, 32,
                                (hipStream_t)stream));
  if (n == 0) return RNNL_OK;
  const int bs = 256;
  hipLaunchKernelGGL(node_weights_kernel, dim3((unsigned)std::min<int64_t>((n + bs - 1) / bs, 2048)), dim3(bs), 0,
                     (hipStream_t)stream, r->d, emb, ld, agg, out);
  if (agg == RNNL_AGG_PNA)
    hipLaunchKernelGGL(pna_fix_kernel, dim3((unsigned)std::min<int64_t>((2 * n + bs - 1) / bs, 4096)), dim3(bs), 0,
                       (hipStream_t)stream, r->d.n_nodes, out);
  if (agg == RNNL_AGG_SUM)
    hipLaunchKernelGGL(node_fix_kernel, dim3((unsigned)std::min<int64_t>((n + bs - 1) / bs, 4096)), dim3(bs), 0,
                       (hipStream_t)stream, r->d.n_nodes, out);
  RNNL_HIP_CHECK(hipGetLastError());
  return RNNL_OK;
}

int rnnl_node_weights_size(rnnl_rules r, int32_t agg, size_t *bytes) {
  if (!r || !bytes || (agg != RNNL_AGG_SUM && agg != RNNL_AGG_PNA)) {
    set_error("rnnl_node_weights_size: bad arguments");
    return RNNL_ERR_INVALID;
  }
  *bytes = (size_t)r->d.n_nodes * (agg == RNNL_AGG_SUM ? kStrideSum : kStridePna) + 64;
  return RNNL_OK;
}

int rnnl_forward_workspace_size(rnnl_graph g, rnnl_rules r, int32_t nq, int32_t scale, size_t *bytes) {
  if (!g || !r || !bytes || nq < 0 || scale < 1) {
    set_error("rnnl_forward_workspace_size: bad arguments");
    return RNNL_ERR_INVALID;
  }
  *bytes = (size_t)make_layout(nq, scale, r->d.n_nodes).total;
  return RNNL_OK;
}

// Graph/rules/rows/workspace part of the launch parameters, shared by the
// forward, the ground-only launch and the COO export.
static int setup_params(const char *who, rnnl_graph g, rnnl_rules r, const int64_t *all_h, const int64_t *all_r,
                        const int64_t *etr, int32_t nq, int32_t *n_cand, void *ws, size_t ws_bytes, int32_t scale,
                        KParams &p) {
  if (!g || !r || !all_h || !all_r || !ws || !n_cand || nq < 0 || scale < 1) {
    set_error(std::string(who) + ": bad arguments");
    return RNNL_ERR_INVALID;
  }
  if ((int64_t)g->d.E > (int64_t)MAXWIN * WIN) {
    set_error(std::string(who) + ": more entities than the kernel's window table supports");
    return RNNL_ERR_INVALID;
  }
  const Layout Ly = make_layout(nq, scale, r->d.n_nodes);
  if ((int64_t)ws_bytes < Ly.total) {
    set_error(std::string(who) + ": workspace too small");
    return RNNL_ERR_INVALID;
  }
  if (Ly.pool_cap >= INT32_MAX) {
    set_error(std::string(who) + ": too many rows for one launch (pool index exceeds 31 bits)");
    return RNNL_ERR_INVALID;
  }
  // packed scratch keys (trie node - head root) << ebits | entity must fit 31 bits
  int ebits = 1;
  while ((1ll << ebits) < (int64_t)g->d.E) ++ebits;
  if (((int64_t)std::max(r->d.max_head_nodes, 1) << ebits) > (int64_t)INT32_MAX) {
    set_error(std::string(who) + ": a head relation's rule trie (" + std::to_string(r->d.max_head_nodes) +
              " nodes) x 2^" + std::to_string(ebits) + " entities exceeds the 31-bit grounding keys");
    return RNNL_ERR_INVALID;
  }
  unsigned char *base = static_cast<unsigned char *>(ws);
  p = KParams{};
  p.g = g->d;
  p.ebits = ebits;
  p.emask = (uint32_t)((1u << ebits) - 1u);
  p.rl = r->d;
  p.all_h = all_h;
  p.all_r = all_r;
  p.etr = etr;
  p.nq = nq;
  p.n_cand = n_cand;
  p.ws = base;
  p.fcap = Ly.fcap;
  p.pcap = Ly.pcap;
  p.pool_cap = Ly.pool_cap;
  p.nslots = (int32_t)Ly.nslots;
  p.slots = base + Ly.off_slots;
  p.q_base = reinterpret_cast<int64_t *>(base + Ly.off_qbase);
  p.q_scale = reinterpret_cast<float *>(base + Ly.off_qscale);
  p.cand = reinterpret_cast<int4 *>(base + Ly.off_cand);
  p.bent = reinterpret_cast<int2 *>(base + Ly.off_bent);
  p.memo = reinterpret_cast<float *>(base + Ly.off_memo);
  p.ptab = nullptr;  // set by launch_score where the pair memo applies
  p.ptab_region = reinterpret_cast<unsigned long long *>(base + Ly.off_ptab);
  p.psbits = (int32_t)Ly.ptab_bits;
  {
    auto bitlen = [](int64_t v) {
      int b = 0;
      while ((1ll << b) <= v) ++b;
      return b;
    };
    p.pbr = bitlen(std::max<int64_t>(g->d.R - 1, 0));
    p.pbo = bitlen(std::max<int64_t>(r->d.max_head_nodes - 1, 0));
    p.pbc = std::min(20, (30 + p.psbits - p.pbr - 2 * p.pbo) / 2);  // K = 31 + psbits, one format bit
    p.pbc3 = std::min(20, (30 + p.psbits - p.pbr - 3 * p.pbo) / 3);
  }
  p.chunks = reinterpret_cast<int2 *>(base + Ly.off_chunk);
  p.chunk_cap = Ly.chunk_cap;
  p.prof = g_prof;
  return RNNL_OK;
}

// Kernel sequences shared by the one-call forward and its two halves.
// `grid` caps the persistent workgroups (0: one per workspace slot, the
// default occupancy); a smaller grid leaves CUs to a concurrent kernel.
static void launch_ground(const KParams &p, int agg, hipStream_t st, int grid = 0) {
  const unsigned g = (unsigned)(grid > 0 ? std::min(grid, p.nslots) : p.nslots);
  if (agg == RNNL_AGG_SUM)
    hipLaunchKernelGGL(ground_kernel<RNNL_AGG_SUM>, dim3(g), dim3(GBS), 0, st, p);
  else
    hipLaunchKernelGGL(ground_kernel<RNNL_AGG_PNA>, dim3(g), dim3(GBS), 0, st, p);
}

static void set_score_params(KParams &p, const rnnl_predictor_params *pp, float *score, uint8_t *mask,
                             uint64_t *digest) {
  p.agg = pp->aggregator;
  p.feature = pp->feature;
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
  p.base_row = pp->base_row;
  p.score = score;
  p.mask = mask;
  p.digest = digest;
}

// RNNL_SCORE_MEMO=0 selects the scoring pass without the single-path memo (A/B)
static bool score_memo_enabled() {
  static const bool on = [] {
    const char *e = getenv("RNNL_SCORE_MEMO");
    return !(e && e[0] == '0');
  }();
  return on;
}

// RNNL_SCORE_PAIRMEMO=0 turns the SUM pair memo off (A/B; bit-identical scores)
static bool pair_memo_enabled() {  // read per launch: tests compare both settings in one process
  const char *e = getenv("RNNL_SCORE_PAIRMEMO");
  return !(e && e[0] == '0');
}

// RNNL_PNA_CHUNKED=0 selects the per-query PNA scoring kernel (A/B)
static bool pna_chunked() {
  static const bool on = [] {
    const char *e = getenv("RNNL_PNA_CHUNKED");
    return !(e && e[0] == '0');
  }();
  return on;
}

// RNNL_SUM_CHUNKED=0 selects the per-query SUM memo scoring kernel (A/B)
static bool sum_chunked() {
  static const bool on = [] {
    const char *e = getenv("RNNL_SUM_CHUNKED");
    return !(e && e[0] == '0');
  }();
  return on;
}

static void launch_score(const KParams &p0, rnnl_rules r, hipStream_t st, int grid = 0) {
  KParams p = p0;
  const int nq = p.nq;
  float *W = reinterpret_cast<float *>(p.ws + HDR_WORDS_BYTES);
  hipLaunchKernelGGL(pack_weights_kernel, dim3((W_FLOATS + 255) / 256), dim3(256), 0, st, p, W);
  if (p.agg == RNNL_AGG_SUM) {
    // staged path while the largest head's leaves fit the LDS budget
    const int64_t base_lds = (int64_t)(WL<RNNL_AGG_SUM>::N + 128) * 4;
    const int64_t stage = sum_stage_bytes(r->d.max_leaves, r->d.max_head_nodes);
    const unsigned sgrid = (unsigned)std::min<int64_t>(
        (nq + QCHUNK - 1) / QCHUNK, grid > 0 ? (int64_t)grid : (int64_t)NUM_CU * RNNL_SCORE_WG_PER_CU);
#ifndef RNNL_STAGE_LIMIT
#define RNNL_STAGE_LIMIT 0  // staging measured slower (lower occupancy); kept for A/B
#endif
    const bool staged = base_lds + stage <= RNNL_STAGE_LIMIT;
    if (!staged && score_memo_enabled() && p.memo) {
      // few rows (e.g. one reference batch per call) with the pair memo on: no memo
      // pass (one workgroup per relation, on the call's critical path); the
      // single-path candidates take pair-memo keys instead — the same outputs
      const bool small = sum_chunked() && !p.digest && pair_memo_enabled() && p.pbc >= 2 && nq <= MEMO_SCAN_ROWS;
      if (small)
        p.memo = nullptr;
      else
        hipLaunchKernelGGL(memo_sum_kernel, dim3((unsigned)std::max(p.g.R, 1)), dim3(BS), 0, st, p,
                           (const float *)W);
      if (sum_chunked()) {
        launch_chunk_list(p, st);
        if (p.digest) (void)hipMemsetAsync(p.digest, 0, sizeof(uint64_t) * (size_t)nq, st);
        // the pair memo (not with the test digest, which needs every candidate's entries); a key
        // needs >= 2 count bits per entry
        if (!p.digest && pair_memo_enabled() && p.pbc >= 2) {
          p.ptab = p.ptab_region;
          (void)hipMemsetAsync(p.ptab, 0, 8ull << p.psbits, st);
        }
        const unsigned cgrid = (unsigned)(grid > 0 ? grid : NUM_CU * RNNL_SCORE_WG_PER_CU);
        // one reference batch per call: the wave-cooperative walk of long entry lists
        // (bit-identical features); large launches keep the per-lane walk
        const bool coop = nq <= MEMO_SCAN_ROWS;
        if (p.digest && coop)
          hipLaunchKernelGGL((score_sum_chunk_kernel<true, true>), dim3(cgrid), dim3(BS), 0, st, p, (const float *)W);
        else if (p.digest)
          hipLaunchKernelGGL((score_sum_chunk_kernel<true, false>), dim3(cgrid), dim3(BS), 0, st, p, (const float *)W);
        else if (coop)
          hipLaunchKernelGGL((score_sum_chunk_kernel<false, true>), dim3(cgrid), dim3(BS), 0, st, p, (const float *)W);
        else
          hipLaunchKernelGGL((score_sum_chunk_kernel<false, false>), dim3(cgrid), dim3(BS), 0, st, p, (const float *)W);
        return;
      }
      if (p.digest)
        hipLaunchKernelGGL((score_sum_memo_kernel<true>), dim3(sgrid), dim3(BS), 0, st, p, (const float *)W);
      else
        hipLaunchKernelGGL((score_sum_memo_kernel<false>), dim3(sgrid), dim3(BS), 0, st, p, (const float *)W);
      return;
    }
    const size_t lds = (size_t)(staged ? base_lds + stage : base_lds);
    if (staged)
      hipLaunchKernelGGL((score_sum_kernel<true, true>), dim3(sgrid), dim3(BS), lds, st, p, (const float *)W);
    else if (p.digest)
      hipLaunchKernelGGL((score_sum_kernel<false, true>), dim3(sgrid), dim3(BS), lds, st, p, (const float *)W);
    else
      hipLaunchKernelGGL((score_sum_kernel<false, false>), dim3(sgrid), dim3(BS), lds, st, p, (const float *)W);
  } else if (pna_chunked()) {
    // per-query digests are sums over the query's chunks
    launch_chunk_list(p, st);
    if (p.digest) (void)hipMemsetAsync(p.digest, 0, sizeof(uint64_t) * (size_t)nq, st);
    const unsigned score_grid = (unsigned)(grid > 0 ? grid : NUM_CU * 8);
    hipLaunchKernelGGL(score_pna_chunk_kernel, dim3(score_grid), dim3(BS), 0, st, p, (const float *)W);
  } else {
    const unsigned score_grid = (unsigned)std::min<int64_t>(nq, (int64_t)NUM_CU * 8);
    hipLaunchKernelGGL(score_kernel<RNNL_AGG_PNA>, dim3(score_grid), dim3(BS), 0, st, p, (const float *)W);
  }
}

static bool bad_params(const rnnl_predictor_params *pp, const float *score) {
  return !pp || !score || !pp->node_w || (pp->aggregator != RNNL_AGG_SUM && pp->aggregator != RNNL_AGG_PNA);
}

int rnnl_predictorplus_forward(rnnl_graph g, rnnl_rules r, const rnnl_predictor_params *pp, const int64_t *all_h,
                               const int64_t *all_r, const int64_t *etr, int32_t nq, float *score, uint8_t *mask,
                               int32_t *n_cand, uint64_t *digest, void *ws, size_t ws_bytes, int32_t scale,
                               void *stream) {
  if (bad_params(pp, score)) {
    set_error("rnnl_predictorplus_forward: bad arguments");
    return RNNL_ERR_INVALID;
  }
  KParams p;
  if (int rc = setup_params("rnnl_predictorplus_forward", g, r, all_h, all_r, etr, nq, n_cand, ws, ws_bytes, scale,
                            p))
    return rc;
  hipStream_t st = (hipStream_t)stream;
  RNNL_HIP_CHECK(hipMemsetAsync(ws, 0, HDR_WORDS_BYTES, st));
  if (nq == 0) return RNNL_OK;
  set_score_params(p, pp, score, mask, digest);
  launch_ground(p, pp->aggregator, st);
  launch_score(p, r, st);
  RNNL_HIP_CHECK(hipGetLastError());
  return RNNL_OK;
}

int rnnl_predictorplus_ground(rnnl_graph g, rnnl_rules r, int32_t aggregator, const int64_t *all_h,
                              const int64_t *all_r, const int64_t *etr, int32_t nq, int32_t *n_cand, void *ws,
                              size_t ws_bytes, int32_t scale, int32_t workgroups, void *stream) {
  if (aggregator != RNNL_AGG_SUM && aggregator != RNNL_AGG_PNA) {
    set_error("rnnl_predictorplus_ground: bad aggregator");
    return RNNL_ERR_INVALID;
  }
  KParams p;
  if (int rc = setup_params("rnnl_predictorplus_ground", g, r, all_h, all_r, etr, nq, n_cand, ws, ws_bytes, scale,
                            p))
    return rc;
  hipStream_t st = (hipStream_t)stream;
  RNNL_HIP_CHECK(hipMemsetAsync(ws, 0, HDR_WORDS_BYTES, st));
  if (nq == 0) return RNNL_OK;
  p.agg = aggregator;
  launch_ground(p, aggregator, st, workgroups);
  RNNL_HIP_CHECK(hipGetLastError());
  return RNNL_OK;
}

int rnnl_predictorplus_score(rnnl_graph g, rnnl_rules r, const rnnl_predictor_params *pp, const int64_t *all_h,
                             const int64_t *all_r, int32_t nq, float *score, uint8_t *mask, int32_t *n_cand,
                             uint64_t *digest, void *ws, size_t ws_bytes, int32_t scale, int32_t workgroups,
                             int32_t deferred, void *stream) {
  if (bad_params(pp, score) || !n_cand || deferred < 0 || deferred > 2 ||
      (deferred == 2 && (mask || pp->feature != RNNL_FEATURE_ADD))) {
    set_error("rnnl_predictorplus_score: bad arguments");
    return RNNL_ERR_INVALID;
  }
  KParams p;
  if (int rc = setup_params("rnnl_predictorplus_score", g, r, all_h, all_r, nullptr, nq, n_cand, ws, ws_bytes,
                            scale, p))
    return rc;
  if (nq == 0) return RNNL_OK;
  set_score_params(p, pp, score, mask, digest);
  if (deferred) {
    p.cand_out = reinterpret_cast<float *>(static_cast<unsigned char *>(ws) + make_layout(nq, scale).off_cout);
    p.atomic_out = deferred == 2;
  }
  hipStream_t st = (hipStream_t)stream;
  RNNL_HIP_CHECK(hipMemsetAsync(p.ws + 4 * H_DEQUEUE2, 0, 4, st));  // the scoring dequeue counter
  launch_score(p, r, st, workgroups);
  RNNL_HIP_CHECK(hipGetLastError());
  return RNNL_OK;
}

int rnnl_predictorplus_apply(void *ws, int32_t nq, int32_t scale, const int32_t *n_cand, int32_t feature,
                             float *score, uint8_t *mask, int32_t n_entities, void *stream) {
  if (!ws || nq < 0 || scale < 1 || !n_cand || !score || n_entities <= 0) {
    set_error("rnnl_predictorplus_apply: bad arguments");
    return RNNL_ERR_INVALID;
  }
  if (nq == 0) return RNNL_OK;
  const Layout Ly = make_layout(nq, scale);
  unsigned char *base = static_cast<unsigned char *>(ws);
  KParams p{};
  p.nq = nq;
  p.g.E = n_entities;
  p.feature = feature;
  p.n_cand = const_cast<int32_t *>(n_cand);
  p.q_base = reinterpret_cast<int64_t *>(base + Ly.off_qbase);
  p.cand = reinterpret_cast<int4 *>(base + Ly.off_cand);
  p.cand_out = reinterpret_cast<float *>(base + Ly.off_cout);
  p.score = score;
  p.mask = mask;
  hipLaunchKernelGGL(apply_kernel, dim3((unsigned)std::min<int64_t>(nq, (int64_t)NUM_CU * 8)), dim3(BS), 0,
                     (hipStream_t)stream, p);
  RNNL_HIP_CHECK(hipGetLastError());
  return RNNL_OK;
}

int rnnl_ground(rnnl_graph g, rnnl_rules r, const int64_t *all_h, const int64_t *all_r, const int64_t *etr,
                int32_t nq, int32_t *n_cand, void *ws, size_t ws_bytes, int32_t scale, void *stream) {
  KParams p;
  if (int rc = setup_params("rnnl_ground", g, r, all_h, all_r, etr, nq, n_cand, ws, ws_bytes, scale, p)) return rc;
  hipStream_t st = (hipStream_t)stream;
  RNNL_HIP_CHECK(hipMemsetAsync(ws, 0, HDR_WORDS_BYTES, st));
  if (nq == 0) return RNNL_OK;
  p.agg = RNNL_AGG_SUM;
  hipLaunchKernelGGL(ground_kernel<RNNL_AGG_SUM>, dim3(p.nslots), dim3(GBS), 0, st, p);
  RNNL_HIP_CHECK(hipGetLastError());
  return RNNL_OK;
}

// Only the workspace carve-up is needed to read the pool back.
static KParams export_params(void *ws, int32_t nq, int32_t scale, const int32_t *n_cand) {
  const Layout Ly = make_layout(nq, scale);
  unsigned char *base = static_cast<unsigned char *>(ws);
  KParams p{};
  p.nq = nq;
  p.n_cand = const_cast<int32_t *>(n_cand);
  p.q_base = reinterpret_cast<int64_t *>(base + Ly.off_qbase);
  p.cand = reinterpret_cast<int4 *>(base + Ly.off_cand);
  p.bent = reinterpret_cast<int2 *>(base + Ly.off_bent);
  return p;
}

int rnnl_ground_export_candidates(void *ws, int32_t nq, int32_t scale, const int32_t *n_cand,
                                  const int64_t *cand_off, int32_t *out_t, int32_t *out_nent, void *stream) {
  if (!ws || nq < 0 || scale < 1 || !n_cand || !cand_off || !out_t || !out_nent) {
    set_error("rnnl_ground_export_candidates: bad arguments");
    return RNNL_ERR_INVALID;
  }
  if (nq == 0) return RNNL_OK;
  const KParams p = export_params(ws, nq, scale, n_cand);
  hipLaunchKernelGGL(export_candidates_kernel, dim3((unsigned)std::min<int64_t>(nq, 4096)), dim3(256), 0,
                     (hipStream_t)stream, p, cand_off, out_t, out_nent);
  RNNL_HIP_CHECK(hipGetLastError());
  return RNNL_OK;
}

int rnnl_ground_export_entries(void *ws, int32_t nq, int32_t scale, const int32_t *n_cand, const int64_t *ent_off,
                               int32_t *out_node, int32_t *out_count, void *stream) {
  if (!ws || nq < 0 || scale < 1 || !n_cand || !ent_off || !out_node || !out_count) {
    set_error("rnnl_ground_export_entries: bad arguments");
    return RNNL_ERR_INVALID;
  }
  if (nq == 0) return RNNL_OK;
  const KParams p = export_params(ws, nq, scale, n_cand);
  hipLaunchKernelGGL(export_entries_kernel, dim3((unsigned)std::min<int64_t>(nq, 4096)), dim3(256), 0,
                     (hipStream_t)stream, p, ent_off, out_node, out_count);
  RNNL_HIP_CHECK(hipGetLastError());
  return RNNL_OK;
}

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
  hipLaunchKernelGGL(ground_kernel<RNNL_AGG_SUM>, dim3(p.nslots), dim3(GBS), 0, st, p);
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
  hipLaunchKernelGGL(ground_kernel<RNNL_AGG_SUM>, dim3(p.nslots), dim3(GBS), 0, st, p);
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
  hipLaunchKernelGGL(predictor_backward_kernel, dim3((unsigned)std::min<int64_t>(nq, 4096)), dim3(BS),
                     (size_t)ld * 8, (hipStream_t)stream, p, grad_score, ld, grad_node);
  RNNL_HIP_CHECK(hipGetLastError());
  return RNNL_OK;
}

int rnnl_debug_profile(void *dev_counters) {
  g_prof = static_cast<unsigned long long *>(dev_counters);
  return RNNL_OK;
}

int rnnl_debug_capacity(int64_t frontier_base, int64_t contrib_base, int64_t pool_per_query) {
  if (frontier_base <= 0 && contrib_base <= 0 && pool_per_query <= 0) {  // restore the defaults
    g_fcap_base = FCAP_BASE;
    g_pcap_base = PCAP_BASE;
    g_pool_per_query = POOL_PER_QUERY;
    return RNNL_OK;
  }
  if (frontier_base < 256 || contrib_base < 256 || frontier_base < contrib_base || pool_per_query < 1 ||
      frontier_base > FCAP_BASE || contrib_base > PCAP_BASE || pool_per_query > POOL_PER_QUERY) {
    set_error("rnnl_debug_capacity: need 256 <= contrib <= frontier <= defaults, 1 <= pool <= default");
    return RNNL_ERR_INVALID;
  }
  g_fcap_base = frontier_base;
  g_pcap_base = contrib_base;
  g_pool_per_query = pool_per_query;
  return RNNL_OK;
}

constexpr int STATUS_WORDS = 18;  // header words 0..17: status, ..., H_NCAND, the pool counter (byte 64)

static int status_from_header(const unsigned int *st, int64_t *totals);

static int forward_status(void *ws, void *stream, int64_t *totals) {
  unsigned int st[STATUS_WORDS] = {0};
  RNNL_HIP_CHECK(hipMemcpyAsync(st, ws, sizeof(st), hipMemcpyDeviceToHost, (hipStream_t)stream));
  RNNL_HIP_CHECK(hipStreamSynchronize((hipStream_t)stream));
  return status_from_header(st, totals);
}

static int status_from_header(const unsigned int *st, int64_t *totals) {
  if (totals) {
    unsigned long long c, e;
    memcpy(&c, st + H_NCAND, 8);
    memcpy(&e, st + 16, 8);
    totals[0] = (int64_t)c;  // candidates (sum of n_cand)
    totals[1] = (int64_t)e;  // bucket entries (every contribution is one entry of its candidate's bucket)
  }
  if (st[H_STATUS] & 2u) {
    const unsigned bits = st[H_ERRBITS];
    if (bits & (ERR_COUNT_WIDTH | ERR_NODE_RANGE | ERR_ACC_RANGE) && !(bits & ERR_WATCHDOG)) {
      std::string msg = "rnnl_predictorplus_forward:";
      if (bits & ERR_COUNT_WIDTH)
        msg += " a path count or PNA degree reached 2^32 (query " + std::to_string(st[H_ERRQ]) + ");";
      if (bits & ERR_NODE_RANGE) msg += " rule-embedding / rule-weight aggregates are non-finite or >= 2^30;";
      if (bits & ERR_ACC_RANGE) msg += " a candidate's path counts sum beyond the exact int64 feature sum;";
      set_error(msg);
      return RNNL_ERR_RANGE;
    }
    set_error("rnnl_predictorplus_forward: internal error bits " + std::to_string(bits) +
              " (4: watchdog) at query " + std::to_string(st[H_ERRQ]));
    return RNNL_ERR_INTERNAL;
  }
  if (st[H_STATUS] & 1u) {
    set_error("rnnl_predictorplus_forward: workspace capacity exceeded");
    return RNNL_ERR_OVERFLOW;
  }
  return RNNL_OK;
}

int rnnl_forward_status(void *ws, void *stream) { return forward_status(ws, stream, nullptr); }

int rnnl_forward_header_bytes(size_t *bytes) {
  if (!bytes) {
    set_error("rnnl_forward_header_bytes: bad arguments");
    return RNNL_ERR_INVALID;
  }
  *bytes = sizeof(unsigned int) * STATUS_WORDS;
  return RNNL_OK;
}

int rnnl_forward_status_host(const void *header, int64_t *totals) {
  if (!header) {
    set_error("rnnl_forward_status_host: bad arguments");
    return RNNL_ERR_INVALID;
  }
  unsigned int st[STATUS_WORDS];
  memcpy(st, header, sizeof(st));
  return status_from_header(st, totals);
}

int rnnl_forward_status_totals(void *ws, void *stream, int64_t *totals) {
  if (!ws || !totals) {
    set_error("rnnl_forward_status_totals: bad arguments");
    return RNNL_ERR_INVALID;
  }
  return forward_status(ws, stream, totals);
}

}  // extern "C"
