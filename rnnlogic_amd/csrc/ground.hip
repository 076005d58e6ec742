// PredictorPlus / Predictor forward for gfx950 (MI355X), K1: the grounding.
//
// ground_kernel — one persistent workgroup (256 lanes) per query at a time,
// dequeued from a device counter:
//   grounding / propagate (ref src/data.py:136-173, torch_scatter scatter-sum)
//       -> level-synchronous walk of the head relation's rule-prefix trie over
//          the vertex-major CSR; every (trie node, entity) path count lives in
//          an LDS hash (integer, exact); the query's own edge is skipped on
//          hops of the query relation (data.py:164-169).
//   candidate set + rule_count stack (ref src/predictors.py:221-244)
//       -> leaf contributions (entity, node, count) are bucketed by entity
//          window and per candidate through LDS tables into a global pool:
//          per query a contiguous run of candidate records (entity, bucket)
//          and (node, count) entries — the COO of the reference's stacked
//          rule_count matrix, candidates in ascending entity order.
// K2 (score.hip) turns each candidate's entries into its score; the EM
// Predictor's linear score is predictor.hip.  Also here: the node-weight
// tables, the scoring chunk list, the COO export and the forward C-ABI.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <map>
#include <cstring>
#include <string>

#include "fwd.h"
#include "hostside.h"

namespace rnnl {

unsigned long long *g_prof = nullptr;
int64_t g_fcap_base = FCAP_BASE, g_pcap_base = PCAP_BASE, g_pool_per_query = POOL_PER_QUERY;
int g_sort_bits = -1;  // rnnl_debug_sort_bits (-1: SORT_WINS windows)

template <int G>
struct __align__(16) SmemT {
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
      int ent_v[G], ent_fch[G], item_off[G];
      uint32_t ent_c[G];
      int it_child[G], it_beg[G], it_flags[G], edge_off[G];
      uint32_t it_c[G];
      // the hash slots occupied at this level, in insertion order (the first
      // OCC_CAP): the level's compaction walks them instead of all HCAP slots
      unsigned short occ[OCC_CAP];
    };
    struct {  // phase B: entity bitmap of one hash pass and its popcount prefix (candidate ranks)
      uint32_t sbits[sort_words(G)];
      unsigned short spre[sort_words(G)];
    };
  };
  int ws[(G / 64) + 1];
  int q, nd, np, ovf, err, root, nocc;
  int nent;   // the query's pool entries used by its passes so far (phase B)
  int nreal;  // of which bucket entries (a merged short bucket leaves a gap behind it)
  long long qbase;
  unsigned long long t0;
  int whist[SORT_WINS], wbeg[SORT_WINS + 1], wfill[SORT_WINS];
  unsigned long long sumlog;
  unsigned long long tp[8];  // diagnostic sub-phase cycles (thread 0)
};

template <int G>
__device__ __forceinline__ void emit_contrib(SmemT<G> &S, const Slot &sl, int64_t pcap, uint32_t key, uint32_t c) {
  const int pos = atomicAdd(&S.np, 1);
  if (pos < pcap) {
    sl.ct[pos] = Ent{key, c};
  } else {
    S.ovf = 1;
  }
}

template <int G>
__device__ __forceinline__ void emit_frontier(SmemT<G> &S, const Slot &sl, int buf, int64_t fcap, uint32_t key,
                                              uint32_t c) {
  const int pos = atomicAdd(&S.nd, 1);
  if (pos < fcap) {
    sl.f(buf)[pos] = Ent{key, c};
  } else {
    S.ovf = 1;
  }
}

// (node, entity) += c in the phase-A hash; false if the table is full.
template <int G>
__device__ __forceinline__ bool hash_add(SmemT<G> &S, int key, uint32_t c) {
  uint32_t h = hash32((uint32_t)key) >> (32 - HBITS);
#pragma unroll 1
  for (int probe = 0; probe < 64; ++probe) {
    const int k = atomicCAS(&S.u.a.key[h], EMPTY, key);
    if (k == EMPTY) {  // a new (node, entity): listed for the level's compaction
      const int i = atomicAdd(&S.nocc, 1);
      if (i < OCC_CAP) S.occ[i] = (unsigned short)h;
    }
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
template <int G>
__device__ __forceinline__ bool watchdog(SmemT<G> &S) {
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
template <int G>
__device__ void ground_query(const KParams &p, SmemT<G> &S, const Slot &sl, int h, int r, int root, int rm_src,
                             int rm_dst) {
  const int tid = threadIdx.x;
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
    for (int cb = 0; cb < n_prev; cb += G) {
      if (watchdog(S)) break;
      const int ne = min(G, n_prev - cb);
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
      const int ioff = block_scan<G>(nch, S.ws, NI);
      S.item_off[tid] = ioff;
      __syncthreads();
      PSTAMP(3);
      for (int ib = 0; ib < NI; ib += G) {
        const int k = ib + tid;
        int deg = 0;
        if (k < NI) {
          const int ent = upper_idx(S.item_off, ne, k);
          const int child = S.ent_fch[ent] + (k - S.item_off[ent]);
          const int4 ci = p.rl.node_info[child];
          const int rel = ci.x;
          const int v = S.ent_v[ent];
          // the (v, rel) edge range from v's relation bitmap word + the dense offsets (L2-sized)
          const uint2 vb = p.g.vbits[(int64_t)v * p.g.W + (rel >> 5)];
          const uint32_t bit = 1u << (rel & 31);
          int beg = 0;
          if (vb.x & bit) {
            const int pos = (int)vb.y + __popc(vb.x & (bit - 1u));
            beg = p.g.dvoff[pos];
            deg = p.g.dvoff[pos + 1] - beg;
          }
          S.it_child[tid] = child;
          S.it_beg[tid] = beg;
          S.it_c[tid] = S.ent_c[ent];
          // bit 0: leaf (rules end here), bit 1: inner (has children),
          // bit 2: this hop may traverse the query's own edge (data.py:143-146)
          S.it_flags[tid] = (ci.w > 0 ? 1 : 0) | (ci.z > 0 ? 2 : 0) |
                            (rel == r && v == rm_src ? 4 : 0);
        }
        int NE;
        const int eoff = block_scan<G>(deg, S.ws, NE);
        S.edge_off[tid] = eoff;
        __syncthreads();
        PSTAMP(4);
        const int nit = min(G, NI - ib);
        // one edge per lane per pass: the edge -> item map is a binary search of
        // the items' edge offsets (2 / 4 edges per lane measured no faster: the
        // loop is bound by its barriers and dependent loads)
        for (int eb = 0; eb < NE; eb += G) {
          const int j = eb + tid;
          if (j < NE) {
            const int it = upper_idx(S.edge_off, nit, j);
            const int tt = p.g.col[S.it_beg[it] + (j - S.edge_off[it])];
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
        __syncthreads();
        PSTAMP(5);
      }
    }
    // compact the hash into the next frontier and clear it
    const int nocc = S.nocc;  // uniform: read after the edge loop's barrier
    if (nocc <= OCC_CAP) {  // the listed slots only (small frontiers: most levels)
      for (int i = tid; i < nocc; i += G) {
        const int s2 = S.occ[i];
        emit_frontier(S, sl, nxt, p.fcap, (uint32_t)S.u.a.key[s2], S.u.a.val[s2]);
        S.u.a.key[s2] = EMPTY;
        S.u.a.val[s2] = 0u;
      }
    } else {
      for (int s2 = tid; s2 < HCAP; s2 += G) {
        const int k = S.u.a.key[s2];
        if (k != EMPTY) {
          emit_frontier(S, sl, nxt, p.fcap, (uint32_t)k, S.u.a.val[s2]);
          S.u.a.key[s2] = EMPTY;
          S.u.a.val[s2] = 0u;
        }
      }
    }
    wg_sync_global();
    PSTAMP(6);
    n_prev = min((int64_t)S.nd, p.fcap);
    __syncthreads();
    if (tid == 0) {
      S.nd = 0;
      S.nocc = 0;
    }
    cur = nxt;
    __syncthreads();
  }
}

// ---------------------------------------------------------------- phase B
// PNA degree += count x rules at the node (u32 in LDS), carry-checked.
template <int G>
__device__ __forceinline__ void degree_add(SmemT<G> &S, uint32_t *cell, uint32_t c, int nrules) {
  const uint64_t v = (uint64_t)c * (uint32_t)nrules;
  const uint32_t old = atomicAdd(cell, (uint32_t)v);
  if ((v >> 32) || old + (uint32_t)v < old) atomicOr(&S.err, ERR_COUNT_WIDTH);
}

// Exclusive scan of WIN ints in place (PER consecutive per thread); returns the total.
template <int G>
__device__ __forceinline__ int scan_win(int *a, int *s_ws) {
  constexpr int PER = WIN / G;
  const int tid = threadIdx.x;
  int loc[PER];
  int sum = 0;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    loc[j] = a[tid * PER + j];
    sum += loc[j];
  }
  int total;
  int base = block_scan<G>(sum, s_ws, total);
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
// its buckets at pool indices qbase + nent + [0, end - beg).  degree_only
// (PNA sweep 1) accumulates sum log(degree) instead.  Returns nc.
// (Duplicate (node, entity) contributions stay separate entries here: a
// register merge of buckets of up to 4 / 8 entries removed 2.5 M / 7 M of
// FB15k-237's 26 M duplicates for +0.3 / +0.45 ms on the bias step —
// tools/sort_ab.py)
template <int G>
__device__ int window_pass(const KParams &p, SmemT<G> &S, const Ent *w, int lo, int beg, int end, int64_t cbase,
                           bool degree_only) {
  // w: contributions (entity | node key, count), window-sorted or (one window) raw
  const int tid = threadIdx.x;
  if (p.prof && tid == 0) S.tp[7] = __builtin_amdgcn_s_memtime();
  for (int i = tid; i < WIN; i += G) S.u.b.map[i] = 0;
  __syncthreads();
  for (int i = beg + tid; i < end; i += G) S.u.b.map[(int)(w[i].k & p.emask) - lo] = 1;  // mark present entities
  __syncthreads();
  for (int i = tid; i < WIN; i += G) S.u.b.cnt[i] = S.u.b.map[i];
  __syncthreads();
  const int nc = scan_win<G>(S.u.b.cnt, S.ws);  // slots in ascending entity order
  for (int i = tid; i < WIN; i += G) {
    if (S.u.b.map[i]) {
      const int slot = S.u.b.cnt[i];
      S.u.b.map[i] = slot;
      S.u.b.st[slot] = lo + i;
    }
  }
  __syncthreads();
  for (int i = tid; i < WIN; i += G) S.u.b.cnt[i] = 0;
  __syncthreads();
  PSTAMP(0);
  if (degree_only) {
    // PNA sweep 1: degree = 1 + sum_rho count (layers.py:99) per candidate
    for (int i = beg + tid; i < end; i += G)
      degree_add(S, reinterpret_cast<uint32_t *>(&S.u.b.cnt[S.u.b.map[(int)(w[i].k & p.emask) - lo]]), w[i].c,
                 p.rl.node_nrules[S.root + (int)(w[i].k >> p.ebits)]);
    __syncthreads();
    for (int s2 = tid; s2 < nc; s2 += G) {
      const float degf = (float)((double)(uint32_t)S.u.b.cnt[s2] + 1.0);
      atomicAdd(&S.sumlog, (unsigned long long)(long long)llrint((double)logf(degf) * 4294967296.0));
    }
    __syncthreads();
    return nc;
  }
  for (int i = beg + tid; i < end; i += G) atomicAdd(&S.u.b.cnt[S.u.b.map[(int)(w[i].k & p.emask) - lo]], 1);  // bucket sizes
  __syncthreads();
  for (int i = tid; i < WIN; i += G) S.u.b.off[i] = S.u.b.cnt[i];
  __syncthreads();
  scan_win<G>(S.u.b.off, S.ws);
  // the pass's entries follow the query's earlier ones
  const int64_t qb = S.qbase + S.nent;
  for (int i = tid; i < WIN; i += G) S.u.b.cnt[i] = 0;
  __syncthreads();
  PSTAMP(1);
  for (int i = beg + tid; i < end; i += G) {  // scatter (node, count) into the buckets
    const int s2 = S.u.b.map[(int)(w[i].k & p.emask) - lo];
    const int64_t pos = qb + S.u.b.off[s2] + atomicAdd(&S.u.b.cnt[s2], 1);
    p.bent[pos] = make_int2(S.root + (int)(w[i].k >> p.ebits), (int)w[i].c);
  }
  __syncthreads();
  // candidate records (bucket sizes: the fill counters)
  for (int s2 = tid; s2 < nc; s2 += G)
    p.cand[cbase + s2] = make_int4(S.u.b.st[s2], (int32_t)(qb + S.u.b.off[s2]), S.u.b.cnt[s2], 0);
  __syncthreads();
  if (tid == 0) {
    S.nent += end - beg;
    S.nreal += end - beg;
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
// than sort_words(G) x 32 entities keeps the hash order (nothing downstream
// depends on the order for correctness: scores scatter by entity, PNA's mean
// and the digests are order-independent sums).
template <int G>
__device__ __forceinline__ int hb_slot(SmemT<G> &S, int t, bool insert) {
  uint32_t h = hash32((uint32_t)t) >> (32 - WBITS);
#pragma unroll 1
  for (int probe = 0; probe < HB; ++probe) {
    const int k = insert ? atomicCAS(&S.u.c.key[h], EMPTY, t) : S.u.c.key[h];
    if (k == t || (insert && k == EMPTY)) return (int)h;
    h = (h + 1) & (HB - 1);
  }
  return -1;  // unreachable: at most HB_LOAD < HB distinct keys
}

template <int G>
__device__ int hash_pass_merged(const KParams &p, SmemT<G> &S, const Ent *w, int beg, int end, int64_t cbase,
                                int lo, int hi);

template <int G>
__device__ int hash_pass(const KParams &p, SmemT<G> &S, const Ent *w, int beg, int end, int64_t cbase,
                         bool degree_only, int lo, int hi) {
  // w: contributions (a = entity, b = node, c = count), window-sorted or raw;
  // every entity lies in [lo, hi)
  const int tid = threadIdx.x;
  const int w0 = lo >> 5, nw = ((hi - 1) >> 5) - w0 + 1;
  // candidates in ascending entity order (the reference's nonzero order, and
  // neighbouring lanes of the scoring pass then touch neighbouring score entries)
  const bool by_rank = !degree_only && nw <= sort_words(G);
  if (by_rank) return hash_pass_merged(p, S, w, beg, end, cbase, lo, hi);
  for (int i = tid; i < HB; i += G) {
    S.u.c.key[i] = EMPTY;
    S.u.c.cnt[i] = 0;
    S.u.c.off[i] = 0;
  }
  if (by_rank)
    for (int i = tid; i < nw; i += G) S.sbits[i] = 0u;
  __syncthreads();
  for (int i = beg + tid; i < end; i += G) atomicAdd(&S.u.c.cnt[hb_slot(S, (int)(w[i].k & p.emask), true)], 1);
  __syncthreads();
  constexpr int PER = HB / G;
  int loc[PER];
  int nc;
  if (by_rank) {
    for (int i = tid; i < HB; i += G) {
      const int k = S.u.c.key[i];
      if (k != EMPTY) atomicOr(&S.sbits[(k >> 5) - w0], 1u << (k & 31));
    }
    __syncthreads();
    // rank of a bit = popcounts of the words before it + of its word below it
    const int per = (nw + G - 1) / G;
    int sum = 0;
    for (int j = 0; j < per; ++j) {
      const int i = tid * per + j;
      if (i < nw) sum += __popc(S.sbits[i]);
    }
    int base = block_scan<G>(sum, S.ws, nc);
    for (int j = 0; j < per; ++j) {
      const int i = tid * per + j;
      if (i < nw) {
        S.spre[i] = (unsigned short)base;
        base += __popc(S.sbits[i]);
      }
    }
    __syncthreads();
    for (int i = tid; i < HB; i += G) {
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
    int run = block_scan<G>(s2, S.ws, tot);
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
    int run = block_scan<G>(sum, S.ws, total);
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
    for (int i = tid; i < HB; i += G) S.u.c.cnt[i] = 0;
    __syncthreads();
    for (int i = beg + tid; i < end; i += G)
      degree_add(S, reinterpret_cast<uint32_t *>(&S.u.c.cnt[hb_slot(S, (int)(w[i].k & p.emask), false)]), w[i].c,
                 p.rl.node_nrules[S.root + (int)(w[i].k >> p.ebits)]);
    __syncthreads();
    for (int i = tid; i < HB; i += G) {
      if (S.u.c.key[i] != EMPTY) {
        const float degf = (float)((double)(uint32_t)S.u.c.cnt[i] + 1.0);
        atomicAdd(&S.sumlog, (unsigned long long)(long long)llrint((double)logf(degf) * 4294967296.0));
      }
    }
    __syncthreads();
    return nc;
  }
  // bucket start of hash slot i: off is indexed by rank (by_rank) or by slot;
  // the pass's entries follow the query's earlier ones
  const int64_t qb = S.qbase + S.nent;
  for (int i = tid; i < HB; i += G) {
    if (S.u.c.key[i] != EMPTY) {
      const int cid = S.u.c.cid[i];
      const int64_t c = cbase + cid;
      p.cand[c] = make_int4(S.u.c.key[i], (int32_t)(qb + S.u.c.off[by_rank ? cid : i]), S.u.c.cnt[i], 0);
    }
  }
  __syncthreads();
  for (int i = tid; i < HB; i += G) S.u.c.cnt[i] = 0;
  __syncthreads();
  for (int i = beg + tid; i < end; i += G) {  // scatter (node, count) into the buckets
    const int sl2 = hb_slot(S, (int)(w[i].k & p.emask), false);
    const int64_t pos = qb + S.u.c.off[by_rank ? S.u.c.cid[sl2] : sl2] + atomicAdd(&S.u.c.cnt[sl2], 1);
    p.bent[pos] = make_int2(S.root + (int)(w[i].k >> p.ebits), (int)w[i].c);
  }
  __syncthreads();
  if (tid == 0) {
    S.nent += end - beg;
    S.nreal += end - beg;
  }
  __syncthreads();
  return nc;
}

// hash_pass with the candidates ranked by entity (the pass's entity range
// within sort_words(G) x 32) and the contributions MERGED: phase A emits a
// rule-end (trie node, entity) once per path prefix that reaches it (its
// hash merges only the inner levels), so one candidate's bucket can hold one
// node several times.  Here the LDS hash is keyed by the whole (node, entity)
// key and sums the counts (u32, carry-checked as in phase A), so every
// bucket holds each node once — the reference's stacked rule_count has one
// entry per (rule, candidate) (predictors.py:239-244).  Counts add exactly,
// and every consumer of the buckets (features, memos, digests, EM scores and
// statistics, backward) is a sum over the entries: results are unchanged.
// Writes the pass's distinct entries after the query's earlier ones.
template <int G>
__device__ int hash_pass_merged(const KParams &p, SmemT<G> &S, const Ent *w, int beg, int end, int64_t cbase,
                                int lo, int hi) {
  const int tid = threadIdx.x;
  const int w0 = lo >> 5, nw = ((hi - 1) >> 5) - w0 + 1;
  constexpr int PER = HB / G;
  for (int i = tid; i < HB; i += G) {
    S.u.c.key[i] = EMPTY;
    S.u.c.cnt[i] = 0;
    S.u.c.off[i] = 0;
  }
  for (int i = tid; i < nw; i += G) S.sbits[i] = 0u;
  __syncthreads();
  // (node, entity) keys (< 2^31: never EMPTY), counts summed
  for (int i = beg + tid; i < end; i += G) {
    const Ent e = w[i];
    const int sl = hb_slot(S, (int)e.k, true);
    const uint32_t old = atomicAdd(reinterpret_cast<uint32_t *>(&S.u.c.cnt[sl]), e.c);
    if (old + e.c < old) atomicOr(&S.err, ERR_COUNT_WIDTH);  // carry out of the u32 path count
  }
  __syncthreads();
  for (int i = tid; i < HB; i += G) {
    const int k = S.u.c.key[i];
    if (k != EMPTY) {
      const int t = k & (int)p.emask;
      atomicOr(&S.sbits[(t >> 5) - w0], 1u << (t & 31));
    }
  }
  __syncthreads();
  // rank of an entity = popcounts of the words before it + of its word below it
  const int per = (nw + G - 1) / G;
  int sum = 0;
  for (int j = 0; j < per; ++j) {
    const int i = tid * per + j;
    if (i < nw) sum += __popc(S.sbits[i]);
  }
  int nc;
  int base = block_scan<G>(sum, S.ws, nc);
  for (int j = 0; j < per; ++j) {
    const int i = tid * per + j;
    if (i < nw) {
      S.spre[i] = (unsigned short)base;
      base += __popc(S.sbits[i]);
    }
  }
  __syncthreads();
  // per key its candidate (rank); bucket sizes (distinct nodes) by rank
  for (int i = tid; i < HB; i += G) {
    const int k = S.u.c.key[i];
    if (k != EMPTY) {
      const int kk = (k & (int)p.emask) - (w0 << 5), wd = kk >> 5;
      const int rank = S.spre[wd] + __popc(S.sbits[wd] & ((1u << (kk & 31)) - 1u));
      S.u.c.cid[i] = rank;
      atomicAdd(&S.u.c.off[rank], 1);
    }
  }
  __syncthreads();
  // exclusive scan of the bucket sizes (rank order): off[rank] = bucket start
  int loc[PER];
  int s2 = 0;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    loc[j] = S.u.c.off[tid * PER + j];
    s2 += loc[j];
  }
  int nd;
  int run = block_scan<G>(s2, S.ws, nd);
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    S.u.c.off[tid * PER + j] = run;
    run += loc[j];
  }
  // this thread's keys' counts to registers: cnt becomes the buckets' fill counters
  uint32_t mine[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) mine[j] = (uint32_t)S.u.c.cnt[tid + j * G];
  __syncthreads();
  for (int i = tid; i < HB; i += G) S.u.c.cnt[i] = 0;
  __syncthreads();
  const int64_t qb = S.qbase + S.nent;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int i = tid + j * G;
    const int k = S.u.c.key[i];
    if (k != EMPTY) {
      const int rank = S.u.c.cid[i];
      const int start = S.u.c.off[rank];
      const int at = atomicAdd(&S.u.c.cnt[rank], 1);
      p.bent[qb + start + at] = make_int2(S.root + (int)((uint32_t)k >> p.ebits), (int)mine[j]);
      if (at == 0) {  // the bucket's first writer writes its candidate record
        const int size = (rank + 1 < nc ? S.u.c.off[rank + 1] : nd) - start;
        p.cand[cbase + rank] = make_int4(k & (int)p.emask, (int32_t)(qb + start), size, 0);
      }
    }
  }
  __syncthreads();
  if (tid == 0) {
    S.nent += nd;
    S.nreal += nd;
  }
  __syncthreads();
  return nc;
}

// Counting sort of the contributions by sort window (2^sbits entities,
// fwd.h SORT_WINS) into the frontier buffer f(0) (free during phase B), then
// consecutive windows in hash passes of up to HB_LOAD contributions (which
// merge duplicate (node, entity) entries, hash_pass_merged), a window of
// more than HB_LOAD contributions alone in the dense window_pass.
template <int G>
__device__ int candidates_phase(const KParams &p, SmemT<G> &S, const Slot &sl, int P, bool degree_only, bool sorted) {
  const int tid = threadIdx.x;
  // all contributions fit one hash pass: no window sort (it exists only to
  // bound the hash load) — one read of the raw list instead of a sorted copy
  if (P <= HB_LOAD) return P > 0 ? hash_pass(p, S, sl.ct, 0, P, S.qbase, degree_only, 0, p.g.E) : 0;
  const int sb = p.sbits;
  const int nwin = (p.g.E + (1 << sb) - 1) >> sb;
  // a graph of at most one window (kinship, UMLS): the dense pass over the
  // raw list, without the window-sorted copy
  if (nwin == 1) return window_pass(p, S, sl.ct, 0, 0, P, S.qbase, degree_only);
  if (!sorted) {
    for (int i = tid; i < nwin; i += G) S.whist[i] = 0;
    __syncthreads();
    for (int i = tid; i < P; i += G) atomicAdd(&S.whist[(int)(sl.ct[i].k & p.emask) >> sb], 1);
    __syncthreads();
    // window starts: a block scan of the histogram (consecutive windows per thread)
    const int per = (nwin + G - 1) / G;
    int loc = 0;
    for (int j = 0; j < per; ++j) {
      const int i = tid * per + j;
      if (i < nwin) loc += S.whist[i];
    }
    int total;
    int acc = block_scan<G>(loc, S.ws, total);
    for (int j = 0; j < per; ++j) {
      const int i = tid * per + j;
      if (i < nwin) {
        S.wbeg[i] = acc;
        S.wfill[i] = acc;
        acc += S.whist[i];
      }
    }
    if (tid == 0) S.wbeg[nwin] = total;
    __syncthreads();
    for (int i = tid; i < P; i += G) {
      const Ent ce = sl.ct[i];
      const int t = (int)(ce.k & p.emask);
      const int pos = atomicAdd(&S.wfill[t >> sb], 1);
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
      ncand += window_pass(p, S, sl.f(0), w << sb, beg, S.wbeg[w + 1], S.qbase + ncand, degree_only);
      ++w;
      continue;
    }
    int w2 = w + 1;
    while (w2 < nwin && S.wbeg[w2 + 1] - beg <= HB_LOAD) ++w2;
    if (S.wbeg[w2] > beg)
      ncand += hash_pass(p, S, sl.f(0), beg, S.wbeg[w2], S.qbase + ncand, degree_only, w << sb,
                         min(w2 << sb, p.g.E));
    w = w2;
  }
  return ncand;
}

template <int G>
__device__ __forceinline__ void flag_error(const KParams &p, unsigned int *hdr, SmemT<G> &S, int q) {
  atomicOr(&hdr[H_STATUS], S.err ? 2u : 1u);
  if (S.err) {
    atomicOr(&hdr[H_ERRBITS], (unsigned)S.err);
    atomicExch(&hdr[H_ERRQ], (unsigned)q);
  }
  if (p.n_cand) p.n_cand[q] = S.err ? -2 : -1;
}

template <int AGG, int G>
// (512 / 1024 lanes: 4 waves per SIMD, two / one workgroups per CU: <= 128 VGPRs)
__global__ __launch_bounds__(G, G >= 512 ? 4 : 1) void ground_kernel(KParams p) {
  __shared__ SmemT<G> S;
  const int tid = threadIdx.x;
  unsigned int *hdr = reinterpret_cast<unsigned int *>(p.ws);
  unsigned long long *pool_ctr = reinterpret_cast<unsigned long long *>(p.ws + 64);
  const Slot sl = make_slot(p.slots, blockIdx.x, p.fcap, p.pcap);
  for (int s = tid; s < HCAP; s += G) {
    S.u.a.key[s] = EMPTY;
    S.u.a.val[s] = 0u;
  }
  unsigned long long pr[6] = {0, 0, 0, 0, 0, 0};
  if (tid < 8) S.tp[tid] = 0ull;
  unsigned long long t_q = 0, t_a = 0;
  __syncthreads();
#pragma unroll 1
  while (true) {
    if (tid == 0) {
      const int qi = (int)atomicAdd(&hdr[H_DEQUEUE], 1u);
      S.q = qi < p.nq && p.order ? p.order[qi] : qi;
    }
    __syncthreads();
    const int q = S.q;
    if (q >= p.nq) break;
    if (p.prof && tid == 0) t_q = __builtin_amdgcn_s_memtime();
    const int h = (int)p.all_h[q];
    const int r = (int)p.all_r[q];
    const int root = p.rl.head_root[r];
    if (tid == 0 && r != (int)p.all_r[0]) atomicOr(&hdr[H_FLAGS], (unsigned)FLAG_MIXED);
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
      S.nocc = 0;
      S.ovf = 0;
      S.nent = 0;
      S.nreal = 0;
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
      for (int s = tid; s < HCAP; s += G) {  // leave the LDS hash clean for the next query
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
      atomicAdd(reinterpret_cast<unsigned long long *>(hdr + H_NENT), (unsigned long long)S.nreal);
      p.q_base[q] = S.qbase;
      if (p.prof) {
        pr[2] += __builtin_amdgcn_s_memtime() - t_a;
        pr[3] += 1;
        pr[4] += P;
        pr[5] += ncand;
      }
    }
    for (int s = tid; s < HCAP; s += G) {  // restore the phase-A hash (phase B reused its LDS)
      S.u.a.key[s] = EMPTY;
      S.u.a.val[s] = 0u;
    }
    __syncthreads();
  }
  if (p.prof && tid == 0) {
#pragma unroll
    for (int k = 0; k < 6; ++k) atomicAdd(&p.prof[k], pr[k]);
#pragma unroll
    for (int k = 0; k < 7; ++k) atomicAdd(&p.prof[6 + k], S.tp[k]);
  }
}

// ---------------------------------------------------------------- scoring chunks
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

// Blocks past nrb (the row blocks) only clear the pair-memo table (when it is
// small: one launch's rows up to a few hundred; larger tables take a memset).
constexpr int PTAB_KERNEL_ZERO_BITS = 16;
__global__ __launch_bounds__(CHB) void chunk_fill_kernel(KParams p, const int *__restrict__ bsum, int nrb) {
  __shared__ int s_ws[CHB / 64];
  __shared__ long long s_pb[CHB / 64], s_pt[CHB / 64];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  // the scoring pass's launch state, cleared here rather than by two
  // dispatches of their own (each one waits for a slot beside RotatE): its
  // chunk dequeue counter and, when it uses one, the pair-memo table
  if (blockIdx.x == 0 && tid == 0) reinterpret_cast<unsigned int *>(p.ws)[H_DEQUEUE2] = 0u;
  if (p.ptab && p.psbits <= PTAB_KERNEL_ZERO_BITS) {
    const int64_t words = (int64_t)1 << (p.psbits - 1);  // 16-B words of the 2^psbits 8-B slots
    uint4 *t = reinterpret_cast<uint4 *>(p.ptab);
    for (int64_t i = (int64_t)blockIdx.x * CHB + tid; i < words; i += (int64_t)gridDim.x * CHB)
      t[i] = make_uint4(0u, 0u, 0u, 0u);
  }
  if ((int)blockIdx.x >= nrb) return;  // block-uniform, before any barrier
  // this block's prefix and the list total from the per-block totals (one
  // block, bsum == nullptr: the total is this block's own sum, below)
  long long pb = 0, pt = 0;
  for (int k = tid; bsum && k < nrb; k += CHB) {
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
    if (!bsum) total = acc;
    if (blockIdx.x == 0)
      *reinterpret_cast<unsigned long long *>(reinterpret_cast<unsigned int *>(p.ws) + H_CHUNKS) = total;
  }
  __syncthreads();
  const long long off = s_pb[0] + s_ws[wid] + v - n;
  for (int k = 0; k < n; ++k) p.chunks[off + k] = make_int2(q, k << 6);
}

void launch_chunk_list(const KParams &p, hipStream_t st) {
  const unsigned nb = (unsigned)((p.nq + CHB - 1) / CHB);
  // extra blocks for a small pair-memo table (2^psbits 8-B slots): ~64 KB
  // each; a larger table (large launches) is cleared by a memset
  const bool zk = p.ptab && p.psbits <= PTAB_KERNEL_ZERO_BITS;
  const unsigned zb = zk ? (unsigned)(((8ll << p.psbits) >> 16) + 1) : 0u;
  if (p.ptab && !zk) (void)hipMemsetAsync(p.ptab, 0, 8ull << p.psbits, st);
  if (nb == 1) {  // one row block (<= 256 rows, e.g. a reference batch per call): one launch
    hipLaunchKernelGGL(chunk_fill_kernel, dim3(1 + zb), dim3(CHB), 0, st, p, (const int *)nullptr, 1);
    return;
  }
  int *bsum = reinterpret_cast<int *>(p.chunks + p.chunk_cap);  // nb ints after the list (layout)
  hipLaunchKernelGGL(chunk_sum_kernel, dim3(nb), dim3(CHB), 0, st, p, bsum);
  hipLaunchKernelGGL(chunk_fill_kernel, dim3(nb + zb), dim3(CHB), 0, st, p, (const int *)bsum, (int)nb);
}

// ---------------------------------------------------------------- node weights
// Grid-stride over (node, dim) pairs; the table-wide max |s1| (the SUM table's
// shift) is reduced per thread, per wave and per block before one atomic per
// block (one atomic per lane on a single word serialised at ~0.5 ms).
// SUM: the record is FuncToNodeSum's Linear(16, 16) weight times the node's
// sum, y[o] = sum_i add_w[o][i] x[i] (fp32, i ascending; x from the node's 16
// lanes by width-16 shuffles): the Linear commutes with the candidate's sum of
// count x record, so the scoring pass adds only its bias.
// Nodes [lo, lo + cnt) (all of them, or one head relation's trie).
__global__ __launch_bounds__(256) void node_weights_kernel(RulesDev rl, int lo, int cnt, const float *__restrict__ emb,
                                                          int ld, int agg, const float *__restrict__ add_w,
                                                          unsigned char *__restrict__ out) {
  const int64_t total = (int64_t)cnt * 16;
  unsigned int m = 0, m2 = 0;
  for (int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; gid < total;
       gid += (int64_t)gridDim.x * blockDim.x) {
    const int n = lo + (int)(gid >> 4), d = (int)(gid & 15);
    float s1 = 0.f, s2 = 0.f, mn = __builtin_huge_valf(), mx = -__builtin_huge_valf();
    for (int k = rl.node_rule_ptr[n]; k < rl.node_rule_ptr[n + 1]; ++k) {
      const float x = emb[(int64_t)rl.node_rules[k] * ld + d];
      s1 += x;
      s2 += x * x;
      mn = fminf(mn, x);
      mx = fmaxf(mx, x);
    }
    if (agg == RNNL_AGG_SUM) {
      // the node's 16 lanes are one aligned width-16 group (total is a multiple of 16)
      float y = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) y = fmaf(__shfl(s1, i, 16), add_w[d * 16 + i], y);
      // f32 for now; node_fix_kernel turns it into int32 fixed point
      reinterpret_cast<float *>(out + (int64_t)n * kStrideSum)[d] = y;
      m = max(m, __float_as_uint(fabsf(y)));
      m2 = max(m2, __float_as_uint(fabsf(s1)));  // the node aggregate itself (range guard, §3.13)
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
    if (m2) atomicMax(trailer + 3, m2);  // PNA: max |sum x^2| bits; SUM: max |sum x| bits (pre-Linear)
  }
}

// PNA records: sum x and sum x^2 to int32 fixed point, each column with its
// own table-wide shift (as the SUM table: every value fits 2^30, so count x
// record is exact in int64); shifts in trailer[1] / trailer[4], trailer[2]
// flags a table that cannot be represented (or held a NaN min / max).
__global__ void pna_fix_kernel(int n_nodes, int lo, int cnt, unsigned char *__restrict__ out) {
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
  const int64_t n = (int64_t)cnt * 32;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t node = lo + (i >> 5);
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

// per query a block: its candidates' buckets in candidate order (a merged
// short bucket leaves a gap behind it in the pool), output offsets by a block
// scan of the bucket lengths
constexpr int EXP_BS = 256;
__global__ __launch_bounds__(EXP_BS) void export_entries_kernel(KParams p, const int64_t *__restrict__ ent_off,
                                                                int32_t *__restrict__ out_node,
                                                                int32_t *__restrict__ out_count) {
  __shared__ int s_ws[EXP_BS / 64 + 1];
  for (int q = blockIdx.x; q < p.nq; q += gridDim.x) {
    const int nc = p.n_cand[q];  // block-uniform
    if (nc <= 0) continue;
    const int64_t qb = p.q_base[q];
    int64_t o = ent_off[q];
    for (int base = 0; base < nc; base += EXP_BS) {
      const int s = base + (int)threadIdx.x;
      const int4 cr = s < nc ? p.cand[qb + s] : make_int4(0, 0, 0, 0);
      int total;
      const int at = block_scan<EXP_BS>(cr.z, s_ws, total);
      for (int i = 0; i < cr.z; ++i) {
        const int2 be = p.bent[cr.y + i];
        out_node[o + at + i] = be.x;
        out_count[o + at + i] = be.y;
      }
      o += total;
    }
  }
}

// SUM records -> int32 fixed point with one shift for the whole table:
// |fix| < 2^30 for the largest |sum|, so a candidate's int64 sum of
// count x fix is exact (deterministic in any entry order) with ~2^-30
// relative resolution.  Trailer: u32 max|x| bits, i32 shift (fix_shift), bad flag, u32 max|sum x| bits
// before the Linear fold (range-checked as well).
__global__ void node_fix_kernel(int n_nodes, int lo, int cnt, unsigned char *__restrict__ out) {
  unsigned int *trailer = reinterpret_cast<unsigned int *>(out + (int64_t)n_nodes * kStrideSum);
  bool bad;
  // trailer[3]: max |sum x| bits before the folded Linear — an aggregate of
  // 2^30 or more fails the launch as it did before the fold
  const int shift = fix_shift(trailer, bad, trailer[3]);
  const float sc = ldexpf(1.f, shift);
  const int64_t n = (int64_t)cnt * 16;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float *f = reinterpret_cast<float *>(out) + (int64_t)lo * 16 + i;
    *reinterpret_cast<int *>(f) = bad ? 0 : (int)rintf(*f * sc);
  }
}

}  // namespace rnnl

namespace rnnl {

// Graph/rules/rows/workspace part of the launch parameters, shared by the
// forward, the ground-only launch and the COO export.
int setup_params(const char *who, rnnl_graph g, rnnl_rules r, const int64_t *all_h, const int64_t *all_r,
                        const int64_t *etr, int32_t nq, int32_t *n_cand, void *ws, size_t ws_bytes, int32_t scale,
                        KParams &p) {
  if (!g || !r || !all_h || !all_r || !ws || !n_cand || nq < 0 || scale < 1) {
    set_error(std::string(who) + ": bad arguments");
    return RNNL_ERR_INVALID;
  }
  if ((int64_t)g->d.E > (int64_t)SORT_WINS << MAX_SBITS) {
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
  // phase B's sort windows: WIN entities (finer windows merge more duplicate
  // entries in hash passes but cost more passes: FB15k-237 bias step 9.2 ms at
  // 2048 entities, 9.8 at 256, 11.1 at 16 — tools/sort_ab.py)
  int min_bits = 0;
  while (((int64_t)g->d.E + (1ll << min_bits) - 1) >> min_bits > SORT_WINS) ++min_bits;
  p.sbits = std::max(min_bits, WBITS);
  if (g_sort_bits >= min_bits && g_sort_bits <= WBITS) p.sbits = g_sort_bits;
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
  p.order = nullptr;  // set by launch_ground on launches of more rows than workgroups
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
// The grounding's dequeue order (RNNL_HEAVY_FIRST; 0 = row order): rows by
// an estimate of their work, heaviest first, so that the launch does not end
// on a workgroup that dequeued a heavy query late — the FB15k-237 split's
// heaviest queries cost ~14x the mean, and in row order the launch's tail is
// ~0.35 ms of ~6.1 (tools/tail_sim.py, from the C oracle's per-query work).
// The estimate is the head's out-degree times the relation's trie size
// (log-correlation 0.79 with the work); the rows are counting-sorted by its
// log2 bucket, descending (two passes of many workgroups).  Only the
// order of the queries changes: every query's outputs are its own, so the
// results are the same.
#ifndef RNNL_HEAVY_FIRST
#define RNNL_HEAVY_FIRST 1
#endif
constexpr int ORDER_BS = 256, ORDER_BUCKETS = 64;

// the row's log2 work bucket, heaviest = 0
__device__ __forceinline__ int order_bucket(const KParams &p, int q) {
  const int h = (int)p.all_h[q], r = (int)p.all_r[q];
  const long long deg = (long long)p.g.off[(int64_t)(h + 1) * p.g.R] - p.g.off[(int64_t)h * p.g.R];
  const int root = p.rl.head_root[r];
  const unsigned long long w = root < 0 ? 0ull : (unsigned long long)(deg + 1) * (unsigned)p.rl.head_nodes[r];
  return ORDER_BUCKETS - 1 - min(ORDER_BUCKETS - 1, 63 - __clzll(w | 1ull));
}

// pass 1: each row's bucket (kept in `bk`) and the buckets' sizes (`cnt`, zeroed by the caller)
__global__ __launch_bounds__(ORDER_BS) void order_count_kernel(KParams p, unsigned char *__restrict__ bk,
                                                               int *__restrict__ cnt) {
  __shared__ int s_hist[ORDER_BUCKETS];
  if (threadIdx.x < ORDER_BUCKETS) s_hist[threadIdx.x] = 0;
  __syncthreads();
  const int q = blockIdx.x * ORDER_BS + threadIdx.x;
  if (q < p.nq) {
    const int b = order_bucket(p, q);
    bk[q] = (unsigned char)b;
    atomicAdd(&s_hist[b], 1);
  }
  __syncthreads();
  if (threadIdx.x < ORDER_BUCKETS && s_hist[threadIdx.x]) atomicAdd(&cnt[threadIdx.x], s_hist[threadIdx.x]);
}

// pass 2: rows scattered by bucket, heaviest buckets first (`cnt` becomes
// the buckets' fill counters past their starts)
__global__ __launch_bounds__(ORDER_BS) void order_fill_kernel(KParams p, const unsigned char *__restrict__ bk,
                                                              int *__restrict__ cnt, int32_t *__restrict__ order) {
  __shared__ int s_base[ORDER_BUCKETS], s_hist[ORDER_BUCKETS], s_off[ORDER_BUCKETS];
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int b = 0; b < ORDER_BUCKETS; ++b) {
      s_base[b] = acc;
      acc += cnt[b];
    }
  }
  if (threadIdx.x < ORDER_BUCKETS) s_hist[threadIdx.x] = 0;
  __syncthreads();
  const int q = blockIdx.x * ORDER_BS + threadIdx.x;
  int b = 0, k = 0;
  if (q < p.nq) {
    b = bk[q];
    k = atomicAdd(&s_hist[b], 1);  // this block's rows of bucket b
  }
  __syncthreads();
  if (threadIdx.x < ORDER_BUCKETS && s_hist[threadIdx.x])  // one global reservation per (block, bucket)
    s_off[threadIdx.x] = atomicAdd(&cnt[ORDER_BUCKETS + threadIdx.x], s_hist[threadIdx.x]);
  __syncthreads();
  if (q < p.nq) order[s_base[b] + s_off[b] + k] = q;
}

void launch_ground(const KParams &p0, int agg, hipStream_t st, int grid) {
  KParams p = p0;
  const unsigned g = (unsigned)(grid > 0 ? std::min(grid, p.nslots) : p.nslots);
  // with the chip to itself (beside RotatE the chain has slack), more rows
  // than workgroups, and a graph of more than one phase-B window (kinship's
  // and UMLS's queries cost alike: there the pass's three dispatches only
  // add ~10 us).  tools/ab_order.sh: WN18RR ground + PNA alone 4.64-5.08 ->
  // 4.12-4.19 ms, FB15k-237 bias 9.27 -> 9.23-9.25 ms, the RotatE steps
  // unchanged within the box's noise.
  if (RNNL_HEAVY_FIRST && grid <= 0 && p.nq > (int)g && p.g.E > WIN) {
    int32_t *order = reinterpret_cast<int32_t *>(p.ws + make_layout(p.nq, 1).off_order);
    // the row buckets and the counters in the slot scratch (free until the grounding starts)
    int *cnt = reinterpret_cast<int *>(p.slots);
    unsigned char *bk = p.slots + 4 * 2 * ORDER_BUCKETS;
    (void)hipMemsetAsync(cnt, 0, sizeof(int) * 2 * ORDER_BUCKETS, st);
    const unsigned nb = (unsigned)((p.nq + ORDER_BS - 1) / ORDER_BS);
    hipLaunchKernelGGL(order_count_kernel, dim3(nb), dim3(ORDER_BS), 0, st, p, bk, cnt);
    hipLaunchKernelGGL(order_fill_kernel, dim3(nb), dim3(ORDER_BS), 0, st, p, (const unsigned char *)bk, cnt, order);
    p.order = order;
  }
  // few rows (a reference batch per call): one 1024-lane workgroup per query,
  // so the batch's heaviest query — the launch's critical path — expands
  // four times the frontier items and edges per pass; beside another kernel
  // (a capped grid) 256-lane workgroups; else 512 lanes (GBS / SOLO_GBS, fwd.h)
  const bool wide = p.nq <= WIDE_ROWS;
  const bool beside = grid > 0;
  if (agg == RNNL_AGG_SUM && wide)
    hipLaunchKernelGGL((ground_kernel<RNNL_AGG_SUM, 1024>), dim3(g), dim3(1024), 0, st, p);
  else if (agg == RNNL_AGG_SUM && beside)
    hipLaunchKernelGGL((ground_kernel<RNNL_AGG_SUM, GBS>), dim3(g), dim3(GBS), 0, st, p);
  else if (agg == RNNL_AGG_SUM)
    hipLaunchKernelGGL((ground_kernel<RNNL_AGG_SUM, SOLO_GBS>), dim3(g), dim3(SOLO_GBS), 0, st, p);
  else if (wide)
    hipLaunchKernelGGL((ground_kernel<RNNL_AGG_PNA, 1024>), dim3(g), dim3(1024), 0, st, p);
  else if (beside)
    hipLaunchKernelGGL((ground_kernel<RNNL_AGG_PNA, GBS>), dim3(g), dim3(GBS), 0, st, p);
  else
    hipLaunchKernelGGL((ground_kernel<RNNL_AGG_PNA, SOLO_GBS>), dim3(g), dim3(SOLO_GBS), 0, st, p);
}

void set_score_params(KParams &p, const rnnl_predictor_params *pp, float *score, uint8_t *mask,
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
  p.packed = pp->packed;
  p.score = score;
  p.mask = mask;
  p.digest = digest;
}

bool bad_params(const rnnl_predictor_params *pp, const float *score) {
  return !pp || !score || !pp->node_w || (pp->aggregator != RNNL_AGG_SUM && pp->aggregator != RNNL_AGG_PNA);
}

// Only the workspace carve-up is needed to read the pool back.
KParams export_params(void *ws, int32_t nq, int32_t scale, const int32_t *n_cand) {
  const Layout Ly = make_layout(nq, scale);
  unsigned char *base = static_cast<unsigned char *>(ws);
  KParams p{};
  p.ws = base;
  p.nq = nq;
  p.n_cand = const_cast<int32_t *>(n_cand);
  p.q_base = reinterpret_cast<int64_t *>(base + Ly.off_qbase);
  p.cand = reinterpret_cast<int4 *>(base + Ly.off_cand);
  p.bent = reinterpret_cast<int2 *>(base + Ly.off_bent);
  return p;
}

}  // namespace rnnl

int rnnl::node_fix_enqueue(rnnl_rules r, void *node_w, void *stream) {
  const int64_t n = (int64_t)r->d.n_nodes * 16;
  if (n == 0) return RNNL_OK;
  const int bs = 256;
  hipLaunchKernelGGL(node_fix_kernel, dim3((unsigned)std::min<int64_t>((n + bs - 1) / bs, 4096)), dim3(bs), 0,
                     (hipStream_t)stream, r->d.n_nodes, 0, r->d.n_nodes, static_cast<unsigned char *>(node_w));
  RNNL_HIP_CHECK(hipGetLastError());
  return RNNL_OK;
}

using namespace rnnl;

extern "C" {

static int node_weights_range(const char *who, rnnl_rules r, int lo, int cnt, const float *emb, int32_t ld,
                              int32_t agg, const float *add_w, void *node_w, void *stream) {
  if (!r || !emb || !node_w || (agg != RNNL_AGG_SUM && agg != RNNL_AGG_PNA) || ld < 16 ||
      (agg == RNNL_AGG_SUM && !add_w)) {
    set_error(std::string(who) + ": bad arguments");
    return RNNL_ERR_INVALID;
  }
  const int64_t n = (int64_t)cnt * 16;
  unsigned char *out = static_cast<unsigned char *>(node_w);
  RNNL_HIP_CHECK(hipMemsetAsync(out + (int64_t)r->d.n_nodes * (agg == RNNL_AGG_SUM ? kStrideSum : kStridePna), 0, 32,
                                (hipStream_t)stream));
  if (n == 0) return RNNL_OK;
  const int bs = 256;
  hipLaunchKernelGGL(node_weights_kernel, dim3((unsigned)std::min<int64_t>((n + bs - 1) / bs, 2048)), dim3(bs), 0,
                     (hipStream_t)stream, r->d, lo, cnt, emb, ld, agg, add_w, out);
  if (agg == RNNL_AGG_PNA)
    hipLaunchKernelGGL(pna_fix_kernel, dim3((unsigned)std::min<int64_t>((2 * n + bs - 1) / bs, 4096)), dim3(bs), 0,
                       (hipStream_t)stream, r->d.n_nodes, lo, cnt, out);
  if (agg == RNNL_AGG_SUM)
    hipLaunchKernelGGL(node_fix_kernel, dim3((unsigned)std::min<int64_t>((n + bs - 1) / bs, 4096)), dim3(bs), 0,
                       (hipStream_t)stream, r->d.n_nodes, lo, cnt, out);
  RNNL_HIP_CHECK(hipGetLastError());
  return RNNL_OK;
}

int rnnl_node_weights(rnnl_rules r, const float *emb, int32_t ld, int32_t agg, const float *add_w, void *node_w,
                      void *stream) {
  if (!r) {
    set_error("rnnl_node_weights: bad arguments");
    return RNNL_ERR_INVALID;
  }
  return node_weights_range("rnnl_node_weights", r, 0, r->d.n_nodes, emb, ld, agg, add_w, node_w, stream);
}

int rnnl_node_weights_head(rnnl_rules r, int32_t head, const float *emb, int32_t ld, int32_t agg,
                           const float *add_w, void *node_w, void *stream) {
  if (!r || head < 0 || head >= (int)r->head_root.size()) {
    set_error("rnnl_node_weights_head: bad arguments");
    return RNNL_ERR_INVALID;
  }
  const int lo = r->head_root[head];
  return node_weights_range("rnnl_node_weights_head", r, lo < 0 ? 0 : lo, lo < 0 ? 0 : r->head_nodes[head], emb, ld,
                            agg, add_w, node_w, stream);
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
  launch_score(p, r->d, st, 0);
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
  if (bad_params(pp, score) || !n_cand || (deferred != 0 && deferred != 2) ||
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
  p.atomic_out = deferred == 2;
  hipStream_t st = (hipStream_t)stream;
  launch_score(p, r->d, st, workgroups);  // (its chunk-list kernel resets the scoring dequeue counter)
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
  launch_ground(p, RNNL_AGG_SUM, st);
  RNNL_HIP_CHECK(hipGetLastError());
  return RNNL_OK;
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
  hipLaunchKernelGGL(export_entries_kernel, dim3((unsigned)std::min<int64_t>(nq, 4096)), dim3(EXP_BS), 0,
                     (hipStream_t)stream, p, ent_off, out_node, out_count);
  RNNL_HIP_CHECK(hipGetLastError());
  return RNNL_OK;
}

int rnnl_debug_pair_memo(int32_t on) {
  g_pair_memo = on != 0;
  return RNNL_OK;
}

int rnnl_debug_sort_bits(int32_t bits) {
  g_sort_bits = bits;
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

// Per (host thread, device) resources of the host side of a forward: a pinned
// copy of the launch header (a status read is one small DMA + one wait) and
// the side streams / events of the RotatE overlap
// (rnnl_predictorplus_forward_rotate).  Created on first use, kept.
struct HostSide {
  unsigned int *pinned = nullptr;
  hipStream_t a = nullptr, b = nullptr;
  hipEvent_t in = nullptr, zero = nullptr, side = nullptr, mask = nullptr;
};

// The HIP device API of hostside.h's keying: the host-side resources, the
// side streams and a null `stream` argument all belong to the current device,
// which need not be the device of the tensors (a caller on cuda:k that never
// called set_device) — every entry point holds a DeviceGuard for the device
// of its stream / graph first.
struct HipDeviceApi {
  static int get_device(int *dev) { return hipGetDevice(dev) == hipSuccess ? 0 : 1; }
  static int set_device(int dev) { return hipSetDevice(dev) == hipSuccess ? 0 : 1; }
  static int stream_device(void *s, int *dev) { return hipStreamGetDevice((hipStream_t)s, dev) == hipSuccess ? 0 : 1; }
};
using DeviceGuard = DeviceGuardT<HipDeviceApi>;
static int stream_device(void *stream) { return stream_device_of<HipDeviceApi>(stream); }

static std::map<int, HostSide> &host_sides() {
  thread_local std::map<int, HostSide> all;
  return all;
}

// The current device's resources (callers hold a DeviceGuard for the device
// of their data / stream).
static HostSide *host_side() {
  HostSide *h = current_device_entry<HipDeviceApi>(host_sides());
  if (!h) return nullptr;
  if (!h->pinned && hipHostMalloc(reinterpret_cast<void **>(&h->pinned), 256, hipHostMallocDefault) != hipSuccess) {
    h->pinned = nullptr;
    return nullptr;
  }
  return h;
}

// The launch header's status words into st (one read-back on `stream`).
static int read_header(void *ws, void *stream, unsigned int (&st)[STATUS_WORDS]) {
  DeviceGuard guard(stream_device(stream));
  HostSide *h = host_side();
  if (!h) {
    set_error("rnnl_forward_status: no pinned header buffer");
    return RNNL_ERR_HIP;
  }
  RNNL_HIP_CHECK(hipMemcpyAsync(h->pinned, ws, sizeof(st), hipMemcpyDeviceToHost, (hipStream_t)stream));
  RNNL_HIP_CHECK(hipStreamSynchronize((hipStream_t)stream));
  memcpy(st, h->pinned, sizeof(st));
  return RNNL_OK;
}

static int forward_status(void *ws, void *stream, int64_t *totals) {
  unsigned int st[STATUS_WORDS] = {0};
  if (int rc = read_header(ws, stream, st)) return rc;
  return status_from_header(st, totals);
}

static int status_from_header(const unsigned int *st, int64_t *totals) {
  if (totals) {
    unsigned long long c, e;
    memcpy(&c, st + H_NCAND, 8);
    memcpy(&e, st + H_NENT, 8);
    totals[0] = (int64_t)c;  // candidates (sum of n_cand)
    totals[1] = (int64_t)e;  // bucket entries (distinct (node, candidate) pairs where phase B merged them)
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

int rnnl_forward_status_flags(void *ws, void *stream, int64_t *totals, uint32_t *flags) {
  if (!ws) {
    set_error("rnnl_forward_status_flags: bad arguments");
    return RNNL_ERR_INVALID;
  }
  unsigned int st[STATUS_WORDS] = {0};
  if (int rc = read_header(ws, stream, st)) return rc;
  if (flags) *flags = st[H_FLAGS];
  return status_from_header(st, totals);
}

// PredictorPlus forward with the RotatE entity feature in one host call: the
// stream choreography of the overlap without a Python step per
// launch.  Side stream B zeroes the score rows, then fills the all-True
// mask beside RotatE; side stream A grounds, then (after the zero fill)
// scores with atomic adds; the caller's stream runs RotatE with atomic adds
// after the zero fill and waits for A and the mask; then the header is read
// back (the only wait).  Ground is
// enqueued before RotatE so its persistent workgroups are resident first.
// The side streams / events of the overlap, created on first use.
static HostSide *overlap_side(const char *who) {
  HostSide *h = host_side();
  if (!h) {
    set_error(std::string(who) + ": no host resources");
    return nullptr;
  }
  if (!h->a) {
    if (hipStreamCreateWithFlags(&h->a, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&h->b, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&h->in, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&h->zero, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&h->side, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&h->mask, hipEventDisableTiming) != hipSuccess) {
      set_error(std::string(who) + ": side stream / event creation failed");
      h->a = nullptr;
      return nullptr;
    }
  }
  return h;
}

// Zero fill of the score rows on side stream B, ordered after `stream`'s work
// so far: issued before the rule encoder, it runs beside it instead of
// lengthening the window before RotatE starts.  The next
// rnnl_predictorplus_forward_rotate with zeroed = 1 waits for it.
int rnnl_forward_rotate_zero(float *score, size_t n_floats, void *stream) {
  if (!score) {
    set_error("rnnl_forward_rotate_zero: bad arguments");
    return RNNL_ERR_INVALID;
  }
  DeviceGuard guard(stream_device(stream));
  HostSide *h = overlap_side("rnnl_forward_rotate_zero");
  if (!h) return RNNL_ERR_HIP;
  RNNL_HIP_CHECK(hipEventRecord(h->in, (hipStream_t)stream));
  RNNL_HIP_CHECK(hipStreamWaitEvent(h->b, h->in, 0));
  RNNL_HIP_CHECK(hipMemsetAsync(score, 0, sizeof(float) * n_floats, h->b));
  RNNL_HIP_CHECK(hipEventRecord(h->zero, h->b));
  return RNNL_OK;
}

// The launches of rnnl_predictorplus_forward_rotate (everything but the
// header read-back).  On an error the caller joins the side streams.
static int forward_rotate_enqueue(HostSide *h, rnnl_graph g, rnnl_rules r, const rnnl_predictor_params *pp,
                                  const rnnl_rotate_args *rot, const int64_t *all_h, const int64_t *all_r,
                                  const int64_t *etr, int32_t nq, float *score, uint8_t *mask, int32_t *n_cand,
                                  uint64_t *digest, void *ws, size_t ws_bytes, int32_t scale, int32_t ground_wg,
                                  int32_t score_wg, int32_t zeroed, void *const *events, hipStream_t main,
                                  int32_t E) {
  // events[0..2] (nullable, timing): before the launches, after RotatE and the
  // mask, after the side stream's work (PredictorPlus.forward_rows `events`)
  auto mark = [&](int k) -> hipError_t {
    return events && events[k] ? hipEventRecord((hipEvent_t)events[k], main) : hipSuccess;
  };
  if (!zeroed)
    if (int rc = rnnl_forward_rotate_zero(score, (size_t)nq * (size_t)E, main)) return rc;
  RNNL_HIP_CHECK(hipEventRecord(h->in, main));
  RNNL_HIP_CHECK(mark(0));
  RNNL_HIP_CHECK(hipStreamWaitEvent(h->a, h->in, 0));
  // B fills `mask`, which the caller allocated after the zero fill was
  // enqueued: B must also be ordered after everything the caller's stream
  // has queued up to now (the allocator may have recycled a block that
  // kernels queued there still read)
  RNNL_HIP_CHECK(hipStreamWaitEvent(h->b, h->in, 0));
  if (int rc = rnnl_predictorplus_ground(g, r, pp->aggregator, all_h, all_r, etr, nq, n_cand, ws, ws_bytes, scale,
                                         ground_wg, h->a))
    return rc;
  // RotatE next, so that it starts while the scoring chain is still being
  // enqueued (that chain waits for the grounding on stream A anyway)
  RNNL_HIP_CHECK(hipStreamWaitEvent(main, h->zero, 0));
  if (int rc = rnnl_rotate_score_pieces(rot->eemb, rot->etab, rot->rtab, rot->dim, rot->gamma, all_h, all_r, nq, E,
                                        score, 2, rot->mode, rot->workspace, rot->workspace_bytes, rot->pieces,
                                        rot->first_share, main))
    return rc;
  RNNL_HIP_CHECK(mark(1));
  if (mask) {  // the all-True mask on side stream B beside RotatE (not behind it on `stream`)
    RNNL_HIP_CHECK(hipMemsetAsync(mask, 1, (size_t)nq * (size_t)E, h->b));
    RNNL_HIP_CHECK(hipEventRecord(h->mask, h->b));
  }
  RNNL_HIP_CHECK(hipStreamWaitEvent(h->a, h->zero, 0));
  if (int rc = rnnl_predictorplus_score(g, r, pp, all_h, all_r, nq, score, nullptr, n_cand, digest, ws, ws_bytes,
                                        scale, score_wg, 2, h->a))
    return rc;
  RNNL_HIP_CHECK(hipEventRecord(h->side, h->a));
  RNNL_HIP_CHECK(hipStreamWaitEvent(main, h->side, 0));
  if (mask) RNNL_HIP_CHECK(hipStreamWaitEvent(main, h->mask, 0));
  RNNL_HIP_CHECK(mark(2));
  return RNNL_OK;
}

int rnnl_predictorplus_forward_rotate(rnnl_graph g, rnnl_rules r, const rnnl_predictor_params *pp,
                                      const rnnl_rotate_args *rot, const int64_t *all_h, const int64_t *all_r,
                                      const int64_t *etr, int32_t nq, float *score, uint8_t *mask, int32_t *n_cand,
                                      uint64_t *digest, void *ws, size_t ws_bytes, int32_t scale, int32_t ground_wg,
                                      int32_t score_wg, int32_t zeroed, void *const *events, void *stream,
                                      int64_t *totals, uint32_t *flags) {
  if (bad_params(pp, score) || !rot || !n_cand || !ws || nq < 0 || pp->feature != RNNL_FEATURE_ADD) {
    set_error("rnnl_predictorplus_forward_rotate: bad arguments");
    return RNNL_ERR_INVALID;
  }
  if (nq == 0) return RNNL_OK;
  // the graph's device: the side streams, the host resources and a null
  // `stream` must all be that device's (the caller's current device may differ)
  DeviceGuard guard(g->device);
  HostSide *h = overlap_side("rnnl_predictorplus_forward_rotate");
  if (!h) return RNNL_ERR_HIP;
  hipStream_t main = (hipStream_t)stream;
  const int32_t E = rot->n_entities;
  const int rc = forward_rotate_enqueue(h, g, r, pp, rot, all_h, all_r, etr, nq, score, mask, n_cand, digest, ws,
                                        ws_bytes, scale, ground_wg, score_wg, zeroed, events, main, E);
  if (rc) {
    // a failed enqueue may leave work on side streams A / B that writes the
    // caller's buffers (score, mask, n_cand, ws): join both into `stream`
    // before returning, so that the caller's allocator (which orders frees on
    // `stream`) cannot hand those buffers out while they are still written
    if (hipEventRecord(h->side, h->a) == hipSuccess) (void)hipStreamWaitEvent(main, h->side, 0);
    if (hipEventRecord(h->mask, h->b) == hipSuccess) (void)hipStreamWaitEvent(main, h->mask, 0);
    (void)hipStreamSynchronize(h->a);
    (void)hipStreamSynchronize(h->b);
    return rc;
  }
  return rnnl_forward_status_flags(ws, main, totals, flags);
}

// Where this thread's forward resources for graph g live (the N-GPU bench's
// self-check): out[0] = the graph's device, out[1] / out[2] = the devices of
// the side streams A / B of g's device (-1: not created yet), out[3] = the
// number of devices this thread holds forward resources for.
int rnnl_forward_host_info(rnnl_graph g, int32_t *out) {
  if (!g || !out) {
    set_error("rnnl_forward_host_info: bad arguments");
    return RNNL_ERR_INVALID;
  }
  out[0] = g->device;
  out[1] = out[2] = -1;
  auto &all = host_sides();
  auto it = all.find(g->device);
  if (it != all.end()) {
    int d = -1;
    if (it->second.a && hipStreamGetDevice(it->second.a, &d) == hipSuccess) out[1] = d;
    if (it->second.b && hipStreamGetDevice(it->second.b, &d) == hipSuccess) out[2] = d;
  }
  out[3] = (int32_t)all.size();
  return RNNL_OK;
}

int rnnl_forward_flags_host(const void *header, uint32_t *flags) {
  if (!header || !flags) {
    set_error("rnnl_forward_flags_host: bad arguments");
    return RNNL_ERR_INVALID;
  }
  *flags = static_cast<const unsigned int *>(header)[H_FLAGS];
  return RNNL_OK;
}

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
