// Rule mining on the GPU: the reference miner's
// RuleMiner::search (miner/rnnlogic.cpp:505-589) — for every train triple
// (h, r, t), every relation path of length <= L from h that reaches t while
// the triple's own edge is removed (KnowledgeGraph::rule_search,
// rnnlogic.cpp:350-382) becomes a rule r <- body; the pool is the set of
// distinct (head, body) over all triples, minus the trivial r <- r.
//
// The reference enumerates every path by DFS (deg^L per triple).  Here one
// workgroup per triple (dynamic dequeue):
//   depth 1  the out-edges of h (coalesced CSR range);
//   depth 2  load-balanced expansion of the depth-1 entities' out-edges
//            (block scan of degrees + binary search, as the grounding kernel);
//   depth 3  never expanded: a path ends at t iff its depth-2 entity y has an
//            edge (y, r3, t), so t's in-edges (sorted by source, staged in LDS)
//            are binary-searched for y — deg^2 work per triple instead of deg^3.
// A walk stops at t (the DFS returns at the goal), and the removed edge
// (h, r, t) is skipped at every depth, as in rule_search.  Rules are keyed
// head | len | b1 | b2 | b3 (15 bits each; numeric key order == the
// reference's std::set<Rule> order within a head) and inserted into a global
// open-addressing set, after a per-triple LDS set that drops the duplicates
// one triple produces.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <numeric>
#include <vector>

#include "internal.h"

struct rnnl_miner_s {
  rnnl::MinerDev d;
  std::vector<void *> bufs;
};

namespace rnnl {

constexpr int MB = 256;             // threads per workgroup
constexpr int ICAP = 2048;          // in-edges of t staged in LDS (else read from global)
constexpr int DBITS = 11;
constexpr int DCAP = 1 << DBITS;    // per-triple dedupe set
constexpr uint64_t KEMPTY = ~0ull;
constexpr int GPROBE = 1 << 14;     // global set probe bound (overflow past it)

__device__ __forceinline__ uint64_t rule_key(int head, int len, int b1, int b2, int b3) {
  return ((uint64_t)head << 47) | ((uint64_t)len << 45) | ((uint64_t)b1 << 30) | ((uint64_t)b2 << 15) |
         (uint64_t)b3;
}

__device__ __forceinline__ uint64_t key_hash(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdULL;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ULL;
  return k ^ (k >> 33);
}

struct MineSmem {
  int in_src[ICAP], in_rel[ICAP];
  unsigned long long dd[DCAP];
  int it_x[MB], it_r1[MB], it_off[MB];
  int ws[MB / 64 + 1];
  int q;
};

__device__ __forceinline__ void global_insert(uint64_t key, unsigned long long *table, int64_t cap,
                                              unsigned long long *flags) {
  uint64_t h = key_hash(key) & (uint64_t)(cap - 1);
  if (__hip_atomic_load(&flags[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;  // already too small
  for (int p = 0; p < GPROBE; ++p) {
    const unsigned long long v = __hip_atomic_load(&table[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (v == key) return;
    if (v == KEMPTY) {
      const unsigned long long old = atomicCAS(&table[h], KEMPTY, (unsigned long long)key);
      if (old == KEMPTY || old == key) return;
    }
    h = (h + 1) & (uint64_t)(cap - 1);
  }
  atomicOr(&flags[1], 1ull);  // set full: the caller retries with a larger table
}

__device__ __forceinline__ void emit_rule(MineSmem &S, uint64_t key, unsigned long long *table, int64_t cap,
                                          unsigned long long *flags) {
  uint32_t h = (uint32_t)key_hash(key) & (DCAP - 1);
  for (int p = 0; p < 32; ++p) {
    const unsigned long long old = atomicCAS(&S.dd[h], KEMPTY, (unsigned long long)key);
    if (old == key) return;  // this triple already produced it
    if (old == KEMPTY) break;
    h = (h + 1) & (DCAP - 1);
  }
  global_insert(key, table, cap, flags);
}

__device__ __forceinline__ int mine_scan(int x, int *s_ws, int &total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int v = x;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(v, o, 64);
    if (lane >= o) v += y;
  }
  if (lane == 63) s_ws[wid] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int w = 0; w < MB / 64; ++w) {
      const int t = s_ws[w];
      s_ws[w] = acc;
      acc += t;
    }
    s_ws[MB / 64] = acc;
  }
  __syncthreads();
  const int res = v - x + s_ws[wid];
  total = s_ws[MB / 64];
  __syncthreads();
  return res;
}

// first index in a[lo, hi) with a[i] >= k
template <typename P>
__device__ __forceinline__ int lower_bound_i(P a, int lo, int hi, int k) {
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (a[mid] < k)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo;
}

__global__ __launch_bounds__(MB) void mine_kernel(MinerDev m, int L, unsigned long long *table, int64_t cap,
                                                  unsigned long long *flags) {
  __shared__ MineSmem S;
  const int tid = threadIdx.x;
#pragma unroll 1
  while (true) {
    __syncthreads();
    if (tid == 0) {
      // a full set ends the search early: the caller retries with a larger table
      const bool full = __hip_atomic_load(&flags[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
      S.q = full ? m.n : (int)atomicAdd(&flags[0], 1ull);
    }
    __syncthreads();
    const int q = S.q;
    if (q >= m.n) break;
    const int h = m.th[q], r = m.tr[q], t = m.tt[q];
    // t's in-edges (sources ascending), staged when they fit
    const int ib = m.in_off[t], nin = m.in_off[t + 1] - ib;
    const bool staged = nin <= ICAP;
    if (staged)
      for (int i = tid; i < nin; i += MB) {
        S.in_src[i] = m.in_src[ib + i];
        S.in_rel[i] = m.in_rel[ib + i];
      }
    for (int i = tid; i < DCAP; i += MB) S.dd[i] = KEMPTY;
    __syncthreads();
    const int *isrc = staged ? S.in_src : m.in_src + ib;
    const int *irel = staged ? S.in_rel : m.in_rel + ib;
    const int ob = m.out_off[h], n1 = m.out_off[h + 1] - ob;
    for (int c1 = 0; c1 < n1; c1 += MB) {
      const int i = c1 + tid;
      int deg = 0;
      S.it_x[tid] = -1;
      if (i < n1) {
        const int x = m.out_dst[ob + i], r1 = m.out_rel[ob + i];
        if (!(r1 == r && x == t)) {  // the triple's own edge (rule_search's removed_triplet)
          if (x == t) {
            if (r1 != r) emit_rule(S, rule_key(r, 1, r1, 0, 0), table, cap, flags);  // r <- r is erased
          } else if (L >= 2) {
            S.it_x[tid] = x;
            S.it_r1[tid] = r1;
            deg = m.out_off[x + 1] - m.out_off[x];
          }
        }
      }
      int NE;
      S.it_off[tid] = mine_scan(deg, S.ws, NE);
      __syncthreads();
      const int nit = min(MB, n1 - c1);
      for (int e0 = 0; e0 < NE; e0 += MB) {
        const int j = e0 + tid;
        if (j < NE) {
          int lo = 0, hi = nit - 1;  // largest item with it_off <= j
          while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (S.it_off[mid] <= j)
              lo = mid;
            else
              hi = mid - 1;
          }
          const int x = S.it_x[lo], r1 = S.it_r1[lo];
          const int k = m.out_off[x] + (j - S.it_off[lo]);
          const int y = m.out_dst[k], r2 = m.out_rel[k];
          if (!(x == h && r2 == r && y == t)) {
            if (y == t) {
              emit_rule(S, rule_key(r, 2, r1, r2, 0), table, cap, flags);
            } else if (L >= 3) {
              for (int a = lower_bound_i(isrc, 0, nin, y); a < nin && isrc[a] == y; ++a) {
                const int r3 = irel[a];
                if (!(y == h && r3 == r)) emit_rule(S, rule_key(r, 3, r1, r2, r3), table, cap, flags);
              }
            }
          }
        }
      }
      __syncthreads();
    }
  }
}

__global__ void compact_kernel(const unsigned long long *__restrict__ table, int64_t cap,
                               unsigned long long *__restrict__ out, int64_t out_cap,
                               unsigned long long *__restrict__ flags) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cap; i += (int64_t)gridDim.x * blockDim.x) {
    const unsigned long long k = table[i];
    if (k != KEMPTY) {
      const unsigned long long pos = atomicAdd(&flags[2], 1ull);
      if ((int64_t)pos < out_cap) out[pos] = k;
    }
  }
}

}  // namespace rnnl

using namespace rnnl;

extern "C" {

int rnnl_miner_create(const int32_t *hrt, int64_t n, int32_t E, int32_t R, rnnl_miner *out) {
  if (!out || n < 0 || E <= 0 || R <= 0 || (n > 0 && !hrt) || R >= (1 << 15) || n >= INT32_MAX) {
    set_error("rnnl_miner_create: bad arguments (R < 32768 required)");
    return RNNL_ERR_INVALID;
  }
  for (int64_t i = 0; i < n; ++i)
    if (hrt[3 * i] < 0 || hrt[3 * i] >= E || hrt[3 * i + 2] < 0 || hrt[3 * i + 2] >= E || hrt[3 * i + 1] < 0 ||
        hrt[3 * i + 1] >= R) {
      set_error("rnnl_miner_create: triple out of range");
      return RNNL_ERR_INVALID;
    }
  // out-edges grouped by source, in-edges grouped by target with sources ascending
  std::vector<int32_t> out_off(E + 1, 0), in_off(E + 1, 0);
  for (int64_t i = 0; i < n; ++i) {
    ++out_off[hrt[3 * i] + 1];
    ++in_off[hrt[3 * i + 2] + 1];
  }
  std::partial_sum(out_off.begin(), out_off.end(), out_off.begin());
  std::partial_sum(in_off.begin(), in_off.end(), in_off.begin());
  std::vector<int32_t> out_dst(n), out_rel(n), fill(out_off.begin(), out_off.end() - 1);
  std::vector<int64_t> by_t(n);
  for (int64_t i = 0; i < n; ++i) {
    const int32_t k = fill[hrt[3 * i]]++;
    out_dst[k] = hrt[3 * i + 2];
    out_rel[k] = hrt[3 * i + 1];
    by_t[i] = i;
  }
  std::stable_sort(by_t.begin(), by_t.end(), [&](int64_t a, int64_t b) {
    if (hrt[3 * a + 2] != hrt[3 * b + 2]) return hrt[3 * a + 2] < hrt[3 * b + 2];
    return hrt[3 * a] < hrt[3 * b];
  });
  std::vector<int32_t> in_src(n), in_rel(n), th(n), tr(n), tt(n);
  for (int64_t i = 0; i < n; ++i) {
    in_src[i] = hrt[3 * by_t[i]];
    in_rel[i] = hrt[3 * by_t[i] + 1];
    th[i] = hrt[3 * i];
    tr[i] = hrt[3 * i + 1];
    tt[i] = hrt[3 * i + 2];
  }
  rnnl_miner_s *mm = new rnnl_miner_s;
  auto up = [&](const std::vector<int32_t> &v, const int32_t *&dst) -> int {
    void *p = nullptr;
    const size_t bytes = std::max<size_t>(4, v.size() * 4);
    if (hipMalloc(&p, bytes) != hipSuccess) return RNNL_ERR_NOMEM;
    mm->bufs.push_back(p);
    if (!v.empty() && hipMemcpy(p, v.data(), v.size() * 4, hipMemcpyHostToDevice) != hipSuccess) return RNNL_ERR_HIP;
    dst = static_cast<const int32_t *>(p);
    return RNNL_OK;
  };
  mm->d.E = E;
  mm->d.R = R;
  mm->d.n = (int32_t)n;
  int rc = RNNL_OK;
  for (auto pr : {std::make_pair(&out_off, &mm->d.out_off), std::make_pair(&out_dst, &mm->d.out_dst),
                  std::make_pair(&out_rel, &mm->d.out_rel), std::make_pair(&in_off, &mm->d.in_off),
                  std::make_pair(&in_src, &mm->d.in_src), std::make_pair(&in_rel, &mm->d.in_rel),
                  std::make_pair(&th, &mm->d.th), std::make_pair(&tr, &mm->d.tr), std::make_pair(&tt, &mm->d.tt)})
    if (rc == RNNL_OK) rc = up(*pr.first, *pr.second);
  if (rc != RNNL_OK) {
    for (void *p : mm->bufs) (void)hipFree(p);
    delete mm;
    set_error("rnnl_miner_create: device allocation/copy failed");
    return rc;
  }
  *out = mm;
  return RNNL_OK;
}

int rnnl_miner_destroy(rnnl_miner m) {
  if (!m) return RNNL_OK;
  for (void *p : m->bufs) (void)hipFree(p);
  delete m;
  return RNNL_OK;
}

int rnnl_rule_search(rnnl_miner m, int32_t max_length, uint64_t *table, int64_t table_cap, uint64_t *rules_out,
                     int64_t out_cap, uint64_t *counters, void *stream) {
  if (!m || max_length < 1 || max_length > 3 || !table || table_cap < 1024 || (table_cap & (table_cap - 1)) ||
      !rules_out || out_cap < 0 || !counters) {
    set_error("rnnl_rule_search: bad arguments (max_length 1..3, table_cap a power of two >= 1024)");
    return RNNL_ERR_INVALID;
  }
  hipStream_t st = (hipStream_t)stream;
  RNNL_HIP_CHECK(hipMemsetAsync(table, 0xff, (size_t)table_cap * 8, st));
  RNNL_HIP_CHECK(hipMemsetAsync(counters, 0, 4 * 8, st));
  unsigned long long *flags = reinterpret_cast<unsigned long long *>(counters);
  if (m->d.n > 0) {
    const unsigned grid = (unsigned)std::min<int64_t>(m->d.n, 256 * 4);
    hipLaunchKernelGGL(mine_kernel, dim3(grid), dim3(MB), 0, st, m->d, (int)max_length,
                       reinterpret_cast<unsigned long long *>(table), table_cap, flags);
  }
  hipLaunchKernelGGL(compact_kernel, dim3(1024), dim3(256), 0, st, reinterpret_cast<const unsigned long long *>(table),
                     table_cap, reinterpret_cast<unsigned long long *>(rules_out), out_cap, flags);
  RNNL_HIP_CHECK(hipGetLastError());
  return RNNL_OK;
}

}  // extern "C"
