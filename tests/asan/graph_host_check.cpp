// Host-side sanitizer check of the graph / rule-trie builders
// (rnnlogic_amd/csrc/graph.cpp: rnnl_graph_create, rnnl_rules_create).
//
// Built with g++ -fsanitize=address,undefined together with graph.cpp by
// tests/test_host_sanitizers.py (CPU, no GPU).  The few HIP runtime calls the
// builders make are replaced below by host stand-ins: hipMalloc is malloc,
// hipMemcpy is memcpy, so the "device" arrays are host memory this program
// reads back and checks against a naive restatement of the reference
// adjacency (ref src/data.py:39-106: per relation, edges in train-file order)
// and rule lists (ref src/predictors.py:165-199).  A countdown makes the k-th
// allocation fail, so every error path's cleanup runs under ASan / LSan.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "../../rnnlogic_amd/csrc/internal.h"

// ---------------------------------------------------------------- HIP stand-ins
static int g_fail_after = -1;  // fail the allocation when this reaches 0 (-1: never)
static long g_live = 0;        // allocations not yet freed

extern "C" {
hipError_t hipMalloc(void **p, size_t n) {
  if (g_fail_after == 0) {
    g_fail_after = -1;
    *p = nullptr;
    return hipErrorOutOfMemory;
  }
  if (g_fail_after > 0) --g_fail_after;
  *p = malloc(n);
  if (!*p) return hipErrorOutOfMemory;
  ++g_live;
  return hipSuccess;
}
hipError_t hipFree(void *p) {
  if (p) --g_live;
  free(p);
  return hipSuccess;
}
hipError_t hipMemcpy(void *d, const void *s, size_t n, hipMemcpyKind) {
  memcpy(d, s, n);
  return hipSuccess;
}
hipError_t hipGetDevice(int *d) {
  *d = 0;
  return hipSuccess;
}
const char *hipGetErrorString(hipError_t) { return "stub error"; }
}

// ---------------------------------------------------------------- checks
static int g_checks = 0;
#define CHECK(c)                                                             \
  do {                                                                       \
    ++g_checks;                                                              \
    if (!(c)) {                                                              \
      fprintf(stderr, "%s:%d: check failed: %s\n", __FILE__, __LINE__, #c); \
      exit(1);                                                               \
    }                                                                        \
  } while (0)

static void check_graph(rnnl_graph g, const std::vector<int32_t> &hrt, int E, int R) {
  const int64_t n = (int64_t)hrt.size() / 3;
  const rnnl::GraphDev &d = g->d;
  CHECK(d.E == E && d.R == R && d.n_edges == n && d.W == (R + 31) / 32);
  // per (h, r): targets in file order
  for (int v = 0; v < E; ++v)
    for (int r = 0; r < R; ++r) {
      std::vector<int32_t> want;
      for (int64_t i = 0; i < n; ++i)
        if (hrt[3 * i] == v && hrt[3 * i + 1] == r) want.push_back(hrt[3 * i + 2]);
      const int64_t o = (int64_t)v * R + r;
      CHECK(d.off[o + 1] - d.off[o] == (int32_t)want.size());
      for (size_t k = 0; k < want.size(); ++k) CHECK(d.col[d.off[o] + k] == want[k]);
      // the compact view gives the same range
      const uint2 p = d.vbits[(size_t)v * d.W + (r >> 5)];
      const bool present = (p.x >> (r & 31)) & 1u;
      CHECK(present == !want.empty());
      if (present) {
        const uint32_t below = p.x & ((1u << (r & 31)) - 1u);
        const int pos = (int)p.y + __builtin_popcount(below);
        CHECK(d.dvoff[pos] == d.off[o] && d.dvoff[pos + 1] == d.off[o + 1]);
      }
    }
  // relation-local edge ids in file order (relation2ht2index, data.py:66-69)
  for (int r = 0; r < R; ++r) {
    int32_t e = d.edge_base[r];
    for (int64_t i = 0; i < n; ++i)
      if (hrt[3 * i + 1] == r) {
        CHECK(d.edge_src[e] == hrt[3 * i] && d.edge_dst[e] == hrt[3 * i + 2]);
        ++e;
      }
    CHECK(e == d.edge_base[r + 1]);
  }
}

static void check_rules(rnnl_rules rs, const std::vector<int32_t> &tok, const std::vector<int64_t> &ptr, int R) {
  const rnnl::RulesDev &d = rs->d;
  const int n_rules = (int)ptr.size() - 1;
  CHECK(d.n_rules == n_rules);
  std::vector<int> seen(n_rules, 0);
  for (int i = 0; i < n_rules; ++i) {
    const int head = tok[ptr[i]];
    int node = d.head_root[head];
    CHECK(node >= 0);
    for (int64_t k = ptr[i] + 1; k < ptr[i + 1]; ++k) {  // walk the body down the trie
      const int4 info = d.node_info[node];
      int next = -1;
      for (int c = info.y; c < info.y + info.z; ++c)
        if (d.node_rel[c] == tok[k]) next = c;
      CHECK(next >= 0);
      node = next;
    }
    CHECK(rs->node_of_rule[i] == node);
    bool member = false;
    for (int j = d.node_rule_ptr[node]; j < d.node_rule_ptr[node + 1]; ++j) member |= d.node_rules[j] == i;
    CHECK(member);
    seen[i]++;
  }
  int leaves = 0;
  for (int r = 0; r < R; ++r) {
    const int root = d.head_root[r];
    if (root < 0) {
      CHECK(d.head_leaf_ptr[r + 1] == d.head_leaf_ptr[r]);
      continue;
    }
    CHECK(d.node_rel[root] == -1);
    for (int nd = root; nd < root + d.head_nodes[r]; ++nd) {
      const int4 info = d.node_info[nd];
      CHECK(info.x == d.node_rel[nd] && info.y == d.node_child[nd] && info.z == d.node_nchild[nd] &&
            info.w == d.node_nrules[nd]);
      for (int c = info.y + 1; c < info.y + info.z; ++c) CHECK(d.node_rel[c] > d.node_rel[c - 1]);
      for (int j = d.node_rule_ptr[nd] + 1; j < d.node_rule_ptr[nd + 1]; ++j)
        CHECK(d.node_rules[j] > d.node_rules[j - 1]);  // members ascending (file order)
      if (info.w > 0) {
        CHECK(d.node_leaf[nd] >= 0 && d.head_leaf_node[d.head_leaf_ptr[r] + d.node_leaf[nd]] == nd);
        ++leaves;
      } else {
        CHECK(d.node_leaf[nd] == -1);
      }
    }
  }
  CHECK(leaves == d.head_leaf_ptr[R]);
}

int main() {
  std::mt19937 rng(7);
  auto U = [&](int lo, int hi) { return std::uniform_int_distribution<int>(lo, hi)(rng); };
  int graphs = 0, rulesets = 0, injected = 0;
  for (int it = 0; it < 60; ++it) {
    const int E = U(1, 40), R = U(1, 70), n = U(0, 300);
    std::vector<int32_t> hrt;
    for (int i = 0; i < n; ++i) {
      hrt.push_back(U(0, E - 1));
      hrt.push_back(U(0, R - 1));
      hrt.push_back(U(0, E - 1));
    }
    rnnl_graph g = nullptr;
    CHECK(rnnl_graph_create(hrt.empty() ? nullptr : hrt.data(), n, E, R, &g) == RNNL_OK);
    check_graph(g, hrt, E, R);
    ++graphs;
    // random rules: bodies of length 0..4 (duplicates allowed: they share a node)
    std::vector<int32_t> tok;
    std::vector<int64_t> ptr(1, 0);
    const int nr = U(0, 200);
    for (int i = 0; i < nr; ++i) {
      tok.push_back(U(0, R - 1));
      const int L = U(0, 4);
      for (int k = 0; k < L; ++k) tok.push_back(U(0, std::min(R - 1, 5)));
      ptr.push_back((int64_t)tok.size());
    }
    rnnl_rules rs = nullptr;
    CHECK(rnnl_rules_create(g, tok.data(), ptr.data(), nr, &rs) == RNNL_OK);
    check_rules(rs, tok, ptr, R);
    ++rulesets;
    std::vector<int32_t> n2r(std::max(nr, 1));
    CHECK(rnnl_rules_node_of_rule(rs, n2r.data()) == RNNL_OK);
    CHECK(rnnl_rules_destroy(rs) == RNNL_OK);
    // every allocation of the rule tables failing in turn: error, no leak
    for (int k = 0; k < 14; ++k) {
      const long live = g_live;
      g_fail_after = k;
      rnnl_rules bad = nullptr;
      CHECK(rnnl_rules_create(g, tok.data(), ptr.data(), nr, &bad) == RNNL_ERR_HIP && bad == nullptr);
      CHECK(g_live == live);
      ++injected;
    }
    g_fail_after = -1;
    // invalid rules: out-of-range head / body, empty rule
    if (nr > 0) {
      std::vector<int32_t> t2 = tok;
      t2[0] = R;
      rnnl_rules bad = nullptr;
      CHECK(rnnl_rules_create(g, t2.data(), ptr.data(), nr, &bad) == RNNL_ERR_INVALID);
      std::vector<int64_t> p2 = ptr;
      p2[1] = p2[0];
      CHECK(rnnl_rules_create(g, tok.data(), p2.data(), 1, &bad) == RNNL_ERR_INVALID);
    }
    CHECK(rnnl_graph_destroy(g) == RNNL_OK);
    // every allocation of the graph failing in turn
    for (int k = 0; k < 7; ++k) {
      const long live = g_live;
      g_fail_after = k;
      rnnl_graph bad = nullptr;
      CHECK(rnnl_graph_create(hrt.empty() ? nullptr : hrt.data(), n, E, R, &bad) == RNNL_ERR_HIP);
      CHECK(g_live == live);
      ++injected;
    }
    g_fail_after = -1;
    if (n > 0) {  // out-of-range triple
      std::vector<int32_t> h2 = hrt;
      h2[3 * (n - 1) + 2] = E;
      rnnl_graph bad = nullptr;
      CHECK(rnnl_graph_create(h2.data(), n, E, R, &bad) == RNNL_ERR_INVALID);
    }
  }
  rnnl_graph bad = nullptr;
  CHECK(rnnl_graph_create(nullptr, 1, 3, 3, &bad) == RNNL_ERR_INVALID);
  CHECK(rnnl_graph_create(nullptr, 0, 0, 3, &bad) == RNNL_ERR_INVALID);
  CHECK(rnnl_rules_create(nullptr, nullptr, nullptr, 0, nullptr) == RNNL_ERR_INVALID);
  CHECK(g_live == 0);
  printf("graph_host_check: %d graphs, %d rule sets, %d injected allocation failures, %d checks, 0 live blocks\n",
         graphs, rulesets, injected, g_checks);
  return 0;
}
