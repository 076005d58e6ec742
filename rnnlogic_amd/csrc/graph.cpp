// Host-side builders for the device-resident knowledge graph and rule tries.
//
//   rnnl_graph_create  <- KnowledgeGraph.__init__ adjacency (ref src/data.py:39-106)
//   rnnl_rules_create  <- PredictorPlus.set_rules           (ref src/predictors.py:165-199)
//
// Both run once per process / rule set, upload immutable arrays and return a
// handle; nothing here is on the timed path.
#include <algorithm>
#include <map>
#include <vector>

#include "internal.h"

namespace rnnl {

static thread_local std::string g_err;
void set_error(const std::string &msg) { g_err = msg; }

static inline uint64_t mix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ULL;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
  return x ^ (x >> 31);
}

template <typename T>
static int upload(const std::vector<T> &h, void **slot, const T **dst) {
  size_t bytes = std::max<size_t>(h.size(), 1) * sizeof(T);
  RNNL_HIP_CHECK(hipMalloc(slot, bytes));
  if (!h.empty()) RNNL_HIP_CHECK(hipMemcpy(*slot, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
  *dst = static_cast<const T *>(*slot);
  return RNNL_OK;
}

}  // namespace rnnl

using namespace rnnl;

extern "C" {

const char *rnnl_last_error(void) { return g_err.c_str(); }
int rnnl_version(void) { return 1; }

int rnnl_graph_create(const int32_t *hrt, int64_t n, int32_t E, int32_t R, rnnl_graph *out) {
  if (!out || E <= 0 || R <= 0 || n < 0 || (n > 0 && !hrt)) {
    set_error("rnnl_graph_create: bad arguments");
    return RNNL_ERR_INVALID;
  }
  if ((int64_t)E * R + 1 > (int64_t)INT32_MAX * 64 || n >= INT32_MAX) {
    set_error("rnnl_graph_create: graph too large for 32-bit offsets");
    return RNNL_ERR_INVALID;
  }
  const int64_t ER = (int64_t)E * R;
  std::vector<int32_t> off(ER + 1, 0), col(n), ebase(R + 1, 0), esrc(n), edst(n);
  for (int64_t i = 0; i < n; ++i) {
    const int32_t h = hrt[3 * i], r = hrt[3 * i + 1], t = hrt[3 * i + 2];
    if (h < 0 || h >= E || t < 0 || t >= E || r < 0 || r >= R) {
      set_error("rnnl_graph_create: triple id out of range");
      return RNNL_ERR_INVALID;
    }
    off[(int64_t)h * R + r + 1]++;
    ebase[r + 1]++;
  }
  for (int64_t i = 0; i < ER; ++i) off[i + 1] += off[i];
  for (int r = 0; r < R; ++r) ebase[r + 1] += ebase[r];
  std::vector<int32_t> fill(off.begin(), off.end() - 1), efill(ebase.begin(), ebase.end() - 1);
  for (int64_t i = 0; i < n; ++i) {
    const int32_t h = hrt[3 * i], r = hrt[3 * i + 1], t = hrt[3 * i + 2];
    col[fill[(int64_t)h * R + r]++] = t;  // train-file order inside (h, r)
    const int32_t e = efill[r]++;         // relation-local id == reference edge id
    esrc[e] = h;
    edst[e] = t;
  }
  // compact per-vertex relation bitmaps + dense offsets (see GraphDev)
  const int W = (R + 31) / 32;
  std::vector<uint2> vbits((size_t)E * W);
  std::vector<int32_t> dvoff;
  dvoff.reserve((size_t)E + (size_t)n + 1);
  for (int64_t v = 0; v < E; ++v) {
    for (int w = 0; w < W; ++w) {
      uint32_t bits = 0;
      const uint32_t first = (uint32_t)dvoff.size();
      for (int b = 0; b < 32; ++b) {
        const int64_t r = (int64_t)w * 32 + b;
        if (r >= R) break;
        const int64_t o = v * R + r;
        if (off[o + 1] > off[o]) {
          bits |= 1u << b;
          dvoff.push_back(off[o]);
        }
      }
      vbits[(size_t)v * W + w] = make_uint2(bits, first);
    }
    dvoff.push_back(off[(v + 1) * R]);  // end of v's edges: the last present relation's end
  }
  auto *g = new rnnl_graph_s;
  (void)hipGetDevice(&g->device);
  g->d.E = E;
  g->d.R = R;
  g->d.W = W;
  g->d.n_edges = n;
  int rc = RNNL_OK;
  if ((rc = upload(off, &g->mem[0], &g->d.off)) || (rc = upload(col, &g->mem[1], &g->d.col)) ||
      (rc = upload(ebase, &g->mem[2], &g->d.edge_base)) || (rc = upload(esrc, &g->mem[3], &g->d.edge_src)) ||
      (rc = upload(edst, &g->mem[4], &g->d.edge_dst)) || (rc = upload(vbits, &g->mem[5], &g->d.vbits)) ||
      (rc = upload(dvoff, &g->mem[6], &g->d.dvoff))) {
    rnnl_graph_destroy(g);
    return rc;
  }
  *out = g;
  return RNNL_OK;
}

int rnnl_graph_destroy(rnnl_graph g) {
  if (!g) return RNNL_OK;
  for (void *p : g->mem)
    if (p) (void)hipFree(p);
  delete g;
  return RNNL_OK;
}

int rnnl_graph_info(rnnl_graph g, int32_t *info) {
  if (!g || !info) return RNNL_ERR_INVALID;
  info[0] = g->d.E;
  info[1] = g->d.R;
  info[2] = (int32_t)(g->d.n_edges & 0x7fffffff);
  info[3] = (int32_t)(g->d.n_edges >> 31);
  return RNNL_OK;
}

int rnnl_rules_create(rnnl_graph g, const int32_t *tok, const int64_t *ptr, int32_t n_rules, rnnl_rules *out) {
  if (!g || !out || n_rules < 0 || (n_rules > 0 && (!tok || !ptr))) {
    set_error("rnnl_rules_create: bad arguments");
    return RNNL_ERR_INVALID;
  }
  const int R = g->d.R;
  // per head: trie with nodes keyed by (parent, relation); rules in file order
  struct TNode {
    int parent, rel, depth;
    std::vector<int> rules;
    std::map<int, int> child;  // relation -> local node (ordered: deterministic BFS)
  };
  std::vector<std::vector<TNode>> tries(R);
  for (int32_t i = 0; i < n_rules; ++i) {
    const int64_t b = ptr[i], e = ptr[i + 1];
    if (e <= b) {
      set_error("rnnl_rules_create: empty rule");
      return RNNL_ERR_INVALID;
    }
    const int head = tok[b];
    if (head < 0 || head >= R) {
      set_error("rnnl_rules_create: head relation out of range");
      return RNNL_ERR_INVALID;
    }
    auto &t = tries[head];
    if (t.empty()) t.push_back(TNode{-1, -1, 0, {}, {}});
    int cur = 0;
    for (int64_t k = b + 1; k < e; ++k) {
      const int rel = tok[k];
      if (rel < 0 || rel >= R) {
        set_error("rnnl_rules_create: body relation out of range");
        return RNNL_ERR_INVALID;
      }
      auto it = t[cur].child.find(rel);
      if (it == t[cur].child.end()) {
        const int id = (int)t.size();
        const int depth = t[cur].depth + 1;
        t.push_back(TNode{cur, rel, depth, {}, {}});
        t[cur].child[rel] = id;
        cur = id;
      } else {
        cur = it->second;
      }
    }
    t[cur].rules.push_back(i);
  }
  // breadth-first renumbering, heads in relation order
  std::vector<int32_t> head_root(R, -1), head_depth(R, 0), head_nodes(R, 0);
  std::vector<int32_t> node_rel, node_child, node_nchild, node_nrules, node_rule_ptr(1, 0), node_rules;
  std::vector<uint64_t> node_fp;
  std::vector<int32_t> node_of_rule(n_rules, -1);
  std::vector<int32_t> node_parent, node_tok, node_depth;
  int max_depth = 0;
  for (int r = 0; r < R; ++r) {
    auto &t = tries[r];
    if (t.empty()) continue;
    const int base = (int)node_rel.size();
    std::vector<int> order;  // local ids in BFS order
    std::vector<int> newid(t.size(), -1);
    order.push_back(0);
    for (size_t q = 0; q < order.size(); ++q)
      for (auto &kv : t[order[q]].child) order.push_back(kv.second);
    for (size_t q = 0; q < order.size(); ++q) newid[order[q]] = base + (int)q;
    head_root[r] = base;
    head_nodes[r] = (int)order.size();
    for (int loc : order) {
      const TNode &nd = t[loc];
      node_rel.push_back(nd.rel);
      node_parent.push_back(nd.parent >= 0 ? newid[nd.parent] : -1);
      node_tok.push_back(nd.parent >= 0 ? nd.rel : r);
      node_depth.push_back(nd.depth);
      node_child.push_back(nd.child.empty() ? 0 : newid[nd.child.begin()->second]);
      node_nchild.push_back((int)nd.child.size());
      node_nrules.push_back((int)nd.rules.size());
      uint64_t fp = 0;
      for (int rid : nd.rules) {
        node_rules.push_back(rid);
        node_of_rule[rid] = newid[loc];
        fp += mix64((uint64_t)rid);
      }
      node_fp.push_back(fp);
      node_rule_ptr.push_back((int32_t)node_rules.size());
      head_depth[r] = std::max(head_depth[r], nd.depth);
    }
    max_depth = std::max(max_depth, head_depth[r]);
    // children of a node must be contiguous in the new numbering (BFS gives it)
    for (int loc : order) {
      int prev = -1;
      for (auto &kv : t[loc].child) {
        const int id = newid[kv.second];
        if (prev >= 0 && id != prev + 1) {
          set_error("rnnl_rules_create: internal BFS numbering error");
          return RNNL_ERR_INVALID;
        }
        prev = id;
      }
    }
    if ((int64_t)head_nodes[r] * g->d.E >= INT32_MAX) {
      set_error("rnnl_rules_create: trie too large for 32-bit (node, entity) keys");
      return RNNL_ERR_INVALID;
    }
  }
  // the scoring kernels address node records with 32-bit byte offsets
  if ((int64_t)node_rel.size() * kStridePna >= ((int64_t)1 << 32)) {
    set_error("rnnl_rules_create: more trie nodes than 32-bit record offsets address");
    return RNNL_ERR_INVALID;
  }
  // leaves per head (nodes where rules end), in node-id order
  const int n_nodes_total = (int)node_rel.size();
  std::vector<int32_t> head_leaf_ptr(R + 1, 0), head_leaf_node, node_leaf(n_nodes_total, -1);
  int max_leaves = 0, max_head_nodes = 0;
  for (int r = 0; r < R; ++r) {
    head_leaf_ptr[r] = (int32_t)head_leaf_node.size();
    if (head_root[r] >= 0) {
      int nl = 0;
      for (int n = head_root[r]; n < head_root[r] + head_nodes[r]; ++n)
        if (node_nrules[n] > 0) {
          node_leaf[n] = nl++;
          head_leaf_node.push_back(n);
        }
      max_leaves = std::max(max_leaves, nl);
      max_head_nodes = std::max(max_head_nodes, head_nodes[r]);
    }
  }
  head_leaf_ptr[R] = (int32_t)head_leaf_node.size();
  // nodes by depth (ascending id within a depth): the encoder's levels
  std::vector<int32_t> level_ptr(max_depth + 2, 0), level_nodes(n_nodes_total);
  for (int n = 0; n < n_nodes_total; ++n) ++level_ptr[node_depth[n] + 1];
  for (int d = 0; d <= max_depth; ++d) level_ptr[d + 1] += level_ptr[d];
  {
    std::vector<int32_t> fill(level_ptr.begin(), level_ptr.end() - 1);
    for (int n = 0; n < n_nodes_total; ++n) level_nodes[fill[node_depth[n]]++] = n;
  }
  auto *rs = new rnnl_rules_s;
  (void)hipGetDevice(&rs->device);
  rs->R = R;
  rs->E = g->d.E;
  rs->d.n_rules = n_rules;
  rs->d.n_nodes = (int32_t)node_rel.size();
  rs->d.max_depth = max_depth;
  rs->d.n_heads = R;
  rs->node_of_rule = std::move(node_of_rule);
  rs->head_root = head_root;
  rs->head_nodes = head_nodes;
  rs->level_ptr = level_ptr;
  rs->d.max_leaves = max_leaves;
  rs->d.max_head_nodes = max_head_nodes;
  std::vector<int32_t> node_info(4 * node_rel.size());
  for (size_t n = 0; n < node_rel.size(); ++n) {
    node_info[4 * n] = node_rel[n];
    node_info[4 * n + 1] = node_child[n];
    node_info[4 * n + 2] = node_nchild[n];
    node_info[4 * n + 3] = node_nrules[n];
  }
  const int32_t *node_info_dev = nullptr;
  int rc = RNNL_OK;
  if ((rc = upload(head_root, &rs->mem[0], &rs->d.head_root)) ||
      (rc = upload(head_depth, &rs->mem[1], &rs->d.head_depth)) ||
      (rc = upload(head_nodes, &rs->mem[2], &rs->d.head_nodes)) ||
      (rc = upload(node_rel, &rs->mem[3], &rs->d.node_rel)) ||
      (rc = upload(node_child, &rs->mem[4], &rs->d.node_child)) ||
      (rc = upload(node_nchild, &rs->mem[5], &rs->d.node_nchild)) ||
      (rc = upload(node_nrules, &rs->mem[6], &rs->d.node_nrules)) ||
      (rc = upload(node_rule_ptr, &rs->mem[7], &rs->d.node_rule_ptr)) ||
      (rc = upload(node_rules, &rs->mem[8], &rs->d.node_rules)) ||
      (rc = upload(node_fp, &rs->mem[9], &rs->d.node_fp)) ||
      (rc = upload(head_leaf_ptr, &rs->mem[10], &rs->d.head_leaf_ptr)) ||
      (rc = upload(head_leaf_node, &rs->mem[11], &rs->d.head_leaf_node)) ||
      (rc = upload(node_leaf, &rs->mem[12], &rs->d.node_leaf)) ||
      (rc = upload(node_info, &rs->mem[13], &node_info_dev)) ||
      (rc = upload(node_parent, &rs->mem[14], &rs->d.node_parent)) ||
      (rc = upload(node_tok, &rs->mem[15], &rs->d.node_tok)) ||
      (rc = upload(level_nodes, &rs->mem[16], &rs->d.level_nodes))) {
    rnnl_rules_destroy(rs);
    return rc;
  }
  rs->d.node_info = reinterpret_cast<const int4 *>(node_info_dev);
  *out = rs;
  return RNNL_OK;
}

int rnnl_rules_destroy(rnnl_rules r) {
  if (!r) return RNNL_OK;
  for (void *p : r->mem)
    if (p) (void)hipFree(p);
  delete r;
  return RNNL_OK;
}

int rnnl_rules_node_of_rule(rnnl_rules r, int32_t *node_of_rule) {
  if (!r || !node_of_rule) {
    set_error("rnnl_rules_node_of_rule: bad arguments");
    return RNNL_ERR_INVALID;
  }
  std::copy(r->node_of_rule.begin(), r->node_of_rule.end(), node_of_rule);
  return RNNL_OK;
}

int rnnl_rules_head_roots(rnnl_rules r, int32_t *head_root, int32_t *max_head_nodes) {
  if (!r || !head_root || !max_head_nodes) {
    set_error("rnnl_rules_head_roots: bad arguments");
    return RNNL_ERR_INVALID;
  }
  std::copy(r->head_root.begin(), r->head_root.end(), head_root);
  *max_head_nodes = r->d.max_head_nodes;
  return RNNL_OK;
}

int rnnl_rules_info(rnnl_rules r, int32_t *info) {
  if (!r || !info) return RNNL_ERR_INVALID;
  info[0] = r->d.n_rules;
  info[1] = r->d.n_nodes;
  info[2] = r->d.max_depth;
  info[3] = kStrideSum;
  info[4] = kStridePna;
  return RNNL_OK;
}

}  // extern "C"
