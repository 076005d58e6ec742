// Internal structures shared by the host builders (graph.cpp) and the HIP
// kernels.  Not part of the C-ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/rnnlogic_hip.h"

namespace rnnl {

// Vertex-major CSR of the train graph: edges (v --rel--> t) for fixed (v, rel)
// are col[off[v*R+rel] .. off[v*R+rel+1]), in train-file order.
struct GraphDev {
  int32_t E = 0, R = 0;
  int64_t n_edges = 0;
  const int32_t *off = nullptr;        // E*R + 1
  const int32_t *col = nullptr;        // n_edges
  // compact per-vertex view of off (L2-sized): for vertex v and relation word
  // w = rel >> 5, vbits[v * W + w] = (bitmap of v's relations with edges in
  // that word, index into dvoff of the word's first present relation); the
  // edges of (v, rel) are col[dvoff[pos] .. dvoff[pos + 1]) with
  // pos = .y + popcount(.x below rel's bit)
  int32_t W = 0;
  const uint2 *vbits = nullptr;        // E * W
  const int32_t *dvoff = nullptr;      // sum over v of (present relations + 1)
  const int32_t *edge_base = nullptr;  // R + 1: start of relation r's edge table
  const int32_t *edge_src = nullptr;   // relation-major, relation-local file order
  const int32_t *edge_dst = nullptr;
};

// Rule miner graph (mine.hip): out-edges grouped by source, in-edges grouped
// by target with sources ascending, and the train triples themselves.
struct MinerDev {
  int32_t E = 0, R = 0, n = 0;
  const int32_t *out_off = nullptr, *out_dst = nullptr, *out_rel = nullptr;  // E + 1, n, n
  const int32_t *in_off = nullptr, *in_src = nullptr, *in_rel = nullptr;     // E + 1, n, n
  const int32_t *th = nullptr, *tr = nullptr, *tt = nullptr;                 // n
};

// Rule bodies as one prefix trie per head relation.  Node ids are global;
// the nodes of one head are contiguous, numbered breadth-first, so the
// children of a node are contiguous too.  Node 0 of a head is its root
// (empty prefix, relation -1).
struct RulesDev {
  int32_t n_rules = 0, n_nodes = 0, max_depth = 0, n_heads = 0;
  const int32_t *head_root = nullptr;   // R: root node id, -1 if the head has no rule
  const int32_t *head_depth = nullptr;  // R: deepest body length of the head
  const int32_t *head_nodes = nullptr;  // R: number of trie nodes of the head
  const int32_t *node_rel = nullptr;    // relation of the edge into the node
  const int32_t *node_child = nullptr;  // first child id
  const int32_t *node_nchild = nullptr;
  const int32_t *node_nrules = nullptr;    // rules whose body ends exactly here
  const int32_t *node_rule_ptr = nullptr;  // n_nodes + 1
  const int32_t *node_rules = nullptr;     // member rule ids, ascending
  const uint64_t *node_fp = nullptr;       // sum of mix64(rule id) of members (digest only)
  // leaves (nodes where >= 1 rule ends), numbered per head for LDS staging
  int32_t max_leaves = 0, max_head_nodes = 0;
  const int32_t *head_leaf_ptr = nullptr;   // R + 1
  const int32_t *head_leaf_node = nullptr;  // leaf node ids, head-major, ascending node id
  const int32_t *node_leaf = nullptr;       // n_nodes: local leaf index within its head, -1 if none
  // the grounding walk's per-node fields in one 16-B load: (rel, first child, nchild, nrules)
  const int4 *node_info = nullptr;
  // the rule encoder over the trie (rnnl_lstm_encode_trie): per node its
  // parent (-1 at a root) and LSTM input token (the head relation at a root,
  // else node_rel); the nodes grouped by depth (level_nodes, host level_ptr)
  const int32_t *node_parent = nullptr;
  const int32_t *node_tok = nullptr;
  const int32_t *level_nodes = nullptr;
};

// Node-weight records (bytes per node); see rnnl_node_weights.
constexpr int kHidden = 16;
constexpr int kStrideSum = 64;   // f32 sum x[16]
constexpr int kStridePna = 256;  // int32 fix(sum x)[16] | int32 fix(sum x^2)[16] | f32 min[16] | f32 max[16]
                                 // (one shift per table and column: trailer[1], trailer[4])

void set_error(const std::string &msg);

// The SUM node records' fixed-point pass (node_fix_kernel, ground.hip) over
// every node of the table (rnnl_lstm_encode_trie_sum's last launch).
int node_fix_enqueue(rnnl_rules r, void *node_w, void *stream);

}  // namespace rnnl

struct rnnl_graph_s {
  rnnl::GraphDev d;
  int device = 0;
  void *mem[7] = {};
};

struct rnnl_rules_s {
  rnnl::RulesDev d;
  int device = 0;
  int32_t R = 0, E = 0;
  void *mem[20] = {};
  std::vector<int32_t> node_of_rule;  // host: trie node where each rule's body ends
  std::vector<int32_t> level_ptr;     // host: max_depth + 2 offsets into d.level_nodes
  std::vector<int32_t> head_root;     // host copy of d.head_root (R)
  std::vector<int32_t> head_nodes;    // host copy of d.head_nodes (R)
};

#define RNNL_HIP_CHECK(expr)                                                              \
  do {                                                                                    \
    hipError_t _e = (expr);                                                               \
    if (_e != hipSuccess) {                                                               \
      rnnl::set_error(std::string(#expr) + ": " + hipGetErrorString(_e));                 \
      return RNNL_ERR_HIP;                                                                \
    }                                                                                     \
  } while (0)
