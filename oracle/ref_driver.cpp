// TEST INFRASTRUCTURE ONLY — never linked into the product.
//
// Thin C-ABI shim over the *reference* C++ miner, compiled from the reference
// sources where they lie (/root/reference/miner/rnnlogic.cpp) by oracle/Makefile
// into oracle/_ref/libref_miner.so.  It exposes exactly three things:
//
//   * ref_rule_destination — KnowledgeGraph::rule_destination
//     (reference miner/rnnlogic.cpp:412-442): per-(query, rule) path counts with
//     the query triple removed at every hop.  Used by tests/ to pin the oracle.
//   * ref_out_test_timed — ReasoningPredictor::out_test (rnnlogic.cpp:1262-1406):
//     the miner's multi-threaded grounding over (a prefix of) the test split.
//     Used only by bench.py's cpu_baseline leg (kind "reference").
//   * ref_rule_search — RuleMiner::search (rnnlogic.cpp:505-589): the rule
//     pool the GPU miner (rnnl_rule_search) must reproduce; tests/ only.
//
// Nothing here re-implements the algorithm; it only marshals plain arrays into
// the reference's own classes.
#include "rnnlogic.h"

#include <chrono>
#include <cstdio>
#include <vector>

namespace {

// Derived classes only to reach the reference's protected members for the
// bounded timing sample; no behaviour is overridden.
struct KG : public KnowledgeGraph {
  void truncate_test(int n) {
    if (n >= 0 && n < static_cast<int>(test_triplets.size())) {
      test_triplets.resize(n);
      test_triplet_size = n;
    }
  }
};

}  // namespace

extern "C" {

void *ref_kg_load(const char *data_path) {
  KG *kg = new KG;
  kg->read_data(const_cast<char *>(data_path));
  return kg;
}

void ref_kg_free(void *kg) { delete static_cast<KG *>(kg); }

int ref_kg_entity_size(void *kg) { return static_cast<KG *>(kg)->get_entity_size(); }
int ref_kg_relation_size(void *kg) { return static_cast<KG *>(kg)->get_relation_size(); }
int ref_kg_test_size(void *kg) { return static_cast<KG *>(kg)->get_test_size(); }

// Path counts of one rule body from entity e; (rm_h, rm_r, rm_t) is skipped at
// every hop (pass rm_r = -1 for "no removal").  Returns the number of
// destinations written (sorted by destination id, as std::map iterates), or
// -(needed) if cap is too small.
int ref_rule_destination(void *kg, int e, const int *body, int len, int rm_h, int rm_r, int rm_t,
                         int *out_dest, int *out_count, int cap) {
  Rule rule;
  rule.r_head = -1;
  rule.type = len;
  for (int i = 0; i < len; ++i) rule.r_body.push_back(body[i]);
  Triplet removed;
  removed.h = rm_h;
  removed.r = rm_r;
  removed.t = rm_t;
  std::map<int, int> dest2count;
  static_cast<KG *>(kg)->rule_destination(e, rule, &dest2count, removed);
  int n = static_cast<int>(dest2count.size());
  if (n > cap) return -n;
  int k = 0;
  for (auto &kv : dest2count) {
    out_dest[k] = kv.first;
    out_count[k] = kv.second;
    ++k;
  }
  return n;
}

// Times ReasoningPredictor::out_test over the first `sample` test triples with
// `threads` pthreads.  Rules are given as a flat (head, len, body...) stream.
// Returns wall seconds; *out_len receives the length of the produced data
// vector (a cheap checksum that the work was done).
double ref_out_test_timed(void *kgp, const int *rules_flat, int n_rules, int threads, int sample,
                          long long *out_len) {
  KG *kg = static_cast<KG *>(kgp);
  kg->truncate_test(sample);
  int R = kg->get_relation_size();
  std::vector<Rule> *rel2rules = new std::vector<Rule>[R];
  const int *p = rules_flat;
  for (int i = 0; i < n_rules; ++i) {
    Rule rule;
    rule.r_head = p[0];
    rule.type = p[1];
    for (int k = 0; k < p[1]; ++k) rule.r_body.push_back(p[2 + k]);
    rel2rules[rule.r_head].push_back(rule);
    p += 2 + rule.type;
  }
  ReasoningPredictor rp;
  rp.init_knowledge_graph(kg);
  rp.set_logic_rules(rel2rules);
  std::vector<int> data;
  auto t0 = std::chrono::steady_clock::now();
  rp.out_test(&data, true, threads);
  auto t1 = std::chrono::steady_clock::now();
  if (out_len) *out_len = static_cast<long long>(data.size());
  delete[] rel2rules;
  return std::chrono::duration<double>(t1 - t0).count();
}

// RuleMiner::search (reference miner/rnnlogic.cpp:505-589, rule_search at
// :350-382) over ALL train triples (portion 1) with `threads` pthreads.  The
// mined pool is written flat as (head, len, body...) in the reference's own
// order (per head relation, std::set<Rule> order).  Returns the number of ints
// written, or -(needed) if cap is too small; *seconds gets the search time.
long long ref_rule_search(void *kgp, int max_length, int threads, int *out_flat, long long cap, double *seconds) {
  KG *kg = static_cast<KG *>(kgp);
  RuleMiner rm;
  rm.init_knowledge_graph(kg);
  auto t0 = std::chrono::steady_clock::now();
  rm.search(max_length, 1.0, threads);
  auto t1 = std::chrono::steady_clock::now();
  if (seconds) *seconds = std::chrono::duration<double>(t1 - t0).count();
  std::vector<Rule> *rel2rules = rm.get_logic_rules();
  long long n = 0;
  for (int r = 0; r < kg->get_relation_size(); ++r)
    for (const Rule &rule : rel2rules[r]) n += 2 + rule.type;
  if (n > cap) return -n;
  long long k = 0;
  for (int r = 0; r < kg->get_relation_size(); ++r)
    for (const Rule &rule : rel2rules[r]) {
      out_flat[k++] = rule.r_head;
      out_flat[k++] = rule.type;
      for (int b : rule.r_body) out_flat[k++] = b;
    }
  return n;
}

}  // extern "C"
