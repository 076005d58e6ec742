/*
 * rnnlogic_hip.h — C-ABI of the MI355X (gfx950) reasoning-predictor hot path.
 *
 * Drop-in boundary for RNNLogic's PredictorPlus forward.  Every entry point
 * takes plain pointers and sizes (device pointers unless marked "host") and an
 * opaque hipStream_t passed as void*.  No torch types cross this line; the
 * Python side (rnnlogic_amd/, ctypes) mirrors the reference's
 * src/{data,predictors,layers,embedding}.py API on top of it.
 *
 * The reference has no FFI on this path: it runs PyTorch eager ops plus
 * torch_scatter.  Each function below names the reference code it replaces.
 *
 * Conventions
 *   - return value: RNNL_OK (0) or an RNNL_ERR_* code; rnnl_last_error()
 *     gives a thread-local message.
 *   - handles (rnnl_graph, rnnl_rules) are immutable after creation and may be
 *     used from several streams at once; one set per GPU / rank.
 *   - all launches are asynchronous on `stream` and capture-safe (no
 *     allocation or synchronisation inside), except the *_create calls, the
 *     status reads (rnnl_forward_status*: one header read-back and wait) and
 *     rnnl_predictorplus_forward_rotate (which ends with that read).
 */
#ifndef RNNLOGIC_HIP_H
#define RNNLOGIC_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RNNL_OK 0
#define RNNL_ERR_INVALID 1   /* bad argument / shape */
#define RNNL_ERR_HIP 2       /* HIP runtime error */
#define RNNL_ERR_OVERFLOW 3  /* workspace capacity exceeded: retry with a larger workspace */
#define RNNL_ERR_NOMEM 4
#define RNNL_ERR_INTERNAL 5  /* kernel self-check failed (message names the query) */
#define RNNL_ERR_RANGE 6     /* integer range: a path count / PNA degree reached 2^32, or the rule
                                aggregates are non-finite or too large for the fixed-point tables */

#define RNNL_AGG_SUM 0       /* FuncToNodeSum   (reference src/layers.py:53-77)  */
#define RNNL_AGG_PNA 1       /* FuncToNode, pna (reference src/layers.py:79-126) */

#define RNNL_FEATURE_ADD 0   /* score = base + mlp  (entity_feature bias / RotatE) */
#define RNNL_FEATURE_NONE 1  /* score = mlp at candidates, base elsewhere (-inf)  */

typedef struct rnnl_graph_s *rnnl_graph;
typedef struct rnnl_rules_s *rnnl_rules;
typedef struct rnnl_miner_s *rnnl_miner;

const char *rnnl_last_error(void);
int rnnl_version(void);

/* ---------------------------------------------------------------- graph --
 * Replaces KnowledgeGraph.__init__'s adjacency (reference src/data.py:39-106):
 * relation2adjacency / relation2ht2index.  Builds a vertex-major CSR
 * (edges of (head v, relation r) contiguous, train-file order inside) and the
 * per-relation edge tables used to resolve `edges_to_remove` ids
 * (relation-local, file order == data.py:68).  train_hrt is host (n_train x 3).
 */
int rnnl_graph_create(const int32_t *train_hrt, int64_t n_train, int32_t n_entities, int32_t n_relations,
                      rnnl_graph *out);
int rnnl_graph_destroy(rnnl_graph g);
/* host out: {n_entities, n_relations, n_edges_lo, n_edges_hi} */
int rnnl_graph_info(rnnl_graph g, int32_t *info4);

/* ---------------------------------------------------------------- rules --
 * Replaces PredictorPlus.set_rules (reference src/predictors.py:165-199).
 * rule_tokens/rule_ptr (host): rule i is tokens[ptr[i] .. ptr[i+1]) =
 * (head, body...).  Builds, per head relation, a prefix trie of the rule
 * bodies (shared prefixes are grounded once; the result is identical).
 */
int rnnl_rules_create(rnnl_graph g, const int32_t *rule_tokens, const int64_t *rule_ptr, int32_t n_rules,
                      rnnl_rules *out);
int rnnl_rules_destroy(rnnl_rules r);
/* host out: {n_rules, n_nodes, max_depth, node record bytes (sum), node record bytes (pna)} */
int rnnl_rules_info(rnnl_rules r, int32_t *info5);
/* host out (n_rules): the trie node where each rule's body ends — several
 * rules share a node when one body is a prefix-equal duplicate; node ids are
 * those of the grounding COO (rnnl_ground_export_entries). */
int rnnl_rules_node_of_rule(rnnl_rules r, int32_t *node_of_rule);
/* host out: head_root (R) = the trie root node of each head relation (-1:
 * no rule), *max_head_nodes = the largest trie (the row stride `ld` of
 * rnnl_predictor_rule_stats). */
int rnnl_rules_head_roots(rnnl_rules r, int32_t *head_root, int32_t *max_head_nodes);

/* Per-node aggregate of rule embeddings (device): rule_emb is n_rules x H
 * (row stride `ld` floats), H == 16.  Writes node_w: n_nodes records of
 * info5[3 + aggregator] bytes, then a trailer.
 *   SUM record: int32 fix_s(W . sum x)[16] — the members' embeddings summed
 *               in rule-id order (f32), times W = add_w (16 x 16 row-major,
 *               rule_to_entity.add_model.layers.0.weight, required for SUM;
 *               f32, inputs in ascending order), then one shift s for the
 *               whole table (|fix| < 2^30).  The Linear commutes with the
 *               candidate's sum of count x record (layers.py:70-74), so the
 *               scoring pass adds only its bias.
 *   PNA record: int32 fix(sum x)[16] | int32 fix(sum x^2)[16] | f32 min x[16] | f32 max x[16]
 *               (one shift per column; add_w unused, nullable)
 * The forward accumulates the fixed-point words exactly (fp64 below a total
 * count of 2^23, int64 past it), so a score does not depend on the order in
 * which the kernel meets a candidate's (node, count) entries.  Buffer size:
 * rnnl_node_weights_size.  Replaces the per-candidate sums of
 * FuncToNodeSum / FuncToNode (reference src/layers.py:53-126). */
int rnnl_node_weights(rnnl_rules r, const float *rule_emb, int32_t ld, int32_t aggregator, const float *add_w,
                      void *node_w, void *stream);
/* rnnl_node_weights for the trie of one head relation only (the records of
 * every other node are left unset; the table's fixed-point shift then covers
 * that head's nodes): a launch whose rows are all of relation `head` (a
 * training batch) reads no other record. */
int rnnl_node_weights_head(rnnl_rules r, int32_t head, const float *rule_emb, int32_t ld, int32_t aggregator,
                           const float *add_w, void *node_w, void *stream);
int rnnl_node_weights_size(rnnl_rules r, int32_t aggregator, size_t *bytes);

/* Rule encoder (reference src/predictors.py:201-208, type 'lstm'): for each
 * rule, the top-layer output of torch.nn.LSTM(16, 16, layers) at its last
 * non-pad token.  vocab: (R+1) x 16 (vocab_emb.weight); w_ih / w_hh:
 * layers x 64 x 16 and b_ih / b_hh: layers x 64 (rnn.weight_ih_l{k} ...,
 * torch gate order i, f, g, o); tokens: n_rules x seq_len int32 padded with
 * `pad`; out: n_rules rows of ld_out floats. */
int rnnl_lstm_encode(const float *vocab, const float *w_ih, const float *w_hh, const float *b_ih, const float *b_hh,
                     int32_t layers, int32_t hidden, const int32_t *tokens, int32_t n_rules, int32_t seq_len,
                     int32_t pad, float *out, int32_t ld_out, void *stream);

/* rnnl_lstm_encode over the rule trie of r (the rules given to
 * rnnl_rules_create, token order [head, body...]): one LSTM step per trie
 * node (prefixes shared by many rules are computed once), one launch per
 * depth.  out: the same n_rules x 16 rows as rnnl_lstm_encode of those
 * rules, bitwise.  The weights come as arrays of `layers` pointers (as for
 * rnnl_lstm_train_forward below: torch's per-layer parameters in place).
 * scratch: rnnl_lstm_encode_trie_scratch bytes (the per-node states). */
int rnnl_lstm_encode_trie_scratch(rnnl_rules r, int32_t layers, size_t *bytes);
int rnnl_lstm_encode_trie(rnnl_rules r, const float *vocab, const float *const *w_ih, const float *const *w_hh,
                          const float *const *b_ih, const float *const *b_hh, int32_t layers, int32_t hidden,
                          float *out, int32_t ld_out, void *scratch, size_t scratch_bytes, void *stream);
/* rnnl_lstm_encode_trie followed by rnnl_node_weights(r, out, ld_out,
 * RNNL_AGG_SUM, add_w, node_w) in the same launches: each trie node's SUM
 * record is formed where its embedding is (the rules ending at a node share
 * its top-layer h), with node_weights' arithmetic — node_w is bitwise that
 * call's table. */
int rnnl_lstm_encode_trie_sum(rnnl_rules r, const float *vocab, const float *const *w_ih, const float *const *w_hh,
                              const float *const *b_ih, const float *const *b_hh, int32_t layers, int32_t hidden,
                              float *out, int32_t ld_out, void *scratch, size_t scratch_bytes, const float *add_w,
                              void *node_w, void *stream);

/* The rule encoder under autograd (training; predictors.py:201-208 and
 * torch.nn.LSTM's backward): the rules ridx[0..n) (int64 rows of `tokens`).
 * Per-layer weights come as arrays of `layers` pointers (w_ih[l]: 64 x 16,
 * w_hh[l]: 64 x 16, b_ih[l] / b_hh[l]: 64), so torch's parameters are used in
 * place.  rnnl_lstm_train_sizes gives the float counts of
 *   act [layers][seq_len][6][n x 16]: i, f, g, o, c_t, h_t of every step,
 *   da  [layers][n seq_len][64]: dL/d(gate pre-activations), 0 at pad steps,
 *   xh  [layers][n seq_len][32]: the step input x_t | h_(t-1), 0 at pad steps,
 *   dvx [n seq_len][16]: dL/d(layer-0 input).
 * forward: out (n x 16) = the top layer's output at each rule's last token,
 * act saved.  backward: for d_out = dL/d out, fills da, xh, dvx (the caller
 * forms dW_l = da_l^T xh_l and db_l = column sums of da_l) and d_vocab
 * (vocab_rows x 16, written whole) = the per-token sums of dvx rows listed
 * by tok_id[u] / tok_pos[tok_ptr[u] .. tok_ptr[u + 1]) (positions row
 * seq_len + t, summed in list order; rows of no listed token are zero). */
int rnnl_lstm_train_sizes(int32_t layers, int32_t hidden, int32_t seq_len, int32_t n, size_t *act_floats,
                          size_t *da_floats, size_t *xh_floats, size_t *dvx_floats);
int rnnl_lstm_train_forward(const float *vocab, const float *const *w_ih, const float *const *w_hh,
                            const float *const *b_ih, const float *const *b_hh, int32_t layers, int32_t hidden,
                            const int32_t *tokens, int32_t seq_len, int32_t pad, const int64_t *ridx, int32_t n,
                            float *out, float *act, void *stream);
int rnnl_lstm_train_backward(const float *vocab, const float *const *w_ih, const float *const *w_hh,
                             const float *const *b_ih, const float *const *b_hh, int32_t layers, int32_t hidden,
                             const int32_t *tokens, int32_t seq_len, int32_t pad, const int64_t *ridx, int32_t n,
                             const float *act, const float *d_out, float *da, float *xh, float *dvx,
                             const int32_t *tok_id, const int32_t *tok_ptr, const int32_t *tok_pos, int32_t n_tok,
                             float *d_vocab, int32_t vocab_rows, void *stream);
/* The weight gradients of the same backward (torch.nn.LSTM's dW_ih, dW_hh,
 * db): dW_l = da_l^T xh_l over the `rows` = n seq_len rows of da / xh as
 * filled above, db_l = column sums of da_l, summed in a fixed order (per
 * 128-row segment, then over segments in order) so that they are bitwise
 * repeatable — a library GEMM with K = n seq_len may split K with atomics.
 * out (floats): [layers][64][16] dW_ih | [layers][64][16] dW_hh |
 * [layers][64] db.  part: rnnl_lstm_weight_grads_scratch floats. */
int rnnl_lstm_weight_grads_scratch(int32_t layers, int64_t rows, size_t *part_floats);
int rnnl_lstm_weight_grads(const float *da, const float *xh, int32_t layers, int64_t rows, float *part,
                           size_t part_floats, float *out, void *stream);

/* ------------------------------------------------------------- forward --
 * Replaces the body of PredictorPlus.forward (reference
 * src/predictors.py:210-271) for n_queries rows — one reference batch, or
 * many batches at once — including grounding/propagate (src/data.py:136-173),
 * torch_scatter's scatter-sum, the rule->entity aggregator (src/layers.py)
 * and score_model (src/layers.py:9-51 MLP(32,[128,1])).
 *
 * score (n_queries x E, row-major) must hold the base score on entry
 * (bias row, RotatE scores or -inf; see rnnl_fill_* / rnnl_rotate_score);
 * candidate entries are updated in place.  mask (nullable, n_queries x E
 * bytes, zeroed by the caller) receives 1 at candidates.  n_cand (nullable)
 * receives the candidate count per query; digest (nullable) an
 * order-independent integer fingerprint of the per-rule path counts
 * (tests only; see oracle/ground_oracle.c).
 */
typedef struct {
  int32_t aggregator;      /* RNNL_AGG_* */
  int32_t feature;         /* RNNL_FEATURE_* */
  const void *node_w;      /* rnnl_node_weights output */
  const float *add_w;      /* rule_to_entity.add_model.layers.0.weight (16 x 16 | 16 x 192) */
  const float *add_b;      /* (16) */
  const float *ln_w;       /* rule_to_entity.layer_norm.weight (16) */
  const float *ln_b;       /* (16) */
  const float *s0_w;       /* score_model.layers.0.weight (128 x 32) */
  const float *s0_b;       /* (128) */
  const float *s1_w;       /* score_model.layers.1.weight (1 x 128) */
  const float *s1_b;       /* (1) */
  const float *rel_emb;    /* relation_emb.weight (R x 16) */
  const float *base_row;   /* nullable: the base score every row starts from (the bias vector, E floats);
                              candidates are then written as out + base_row[t] without reading score */
  const float *packed;     /* nullable: the weights above already packed by rnnl_pack_weights (kept by
                              the caller while they do not change); NULL: packed per launch */
} rnnl_predictor_params;
/* Packs the score_model / rule_to_entity weights of p (rnnl_pack_weights_floats
 * floats) for the scoring kernels, so that repeated launches with the same
 * weights (one reference batch per call) skip the packing launch. */
int rnnl_pack_weights_floats(size_t *n_floats);
int rnnl_pack_weights(const rnnl_predictor_params *p, float *out, void *stream);

/* Workspace bytes for one launch of rnnl_predictorplus_forward (host). */
int rnnl_forward_workspace_size(rnnl_graph g, rnnl_rules r, int32_t n_queries, int32_t capacity_scale,
                                size_t *bytes);
int rnnl_predictorplus_forward(rnnl_graph g, rnnl_rules r, const rnnl_predictor_params *p, const int64_t *all_h,
                               const int64_t *all_r, const int64_t *edges_to_remove, int32_t n_queries,
                               float *score, uint8_t *mask, int32_t *n_cand, uint64_t *digest, void *workspace,
                               size_t workspace_bytes, int32_t capacity_scale, void *stream);
/* The same forward in two halves, so that the grounding (independent of the
 * base score) can run on a second stream beside rnnl_rotate_score:
 * rnnl_predictorplus_ground fills the workspace (grounding + candidate
 * buckets, and for PNA the per-row mean log-degree) and n_cand;
 * rnnl_predictorplus_score then updates score / mask from that workspace
 * (same n_queries, capacity_scale, rows).  rnnl_predictorplus_forward ==
 * ground then score on one stream. */
int rnnl_predictorplus_ground(rnnl_graph g, rnnl_rules r, int32_t aggregator, const int64_t *all_h,
                              const int64_t *all_r, const int64_t *edges_to_remove, int32_t n_queries,
                              int32_t *n_cand, void *workspace, size_t workspace_bytes, int32_t capacity_scale,
                              int32_t workgroups, void *stream);
int rnnl_predictorplus_score(rnnl_graph g, rnnl_rules r, const rnnl_predictor_params *p, const int64_t *all_h,
                             const int64_t *all_r, int32_t n_queries, float *score, uint8_t *mask, int32_t *n_cand,
                             uint64_t *digest, void *workspace, size_t workspace_bytes, int32_t capacity_scale,
                             int32_t workgroups, int32_t deferred, void *stream);
/* workgroups: cap on the persistent workgroups of the launch (0 = the full
 * default occupancy); a smaller grid leaves room on the CUs for a kernel on
 * another stream (the RotatE overlap).
 * deferred: 0 = add each candidate's output into the finished base score in
 * `score` and set mask; 2 = (feature add, mask NULL) add the outputs
 * atomically into `score`, which the caller zeroed and whose base score
 * arrives by atomic adds too (rnnl_rotate_score accumulate == 2): the pass
 * then does not wait for the base score and runs beside rnnl_rotate_score;
 * two addends on an exact zero round to fl(base + out) in either order, so
 * the result is deferred == 0's bit for bit. */
/* After a forward: RNNL_OK, or RNNL_ERR_OVERFLOW if any query exceeded the
 * workspace (those rows are incomplete; rerun with a larger capacity_scale).
 * Synchronises `stream`. */
int rnnl_forward_status(void *workspace, void *stream);
/* rnnl_forward_status plus the grounding's totals from the same read-back:
 * totals[0] = candidates (sum of n_cand), totals[1] = bucket entries (the
 * (trie node, path count) entries of the COO), so a caller sizing the COO
 * export needs no further synchronisation.  Valid when RNNL_OK. */
int rnnl_forward_status_totals(void *workspace, void *stream, int64_t *totals);
/* The same status from a host copy of the workspace's first
 * rnnl_forward_header_bytes bytes (copied by the caller on its stream, e.g.
 * asynchronously into pinned memory): no synchronisation here.  totals as
 * for rnnl_forward_status_totals (nullable). */
int rnnl_forward_header_bytes(size_t *bytes);
int rnnl_forward_status_host(const void *header, int64_t *totals);
/* The status with the launch's flags from the same read-back (totals and
 * flags nullable): flags bit 0 (RNNL_FLAG_MIXED) = the rows hold more than one
 * relation — the reference forward's one-relation-per-batch assertion
 * (predictors.py:54-55, 211-212) without a separate reduction.  The _host
 * form decodes the flags of a header copy. */
#define RNNL_FLAG_MIXED 1
int rnnl_forward_status_flags(void *workspace, void *stream, int64_t *totals, uint32_t *flags);
int rnnl_forward_flags_host(const void *header, uint32_t *flags);
/* Where the calling thread's forward resources for graph g live (a
 * multi-GPU self-check): out[0] = g's device, out[1] / out[2] = the devices
 * of the RotatE overlap's side streams for g's device (-1: not created),
 * out[3] = the number of devices this thread holds forward resources for. */
int rnnl_forward_host_info(rnnl_graph g, int32_t *out);
/* Grounding only (reference data.py:136-173 for every rule of every row,
 * predictors.py:221-244): fills the workspace's COO of the stacked rule_count
 * matrix and n_cand (per row candidate count, -1/-2 on overflow/error; check
 * rnnl_forward_status).  Used by the differentiable training path, which
 * exports the COO and evaluates the aggregator/MLP with autograd. */
int rnnl_ground(rnnl_graph g, rnnl_rules r, const int64_t *all_h, const int64_t *all_r,
                const int64_t *edges_to_remove, int32_t n_queries, int32_t *n_cand, void *workspace,
                size_t workspace_bytes, int32_t capacity_scale, void *stream);
/* COO export after rnnl_ground or rnnl_predictorplus_forward (same n_queries /
 * capacity_scale).  cand_off (n_queries + 1, exclusive prefix of n_cand):
 * out_t[cand_off[q] + s] = entity of row q's s-th candidate (ascending entity
 * order = the reference's row-major nonzero), out_nent = its bucket size.
 * ent_off (n_queries + 1): prefix of the per-row sums of out_nent; the
 * entries (trie node, path count) of row q's candidates, candidate-major, land
 * at out_node/out_count[ent_off[q] ..]. */
int rnnl_ground_export_candidates(void *workspace, int32_t n_queries, int32_t capacity_scale, const int32_t *n_cand,
                                  const int64_t *cand_off, int32_t *out_t, int32_t *out_nent, void *stream);
int rnnl_ground_export_entries(void *workspace, int32_t n_queries, int32_t capacity_scale, const int32_t *n_cand,
                               const int64_t *ent_off, int32_t *out_node, int32_t *out_count, void *stream);
/* Diagnostic: when non-NULL, later forward launches add per-phase cycle
 * counters into dev_counters (13 x uint64: prologue, grounding, candidates,
 * queries, contributions, candidates, then the candidate and grounding
 * sub-phases; tools/profile_phases.py). */
int rnnl_debug_profile(void *dev_counters);
/* Diagnostic: when non-NULL, later RotatE launches add (shader-clock ticks,
 * 100 MHz real-time ticks) of every block into dev_counters (2 x uint64); the
 * ratio x 0.1 GHz is the effective shader clock under that kernel's load. */
int rnnl_debug_clock(void *dev_counters);

/* Test hook: lower the per-slot frontier / contribution capacities and the
 * per-query bucket-pool entries of the grounding workspace (at
 * capacity_scale 1; all three <= 0 restores the defaults), so that a test can
 * force RNNL_ERR_OVERFLOW and the host's doubled-capacity_scale retry.
 * Affects the sizes computed by later rnnl_forward_workspace_size / launches
 * in this process. */
int rnnl_debug_capacity(int64_t frontier_base, int64_t contrib_base, int64_t pool_per_query);
/* Phase B's sort-window width 2^bits entities for launches after the call
 * (A/B measurements; -1 = the default: the smallest width giving at most
 * 1024 windows).  Results do not depend on it. */
int rnnl_debug_sort_bits(int32_t bits);
/* Test hook: turn the SUM scoring pass's pair memo (score_model outputs
 * reused between candidates with equal bucket entries) off (0) or on (1,
 * the default), so that a test can compare the outputs both ways. */
int rnnl_debug_pair_memo(int32_t on);

/* ------------------------------------------------------- EM Predictor --
 * The EM loop's rule-weight predictor (reference src/predictors.py:17-119,
 * Predictor.forward / compute_H; run_rnnlogic.py:72-83).
 *
 * rnnl_linear_node_weights: per trie node, the sum of its rules' weights
 * (rule_weights: n_rules floats, fp64 sum) as int32 fixed point with one
 * shift for the table (trailer after the n_nodes values); buffer size from
 * rnnl_linear_node_weights_size.  Replaces the per-rule `x * rule_weights[i]`
 * products of predictors.py:62-66: rules ending at one node share its counts.
 *
 * rnnl_predictor_forward: grounding (as rnnl_ground, with the batch's edge
 * removal) + score[q, t] (+)= sum over the candidate's (node, count) entries
 * of count x node weight, exact int64 sums.  feature RNNL_FEATURE_ADD adds
 * into pre-filled bias rows (rnnl_fill_rows; predictors.py:73-75),
 * RNNL_FEATURE_NONE writes candidates into -inf-filled rows and sets mask
 * (predictors.py:76-78).  The whole-batch early return (predictors.py:68-72)
 * is the caller's (it needs the batch boundaries).
 *
 * rnnl_predictor_rule_stats: after rnnl_ground / rnnl_predictor_forward on
 * the same workspace, per row q and per node k of its head's trie (local
 * index node - root < ld, ld >= max_head_nodes): pos[q*ld + k] = path count
 * of node k at all_t[q], tot[q*ld + k] = its sum over all candidates.  The
 * caller zero-fills pos.  compute_H's pos_score / neg_score
 * (predictors.py:106-113) are w x pos and w x tot / n_cand.
 *
 * rnnl_predictor_backward: after rnnl_predictor_forward on the same
 * workspace, the gradient of the scores with respect to the per-node weight
 * sums: grad_node[n] += sum over every (q, t) of count_n(q, t) x
 * grad_score[q * n_entities + t] (fp64; caller zero-fills n_nodes values;
 * summed as int64 fixed point at one scale per launch, so the result is
 * run-to-run bitwise; the workspace header's words 20..23 hold the scale's
 * statistics).
 * A rule's weight gradient is its node's (rules ending at one node share their
 * counts) — the backward of `score += x * rule_weights[index]`
 * (predictors.py:62-66) that trainer.py:90's loss.backward() takes. */
int rnnl_linear_node_weights_size(rnnl_rules r, size_t *bytes);
int rnnl_linear_node_weights(rnnl_rules r, const float *rule_weights, int32_t n_rules, void *node_w, void *stream);
int rnnl_predictor_forward(rnnl_graph g, rnnl_rules r, const void *node_w, int32_t feature, const int64_t *all_h,
                           const int64_t *all_r, const int64_t *edges_to_remove, int32_t n_queries, float *score,
                           uint8_t *mask, int32_t *n_cand, void *workspace, size_t workspace_bytes,
                           int32_t capacity_scale, void *stream);
/* rnnl_predictor_forward in two halves (training lookahead: the grounding of
 * the next batches, which does not depend on the weights, runs on a second
 * stream while the current batch scores and steps): rnnl_predictor_ground
 * fills the workspace (grounding + the scoring chunk list) and n_cand;
 * rnnl_predictor_score then scores from it (same rows, n_queries,
 * capacity_scale; score pre-filled as for rnnl_predictor_forward).  The
 * overflow status is the workspace's, read after the score half. */
int rnnl_predictor_ground(rnnl_graph g, rnnl_rules r, const int64_t *all_h, const int64_t *all_r,
                          const int64_t *edges_to_remove, int32_t n_queries, int32_t *n_cand, void *workspace,
                          size_t workspace_bytes, int32_t capacity_scale, void *stream);
int rnnl_predictor_score(rnnl_graph g, rnnl_rules r, const void *node_w, int32_t feature, const int64_t *all_h,
                         const int64_t *all_r, int32_t n_queries, float *score, uint8_t *mask, int32_t *n_cand,
                         void *workspace, size_t workspace_bytes, int32_t capacity_scale, void *stream);
int rnnl_predictor_rule_stats(void *workspace, int32_t n_queries, int32_t capacity_scale, const int32_t *n_cand,
                              rnnl_rules r, const int64_t *all_r, const int64_t *all_t, int32_t ld, int64_t *pos,
                              int64_t *tot, void *stream);
int rnnl_predictor_backward(void *workspace, int32_t n_queries, int32_t capacity_scale, const int32_t *n_cand,
                            rnnl_rules r, const int64_t *all_r, int32_t n_entities, const float *grad_score,
                            int32_t ld, double *grad_node, void *stream);

/* --------------------------------------------------------- entity feature --
 * Base-score fills (reference src/predictors.py:260-269). */
int rnnl_fill_rows(const float *row, int32_t n_queries, int32_t n_entities, float *score, void *stream);
int rnnl_fill_value(float value, int64_t n, float *score, void *stream);

/* RotatE entity feature (reference src/embedding.py:28-70):
 * score[q][e] = gamma - sum_d |(h_q o r_q)_d - e_d|, complex entries stored
 * [re(0:D) | im(D:2D)]; relation ids >= n_rel_fwd use the negated half
 * (embedding.py:26).  Two kernels (mode):
 *   RNNL_ROTATE_DIRECT (default)  the reference's arithmetic term by term
 *                                 (differences, squares, sqrt) on the VALU;
 *   RNNL_ROTATE_MFMA              |hr - t|^2 expanded into a bf16x3 MFMA
 *                                 contraction: ~1.7x faster, but the
 *                                 expansion cancels when h o r ~= t (error up
 *                                 to ~sqrt(2^-24 (|hr|^2+|t|^2)) per dim;
 *                                 DESIGN.md "RotatE numerics").
 * Weight-derived device tables, built once per weight version:
 *   entity table    mode-specific layout (rnnl_rotate_entity_table, from eemb
 *                   (E x 2 dim)); size from rnnl_rotate_table_sizes;
 *   relation table  [n_rel_total][dim][2] (cos, sin) of the relation phase
 *                   (rnnl_rotate_relation_table, from remb (n_rel_total x dim)).
 * rnnl_rotate_score replaces RotatE.forward (embedding.py:45-70); it needs a
 * per-call workspace of rnnl_rotate_workspace_size bytes (h o r of every
 * query in DIRECT mode, plus per-32-dim chunk sums when a launch has few rows
 * — the split form, bitwise equal to the one-pass kernel; 0 for MFMA).
 * accumulate: 0 stores, 1 adds into score, 2 adds atomically (a zeroed score
 * shared with rnnl_predictorplus_score deferred == 2 on another stream). */
#define RNNL_ROTATE_DIRECT 0
#define RNNL_ROTATE_MFMA 1
int rnnl_rotate_table_sizes(int32_t n_entities, int32_t dim, int32_t n_rel_total, int32_t mode,
                            size_t *entity_bytes, size_t *relation_bytes);
int rnnl_rotate_entity_table(const float *eemb, int32_t n_entities, int32_t dim, int32_t mode, void *entity_table,
                             void *stream);
int rnnl_rotate_relation_table(const float *remb, int32_t n_rel_total, int32_t dim, float gamma,
                               float *relation_table, void *stream);
int rnnl_rotate_workspace_size(int32_t n_queries, int32_t n_entities, int32_t dim, int32_t mode, size_t *bytes);
int rnnl_rotate_score(const float *eemb, const void *entity_table, const float *relation_table, int32_t dim,
                      float gamma, const int64_t *all_h, const int64_t *all_r, int32_t n_queries,
                      int32_t n_entities, float *score, int32_t accumulate, int32_t mode, void *workspace,
                      size_t workspace_bytes, void *stream);
/* The same scores, bitwise, from `pieces` back-to-back launches over
 * consecutive ranges of the one-pass grid (the first one `first_share` of it,
 * 0 = equal pieces; DIRECT mode with enough rows, otherwise one launch).  A
 * launch boundary lets workgroups of another stream that wait for registers
 * RotatE's waves hold become resident (the PNA scoring pass
 * beside RotatE).  rnnl_rotate_score == pieces 1. */
int rnnl_rotate_score_pieces(const float *eemb, const void *entity_table, const float *relation_table, int32_t dim,
                             float gamma, const int64_t *all_h, const int64_t *all_r, int32_t n_queries,
                             int32_t n_entities, float *score, int32_t accumulate, int32_t mode, void *workspace,
                             size_t workspace_bytes, int32_t pieces, float first_share, void *stream);

/* PredictorPlus.forward with the RotatE entity feature (reference
 * src/predictors.py:210-271 with embedding.py:64-70 as the base score) in one
 * host call: rnnl_predictorplus_ground and rnnl_predictorplus_score
 * (deferred 2) on a side stream beside rnnl_rotate_score_pieces
 * (accumulate 2) on `stream`, into score rows zeroed on a second side
 * stream; mask (nullable, n_queries x E bytes) is filled with 1 (on the
 * second side stream, beside RotatE); then one
 * header read-back, the result as rnnl_forward_status_flags (RNNL_ERR_OVERFLOW:
 * call again with zeroed 0 and a doubled capacity_scale).  zeroed: 0 = the
 * call zeroes the rows first; 1 = rnnl_forward_rotate_zero(score, ...) was
 * issued earlier on this thread (e.g. before the rule encoder, so the fill
 * runs beside it).  The side streams and events are the library's own (per
 * host thread and device).
 * events (nullable, 3 hipEvent_t, each nullable): recorded on `stream` before
 * the launches, after RotatE and the mask, and after the side stream's work
 * (timing).  Same scores as the one-stream path, bit for bit. */
typedef struct {
  const float *eemb;       /* RotatE.eemb (n_entities x 2 dim) */
  const void *etab;        /* rnnl_rotate_entity_table */
  const float *rtab;       /* rnnl_rotate_relation_table */
  int32_t dim, n_entities;
  float gamma;
  int32_t mode;            /* RNNL_ROTATE_* */
  void *workspace;         /* rnnl_rotate_workspace_size bytes (nullable when 0) */
  size_t workspace_bytes;
  int32_t pieces;          /* as rnnl_rotate_score_pieces */
  float first_share;
} rnnl_rotate_args;
int rnnl_predictorplus_forward_rotate(rnnl_graph g, rnnl_rules r, const rnnl_predictor_params *p,
                                      const rnnl_rotate_args *rotate, const int64_t *all_h, const int64_t *all_r,
                                      const int64_t *edges_to_remove, int32_t n_queries, float *score, uint8_t *mask,
                                      int32_t *n_cand, uint64_t *digest, void *workspace, size_t workspace_bytes,
                                      int32_t capacity_scale, int32_t ground_workgroups, int32_t score_workgroups,
                                      int32_t zeroed, void *const *events, void *stream, int64_t *totals,
                                      uint32_t *flags);
int rnnl_forward_rotate_zero(float *score, size_t n_floats, void *stream);

/* Backward of the RotatE score (training; embedding.py:45-70 under autograd):
 * for grad = dL/dscore (n_queries x E, row-major), hr = h o r per query
 * (n_queries x 2 dim: re | im, as torch forms it) and the entity planes
 * (dim x 2 x ld: planes[(2 d + part) * ld + e], ld >= E), writes
 *   d_tail (dim x 2 x E, same plane order) = dL/d(tail entity embedding)
 *   (d_tail may be NULL when the entity table is frozen)
 * and accumulates (atomically; zero it first) d_hr (n_queries x 2 dim) +=
 * dL/d(h o r).  torch.norm's convention: zero gradient where |hr - t| = 0. */
int rnnl_rotate_backward(const float *planes, int32_t ld, const float *hr, const float *grad, int32_t n_queries,
                         int32_t n_entities, int32_t dim, float *d_hr, float *d_tail, void *stream);

/* The RotatE parameter gradients in one call (training; embedding.py:45-70
 * and the h o r product of :55-61 under autograd): for grad = dL/dscore
 * (n_queries x E) of score = gamma - dist(eemb[h] o rot(remb[r]), eemb[e]),
 *   d_eemb (E x 2 dim, eemb's layout; NULL: frozen table) = the tail term of
 *     rnnl_rotate_backward plus the head rows' chain rule,
 *   d_remb (n_rel_total x dim; NULL: frozen) = the phase chain rule,
 * both written whole (no accumulation into the caller's buffers).  planes /
 * ld: the direct-mode entity planes of eemb (rnnl_rotate_entity_table) or any
 * dim x 2 x ld copy; rtab: rnnl_rotate_relation_table of remb and gamma.
 * scratch: rnnl_rotate_param_grads_scratch bytes (with_eemb = d_eemb given).
 * Head rows and relations that repeat in the batch are summed in row order. */
int rnnl_rotate_param_grads_scratch(int32_t n_queries, int32_t n_entities, int32_t dim, int32_t with_eemb,
                                    size_t *bytes);
int rnnl_rotate_param_grads(const float *eemb, const float *planes, int32_t ld, const float *rtab, float gamma,
                            const int64_t *all_h, const int64_t *all_r, int32_t n_queries, int32_t n_entities,
                            int32_t dim, int32_t n_rel_total, const float *grad, void *scratch, size_t scratch_bytes,
                            float *d_eemb, float *d_remb, void *stream);

/* ------------------------------------------------------ training batches --
 * Device-side TrainDataset rows (reference src/data.py:201-219, the target
 * part): out (n_rows x width, f32, row-major) = multi-hot of the value list
 * of row_keys[i] in a CSR map (keys ascending, offs n_keys + 1, vals int32).
 * A key not in the map gives a zero row.  With keys = r * |E| + h and the
 * hr2o lists this is TrainDataset's `target`. */
/* One training batch (TrainDataset.__getitem__, data.py:201-219) in one
 * launch: rows row0 .. row0 + n_rows - 1 of the (n, 3) int64 (h, r, t) table
 * into out_h / out_r / out_t, each row's own relation-local edge id into
 * out_etr (the sorted edge keys (r |E| + t) |E| + h and their ids:
 * relation2ht2index), and the multi-hot target over hr2o (the CSR of
 * rnnl_multi_hot) into out_target (n_rows x n_entities floats). */
int rnnl_train_batch(const int64_t *table, int64_t row0, int32_t n_rows, const int64_t *keys, const int64_t *offs,
                     const int32_t *vals, int64_t n_keys, const int64_t *edge_keys, const int64_t *edge_ids,
                     int64_t n_edges, int32_t n_entities, int64_t *out_h, int64_t *out_r, int64_t *out_t,
                     int64_t *out_etr, float *out_target, void *stream);
int rnnl_multi_hot(const int64_t *keys, const int64_t *offs, const int32_t *vals, int64_t n_keys,
                   const int64_t *row_keys, int32_t n_rows, int32_t width, float *out, void *stream);

/* Evaluation filter rows (reference ValidDataset / TestDataset.__getitem__,
 * src/data.py:250-255 and 287-291): out (n_rows x width, u8 0/1) is 1 except
 * at the values listed for row_keys[i] — with the hr2oo / hr2ooo lists, the
 * reference's `flag` (true = a ranked competitor). Same map layout as
 * rnnl_multi_hot. */
int rnnl_filter_flags(const int64_t *keys, const int64_t *offs, const int32_t *vals, int64_t n_keys,
                      const int64_t *row_keys, int32_t n_rows, int32_t width, uint8_t *out, void *stream);

/* evaluate()'s filtered rank bounds (reference src/trainer.py:191-203) in one
 * pass per row: for row i with target t = all_t[i], L[i] = #(flag & score >
 * score[t]) + 1 and H[i] = #(flag & score >= score[t]) + 2 when mask[i][t],
 * else (1, n_entities + 1).  score f32, mask / flag bytes, all n_rows x
 * n_entities row-major. */
int rnnl_filtered_ranks(const float *score, const uint8_t *mask, const uint8_t *flag, const int64_t *all_t,
                        int32_t n_rows, int32_t n_entities, int64_t *L, int64_t *H, void *stream);

/* ---------------------------------------------------------- rule mining --
 * The reference miner's RuleMiner::search (miner/rnnlogic.cpp:505-589 with
 * KnowledgeGraph::rule_search :350-382) on the GPU: for every train triple
 * (h, r, t), every relation path of length <= max_length (1..3) from h to t
 * with the triple's own edge removed gives the rule r <- path; the pool is the
 * set over all triples minus r <- r.
 *   rnnl_miner_create: host triples (n x 3 int32, train-file order); R < 2^15.
 *   rnnl_rule_search: table = device scratch of table_cap (power of two)
 *     uint64 slots; rules_out receives the distinct rules as keys
 *     head<<47 | len<<45 | b1<<30 | b2<<15 | b3 (numeric order == the
 *     reference's order); counters (4 x uint64, device): [1] != 0 if the table
 *     was too small (retry larger), [2] = number of rules (may exceed out_cap:
 *     retry with a larger rules_out). */
int rnnl_miner_create(const int32_t *hrt, int64_t n_triples, int32_t n_entities, int32_t n_relations,
                      rnnl_miner *out);
int rnnl_miner_destroy(rnnl_miner m);
int rnnl_rule_search(rnnl_miner m, int32_t max_length, uint64_t *table, int64_t table_cap, uint64_t *rules_out,
                     int64_t out_cap, uint64_t *counters, void *stream);

/* ------------------------------------------------------- training loss --
 * TrainerPredictor.train's loss (reference src/trainer.py:84-90) for a model
 * whose mask is all True (bias / RotatE features): with
 * target' = target * smoothing + one_hot(all_t) * (1 - smoothing),
 * loss = -sum log(softmax(logits) + 1e-8) * target' / max(sum target', 1)
 * over the (B, E) rows.  loss: 2 floats (the loss, then the clamped target
 * sum the backward needs).  aux: rnnl_nll_aux_bytes(B) bytes of per-row
 * statistics, kept for the backward.  counter: one uint32 that is zero
 * between launches (the kernel resets it; zero it once, and use it for one
 * launch at a time).  rnnl_nll_backward writes d loss / d logits * grad_out
 * into grad (B, E). */
int rnnl_nll_aux_bytes(int32_t B, size_t *bytes);
int rnnl_nll_forward(const float *logits, const float *target, const int64_t *all_t, int32_t B, int32_t E,
                     float smoothing, uint32_t *counter, void *aux, float *loss, void *stream);
int rnnl_nll_backward(const float *logits, const float *target, const int64_t *all_t, int32_t B, int32_t E,
                      float smoothing, const void *aux, const float *loss, const float *grad_out, float *grad,
                      void *stream);

/* ------------------------------------------------ training backward (K2^T) --
 * The gradient of PredictorPlus's rule part for the SUM aggregator: replaces
 * torch autograd over the reference's forward (src/predictors.py:238-271,
 * src/layers.py:9-77: rule_to_entity = relu(LayerNorm(Linear(sum of count x
 * rule embedding))), cat with relation_emb, score_model MLP(32, [128, 1]),
 * scatter into the score rows) as called by TrainerPredictor.train
 * (src/trainer.py:84-93).  After rnnl_predictorplus_forward over the same
 * rows (its workspace, capacity_scale and n_cand hold the grounding COO and
 * the scoring chunk list; p is that forward's parameter block, node_w from
 * rnnl_node_weights over `emb`; n_cand_total: that forward's candidate total,
 * rnnl_forward_status_totals), given grad_score = dL/d score (n_queries x E),
 * writes dL/d parameter for every parameter of the rule part:
 *   emb: (n_rules x emb_ld) rows of the rule-embedding table the node weights
 *        were built from (rules outside the launch's rows get 0);
 *   add_w (16 x 16), add_b, ln_w, ln_b (16), s0_w (128 x 32), s0_b (128),
 *   s1_w (128), s1_b (1), rel_emb (R x 16).
 * The entity feature's gradient (bias: column sums of grad_score; RotatE:
 * rnnl_rotate_backward) is the caller's.  head >= 0: every row is of that
 * relation (a training batch; only its trie is touched), -1: any rows.
 * scratch: rnnl_predictorplus_backward_size bytes; rows_scratch:
 * rnnl_predictorplus_backward_rows_size(n_queries, n_cand_total) bytes (one
 * dL/dy slot per scoring chunk).  Run-to-run deterministic for head >= 0 (a
 * training batch): fixed-order partial sums, and the per-node gradients as
 * int64 fixed-point sums at one scale per launch (order-independent integer
 * adds); with head = -1 the relation_emb gradient takes fp64 atomics per
 * relation run (order-dependent in the last fp64 bits). */
typedef struct {
  float *emb;
  int32_t emb_ld;
  float *add_w, *add_b, *ln_w, *ln_b, *s0_w, *s0_b, *s1_w, *s1_b, *rel_emb;
} rnnl_sum_grads;
int rnnl_predictorplus_backward_size(rnnl_rules r, int32_t n_relations, size_t *bytes);
int rnnl_predictorplus_backward_rows_size(int32_t n_queries, int64_t n_cand_total, size_t *bytes);
int rnnl_predictorplus_backward(rnnl_graph g, rnnl_rules r, const rnnl_predictor_params *p, const float *emb,
                                int32_t emb_ld, const int64_t *all_r, int32_t n_queries, const float *grad_score,
                                const int32_t *n_cand, int64_t n_cand_total, void *workspace, size_t workspace_bytes,
                                int32_t capacity_scale, int32_t head, void *scratch, size_t scratch_bytes,
                                void *rows_scratch, size_t rows_bytes, const rnnl_sum_grads *grads, void *stream);

/* PNA (FuncToNode) training path (reference src/layers.py:89-101 under
 * autograd): the per-candidate statistics of the grounding in `workspace`
 * (after rnnl_ground / rnnl_predictorplus_ground), candidates in row-major
 * order at cand_off[q] = exclusive prefix of n_cand (n_queries + 1):
 *   wsum / wsq (C x 16) = sum over the candidate's (node, count) entries of
 *     count x (sum over the node's rules of x / of x^2) — exact, one rounding,
 *   mn / mx (C x 16) = min / max of x over the rules reaching it,
 *   deg (C) = 1 + sum of count x rules, row / ent (C) its row and entity,
 *   row_scale (n_queries) = the row's mean log(deg) over its candidates
 *     (layers.py:108-114, one order-free fixed-point sum; 0 without any).
 * node_w: rnnl_node_weights(..., RNNL_AGG_PNA, ...) of the same embeddings.
 * A table the fixed-point records cannot hold, or a candidate past 2^33
 * paths, sets the workspace header's range bits (rnnl_forward_status:
 * RNNL_ERR_RANGE).
 * rnnl_pna_features_backward: d_x (n_rules x 16, written whole) from the
 * gradients of the four statistics — per node sum count x gradient (each
 * gradient rounded to the fixed-point grid once per candidate, times the
 * integer count), a candidate's min / max gradient whole to the smallest trie
 * node tied at its min / max (the reference's .min(1) / .max(1) route it to
 * one index, layers.py:100-101) and split evenly among that node's tied
 * rules; int64 fixed point at one scale per launch: run-to-run bitwise,
 * whatever the split of a (node, candidate) pair over bucket entries.
 * head >= 0: every row is of that relation (only its trie is touched), -1:
 * any rows.  scratch: rnnl_pna_features_backward_scratch bytes. */
int rnnl_pna_features(rnnl_rules r, const void *node_w, void *workspace, int32_t n_queries, int32_t capacity_scale,
                      const int32_t *n_cand, const int64_t *cand_off, int64_t n_cand_total, float *wsum, float *wsq,
                      float *mn, float *mx, float *deg, int64_t *row, int64_t *ent, float *row_scale,
                      void *row_scratch /* n_queries x 8 bytes */, void *stream);
int rnnl_pna_features_backward_scratch(rnnl_rules r, size_t *bytes);
int rnnl_pna_features_backward(rnnl_rules r, const void *node_w, const float *x, int32_t ld, void *workspace,
                               int32_t n_queries, int32_t capacity_scale, const int64_t *all_r, const int32_t *n_cand,
                               const int64_t *cand_off, int64_t n_cand_total, const float *mn, const float *mx,
                               const float *d_wsum,
                               const float *d_wsq, const float *d_mn, const float *d_mx, int32_t head, void *scratch,
                               size_t scratch_bytes, float *d_x, void *stream);

/* ------------------------------------------------ 64-bit path counts --
 * Rows whose path counts (or PNA degree) reach 2^32 fail the forward with
 * RNNL_ERR_RANGE (the grounding kernel sums u32) and n_cand = -2; the
 * reference counts in int64 (src/data.py:139-171).  rnnl_ground_wide grounds
 * rows[0 .. n_rows) again with exact u64 counts, rule-end trie node by node
 * (slow: O(|E|) per hop, for those rows only), appending (row, entity, node,
 * count) entries in no particular order; *cursor receives the entry total
 * (compare with cap; rerun with a larger buffer when it exceeds it).
 * scratch: rnnl_ground_wide_scratch_bytes(n_rows).
 * rnnl_forward_error_bits: the failed launch's error bits (synchronises):
 * 8 count width, 16 node-table range, 32 feature-sum range. */
int rnnl_ground_wide_scratch_bytes(rnnl_graph g, int32_t n_rows, size_t *bytes);
int rnnl_ground_wide(rnnl_graph g, rnnl_rules r, const int64_t *all_h, const int64_t *all_r,
                     const int64_t *edges_to_remove, const int32_t *rows, int32_t n_rows, void *scratch,
                     size_t scratch_bytes, int32_t *out_row, int32_t *out_entity, int32_t *out_node,
                     uint64_t *out_count, int64_t cap, uint64_t *cursor, void *stream);
int rnnl_forward_error_bits(void *workspace, void *stream, uint32_t *bits);

#ifdef __cplusplus
}
#endif
#endif /* RNNLOGIC_HIP_H */
