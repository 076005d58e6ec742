"""TEST INFRASTRUCTURE ONLY — CPU restatement of the reference hot path.

Plain NumPy, written op-for-op after the reference so that tests/ can check the
HIP path against it on the same seeded inputs.  Only tests/, bench.py's
cpu_baseline leg and __graft_entry__.smoke() may import this module; the
product (rnnlogic_amd/) never does.

Pinned against the reference itself: tests/test_oracle.py checks every function
here against tests/golden/*.npz, which tools/make_golden.py produced by running
the reference's own Python (/root/reference/src) in the build container.

Reference anchors (file:line in /root/reference):
  load_graph            src/data.py:10-108    (ids, adjacency in train-file order, hr2o/oo/ooo)
  grounding/propagate   src/data.py:136-173   (dense one-hot chain, per-batch edge drop)
  make_*_batches        src/data.py:186-196, 232-238, 269-275 (python `random` call order)
  lstm_encode           src/predictors.py:201-208 (3-layer LSTM, output at last non-pad token)
  predictorplus_forward src/predictors.py:210-271
  predictor_forward     src/predictors.py:53-80   (EM rule-weight Predictor)
  predictor_compute_H   src/predictors.py:82-119
  func_to_node_sum      src/layers.py:63-77
  func_to_node_pna      src/layers.py:89-126
  mlp                   src/layers.py:35-51
  rotate_forward        src/embedding.py:28-70
  rule_search_pool      miner/rnnlogic.cpp:350-382, 505-589 (the miner's rule search)
  rank_metrics          src/trainer.py:189-238
"""
import json
import os
import random

import numpy as np

PI = 3.141592653589793238462643383279


# --------------------------------------------------------------------------- graph
class Graph:
    def __init__(self, path):
        def rd(fn):
            m = {}
            with open(os.path.join(path, fn)) as f:
                for line in f:
                    i, name = line.strip().split("\t")
                    m[name] = int(i)
            return m

        self.entity2id = rd("entities.dict")
        self.relation2id = rd("relations.dict")
        self.entity_size = len(self.entity2id)
        self.relation_size = len(self.relation2id)

        def trip(fn):
            out = []
            with open(os.path.join(path, fn)) as f:
                for line in f:
                    h, r, t = line.strip().split("\t")
                    out.append((self.entity2id[h], self.relation2id[r], self.entity2id[t]))
            return out

        self.train_facts = trip("train.txt")
        self.valid_facts = trip("valid.txt")
        self.test_facts = trip("test.txt")
        E = self.entity_size
        self.hr2o, self.hr2oo, self.hr2ooo = {}, {}, {}
        for h, r, t in self.train_facts:
            for d in (self.hr2o, self.hr2oo, self.hr2ooo):
                d.setdefault(r * E + h, []).append(t)
        for h, r, t in self.valid_facts:
            for d in (self.hr2oo, self.hr2ooo):
                d.setdefault(r * E + h, []).append(t)
        for h, r, t in self.test_facts:
            self.hr2ooo.setdefault(r * E + h, []).append(t)
        tr = np.asarray(self.train_facts, dtype=np.int64).reshape(-1, 3)
        # per relation: (heads, tails) in file order == relation-local edge ids
        self.adj = []
        self.ht2index = []
        for r in range(self.relation_size):
            sel = tr[tr[:, 1] == r]
            self.adj.append((sel[:, 0].copy(), sel[:, 2].copy()))
            self.ht2index.append({int(t) * E + int(h): i for i, (h, t) in enumerate(zip(sel[:, 0], sel[:, 2]))})


def grounding(g, h, r, body, edges_to_remove):
    """(B, |E|) int64 path counts of `body` from each h (data.py:136-173)."""
    h = np.asarray(h, dtype=np.int64)
    B = len(h)
    x = np.zeros((g.entity_size, B), dtype=np.int64)
    x[h, np.arange(B)] = 1
    for rel in body:
        heads, tails = g.adj[rel]
        msg = x[heads]  # (E_r, B)
        if rel == r and edges_to_remove is not None:
            msg[np.asarray(edges_to_remove, dtype=np.int64), np.arange(B)] = 0
        x = np.zeros_like(x)
        np.add.at(x, tails, msg)
    return x.T.copy()


# --------------------------------------------------------------------------- datasets
def make_train_batches(g, batch_size, r2instances=None):
    """TrainDataset.__init__ + make_batches (data.py:176-196): consumes `random`."""
    if r2instances is None:
        r2instances = [[] for _ in range(g.relation_size)]
        for h, r, t in g.train_facts:
            r2instances[r].append((h, r, t))
    for r in range(g.relation_size):
        random.shuffle(r2instances[r])
    batches = []
    for inst in r2instances:
        for k in range(0, len(inst), batch_size):
            batches.append(inst[k:min(k + batch_size, len(inst))])
    random.shuffle(batches)
    return batches, r2instances


def make_eval_batches(g, facts, batch_size):
    """Valid/TestDataset.__init__ (data.py:222-238, 259-275)."""
    r2inst = [[] for _ in range(g.relation_size)]
    for h, r, t in facts:
        r2inst[r].append((h, r, t))
    batches = []
    for inst in r2inst:
        random.shuffle(inst)
        for k in range(0, len(inst), batch_size):
            batches.append(inst[k:min(k + batch_size, len(inst))])
    return batches


# --------------------------------------------------------------------------- model pieces
def _sigmoid(x):
    return (1.0 / (1.0 + np.exp(-x))).astype(np.float32)


def lstm_encode(sd, rule_features, num_relations, num_layers=3):
    """encode_rules (predictors.py:201-208) with torch.nn.LSTM semantics (i,f,g,o)."""
    x = sd["vocab_emb.weight"][rule_features].astype(np.float32)  # (N, L, H)
    N, L, H = x.shape
    for layer in range(num_layers):
        Wi, Wh = sd["rnn.weight_ih_l%d" % layer], sd["rnn.weight_hh_l%d" % layer]
        b = sd["rnn.bias_ih_l%d" % layer] + sd["rnn.bias_hh_l%d" % layer]
        h = np.zeros((N, H), np.float32)
        c = np.zeros((N, H), np.float32)
        outs = []
        for t in range(L):
            z = x[:, t] @ Wi.T + h @ Wh.T + b
            i, f, gg, o = np.split(z, 4, axis=1)
            c = _sigmoid(f) * c + _sigmoid(i) * np.tanh(gg)
            h = _sigmoid(o) * np.tanh(c)
            outs.append(h)
        x = np.stack(outs, 1).astype(np.float32)
    idx = (rule_features != num_relations).sum(-1) - 1
    return x[np.arange(N), idx]


def mlp(sd, prefix, x, n_layers):
    """MLP.forward (layers.py:35-51): Linear, relu between layers, none at the end."""
    for i in range(n_layers):
        x = x @ sd["%s.layers.%d.weight" % (prefix, i)].T + sd["%s.layers.%d.bias" % (prefix, i)]
        if i < n_layers - 1:
            x = np.maximum(x, 0)
    return x.astype(np.float32)


def layer_norm(x, w, b, eps=1e-5):
    mu = x.mean(-1, keepdims=True)
    var = ((x - mu) ** 2).mean(-1, keepdims=True)
    return ((x - mu) / np.sqrt(var + eps) * w + b).astype(np.float32)


def func_to_node_sum(sd, A, x_f):
    """FuncToNodeSum.forward (layers.py:63-77)."""
    feat = (A.T[:, :, None] * x_f[None]).sum(1)
    out = mlp(sd, "rule_to_entity.add_model", feat, 1)
    out = layer_norm(out, sd["rule_to_entity.layer_norm.weight"], sd["rule_to_entity.layer_norm.bias"])
    return np.maximum(out, 0)


def func_to_node_pna(sd, A, x_f, b_n, eps=1e-6):
    """FuncToNode.forward (layers.py:89-126)."""
    batch_size = int(b_n.max()) + 1
    degree = A.sum(0) + 1
    w = A.T[:, :, None]
    msg = x_f[None]
    s = (msg * w).sum(1)
    sq = ((msg ** 2) * w).sum(1)
    zero = np.broadcast_to(w == 0, (w.shape[0], w.shape[1], msg.shape[2]))
    full = np.broadcast_to(msg, zero.shape)
    mn = np.where(zero, np.inf, full).min(1)
    mx = np.where(zero, -np.inf, full).max(1)
    d = degree[:, None].astype(np.float32)
    mean = s / np.maximum(d, eps)
    sq_mean = sq / np.maximum(d, eps)
    std = np.sqrt(np.maximum(sq_mean - mean ** 2, eps))
    features = np.concatenate([mean, mn, mx, std], -1).astype(np.float32)
    scale = np.log(d)
    sum_scale = np.zeros(batch_size, np.float32)
    cn = np.zeros(batch_size, np.float32)
    np.add.at(sum_scale, b_n, scale[:, 0])
    np.add.at(cn, b_n, 1.0)
    mean_scale = sum_scale / np.maximum(cn, eps)
    scale = scale / np.maximum(mean_scale[b_n][:, None], eps)
    scales = np.concatenate([np.ones_like(scale), scale, 1 / np.maximum(scale, eps)], -1)
    upd = (features[:, :, None] * scales[:, None, :]).reshape(len(features), -1).astype(np.float32)
    out = mlp(sd, "rule_to_entity.add_model", upd, 1)
    out = layer_norm(out, sd["rule_to_entity.layer_norm.weight"], sd["rule_to_entity.layer_norm.bias"])
    return np.maximum(out, 0)


def load_rotate(path):
    """RotatE.__init__ (embedding.py:7-26): returns (eemb, remb_with_negated_half, gamma, dim)."""
    with open(os.path.join(path, "config.json")) as f:
        cfg = json.load(f)
    eemb = np.load(os.path.join(path, "entity_embedding.npy")).astype(np.float32)
    remb = np.load(os.path.join(path, "relation_embedding.npy")).astype(np.float32)
    return eemb, np.concatenate([remb, -remb], 0), float(cfg["gamma"]), int(cfg["hidden_dim"])


def rotate_forward(eemb, remb, gamma, dim, h, r):
    """RotatE.forward (embedding.py:64-70): (B, |E|) = gamma - sum_d |h∘r - e|."""
    rng = np.float32((gamma + 2.0) / dim / PI)
    ph = remb[np.asarray(r)] / rng
    re_r, im_r = np.cos(ph), np.sin(ph)
    he = eemb[np.asarray(h)]
    re_h, im_h = he[:, :dim], he[:, dim:]
    re = re_h * re_r - im_h * im_r
    im = re_h * im_r + im_h * re_r
    dre = re[:, None, :] - eemb[None, :, :dim]
    dim_ = im[:, None, :] - eemb[None, :, dim:]
    dist = np.sqrt(dre * dre + dim_ * dim_).sum(-1, dtype=np.float32)
    return (np.float32(gamma) - dist).astype(np.float32)


def rule_search_pool(g, max_length):
    """RuleMiner::search (miner/rnnlogic.cpp:505-589) with the DFS of
    KnowledgeGraph::rule_search (:350-382): for every train triple (h, r, t),
    every relation path of length <= max_length from h that reaches t (a walk
    stops at t), the triple's own edge skipped at every hop, is the rule
    r <- path; r <- r is dropped (:532-539).  Returns [(head, body tuple)] per
    head in std::set<Rule> order (length, then body).  Pure Python: small
    graphs only."""
    adj = {}
    for h, r, t in g.train_facts:
        adj.setdefault(h, []).append((r, t))
    pool = [set() for _ in range(g.relation_size)]

    def dfs(e, goal, path, head, removed):
        if e == goal:
            pool[head].add(tuple(path))
            return
        if len(path) == max_length:
            return
        for rel, nxt in adj.get(e, ()):
            if (e, rel, nxt) == removed:
                continue
            dfs(nxt, goal, path + [rel], head, removed)

    for h, r, t in g.train_facts:
        found = set()
        pool_r, pool[r] = pool[r], found
        dfs(h, t, [], r, (h, r, t))
        found.discard((r,))  # the per-triple set loses r <- r before the merge
        pool[r] = pool_r | found
    return [(hd, b) for hd in range(g.relation_size) for b in sorted(pool[hd], key=lambda x: (len(x), x))]


class Rules:
    """set_rules (predictors.py:165-199) on a list of token lists or a file."""

    def __init__(self, source, num_relations):
        if isinstance(source, str):
            with open(source) as f:
                toks = [[int(x) for x in line.split()] for line in f]
        else:
            toks = [list(map(int, x)) for x in source]
        self.rules = [(t[0], t[1:]) for t in toks]
        self.max_length = max(len(b) for _, b in self.rules)
        self.relation2rules = [[] for _ in range(num_relations)]
        for i, (hd, body) in enumerate(self.rules):
            self.relation2rules[hd].append((i, (hd, body)))
        self.features = np.asarray([[hd] + body + [num_relations] * (self.max_length - len(body))
                                    for hd, body in self.rules], dtype=np.int64)


def predictorplus_forward(sd, cfg, g, rules, h, r, edges_to_remove, rotate=None):
    """PredictorPlus.forward (predictors.py:210-271) -> (score (B,|E|) f32, mask bool)."""
    h = np.asarray(h, dtype=np.int64)
    r = np.asarray(r, dtype=np.int64)
    q = int(r[0])
    assert (r != q).sum() == 0
    B, E = len(h), g.entity_size
    idx, counts = [], []
    mask = np.zeros((B, E), np.float32)
    for i, (hd, body) in rules.relation2rules[q]:
        c = grounding(g, h, hd, body, edges_to_remove).astype(np.float32)
        mask += c
        idx.append(i)
        counts.append(c)
    feat = cfg["entity_feature"]
    if mask.sum() == 0:
        if feat == "bias":
            return mask + sd["bias"][None], (1 - mask).astype(bool)
        if feat == "RotatE":
            return mask + rotate_forward(*rotate, h, r), (1 - mask).astype(bool)
        return mask - float("-inf"), mask.astype(bool)
    cand = np.nonzero(mask.reshape(-1))[0]
    b_n = cand // E
    A = np.stack(counts, 0).reshape(len(idx), -1)[:, cand]
    idx = np.asarray(idx, dtype=np.int64)
    if cfg["type"] == "emb":
        x_f = sd["rule_emb"][idx]
    else:
        x_f = lstm_encode(sd, rules.features[idx], g.relation_size, cfg.get("num_layers", 3))
    if cfg["aggregator"] == "sum":
        out = func_to_node_sum(sd, A, x_f)
    else:
        out = func_to_node_pna(sd, A, x_f, b_n)
    rel = np.broadcast_to(sd["relation_emb.weight"][q], (len(out), out.shape[1]))
    out = mlp(sd, "score_model", np.concatenate([out, rel], -1), 2)[:, 0]
    score = np.zeros(B * E, np.float32)
    score[cand] = out
    score = score.reshape(B, E)
    if feat == "bias":
        return score + sd["bias"][None], np.ones((B, E), bool)
    if feat == "RotatE":
        return score + rotate_forward(*rotate, h, r), np.ones((B, E), bool)
    m = mask != 0
    return np.where(m, score, -np.inf).astype(np.float32), m


def predictor_forward(sd, feature, g, rules, h, r, edges_to_remove):
    """Predictor.forward (predictors.py:53-80) -> (score (B,|E|) f32, mask bool):
    score = sum over the relation's rules, in rule order, of count * weight (fp32)."""
    h = np.asarray(h, dtype=np.int64)
    r = np.asarray(r, dtype=np.int64)
    q = int(r[0])
    assert (r != q).sum() == 0
    B, E = len(h), g.entity_size
    w = sd["rule_weights"].astype(np.float32)
    score = np.zeros((B, E), np.float32)
    mask = np.zeros((B, E), np.float32)
    for i, (hd, body) in rules.relation2rules[q]:
        x = grounding(g, h, hd, body, edges_to_remove)
        score += x.astype(np.float32) * w[i]
        mask += x
    if mask.sum() == 0:
        if feature == "bias":
            return mask + sd["bias"][None], (1 - mask).astype(bool)
        return mask - float("-inf"), mask.astype(bool)
    if feature == "bias":
        return score + sd["bias"][None], np.ones((B, E), bool)
    m = mask != 0
    return np.where(m, score, -np.inf).astype(np.float32), m


def predictor_compute_H(sd, g, rules, h, r, t, edges_to_remove):
    """Predictor.compute_H (predictors.py:82-119) -> (H (R_q,) f32, rule index) or (None, None):
    per row, pos = count at t times w, neg = sum over candidates of count times w
    divided by the candidate count; softmax over the rules, summed over rows."""
    h = np.asarray(h, dtype=np.int64)
    r = np.asarray(r, dtype=np.int64)
    t = np.asarray(t, dtype=np.int64)
    q = int(r[0])
    B, E = len(h), g.entity_size
    w = sd["rule_weights"].astype(np.float32)
    scores, index = [], []
    mask = np.zeros((B, E), np.float32)
    for i, (hd, body) in rules.relation2rules[q]:
        x = grounding(g, h, hd, body, edges_to_remove)
        scores.append(x.astype(np.float32) * w[i])
        index.append(i)
        mask += x
    if not scores:
        return None, None
    neg = mask != 0
    nneg = np.maximum(neg.sum(1), 1).astype(np.float32)
    rows = np.arange(B)
    Hs = np.stack([s[rows, t] - (s * neg).sum(1, dtype=np.float32) / nneg for s in scores], -1)
    Hs = Hs - Hs.max(-1, keepdims=True)
    e = np.exp(Hs.astype(np.float64))
    return (e / e.sum(-1, keepdims=True)).sum(0).astype(np.float32), np.asarray(index, dtype=np.int64)


def predictor_H_rows(w, pos, tot, ncand):
    """Per-row compute_H terms (predictors.py:109-117) from integer path
    statistics of one row's rules: pos = count at t, tot = sum of counts over
    candidates, ncand = #candidates, w = the rules' weights.  Returns the
    row's softmax over its rules (float64): pos_score = w * pos (one-hot
    divided by 1), neg_score = w * tot / max(ncand, 1)."""
    w = np.asarray(w, np.float64)
    h = w * np.asarray(pos, np.float64) - w * np.asarray(tot, np.float64) / max(int(ncand), 1)
    h = np.exp(h - h.max())
    return h / h.sum()


# --------------------------------------------------------------------------- evaluation
def query_ranks(logits, mask, flag, t):
    """(L, H) per query (trainer.py:190-201)."""
    out = []
    for k in range(len(t)):
        tk = int(t[k])
        if mask[k, tk]:
            val = logits[k, tk]
            row = logits[k][flag[k]]
            out.append((int((row > val).sum()) + 1, int((row >= val).sum()) + 2))
        else:
            out.append((1, flag.shape[1] + 1))
    return out


def test_flags(g, b):
    """TestDataset.__getitem__ mask (data.py:287-291): False at every known answer."""
    flag = np.ones((len(b), g.entity_size), bool)
    for k, (h, r, t) in enumerate(np.asarray(b).tolist()):
        flag[k, g.hr2ooo[r * g.entity_size + h]] = False
    return flag


def near_tie_count(logits, flag, t, tol):
    """Per query: #filtered entities whose score is within tol of the target's.
    Ranks computed from two fp32 evaluations of the same model can differ by at
    most this many places (ties are resolved by exact float equality,
    trainer.py:196-197)."""
    out = []
    for k in range(len(t)):
        row = logits[k][flag[k]]
        v = logits[k, int(t[k])]
        out.append(int((np.abs(row - v) <= tol * max(1.0, abs(float(v)))).sum()) if np.isfinite(v) else 0)
    return out


def rank_metrics(keys_LH, n_total, expectation=True):
    """Metrics of trainer.py:207-238; keys_LH = [(h, r, t, L, H)], n_total = len(ranks)."""
    q2 = {}
    for h, r, t, L, H in keys_LH:
        q2[(h, r, t)] = (L, H)
    hit1 = hit3 = hit10 = mr = mrr = 0.0
    for L, H in q2.values():
        if expectation:
            for rank in range(L, H):
                w = 1.0 / (H - L)
                hit1 += w if rank <= 1 else 0.0
                hit3 += w if rank <= 3 else 0.0
                hit10 += w if rank <= 10 else 0.0
                mr += rank * w
                mrr += 1.0 / rank * w
        else:
            rank = H - 1
            hit1 += rank <= 1
            hit3 += rank <= 3
            hit10 += rank <= 10
            mr += rank
            mrr += 1.0 / rank
    return dict(Hit1=hit1 / n_total, Hit3=hit3 / n_total, Hit10=hit10 / n_total, MR=mr / n_total,
                MRR=mrr / n_total, Data=len(q2))


def rotate_kat_mrr(g, eemb, remb, gamma, dim):
    """Filtered link-prediction MRR/H@10 of a RotatE table, the protocol of the
    shipped train.log files: tail (h, r) and head (t, r + |R|) queries, filter
    train ∪ valid ∪ test, rank = 1 + #(score > true) — known-answer test."""
    R = g.relation_size
    allt = set(g.train_facts) | set(g.valid_facts) | set(g.test_facts)
    rr, h10 = [], []
    test = np.asarray(g.test_facts)
    for side in ("tail", "head"):
        hh = test[:, 0] if side == "tail" else test[:, 2]
        rel = test[:, 1] if side == "tail" else test[:, 1] + R
        tt = test[:, 2] if side == "tail" else test[:, 0]
        s = rotate_forward(eemb, remb, gamma, dim, hh, rel)
        for k in range(len(test)):
            row = s[k].copy()
            h0, r0, t0 = (int(x) for x in test[k])
            for e in range(g.entity_size):
                trip = (h0, r0, e) if side == "tail" else (e, r0, t0)
                if e != tt[k] and trip in allt:
                    row[e] = -np.inf
            rank = 1 + int((row > row[tt[k]]).sum())
            rr.append(1.0 / rank)
            h10.append(rank <= 10)
    return float(np.mean(rr)), float(np.mean(h10))
