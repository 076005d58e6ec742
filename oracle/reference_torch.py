"""TEST / BASELINE INFRASTRUCTURE ONLY — the reference PyTorch predictor,
restated in torch eager so it runs on any device (CPU here, the MI355X on the
GPU box): the "reference PyTorch predictor on the same box" that
BASELINE.json's north_star asks to be timed beside the HIP path.

Op for op after the reference (the dense formulation, NOT the HIP path's):
  grounding/propagate  src/data.py:136-173  one-hot (|E|, B, 1) int64 state,
                       gather x[head], per-batch-element edge drop
                       (msg.view(-1, 1)[e_b * B + b] = 0), scatter-sum onto the
                       tails (torch_scatter.scatter(..., reduce='sum') ==
                       index_add_, the only reduce the reference uses)
  forward              src/predictors.py:210-271  rule loop, stacked counts,
                       nonzero candidates, rule_to_entity, score_model, scatter
  encode_rules         src/predictors.py:201-208  torch.nn.LSTM, last non-pad
  FuncToNodeSum        src/layers.py:63-77
  FuncToNode (pna)     src/layers.py:89-126
  MLP                  src/layers.py:35-51
  RotatE.forward       src/embedding.py:45-70  (dense (B, |E|, D) expansion)

Only tests/ and bench.py's baseline leg import this module; the product
(rnnlogic_amd/) never does.  Pinned by tests/test_oracle.py against the
reference's own outputs (tests/golden/*.npz).
"""
import torch
import torch.nn.functional as F

from . import reference_np as ref

PI = 3.141592653589793238462643383279


class TorchGraph:
    """Per-relation (heads, tails) in train-file order (data.py:39-106) on `device`."""

    def __init__(self, g, device):
        self.entity_size = g.entity_size
        self.relation_size = g.relation_size
        self.adj = [(torch.as_tensor(h, device=device), torch.as_tensor(t, device=device)) for h, t in g.adj]
        self.device = device


def grounding(tg, h, r, body, edges_to_remove):
    """(B, |E|) int64 path counts (data.py:136-147 + propagate 149-173)."""
    B = h.numel()
    ar = torch.arange(B, device=tg.device)
    x = torch.zeros((tg.entity_size, B, 1), dtype=torch.int64, device=tg.device)
    x[h, ar, 0] = 1
    for rel in body:
        heads, tails = tg.adj[rel]
        msg = x[heads]  # (E_r, B, 1)
        if rel == r and edges_to_remove is not None:
            msg.view(-1, 1)[edges_to_remove * B + ar] = 0
        x = torch.zeros_like(x).index_add_(0, tails, msg)
    return x.squeeze(-1).t()


class Model:
    """PredictorPlus with the reference's parameters (a state_dict of numpy
    arrays or tensors) on `device`."""

    def __init__(self, sd, cfg, g, rules, device, rotate=None):
        self.cfg = dict(cfg)
        self.device = device
        self.tg = TorchGraph(g, device)
        self.rules = rules
        self.sd = {k: torch.as_tensor(v).to(device) for k, v in sd.items()}
        self.features = torch.as_tensor(rules.features, device=device)
        self.lstm = None
        if self.cfg.get("type", "emb") != "emb":
            L = self.cfg.get("num_layers", 3)
            self.lstm = torch.nn.LSTM(16, 16, L, batch_first=True).to(device)
            self.lstm.load_state_dict({k[4:]: v for k, v in self.sd.items() if k.startswith("rnn.")})
        self.rotate = None
        if rotate is not None:
            eemb, remb, gamma, dim = rotate
            self.rotate = (torch.as_tensor(eemb, device=device), torch.as_tensor(remb, device=device), gamma, dim)

    def encode_rules(self, idx):
        """predictors.py:201-208."""
        feats = self.features[idx]
        mask = feats != self.tg.relation_size
        out, _ = self.lstm(F.embedding(feats, self.sd["vocab_emb.weight"]))
        last = (mask.sum(-1) - 1).long()
        return out.gather(1, last.view(-1, 1, 1).expand(-1, 1, out.size(-1))).squeeze(1)

    def linear(self, prefix, x):
        return F.linear(x, self.sd[prefix + ".weight"], self.sd[prefix + ".bias"])

    def func_to_node_sum(self, A, x_f):
        """layers.py:63-77."""
        feat = (A.t().unsqueeze(-1) * x_f.unsqueeze(0)).sum(1)
        out = self.linear("rule_to_entity.add_model.layers.0", feat)
        out = F.layer_norm(out, (out.size(-1),), self.sd["rule_to_entity.layer_norm.weight"],
                           self.sd["rule_to_entity.layer_norm.bias"])
        return F.relu(out)

    def func_to_node_pna(self, A, x_f, b_n, eps=1e-6):
        """layers.py:89-126."""
        batch_size = int(b_n.max().item()) + 1
        degree = A.sum(0) + 1
        w = A.t().unsqueeze(-1)
        msg = x_f.unsqueeze(0)
        s = (msg * w).sum(1)
        sq = ((msg ** 2) * w).sum(1)
        zero = (w == 0).expand(-1, -1, msg.size(-1))
        full = msg.expand_as(zero)
        mn = full.masked_fill(zero, float("inf")).min(1)[0]
        mx = full.masked_fill(zero, float("-inf")).max(1)[0]
        d = degree.unsqueeze(-1)
        mean = s / d.clamp(min=eps)
        sq_mean = sq / d.clamp(min=eps)
        std = (sq_mean - mean ** 2).clamp(min=eps).sqrt()
        features = torch.cat([mean, mn, mx, std], -1)
        scale = d.log()
        sum_scale = torch.zeros(batch_size, device=A.device).index_add_(0, b_n, scale.squeeze(-1))
        cn = torch.zeros(batch_size, device=A.device).index_add_(0, b_n, torch.ones_like(scale.squeeze(-1)))
        mean_scale = sum_scale / cn.clamp(min=eps)
        scale = scale / mean_scale[b_n].unsqueeze(-1).clamp(min=eps)
        scales = torch.cat([torch.ones_like(scale), scale, 1 / scale.clamp(min=eps)], -1)
        upd = (features.unsqueeze(-1) * scales.unsqueeze(-2)).flatten(1)
        out = self.linear("rule_to_entity.add_model.layers.0", upd)
        out = F.layer_norm(out, (out.size(-1),), self.sd["rule_to_entity.layer_norm.weight"],
                           self.sd["rule_to_entity.layer_norm.bias"])
        return F.relu(out)

    def rotate_forward(self, h, r):
        """embedding.py:45-70, the dense expansion."""
        eemb, remb, gamma, dim = self.rotate
        phase = remb[r] / ((gamma + 2.0) / dim / PI)
        re_r, im_r = torch.cos(phase), torch.sin(phase)
        he = eemb[h]
        re_h, im_h = he[:, :dim], he[:, dim:]
        re = re_h * re_r - im_h * im_r
        im = re_h * im_r + im_h * re_r
        dre = re.unsqueeze(1) - eemb[:, :dim].unsqueeze(0)
        dim_ = im.unsqueeze(1) - eemb[:, dim:].unsqueeze(0)
        dist = torch.stack([dre, dim_], 0).norm(dim=0).sum(-1)
        return gamma - dist

    @torch.no_grad()
    def forward(self, h, r, edges_to_remove):
        """predictors.py:210-271 -> (score (B, |E|) f32, mask bool)."""
        h = torch.as_tensor(h, device=self.device)
        r = torch.as_tensor(r, device=self.device)
        etr = torch.as_tensor(edges_to_remove, device=self.device) if edges_to_remove is not None else None
        q = int(r[0].item())
        B, E = h.numel(), self.tg.entity_size
        feat = self.cfg["entity_feature"]
        idx, counts = [], []
        mask = torch.zeros((B, E), device=self.device)
        for i, (hd, body) in self.rules.relation2rules[q]:
            c = grounding(self.tg, h, hd, body, etr).float()
            mask += c
            idx.append(i)
            counts.append(c)
        if mask.sum().item() == 0:
            if feat == "bias":
                return mask + self.sd["bias"].unsqueeze(0), (1 - mask).bool()
            if feat == "RotatE":
                return mask + self.rotate_forward(h, r), (1 - mask).bool()
            return mask - float("-inf"), mask.bool()
        cand = torch.nonzero(mask.view(-1)).view(-1)
        b_n = cand // E
        A = torch.stack(counts, 0).view(len(idx), -1)[:, cand]
        idx = torch.as_tensor(idx, dtype=torch.long, device=self.device)
        x_f = self.sd["rule_emb"][idx] if self.lstm is None else self.encode_rules(idx)
        if self.cfg["aggregator"] == "sum":
            out = self.func_to_node_sum(A, x_f)
        else:
            out = self.func_to_node_pna(A, x_f, b_n)
        rel = self.sd["relation_emb.weight"][q].unsqueeze(0).expand(out.size(0), -1)
        out = self.linear("score_model.layers.1", F.relu(self.linear("score_model.layers.0",
                                                                     torch.cat([out, rel], -1)))).squeeze(-1)
        score = torch.zeros(B * E, device=self.device).scatter_(0, cand, out).view(B, E)
        if feat == "bias":
            return score + self.sd["bias"].unsqueeze(0), torch.ones((B, E), dtype=torch.bool, device=self.device)
        if feat == "RotatE":
            return score + self.rotate_forward(h, r), torch.ones((B, E), dtype=torch.bool, device=self.device)
        m = mask != 0
        return score.masked_fill(~m, float("-inf")), m


def from_fixture(fx, device):
    """A Model with a golden fixture's graph, rules, state_dict and RotatE."""
    g = ref.Graph(fx.dataset_path())
    rules = ref.Rules(fx.rule_path(), g.relation_size)
    rot = ref.load_rotate(fx.rotate_path()) if fx.rotate_path() else None
    return Model(fx.sd, fx.cfg["model"], g, rules, device, rot)
