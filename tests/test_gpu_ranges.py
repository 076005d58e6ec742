"""Integer / fixed-point range guards and the workspace-overflow retry of the
HIP forward.

* Path counts are u32 in the grounding kernel's LDS hash (the reference counts
  in int64, src/data.py:139-171).  A layered graph whose path count reaches
  2^32 is flagged (RNNL_ERR_RANGE) and grounded again with exact u64 counts
  (rnnl_ground_wide): it must match the oracle, as must one just below
  (255^4 paths, above 2^31) through the fused kernels.
* Rule-embedding / rule-weight aggregates that are non-finite or too large
  for the fixed-point node tables, and feature sums past int64, are recomputed
  with the reference's fp32 arithmetic on the grounding COO (infinities and
  NaNs propagate as in the reference).
* A forward whose workspace is too small (capacities lowered with
  rnnl_debug_capacity) reports RNNL_ERR_OVERFLOW, the host retries with a
  doubled capacity_scale, and the result is bit-identical to a forward with
  the default capacities.
"""
import os

import numpy as np
import pytest
import torch

from oracle import reference_np as ref
from rnnlogic_amd import _native, datasets
from rnnlogic_amd.data import KnowledgeGraph
from rnnlogic_amd.predictors import Predictor, PredictorPlus

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def chain_graph(tmp_path, m, w5=1):
    """A layered graph e0 -r1-> L1 -r1-> L2 -r1-> L3 -r1-> L4 -r1-> L5 -r1-> e6
    with m entities in L1..L4 and w5 in L5, consecutive layers wired complete
    bipartite (the reference rejects parallel edges, data.py:68), plus the
    query edge e0 -r0-> e6, and the rule r0 <- r1^6.  Each L5 entity is
    reached by m^4 paths, summed in the grounding kernel's phase-A hash at the
    inner depth-5 trie node (m path counts of m^3 each); e6 then gets w5
    (depth-6, rule-end) entries of m^4 each."""
    d = tmp_path / ("layers%d_%d" % (m, w5))
    d.mkdir()
    layers = [["e0"]] + [["l%d_%d" % (k, i) for i in range(m)] for k in range(1, 5)]
    layers += [["l5_%d" % i for i in range(w5)], ["e6"]]
    ents = [e for layer in layers for e in layer]
    (d / "entities.dict").write_text("".join("%d\t%s\n" % (i, e) for i, e in enumerate(ents)))
    (d / "relations.dict").write_text("0\tr0\n1\tr1\n")
    lines = []
    for a, b in zip(layers[:-1], layers[1:]):
        lines += ["%s\tr1\t%s\n" % (x, y) for x in a for y in b]
    lines.append("e0\tr0\te6\n")
    (d / "train.txt").write_text("".join(lines))
    (d / "valid.txt").write_text("e0\tr0\te6\n")
    (d / "test.txt").write_text("e0\tr0\te6\n")
    rules = d / "rules.txt"
    rules.write_text("0 1 1 1 1 1 1\n")
    return str(d), str(rules)


def _emb_model(graph, rule_path, dev, aggregator="sum"):
    torch.manual_seed(0)
    model = PredictorPlus(graph, type="emb", entity_feature="bias", aggregator=aggregator)
    model.set_rules(rule_path)
    return model.to(dev).eval()


@pytest.mark.parametrize("aggregator", ["sum", "pna"])
@pytest.mark.parametrize("m,w5", [(256, 1), (256, 3)])
def test_path_count_at_2_32_matches_oracle(tmp_path, dev, aggregator, m, w5):
    """256^4 = 2^32 paths e0 -> each L5 entity: past the grounding kernel's u32
    sums (RNNL_ERR_RANGE, n_cand -2), the row is grounded again with exact u64
    counts (rnnl_ground_wide) and scored by the reference's fp32 arithmetic on
    that COO: the oracle's int64 counts (reference data.py:139-171) and scores."""
    path, rules = chain_graph(tmp_path, m, w5)
    graph = KnowledgeGraph(path)
    model = _emb_model(graph, rules, dev, aggregator)
    h = torch.tensor([0], device=dev)
    r = torch.tensor([0], device=dev)
    with torch.no_grad():
        model.bias.normal_()
        score, mask = model(h, r, None)
    g = ref.Graph(path)
    sd = {k: v.detach().cpu().numpy() for k, v in model.state_dict().items()}
    want, wmask = ref.predictorplus_forward(sd, dict(type="emb", aggregator=aggregator, entity_feature="bias"), g,
                                           ref.Rules(rules, g.relation_size), np.asarray([0]), np.asarray([0]), None)
    assert np.array_equal(mask.cpu().numpy(), wmask)
    np.testing.assert_allclose(score.cpu().numpy(), want, atol=1e-4, rtol=1e-5)
    # the COO's int64 counts: w5 x 2^32 paths to e6, one (candidate, node) entry (the oracle's grounding)
    row, ent, ce, node, count = model.ground_coo(h, r)
    assert ent.tolist() == [graph.entity_size - 1] and count.tolist() == [w5 * m ** 4]
    x = ref.grounding(g, np.asarray([0]), 0, [1] * 6, None)
    assert int(x[0, graph.entity_size - 1]) == w5 * m ** 4
    # the training path (autograd on the COO) takes the same counts
    model.train()
    loss = model(h, r, torch.tensor([0], device=dev))[0].logsumexp(1).sum()
    loss.backward()
    assert model.rule_emb.grad is not None and torch.isfinite(model.rule_emb.grad).all()


def test_em_predictor_path_count_at_2_32(tmp_path, dev):
    """The EM Predictor (score = sum of count x rule weight) past 2^32 paths:
    the reference's int64 counts on the wide grounding COO."""
    path, rules = chain_graph(tmp_path, 256, 2)
    graph = KnowledgeGraph(path)
    pred = Predictor(graph, entity_feature="bias")
    pred.set_rules(rules)
    with torch.no_grad():
        pred.rule_weights.fill_(1e-9)
    pred = pred.to(dev).eval()
    g = ref.Graph(path)
    sd = {k: v.detach().cpu().numpy() for k, v in pred.state_dict().items()}
    want, wmask = ref.predictor_forward(sd, "bias", g, ref.Rules(rules, g.relation_size), np.asarray([0]),
                                        np.asarray([0]), None)
    with torch.no_grad():
        score, mask, n_cand = pred.forward_rows(torch.tensor([0], device=dev), torch.tensor([0], device=dev), None,
                                                return_ncand=True)
    assert np.array_equal(mask.cpu().numpy(), wmask)
    np.testing.assert_allclose(score.cpu().numpy(), want, rtol=1e-6, atol=1e-6)
    assert n_cand.tolist() == [1]


@pytest.mark.parametrize("aggregator", ["sum", "pna"])
@pytest.mark.parametrize("m,w5", [(255, 1), (100, 3)])
def test_path_count_above_2_31_matches_oracle(tmp_path, dev, aggregator, m, w5):
    # (255, 1): 255^4 = 4.23e9 paths, above 2^31, below 2^32; (100, 3): three
    # entries of 1e8 at e6 — both past the 2^23 total count below which the
    # scoring kernels' fp64 feature sums are exact (their int64 fallback)
    path, rules = chain_graph(tmp_path, m, w5)
    graph = KnowledgeGraph(path)
    model = _emb_model(graph, rules, dev, aggregator)
    with torch.no_grad():
        model.bias.normal_()
        score, mask = model(torch.tensor([0], device=dev), torch.tensor([0], device=dev), None)
    g = ref.Graph(path)
    sd = {k: v.detach().cpu().numpy() for k, v in model.state_dict().items()}
    want, wmask = ref.predictorplus_forward(sd, dict(type="emb", aggregator=aggregator, entity_feature="bias"), g,
                                           ref.Rules(rules, g.relation_size), np.asarray([0]), np.asarray([0]), None)
    assert np.array_equal(mask.cpu().numpy(), wmask)
    np.testing.assert_allclose(score.cpu().numpy(), want, atol=1e-4, rtol=1e-5)
    # the training path's COO carries the same u32 count (not a negative int32):
    # the rule's one (candidate, node) entry, its w5 paths' counts merged in
    # phase B into the reference's single rule_count cell (w5 x m^4 < 2^32)
    row, ent, ce, node, count = model.ground_coo(torch.tensor([0], device=dev), torch.tensor([0], device=dev))
    assert sorted(set(ent.tolist())) == [graph.entity_size - 1] and count.tolist() == [w5 * m ** 4]


@pytest.mark.parametrize("aggregator", ["sum", "pna"])
def test_count_sum_past_int64_features_matches_oracle(tmp_path, dev, aggregator):
    # three depth-6 entries of 255^4 at e6: the counts sum to 1.27e10 >= 2^33,
    # past what the int64 fixed-point feature sums hold exactly (SUM); for PNA
    # the u32 degree (sum of count x rules) wraps first.  The launch reports
    # RNNL_ERR_RANGE and the rows are recomputed on the grounding COO with the
    # reference's fp32 arithmetic
    path, rules = chain_graph(tmp_path, 255, w5=3)
    graph = KnowledgeGraph(path)
    model = _emb_model(graph, rules, dev, aggregator)
    with torch.no_grad():
        score, mask = model(torch.tensor([0], device=dev), torch.tensor([0], device=dev), None)
    g = ref.Graph(path)
    sd = {k: v.detach().cpu().numpy() for k, v in model.state_dict().items()}
    want, wmask = ref.predictorplus_forward(sd, dict(type="emb", aggregator=aggregator, entity_feature="bias"), g,
                                           ref.Rules(rules, g.relation_size), np.asarray([0]), np.asarray([0]), None)
    assert np.array_equal(mask.cpu().numpy(), wmask)
    np.testing.assert_allclose(score.cpu().numpy(), want, atol=1e-4, rtol=1e-5)


@pytest.mark.parametrize("bad", [float("nan"), float("inf"), 2.0 ** 31])
@pytest.mark.parametrize("aggregator", ["sum", "pna"])
def test_node_table_out_of_range_matches_oracle(bad, aggregator, dev):
    """Rule embeddings the fixed-point node tables cannot hold (non-finite, or
    an aggregate >= 2^30): the launch reports RNNL_ERR_RANGE and the rows are
    recomputed with the reference's fp32 arithmetic on the grounding COO,
    which propagates infinities and NaNs as the reference does
    (layers.py:68-75): the same non-finite pattern, the finite scores close."""
    path = datasets.materialize("umls")
    graph = KnowledgeGraph(path)
    model = _emb_model(graph, datasets.rule_file("umls"), dev, aggregator)
    with torch.no_grad():
        model.rule_emb[3, 5] = bad
    r0 = int(model.rules[3][0])
    facts = [f for f in graph.test_facts if f[1] == r0][:8]
    h = np.asarray([f[0] for f in facts])
    r = np.asarray([f[1] for f in facts])
    with torch.no_grad():
        score, mask = model(torch.from_numpy(h).to(dev), torch.from_numpy(r).to(dev), None)
    g = ref.Graph(path)
    sd = {k: v.detach().cpu().numpy() for k, v in model.state_dict().items()}
    with np.errstate(all="ignore"):
        want, wmask = ref.predictorplus_forward(sd, dict(type="emb", aggregator=aggregator, entity_feature="bias"),
                                               g, ref.Rules(datasets.rule_file("umls"), g.relation_size), h, r, None)
    score = score.cpu().numpy()
    assert np.array_equal(mask.cpu().numpy(), wmask)
    assert np.array_equal(np.isnan(score), np.isnan(want)) and np.array_equal(np.isinf(score), np.isinf(want))
    fin = np.isfinite(want)
    np.testing.assert_allclose(score[fin], want[fin], atol=1e-4, rtol=1e-5)
    assert (~np.isfinite(want)).any() or bad == 2.0 ** 31


def test_em_predictor_weights_out_of_range_match_oracle(dev):
    path = datasets.materialize("umls")
    graph = KnowledgeGraph(path)
    pred = Predictor(graph, entity_feature="bias")
    pred.set_rules(datasets.rule_file("umls"))
    with torch.no_grad():
        pred.rule_weights.normal_()
        pred.rule_weights[7] = float("nan")
    pred = pred.to(dev).eval()
    r7 = int(pred.rules[7][0])
    facts = [f for f in graph.test_facts if f[1] == r7][:16]  # one relation per batch, with the NaN rule
    h = np.asarray([f[0] for f in facts])
    r = np.asarray([f[1] for f in facts])
    with torch.no_grad():
        score, mask = pred.forward_rows(torch.from_numpy(h).to(dev), torch.from_numpy(r).to(dev), None)
    g = ref.Graph(path)
    sd = {k: v.detach().cpu().numpy() for k, v in pred.state_dict().items()}
    with np.errstate(all="ignore"):
        want, wmask = ref.predictor_forward(sd, "bias", g, ref.Rules(datasets.rule_file("umls"), g.relation_size),
                                            h, r, None)
    score = score.cpu().numpy()
    assert np.array_equal(np.isnan(score), np.isnan(want))
    fin = np.isfinite(want)
    np.testing.assert_allclose(score[fin], want[fin], atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize("case", [("umls", "lstm", "sum", "bias"), ("kinship", "emb", "pna", "bias"),
                                  ("umls", "lstm", "sum", "RotatE")])
def test_workspace_overflow_retry_is_bit_identical(case, dev):
    """The RotatE case retries inside the one-call overlap forward
    (rnnl_predictorplus_forward_rotate, rows re-zeroed)."""
    data, typ, agg, feature = case
    path = datasets.materialize(data)
    graph = KnowledgeGraph(path)
    torch.manual_seed(0)
    model = PredictorPlus(graph, type=typ, entity_feature=feature, aggregator=agg,
                          embedding_path=datasets.rotate_path(data) if feature == "RotatE" else None)
    model.set_rules(datasets.rule_file(data))
    if feature == "bias":
        with torch.no_grad():
            model.bias.normal_()
    model = model.to(dev).eval()
    rows = np.asarray(graph.test_facts[:512], dtype=np.int64)
    h = torch.from_numpy(rows[:, 0]).to(dev)
    r = torch.from_numpy(rows[:, 1]).to(dev)
    with torch.no_grad():
        want, wmask, wnc = model.forward_rows(h, r, None, return_ncand=True)
    torch.cuda.synchronize()
    _native.call("rnnl_debug_capacity", 1024, 1024, 64)
    try:
        model.capacity_scale = 1
        model._ws, model._ws_chunks = {}, {}
        with torch.no_grad():
            got, gmask, gnc = model.forward_rows(h, r, None, return_ncand=True)
        torch.cuda.synchronize()
        retried = model.capacity_scale
    finally:
        _native.call("rnnl_debug_capacity", 0, 0, 0)
        model.capacity_scale = 1
        model._ws, model._ws_chunks = {}, {}
    assert retried > 1, "the lowered capacities did not overflow"
    assert torch.equal(gnc, wnc)
    assert torch.equal(gmask, wmask)
    assert torch.equal(got, want), float((got - want).abs().max())
    print("%s: retried up to capacity_scale %d, bit-identical" % (data, retried))


def test_em_compute_H_path_count_at_2_32(tmp_path, dev):
    """compute_H / compute_H_rows (the E-step's rule statistics) past 2^32
    paths: int64 counts from the wide grounding COO against the oracle."""
    path, rules = chain_graph(tmp_path, 256, 2)
    with open(rules, "a") as f:  # a second rule: 2^32 paths to each L5 entity, none to the tail
        f.write("0 1 1 1 1 1\n")
    graph = KnowledgeGraph(path)
    pred = Predictor(graph, entity_feature="bias")
    pred.set_rules(rules)
    with torch.no_grad():
        pred.rule_weights.copy_(torch.tensor([1e-10, 3e-10]))
    pred = pred.to(dev).eval()
    g = ref.Graph(path)
    sd = {k: v.detach().cpu().numpy() for k, v in pred.state_dict().items()}
    h, r, t = np.asarray([0]), np.asarray([0]), np.asarray([graph.entity_size - 1])
    want = ref.predictor_compute_H(sd, g, ref.Rules(rules, g.relation_size), h, r, t, None)
    got, idx = pred.compute_H(torch.from_numpy(h).to(dev), torch.from_numpy(r).to(dev),
                              torch.from_numpy(t).to(dev), None)
    want_h = np.asarray(want[0] if isinstance(want, tuple) else want, dtype=np.float64).reshape(-1)
    np.testing.assert_allclose(got.cpu().numpy().reshape(-1), want_h, rtol=1e-5, atol=1e-7)
    rows = pred.compute_H_rows(torch.from_numpy(h).to(dev), torch.from_numpy(r).to(dev), torch.from_numpy(t).to(dev),
                               None)
    np.testing.assert_allclose(rows[idx].cpu().numpy(), got.cpu().numpy(), rtol=1e-6, atol=1e-8)
