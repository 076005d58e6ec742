"""Integer / fixed-point range guards and the workspace-overflow retry of the
HIP forward.

* Path counts are u32 in the grounding kernel's LDS hash (the reference counts
  in int64, src/data.py:139-171).  A layered graph whose path
  count reaches 2^32 must fail loudly (RNNL_ERR_RANGE), and one just below
  (255^4 paths, above 2^31) must match the oracle.
* Rule-embedding / rule-weight aggregates that are non-finite or too large
  for the fixed-point node tables fail loudly instead of converting.
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


def test_path_count_at_2_32_fails_loudly(tmp_path, dev):
    path, rules = chain_graph(tmp_path, 256)  # 256^4 = 2^32 paths e0 -> each L5 entity
    model = _emb_model(KnowledgeGraph(path), rules, dev)
    h = torch.tensor([0], device=dev)
    r = torch.tensor([0], device=dev)
    with pytest.raises(_native.NativeError) as ei:
        with torch.no_grad():
            model(h, r, None)
    assert ei.value.code == _native.RNNL_ERR_RANGE, str(ei.value)


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
    # the training path's COO carries the same u32 count (not a negative int32)
    row, ent, ce, node, count = model.ground_coo(torch.tensor([0], device=dev), torch.tensor([0], device=dev))
    assert sorted(set(ent.tolist())) == [graph.entity_size - 1] and count.tolist() == [m ** 4] * w5


@pytest.mark.parametrize("aggregator", ["sum", "pna"])
def test_count_sum_past_int64_features_fails_loudly(tmp_path, dev, aggregator):
    # three depth-6 entries of 255^4 at e6: the counts sum to 1.27e10 >= 2^33,
    # past what the int64 fixed-point feature sums hold exactly (SUM); for PNA
    # the u32 degree (sum of count x rules) wraps first
    path, rules = chain_graph(tmp_path, 255, w5=3)
    model = _emb_model(KnowledgeGraph(path), rules, dev, aggregator)
    with pytest.raises(_native.NativeError) as ei:
        with torch.no_grad():
            model(torch.tensor([0], device=dev), torch.tensor([0], device=dev), None)
    assert ei.value.code == _native.RNNL_ERR_RANGE, str(ei.value)


@pytest.mark.parametrize("bad", [float("nan"), float("inf"), 2.0 ** 31])
@pytest.mark.parametrize("aggregator", ["sum", "pna"])
def test_node_table_out_of_range_fails_loudly(bad, aggregator, dev):
    path = datasets.materialize("umls")
    graph = KnowledgeGraph(path)
    model = _emb_model(graph, datasets.rule_file("umls"), dev, aggregator)
    with torch.no_grad():
        model.rule_emb[3, 5] = bad
    r0 = int(model.rules[3][0])
    facts = [f for f in graph.test_facts if f[1] == r0][:8]
    h = torch.tensor([f[0] for f in facts], device=dev)
    r = torch.tensor([f[1] for f in facts], device=dev)
    with pytest.raises(_native.NativeError) as ei:
        with torch.no_grad():
            model(h, r, None)
    assert ei.value.code == _native.RNNL_ERR_RANGE, str(ei.value)


def test_em_predictor_weights_out_of_range_fail_loudly(dev):
    path = datasets.materialize("umls")
    graph = KnowledgeGraph(path)
    pred = Predictor(graph, entity_feature="bias")
    pred.set_rules(datasets.rule_file("umls"))
    with torch.no_grad():
        pred.rule_weights.normal_()
        pred.rule_weights[7] = float("nan")
    pred = pred.to(dev).eval()
    facts = graph.test_facts[:16]
    with pytest.raises(_native.NativeError) as ei:
        with torch.no_grad():
            pred.forward_rows(torch.tensor([f[0] for f in facts], device=dev),
                              torch.tensor([f[1] for f in facts], device=dev), None)
    assert ei.value.code == _native.RNNL_ERR_RANGE, str(ei.value)


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
