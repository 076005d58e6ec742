"""Edge cases of the PredictorPlus forward on the HIP path, against the CPU
oracle (oracle/reference_np.py, a restatement of predictors.py:210-271):

  * a batch whose relation has no rules — the reference's early return
    (predictors.py:230-237): bias rows / RotatE with the mask all True, and for
    entity_feature 'none' `mask - float('-inf')` = +inf with the mask all False;
  * a batch mixing heads with and without candidates (rows without any path
    keep the base score, or -inf for 'none');
  * an empty row set through forward_rows.
"""
import numpy as np
import pytest
import torch

from oracle import reference_np as ref
from rnnlogic_amd import datasets
from rnnlogic_amd.data import KnowledgeGraph
from rnnlogic_amd.predictors import PredictorPlus

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def umls():
    path = datasets.materialize("umls")
    return path, KnowledgeGraph(path), ref.Graph(path)


def subset_rules(tmp_path, keep_heads):
    """The shipped UMLS rule file restricted to the given head relations."""
    out = tmp_path / "rules_subset.txt"
    with open(datasets.rule_file("umls")) as f, open(out, "w") as g:
        for line in f:
            tok = line.split()
            if tok and int(tok[0]) in keep_heads:
                g.write(line)
    return str(out)


def build(graph, rule_path, feature, dev):
    torch.manual_seed(0)
    model = PredictorPlus(graph, type="emb", entity_feature=feature, aggregator="sum")
    model.set_rules(rule_path)
    if feature == "bias":
        with torch.no_grad():
            model.bias.normal_()
    return model.to(dev).eval()


def oracle(model, g, rule_path, feature, h, r):
    rules = ref.Rules(rule_path, g.relation_size)
    sd = {k: v.detach().cpu().numpy() for k, v in model.state_dict().items()}
    return ref.predictorplus_forward(sd, dict(type="emb", aggregator="sum", entity_feature=feature), g, rules,
                                     np.asarray(h), np.asarray(r), None)


def check(model, g, rule_path, feature, h, r, dev):
    with torch.no_grad():
        score, mask = model(torch.tensor(h, device=dev), torch.tensor(r, device=dev), None)
    want, wmask = oracle(model, g, rule_path, feature, h, r)
    got = score.cpu().numpy()
    assert np.array_equal(mask.cpu().numpy(), wmask)
    fin = np.isfinite(want)
    assert np.array_equal(np.isfinite(got), fin)
    assert np.array_equal(got[~fin], want[~fin])  # +inf / -inf where the reference has them
    assert np.abs(got[fin] - want[fin]).max(initial=0.0) <= 1e-4


@pytest.mark.parametrize("feature", ["bias", "none"])
def test_relation_without_rules(feature, umls, tmp_path):
    dev = torch.device("cuda:0")
    path, graph, g = umls
    heads = sorted({int(line.split()[0]) for line in open(datasets.rule_file("umls")) if line.strip()})
    keep = set(heads[: len(heads) // 2])
    rule_path = subset_rules(tmp_path, keep)
    model = build(graph, rule_path, feature, dev)
    q = next(x for x in range(g.relation_size) if x not in keep)
    h = list(range(16))
    check(model, g, rule_path, feature, h, [q] * len(h), dev)
    if feature == "none":  # the reference's +inf early return, mask all False
        with torch.no_grad():
            score, mask = model(torch.tensor(h, device=dev), torch.tensor([q] * len(h), device=dev), None)
        assert torch.isposinf(score).all() and not mask.any()


@pytest.mark.parametrize("feature", ["bias", "none"])
def test_batch_mixing_heads_with_and_without_candidates(feature, umls, tmp_path):
    dev = torch.device("cuda:0")
    path, graph, g = umls
    rule_path = datasets.rule_file("umls")
    model = build(graph, rule_path, feature, dev)
    # a relation where some heads reach no candidate at all
    for q in range(g.relation_size):
        h_all = list(range(g.entity_size))
        _, m = oracle(model, g, rule_path, "none", h_all, [q] * len(h_all))
        empty = [x for x in h_all if not m[x].any()]
        full = [x for x in h_all if m[x].any()]
        if empty and full:
            break
    else:
        pytest.skip("no relation with both kinds of heads")
    h = (full[:10] + empty[:6]) * 2
    check(model, g, rule_path, feature, h, [q] * len(h), dev)


@pytest.mark.parametrize("kind", ["predictorplus", "predictor"])
def test_empty_row_set(kind, umls):
    from rnnlogic_amd.predictors import Predictor
    dev = torch.device("cuda:0")
    path, graph, g = umls
    if kind == "predictor":
        model = Predictor(graph, entity_feature="bias")
        model.set_rules(datasets.rule_file("umls"))
        model = model.to(dev).eval()
    else:
        model = build(graph, datasets.rule_file("umls"), "bias", dev)
    e = torch.empty(0, dtype=torch.int64, device=dev)
    with torch.no_grad():
        score, mask = model.forward_rows(e, e, None)
    torch.cuda.synchronize()
    assert tuple(score.shape) == (0, g.entity_size) and tuple(mask.shape) == (0, g.entity_size)


def test_mixed_relation_batch_fails_like_the_reference(umls):
    """forward() keeps the reference's one-relation-per-batch assertion
    (predictors.py:54-55, 211-212), now read from the grounding launch's
    header flag: PredictorPlus (fused and overlapped RotatE-free path) and
    the EM Predictor raise on a batch mixing relations and accept a
    single-relation batch; forward_rows accepts mixed rows."""
    from rnnlogic_amd.predictors import Predictor
    path, graph, _ = umls
    dev = torch.device("cuda:0")
    facts = np.asarray(graph.test_facts, dtype=np.int64)
    r0, r1 = int(facts[0, 1]), int(next(f[1] for f in facts if f[1] != facts[0, 1]))
    one = facts[facts[:, 1] == r0][:6]
    mixed = np.concatenate([one[:3], facts[facts[:, 1] == r1][:3]])
    torch.manual_seed(0)
    plus = PredictorPlus(graph, type="emb", entity_feature="bias", aggregator="sum")
    plus.set_rules(datasets.rule_file("umls"))
    pred = Predictor(graph, entity_feature="bias")
    pred.set_rules(datasets.rule_file("umls"))
    plus, pred = plus.to(dev).eval(), pred.to(dev).eval()
    t = lambda a: torch.from_numpy(a).to(dev)  # noqa: E731
    with torch.no_grad():
        for model in (plus, pred):
            model(t(one[:, 0]), t(one[:, 1]), None)
            with pytest.raises(AssertionError):
                model(t(mixed[:, 0]), t(mixed[:, 1]), None)
            model(t(one[:, 0]), t(one[:, 1]), None)  # the flag does not stick
        plus.forward_rows(t(mixed[:, 0]), t(mixed[:, 1]), None)


@pytest.mark.skipif(not torch.cuda.is_available() or torch.cuda.device_count() < 2, reason="needs two GPUs")
def test_forward_on_second_device_with_current_device_elsewhere(umls):
    """a model and rows on cuda:1 while the current device is
    cuda:0 (the reference trainer picks cuda:k without set_device).  The
    overlap's side streams, the header read-back and torch's null stream must
    all be cuda:1's: the scores equal the same forward run on cuda:0."""
    path, graph, _ = umls
    outs = []
    for k in (0, 1):
        torch.cuda.set_device(0)
        dev = torch.device("cuda", k)
        torch.manual_seed(0)
        model = PredictorPlus(graph, type="lstm", entity_feature="RotatE", aggregator="sum",
                              embedding_path=datasets.rotate_path("umls", 200))
        model.set_rules(datasets.rule_file("umls"))
        model = model.to(dev).eval()
        h = torch.arange(0, 64, device=dev) % graph.entity_size
        r = torch.full_like(h, 3)
        with torch.no_grad():
            score, mask = model.forward_rows(h, r, None)
        assert torch.cuda.current_device() == 0
        outs.append((score.cpu(), mask.cpu()))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
