"""One FB15k-237 EM iteration at full size on the GPU (BASELINE.json config 5:
config/FB15k-237.yaml through run_rnnlogic.py:56-91), checked phase by phase.

The graph is the seeded synthetic FB15k-237 train graph with the real test
split; the pre-training rule set is rnnlogic_rules.txt with synthetic weights
(FB's mined_rules.txt needs the absent train.txt), and pre-training runs
PRE_EPOCHS of the config's 10,000 epochs.  The rest is the config's:
  sample      TrainerGenerator.sample(100, 3) in the reference's draw order:
              per head relation <= 100 distinct rules of body length <= 3,
              a rule closed by END before length 3 carrying the generator's
              own log_probability of it;
  E-step      Predictor.compute_H_rows over the rows of the first H_BATCHES
              train batches (sampler order, edge removal) against the C
              oracle's per-rule path counts (oracle_query_stats, pinned to
              the reference's compute_H by test_c_oracle_predictor_stats)
              through the reference's softmax, and compute_H per batch on a
              few batches;
  forward     Predictor.forward_rows over all 40,932 test rows: candidate
              counts equal the oracle's on every row, the grounding's
              path-count digests equal the oracle's on every row (the same
              rules through the digest path), and the scores at every
              candidate of every SCORE_STRIDE-th row equal the oracle's
              sum count x weight + bias to 1e-5;
  train/eval  TrainerPredictor.train over TRAIN_BATCHES batches (finite,
              logged losses), evaluate('valid') / evaluate('test');
  M-step      TrainerPredictor.compute_H over every train row, the posterior
              and TrainerGenerator.train(num_epoch=100, lr=1e-5) on it.
"""
import io
import logging

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

PRE_EPOCHS = 200
H_BATCHES = 300
TRAIN_BATCHES = 300
SCORE_STRIDE = 8


def _logged(fn):
    stream = io.StringIO()
    h = logging.StreamHandler(stream)
    root = logging.getLogger()
    old = root.level
    root.addHandler(h)
    root.setLevel(logging.INFO)
    try:
        fn()
    finally:
        root.removeHandler(h)
        root.setLevel(old)
    return [float(p[2]) for p in (line.split() for line in stream.getvalue().splitlines())
            if len(p) >= 3 and p[0].isdigit()]


def test_fb15k237_em_iteration():
    from oracle import ground_c
    from oracle import reference_np as ref
    from rnnlogic_amd import datasets
    from rnnlogic_amd.data import KnowledgeGraph, RuleDataset, TestDataset, TrainDataset, ValidDataset
    from rnnlogic_amd.generators import Generator
    from rnnlogic_amd.predictors import Predictor, PredictorPlus
    from rnnlogic_amd.trainer import TrainerGenerator, TrainerPredictor
    from rnnlogic_amd.utils import set_seed
    from torch.utils import data as torch_data

    dev = torch.device("cuda:0")
    path = datasets.materialize("FB15k-237")
    set_seed(1)
    graph = KnowledgeGraph(path)
    train_set, valid_set, test_set = TrainDataset(graph, 32), ValidDataset(graph, 32), TestDataset(graph, 32)
    mined = [[int(x) for x in line.split()] for line in open(datasets.rule_file("FB15k-237"))]
    dataset = RuleDataset(graph.relation_size, [r + [0.25 * ((i * 37) % 11) - 1.0] for i, r in enumerate(mined)])

    # ---- generator pre-training + sample(num_rules=100, max_length=3)
    gen = Generator(graph, num_layers=1, embedding_dim=512, hidden_dim=256)
    solver_g = TrainerGenerator(gen, gpu=0)
    losses = _logged(lambda: solver_g.train(dataset, num_epoch=PRE_EPOCHS, lr=1e-3, print_every=100,
                                            batch_size=512))
    assert len(losses) == PRE_EPOCHS // 100 and np.isfinite(losses).all()
    sampled = solver_g.sample(100, 3)
    per_rel = {}
    for rule in sampled:
        body = rule[1:-1]
        assert 0 <= rule[0] < graph.relation_size and len(body) <= 3
        assert all(0 <= x < graph.relation_size for x in body)
        per_rel.setdefault(rule[0], set()).add(tuple(rule[:-1]))
    assert len(per_rel) == graph.relation_size
    assert all(len(v) <= 100 for v in per_rel.values())
    assert sum(len(v) for v in per_rel.values()) == len(sampled)  # deduplicated per relation
    # a sequence closed by END before max_length carries END's log p, as
    # log_probability does; full-length ones stop without it (trainer.py:428-445)
    probe = [r for r in sampled if len(r) - 2 < 3][::97][:40]
    assert probe
    lp = solver_g.log_probability([list(r[:-1]) for r in probe])
    np.testing.assert_allclose([r[-1] for r in probe], lp, atol=1e-4, rtol=0)
    prior = [rule[-1] for rule in sampled]
    rules = [rule[0:-1] for rule in sampled]

    # ---- the E-step's Predictor on the sampled rules (weights seeded, nonzero)
    predictor = Predictor(graph, entity_feature="bias")
    predictor.set_rules([list(r) for r in rules])
    torch.manual_seed(5)
    with torch.no_grad():
        predictor.rule_weights.normal_()
        predictor.bias.normal_(std=0.1)
    predictor = predictor.to(dev).eval()
    g = ref.Graph(path)
    orc = ground_c.Oracle(ground_c.CGraph(g.entity_size, g.relation_size, g.train_facts),
                          [(r[0], list(r[1:])) for r in rules], g.relation_size)
    w = predictor.rule_weights.detach().cpu().numpy().astype(np.float64)
    heads = np.asarray([r[0] for r in rules])
    rule_ids = [np.nonzero(heads == q)[0] for q in range(graph.relation_size)]

    sampler = torch_data.DistributedSampler(train_set, 1, 0)
    order = list(iter(sampler))[:H_BATCHES]
    rows = np.asarray([x for i in order for x in train_set.batches[i]], dtype=np.int64)
    etr = np.asarray([graph.relation2ht2index[r][graph.encode_ht(h, t)] for h, r, t in rows], dtype=np.int64)
    rm_src = np.asarray([g.adj[r][0][e] for (_, r, _), e in zip(rows, etr)])
    rm_dst = np.asarray([g.adj[r][1][e] for (_, r, _), e in zip(rows, etr)])
    rq_ptr, pos, tot = orc.query_stats(rows[:, 0], rows[:, 1], rows[:, 2], rm_src, rm_dst)
    _, ncand = orc.digests(rows[:, 0], rows[:, 1], rm_src, rm_dst)
    want_H = np.zeros(len(rules))
    for i in range(len(rows)):
        ids = rule_ids[rows[i, 1]]
        if len(ids):
            want_H[ids] += ref.predictor_H_rows(w[ids], pos[rq_ptr[i]:rq_ptr[i + 1]], tot[rq_ptr[i]:rq_ptr[i + 1]],
                                                ncand[i])
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    got_H = predictor.compute_H_rows(t(rows[:, 0]), t(rows[:, 1]), t(rows[:, 2]), t(etr)).cpu().numpy()
    np.testing.assert_allclose(got_H, want_H, atol=2e-4, rtol=1e-5)
    # the per-batch reference API on a few batches
    off = 0
    for k, i in enumerate(order[:5]):
        n = len(train_set.batches[i])
        sl = slice(off, off + n)
        off += n
        Hb, index = predictor.compute_H(t(rows[sl, 0]), t(rows[sl, 1]), t(rows[sl, 2]), t(etr[sl]))
        q = int(rows[sl.start, 1])
        if len(rule_ids[q]) == 0:
            assert Hb is None
            continue
        np.testing.assert_array_equal(index.cpu().numpy(), rule_ids[q])
        want = sum(ref.predictor_H_rows(w[rule_ids[q]], pos[rq_ptr[j]:rq_ptr[j + 1]], tot[rq_ptr[j]:rq_ptr[j + 1]],
                                        ncand[j]) for j in range(sl.start, sl.stop))
        np.testing.assert_allclose(Hb.cpu().numpy(), want, atol=1e-5, rtol=0)

    # ---- forward over the full test split
    test = np.asarray(g.test_facts, dtype=np.int64)
    want_d, want_n = orc.digests(test[:, 0], test[:, 1])
    with torch.no_grad():
        score, mask, n_cand = predictor.forward_rows(t(test[:, 0]), t(test[:, 1]), None, return_ncand=True)
    np.testing.assert_array_equal(n_cand.cpu().numpy(), want_n)
    assert bool(mask.all())  # bias feature: every entity is scored (predictors.py:73-75)
    sub = np.arange(0, len(test), SCORE_STRIDE)
    _, _, _, cptr, cand, sc = orc.query_stats(test[sub, 0], test[sub, 1], test[sub, 2], weights=w)
    bias = predictor.bias.detach().cpu().numpy().astype(np.float64)
    rows_c = np.repeat(sub, np.diff(cptr))
    got = score[t(rows_c), t(cand.astype(np.int64))].cpu().numpy().astype(np.float64)
    np.testing.assert_allclose(got, sc + bias[cand], atol=1e-5, rtol=1e-6)
    # the same rules through the path-count digest (grounding bit-exactness, every row)
    pp = PredictorPlus(graph, type="emb", entity_feature="bias", aggregator="sum")
    pp.set_rules([list(r) for r in rules])
    pp = pp.to(dev).eval()
    dig = torch.zeros(len(test), dtype=torch.int64, device=dev)
    with torch.no_grad():
        _, _, n2 = pp.forward_rows(t(test[:, 0]), t(test[:, 1]), None, return_ncand=True, digest=dig)
    np.testing.assert_array_equal(n2.cpu().numpy(), want_n)
    np.testing.assert_array_equal(dig.cpu().numpy().view(np.uint64), want_d)
    del score, mask, pp

    # ---- predictor training, evaluation, E-step over the whole split, M-step
    predictor = Predictor(graph, entity_feature="bias")
    predictor.set_rules([list(r) for r in rules])
    optim = torch.optim.Adam(predictor.parameters(), lr=1e-3, weight_decay=0)
    solver_p = TrainerPredictor(predictor, train_set, valid_set, test_set, optim, gpus=[0])
    losses = _logged(lambda: solver_p.train(batch_per_epoch=TRAIN_BATCHES, smoothing=0.2, print_every=100))
    assert len(losses) == TRAIN_BATCHES // 100 and np.isfinite(losses).all()
    for split in ("valid", "test"):
        mrr = solver_p.evaluate(split, expectation=True)
        assert 0.0 < mrr <= 1.0
    likelihood = solver_p.compute_H(print_every=1000)
    assert len(likelihood) == len(rules) and np.isfinite(likelihood).all()
    posterior = [lh + p * 0.001 for lh, p in zip(likelihood, prior)]
    for i in range(len(rules)):
        rules[i].append(posterior[i])
    losses = _logged(lambda: solver_g.train(RuleDataset(graph.relation_size, rules), num_epoch=100, lr=1e-5,
                                            print_every=50, batch_size=512))
    assert len(losses) == 2 and np.isfinite(losses).all()
