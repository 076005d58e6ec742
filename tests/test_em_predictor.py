"""EM rule-weight Predictor (reference src/predictors.py:17-119).

CPU: the oracle (oracle/reference_np.py predictor_forward / predictor_compute_H)
against the reference's own outputs (tests/golden/pred_*.npz, made by
tools/make_golden_predictor.py).
GPU: the HIP path (rnnl_predictor_forward, rnnl_predictor_rule_stats, the
COO autograd path) against the same fixtures: scores within 1e-4 abs (fp32),
masks identical, compute_H within 1e-5, TrainerPredictor.compute_H over the
whole train split and the first Adam steps' losses / gradients.
"""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, PRED_CASES
from oracle import reference_np as ref

SCORE_TOL = 1e-4


class PredFixture:
    def __init__(self, name):
        self.z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
        self.cfg = json.loads(str(self.z["cfg"]))
        self.sd = {k[3:]: self.z[k] for k in self.z.files if k.startswith("sd/")}
        self.ncalls = int(self.z["ncalls"])
        self.nH = int(self.z["nH"])

    def call(self, k):
        p = "q%d/" % k
        split = str(self.z[p + "split"])
        return dict(split=split, h=self.z[p + "h"], r=self.z[p + "r"], t=self.z[p + "t"],
                    etr=self.z[p + "etr"] if split == "train" else None, score=self.z[p + "score"],
                    mask=self.z[p + "mask"])

    def hcall(self, k):
        p = "H%d/" % k
        return {n: self.z[p + n] for n in ("h", "r", "t", "etr", "H", "index")}

    def paths(self):
        from rnnlogic_amd import datasets
        return datasets.materialize(self.cfg["data"]), datasets.rule_file(self.cfg["data"])


_cache = {}


def _fixture(name):
    if name not in _cache:
        fx = PredFixture(name)
        dpath, rpath = fx.paths()
        g = ref.Graph(dpath)
        _cache[name] = (fx, g, ref.Rules(rpath, g.relation_size))
    return _cache[name]


def _check_scores(score, mask, want_score, want_mask, tol):
    np.testing.assert_array_equal(mask, want_mask)
    fin = np.isfinite(want_score)
    np.testing.assert_array_equal(np.isfinite(score), fin)
    np.testing.assert_array_equal(score[~fin], want_score[~fin])
    np.testing.assert_allclose(score[fin], want_score[fin], atol=tol, rtol=0)


# ----------------------------------------------------------------------------- CPU: oracle pinning
@pytest.mark.parametrize("case", PRED_CASES)
def test_oracle_predictor_forward(case):
    fx, g, rules = _fixture(case)
    for k in range(0, fx.ncalls, 3):
        c = fx.call(k)
        score, mask = ref.predictor_forward(fx.sd, fx.cfg["feature"], g, rules, c["h"], c["r"], c["etr"])
        _check_scores(score, mask, c["score"], c["mask"], 1e-5)


@pytest.mark.parametrize("case", PRED_CASES)
def test_oracle_predictor_compute_H(case):
    fx, g, rules = _fixture(case)
    for k in range(fx.nH):
        c = fx.hcall(k)
        H, index = ref.predictor_compute_H(fx.sd, g, rules, c["h"], c["r"], c["t"], c["etr"])
        if c["index"].size == 0:
            assert H is None
            continue
        np.testing.assert_array_equal(index, c["index"])
        np.testing.assert_allclose(H, c["H"], atol=1e-5, rtol=0)


# ----------------------------------------------------------------------------- GPU: the HIP path
def _model(fx, device):
    from rnnlogic_amd.data import KnowledgeGraph
    from rnnlogic_amd.predictors import Predictor
    dpath, rpath = fx.paths()
    graph = KnowledgeGraph(dpath)
    model = Predictor(graph, entity_feature=fx.cfg["feature"])
    model.set_rules(rpath)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in fx.sd.items()})
    return model.to(device), graph


@pytest.mark.gpu
@pytest.mark.parametrize("case", PRED_CASES)
def test_predictor_forward_hip(case):
    fx, _, _ = _fixture(case)
    dev = torch.device("cuda:0")
    model, _ = _model(fx, dev)
    model.eval()
    with torch.no_grad():
        for k in range(fx.ncalls):
            c = fx.call(k)
            etr = torch.from_numpy(c["etr"]).to(dev) if c["etr"] is not None else None
            score, mask = model(torch.from_numpy(c["h"]).to(dev), torch.from_numpy(c["r"]).to(dev), etr)
            _check_scores(score.cpu().numpy(), mask.cpu().numpy(), c["score"], c["mask"], SCORE_TOL)
    # every test batch of the fixture in ONE launch (rows of mixed relations)
    rows = [fx.call(k) for k in range(fx.ncalls) if fx.call(k)["split"] == "test"]
    h = torch.from_numpy(np.concatenate([c["h"] for c in rows])).to(dev)
    r = torch.from_numpy(np.concatenate([c["r"] for c in rows])).to(dev)
    with torch.no_grad():
        score, mask, n_cand = model.forward_rows(h, r, None, return_ncand=True)
    score, mask, off = score.cpu().numpy(), mask.cpu().numpy(), 0
    for c in rows:
        n = len(c["h"])
        if fx.cfg["feature"] != "bias" and not c["mask"].any():
            off += n  # whole-batch early return (+inf) is a per-batch property: checked above
            continue
        _check_scores(score[off:off + n], mask[off:off + n], c["score"], c["mask"], SCORE_TOL)
        off += n


@pytest.mark.gpu
@pytest.mark.parametrize("case", PRED_CASES)
def test_predictor_compute_H_hip(case):
    fx, _, _ = _fixture(case)
    dev = torch.device("cuda:0")
    model, _ = _model(fx, dev)
    model.eval()
    with torch.no_grad():
        for k in range(fx.nH):
            c = fx.hcall(k)
            H, index = model.compute_H(torch.from_numpy(c["h"]).to(dev), torch.from_numpy(c["r"]).to(dev),
                                       torch.from_numpy(c["t"]), torch.from_numpy(c["etr"]).to(dev))
            if c["index"].size == 0:
                assert H is None
                continue
            np.testing.assert_array_equal(index.cpu().numpy(), c["index"])
            np.testing.assert_allclose(H.cpu().numpy(), c["H"], atol=1e-5, rtol=0)


@pytest.mark.gpu
@pytest.mark.parametrize("case", PRED_CASES)
def test_predictor_trainer_hip(case):
    """TrainerPredictor on the GPU: compute_H over the whole train split,
    evaluate('test') metrics, and the first Adam steps of train()'s loop
    (trainer.py:48-105) with the reference's batch order."""
    from torch.utils import data as torch_data
    from rnnlogic_amd.data import KnowledgeGraph, TestDataset, TrainDataset, ValidDataset
    from rnnlogic_amd.predictors import Predictor
    from rnnlogic_amd.trainer import TrainerPredictor
    from rnnlogic_amd.utils import set_seed
    fx, _, _ = _fixture(case)
    dev = torch.device("cuda:0")
    dpath, rpath = fx.paths()
    set_seed(1)  # the fixture generator's order: graph, datasets, model
    graph = KnowledgeGraph(dpath)
    train_set, valid_set, test_set = TrainDataset(graph, 32), ValidDataset(graph, 32), TestDataset(graph, 32)
    model = Predictor(graph, entity_feature=fx.cfg["feature"])
    model.set_rules(rpath)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in fx.sd.items()})
    solver = TrainerPredictor(model, train_set, valid_set, test_set, None, gpus=[dev])
    Hall = np.asarray(solver.compute_H(print_every=1000000), dtype=np.float32)
    np.testing.assert_allclose(Hall, fx.z["Hall"], atol=1e-6, rtol=1e-4)
    mrr = solver.evaluate("test", expectation=True)
    assert abs(mrr - float(fx.z["eval/mrr"])) < 1e-6, (mrr, float(fx.z["eval/mrr"]))
    model = solver.model
    optim = torch.optim.Adam(model.parameters(), lr=fx.cfg["lr"], weight_decay=0)
    train_set.make_batches()
    sampler = torch_data.DistributedSampler(train_set, 1, 0)
    sampler.set_epoch(0)
    order = list(iter(sampler))[:len(fx.z["order"])]
    np.testing.assert_array_equal(order, fx.z["order"])
    model.train()
    for k, idx in enumerate(order):
        all_h, all_r, all_t, target, etr = train_set[idx]
        p = "s%d/" % k
        for name, got in (("h", all_h), ("r", all_r), ("t", all_t), ("etr", etr)):
            np.testing.assert_array_equal(got.numpy(), fx.z[p + name])
        target = (target * 0.2 + torch.nn.functional.one_hot(all_t, graph.entity_size) * 0.8).to(dev)
        logits, mask = model(all_h.to(dev), all_r.to(dev), etr.to(dev))
        want = float(fx.z[p + "loss"])
        if mask.sum().item() == 0:
            assert np.isnan(want)
            continue
        logits = (torch.softmax(logits, dim=1) + 1e-8).log()
        loss = -(logits[mask] * target[mask]).sum() / torch.clamp(target[mask].sum(), min=1)
        loss.backward()
        assert abs(loss.item() - want) <= 1e-5 * max(1.0, abs(want)), (case, k, loss.item(), want)
        if k == 0:
            for n, prm in model.named_parameters():
                want_g = fx.z["g/" + n]
                atol = 1e-6 * max(1.0, float(np.abs(want_g).max()))
                np.testing.assert_allclose(prm.grad.detach().cpu().numpy(), want_g, atol=atol, rtol=1e-5)
        optim.step()
        optim.zero_grad()


# ----------------------------------------------------------------------------- CPU: the C oracle's EM statistics
@pytest.mark.parametrize("case", PRED_CASES)
def test_c_oracle_predictor_stats(case):
    """oracle_query_stats (per-rule path counts at the true tail and in
    total, and the Predictor score per candidate) against the reference's
    compute_H and forward outputs (tests/golden/pred_*.npz) — the checker the
    FB15k-237 EM test uses at full size."""
    from oracle import ground_c
    fx, g, rules = _fixture(case)
    cg = ground_c.CGraph(g.entity_size, g.relation_size, g.train_facts)
    orc = ground_c.Oracle(cg, [(hd, list(b)) for hd, b in rules.rules], g.relation_size)
    w = fx.sd["rule_weights"].astype(np.float64)
    heads = np.asarray([hd for hd, _ in rules.rules])
    for k in range(fx.nH):
        c = fx.hcall(k)
        if c["index"].size == 0:
            continue
        q = int(c["r"][0])
        rm_src, rm_dst = g.adj[q][0][c["etr"]], g.adj[q][1][c["etr"]]
        rq_ptr, pos, tot = orc.query_stats(c["h"], c["r"], c["t"], rm_src, rm_dst)
        # candidates per row (over all the relation's rules)
        _, ncand = orc.digests(c["h"], c["r"], rm_src, rm_dst)
        ids = np.nonzero(heads == q)[0]
        np.testing.assert_array_equal(ids, c["index"])
        H = sum(ref.predictor_H_rows(w[ids], pos[rq_ptr[i]:rq_ptr[i + 1]], tot[rq_ptr[i]:rq_ptr[i + 1]], ncand[i])
                for i in range(len(c["h"])))
        np.testing.assert_allclose(H, c["H"], atol=1e-5, rtol=0)
    for k in range(0, fx.ncalls, 3):
        c = fx.call(k)
        if not c["mask"].any() and fx.cfg["feature"] != "bias":
            continue
        q = int(c["r"][0])
        rm = (g.adj[q][0][c["etr"]], g.adj[q][1][c["etr"]]) if c["etr"] is not None else (None, None)
        rq_ptr, pos, tot, cptr, cand, sc = orc.query_stats(c["h"], c["r"], c["t"], rm[0], rm[1], weights=w)
        for i in range(len(c["h"])):
            e, v = cand[cptr[i]:cptr[i + 1]], sc[cptr[i]:cptr[i + 1]]
            if fx.cfg["feature"] == "bias":
                v = v + fx.sd["bias"][e]
            else:
                np.testing.assert_array_equal(np.nonzero(c["mask"][i])[0], e)
            np.testing.assert_allclose(c["score"][i, e], v, atol=1e-5, rtol=1e-6)


@pytest.mark.gpu
def test_predictor_batch_without_candidates_gives_no_rule_gradient():
    """predictors.py:67-71: a batch with no candidate returns `mask + bias`,
    so the rule weights are outside its graph and keep grad None (Adam then
    skips them; a zero gradient would still move them through its moments).
    A batch with candidates gives them a gradient."""
    from rnnlogic_amd import datasets
    from rnnlogic_amd.data import KnowledgeGraph
    from rnnlogic_amd.predictors import Predictor
    dev = torch.device("cuda:0")
    graph = KnowledgeGraph(datasets.materialize("umls"))
    facts = np.asarray(graph.train_facts, dtype=np.int64)
    r0 = int(facts[0, 1])
    model = Predictor(graph, entity_feature="bias")
    model.set_rules([[r0, r0], [r0, r0, r0]])  # rules for one relation only
    model = model.to(dev).train()
    r1 = int(facts[facts[:, 1] != r0][0, 1])
    other = facts[facts[:, 1] == r1][:8]  # one relation without rules
    for rows, want_grad in ((other, False), (facts[facts[:, 1] == r0][:8], True)):
        model.zero_grad(set_to_none=True)
        h, r = torch.from_numpy(rows[:, 0]).to(dev), torch.from_numpy(rows[:, 1]).to(dev)
        score, mask = model(h, r, None)
        assert bool(mask.all())
        (torch.softmax(score, 1)[:, 0].sum()).backward()
        assert (model.rule_weights.grad is not None) == want_grad
        assert model.bias.grad is not None


@pytest.mark.gpu
@pytest.mark.parametrize("overflow", [False, True])
def test_predictor_train_lookahead_is_bit_identical(overflow):
    """TrainerPredictor.train grounds the next batches ahead on a side stream
    (Predictor.prefetch, rnnl_predictor_ground / rnnl_predictor_score): the
    trained weights and the logged losses equal those of the one-call forward
    (prefetch_depth 0) — also when lowered workspace capacities make
    prefetched groundings overflow and fall back to the retried path.  The
    weights are held to a tight tolerance, not bitwise: the backward
    (predictor_backward_kernel) sums each node's count x gradient with fp64
    atomics, whose order may differ between two runs, so a node's gradient
    can differ in its last fp64 bits and, rarely, its fp32 rounding."""
    import io
    import logging
    import random

    from rnnlogic_amd import _native, datasets
    from rnnlogic_amd.data import KnowledgeGraph, TestDataset, TrainDataset, ValidDataset
    from rnnlogic_amd.predictors import Predictor
    from rnnlogic_amd.trainer import TrainerPredictor
    from rnnlogic_amd.utils import set_seed
    dev = torch.device("cuda:0")
    set_seed(1)
    graph = KnowledgeGraph(datasets.materialize("FB15k-237"))
    train_set, valid_set, test_set = TrainDataset(graph, 32), ValidDataset(graph, 32), TestDataset(graph, 32)
    rules = [[int(x) for x in line.split()] for line in open(datasets.rule_file("FB15k-237"))][::4]
    model = Predictor(graph, entity_feature="bias")
    model.set_rules(rules)
    torch.manual_seed(3)
    with torch.no_grad():
        model.rule_weights.normal_(std=0.1)
    init = {k: v.clone() for k, v in model.state_dict().items()}
    rng = (random.getstate(), np.random.get_state(), torch.get_rng_state())
    r2i = [list(x) for x in train_set.r2instances]  # make_batches shuffles these lists in place
    runs = []
    for depth in (0, 2):
        model.load_state_dict(init)
        train_set.r2instances = [list(x) for x in r2i]
        random.setstate(rng[0])
        np.random.set_state(rng[1])
        torch.set_rng_state(rng[2])
        model.prefetch_depth = depth
        model.capacity_scale = 1
        optim = torch.optim.Adam(model.parameters(), lr=1e-3, weight_decay=0)
        solver = TrainerPredictor(model, train_set, valid_set, test_set, optim, gpus=[dev])
        stream = io.StringIO()
        h = logging.StreamHandler(stream)
        root = logging.getLogger()
        old = root.level
        root.addHandler(h)
        root.setLevel(logging.INFO)
        if overflow:
            _native.call("rnnl_debug_capacity", 8192, 8192, 1024)  # 1/8 of the defaults
        try:
            solver.train(batch_per_epoch=60, smoothing=0.2, print_every=20)
            torch.cuda.synchronize()
        finally:
            _native.call("rnnl_debug_capacity", 0, 0, 0)
            root.removeHandler(h)
            root.setLevel(old)
        losses = [line for line in stream.getvalue().splitlines() if line[:1].isdigit()]
        runs.append(({k: v.detach().cpu().clone() for k, v in solver.model.state_dict().items()}, losses,
                     model.capacity_scale))
        model = solver.model
    (w0, l0, s0), (w1, l1, s1) = runs
    assert len(l0) == 3 and l0 == l1
    if overflow:
        assert s0 > 1 and s1 > 1, (s0, s1)
    for k in w0:
        torch.testing.assert_close(w0[k], w1[k], rtol=1e-6, atol=1e-8, msg=k)
