"""HIP path parity (runs on the MI355X box).

Every forward goes through the C-ABI library (rnnlogic_amd/_build/
librnnlogic_hip.so).  Checks, against the reference's own outputs
(tests/golden) and the C oracle (oracle/ground_oracle.c):
  * entity scores within 1e-4 (fp32, abs) and identical masks;
  * exact integer parity of the per-rule path counts, through the
    order-independent digest of (candidate, sum of counts, rule fingerprint)
    — on the fixture batches and on the FULL synthetic FB15k-237 test split;
  * candidate counts per query;
  * RotatE known-answer MRRs of the shipped embeddings (train.log values).
"""
import numpy as np
import pytest
import torch

from conftest import ALL_CASES, Fixture
from oracle import ground_c
from oracle import reference_np as ref

pytestmark = pytest.mark.gpu

TOL = 1e-4  # north_star: entity scores within 1e-4 fp32

_graphs, _oracles = {}, {}


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def graph_for(path):
    from rnnlogic_amd.data import KnowledgeGraph
    if path not in _graphs:
        _graphs[path] = KnowledgeGraph(path)
    return _graphs[path]


def oracle_for(fx):
    p = fx.dataset_path()
    if p not in _oracles:
        g = ref.Graph(p)
        rules = ref.Rules(fx.rule_path(), g.relation_size)
        cg = ground_c.CGraph(g.entity_size, g.relation_size, g.train_facts)
        _oracles[p] = (g, ground_c.Oracle(cg, rules.rules, g.relation_size))
    return _oracles[p]


def build_model(fx, dev):
    from rnnlogic_amd.predictors import PredictorPlus
    graph = graph_for(fx.dataset_path())
    cfg = dict(fx.cfg["model"])
    model = PredictorPlus(graph, embedding_path=fx.rotate_path(), **cfg)
    model.set_rules(fx.rule_path())
    sd = {k: torch.from_numpy(v) for k, v in fx.sd.items()}
    missing, unexpected = model.load_state_dict(sd, strict=False)
    assert not unexpected and all(k.startswith("RotatE.") for k in missing), (missing, unexpected)
    return model.to(dev).eval()


@pytest.mark.parametrize("case", ALL_CASES)
def test_forward_matches_reference(case, dev):
    fx = Fixture(case)
    model = build_model(fx, dev)
    worst = 0.0
    for k in range(fx.ncalls):
        c = fx.call(k)
        h = torch.from_numpy(c["h"]).to(dev)
        r = torch.from_numpy(c["r"]).to(dev)
        etr = torch.from_numpy(c["etr"]).to(dev) if c["etr"] is not None else None
        with torch.no_grad():
            score, mask = model(h, r, etr)
        score = score.cpu().numpy()
        np.testing.assert_array_equal(mask.cpu().numpy(), c["mask"], err_msg="%s call %d mask" % (case, k))
        want = c["score"]
        fin = np.isfinite(want)
        np.testing.assert_array_equal(np.isfinite(score), fin)
        np.testing.assert_array_equal(score[~fin], want[~fin])
        if fin.any():
            err = float(np.abs(score[fin] - want[fin]).max())
            worst = max(worst, err)
            assert err <= TOL, "%s call %d: max |score - reference| = %g" % (case, k, err)
    print("%s: %d calls, max abs err %.3g" % (case, fx.ncalls, worst))


@pytest.mark.parametrize("case", ALL_CASES)
def test_path_count_digests(case, dev):
    """Exact integer parity of the grounding for every fixture batch."""
    fx = Fixture(case)
    model = build_model(fx, dev)
    g, orc = oracle_for(fx)
    for k in range(fx.ncalls):
        c = fx.call(k)
        rs = rd = None
        if c["etr"] is not None:
            q = int(c["r"][0])
            heads, tails = g.adj[q]
            rs, rd = heads[c["etr"]], tails[c["etr"]]
        want_d, want_n = orc.digests(c["h"], c["r"], rs, rd, threads=4)
        h = torch.from_numpy(c["h"]).to(dev)
        r = torch.from_numpy(c["r"]).to(dev)
        etr = torch.from_numpy(c["etr"]).to(dev) if c["etr"] is not None else None
        dig = torch.zeros(len(h), dtype=torch.int64, device=dev)
        with torch.no_grad():
            _, _, ncand = model.forward_rows(h, r, etr, return_ncand=True, digest=dig)
        np.testing.assert_array_equal(ncand.cpu().numpy(), want_n)
        np.testing.assert_array_equal(dig.cpu().numpy().view(np.uint64), want_d)


def test_full_fb15k237_test_split_digests(dev):
    """Size-independent property at full size: every one of the 40,932 test
    queries of the synthetic FB15k-237 graph grounds to exactly the oracle's
    path counts (digest + candidate count), in one multi-batch launch."""
    fx = Fixture("fb_lstm_sum_bias")
    model = build_model(fx, dev)
    g, orc = oracle_for(fx)
    test = np.asarray(g.test_facts, dtype=np.int64)
    want_d, want_n = orc.digests(test[:, 0], test[:, 1])
    h = torch.from_numpy(test[:, 0]).to(dev)
    r = torch.from_numpy(test[:, 1]).to(dev)
    got_d, got_n = [], []
    for s in range(0, len(test), 8192):
        dig = torch.zeros(min(8192, len(test) - s), dtype=torch.int64, device=dev)
        with torch.no_grad():
            _, _, n = model.forward_rows(h[s:s + 8192], r[s:s + 8192], None, return_ncand=True, digest=dig)
        got_d.append(dig.cpu().numpy().view(np.uint64))
        got_n.append(n.cpu().numpy())
    np.testing.assert_array_equal(np.concatenate(got_n), want_n)
    np.testing.assert_array_equal(np.concatenate(got_d), want_d)


@pytest.mark.parametrize("data,dim,mrr", [("umls", 200, 0.659847), ("umls", 50, 0.344034),
                                          ("kinship", 1000, 0.637454)])
def test_rotate_known_answer_mrr(data, dim, mrr, dev):
    """RotatE HIP scorer reproduces the shipped train.log test MRR (KAT)."""
    from rnnlogic_amd import datasets
    from rnnlogic_amd.embedding import RotatE
    g = ref.Graph(datasets.materialize(data))
    rot = RotatE(datasets.rotate_path(data, dim)).to(dev)
    R = g.relation_size
    test = np.asarray(g.test_facts)
    allt = set(g.train_facts) | set(g.valid_facts) | set(g.test_facts)
    rr = []
    for side in ("tail", "head"):
        hh = test[:, 0] if side == "tail" else test[:, 2]
        rel = test[:, 1] if side == "tail" else test[:, 1] + R
        tt = test[:, 2] if side == "tail" else test[:, 0]
        with torch.no_grad():
            s = rot(torch.from_numpy(hh).to(dev), torch.from_numpy(rel).to(dev)).cpu().numpy()
        for k in range(len(test)):
            row = s[k].copy()
            h0, r0, t0 = (int(x) for x in test[k])
            for e in range(g.entity_size):
                trip = (h0, r0, e) if side == "tail" else (e, r0, t0)
                if e != tt[k] and trip in allt:
                    row[e] = -np.inf
            rr.append(1.0 / (1 + int((row > row[tt[k]]).sum())))
    assert abs(float(np.mean(rr)) - mrr) < 5e-7, (float(np.mean(rr)), mrr)
