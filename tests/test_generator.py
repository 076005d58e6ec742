"""Rule generator + TrainerGenerator (reference src/generators.py:3-37,
src/trainer.py:291-485) against the reference's own run of the
run_rnnlogic.py sequence on UMLS (tests/golden/em_umls.npz, made by
tools/make_golden_em.py).

CPU: seeded init identical; generator pre-training (losses, weights, global
RNG probes — the batch order comes from the same DataLoader draws);
log_probability, next_relation_log_probability, beam_search, and sample()
(run_rnnlogic.py:68): the same rules per relation, their log-probabilities to
1e-6, the reference's rule order whenever the log-probabilities are bitwise
equal (the reference dedupes through a Python set, whose order follows the
float hashes), and the same global-RNG consumption.
GPU: the generator chain on cuda:0; then one EM iteration started from the
CPU generator's sample() (the fixture's draws come from the CPU RNG) with the
Predictor on the HIP path: predictor losses, MRRs, H scores, posterior, the
M-step's generator losses and final log-probabilities.

Tolerances: the generator and the EM Predictor train in fp32 with a few
dozen Adam steps, so weights and losses are compared at 2e-5 (abs, plus 1e-6
for the reference's 6-decimal log lines); RNG probes, rules and mined-rule
pools are exact.
"""
import numpy as np
import pytest
import torch

import em_chain

W_TOL = 2e-5


def _close(a, b, tol):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    assert a.shape == b.shape, (a.shape, b.shape)
    err = float(np.abs(a - b).max()) if a.size else 0.0
    assert err <= tol, "max |err| %g > %g" % (err, tol)
    return err


def _check_states(got, want, tol):
    assert sorted(got) == sorted(want)
    for k in want:
        _close(got[k], want[k], tol)


def _check_generator_part(z, got, w_tol=W_TOL):
    _check_states(got["gen_init"], em_chain.state(z, "gen_init"), 0.0)
    _close(got["pre_train/loss"], z["pre_train/loss"], w_tol + 1e-6)
    assert np.array_equal(got["probe/pre_train"], z["probe/pre_train"])
    _check_states(got["gen_pre"], em_chain.state(z, "gen_pre"), w_tol)
    _close(got["pre/log_prob"], z["pre/log_prob"], 1e-4)
    _close(got["pre/next_logp"], z["pre/next_logp"], 1e-4)
    import json
    em_chain.check_beam(got["pre/beam"], json.loads(str(z["pre/beam"])), 1e-4)
    assert np.array_equal(got["probe/beam"], z["probe/beam"])


def _check_sample(got, want_json, tol=1e-6):
    """Same rules per head relation (as sets), log p within `tol`, and the
    reference's order when every log p is bitwise equal."""
    import json
    want = json.loads(str(want_json))
    assert len(got) == len(want)
    key = lambda rule: tuple(int(x) for x in rule[:-1])  # noqa: E731
    gmap, wmap = {key(r): r[-1] for r in got}, {key(r): r[-1] for r in want}
    assert len(gmap) == len(got) and set(gmap) == set(wmap)
    _close([gmap[k] for k in wmap], [wmap[k] for k in wmap], tol)
    if all(gmap[k] == wmap[k] for k in wmap):
        assert [key(r) for r in got] == [key(r) for r in want]
        return True
    return False


def test_generator_chain_cpu():
    z, got = em_chain.run(torch.device("cpu"))
    # on the CPU model the fixture was made on, the pre-training reproduces the
    # reference's weights bitwise (same batches, same gathered loss sums, same
    # Adam), hence sample()'s log-probabilities and its set order too; another
    # CPU's vector code rounds the LSTM GEMMs differently (W_TOL then)
    same_cpu = "cpu" in z.files and str(z["cpu"]) == em_chain.cpu_model()
    _check_generator_part(z, got, w_tol=0.0 if same_cpu else W_TOL)
    exact = _check_sample(got["em/sampled"], z["em/sampled"])
    print("sample(): %d rules, bitwise log p and order: %s (fixture CPU: %s)" % (len(got["em/sampled"]), exact,
                                                                               "same" if same_cpu else "other"))
    assert exact or not same_cpu
    assert np.array_equal(got["probe/sample"], z["probe/sample"])


@pytest.mark.gpu
def test_generator_chain_gpu():
    """The generator chain on cuda:0 (sample() draws from the device RNG
    there, so only its contract is checked)."""
    z, got = em_chain.run(torch.device("cuda:0"))
    _check_generator_part(z, got)
    assert len(got["em/sampled"]) > 0


def test_generator_state_dict_names():
    from rnnlogic_amd import datasets
    from rnnlogic_amd.data import KnowledgeGraph
    from rnnlogic_amd.generators import Generator
    z, cfg = em_chain.fixture()
    g = Generator(KnowledgeGraph(datasets.materialize("umls")), **cfg["gen"])
    want = em_chain.state(z, "gen_init")
    assert {k: tuple(v.shape) for k, v in g.state_dict().items()} == {k: v.shape for k, v in want.items()}


def test_rule_dataset_and_table_match_collate():
    """_RuleTable.batch gives the tensors RuleDataset.collate_fn gives."""
    from rnnlogic_amd.data import RuleDataset
    from rnnlogic_amd.trainer import _RuleTable
    rules = [[3, 1, 2, 0.5], [4, 7, -1.25], [1, 2, 3, 4, 2.0], [5, 0.0]]
    ds = RuleDataset(10, rules)
    table = _RuleTable(ds, torch.device("cpu"))
    for idx in ([0, 1, 2, 3], [1, 3], [2], [3, 0]):
        want = RuleDataset.collate_fn([ds[i] for i in idx])
        got = table.batch(torch.tensor(idx))
        for a, b in zip(got, want):
            assert torch.equal(a, b), (idx, a, b)


@pytest.mark.parametrize("batched", [False, True])
def test_sample_shapes_and_dedupe_cpu(batched):
    """The output contract of both draw orders (the reference order is pinned
    by test_generator_chain_cpu): [head, body..., log p], body ≤ max_len, one
    entry per distinct sequence and head, log p = the generator's own
    log_probability of the rule."""
    from rnnlogic_amd import datasets
    from rnnlogic_amd.data import KnowledgeGraph
    from rnnlogic_amd.generators import Generator
    from rnnlogic_amd.trainer import TrainerGenerator
    torch.manual_seed(0)
    g = Generator(KnowledgeGraph(datasets.materialize("umls")), num_layers=1, embedding_dim=16, hidden_dim=16)
    solver = TrainerGenerator(g, gpu=None)
    out = solver.sample(20, 3, batched=batched)
    seen = set()
    for rule in out:
        body = rule[1:-1]
        assert 0 <= rule[0] < g.num_relations and len(body) <= 3
        assert all(0 <= x < g.num_relations for x in body)
        assert tuple(rule) not in seen
        seen.add(tuple(rule))
    # a sequence closed by END before max_len carries END's log p, as log_probability does
    closed = [r for r in out if len(r) - 2 < 3][:50]
    assert closed
    lp = solver.log_probability([list(r[:-1]) for r in closed])
    _close([r[-1] for r in closed], lp, 1e-4)


@pytest.mark.gpu
def test_em_iteration_gpu():
    """run_rnnlogic.py:45-91 through the package vs the reference run: the
    generator on the CPU (its sample() must draw the fixture's rules), the
    EM iteration's Predictor on cuda:0."""
    z, got = em_chain.run(torch.device("cuda:0"), em=True, gen_device=torch.device("cpu"))
    _check_generator_part(z, got)
    # bitwise on the fixture's CPU model (test_generator_chain_cpu); on another
    # CPU the pre-trained weights differ in the last bits, so log p does too
    same_cpu = "cpu" in z.files and str(z["cpu"]) == em_chain.cpu_model()
    _check_sample(got["em/sampled"], z["em/sampled"], 1e-6 if same_cpu else 1e-5)
    assert np.array_equal(got["probe/sample"], z["probe/sample"])
    err = lambda a, b: float(np.abs(np.asarray(a, np.float64) - np.asarray(b, np.float64)).max())  # noqa: E731
    print("EM errors: train_loss %.3g, pred_trained %s, H %.3g, posterior %.3g, m_step loss %.3g, gen_m %s" % (
        err(got["em/train_loss"], z["em/train_loss"]),
        {k: "%.3g" % err(v, em_chain.state(z, "pred_trained")[k]) for k, v in got["pred_trained"].items()},
        err(got["em/H"], z["em/H"]), err(got["em/posterior"], z["em/posterior"]),
        err(got["m_step/loss"], z["m_step/loss"]),
        max(err(v, em_chain.state(z, "gen_m")[k]) for k, v in got["gen_m"].items())))
    _check_states(got["pred_init"], em_chain.state(z, "pred_init"), 0.0)
    _close(got["em/train_loss"], z["em/train_loss"], W_TOL + 1e-6)
    assert np.array_equal(got["probe/em_train"], z["probe/em_train"])
    _check_states(got["pred_trained"], em_chain.state(z, "pred_trained"), W_TOL)
    print("EM: valid MRR %.9f (ref %.9f), test MRR %.9f (ref %.9f)" % (
        got["em/valid_mrr"], z["em/valid_mrr"], got["em/test_mrr"], z["em/test_mrr"]))
    _close(got["em/valid_mrr"], z["em/valid_mrr"], 1e-4)
    _close(got["em/test_mrr"], z["em/test_mrr"], 1e-4)
    _close(got["em/H"], z["em/H"], 1e-5)
    _close(got["em/posterior"], z["em/posterior"], 1e-5)
    assert np.array_equal(got["probe/em_H"], z["probe/em_H"])
    _close(got["m_step/loss"], z["m_step/loss"], W_TOL + 1e-6)
    assert np.array_equal(got["probe/m_step"], z["probe/m_step"])
    _close(got["m_step/log_prob"], z["m_step/log_prob"], 1e-4)
    _check_states(got["gen_m"], em_chain.state(z, "gen_m"), W_TOL)


def test_padded_rule_batch_gives_the_same_loss_cpu():
    """TrainerGenerator.train on a GPU pads every batch to batch_size rows
    (weight 0) and the table's full width (one LSTM shape); the loss is the
    unpadded batch's."""
    from rnnlogic_amd import datasets
    from rnnlogic_amd.data import KnowledgeGraph, RuleDataset
    from rnnlogic_amd.generators import Generator
    from rnnlogic_amd.trainer import _RuleTable
    torch.manual_seed(0)
    graph = KnowledgeGraph(datasets.materialize("umls"))
    g = Generator(graph, num_layers=1, embedding_dim=16, hidden_dim=16)
    mined = [[int(x) for x in line.split()] for line in open(datasets.rule_file("umls"))][:300]
    ds = RuleDataset(graph.relation_size, [r + [0.1 + (i % 7)] for i, r in enumerate(mined)])
    table = _RuleTable(ds, torch.device("cpu"))
    idx = torch.tensor([5, 17, 2, 250, 99])
    zero = lambda n: (torch.zeros(1, n, 16), torch.zeros(1, n, 16))  # noqa: E731
    a = table.batch(idx)
    b = table.batch(idx, pad_rows=16)
    assert b[0].shape == (16, table.inputs.size(1))
    with torch.no_grad():
        la = g.loss(*a, zero(a[0].size(0)))
        lb = g.loss(*b, zero(16))
    assert abs(float(la) - float(lb)) <= 1e-6 * max(1.0, abs(float(la)))
