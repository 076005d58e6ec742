"""The run_predictorplus.py flow end to end on the GPU:
reference src/run_predictorplus.py:45-68 — seeded model, Adam, ITERS x
(TrainerPredictor.train(batch_per_epoch) -> evaluate('valid') ->
evaluate('test')) — through the package on UMLS, against the reference's own
run of the same flow in this container (tests/golden/flow_umls.npz, made by
tools/make_golden_flow.py).

Checked: the seeded initial weights (exact), every training loss (the
reference's 6-decimal log lines), the trained weights, and after every
iteration every valid/test query's filtered rank bounds (L, H) and
evaluate()'s MRR, held to the score error measured at that iteration
(tests/rank_parity.py: a row moves only by the competitors within 2 eps of
its target, exactly accounted where the probes cover them; |dMRR| within the
per-row bound, and evaluate()'s own return value equal to the metric over the
device ranks).  Observed deltas are printed.
"""
import logging
import os

import numpy as np
import pytest
import torch

import rank_parity
from conftest import GOLDEN

# trained weights differ from the reference's by <= 1e-4 (asserted), so the
# per-batch score error is wider than at fixed weights
EPS_MAX = 2.5e-3


def _ranks_vs_reference(model, ds, z, prefix, dev, graph):
    from rnnlogic_amd.data import DeviceEvalBatches
    from rnnlogic_amd.trainer import TrainerPredictor
    want = z[prefix + "rows"]
    h, r, t, flag = DeviceEvalBatches(ds, dev).rows(list(range(len(ds))))
    np.testing.assert_array_equal(torch.stack([h, r, t], 1).cpu().numpy(), want[:, :3])
    with torch.no_grad():
        logits, mask = model.forward_rows(h, r, None)
    L, H = TrainerPredictor.filtered_ranks(logits, mask, flag, t, graph.entity_size)
    L, H = L.cpu().numpy(), H.cpu().numpy()
    n = len(want)
    pe = z[prefix + "probe_ent"].astype(np.int64)
    rows_i = torch.arange(n, device=dev)
    hip_t = logits[rows_i, t].cpu().numpy().astype(np.float64)
    hip_p = logits.gather(1, torch.from_numpy(np.maximum(pe, 0)).to(dev)).cpu().numpy().astype(np.float64)
    hit = mask[rows_i, t].cpu().numpy()
    rep = rank_parity.check(want, L, H, hip_t, hip_p, hit, z[prefix + "s_t"].astype(np.float64),
                            z[prefix + "probe_score"].astype(np.float64), pe, z[prefix + "near_w"],
                            z[prefix + "windows"], z[prefix + "batch_ptr"], eps_max=EPS_MAX, nclose=pe.shape[1] - 4)
    return rep, np.stack([want[:, 0], want[:, 1], want[:, 2], L, H], 1)

pytestmark = pytest.mark.gpu


class _Losses(logging.Handler):
    def __init__(self):
        super().__init__()
        self.vals = []

    def emit(self, record):
        parts = record.getMessage().split()
        if len(parts) == 4:
            try:
                self.vals.append(float(parts[2]))
            except ValueError:
                pass


def test_run_predictorplus_flow_matches_reference():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from rnnlogic_amd import datasets
    from rnnlogic_amd.data import DeviceEvalBatches, KnowledgeGraph, TestDataset, TrainDataset, ValidDataset  # noqa
    from rnnlogic_amd.predictors import PredictorPlus
    from rnnlogic_amd.trainer import TrainerPredictor
    from rnnlogic_amd.utils import set_seed
    z = np.load(os.path.join(GOLDEN, "flow_umls.npz"))
    iters = len([k for k in z.files if k.endswith("/valid_mrr")])
    set_seed(1)
    graph = KnowledgeGraph(datasets.materialize("umls"))
    train_set, valid_set, test_set = TrainDataset(graph, 32), ValidDataset(graph, 32), TestDataset(graph, 32)
    model = PredictorPlus(graph, type="lstm", num_layers=3, hidden_dim=16, entity_feature="bias", aggregator="sum",
                          embedding_path=None)
    model.set_rules(datasets.rule_file("umls"))
    for k, v in model.state_dict().items():
        np.testing.assert_array_equal(v.numpy(), z["sd0/" + k], err_msg=k)
    optim = torch.optim.Adam(model.parameters(), lr=0.005, weight_decay=0)
    solver = TrainerPredictor(model, train_set, valid_set, test_set, optim, gpus=[0])
    handler = _Losses()
    root = logging.getLogger()
    root.addHandler(handler)
    level = root.level
    root.setLevel(logging.INFO)
    report = []
    dev = torch.device("cuda:0")
    try:
        for it in range(iters):
            handler.vals = []
            solver.train(batch_per_epoch=len(z["it%d/loss" % it]), smoothing=0.2, print_every=1)
            want = z["it%d/loss" % it]
            got = np.asarray(handler.vals)
            assert got.shape == want.shape
            dl = float(np.abs(got - want).max())
            assert dl <= 2e-5, (it, got, want)
            vm, tm = solver.evaluate("valid"), solver.evaluate("test")
            report.append("iteration %d: max |loss delta| %.2g" % (it, dl))
            for name, ds, got in (("valid", valid_set, vm), ("test", test_set, tm)):
                rep, rows = _ranks_vs_reference(model, ds, z, "it%d/%s/" % (it, name), dev, graph)
                want_mrr = float(z["it%d/%s_mrr" % (it, name)])
                # evaluate()'s return value is the metric over these ranks
                m = TrainerPredictor.rank_metrics(rows.tolist(), True)
                assert abs(got - m["MRR"]) <= 1e-12, (it, name, got, m["MRR"])
                assert abs((got - want_mrr) - rep["d_mrr"]) <= 1e-10, (it, name, got - want_mrr, rep["d_mrr"])
                report.append("  %s: MRR delta %.3g; %s" % (name, got - want_mrr, rank_parity.describe(rep)))
    finally:
        root.removeHandler(handler)
        root.setLevel(level)
    sd = {k: v.detach().cpu().numpy() for k, v in model.state_dict().items()}
    wd = max(float(np.abs(sd[k] - z["sd1/" + k]).max()) for k in sd)
    assert wd <= 1e-4, wd
    report.append("trained weights: max |delta| %.3g" % wd)
    for name, ds in (("valid", valid_set), ("test", test_set)):
        want = z["final/%s/rows" % name]
        h, r, t, flag = DeviceEvalBatches(ds, dev).rows(list(range(len(ds))))
        np.testing.assert_array_equal(torch.stack([h, r, t], 1).cpu().numpy(), want[:, :3])
        with torch.no_grad():
            logits, mask = model.forward_rows(h, r, None)
        L, H = TrainerPredictor.filtered_ranks(logits, mask, flag, t, graph.entity_size)
        L, H = L.cpu().numpy(), H.cpu().numpy()
        dL, dH = np.abs(L - want[:, 3]), np.abs(H - want[:, 4])
        bad = np.nonzero((dL > want[:, 5]) | (dH > want[:, 5]))[0]
        m = TrainerPredictor.rank_metrics(np.stack([want[:, 0], want[:, 1], want[:, 2], L, H], 1).tolist(), True)
        report.append("%s: %d rows, %d with differing (L, H), all within near-ties: %s; " % (
            name, len(want), int(((dL > 0) | (dH > 0)).sum()), "yes" if len(bad) == 0 else "NO") + ", ".join(
            "%s delta %.3g" % (k, m[k] - float(z["final/%s/metric/%s" % (name, k)]))
            for k in ("MRR", "Hit1", "Hit3", "Hit10", "MR")))
        assert len(bad) == 0, (name, bad[:10], L[bad[:10]], H[bad[:10]], want[bad[:10]])
    print("\n".join(report))
