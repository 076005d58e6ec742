"""Evaluation parity on the GPU.

* DeviceEvalBatches (rows + filter flags by rnnl_filter_flags) equals
  ValidDataset / TestDataset.__getitem__ (reference src/data.py:250-255,
  287-291).
* The reference's own scores and masks (tests/golden/umls_lstm_sum_bias.npz)
  through TrainerPredictor.filtered_ranks on the device and rank_metrics give
  the reference's evaluate() metrics to 1e-12.
* Per-query ranks of the HIP forward against the reference's per-query
  (L, H) (tests/golden/eval_<case>.npz, tools/make_golden_eval.py): a query's
  bounds may differ only by the number of flagged competitors whose reference
  score lies within 1e-4 (the forward's score tolerance) of the target's,
  and MRR / Hits deltas are logged.
"""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, Fixture

pytestmark = pytest.mark.gpu

EVAL_CASES = sorted(f[5:-4] for f in os.listdir(GOLDEN) if f.startswith("eval_") and f.endswith(".npz"))


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def _datasets(data):
    from rnnlogic_amd import datasets
    from rnnlogic_amd.data import KnowledgeGraph, TestDataset, TrainDataset, ValidDataset
    from rnnlogic_amd.utils import set_seed
    set_seed(1)
    graph = KnowledgeGraph(datasets.materialize(data))
    return graph, TrainDataset(graph, 32), ValidDataset(graph, 32), TestDataset(graph, 32)


@pytest.mark.parametrize("data", ["umls", "FB15k-237"])
def test_device_eval_batches_match_dataset(data, dev):
    from rnnlogic_amd.data import DeviceEvalBatches
    graph, _, valid_set, test_set = _datasets(data)
    for ds in (valid_set, test_set):
        db = DeviceEvalBatches(ds, dev)
        idx = list(range(0, len(ds), max(1, len(ds) // 40)))[:40]
        for i in idx:
            for w, g in zip(ds[i], db[i]):
                np.testing.assert_array_equal(g.cpu().numpy(), w.numpy())
        # many batches in one launch == their concatenation
        h, r, t, flag = db.rows(idx)
        want = [torch.cat(x) for x in zip(*[ds[i] for i in idx])]
        for w, g in zip(want, (h, r, t, flag)):
            np.testing.assert_array_equal(g.cpu().numpy(), w.numpy())


def test_reference_scores_through_device_ranks(dev):
    """the reference's logits and masks through the device ranking
    and the metric code reproduce its evaluate() metrics exactly."""
    from rnnlogic_amd.trainer import TrainerPredictor
    fx = Fixture("umls_lstm_sum_bias")
    graph, _, _, test_set = _datasets("umls")
    table = {}
    for k in range(fx.ncalls):
        c = fx.call(k)
        if c["split"] == "test":
            table[(int(c["r"][0]),) + tuple(int(x) for x in c["h"])] = (c["score"], c["mask"])
    ranks = []
    # the reference evaluate()'s DistributedSampler order: a (h, r, t) that
    # occurs in two batches keeps its later row, and the reference's scores
    # of one (h, r) may differ in the last bits between batches
    for i in torch.utils.data.DistributedSampler(test_set, 1, 0):
        h, r, t, flag = test_set[i]
        s, m = table[(int(r[0]),) + tuple(int(x) for x in h)]
        L, H = TrainerPredictor.filtered_ranks(torch.from_numpy(s).to(dev), torch.from_numpy(m).to(dev),
                                               flag.to(dev), t.to(dev), graph.entity_size)
        ranks.append(torch.stack([h.to(dev), r.to(dev), t.to(dev), L, H], 1))
    m = TrainerPredictor.rank_metrics(torch.cat(ranks).cpu().numpy().tolist(), True)
    # eval/mrr is evaluate()'s return value (float64); the other metrics are
    # the reference's log lines, printed to 6 decimals
    assert abs(m["MRR"] - float(fx.z["eval/mrr"])) <= 1e-12
    for key in ("MRR", "Hit1", "Hit3", "Hit10", "MR"):
        assert abs(m[key] - float(fx.z["eval/" + key])) <= 5e-7, key


@pytest.mark.parametrize("case", EVAL_CASES)
def test_per_query_ranks_vs_reference(case, dev):
    from rnnlogic_amd import datasets
    from rnnlogic_amd.data import DeviceEvalBatches
    from rnnlogic_amd.predictors import PredictorPlus
    from rnnlogic_amd.trainer import TrainerPredictor
    z = np.load(os.path.join(GOLDEN, "eval_%s.npz" % case))
    fx = Fixture(case)
    graph, _, _, test_set = _datasets(fx.cfg["data"])
    model = PredictorPlus(graph, embedding_path=fx.rotate_path(), **fx.cfg["model"])
    model.set_rules(datasets.rule_file(fx.cfg["data"]))
    # the fixture's state_dict omits the RotatE tables (loaded from embedding_path)
    missing, unexpected = model.load_state_dict({k: torch.from_numpy(v) for k, v in fx.sd.items()}, strict=False)
    assert not unexpected and all(k.startswith("RotatE.") for k in missing), (missing, unexpected)
    model = model.to(dev).eval()
    nb = int(z["batches"])
    want = z["rows"]
    h, r, t, flag = DeviceEvalBatches(test_set, dev).rows(list(range(nb)))
    np.testing.assert_array_equal(torch.stack([h, r, t], 1).cpu().numpy(), want[:, :3])
    with torch.no_grad():
        logits, mask = model.forward_rows(h, r, None)
    L, H = TrainerPredictor.filtered_ranks(logits, mask, flag, t, graph.entity_size)
    L, H = L.cpu().numpy(), H.cpu().numpy()
    dL, dH = np.abs(L - want[:, 3]), np.abs(H - want[:, 4])
    near = want[:, 5]
    diff = (dL > 0) | (dH > 0)
    bad = np.nonzero((dL > near) | (dH > near))[0]
    got_m = TrainerPredictor.rank_metrics(np.stack([want[:, 0], want[:, 1], want[:, 2], L, H], 1).tolist(), True)
    msg = "%s: %d rows, %d with differing (L, H) (all within their near-tie counts: %s); " % (
        case, len(want), int(diff.sum()), "yes" if len(bad) == 0 else "NO")
    msg += ", ".join("%s delta %.3g" % (k, got_m[k] - float(z["metric/" + k]))
                     for k in ("MRR", "Hit1", "Hit3", "Hit10", "MR"))
    print(msg)
    assert len(bad) == 0, (bad[:10], L[bad[:10]], H[bad[:10]], want[bad[:10]])
    if not diff.any():
        assert abs(got_m["MRR"] - float(z["metric/MRR"])) <= 1e-12
