"""Golden vectors for the run_predictorplus.py flow (SURVEY §8(c) vector (5),
VERDICT r1 item 9): the reference's own training + evaluation loop
(src/run_predictorplus.py:45-68 with the FB15k-237_predictorplus.yaml
predictor settings: PredictorPlus(lstm, 3, 16, bias, sum), Adam lr 0.005,
smoothing 0.2, expectation ranks) on UMLS, seed 1, for ITERS iterations of
BATCHES training batches each (batch_per_epoch), run on CPU in this container
by importing the reference (tools/ref_shims stand in for torch_scatter /
easydict, as in tools/make_golden.py).

Stored in tests/golden/flow_umls.npz:
  sd0/<name>             initial state_dict (equals the package's seeded init)
  sd1/<name>             state_dict after the last iteration
  it<k>/loss             per-step training losses of iteration k (the
                         reference's log lines with print_every=1, 6 decimals)
  it<k>/valid_mrr, it<k>/test_mrr   evaluate()'s return values
  final/<split>/rows     per query of the trained model: h, r, t, L, H, near
                         (the rank bounds of trainer.py:191-203 and the number
                         of flagged competitors within 1e-4 of the target's
                         score), TestDataset / ValidDataset batch order
  final/<split>/metric/<k>   the reference formula over those rows
  it<k>/<split>/...      per iteration k, every valid / test query's record
                         of tools/make_golden_eval.py (`batch_records`: L, H,
                         near_w over FLOW_WINDOWS, probe entities and their
                         reference scores), so that tests/test_gpu_flow.py
                         holds each iteration's ranks and MRR to the score
                         error it measures (tests/rank_parity.py)

Usage: python tools/make_golden_flow.py
"""
import logging
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)
sys.dont_write_bytecode = True
sys.path[:0] = [os.path.join(HERE, "ref_shims"), "/root/reference/src"]

import torch  # noqa: E402

import data as R_data  # noqa: E402  (reference src/data.py)
import predictors as R_pred  # noqa: E402
import trainer as R_trainer  # noqa: E402
import utils as R_utils  # noqa: E402

from make_golden_eval import WINDOWS, batch_records, metrics  # noqa: E402
from rnnlogic_amd import datasets  # noqa: E402

OUT = os.path.join(REPO, "tests", "golden", "flow_umls.npz")
ITERS = 2
BATCHES = 20
TOL = 1e-4
# trained weights differ from the reference's by ~1e-5 after 20 Adam steps, so the
# score error is wider than a fixed-weight forward's: windows up to 5e-3
FLOW_WINDOWS = WINDOWS + (2e-4, 5e-4, 1e-3, 2e-3, 5e-3)


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


def ranks(model, ds, graph):
    rows = []
    model.eval()
    with torch.no_grad():
        for i in range(len(ds)):
            all_h, all_r, all_t, flag = ds[i]
            score, mask = model(all_h, all_r, None)
            for k in range(all_t.numel()):
                t = int(all_t[k])
                if bool(mask[k, t]):
                    val = score[k, t]
                    s = score[k][flag[k]]
                    L, H = int((s > val).sum()) + 1, int((s >= val).sum()) + 2
                    near = int(((s - val).abs() <= TOL).sum())
                else:
                    L, H, near = 1, graph.entity_size + 1, 0
                rows.append((int(all_h[k]), int(all_r[k]), t, L, H, near))
    return np.asarray(rows, dtype=np.int64)


def records(model, ds, graph, out, prefix):
    """Per-row parity records of one split (make_golden_eval.batch_records)."""
    rows, ptr = [], [0]
    model.eval()
    with torch.no_grad():
        for i in range(len(ds)):
            all_h, all_r, all_t, flag = ds[i]
            score, mask = model(all_h, all_r, None)
            rows += batch_records(score, mask, all_h, all_r, all_t, flag, graph.entity_size,
                                  np.random.RandomState(1000 + i), FLOW_WINDOWS)
            ptr.append(len(rows))
    out[prefix + "rows"] = np.asarray([r[:6] for r in rows], dtype=np.int64)
    out[prefix + "s_t"] = np.asarray([r[6] for r in rows], dtype=np.float32)
    out[prefix + "near_w"] = np.stack([r[7] for r in rows])
    out[prefix + "probe_ent"] = np.stack([r[8] for r in rows]).astype(np.int32)
    out[prefix + "probe_score"] = np.stack([r[9] for r in rows])
    out[prefix + "batch_ptr"] = np.asarray(ptr, dtype=np.int64)
    out[prefix + "windows"] = np.asarray(FLOW_WINDOWS, np.float64)


def main():
    torch.set_num_threads(8)
    R_utils.set_seed(1)
    graph = R_data.KnowledgeGraph(datasets.materialize("umls"))
    train_set = R_data.TrainDataset(graph, 32)
    valid_set = R_data.ValidDataset(graph, 32)
    test_set = R_data.TestDataset(graph, 32)
    model = R_pred.PredictorPlus(graph, type="lstm", num_layers=3, hidden_dim=16, entity_feature="bias",
                                 aggregator="sum", embedding_path=None)
    model.set_rules(datasets.rule_file("umls"))
    out = {"sd0/" + k: v.detach().numpy().copy() for k, v in model.state_dict().items()}
    optim = torch.optim.Adam(model.parameters(), lr=0.005, weight_decay=0)
    solver = R_trainer.TrainerPredictor(model, train_set, valid_set, test_set, optim, gpus=None)
    handler = _Losses()
    logging.getLogger().addHandler(handler)
    logging.getLogger().setLevel(logging.INFO)
    for k in range(ITERS):
        handler.vals = []
        solver.train(batch_per_epoch=BATCHES, smoothing=0.2, print_every=1)
        out["it%d/loss" % k] = np.asarray(handler.vals, dtype=np.float64)
        out["it%d/valid_mrr" % k] = np.float64(solver.evaluate("valid", expectation=True))
        out["it%d/test_mrr" % k] = np.float64(solver.evaluate("test", expectation=True))
        for name, ds in (("valid", valid_set), ("test", test_set)):
            records(model, ds, graph, out, "it%d/%s/" % (k, name))
        print("iteration %d: %d steps, valid MRR %.6f, test MRR %.6f" % (
            k, len(handler.vals), out["it%d/valid_mrr" % k], out["it%d/test_mrr" % k]), flush=True)
    for k, v in model.state_dict().items():
        out["sd1/" + k] = v.detach().numpy().copy()
    for name, ds in (("valid", valid_set), ("test", test_set)):
        rows = ranks(model, ds, graph)
        out["final/%s/rows" % name] = rows
        for key, val in metrics(rows[:, :5].tolist()).items():
            out["final/%s/metric/%s" % (name, key)] = np.float64(val)
    np.savez_compressed(OUT, **out)
    print(OUT, os.path.getsize(OUT))


if __name__ == "__main__":
    main()
