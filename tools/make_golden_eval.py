"""Per-query reference ranks for evaluate() parity (SURVEY §8c vector (5)/(a14)).

Runs the *reference* PredictorPlus (imported from /root/reference/src with the
test-only shims, exactly as tools/make_golden.py does) over the test split of a
case and records, per query row, the reference's filtered rank bounds
(trainer.py:191-203):

    L = #(flagged scores > s_t) + 1,  H = #(flagged scores >= s_t) + 2
    (or L = 1, H = |E| + 1 when t is not a candidate)

plus s_t and `near`, the number of flagged competitors whose score lies within
`TOL` = 1e-4 of s_t — the tolerance the forward is held to, so a HIP rank may
differ from the reference's only by that many positions.  The metrics of the
reference's own formula over these rows (world size 1, no sampler padding) are
stored beside them.  Weights are the seeded state_dict of the same case in
tests/golden/<case>.npz (checked equal here).

Output: tests/golden/eval_<case>.npz.  Long runs: FB15k-237 full test split
(40,932 rows) takes ~25 min on 8 cores; rows are split over worker processes.

Usage: python tools/make_golden_eval.py <case> [--batches N] [--workers W]
"""
import argparse
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as MG  # noqa: E402  (sets up the reference import path + shims)

import torch  # noqa: E402

TOL = 1e-4
_STATE = {}


def _build(name):
    spec = MG.CASES[name]
    dpath = MG.datasets.materialize(spec["data"])
    rules = MG.datasets.rule_file(spec["data"])
    kw = dict(type="lstm", num_layers=3, hidden_dim=16, entity_feature="bias", aggregator="sum", embedding_path=None)
    kw.update(spec["model"])
    if kw.get("embedding_path"):
        kw["embedding_path"] = MG._rotate_dir(spec["data"], kw["embedding_path"])
    MG.R_utils.set_seed(1)
    graph = MG.R_data.KnowledgeGraph(dpath)
    MG.R_data.TrainDataset(graph, 32)
    MG.R_data.ValidDataset(graph, 32)
    test_set = MG.R_data.TestDataset(graph, 32)
    model = MG.R_pred.PredictorPlus(graph, **kw)
    model.set_rules(rules)
    model.eval()
    return graph, test_set, model


def _ranks_of_batch(i):
    graph, test_set, model = _STATE["g"], _STATE["t"], _STATE["m"]
    all_h, all_r, all_t, flag = test_set[i]
    with torch.no_grad():
        score, mask = model(all_h, all_r, None)
    out = []
    for k in range(all_t.numel()):
        t = int(all_t[k])
        if bool(mask[k, t]):
            val = score[k, t]
            s = score[k][flag[k]]
            L = int((s > val).sum()) + 1
            H = int((s >= val).sum()) + 2
            near = int(((s - val).abs() <= TOL).sum())
            st = float(val)
        else:
            L, H, near, st = 1, graph.entity_size + 1, 0, float("nan")
        out.append((int(all_h[k]), int(all_r[k]), t, L, H, near, st))
    return i, out


def _worker(args):
    idx, threads = args
    torch.set_num_threads(threads)
    res = []
    t0 = time.time()
    for j, i in enumerate(idx):
        res.append(_ranks_of_batch(i))
        if j % 50 == 0:
            print("  worker %d: %d/%d batches, %.0f s" % (os.getpid(), j, len(idx), time.time() - t0), flush=True)
    return res


def metrics(rows, expectation=True):
    """The reference formula (trainer.py:207-238) over [h, r, t, L, H] rows."""
    q = {}
    for h, r, t, L, H in rows:
        q[(h, r, t)] = (L, H)
    hit1 = hit3 = hit10 = mr = mrr = 0.0
    for L, H in q.values():
        for rank in range(L, H):
            w = 1.0 / (H - L)
            hit1 += w if rank <= 1 else 0.0
            hit3 += w if rank <= 3 else 0.0
            hit10 += w if rank <= 10 else 0.0
            mr += rank * w
            mrr += w / rank
    n = len(rows)
    return dict(Hit1=hit1 / n, Hit3=hit3 / n, Hit10=hit10 / n, MR=mr / n, MRR=mrr / n)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("case")
    ap.add_argument("--batches", type=int, default=0, help="prefix of test batches (0 = all)")
    ap.add_argument("--workers", type=int, default=4)
    ap.add_argument("--threads", type=int, default=2)
    a = ap.parse_args()
    graph, test_set, model = _build(a.case)
    fx = np.load(os.path.join(MG.OUT, a.case + ".npz"))
    for k, v in model.state_dict().items():
        if "sd/" + k in fx.files:
            assert np.array_equal(v.detach().numpy(), fx["sd/" + k]), k
    _STATE.update(g=graph, t=test_set, m=model)
    nb = len(test_set) if a.batches <= 0 else min(a.batches, len(test_set))
    order = list(range(nb))
    chunks = [order[w::a.workers] for w in range(a.workers)]
    t0 = time.time()
    import multiprocessing as mp
    with mp.get_context("fork").Pool(a.workers) as pool:
        parts = pool.map(_worker, [(c, a.threads) for c in chunks])
    res = dict(x for p in parts for x in p)
    rows = [row for i in range(nb) for row in res[i]]
    arr = np.asarray([r[:6] for r in rows], dtype=np.int64)
    st = np.asarray([r[6] for r in rows], dtype=np.float32)
    m = metrics(arr[:, :5].tolist())
    out = dict(batches=np.int64(nb), rows=arr, s_t=st, tol=np.float64(TOL),
               batch_ptr=np.cumsum([0] + [len(res[i]) for i in range(nb)]).astype(np.int64))
    for k, v in m.items():
        out["metric/" + k] = np.float64(v)
    path = os.path.join(MG.OUT, "eval_%s.npz" % a.case)
    np.savez_compressed(path, **out)
    print("%s: %d batches, %d rows in %.0f s -> %s (%d B); MRR %.6f, rows with near-ties %d" % (
        a.case, nb, len(rows), time.time() - t0, path, os.path.getsize(path), m["MRR"], int((arr[:, 5] > 0).sum())))


if __name__ == "__main__":
    main()
