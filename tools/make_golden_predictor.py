"""Golden vectors for the EM loop's rule-weight Predictor,
made by running the *reference* Python on CPU in the build container
(tools/ref_shims stand in for torch_scatter / easydict; see make_golden.py).

Per case (reference src/predictors.py:17-119, trainer.py:48-143, 145-248):
  cfg                 json: dataset, entity_feature, seed, lr
  sd/<name>           state_dict after the seeded re-draw of the weights (the
                      reference initialises rule_weights and bias to zero,
                      which would make every score identical)
  q<k>/h,r,t,etr      forward inputs (test batches without, train batches with
                      edge removal); q<k>/score, q<k>/mask the outputs
  H<k>/h,r,t,etr      compute_H inputs on train batches; H<k>/H, H<k>/index
  Hall                TrainerPredictor.compute_H over the whole train split
  eval/<metric>       TrainerPredictor.evaluate('test') with these weights
  s<k>/...            the first K Adam steps of TrainerPredictor.train's loop:
                      sampler order, per-step loss, step-0 gradients

Usage:  python tools/make_golden_predictor.py [case ...]
"""
import io
import json
import logging
import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
sys.dont_write_bytecode = True
sys.path[:0] = [os.path.join(HERE, "ref_shims"), "/root/reference/src"]

import torch  # noqa: E402
from torch.utils import data as torch_data  # noqa: E402

import data as R_data  # noqa: E402  (reference src/data.py)
import predictors as R_pred  # noqa: E402
import trainer as R_trainer  # noqa: E402
import utils as R_utils  # noqa: E402

from rnnlogic_amd import datasets  # noqa: E402

OUT = os.path.join(REPO, "tests", "golden")
K = 3
SMOOTHING = 0.2

CASES = {
    "pred_umls_bias": dict(data="umls", feature="bias", test_batches=40, train_batches=6, h_batches=8, lr=0.001),
    "pred_kinship_none": dict(data="kinship", feature="none", test_batches=30, train_batches=6, h_batches=8,
                              lr=0.001),
}


def _draw_weights(model, seed):
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        model.rule_weights.copy_(torch.randn(model.num_rules, generator=g) * 0.5)
        if model.entity_feature == "bias":
            model.bias.copy_(torch.randn(model.num_entities, generator=g) * 0.1)


def _metrics(solver, split):
    stream = io.StringIO()
    h = logging.StreamHandler(stream)
    logging.getLogger().addHandler(h)
    logging.getLogger().setLevel(logging.INFO)
    mrr = solver.evaluate(split, expectation=True)
    logging.getLogger().removeHandler(h)
    vals = {"mrr": mrr}
    for line in stream.getvalue().splitlines():
        for key in ("Hit1", "Hit3", "Hit10", "MR", "MRR", "Data"):
            if line.startswith(key + " ") or line.startswith(key + ":"):
                vals[key] = float(line.split(":")[1])
    return vals


def run_case(name, spec):
    dpath = datasets.materialize(spec["data"])
    rules = datasets.rule_file(spec["data"])
    R_utils.set_seed(1)
    graph = R_data.KnowledgeGraph(dpath)
    train_set = R_data.TrainDataset(graph, 32)
    valid_set = R_data.ValidDataset(graph, 32)
    test_set = R_data.TestDataset(graph, 32)
    model = R_pred.Predictor(graph, entity_feature=spec["feature"])
    model.set_rules(rules)
    _draw_weights(model, 5)
    out = {"cfg": np.array(json.dumps(dict(data=spec["data"], feature=spec["feature"], seed=1, weight_seed=5,
                                           lr=spec["lr"], batch_size=32)))}
    for k, v in model.state_dict().items():
        out["sd/" + k] = v.detach().cpu().numpy().copy()

    rng = random.Random(11)
    sel = sorted(rng.sample(range(len(test_set)), min(spec["test_batches"], len(test_set))))
    calls = [("test", i) for i in sel] + [("train", i) for i in range(spec["train_batches"])]
    k = 0
    with torch.no_grad():
        for split, i in calls:
            if split == "test":
                all_h, all_r, all_t, flag = test_set[i]
                etr = None
            else:
                all_h, all_r, all_t, target, etr = train_set[i]
            score, mask = model(all_h, all_r, etr)
            p = "q%d/" % k
            out[p + "split"] = np.array(split)
            out[p + "h"], out[p + "r"], out[p + "t"] = all_h.numpy(), all_r.numpy(), all_t.numpy()
            out[p + "etr"] = etr.numpy() if etr is not None else np.zeros(0, np.int64)
            out[p + "score"] = score.numpy().astype(np.float32)
            out[p + "mask"] = mask.numpy()
            k += 1
        out["ncalls"] = np.int64(k)
        nh = 0
        for i in range(spec["h_batches"]):
            all_h, all_r, all_t, target, etr = train_set[i]
            H, index = model.compute_H(all_h, all_r, all_t, etr)
            p = "H%d/" % nh
            out[p + "h"], out[p + "r"], out[p + "t"], out[p + "etr"] = (all_h.numpy(), all_r.numpy(), all_t.numpy(),
                                                                        etr.numpy())
            out[p + "H"] = H.numpy() if H is not None else np.zeros(0, np.float32)
            out[p + "index"] = index.numpy() if index is not None else np.zeros(0, np.int64)
            nh += 1
        out["nH"] = np.int64(nh)

    solver = R_trainer.TrainerPredictor(model, train_set, valid_set, test_set, None, gpus=None)
    out["Hall"] = np.asarray(solver.compute_H(print_every=1000000), dtype=np.float32)
    for key, v in _metrics(solver, "test").items():
        out["eval/" + key] = np.float64(v)

    # trainer.py:48-105, first K steps
    optim = torch.optim.Adam(model.parameters(), lr=spec["lr"], weight_decay=0)
    train_set.make_batches()
    sampler = torch_data.DistributedSampler(train_set, 1, 0)
    sampler.set_epoch(0)
    order = list(iter(sampler))[:K]
    out["order"] = np.asarray(order, dtype=np.int64)
    model.train()
    for s, idx in enumerate(order):
        all_h, all_r, all_t, target, etr = train_set[idx]
        target_t = torch.nn.functional.one_hot(all_t, graph.entity_size)
        target = target * SMOOTHING + target_t * (1 - SMOOTHING)
        logits, mask = model(all_h, all_r, etr)
        p = "s%d/" % s
        out[p + "h"], out[p + "r"], out[p + "t"], out[p + "etr"] = (all_h.numpy(), all_r.numpy(), all_t.numpy(),
                                                                    etr.numpy())
        if mask.sum().item() != 0:
            logits = (torch.softmax(logits, dim=1) + 1e-8).log()
            loss = -(logits[mask] * target[mask]).sum() / torch.clamp(target[mask].sum(), min=1)
            loss.backward()
            out[p + "loss"] = np.float64(loss.item())
            if s == 0:
                for n, prm in model.named_parameters():
                    if prm.grad is not None:
                        out["g/" + n] = prm.grad.detach().numpy().copy()
            optim.step()
            optim.zero_grad()
        else:
            out[p + "loss"] = np.float64("nan")
    path = os.path.join(OUT, name + ".npz")
    np.savez_compressed(path, **out)
    print(name, "calls", k, "H", nh, "->", path, os.path.getsize(path), "mrr", out["eval/mrr"],
          "losses", [float(out["s%d/loss" % s]) for s in range(K)])


if __name__ == "__main__":
    os.makedirs(OUT, exist_ok=True)
    torch.set_num_threads(8)
    for n in sys.argv[1:] or list(CASES):
        run_case(n, CASES[n])
