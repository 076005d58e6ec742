"""One EM iteration of run_rnnlogic.py (src/run_rnnlogic.py:56-91, config
config/FB15k-237.yaml) on FB15k-237 through the package, timed per phase on
one GPU (BASELINE.json config 5; synthetic train graph, real test split).

Phases, with the config's settings unless noted:
  pre-train   TrainerGenerator.train over a rule dataset (rnnlogic_rules.txt with
              synthetic weights: FB's mined_rules.txt needs the real train.txt),
              PRE_EPOCHS of the config's 10,000 epochs (per-epoch time reported)
  sample      TrainerGenerator.sample(100, 3): 100 rules per relation
  p-train     TrainerPredictor.train with the sampled rules (Predictor, bias):
              TRAIN_BATCHES of the train split's batches (the config runs all)
  evaluate    evaluate('valid') + evaluate('test')
  E-step      TrainerPredictor.compute_H over every train batch
  M-step      TrainerGenerator.train(num_epoch=100) on the posterior-weighted rules
Writes one JSON line (stdout): per-phase seconds, rates, and the full-iteration
time with the capped phases scaled to the config's counts.

Usage (GPU box): python tools/em_iteration_fb.py [PRE_EPOCHS] [TRAIN_BATCHES]
"""
import contextlib
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rnnlogic_amd import datasets  # noqa: E402
from rnnlogic_amd.data import KnowledgeGraph, RuleDataset, TestDataset, TrainDataset, ValidDataset  # noqa: E402
from rnnlogic_amd.generators import Generator  # noqa: E402
from rnnlogic_amd.predictors import Predictor  # noqa: E402
from rnnlogic_amd.trainer import TrainerGenerator, TrainerPredictor  # noqa: E402
from rnnlogic_amd.utils import set_seed  # noqa: E402

PRE_EPOCHS = int(sys.argv[1]) if len(sys.argv) > 1 else 500
TRAIN_BATCHES = int(sys.argv[2]) if len(sys.argv) > 2 else 2000


def timed(fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = fn()
    torch.cuda.synchronize()
    return out, time.perf_counter() - t0


def main():
    dev = torch.device("cuda:0")
    res = {"workload": "FB15k-237 (seeded synthetic train graph), config/FB15k-237.yaml EM iteration on 1 GPU"}
    with contextlib.redirect_stdout(sys.stderr):
        set_seed(1)
        graph = KnowledgeGraph(datasets.materialize("FB15k-237"))
        train_set = TrainDataset(graph, 32)
        valid_set = ValidDataset(graph, 32)
        test_set = TestDataset(graph, 32)
    rules = [[int(x) for x in line.split()] for line in open(datasets.rule_file("FB15k-237"))]
    dataset = RuleDataset(graph.relation_size, [r + [0.25 * ((i * 37) % 11) - 1.0] for i, r in enumerate(rules)])
    gen = Generator(graph, num_layers=1, embedding_dim=512, hidden_dim=256)
    solver_g = TrainerGenerator(gen, gpu=0)
    _, t = timed(lambda: solver_g.train(dataset, num_epoch=PRE_EPOCHS, lr=1e-3, print_every=1000, batch_size=512))
    res["pre_train"] = {"epochs": PRE_EPOCHS, "s": round(t, 3), "ms_per_epoch": round(t / PRE_EPOCHS * 1e3, 3),
                        "config_epochs": 10000, "config_s": round(t / PRE_EPOCHS * 10000, 1)}
    sampled, t = timed(lambda: solver_g.sample(100, 3))
    res["sample"] = {"s": round(t, 3), "rules": len(sampled)}
    prior = [r[-1] for r in sampled]
    rules = [r[:-1] for r in sampled]
    predictor = Predictor(graph, entity_feature="bias")
    with contextlib.redirect_stdout(sys.stderr):
        predictor.set_rules(rules)
    optim = torch.optim.Adam(predictor.parameters(), lr=1e-3, weight_decay=0)
    solver_p = TrainerPredictor(predictor, train_set, valid_set, test_set, optim, gpus=[0])
    n_batches = len(train_set)
    nb = min(TRAIN_BATCHES, n_batches)
    _, t = timed(lambda: solver_p.train(batch_per_epoch=nb, smoothing=0.2, print_every=1000))
    res["predictor_train"] = {"batches": nb, "s": round(t, 3), "ms_per_batch": round(t / nb * 1e3, 3),
                              "config_batches": n_batches, "config_s": round(t / nb * n_batches, 1)}
    (vm, tm), t = timed(lambda: (solver_p.evaluate("valid"), solver_p.evaluate("test")))
    res["evaluate"] = {"s": round(t, 3), "valid_mrr": vm, "test_mrr": tm}
    H, t = timed(lambda: solver_p.compute_H(print_every=100000))
    res["e_step_compute_H"] = {"s": round(t, 3), "batches": n_batches,
                               "queries_per_s": round(len(graph.train_facts) / t, 1)}
    posterior = [h + p * 0.001 for h, p in zip(H, prior)]
    for i in range(len(rules)):
        rules[i].append(posterior[i])
    _, t = timed(lambda: solver_g.train(RuleDataset(graph.relation_size, rules), num_epoch=100, lr=1e-5,
                                        print_every=1000, batch_size=512))
    res["m_step"] = {"epochs": 100, "s": round(t, 3)}
    res["iteration_s_config"] = round(res["sample"]["s"] + res["predictor_train"]["config_s"] + res["evaluate"]["s"]
                                      + res["e_step_compute_H"]["s"] + res["m_step"]["s"], 1)
    res["note"] = ("iteration_s_config: one EM iteration at the config's counts (predictor training over all "
                   "%d train batches scaled from %d; pre-training, once per run, is %.0f s at 10,000 epochs)"
                   % (n_batches, nb, res["pre_train"]["config_s"]))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
