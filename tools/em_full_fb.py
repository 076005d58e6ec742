"""Config 5 end to end on one GPU (diagnostic; GPU box): the whole
run_rnnlogic.py flow (reference src/run_rnnlogic.py:45-139) through the
package with config/FB15k-237.yaml's settings on the seeded synthetic
FB15k-237 graph — generator pre-training, the EM iterations (sample, a new
Predictor trained over every train batch, evaluate, compute_H, M-step), the
generator's post-training on the replay buffer, beam search, and the final
PredictorPlus stage (train over every train batch + evaluate, per
iteration).  Prints one JSON line with the wall time of every phase and the
MRRs.  Pre-training uses rnnlogic_rules.txt with synthetic weights (the
config's mined_rules.txt needs the absent train.txt), as bench.py's
em_iteration line does.

Usage: python tools/em_full_fb.py [--em-iters 5] [--final-iters 5]
       [--pre-epochs 10000]"""
import argparse
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
from rnnlogic_amd.predictors import Predictor, PredictorPlus  # noqa: E402
from rnnlogic_amd.trainer import TrainerGenerator, TrainerPredictor  # noqa: E402
from rnnlogic_amd.utils import set_seed  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--em-iters", type=int, default=5)      # config EM.num_iters
    ap.add_argument("--final-iters", type=int, default=5)   # config final_prediction.num_iters
    ap.add_argument("--pre-epochs", type=int, default=10000)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    times, mrr = {}, {}

    def timed(name, fn):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        out = fn()
        torch.cuda.synchronize(dev)
        times[name] = round(times.get(name, 0.0) + time.perf_counter() - t0, 3)
        print("%s %.1f s" % (name, times[name]), file=sys.stderr, flush=True)
        return out

    t_all = time.perf_counter()
    with contextlib.redirect_stdout(sys.stderr):
        set_seed(1)
        graph = KnowledgeGraph(datasets.materialize("FB15k-237"))
        train_set, valid_set, test_set = TrainDataset(graph, 32), ValidDataset(graph, 32), TestDataset(graph, 32)
    mined = [[int(x) for x in line.split()] for line in open(datasets.rule_file("FB15k-237"))]
    dataset = RuleDataset(graph.relation_size, [r + [0.25 * ((i * 37) % 11) - 1.0] for i, r in enumerate(mined)])
    gen = Generator(graph, num_layers=1, embedding_dim=512, hidden_dim=256)
    solver_g = TrainerGenerator(gen, gpu=0)
    timed("pre_train", lambda: solver_g.train(dataset, num_epoch=args.pre_epochs, lr=1e-3, print_every=1000000,
                                              batch_size=512))
    replay = []
    for k in range(args.em_iters):  # run_rnnlogic.py:61-91
        sampled = timed("em_sample", lambda: solver_g.sample(100, 3))
        prior = [r[-1] for r in sampled]
        rules = [r[:-1] for r in sampled]
        predictor = Predictor(graph, entity_feature="bias")
        with contextlib.redirect_stdout(sys.stderr):
            predictor.set_rules(rules)
        optim = torch.optim.Adam(predictor.parameters(), lr=1e-3, weight_decay=0)
        solver_p = TrainerPredictor(predictor, train_set, valid_set, test_set, optim, gpus=[0])
        timed("em_predictor_train", lambda: solver_p.train(batch_per_epoch=1000000, smoothing=0.2,
                                                           print_every=1000000))
        v, t = timed("em_evaluate", lambda: (solver_p.evaluate("valid"), solver_p.evaluate("test")))
        mrr["em_iter%d" % k] = {"valid": v, "test": t, "rules": len(rules)}
        H = timed("em_compute_H", lambda: solver_p.compute_H(print_every=1000000))
        posterior = [h + p * 0.001 for h, p in zip(H, prior)]
        for i in range(len(rules)):
            rules[i].append(posterior[i])
        replay += rules
        timed("em_m_step", lambda: solver_g.train(RuleDataset(graph.relation_size, rules), num_epoch=100, lr=1e-5,
                                                  print_every=1000000, batch_size=512))
        del solver_p, predictor, optim
    if replay:  # run_rnnlogic.py:93-99
        timed("post_train", lambda: solver_g.train(RuleDataset(graph.relation_size, replay), num_epoch=1000,
                                                   lr=1e-5, print_every=1000000, batch_size=512))
    sampled = timed("beam_search", lambda: solver_g.beam_search(100, 3))  # run_rnnlogic.py:101-110
    rules = [r[:-1] for r in sampled]
    predictor = PredictorPlus(graph, hidden_dim=16)  # run_rnnlogic.py:112-139 (config predictorplus.model)
    with contextlib.redirect_stdout(sys.stderr):
        predictor.set_rules(rules)
    optim = torch.optim.Adam(predictor.parameters(), lr=0.005, weight_decay=0)
    solver_p = TrainerPredictor(predictor, train_set, valid_set, test_set, optim, gpus=[0])
    best_valid, test_at_best = 0.0, 0.0
    for k in range(args.final_iters):
        timed("final_train", lambda: solver_p.train(batch_per_epoch=1000000, smoothing=0.2, print_every=1000000))
        v, t = timed("final_evaluate", lambda: (solver_p.evaluate("valid"), solver_p.evaluate("test")))
        mrr["final_iter%d" % k] = {"valid": v, "test": t}
        if v > best_valid:
            best_valid, test_at_best = v, t
    out = {"workload": "config 5 (run_rnnlogic.py, config/FB15k-237.yaml) on one MI355X: seeded synthetic FB15k-237 "
                       "train graph; generator pre-trained on rnnlogic_rules.txt with synthetic weights",
           "em_iters": args.em_iters, "final_iters": args.final_iters, "pre_epochs": args.pre_epochs,
           "wall_s": round(time.perf_counter() - t_all, 1), "phases_s": times,
           "final_rules": len(rules), "best_valid_mrr": best_valid, "test_mrr_at_best_valid": test_at_best,
           "mrr": mrr}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
