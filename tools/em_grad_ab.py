"""Per-step gradient A/B of the EM Predictor (GPU box): on the UMLS EM
fixture's sampled rules, for each of the first 40 training batches, the rule
weight / bias gradients of the HIP backward (_PredictorLinear) against torch
autograd on the grounding COO (forward_autograd), the trajectory following the
COO path.  Usage: python tools/em_grad_ab.py"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import em_chain  # noqa: E402
from rnnlogic_amd import datasets  # noqa: E402
from rnnlogic_amd.data import DeviceTrainBatches, KnowledgeGraph, TrainDataset  # noqa: E402
from rnnlogic_amd.predictors import Predictor  # noqa: E402

z, cfg = em_chain.fixture()
dev = torch.device("cuda:0")
graph = KnowledgeGraph(datasets.materialize("umls"))
train_set = TrainDataset(graph, 32)
rules = [r[:-1] for r in json.loads(str(z["em/sampled"]))]
pred = Predictor(graph, entity_feature="bias")
pred.set_rules(rules)
pred = pred.to(dev).train()
opt = torch.optim.Adam(pred.parameters(), lr=1e-3)
dtb = DeviceTrainBatches(train_set, dev)
E = graph.entity_size


def loss_of(logits, target, t):
    target_t = torch.zeros_like(target).scatter_(1, t.view(-1, 1), 1.0)
    tg = target * 0.2 + target_t * 0.8
    lp = (torch.softmax(logits, dim=1) + 1e-8).log()
    return -(lp.reshape(-1) * tg.reshape(-1)).sum() / torch.clamp(tg.sum(), min=1)


for step in range(40):
    h, r, t, target, etr = dtb[step]
    logits, _ = pred(h, r, etr)
    loss_of(logits, target, t).backward()
    gh = pred.rule_weights.grad
    gh = torch.full_like(pred.rule_weights, float("nan")) if gh is None else gh.clone()
    bh = pred.bias.grad.clone()
    opt.zero_grad()
    logits2, _ = pred.forward_autograd(h, r, etr)
    s_err = float((logits - logits2).abs().max())
    loss_of(logits2, target, t).backward()
    gc = pred.rule_weights.grad
    if gc is None or torch.isnan(gh).any():
        print("step %2d: rule grads %s (HIP) / %s (COO)" % (step, "None" if torch.isnan(gh).any() else "set",
                                                              "None" if gc is None else "set"), flush=True)
        opt.step()
        opt.zero_grad()
        continue
    gc = gc.clone()
    d = (gh - gc).abs()
    flip = ((gh > 0) != (gc > 0)) & ((gh != 0) | (gc != 0))
    print("step %2d: score diff %.3g | rule grad max |d| %.3g (max |g| %.3g), sign flips %d (max |g| among them %.3g)"
          " | bias grad max |d| %.3g" % (step, s_err, float(d.max()), float(gc.abs().max()), int(flip.sum()),
                                         float(gc[flip].abs().max()) if flip.any() else 0.0,
                                         float((bh - pred.bias.grad).abs().max())), flush=True)
    opt.step()
    opt.zero_grad()
