"""Why train_kinship_lstm_sum_none's step-1 loss drifts ~1e-4 from the
reference while step 0 agrees to ~1e-7 (diagnostic; GPU box).  Adam's first
update is lr * g / (|g| + eps) per element: an element whose true gradient is
zero but whose computed one is rounding noise moves by up to lr in the
noise's direction.  This replays step 0 of the fixture, counts such elements
whose sign differs from the reference's gradient, and then takes the Adam
step twice — with our gradients and with the reference's (from the fixture)
— and prints both step-1 losses against the reference's.
Usage: python tools/train_drift.py [case]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from conftest import GOLDEN, TRAIN_SPECS  # noqa: E402
from rnnlogic_amd import datasets  # noqa: E402
from rnnlogic_amd.data import KnowledgeGraph, TestDataset, TrainDataset, ValidDataset  # noqa: E402
from rnnlogic_amd.predictors import PredictorPlus  # noqa: E402
from rnnlogic_amd.utils import set_seed  # noqa: E402
from torch.utils import data as torch_data  # noqa: E402

case = sys.argv[1] if len(sys.argv) > 1 else "train_kinship_lstm_sum_none"
dev = torch.device("cuda:0")
z = np.load(os.path.join(GOLDEN, case + ".npz"), allow_pickle=False)
data, kw, dim = TRAIN_SPECS[case]


def build():
    set_seed(1)
    graph = KnowledgeGraph(datasets.materialize(data))
    train_set = TrainDataset(graph, 32)
    ValidDataset(graph, 32)
    TestDataset(graph, 32)
    model = PredictorPlus(graph, num_layers=3, hidden_dim=16,
                          embedding_path=datasets.rotate_path(data, dim) if dim else None, **kw)
    model.set_rules(datasets.rule_file(data))
    sd = {k[3:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("sd/")}
    model.load_state_dict(sd, strict=False)
    model = model.to(dev).train()
    train_set.make_batches()
    sampler = torch_data.DistributedSampler(train_set, 1, 0)
    sampler.set_epoch(0)
    return graph, train_set, model, list(iter(sampler))[:len(z["order"])]


def loss_of(graph, train_set, model, idx):
    all_h, all_r, all_t, target, etr = train_set[idx]
    logits, mask = model(all_h.to(dev), all_r.to(dev), etr.to(dev))
    target_t = torch.nn.functional.one_hot(all_t, graph.entity_size)
    target = (target * 0.2 + target_t * 0.8).to(dev)
    logits = (torch.softmax(logits, dim=1) + 1e-8).log()
    return -(logits[mask] * target[mask]).sum() / torch.clamp(target[mask].sum(), min=1)


for use_ref in (False, True):
    graph, train_set, model, order = build()
    optim = torch.optim.Adam(model.parameters(), lr=0.005, weight_decay=0)
    loss = loss_of(graph, train_set, model, order[0])
    loss.backward()
    flips, tiny = 0, 0
    for n, p in model.named_parameters():
        key = "g/" + n
        if key not in z.files or p.grad is None:
            continue
        g, w = p.grad.detach().cpu().numpy(), z[key]
        small = np.abs(w) < 1e-6 * np.abs(w).max()
        tiny += int(small.sum())
        f = int((np.sign(g[small]) != np.sign(w[small])).sum())
        flips += f
        if use_ref:
            p.grad.copy_(torch.from_numpy(w).to(dev))
        elif f:
            print("  %s: %d of %d near-zero gradient elements differ in sign" % (n, f, int(small.sum())))
    optim.step()
    optim.zero_grad()
    l1 = loss_of(graph, train_set, model, order[1]).item()
    want = float(z["s1/loss"])
    print("%s: step-0 loss %.9g (reference %.9g); Adam on %s gradients -> step-1 loss %.9g, reference %.9g, "
          "relative delta %.3g; near-zero elements %d, sign flips %d"
          % (case, loss.item(), float(z["s0/loss"]), "the reference's" if use_ref else "our", l1, want,
             abs(l1 - want) / abs(want), tiny, flips))
