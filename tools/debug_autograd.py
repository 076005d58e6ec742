"""Diagnostic: PredictorPlus.forward_autograd (training path) against the
fused HIP forward on the same rows, for every training fixture case."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
from conftest import GOLDEN, TRAIN_CASES, TRAIN_SPECS  # noqa: E402
from rnnlogic_amd import datasets  # noqa: E402
from rnnlogic_amd.data import KnowledgeGraph, TestDataset, TrainDataset, ValidDataset  # noqa: E402
from rnnlogic_amd.predictors import PredictorPlus  # noqa: E402
from rnnlogic_amd.utils import set_seed  # noqa: E402

dev = torch.device("cuda:0")
for case in TRAIN_CASES:
    z = np.load(os.path.join(GOLDEN, case + ".npz"), allow_pickle=False)
    data, kw, dim = TRAIN_SPECS[case]
    set_seed(1)
    graph = KnowledgeGraph(datasets.materialize(data))
    model = PredictorPlus(graph, num_layers=3, hidden_dim=16,
                          embedding_path=datasets.rotate_path(data, dim) if dim else None, **kw)
    model.set_rules(datasets.rule_file(data))
    sd = {k[3:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("sd/")}
    model.load_state_dict(sd, strict=False)
    model = model.to(dev)
    h = torch.from_numpy(z["s0/h"]).to(dev)
    r = torch.from_numpy(z["s0/r"]).to(dev)
    etr = torch.from_numpy(z["s0/etr"]).to(dev)
    sa, ma = model.forward_autograd(h, r, etr)
    with torch.no_grad():
        sb, mb = model.forward_rows(h, r, etr)
    fin = torch.isfinite(sb)
    print(case, "mask equal", bool((ma == mb).all()), "finite equal", bool((torch.isfinite(sa) == fin).all()),
          "max |diff|", float((sa.detach() - sb)[fin].abs().max()))
    row, ent, ce, node, count = model.ground_coo(h, r, etr)
    print("   C", ent.numel(), "P", node.numel(), "rows", int(row.max()) + 1 if row.numel() else 0)
