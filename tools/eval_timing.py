"""Where evaluate('test') spends its time on FB15k-237 (diagnostic; GPU box)."""
import contextlib
import os
import sys
import time

import torch
from torch.utils import data as torch_data

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from rnnlogic_amd.data import DeviceEvalBatches  # noqa: E402
from rnnlogic_amd.trainer import TrainerPredictor  # noqa: E402

dev = torch.device("cuda:0")
with contextlib.redirect_stdout(sys.stderr):
    graph, test_set, model, rows = bench.build_workload(sys.argv[1] if len(sys.argv) > 1 else "RotatE")
model = model.to(dev).eval()
solver = TrainerPredictor(model, model.train_set, None, test_set, None, gpus=[0])
solver.evaluate("test")
T = {}


def lap(name, t0):
    torch.cuda.synchronize()
    T[name] = T.get(name, 0.0) + time.perf_counter() - t0
    return time.perf_counter()


for _ in range(3):
    t = time.perf_counter()
    sampler = torch_data.DistributedSampler(test_set, 1, 0)
    db = solver._dev_eval[id(test_set)]
    h, r, tt, flag = db.rows(list(iter(sampler)))
    t = lap("rows+flags", t)
    with torch.no_grad():
        logits, mask = model.forward_rows(h, r, None)
    t = lap("forward", t)
    L, H = TrainerPredictor.filtered_ranks(logits, mask, flag, tt, graph.entity_size)
    t = lap("ranks", t)
    ranks = torch.stack([h, r, tt, L, H], 1).to(torch.long).cpu().numpy()
    t = lap("to_host", t)
    TrainerPredictor.rank_metrics(ranks, True)
    t = lap("metrics", t)
    t = time.perf_counter()
    solver.evaluate("test")
    t = lap("evaluate_total", t)
print({k: round(v / 3 * 1e3, 2) for k, v in T.items()})
