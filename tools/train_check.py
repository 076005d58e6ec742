"""Training-step timings on the GPU box: config 3's WN18RR step (PNA
statistics in HIP vs the autograd-COO path, bench.wn18rr_train_line) and the
headline model's FB15k-237 step (bench.train_step_line)."""
import contextlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from rnnlogic_amd.trainer import TrainerPredictor  # noqa: E402

dev = torch.device("cuda:0")
out = {"wn18rr_train_step": bench.wn18rr_train_line(dev)}
with contextlib.redirect_stdout(sys.stderr):
    graph, test_set, model, rows = bench.build_workload("RotatE")
model = model.to(dev)
solver = TrainerPredictor(model, model.train_set, None, test_set, None, gpus=[0])
bench.train_step_line(model, solver, dev)
out["fb_train_step"] = bench.train_step_line(model, solver, dev)
print(json.dumps(out))
