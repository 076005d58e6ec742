"""Where a PredictorPlus training step (bench.py's train_step line: FB15k-237,
B = 32, edge removal, RotatE feature, Adam) spends its time (diagnostic; GPU
box): torch.profiler over 10 steps, top ops by device and by host time.
`emb`: the final PredictorPlus stage of run_rnnlogic.py instead
(PredictorPlus(graph, hidden_dim=16): emb / bias / sum, rnnlogic_rules.txt).
Usage: python tools/train_profile.py [emb]"""
import contextlib
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from rnnlogic_amd.data import DeviceTrainBatches  # noqa: E402
from rnnlogic_amd.trainer import TrainerPredictor  # noqa: E402

dev = torch.device("cuda:0")
with contextlib.redirect_stdout(sys.stderr):
    graph, test_set, model, rows = bench.build_workload("RotatE")
    if len(sys.argv) > 1 and sys.argv[1] == "emb":
        from rnnlogic_amd.predictors import PredictorPlus
        train_set = model.train_set
        model = PredictorPlus(graph, hidden_dim=16)
        model.set_rules(bench.datasets.rule_file("FB15k-237"))
        model.train_set = train_set
model = model.to(dev)
solver = TrainerPredictor(model, model.train_set, None, test_set, None, gpus=[0])
solver.optimizer = torch.optim.Adam(model.parameters(), lr=5e-3)
dtb = DeviceTrainBatches(model.train_set, dev)
model.train()
batches = [[x.unsqueeze(0) for x in dtb[i]] for i in range(22)]
for b in batches[:2]:
    solver.train_step(model, b, 0.2)
torch.cuda.synchronize()
t = time.perf_counter()
for b in batches[2:12]:
    solver.train_step(model, b, 0.2)
torch.cuda.synchronize()
print("ms per step (no profiler): %.3f" % ((time.perf_counter() - t) * 100))
acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
with torch.profiler.profile(activities=acts) as prof:
    for b in batches[12:22]:
        solver.train_step(model, b, 0.2)
    torch.cuda.synchronize()
ka = prof.key_averages()
print(ka.table(sort_by="self_cuda_time_total", row_limit=18, max_name_column_width=60))
print(ka.table(sort_by="self_cpu_time_total", row_limit=18, max_name_column_width=60))
