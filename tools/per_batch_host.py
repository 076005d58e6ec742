"""Host-side profile (cProfile) of the per-batch PredictorPlus.forward loop
(tools/per_batch_forward.py's workload) — where a call's Python / launch time
goes (GPU box).  Usage: python tools/per_batch_host.py [N_BATCHES]"""
import contextlib
import cProfile
import os
import pstats
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 300
dev = torch.device("cuda:0")
with contextlib.redirect_stdout(sys.stderr):
    graph, test_set, model, rows = bench.build_workload("RotatE")
model = model.to(dev).eval()
batches = test_set.batches[:N]
hs = [torch.tensor([x[0] for x in b], device=dev) for b in batches]
rs = [torch.tensor([x[1] for x in b], device=dev) for b in batches]
with torch.no_grad():
    for k in range(3):
        model(hs[k], rs[k], None)
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for h, r in zip(hs, rs):
        model(h, r, None)
    torch.cuda.synchronize()
    pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
