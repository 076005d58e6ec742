"""The reference API's call pattern (trainer.py:150-173): PredictorPlus.forward
once per TestDataset batch (B <= 32, one relation) over the FB15k-237 test
split, the bench model (lstm/sum + RotatE D = 1000) — diagnostic timing of the
per-call cost beside bench.py's one-launch forward_rows.
Usage (GPU box): python tools/per_batch_forward.py [N_BATCHES [FEATURE]]"""
import contextlib
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 0
FEATURE = sys.argv[2] if len(sys.argv) > 2 else "RotatE"  # or "bias"
dev = torch.device("cuda:0")
with contextlib.redirect_stdout(sys.stderr):
    graph, test_set, model, rows = bench.build_workload(FEATURE)
model = model.to(dev).eval()
if "ZERO_EARLY" in os.environ:  # A/B of the zero fill's issue point
    model.zero_early = os.environ["ZERO_EARLY"] == "1"
batches = test_set.batches[:N] if N else test_set.batches
hs = [torch.tensor([x[0] for x in b], device=dev) for b in batches]
rs = [torch.tensor([x[1] for x in b], device=dev) for b in batches]
with torch.no_grad():
    for k in range(3):
        model(hs[k], rs[k], None)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for h, r in zip(hs, rs):
        model(h, r, None)
    torch.cuda.synchronize()
    sec = time.perf_counter() - t0
n = sum(len(b) for b in batches)
print("per-batch forward: %d batches, %d queries, %.3f s, %.1f queries/s, %.3f ms/call" % (
    len(batches), n, sec, n / sec, sec / len(batches) * 1e3))
