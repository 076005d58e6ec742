"""Where the reference call pattern's time goes (diagnostic, GPU box): per
PredictorPlus.forward call on 32-row FB15k-237 test batches (the bench
model), the time inside the one C call (rnnl_predictorplus_forward_rotate:
enqueue + header read-back wait) against the whole call (the Python
mirror's own work = the rest)."""
import contextlib
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from rnnlogic_amd import _native  # noqa: E402

dev = torch.device("cuda:0")
with contextlib.redirect_stdout(sys.stderr):
    graph, test_set, model, rows = bench.build_workload("RotatE")
model = model.to(dev).eval()
batches = test_set.batches[:600]
hs = [torch.tensor([x[0] for x in b], device=dev) for b in batches]
rs = [torch.tensor([x[1] for x in b], device=dev) for b in batches]
L = _native.lib()
inner = L.rnnl_predictorplus_forward_rotate
acc = [0.0]


def timed(*a):
    t = time.perf_counter()
    rc = inner(*a)
    acc[0] += time.perf_counter() - t
    return rc


L.rnnl_predictorplus_forward_rotate = timed
with torch.no_grad():
    for k in range(5):
        model(hs[k], rs[k], None)
    torch.cuda.synchronize()
    acc[0] = 0.0
    t0 = time.perf_counter()
    for h, r in zip(hs, rs):
        model(h, r, None)
    torch.cuda.synchronize()
    sec = time.perf_counter() - t0
n = len(hs)
print("calls %d: %.1f us/call total, %.1f us in the C call (enqueue + wait), %.1f us Python mirror"
      % (n, sec / n * 1e6, acc[0] / n * 1e6, (sec - acc[0]) / n * 1e6))
