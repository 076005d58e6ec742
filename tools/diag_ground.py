"""Grounding diagnostics on the GPU box: the FB15k-237 test rows through
PredictorPlus.ground at capacity_scale 1 (no retry), the rows the launch
flags (n_cand -1: overflow, -2: range), the candidate / bucket-entry totals.
Usage: python tools/diag_ground.py [rows]   (run under tools/ab_run.py for a variant)"""
import contextlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from rnnlogic_amd import _native  # noqa: E402

dev = torch.device("cuda:0")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 40932
with contextlib.redirect_stdout(sys.stderr):
    graph, test_set, model, rows = bench.build_workload("bias")
model = model.to(dev).eval()
h = torch.from_numpy(np.ascontiguousarray(rows[:n, 0])).to(dev)
r = torch.from_numpy(np.ascontiguousarray(rows[:n, 1])).to(dev)
model.capacity_scale = 1
with torch.no_grad():
    g, nr = model.graph.device_graph(dev), model.native_rules(dev)
    ws = model._workspace(dev, n, 1)
    n_cand = torch.empty(n, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    _native.call("rnnl_ground", g, nr.ptr, h.data_ptr(), r.data_ptr(), None, n, n_cand.data_ptr(), ws.data_ptr(),
                 ws.numel(), 1, stream)
    tot = np.zeros(2, dtype=np.int64)
    rc = model._status(ws, stream, tot)
nc = n_cand.cpu().numpy()
bad = np.nonzero(nc < 0)[0]
print("rows %d rc %d candidates %d entries %d flagged %d (overflow %d, range %d)" %
      (n, rc, tot[0], tot[1], len(bad), int((nc == -1).sum()), int((nc == -2).sum())))
for q in bad[:10]:
    print("  row %d h %d r %d n_cand %d" % (q, int(h[q]), int(r[q]), nc[q]))
