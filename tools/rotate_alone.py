"""The bench's RotatE launch alone (no grounding / scoring beside it), for
rocprofv3 counter passes (diagnostic; GPU box): python tools/rotate_alone.py"""
import contextlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

dev = torch.device("cuda:0")
with contextlib.redirect_stdout(sys.stderr):
    graph, test_set, model, rows = bench.build_workload("RotatE")
model = model.to(dev).eval()
h = torch.from_numpy(rows[:, 0]).to(dev)
r = torch.from_numpy(rows[:, 1]).to(dev)
out = torch.empty((len(rows), graph.entity_size), dtype=torch.float32, device=dev)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
with torch.no_grad():
    for k in range(4):
        if k == 1:
            e0.record()
        model.RotatE.score_into(h, r, out)
    e1.record()
torch.cuda.synchronize()
print("rotate alone: %.3f ms per launch" % (e0.elapsed_time(e1) / 3))
