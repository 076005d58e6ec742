"""WN18RR (config 3) forward steps only, for a rocprofv3 --kernel-trace
timeline (diagnostic; GPU box): python tools/wn_steps.py; then
python tools/step_trace.py <trace dir>."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

dev = torch.device("cuda:0")
model, h, r = bench.wn18rr_model(dev)
for _ in range(12):
    model.invalidate_cache()
    with torch.no_grad():
        model.forward_rows(h, r, None)
torch.cuda.synchronize()
