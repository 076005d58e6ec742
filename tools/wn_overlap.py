"""WN18RR (config 3) step time under overlap settings (diagnostic; GPU box):
python tools/wn_overlap.py — prints one line per setting."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

dev = torch.device("cuda:0")
for env in ({"RNNL_OVERLAP_GROUND_WG": "256"}, {"RNNL_OVERLAP_GROUND_WG": "512"},
            {"RNNL_OVERLAP_GROUND_WG": "768"}, {"RNNL_OVERLAP": "0"}):
    os.environ.update(env)
    line = bench.wn18rr_line(dev)
    print(json.dumps({"env": env, "ms": line["ms_per_step"], "kernels": line["kernels_ms"]}), flush=True)
    for k in env:
        del os.environ[k]
