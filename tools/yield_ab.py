"""WN18RR step time against the RotatE yield point (diagnostic; GPU box):
python tools/yield_ab.py — the share of RotatE's grid in the first of its two
launches (PredictorPlus.rotate_share), and one launch (no yield)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

dev = torch.device("cuda:0")
model, h, r = bench.wn18rr_model(dev)


def step():
    model.invalidate_cache()
    with torch.no_grad():
        return model.forward_rows(h, r, None)


for rep in range(2):
    for share in (0.35, 0.5, 0.65, 0.8, None):
        model.rotate_yield = share is not None
        if share is not None:
            model.rotate_share = share
        ms = bench.time_forward(step, 10) * 1e3
        print("share %s: %.3f ms" % (share, ms), flush=True)
