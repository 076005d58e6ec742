"""cProfile of the bench step's host side (diagnostic; GPU box):
python tools/host_profile.py [--feature RotatE|bias]"""
import cProfile
import contextlib
import os
import pstats
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

feature = sys.argv[2] if len(sys.argv) > 2 else "RotatE"
with contextlib.redirect_stdout(sys.stderr):
    graph, test_set, model, rows = bench.build_workload(feature)
dev = torch.device("cuda:0")
model = model.to(dev).eval()
h = torch.from_numpy(rows[:, 0]).to(dev)
r = torch.from_numpy(rows[:, 1]).to(dev)


def step():
    model.invalidate_cache()
    with torch.no_grad():
        model.forward_rows(h, r, None)


for _ in range(2):
    step()
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
for _ in range(3):
    step()
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("cumulative").print_stats(25)
