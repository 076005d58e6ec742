"""Run-to-run stability of the bench step with and without the stream
overlap (diagnostic; GPU box): 6 blocks of 8 back-to-back steps per mode."""
import contextlib
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

with contextlib.redirect_stdout(sys.stderr):
    graph, test_set, model, rows = bench.build_workload("RotatE")
dev = torch.device("cuda:0")
model = model.to(dev).eval()
h = torch.from_numpy(rows[:, 0]).to(dev)
r = torch.from_numpy(rows[:, 1]).to(dev)


def block(n):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        model.invalidate_cache()
        with torch.no_grad():
            model.forward_rows(h, r, None)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


for mode in os.environ.get("MODES", "overlap single overlap single").split():
    model.overlap = mode.startswith("overlap")
    if mode.startswith("overlap") and ":" in mode:
        model.overlap_chunks = int(mode.split(":")[1])
    block(2)
    print(mode, " ".join("%.1f" % block(8) for _ in range(5)), flush=True)
