"""One DistributedSampler shard of the bench workload (default: N = 8, rank 3,
the slowest in round 4/5's shard_balance) stepped as bench.py's
shard_balance times it (rule aggregates recomputed, RotatE + grounding +
scoring) — for a kernel trace of one rank's step at N = 8 (diagnostic; GPU
box): rocprofv3 --kernel-trace --output-format csv -d DIR -- python
tools/shard_run.py [N RANK STEPS], then python tools/step_trace.py DIR."""
import contextlib
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

world = int(sys.argv[1]) if len(sys.argv) > 1 else 8
rank = int(sys.argv[2]) if len(sys.argv) > 2 else 3
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 8
wgs = [(int(a), int(b)) for a, b in (x.split("/") for x in sys.argv[4:])] or [None]  # ground/score workgroups
dev = torch.device("cuda:0")
with contextlib.redirect_stdout(sys.stderr):
    graph, test_set, model, full = bench.build_workload("RotatE")
model = model.to(dev).eval()
if "ZERO_EARLY" in os.environ:  # A/B of the zero fill's issue point
    model.zero_early = os.environ["ZERO_EARLY"] == "1"
rows = bench.shard_rows(test_set, world, rank)[0] if world > 1 else full  # N = 1: the bench's row order
sh = torch.from_numpy(np.ascontiguousarray(rows[:, 0])).to(dev)
sr = torch.from_numpy(np.ascontiguousarray(rows[:, 1])).to(dev)


def st():
    model.invalidate_cache()
    with torch.no_grad():
        return model.forward_rows(sh, sr, None)


for wg in wgs:
    if wg is not None:
        model.overlap_ground_wg, model.overlap_score_wg = wg
    for _ in range(2):
        st()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        st()
    torch.cuda.synchronize()
    print("N=%d rank %d: %d rows, %.3f ms per step (ground / score workgroups %d / %d, zero_early %d)"
          % (world, rank, len(rows), (time.perf_counter() - t) * 1e3 / steps, model.overlap_ground_wg,
             model.overlap_score_wg, model.zero_early))
