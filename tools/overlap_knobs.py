"""Sweep of the RotatE-overlap launch knobs (PredictorPlus.rotate_yield,
rotate_share, overlap_ground_wg, overlap_score_wg, zero_early) on the WN18RR
config-3 step (PNA) or the FB15k-237 headline step (SUM), one process, two
rounds so that box drift shows.  GPU box; diagnostic only.
Usage: python tools/overlap_knobs.py wn|fb "yield,share,gwg,swg,zero_early" ..."""
import contextlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

dev = torch.device("cuda:0")
which = sys.argv[1]
confs = [tuple(c.split(",")) for c in sys.argv[2:]]
with contextlib.redirect_stdout(sys.stderr):
    if which == "wn":
        model, h, r = bench.wn18rr_model(dev)
        reps = 20
    else:
        _, _, model, rows = bench.build_workload("RotatE")
        model = model.to(dev).eval()
        h = torch.from_numpy(np.ascontiguousarray(rows[:, 0])).to(dev)
        r = torch.from_numpy(np.ascontiguousarray(rows[:, 1])).to(dev)
        reps = 6


def step():
    model.invalidate_cache()
    with torch.no_grad():
        return model.forward_rows(h, r, None)


ref = step()[0].clone()
for rnd in range(2):
    for c in confs:
        model.rotate_yield = c[0] == "1"
        model.rotate_share = float(c[1])
        model.overlap_ground_wg = int(c[2])
        model.overlap_score_wg = int(c[3])
        model.zero_early = c[4] == "1"
        same = bool(torch.equal(step()[0], ref))
        ms = bench.time_forward(step, reps) * 1e3
        print("round %d %s yield %s share %s ground_wg %s score_wg %s zero_early %s: %.3f ms (bitwise %s)"
              % (rnd, which, *c, ms, same), flush=True)
