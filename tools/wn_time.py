"""WN18RR (config 3) forward step time, as bench.py's wn18rr_forward times it
(diagnostic; GPU box; A/B builds through tools/ab_run.py)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

dev = torch.device("cuda:0")
model, h, r = bench.wn18rr_model(dev)
if "ROTATE_SHARE" in os.environ:  # A/B of the PNA yield point
    model.rotate_share = float(os.environ["ROTATE_SHARE"])
if "ZERO_EARLY" in os.environ:  # A/B of the zero fill's issue point
    model.zero_early = os.environ["ZERO_EARLY"] == "1"


def step():
    model.invalidate_cache()
    with torch.no_grad():
        return model.forward_rows(h, r, None)


ms = [bench.time_forward(step, 10) * 1e3 for _ in range(3)]
print("%s share %.2f zero_early %d: WN18RR step %s ms" % (os.path.basename(__import__("rnnlogic_amd._native")._native.LIB_PATH),
                                model.rotate_share, model.zero_early,
                                " / ".join("%.3f" % x for x in ms)))
