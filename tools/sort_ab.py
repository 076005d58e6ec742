"""A/B of phase B's sort-window width (rnnl_debug_sort_bits) on the GPU box.
Per width: the FB15k-237 bias-feature grounding + scoring alone (one
one-stream launch over the split, bench.isolated_ground_ms) and its bucket
entries; the headline step (RotatE overlap, the bench's timed step); the
WN18RR step and its ground + PNA alone; the kinship step.
Usage: python tools/sort_ab.py [bits ...]   (-1 = the default)"""
import contextlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from rnnlogic_amd import _native  # noqa: E402

dev = torch.device("cuda:0")
bits_list = [int(x) for x in sys.argv[1:]] or [-1, 11]


def rows_of(rows):
    return (torch.from_numpy(np.ascontiguousarray(rows[:, 0])).to(dev),
            torch.from_numpy(np.ascontiguousarray(rows[:, 1])).to(dev))


def stepper(model, h, r):
    def step():
        model.invalidate_cache()
        with torch.no_grad():
            return model.forward_rows(h, r, None)
    return step


with contextlib.redirect_stdout(sys.stderr):
    graph, test_set, model, rows = bench.build_workload("bias")
    rgraph, _, rmodel, rrows = bench.build_workload("RotatE")
    wmodel, wh, wr, wgraph, _, _ = bench.wn18rr_model(dev, full=True)
    kin = bench.kinship_line  # (its own model; timed below through the same line)
model, rmodel = model.to(dev).eval(), rmodel.to(dev).eval()
h, r = rows_of(rows)
rh, rr = rows_of(rrows)
fb_step, rot_step, wn_step = stepper(model, h, r), stepper(rmodel, rh, rr), stepper(wmodel, wh, wr)
for f in (fb_step, rot_step, wn_step):  # capacity_scale settles (overflow retries) before the timed launches
    f()
torch.cuda.synchronize()
for bits in bits_list * 2:  # two rounds: box drift shows as a round difference
    _native.call("rnnl_debug_sort_bits", bits)
    ms = [bench.isolated_ground_ms(model, graph, h, r, dev) for _ in range(4)][1:]
    tot = np.zeros(2, dtype=np.int64)
    with torch.no_grad():
        model.ground(h, r, None, totals=tot)
    wms = [bench.isolated_ground_ms(wmodel, wgraph, wh, wr, dev) for _ in range(4)][1:]
    head = bench.time_forward(rot_step, 5) * 1e3
    wn = bench.time_forward(wn_step, 10) * 1e3
    with contextlib.redirect_stdout(sys.stderr):
        k = kin(dev, reps=50)["ms_per_step"]
    print("bits %3d: FB bias ground+score %s ms, entries %d | headline %.3f ms | WN step %.3f, ground+pna %s ms "
          "| kinship %.3f ms" % (bits, " ".join("%.3f" % x for x in ms), tot[1], head, wn,
                                 " ".join("%.3f" % x for x in wms), k), flush=True)
_native.call("rnnl_debug_sort_bits", -1)
