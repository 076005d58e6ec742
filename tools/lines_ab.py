"""A/B of a library build (run through tools/ab_run.py per variant) on the
secondary lines a scoring / grounding change moves: the FB15k-237 bias
grounding + scoring alone, the headline step, the WN18RR step and its
ground + PNA alone, the kinship step — plus sha1 digests of the WN18RR and
FB15k-237 bias score matrices, so that variants meant to be bitwise equal
can be checked against each other.
Usage: python tools/ab_run.py <variant.so> tools/lines_ab.py [rounds]"""
import contextlib
import hashlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from rnnlogic_amd import _native  # noqa: E402

dev = torch.device("cuda:0")
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
tag = os.path.basename(_native.LIB_PATH)


def rows_of(rows):
    return (torch.from_numpy(np.ascontiguousarray(rows[:, 0])).to(dev),
            torch.from_numpy(np.ascontiguousarray(rows[:, 1])).to(dev))


def stepper(model, h, r):
    def step():
        model.invalidate_cache()
        with torch.no_grad():
            return model.forward_rows(h, r, None)
    return step


def sha(t):
    return hashlib.sha1(t.detach().contiguous().cpu().numpy().tobytes()).hexdigest()[:12]


if os.environ.get("AB_ONLY_WN"):  # the WN18RR lines alone (PNA changes)
    with contextlib.redirect_stdout(sys.stderr):
        wmodel, wh, wr, wgraph, _, _ = bench.wn18rr_model(dev, full=True)
    if os.environ.get("AB_PNA_WG"):
        wmodel.overlap_score_wg = int(os.environ["AB_PNA_WG"])
        tag += " wg%d" % wmodel.overlap_score_wg
    wn_step = stepper(wmodel, wh, wr)
    wn_step()
    d = sha(wn_step()[0])
    for rd in range(rounds):
        wms = [bench.isolated_ground_ms(wmodel, wgraph, wh, wr, dev) for _ in range(4)][1:]
        wn = [bench.time_forward(wn_step, 10) * 1e3 for _ in range(2)]
        print("%s r%d: WN step %s, ground+pna %s ms | wn %s" % (tag, rd, " ".join("%.3f" % x for x in wn),
                                                                 " ".join("%.3f" % x for x in wms), d), flush=True)
    sys.exit(0)
with contextlib.redirect_stdout(sys.stderr):
    graph, test_set, model, rows = bench.build_workload("bias")
    rgraph, _, rmodel, rrows = bench.build_workload("RotatE")
    wmodel, wh, wr, wgraph, _, _ = bench.wn18rr_model(dev, full=True)
model, rmodel = model.to(dev).eval(), rmodel.to(dev).eval()
if os.environ.get("AB_PNA_WG"):  # the PNA scoring pass's workgroups beside RotatE
    wmodel.overlap_score_wg = int(os.environ["AB_PNA_WG"])
    tag += " wg%d" % wmodel.overlap_score_wg
h, r = rows_of(rows)
rh, rr = rows_of(rrows)
fb_step, rot_step, wn_step = stepper(model, h, r), stepper(rmodel, rh, rr), stepper(wmodel, wh, wr)
for f in (fb_step, rot_step, wn_step):  # capacity_scale settles (overflow retries) before the timed launches
    f()
torch.cuda.synchronize()
digests = "wn %s fb-bias %s" % (sha(wn_step()[0]), sha(fb_step()[0]))
for rd in range(rounds):
    ms = [bench.isolated_ground_ms(model, graph, h, r, dev) for _ in range(4)][1:]
    wms = [bench.isolated_ground_ms(wmodel, wgraph, wh, wr, dev) for _ in range(4)][1:]
    head = bench.time_forward(rot_step, 5) * 1e3
    wn = bench.time_forward(wn_step, 10) * 1e3
    with contextlib.redirect_stdout(sys.stderr):
        k = bench.kinship_line(dev, reps=50)["ms_per_step"]
    print("%s r%d: FB bias ground+score %s ms | headline %.3f ms | WN step %.3f, ground+pna %s ms | kinship %.3f ms "
          "| %s" % (tag, rd, " ".join("%.3f" % x for x in ms), head, wn, " ".join("%.3f" % x for x in wms), k,
                    digests), flush=True)
