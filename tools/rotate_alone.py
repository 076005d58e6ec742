"""The bench's RotatE launch alone (no grounding / scoring beside it), for
rocprofv3 counter passes (diagnostic; GPU box): python tools/rotate_alone.py
[N RANK] — with N, the rows of one DistributedSampler shard.  Three timed
rounds of three launches: the first round of a process reads 0.3-0.5 ms high
per launch on a shard (clock ramp), so compare the later ones."""
import contextlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from rnnlogic_amd import _native  # noqa: E402

if os.environ.get("RNNL_LIB"):  # an A/B build (tools/build_variants.sh)
    _native.LIB_PATH = os.path.abspath(os.environ["RNNL_LIB"])

dev = torch.device("cuda:0")
with contextlib.redirect_stdout(sys.stderr):
    graph, test_set, model, rows = bench.build_workload("RotatE")
model = model.to(dev).eval()
if len(sys.argv) > 2:
    rows, _ = bench.shard_rows(test_set, int(sys.argv[1]), int(sys.argv[2]))
h = torch.from_numpy(rows[:, 0].copy()).to(dev)
r = torch.from_numpy(rows[:, 1].copy()).to(dev)
out = torch.empty((len(rows), graph.entity_size), dtype=torch.float32, device=dev)
for rnd in range(3):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.no_grad():
        for k in range(4):
            if k == 1:
                e0.record()
            model.RotatE.score_into(h, r, out)
        e1.record()
    torch.cuda.synchronize()
    print("rotate alone, %d rows, round %d: %.3f ms per launch" % (len(rows), rnd, e0.elapsed_time(e1) / 3))
