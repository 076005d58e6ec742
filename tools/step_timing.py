"""Per-step wall time of the bench step and where the host waits
(diagnostic; GPU box): python tools/step_timing.py [steps]"""
import contextlib
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from rnnlogic_amd import _native  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 6
with contextlib.redirect_stdout(sys.stderr):
    graph, test_set, model, rows = bench.build_workload("RotatE")
dev = torch.device("cuda:0")
model = model.to(dev).eval()
h = torch.from_numpy(rows[:, 0]).to(dev)
r = torch.from_numpy(rows[:, 1]).to(dev)
host = {}


def wrap(obj, name):
    f = getattr(obj, name)

    def g(*a, **k):
        t = time.perf_counter()
        try:
            return f(*a, **k)
        finally:
            host[name] = host.get(name, 0.0) + time.perf_counter() - t
    setattr(obj, name, g)


for nm in ("node_weights", "_params", "_forward_overlap", "_chunk_workspace", "_side_streams", "all_rule_embeddings"):
    wrap(model, nm)
wrap(model.RotatE, "score_into")
wrap(model.RotatE, "_device_tables")
wrap(model.RotatE, "_workspace")
_empty = torch.empty


def empty(*a, **k):
    t = time.perf_counter()
    try:
        return _empty(*a, **k)
    finally:
        host["torch.empty"] = host.get("torch.empty", 0.0) + time.perf_counter() - t


torch.empty = empty
for i in range(steps):
    host.clear()
    t0 = time.perf_counter()
    model.invalidate_cache()
    ev = {}
    with torch.no_grad():
        out = model.forward_rows(h, r, None, events=ev)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    del out
    t3 = time.perf_counter()
    print("step %d: forward %.1f ms, trailing sync %.1f ms, free %.1f ms | events start-base %.1f base-ground %.1f "
          "ground-end %.1f" % (i, (t1 - t0) * 1e3, (t2 - t1) * 1e3, (t3 - t2) * 1e3,
                               ev["start"].elapsed_time(ev["base"]), ev["base"].elapsed_time(ev["ground"]),
                               ev["ground"].elapsed_time(ev["end"])), flush=True)
    print("   host ms: " + ", ".join("%s %.1f" % (k, v * 1e3) for k, v in sorted(host.items())), flush=True)
t0 = time.perf_counter()
for i in range(steps):
    model.invalidate_cache()
    with torch.no_grad():
        model.forward_rows(h, r, None)
torch.cuda.synchronize()
print("back-to-back: %.1f ms/step" % ((time.perf_counter() - t0) / steps * 1e3), flush=True)
t0 = time.perf_counter()
for i in range(steps):
    model.invalidate_cache()
    with torch.no_grad():
        out = model.forward_rows(h, r, None)
    del out
torch.cuda.synchronize()
print("back-to-back, explicit del: %.1f ms/step" % ((time.perf_counter() - t0) / steps * 1e3), flush=True)
