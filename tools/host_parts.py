"""Host time of the pieces of one per-batch PredictorPlus.forward call (the
reference call pattern, tools/per_batch_forward.py's model) — each piece
timed alone over many calls with the caches warm (diagnostic; GPU box)."""
import contextlib
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

dev = torch.device("cuda:0")
with contextlib.redirect_stdout(sys.stderr):
    graph, test_set, model, rows = bench.build_workload("RotatE")
model = model.to(dev).eval()
b = test_set.batches[100]
h = torch.tensor([x[0] for x in b], device=dev)
r = torch.tensor([x[1] for x in b], device=dev)
N = 2000


def t(name, fn):
    with torch.no_grad():
        for _ in range(20):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(N):
            fn()
        el = time.perf_counter() - t0
        torch.cuda.synchronize()
    print("%-40s %8.2f us per call" % (name, el / N * 1e6))


with torch.no_grad():
    model(h, r, None)
nw = model.node_weights(dev)
t("forward (whole call, GPU-synchronised)", lambda: model(h, r, None))
t("node_weights (cache hit)", lambda: model.node_weights(dev))
t("_params (cache hit)", lambda: model._params(dev, nw))
t("RotatE.native_args", lambda: model.RotatE.native_args(h.numel(), 1, 0.0))
t("torch.empty (32 x |E|) f32", lambda: torch.empty((32, model.num_entities), device=dev))
t("_needs_grad", lambda: model._needs_grad())
t("graph.device_graph + native_rules", lambda: (model.graph.device_graph(dev), model.native_rules(dev)))
t("torch.cuda.current_stream", lambda: torch.cuda.current_stream(dev).cuda_stream)


def recompute():
    model.invalidate_cache()
    w = model.node_weights(dev)
    return model._params(dev, w)


t("invalidate + node_weights + _params", recompute)
t("_encode_rules_hip", lambda: model._encode_rules_hip(dev))
big_h = torch.cat([torch.tensor([x[0] for x in bb], device=dev) for bb in test_set.batches[:200]])
big_r = torch.cat([torch.tensor([x[1] for x in bb], device=dev) for bb in test_set.batches[:200]])


def step():
    model.invalidate_cache()
    return model.forward_rows(big_h, big_r, None)


ev = {}
with torch.no_grad():
    for _ in range(3):
        model.invalidate_cache()
        model.forward_rows(big_h, big_r, None, events=ev)
torch.cuda.synchronize()
print("events start->base (the step's head on the GPU timeline): %.3f ms" % ev["start"].elapsed_time(ev["base"]))
