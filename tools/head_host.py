"""Host (CPU) time of the per-step head of the bench step — invalidate_cache,
the rule encoder with the node records, the parameter block — enqueued
without synchronising, so the figure is the Python + launch cost alone
(diagnostic; GPU box): python tools/head_host.py"""
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
N = 200


def host(name, fn):
    with torch.no_grad():
        for _ in range(10):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(N):
            fn()
        el = time.perf_counter() - t0
        torch.cuda.synchronize()
    print("%-45s %8.1f us host per call" % (name, el / N * 1e6))


def head():
    model.invalidate_cache()
    w = model.node_weights(dev)
    return model._params(dev, w)


host("invalidate + node_weights + _params", head)
host("node_weights (cache hit) + _params", lambda: model._params(dev, model.node_weights(dev)))
host("_encode_rules_hip (trie, no records)", lambda: model._encode_rules_hip(dev))
host("torch.cuda.current_stream", lambda: torch.cuda.current_stream(dev).cuda_stream)
