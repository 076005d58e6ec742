"""Config 2 (kinship lstm/sum/none) diagnostics on the GPU box: the grounding
kernel's per-phase cycles (rnnl_debug_profile) and the step's kernels under
rocprofv3 --kernel-trace (run it under the profiler; steps split by
tools/step_trace.py DIR lstm_trie_level_kernel 3).
Usage: python tools/kinship_profile.py"""
import contextlib
import os
import random
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from rnnlogic_amd import _native, datasets  # noqa: E402
from rnnlogic_amd.data import KnowledgeGraph, TestDataset, TrainDataset, ValidDataset  # noqa: E402
from rnnlogic_amd.predictors import PredictorPlus  # noqa: E402

dev = torch.device("cuda:0")
random.seed(1)
np.random.seed(1)
torch.manual_seed(1)
with contextlib.redirect_stdout(sys.stderr):
    graph = KnowledgeGraph(datasets.materialize("kinship"))
    TrainDataset(graph, 32)
    ValidDataset(graph, 32)
    test_set = TestDataset(graph, 32)
    model = PredictorPlus(graph, type="lstm", num_layers=3, hidden_dim=16, entity_feature="none", aggregator="sum")
    model.set_rules(datasets.rule_file("kinship"))
model = model.to(dev).eval()
rows = np.asarray([x for b in test_set.batches for x in b], dtype=np.int64)
h = torch.from_numpy(np.ascontiguousarray(rows[:, 0])).to(dev)
r = torch.from_numpy(np.ascontiguousarray(rows[:, 1])).to(dev)


def step():
    model.invalidate_cache()
    with torch.no_grad():
        return model.forward_rows(h, r, None)


for pm in (0, 1):  # the SUM scoring pass's pair memo off / on (rnnl_debug_pair_memo)
    _native.call("rnnl_debug_pair_memo", pm)
    print("kinship step, pair memo %d: %.3f ms" % (pm, bench.time_forward(step, 50) * 1e3))
ms = bench.time_forward(step, 50) * 1e3
with torch.no_grad():
    prof = torch.zeros(13, dtype=torch.int64, device=dev)
    _native.call("rnnl_debug_profile", prof.data_ptr())
    model.ground_early = False
    step()
    torch.cuda.synchronize()
    _native.call("rnnl_debug_profile", None)
    model.ground_early = True
p = prof.cpu().tolist()
nq = max(p[3], 1)
print("kinship step %.3f ms; queries %d  contributions/q %.1f  candidates/q %.1f" % (ms, p[3], p[4] / nq, p[5] / nq))
for name, v in zip(["prologue", "grounding(A)", "candidates(B)"], p[:3]):
    print("  %-14s %10.0f cycles/query" % (name, v / nq))
for name, v in zip(["B mark+slots", "B count+records", "B scatter", "A node+scan", "A item+scan", "A edges",
                    "A compaction"], p[6:13]):
    print("  %-14s %10.0f cycles/query" % (name, v / nq))
