"""Bucket-entry statistics of the scoring pass's work units (diagnostic; GPU
box): python tools/entry_stats.py [fb|wn]

Per candidate its bucket-entry count (rules-with-paths); per 64-candidate
chunk of a query (the scoring pass's wave unit) the maximum over its lanes —
a lane-per-candidate walk costs the wave max, not the mean.  Prints totals and
what a cooperative walk of long lists (> T entries, the whole wave on one
candidate) would leave."""
import contextlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

dev = torch.device("cuda:0")
WN = len(sys.argv) > 1 and sys.argv[1] == "wn"
with contextlib.redirect_stdout(sys.stderr):
    if WN:
        from rnnlogic_amd.data import KnowledgeGraph, TestDataset, TrainDataset, ValidDataset
        from rnnlogic_amd.predictors import PredictorPlus
        path = bench.datasets.materialize("wn18rr", with_rotate=True)
        graph = KnowledgeGraph(path)
        TrainDataset(graph, 32)
        ValidDataset(graph, 32)
        test_set = TestDataset(graph, 32)
        model = PredictorPlus(graph, type="emb", num_layers=3, hidden_dim=16, entity_feature="RotatE",
                              aggregator="pna", embedding_path=bench.datasets.rotate_path("wn18rr"))
        model.set_rules(bench.datasets.rule_file("wn18rr"))
        rows = np.asarray([x for b in test_set.batches for x in b], dtype=np.int64)
    else:
        graph, test_set, model, rows = bench.build_workload("RotatE")
model = model.to(dev).eval()
h = torch.from_numpy(rows[:, 0]).to(dev)
r = torch.from_numpy(rows[:, 1]).to(dev)
with torch.no_grad():
    row, ent, ce, node, count = model.ground_coo(h, r)
row = row.cpu().numpy()
nent = np.bincount(ce.cpu().numpy(), minlength=len(row))
C, P = len(row), int(nent.sum())
# candidate index within its row -> chunk id (row, idx // 64)
starts = np.r_[0, np.flatnonzero(np.diff(row)) + 1]
idx = np.arange(C) - np.repeat(starts, np.diff(np.r_[starts, C]))
chunk = np.unique(row * 1_000_000 + idx // 64, return_inverse=True)[1]
nch = chunk.max() + 1
cmax = np.zeros(nch, dtype=np.int64)
np.maximum.at(cmax, chunk, nent)
print("candidates %d, entries %d (%.2f per candidate), chunks %d" % (C, P, P / C, nch))
nn = max(model.native_rules(dev).n_nodes, 1)
distinct = len(np.unique(ce.cpu().numpy().astype(np.int64) * nn + node.cpu().numpy()))
print("distinct (candidate, trie node) pairs %d: entries / distinct = %.4f" % (distinct, P / distinct))
print("entries per candidate: p50 %d p90 %d p99 %d p99.9 %d max %d" % tuple(
    np.percentile(nent, [50, 90, 99, 99.9]).tolist() + [nent.max()]))
print("lane-per-candidate walk: sum over chunks of max entries %d (%.1f per chunk; %.1fx the entries / 64)"
      % (cmax.sum(), cmax.mean(), cmax.sum() / (P / 64)))
for T in (8, 16, 32, 64):
    small = np.where(nent <= T, nent, 0)
    smax = np.zeros(nch, dtype=np.int64)
    np.maximum.at(smax, chunk, small)
    big = nent[nent > T]
    coop = np.ceil(big / 64).sum()
    print("T=%d: %d long candidates (%.3f%%), per-lane part %d + cooperative rounds %d = %d wave-steps"
          % (T, len(big), 100 * len(big) / C, smax.sum(), coop, smax.sum() + coop))
