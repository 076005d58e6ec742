"""Time the HIP LSTM rule encoder on the FB15k-237 bench model's 131,883
rules (diagnostic; GPU box) and check it against torch's LSTM:
python tools/enc_time.py — the trie form (one step per prefix node) and the
per-rule form, and the encoder + node-weight records as the bench's head."""
import contextlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

dev = torch.device("cuda:0")
with contextlib.redirect_stdout(sys.stderr):
    graph, test_set, model, rows = bench.build_workload("RotatE")
model = model.to(dev).eval()
with torch.no_grad():
    res = {}
    for trie in (True, False):
        model.encoder_trie = trie
        res[trie] = bench.time_forward(lambda: model._encode_rules_hip(dev), 20) * 1e3
    got = model._encode_rules_hip(dev)
    want = model.encode_rules(model.rule_features.to(dev))
    model.encoder_trie = True  # the bench's head: the trie encoder with the SUM records in its launches
    nw = bench.time_forward(lambda: (model.invalidate_cache(), model.node_weights(dev)), 20) * 1e3
print("encoder: trie %.3f ms, per-rule %.3f ms; encoder + node weights %.3f ms; max |hip - torch| %.2e"
      % (res[True], res[False], nw, (got - want).abs().max().item()))
