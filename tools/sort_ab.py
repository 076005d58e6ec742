"""A/B of phase B's sort-window width (rnnl_debug_sort_bits) on the GPU box:
per width, the FB15k-237 bias-feature grounding + scoring alone (one
untimed-stream launch over the split, bench.isolated_ground_ms), its bucket
entries, the WN18RR ground + PNA alone, the kinship step and the
reference-API per-batch loop (first 300 FB15k-237 test batches).
Usage: python tools/sort_ab.py [bits ...]   (-1 = the default)"""
import contextlib
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from rnnlogic_amd import _native  # noqa: E402

dev = torch.device("cuda:0")
bits_list = [int(x) for x in sys.argv[1:]] or [-1, 11]
with contextlib.redirect_stdout(sys.stderr):
    graph, test_set, model, rows = bench.build_workload("bias")
    wmodel, wh, wr, wgraph, _, _ = bench.wn18rr_model(dev, full=True)
model = model.to(dev).eval()
h = torch.from_numpy(np.ascontiguousarray(rows[:, 0])).to(dev)
r = torch.from_numpy(np.ascontiguousarray(rows[:, 1])).to(dev)
hs = [torch.tensor([x[0] for x in b], device=dev) for b in test_set.batches[:300]]
rs = [torch.tensor([x[1] for x in b], device=dev) for b in test_set.batches[:300]]
for bits in bits_list * 2:  # two rounds: box drift shows as a round difference
    _native.call("rnnl_debug_sort_bits", bits)
    ms = [bench.isolated_ground_ms(model, graph, h, r, dev) for _ in range(4)][1:]
    tot = np.zeros(2, dtype=np.int64)
    with torch.no_grad():
        model.ground(h, r, None, totals=tot)
    wms = [bench.isolated_ground_ms(wmodel, wgraph, wh, wr, dev) for _ in range(4)][1:]
    with torch.no_grad():
        for k in range(3):
            model(hs[k], rs[k], None)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for a, b in zip(hs, rs):
            model(a, b, None)
        torch.cuda.synchronize()
        pb = (time.perf_counter() - t0) / len(hs) * 1e3
    print("bits %3d: FB ground+score %s ms, entries %d, candidates %d | WN ground+pna %s ms | per-batch %.4f ms"
          % (bits, " ".join("%.3f" % x for x in ms), tot[1], tot[0], " ".join("%.3f" % x for x in wms), pb),
          flush=True)
_native.call("rnnl_debug_sort_bits", -1)
