"""Where the FB15k-237 RotatE pass loses time beside the side-stream kernels
(diagnostic; GPU box): python tools/interference.py [fb|wn]
(wn: the WN18RR config-3 model, PNA aggregator, RotatE D = 500)

Times the bench's RotatE launch (HIP events on its stream) in five settings:
  store       alone, plain stores (RotatE.score_into)
  atomic      alone, atomic adds into zeroed rows (the overlap's mode)
  +ground     atomic, ground_kernel on a side stream beside it (256 workgroups)
  +score      atomic, the grounding done first, the scoring pass beside it
  +score_late the same, the scoring pass enqueued after RotatE's launch
  +both       atomic, grounding then scoring on the side stream (the forward's order)
  forward     the whole overlapped forward (forward_rows), RotatE's events
and the side kernel's own time where there is one."""
import contextlib
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from rnnlogic_amd import _native  # noqa: E402

dev = torch.device("cuda:0")
WN = len(sys.argv) > 1 and sys.argv[1] == "wn"
with contextlib.redirect_stdout(sys.stderr):
    if WN:
        import numpy as np
        from rnnlogic_amd.data import KnowledgeGraph, TestDataset, TrainDataset, ValidDataset
        from rnnlogic_amd.predictors import PredictorPlus
        path = bench.datasets.materialize("wn18rr", with_rotate=True)
        torch.manual_seed(1)
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
AGG = _native.AGG_PNA if WN else _native.AGG_SUM
h = torch.from_numpy(rows[:, 0]).to(dev)
r = torch.from_numpy(rows[:, 1]).to(dev)
nq, E = h.numel(), graph.entity_size
out = torch.empty((nq, E), dtype=torch.float32, device=dev)
main = torch.cuda.current_stream(dev)
side = torch.cuda.Stream(dev)
g = model.graph.device_graph(dev)
nr = model.native_rules(dev)
REPS = 3


def ev():
    return torch.cuda.Event(enable_timing=True)


def ground(stream, wg):
    ncs = torch.empty(nq, dtype=torch.int32, device=dev)
    ws = model._workspace(dev, nq, model.capacity_scale)
    _native.call("rnnl_predictorplus_ground", g, nr.ptr, AGG, h.data_ptr(), r.data_ptr(), None, nq,
                 ncs.data_ptr(), ws.data_ptr(), ws.numel(), model.capacity_scale, wg, stream.cuda_stream)
    return ws, ncs


def score(stream, ws, ncs, params, wg):
    _native.call("rnnl_predictorplus_score", g, nr.ptr, ctypes.byref(params), h.data_ptr(), r.data_ptr(), nq,
                 out.data_ptr(), None, ncs.data_ptr(), None, ws.data_ptr(), ws.numel(), model.capacity_scale, wg, 2,
                 stream.cuda_stream)


res = {}
with torch.no_grad():
    params, keep = model._params(dev, model.node_weights(dev))
    for mode in ("store", "atomic", "+ground", "+score", "+score_late", "+both", "forward", "forward_1piece"):
        rot, sid = [], []
        for k in range(REPS + 1):
            if mode.startswith("forward"):
                model.rotate_yield = mode == "forward"
                evs = {}
                model.invalidate_cache()
                model.forward_rows(h, r, None, events=evs)
                torch.cuda.synchronize(dev)
                if k:
                    rot.append(evs["base"].elapsed_time(evs["ground"]))
                    sid.append(evs["base"].elapsed_time(evs["end"]))
                continue
            if mode != "store":
                out.zero_()
            pre = None
            if mode in ("+score", "+score_late"):
                pre = ground(main, 0)
            torch.cuda.synchronize(dev)
            a0, a1, s0, s1 = ev(), ev(), ev(), ev()
            if mode in ("+ground", "+score", "+both"):
                side.wait_stream(main)
                with torch.cuda.stream(side):
                    s0.record(side)
                    if mode == "+ground":
                        ground(side, 256)
                    elif mode == "+both":
                        ws, ncs = ground(side, 256)
                        score(side, ws, ncs, params, 256)
                    else:
                        score(side, pre[0], pre[1], params, 256)
                    s1.record(side)
            a0.record(main)
            model.RotatE.score_into(h, r, out, accumulate=(False if mode == "store" else 2))
            a1.record(main)
            if mode == "+score_late":  # enqueued behind RotatE's launch: its workgroups wait for room
                with torch.cuda.stream(side):
                    s0.record(side)
                    score(side, pre[0], pre[1], params, 256)
                    s1.record(side)
            torch.cuda.synchronize(dev)
            if k:
                rot.append(a0.elapsed_time(a1))
                if mode not in ("store", "atomic"):
                    sid.append(s0.elapsed_time(s1))
        res[mode] = (sum(rot) / len(rot), sum(sid) / len(sid) if sid else None)
        print("%-8s rotate %.3f ms%s" % (mode, res[mode][0],
                                          "  side %.3f ms" % res[mode][1] if res[mode][1] else ""), flush=True)
