"""Wall time per batch of TrainerPredictor.train on FB15k-237 (diagnostic; GPU
box): the bench model (PredictorPlus(lstm, sum) + RotatE D = 1000) and the
final PredictorPlus stage of run_rnnlogic.py (emb, sum, bias), each with the
training lookahead on (prefetch_depth 2, the default) and off (0).
Usage: python tools/train_timing.py [n_batches] [profile]
`profile`: torch.profiler over one train() call of each model (depth 2)
instead, top ops by host time; `cprofile`: the Python profiler over it
(where the host time of a step goes, by function)."""
import contextlib
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from rnnlogic_amd.predictors import PredictorPlus  # noqa: E402
from rnnlogic_amd.trainer import TrainerPredictor  # noqa: E402

nb = int(sys.argv[1]) if len(sys.argv) > 1 else 200
prof = sys.argv[2] if len(sys.argv) > 2 else None
dev = torch.device("cuda:0")
with contextlib.redirect_stdout(sys.stderr):
    graph, test_set, rot_model, rows = bench.build_workload("RotatE")
    train_set = rot_model.train_set
    emb_model = PredictorPlus(graph, hidden_dim=16)
    emb_model.set_rules(bench.datasets.rule_file("FB15k-237"))
for name, model in (("emb_sum_bias", emb_model), ("lstm_sum_rotate", rot_model)):
    model = model.to(dev)
    if prof:
        model.prefetch_depth = 2
        opt = torch.optim.Adam(model.parameters(), lr=5e-3)
        solver = TrainerPredictor(model, train_set, None, test_set, opt, gpus=[0])
        solver.train(batch_per_epoch=nb, smoothing=0.2, print_every=10 ** 9)
        torch.cuda.synchronize()
        print("== %s, %d batches" % (name, nb))
        if prof == "cprofile":
            import cProfile
            import pstats
            pr = cProfile.Profile()
            pr.enable()
            solver.train(batch_per_epoch=nb, smoothing=0.2, print_every=10 ** 9)
            torch.cuda.synchronize()
            pr.disable()
            pstats.Stats(pr, stream=sys.stdout).sort_stats("tottime").print_stats(45)
            continue
        acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
        with torch.profiler.profile(activities=acts) as p:
            solver.train(batch_per_epoch=nb, smoothing=0.2, print_every=10 ** 9)
            torch.cuda.synchronize()
        print(p.key_averages().table(sort_by="self_cpu_time_total", row_limit=30, max_name_column_width=60))
        continue
    for depth in (2, 0):
        model.prefetch_depth = depth
        opt = torch.optim.Adam(model.parameters(), lr=5e-3)
        solver = TrainerPredictor(model, train_set, None, test_set, opt, gpus=[0])
        solver.train(batch_per_epoch=20, smoothing=0.2, print_every=10 ** 9)  # warm-up (shapes, tables)
        wall = []
        for n in (nb, 2 * nb):  # the difference: per-batch cost without train()'s fixed epoch setup
            torch.cuda.synchronize()
            t = time.perf_counter()
            solver.train(batch_per_epoch=n, smoothing=0.2, print_every=10 ** 9)
            torch.cuda.synchronize()
            wall.append(time.perf_counter() - t)
        ms = (wall[1] - wall[0]) * 1e3 / nb
        fixed = (2 * wall[0] - wall[1]) * 1e3
        print("%s prefetch_depth %d: %.3f ms per batch (train() over %d and %d batches: %.3f / %.3f s; fixed "
              "per-call setup %.0f ms: make_batches + the row table; dropped lookaheads %d)"
              % (name, depth, ms, nb, 2 * nb, wall[0], wall[1], fixed, getattr(model, "prefetch_dropped", 0)),
              flush=True)
