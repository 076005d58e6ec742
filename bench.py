"""Benchmark: PredictorPlus forward queries/sec on FB15k-237 (BASELINE.json).

Workload (one "step"): the PredictorPlus forward over every batch of the
FB15k-237 test split as TestDataset builds them (1514 single-relation batches
of <= 32 queries, 40,932 queries), eval mode, edges_to_remove=None — the
reference's evaluate() forward (src/trainer.py:161-180).  Model = config 4 of
BASELINE.json: PredictorPlus(type=lstm, num_layers=3, hidden_dim=16,
aggregator=sum) from config/FB15k-237_predictorplus.yaml with the RotatE
entity feature (D=1000, gamma=9), rules = data/FB15k-237/rnnlogic_rules.txt
(131,883 rules, body length <= 3).  The FB15k-237 train graph and RotatE
tables are absent from the reference mount, so both are seeded synthetic
(rnnlogic_amd/datasets.py); the test split and rules are real.

Timed region per step: rule embeddings (LSTM over all rules) + node
aggregates, the RotatE base-score kernel and the fused grounding/aggregation/
MLP kernel over all rows, and the overflow status check — inputs already in
HBM.  N ranks (torchrun, one per GPU) split the test batches with the
reference evaluate()'s DistributedSampler(test_set, N, rank) (shuffled with
seed 0, padded by repeating batches so every rank holds the same count;
src/trainer.py:150), the KG replicated on every GPU: the total work is fixed
("scaling": "strong") and `value` counts each of the split's 40,932 queries
once (the sampler's padding duplicates are extra work, not extra queries).
There is no collective in the timed region (queries are independent;
DESIGN.md "Multi-GPU").  At N > 1 a secondary line `weak_replicated` times
every rank on the whole split.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--feature RotatE|bias]
"""
import argparse
import contextlib
import json
import os
import random
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from rnnlogic_amd import datasets  # noqa: E402
from rnnlogic_amd.data import KnowledgeGraph, TestDataset, TrainDataset, ValidDataset  # noqa: E402
from rnnlogic_amd.predictors import PredictorPlus  # noqa: E402

METRIC = "queries/sec PredictorPlus forward, FB15k-237, 1/2/4/8 GPU; MRR parity"
HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md: 8.0 TB/s spec
FP32_PEAK_TFS = 157.3     # MI355X_MICROARCH.md: FP32 vector == FP32 matrix peak


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def build_workload(feature):
    path = datasets.materialize("FB15k-237", with_rotate=(feature == "RotatE"))
    # run_predictorplus.py order: set_seed, graph, train/valid/test datasets, model
    random.seed(1)
    np.random.seed(1)
    torch.manual_seed(1)
    graph = KnowledgeGraph(path)
    train_set = TrainDataset(graph, 32)
    ValidDataset(graph, 32)
    test_set = TestDataset(graph, 32)
    model = PredictorPlus(graph, type="lstm", num_layers=3, hidden_dim=16, entity_feature=feature,
                          aggregator="sum",
                          embedding_path=datasets.rotate_path("FB15k-237") if feature == "RotatE" else None)
    model.set_rules(datasets.rule_file("FB15k-237"))
    rows = np.asarray([x for b in test_set.batches for x in b], dtype=np.int64)
    model.train_set = train_set  # for the train-mode line (not a module attribute of the reference)
    return graph, test_set, model, rows


def shard_rows(test_set, world, rank):
    """Rows of this rank's batches under the reference evaluate()'s sampler:
    DistributedSampler(test_set, world, rank) — shuffle with seed 0, epoch 0,
    padded by repeating indices so len % world == 0 (src/trainer.py:150).
    Returns (rows (n, 3) int64, batch indices)."""
    from torch.utils import data as torch_data
    idx = list(iter(torch_data.DistributedSampler(test_set, world, rank)))
    rows = np.asarray([x for i in idx for x in test_set.batches[i]], dtype=np.int64).reshape(-1, 3)
    return rows, idx


def shard_balance_line(model, test_set, dev, full_ms, worlds=(2, 4, 8), reps=3):
    """Prediction of the N-GPU load balance on one GPU (no scaling claim):
    each DistributedSampler(test_set, N, k) shard (the rows rank k of an
    N-GPU bench runs, sampler padding included) timed alone on cuda:0 with
    the same step as `value` (rule aggregates recomputed, RotatE + grounding +
    scoring).  The N-GPU step is the slowest shard (ranks are independent
    until the closing barrier), so the implied strong-scaling efficiency is
    T_1 / (N x max_k T_k); the shards' RotatE and grounding times show which
    one sets it.  Plus the DDP gradient size of the headline model's training
    step (every trainable parameter is all-reduced each step)."""
    out = {}
    for world in worlds:
        shard_ms, shard_rows_n, rot_ms, ground_ms = [], [], [], []
        for k in range(world):
            rows, _ = shard_rows(test_set, world, k)
            sh = torch.from_numpy(np.ascontiguousarray(rows[:, 0])).to(dev)
            sr = torch.from_numpy(np.ascontiguousarray(rows[:, 1])).to(dev)

            def st(ev=None):
                model.invalidate_cache()
                with torch.no_grad():
                    return model.forward_rows(sh, sr, None, events=ev)
            shard_ms.append(time_forward(st, reps) * 1e3)
            ev = {}
            st(ev)
            torch.cuda.synchronize(dev)
            rot_ms.append(ev["base"].elapsed_time(ev["ground"]))
            ground_ms.append(isolated_ground_ms(model, model.graph, sh, sr, dev))
            shard_rows_n.append(len(rows))
            del sh, sr
        mx, mean = max(shard_ms), float(np.mean(shard_ms))
        slow = int(np.argmax(shard_ms))
        out["N=%d" % world] = {
            "shard_ms": [round(x, 3) for x in shard_ms], "shard_rows": shard_rows_n,
            "rotate_ms": [round(x, 3) for x in rot_ms], "ground_score_alone_ms": [round(x, 3) for x in ground_ms],
            "max_ms": round(mx, 3), "mean_ms": round(mean, 3), "balance_mean_over_max": round(mean / mx, 4),
            "implied_strong_efficiency": round(full_ms / (world * mx), 4),
            "slowest_shard": slow,
            "slowest_grounding_outlasts_rotate": bool(ground_ms[slow] > rot_ms[slow])}
    n_grad = sum(p.numel() for p in model.parameters())
    out["ddp_gradient"] = {
        "parameters": int(n_grad), "bytes_per_step": int(4 * n_grad),
        "rotate_share": round(float(model.RotatE.eemb.numel() + model.RotatE.remb.numel()) / n_grad, 4)
        if hasattr(model, "RotatE") else 0.0,
        "note": "fp32 gradients all-reduced by DDP each training step (trainer.py:56-60; every parameter, "
                "find_unused_parameters=True); not measured here (no multi-GPU run from this box)"}
    out["note"] = ("each DistributedSampler shard timed alone on one GPU (the N-GPU step is the slowest shard); "
                   "T_1 = the full split's step on the same GPU; prediction only, not a scaling measurement")
    return out


def rank_info(model, dev, local, world, backend):
    """This rank's placement: LOCAL_RANK, the device it runs on, the device
    of its graph handle and of the forward's side streams
    (rnnl_forward_host_info), and the process group's world size."""
    import ctypes
    import socket
    from rnnlogic_amd import _native
    info = (ctypes.c_int32 * 4)()
    _native.call("rnnl_forward_host_info", model.graph.device_graph(dev), info)
    return {"rank": dist.get_rank() if dist.is_initialized() else 0, "local_rank": local,
            "host": socket.gethostname(), "cuda_device": dev.index,
            "graph_device": int(info[0]), "side_stream_devices": [int(info[1]), int(info[2])],
            "devices_with_forward_resources": int(info[3]),
            "world_size_seen": dist.get_world_size() if dist.is_initialized() else 1,
            "world_size_env": world, "backend": dist.get_backend() if dist.is_initialized() else None,
            "placement_ok": int(info[0]) == dev.index and all(x in (-1, dev.index) for x in info[1:3])}


def train_rows(train_set, n_rows):
    """The first train batches (sampler order of trainer.py:51-56 is a
    permutation; batch order does not matter for throughput) up to n_rows:
    (h, r, edges_to_remove) — the train-mode forward input (data.py:201-219)."""
    hs, rs, es, n = [], [], [], 0
    for i in range(len(train_set)):
        all_h, all_r, _, _, etr = train_set[i]
        hs.append(all_h)
        rs.append(all_r)
        es.append(etr)
        n += len(all_h)
        if n >= n_rows:
            break
    return torch.cat(hs), torch.cat(rs), torch.cat(es), i + 1


def time_forward(fn, reps, warmup=2):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def host_cores():
    """The host's CPU count (nproc), the CPUs this process may run on (its
    affinity mask) and the cgroup CPU quota, if any; `usable` = the smallest."""
    nproc = os.cpu_count() or 1
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = nproc
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(period)))
    except (OSError, ValueError):
        pass
    usable = min(affinity, quota) if quota else affinity
    return {"nproc": nproc, "affinity": affinity, "cgroup_quota": quota, "usable": usable}


def cpu_baseline(path, model, rows, threads, cores, budget_s=20.0):
    """The reference's own C++ path counter (miner/rnnlogic.cpp rule_destination
    via ReasoningPredictor::out_test, compiled from the reference sources into
    oracle/_ref) on the host cores, over a bounded prefix of the test split."""
    from oracle import ground_c
    if not os.path.exists(ground_c.REF_LIB):
        return None
    miner = ground_c.RefMiner(path)
    try:
        sample = 2048
        sec, _ = miner.out_test_timed(model.rules, threads, sample)
        # scale the sample to ~budget_s of CPU work (bounded by the split size)
        target = int(min(len(rows), max(sample, sample * budget_s / max(sec, 1e-3))))
        if target > sample:
            miner.close()
            miner = ground_c.RefMiner(path)
            sec, _ = miner.out_test_timed(model.rules, threads, target)
            sample = target
    finally:
        miner.close()
    return {"value": round(sample / sec, 1), "unit": "queries/s", "cores": threads, "kind": "reference",
            "host": cores,
            "sample": "first %d FB15k-237 test triples, grounding only (ReasoningPredictor::out_test, "
                      "%d pthreads = the CPUs this process may use; host nproc %d), %.1f s"
                      % (sample, threads, cores["nproc"], sec)}


def reference_pytorch_baseline(model, graph, test_set, dev, feature, budget_s=15.0):
    """The reference PyTorch predictor (its dense torch-eager formulation,
    oracle/reference_torch.py, op for op after src/data.py:136-173 and
    src/predictors.py:210-271) on the same GPU, same weights and rules, over
    the first test batches in TestDataset order until ~budget_s elapse."""
    from oracle import reference_np as ref
    from oracle import reference_torch as rt
    g = ref.Graph(graph.data_path)
    rules = ref.Rules(datasets.rule_file("FB15k-237"), g.relation_size)
    rot = ref.load_rotate(datasets.rotate_path("FB15k-237")) if feature == "RotatE" else None
    sd = {k: v.detach().cpu().numpy() for k, v in model.state_dict().items() if not k.startswith("RotatE.")}
    m = rt.Model(sd, {"type": model.type, "num_layers": model.num_layers, "aggregator": model.aggregator,
                      "entity_feature": feature}, g, rules, dev, rot)
    b0 = test_set.batches[0]
    m.forward([x[0] for x in b0], [x[1] for x in b0], None)  # warm-up (allocator, kernels)
    torch.cuda.synchronize(dev)
    n, nb, t0 = 0, 0, time.perf_counter()
    for b in test_set.batches:
        m.forward([x[0] for x in b], [x[1] for x in b], None)
        n += len(b)
        nb += 1
        if time.perf_counter() - t0 > budget_s:
            break
    torch.cuda.synchronize(dev)
    sec = time.perf_counter() - t0
    return {"value": round(n / sec, 2), "unit": "queries/s", "device": "cuda:0 (same GPU)", "kind": "port",
            "sample": "first %d FB15k-237 test batches (%d queries) in TestDataset order, %.1f s" % (nb, n, sec),
            "note": "reference PyTorch predictor, dense torch-eager (oracle/reference_torch.py)"}


def csrc_fingerprint():
    """sha256 over the HIP/C++ sources of the library (rnnlogic_amd/csrc),
    name-ordered: the stamp tools/pmc_traffic.py writes into the committed
    traffic summaries (no git on the GPU box)."""
    import hashlib
    d = os.path.join(REPO, "rnnlogic_amd", "csrc")
    h = hashlib.sha256()
    for name in sorted(os.listdir(d)):
        if name.endswith((".hip", ".cpp", ".h")) or name == "Makefile":
            h.update(name.encode())
            with open(os.path.join(d, name), "rb") as f:
                h.update(f.read())
    return h.hexdigest()


def isolated_ground_ms(model, graph, h, r, dev):
    """Device time of the rule part of a bias-feature forward alone: one
    untimed one-stream launch over all rows — the bias-row fill of the score
    rows (rnnl_fill_rows: SURVEY §8(d)'s 4 B |E| score write) then
    rnnl_predictorplus_forward (grounding + scoring) — so that the time, the
    algorithmic bytes and the counter traffic (fill_rows_kernel included)
    describe the same kernels."""
    import ctypes
    from rnnlogic_amd import _native
    nq = h.numel()
    with torch.no_grad():
        scratch = torch.empty((nq, graph.entity_size), dtype=torch.float32, device=dev)
        ncs = torch.empty(nq, dtype=torch.int32, device=dev)
        params, keep = model._params(dev, model.node_weights(dev))
        ws = model._workspace(dev, nq, model.capacity_scale)
        bias = torch.randn(graph.entity_size, device=dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        st = torch.cuda.current_stream(dev).cuda_stream
        torch.cuda.synchronize(dev)
        e0.record()
        _native.call("rnnl_fill_rows", bias.data_ptr(), nq, graph.entity_size, scratch.data_ptr(), st)
        _native.call("rnnl_predictorplus_forward", model.graph.device_graph(dev), model.native_rules(dev).ptr,
                     ctypes.byref(params), h.data_ptr(), r.data_ptr(), None, nq, scratch.data_ptr(), None,
                     ncs.data_ptr(), None, ws.data_ptr(), ws.numel(), model.capacity_scale, st)
        e1.record()
        _native.check(_native.lib().rnnl_forward_status(ws.data_ptr(), st))
        del scratch, keep
        return e0.elapsed_time(e1)


def wn18rr_model(dev, full=False):
    """The config-3 model (PredictorPlus(emb, pna) + RotatE D = 500) and the
    WN18RR test split's rows on `dev`, in run_predictorplus.py's order."""
    path = datasets.materialize("wn18rr", with_rotate=True)
    random.seed(1)
    np.random.seed(1)
    torch.manual_seed(1)
    with contextlib.redirect_stdout(sys.stderr):
        graph = KnowledgeGraph(path)
        TrainDataset(graph, 32)
        ValidDataset(graph, 32)
        test_set = TestDataset(graph, 32)
        model = PredictorPlus(graph, type="emb", num_layers=3, hidden_dim=16, entity_feature="RotatE",
                              aggregator="pna", embedding_path=datasets.rotate_path("wn18rr"))
        model.set_rules(datasets.rule_file("wn18rr"))
    model = model.to(dev).eval()
    rows = np.asarray([x for b in test_set.batches for x in b], dtype=np.int64)
    h = torch.from_numpy(np.ascontiguousarray(rows[:, 0])).to(dev)
    r = torch.from_numpy(np.ascontiguousarray(rows[:, 1])).to(dev)
    return (model, h, r, graph, test_set, rows) if full else (model, h, r)


def wn18rr_line(dev, reps=10):
    """Config 3 of BASELINE.json as a secondary line: PredictorPlus(emb, pna)
    + RotatE(D=500, gamma=6) over the WN18RR test split (206 batches, 6,268
    queries, real rnnlogic_rules.txt: 7,386 rules, L <= 5), seeded synthetic
    train graph and RotatE tables — the same timed step as `value` (rule
    aggregates recomputed, RotatE + grounding + PNA scoring), plus the
    grounding/scoring kernels alone and the RotatE kernel's VALU roofline."""
    model, h, r, graph, test_set, rows = wn18rr_model(dev, full=True)

    def step():
        model.invalidate_cache()
        with torch.no_grad():
            return model.forward_rows(h, r, None)
    sec = time_forward(step, reps)
    nq, E, D = len(rows), graph.entity_size, model.RotatE.emb_dim
    with torch.no_grad():
        tmp = torch.empty((nq, E), dtype=torch.float32, device=dev)
        rot_ms = time_forward(lambda: model.RotatE.score_into(h, r, tmp), reps) * 1e3
        del tmp
    ground_ms = isolated_ground_ms(model, graph, h, r, dev)
    flops = 7.0 * nq * E * D
    groof = grounding_roofline(algorithmic_work(model, graph, rows, name="wn18rr"), nq, E, ground_ms,
                               "ground_kernel<PNA> + score_pna_chunk_kernel",
                               measured="one untimed one-stream launch over all rows (isolated from RotatE)")
    return {"queries_per_s": round(nq / sec, 1), "ms_per_step": round(sec * 1e3, 3), "rows": nq,
            "batches": len(test_set), "rules": model.num_rules, "roofline_grounding": groof,
            "kernels_ms": {"rotate_alone": round(rot_ms, 3), "ground+score_isolated": round(ground_ms, 3)},
            "roofline_rotate": {"bound": "valu", "achieved": round(flops / (rot_ms * 1e-3) / 1e12, 2),
                                "peak": FP32_PEAK_TFS, "unit": "TFLOP/s",
                                "frac": round(flops / (rot_ms * 1e-3) / 1e12 / FP32_PEAK_TFS, 4),
                                "alg_flops": flops, "kernel": "rotate_direct_kernel (alone, one launch)"},
            "workload": "WN18RR test split, PredictorPlus(emb,3,16,pna) + RotatE(D=500,gamma=6); "
                        "rnnlogic_rules.txt (L<=5); seeded synthetic train graph and RotatE tables"}


def kinship_line(dev, reps=50):
    """Config 2 of BASELINE.json as a secondary line: PredictorPlus(lstm, 3,
    16, sum) without an entity feature on the kinship test split (178 batches,
    5,343 queries; the mined L <= 3 rule file, top 100 per relation: 2,500
    rules), real kinship train graph — the same timed step as `value`."""
    path = datasets.materialize("kinship")
    random.seed(1)
    np.random.seed(1)
    torch.manual_seed(1)
    with contextlib.redirect_stdout(sys.stderr):
        graph = KnowledgeGraph(path)
        TrainDataset(graph, 32)
        ValidDataset(graph, 32)
        test_set = TestDataset(graph, 32)
        model = PredictorPlus(graph, type="lstm", num_layers=3, hidden_dim=16, entity_feature="none",
                              aggregator="sum")
        model.set_rules(datasets.rule_file("kinship"))
    model = model.to(dev).eval()
    rows = np.asarray([x for b in test_set.batches for x in b], dtype=np.int64)
    h = torch.from_numpy(np.ascontiguousarray(rows[:, 0])).to(dev)
    r = torch.from_numpy(np.ascontiguousarray(rows[:, 1])).to(dev)

    def step():
        model.invalidate_cache()
        with torch.no_grad():
            return model.forward_rows(h, r, None)
    sec = time_forward(step, reps)
    roof = grounding_roofline(algorithmic_work(model, graph, rows, name="kinship"), len(rows), graph.entity_size,
                              sec * 1e3, "ground_kernel + scoring (whole step: no entity feature)",
                              measured="the timed step (rule embeddings + node aggregates + grounding + scoring)")
    return {"queries_per_s": round(len(rows) / sec, 1), "ms_per_step": round(sec * 1e3, 3), "rows": len(rows),
            "batches": len(test_set), "rules": model.num_rules, "roofline": roof,
            "workload": "kinship test split, PredictorPlus(lstm,3,16,sum), entity_feature none; mined rules "
                        "(L<=3, top 100 per relation); real train graph"}


def per_batch_line(model, graph, test_set, dev):
    """The reference API's call pattern (src/trainer.py:150-173): one
    PredictorPlus.forward(all_h, all_r, None) per TestDataset batch (B <= 32,
    one relation) over the whole split, inputs already on the device.  Its
    roofline: the RotatE flops of every call over the loop's time (the same
    kernel as `value`, launched 1,514 times on 32 rows each)."""
    hs = [torch.tensor([x[0] for x in b], device=dev) for b in test_set.batches]
    rs = [torch.tensor([x[1] for x in b], device=dev) for b in test_set.batches]
    with torch.no_grad():
        for k in range(3):
            model(hs[k], rs[k], None)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for h, r in zip(hs, rs):
            model(h, r, None)
        torch.cuda.synchronize(dev)
        sec = time.perf_counter() - t0
    n = sum(len(b) for b in test_set.batches)
    out = {"queries_per_s": round(n / sec, 1), "ms": round(sec * 1e3, 3), "calls": len(hs),
           "ms_per_call": round(sec / len(hs) * 1e3, 4), "rows": n,
           "note": "PredictorPlus.forward once per TestDataset batch (the reference evaluate()'s loop), "
                   "device-resident inputs; same model as value"}
    if model.entity_feature == "RotatE":
        fl = 7.0 * n * graph.entity_size * model.RotatE.emb_dim
        out["roofline"] = {"bound": "valu", "achieved": round(fl / sec / 1e12, 2), "peak": FP32_PEAK_TFS,
                           "unit": "TFLOP/s", "frac": round(fl / sec / 1e12 / FP32_PEAK_TFS, 4),
                           "kernel": "rotate_direct_kernel (RotatE flops of all calls / loop time)"}
    return out


def train_step_line(model, solver, dev, n_steps=10, warmup=2):
    """TrainerPredictor.train_step (src/trainer.py:72-98) on FB15k-237 train
    batches with the bench model: per-step times of every timed step (a
    first-use cost of a new shape shows as an outlier, a steady cost does not)."""
    from rnnlogic_amd.data import DeviceTrainBatches
    opt = torch.optim.Adam(model.parameters(), lr=5e-3)
    solver.optimizer = opt
    dtb = DeviceTrainBatches(model.train_set, dev)
    model.train()
    batches = [[x.unsqueeze(0) for x in dtb[i]] for i in range(warmup + n_steps)]
    for b in batches[:warmup]:
        solver.train_step(model, b, 0.2)
    times, nrow = [], 0
    for b in batches[warmup:]:
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        solver.train_step(model, b, 0.2, sync=False)
        torch.cuda.synchronize(dev)
        times.append((time.perf_counter() - t) * 1e3)
        nrow += b[0].numel()
    model.eval()
    sec = sum(times) * 1e-3
    return {"queries_per_s": round(nrow / sec, 1), "ms_per_batch": round(sec * 1e3 / n_steps, 3),
            "ms_per_step": [round(x, 3) for x in times], "batches": n_steps, "rows": nrow,
            "note": "TrainerPredictor.train_step on FB15k-237 train batches (B=32, edge removal, RotatE feature, "
                    "Adam): forward + loss + backward + step, each step synchronised"}


def wn18rr_train_line(dev, n_steps=10, warmup=3):
    """Config 3's training step: TrainerPredictor.train_step on WN18RR train
    batches (B = 32, edge removal, Adam) for PredictorPlus(emb, 3, 16, pna) +
    RotatE(D = 500) — FuncToNode's statistics and their backward on the HIP
    path (predictors._PnaStats, csrc/pna_grad.hip), beside the same steps
    through torch autograd over the exported grounding COO (the round-5 path)."""
    from rnnlogic_amd.trainer import TrainerPredictor
    path = datasets.materialize("wn18rr", with_rotate=True)
    random.seed(1)
    np.random.seed(1)
    torch.manual_seed(1)
    with contextlib.redirect_stdout(sys.stderr):
        graph = KnowledgeGraph(path)
        train_set = TrainDataset(graph, 32)
        ValidDataset(graph, 32)
        test_set = TestDataset(graph, 32)
        model = PredictorPlus(graph, type="emb", num_layers=3, hidden_dim=16, entity_feature="RotatE",
                              aggregator="pna", embedding_path=datasets.rotate_path("wn18rr"))
        model.set_rules(datasets.rule_file("wn18rr"))
    model = model.to(dev)
    model.train_set = train_set
    solver = TrainerPredictor(model, train_set, None, test_set, None, gpus=[dev.index or 0])
    # a first pass over the batches: the dense layers' GEMM shapes (one per
    # candidate count) are selected on first use, for both paths alike
    train_step_line(model, solver, dev, n_steps=n_steps, warmup=warmup)
    model.fused_backward = False
    coo = train_step_line(model, solver, dev, n_steps=n_steps, warmup=warmup)
    model.fused_backward = True
    out = train_step_line(model, solver, dev, n_steps=n_steps, warmup=warmup)
    out["autograd_coo_ms_per_batch"] = coo["ms_per_batch"]
    out["note"] = ("TrainerPredictor.train_step on WN18RR train batches (B=32, edge removal, RotatE D=500 trainable, "
                   "Adam), each step synchronised: PNA statistics + backward in HIP (csrc/pna_grad.hip); "
                   "autograd_coo_ms_per_batch: the same steps through torch autograd over the grounding COO")
    return out


def recorded_em_full(path=os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles",
                                        "r05_em_full_fb.json")):
    """Config 5 end to end (tools/em_full_fb.py: the whole run_rnnlogic.py flow
    with config/FB15k-237.yaml's settings, 5 EM + 5 final iterations) — a
    recorded run (~170 s on one MI355X, too long for the default bench), read
    from profiles/, with the final PredictorPlus stage per batch."""
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    ph = d.get("phases_s", {})
    n_batches = 17258 * d.get("final_iters", 5)  # FB15k-237 train batches per final iteration
    return {"s": d.get("wall_s"), "phases_s": ph,
            "final_train_ms_per_batch": round(ph.get("final_train", 0.0) * 1e3 / n_batches, 3),
            "best_valid_mrr": d.get("best_valid_mrr"), "source": os.path.relpath(path, os.path.dirname(path) + "/.."),
            "note": "recorded run of tools/em_full_fb.py (not re-run by bench.py); " + d.get("workload", "")}


def em_iteration_line(dev, pre_epochs=200):
    """One EM iteration of run_rnnlogic.py (src/run_rnnlogic.py:61-91) with
    config/FB15k-237.yaml's settings on FB15k-237 (BASELINE.json config 5):
    sample(100, 3) from the generator, a new Predictor(bias) + Adam trained
    over every train batch (the config's batch_per_epoch 1e6 = all 17,258),
    evaluate('valid') and ('test'), compute_H over every train row, the
    posterior and the M-step (generator.train, 100 epochs).  The generator is
    first pre-trained for `pre_epochs` of the config's 10,000 epochs on
    rnnlogic_rules.txt with synthetic weights (pre-training happens once per
    run, before the EM loop; FB's mined_rules.txt needs the absent
    train.txt) — reported separately, not part of the iteration."""
    from rnnlogic_amd.data import RuleDataset
    from rnnlogic_amd.generators import Generator
    from rnnlogic_amd.predictors import Predictor
    from rnnlogic_amd.trainer import TrainerGenerator, TrainerPredictor
    from rnnlogic_amd.utils import set_seed

    def timed(fn):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        out = fn()
        torch.cuda.synchronize(dev)
        return out, time.perf_counter() - t0
    with contextlib.redirect_stdout(sys.stderr):
        set_seed(1)
        graph = KnowledgeGraph(datasets.materialize("FB15k-237"))
        train_set, valid_set, test_set = TrainDataset(graph, 32), ValidDataset(graph, 32), TestDataset(graph, 32)
    mined = [[int(x) for x in line.split()] for line in open(datasets.rule_file("FB15k-237"))]
    dataset = RuleDataset(graph.relation_size, [r + [0.25 * ((i * 37) % 11) - 1.0] for i, r in enumerate(mined)])
    gen = Generator(graph, num_layers=1, embedding_dim=512, hidden_dim=256)
    solver_g = TrainerGenerator(gen, gpu=dev.index or 0)
    _, t_pre = timed(lambda: solver_g.train(dataset, num_epoch=pre_epochs, lr=1e-3, print_every=1000000,
                                            batch_size=512))
    res = {}
    sampled, res["sample_s"] = timed(lambda: solver_g.sample(100, 3))
    prior = [r[-1] for r in sampled]
    rules = [r[:-1] for r in sampled]
    predictor = Predictor(graph, entity_feature="bias")
    with contextlib.redirect_stdout(sys.stderr):
        predictor.set_rules(rules)
    optim = torch.optim.Adam(predictor.parameters(), lr=1e-3, weight_decay=0)
    solver_p = TrainerPredictor(predictor, train_set, valid_set, test_set, optim, gpus=[dev.index or 0])
    _, res["predictor_train_s"] = timed(lambda: solver_p.train(batch_per_epoch=1000000, smoothing=0.2,
                                                               print_every=1000000))
    (vm, tm), res["evaluate_s"] = timed(lambda: (solver_p.evaluate("valid"), solver_p.evaluate("test")))
    H, res["e_step_compute_H_s"] = timed(lambda: solver_p.compute_H(print_every=1000000))
    posterior = [h + p * 0.001 for h, p in zip(H, prior)]
    for i in range(len(rules)):
        rules[i].append(posterior[i])
    _, res["m_step_s"] = timed(lambda: solver_g.train(RuleDataset(graph.relation_size, rules), num_epoch=100,
                                                      lr=1e-5, print_every=1000000, batch_size=512))
    total = sum(res.values())
    nb = len(train_set)
    out = {"s": round(total, 3), "phases_s": {k: round(v, 3) for k, v in res.items()},
           "rules_sampled": len(sampled), "train_batches": nb,
           "predictor_ms_per_batch": round(res["predictor_train_s"] / nb * 1e3, 3),
           "valid_mrr": vm, "test_mrr": tm,
           "pre_train": {"epochs": pre_epochs, "s": round(t_pre, 3), "ms_per_epoch": round(t_pre / pre_epochs * 1e3, 3),
                         "note": "once per run, before the EM loop; not in `s`"},
           "workload": "config/FB15k-237.yaml EM iteration (EM.num_rules 100, max_length 3; predictor over all "
                       "train batches; M-step 100 epochs) on the seeded synthetic FB15k-237 train graph, 1 GPU"}
    del solver_p, predictor, solver_g, gen
    return out


WORK_FILES = {"FB15k-237": "fb15k237_work.json", "kinship": "kinship_work.json", "wn18rr": "wn18rr_work.json"}


def algorithmic_work(model, graph, rows, threads=None, name="FB15k-237"):
    """Exact per-rule work counts of the SURVEY §8(d) formula: F (frontier
    expansions), T (edge traversals), P ((rule, dest) pairs) and C
    (candidates) of a workload, from tests/golden/<name>_work.json (made by
    tools/make_work_counts.py with the C oracle; a prefix is re-derived by
    tests/test_oracle_c.py).  The file must describe exactly these rows."""
    import hashlib
    fn = os.path.join(REPO, "tests", "golden", WORK_FILES[name])
    with open(fn) as f:
        w = json.load(f)
    dig = hashlib.sha256(np.ascontiguousarray(rows[:, :2], dtype=np.int64).tobytes()).hexdigest()
    if w["rows_sha256"] != dig or w["rules"] != model.num_rules:
        raise RuntimeError("%s does not describe this workload: rerun tools/make_work_counts.py" % fn)
    return (w["F"], w["T"], w["P"]), w["C"]


def grounding_roofline(work, nq, E, ms, kernel, extra_bytes=0.0, measured=""):
    """HBM roofline of a grounding + scoring launch: SURVEY §8(d)'s
    ALG_BYTES = 12 F + 12 T + 8 P + 4 B |E| (+ X: the bias row or other base
    reads) over the measured time."""
    (F, T, P), C = work
    alg = 12 * F + 12 * T + 8 * P + 4 * nq * E + extra_bytes
    ach = alg / (ms * 1e-3) / 1e9
    return {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4), "ms": round(ms, 3), "kernel": kernel, "measured": measured,
            "alg_bytes": int(alg), "work": {"F": int(F), "T": int(T), "P": int(P), "C": int(C)}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--feature", default="RotatE", choices=["RotatE", "bias"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=None,
                    help="threads of the CPU baseline (default: every core this process may run on)")
    ap.add_argument("--profile-only", action="store_true",
                    help="only the timed steps (no extra lines, baselines or clock probe): the command the "
                         "committed rocprofv3 summaries profile, so every launch of a kernel has the same shape")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world:
        raise SystemExit("bench.py --gpus %d but WORLD_SIZE=%d: launch N>1 with torch.distributed.run "
                         "--nproc-per-node N" % (args.gpus, world))
    # rehearsal of the N > 1 path on a one-GPU box (never for measurements):
    # RNNL_BENCH_ONE_DEVICE=1 puts every rank on cuda:0, RNNL_BENCH_BACKEND=gloo
    # replaces RCCL (which refuses two ranks on one device)
    if os.environ.get("RNNL_BENCH_ONE_DEVICE") == "1":
        local = 0
    backend = os.environ.get("RNNL_BENCH_BACKEND", "nccl")
    # a process group whenever torch.distributed.run launched this process
    # (also at --nproc-per-node 1: RCCL then runs its one-rank communicator
    # through the same barriers / all-reduce / all-gather as at N > 1)
    distributed = world > 1 or "TORCHELASTIC_RUN_ID" in os.environ
    if distributed:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    if rank == 0:
        datasets.materialize("FB15k-237", with_rotate=(args.feature == "RotatE"))
    if distributed:
        dist.barrier()

    with contextlib.redirect_stdout(sys.stderr):  # stdout carries only the JSON line
        graph, test_set, model, all_rows = build_workload(args.feature)
    model = model.to(dev).eval()
    n_split = len(all_rows)
    rows, shard = (all_rows, list(range(len(test_set)))) if world == 1 else shard_rows(test_set, world, rank)
    h = torch.from_numpy(np.ascontiguousarray(rows[:, 0])).to(dev)
    r = torch.from_numpy(np.ascontiguousarray(rows[:, 1])).to(dev)
    nq = len(rows)
    torch.cuda.synchronize(dev)

    def step(ev=None):
        model.invalidate_cache()  # rule embeddings + node aggregates recomputed every step
        with torch.no_grad():
            return model.forward_rows(h, r, None, events=ev)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if distributed:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if distributed:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if distributed:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    rows_per_rank = [nq]
    shards = None
    if distributed:
        cnt = torch.tensor([nq], dtype=torch.int64, device=dev)
        parts = [torch.empty_like(cnt) for _ in range(world)]
        dist.all_gather(parts, cnt)
        rows_per_rank = [int(x.item()) for x in parts]
        # every rank's batch indices: their union must be the split, the
        # surplus the sampler's padding (repeated batches, trainer.py:150)
        idx_all = [None] * world
        dist.all_gather_object(idx_all, list(shard))
        flat = [i for part in idx_all for i in part]
        # per-rank self-check: the rank's device, where its graph handle and the
        # forward's side streams live, and the world the process group saw
        me = rank_info(model, dev, local, world, backend)
        info_all = [None] * world
        dist.all_gather_object(info_all, me)
        shards = {"batches_per_rank": [len(x) for x in idx_all],
                  "ranks": info_all,
                  "devices_distinct": len({(x["host"], x["cuda_device"]) for x in info_all}) == world,
                  "union_is_split": sorted(set(flat)) == list(range(len(test_set))),
                  "padding_batches": len(flat) - len(test_set),
                  "rows_total_with_padding": int(sum(rows_per_rank)), "rows_counted": n_split}

    # secondary at N > 1: every rank on the whole split (replicated, weak scaling)
    weak = None
    if world > 1 and not args.profile_only:
        ah = torch.from_numpy(np.ascontiguousarray(all_rows[:, 0])).to(dev)
        ar = torch.from_numpy(np.ascontiguousarray(all_rows[:, 1])).to(dev)

        def full_step():
            model.invalidate_cache()
            with torch.no_grad():
                return model.forward_rows(ah, ar, None)
        full_step()
        torch.cuda.synchronize(dev)
        dist.barrier()
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        for _ in range(args.steps):
            full_step()
        torch.cuda.synchronize(dev)
        dist.barrier()
        torch.cuda.synchronize(dev)
        tw = torch.tensor([time.perf_counter() - t1], dtype=torch.float64, device=dev)
        dist.all_reduce(tw, op=dist.ReduceOp.MAX)
        weak = {"queries_per_s": round(n_split * args.steps * world / float(tw.item()), 1),
                "ms_per_step": round(float(tw.item()) / args.steps * 1e3, 3), "rows_per_rank": n_split,
                "scaling": "weak",
                "note": "every rank runs the whole test split (replicated work; value counts world x rows)"}
        del ah, ar

    # per-kernel device time (HIP events on the launch stream).  With the
    # RotatE feature the forward overlaps: the grounding runs on a side stream
    # beside the RotatE chunks (predictors.PredictorPlus._forward_overlap), so
    # base -> ground brackets the RotatE launches on the main stream and
    # ground -> end is the scoring tail left after the last RotatE chunk.
    # (measured on 3 extra, untimed steps: the events stay out of the timed region)
    evs = []
    for _ in range(3):
        ev = {}
        step(ev)
        evs.append(ev)
    torch.cuda.synchronize(dev)
    nodes_ms = float(np.mean([e["start"].elapsed_time(e["base"]) for e in evs]))
    base_ms = float(np.mean([e["base"].elapsed_time(e["ground"]) for e in evs]))
    tail_ms = float(np.mean([e["ground"].elapsed_time(e["end"]) for e in evs]))
    overlapped = args.feature == "RotatE" and model.overlap
    n_rot = 1  # RotatE launches per step
    # the grounding + scoring kernels alone (one untimed one-stream launch), for their roofline
    if world > 1:  # the work-count fixture describes the whole split, not a shard
        ground_ms, ground_how = None, None
    elif not args.profile_only:
        ground_ms, ground_how = isolated_ground_ms(model, graph, h, r, dev), \
            "one untimed one-stream launch over all rows (isolated from RotatE)"
    elif args.feature != "RotatE":
        ground_ms, ground_how = base_ms + tail_ms, "timed steps (one stream: bias-row fill + ground + score)"
    else:
        ground_ms, ground_how = None, None

    # effective shader clock under the RotatE kernel's load (one extra, untimed
    # launch with the kernel's per-block clock stamps on; rnnl_debug_clock)
    clock_ghz = None
    if args.feature == "RotatE" and not args.profile_only:
        from rnnlogic_amd import _native
        clk = torch.zeros(2, dtype=torch.int64, device=dev)
        _native.call("rnnl_debug_clock", clk.data_ptr())
        try:
            with torch.no_grad():
                tmp = torch.empty((nq, graph.entity_size), dtype=torch.float32, device=dev)
                model.RotatE.score_into(h, r, tmp)
            torch.cuda.synchronize(dev)
        finally:
            _native.call("rnnl_debug_clock", None)
        ticks, real = clk.tolist()
        clock_ghz = 0.1 * ticks / max(real, 1)
        del tmp

    # HBM traffic per launch from the committed PMC summary of this workload
    # (tools/pmc_traffic.py; bench.py cannot read counters itself).  RotatE
    # kernels: traffic_rotate.json (the overlapped launches, as timed);
    # grounding kernels: traffic_bias.json (one launch over all rows, as the
    # isolated grounding time).  A summary is used only when its stamp
    # matches the kernel sources this run executes (csrc_fingerprint):
    # counters of an older tree are not reported as this tree's traffic.
    traffic_note = {}

    def load_traffic(name):
        tpath = os.path.join(REPO, "profiles", "traffic_%s.json" % name)
        if not os.path.exists(tpath):
            traffic_note[name] = "missing"
            return {}
        with open(tpath) as f:
            tj = json.load(f)
        if tj.get("csrc_sha256") != csrc_fingerprint():
            traffic_note[name] = "stale (captured at %s; kernel sources changed since)" % tj.get("commit", "?")
            return {}
        traffic_note[name] = "captured at %s" % tj.get("commit", "?")
        return {k.split("::")[-1].split("<")[0]: v["bytes"] for k, v in tj.get("kernels", {}).items()}
    # (the committed PMC summaries describe the one-rank workload: no traffic figure for a shard)
    traffic = load_traffic(args.feature.lower()) if world == 1 else {}
    gtraffic = load_traffic("bias") if world == 1 else {}

    # secondary lines (untimed by the driver; not `value`): the train-mode
    # forward with per-row edge removal, and the EM loop's
    # rule-weight Predictor over the same test split (a12)
    extra = {}
    if rank == 0 and world == 1 and not args.profile_only:
        # the same step with duplicate (h, r) rows computed once (bit-identical
        # output; forward_rows(dedupe=True)) — reported beside `value`, not as it
        def dd_step():
            model.invalidate_cache()
            return model.forward_rows(h, r, None, dedupe=True)
        with torch.no_grad():
            sec = time_forward(dd_step, 3)
        nu = int(torch.unique(r * graph.entity_size + h).numel())
        extra["dedup_forward"] = {"queries_per_s": round(nq / sec, 1), "ms": round(sec * 1e3, 3), "rows": nq,
                                  "distinct_rows": nu,
                                  "note": "eval rows with equal (h, r) computed once and copied (bit-identical)"}
        with contextlib.redirect_stdout(sys.stderr):
            th, tr, te, nb = train_rows(model.train_set, nq)
        th, tr, te = th.to(dev), tr.to(dev), te.to(dev)
        with torch.no_grad():
            sec = time_forward(lambda: model.forward_rows(th, tr, te), 3)
        extra["train_mode_forward"] = {"queries_per_s": round(len(th) / sec, 1), "ms": round(sec * 1e3, 3),
                                       "rows": len(th), "batches": nb,
                                       "note": "forward_rows with edges_to_remove (train batches), no autograd"}
        from rnnlogic_amd.predictors import Predictor
        pred = Predictor(graph, entity_feature="bias")
        with contextlib.redirect_stdout(sys.stderr):
            pred.set_rules(datasets.rule_file("FB15k-237"))
        with torch.no_grad():
            pred.rule_weights.normal_()
            pred.bias.normal_()
        pred = pred.to(dev).eval()
        with torch.no_grad():
            sec = time_forward(lambda: pred.forward_rows(h, r, None), 3)
        extra["em_predictor_forward"] = {
            "queries_per_s": round(nq / sec, 1), "ms": round(sec * 1e3, 3), "rows": nq,
            "roofline": grounding_roofline(algorithmic_work(model, graph, all_rows), nq, graph.entity_size, sec * 1e3,
                                           "ground_kernel + score_linear_kernel (+ bias row fill)",
                                           extra_bytes=4.0 * graph.entity_size,
                                           measured="the timed forward_rows (node weights + fill + ground + score)"),
            "note": "Predictor(bias) over the test split, same rules (same grounding work as value)"}
        del pred
        if args.feature == "RotatE":
            extra["shard_balance"] = shard_balance_line(model, test_set, dev, elapsed / args.steps * 1e3)
        extra["wn18rr_forward"] = wn18rr_line(dev)
        extra["wn18rr_train_step"] = wn18rr_train_line(dev)
        extra["kinship_forward"] = kinship_line(dev)
        # end-to-end evaluate('test') (trainer.py:145-248): device rows + filter
        # flags, one forward over the split, device ranks, host metrics
        from rnnlogic_amd.trainer import TrainerPredictor
        solver = TrainerPredictor(model, model.train_set, None, test_set, None, gpus=[local])
        t_first = time.perf_counter()
        solver.evaluate("test")
        torch.cuda.synchronize(dev)
        t_first = time.perf_counter() - t_first
        sec = time_forward(lambda: solver.evaluate("test"), 3)
        extra["evaluate_test"] = {"queries_per_s": round(n_split / sec, 1), "ms": round(sec * 1e3, 3),
                                  "first_call_ms": round(t_first * 1e3, 3), "rows": n_split,
                                  "note": "TrainerPredictor.evaluate('test') end to end (MRR/Hits on the host); "
                                          "the first call also uploads the split's rows and filter lists"}
        # the reference API's per-batch forward (trainer.py:150-173)
        extra["per_batch_forward"] = per_batch_line(model, graph, test_set, dev)
        # training steps (trainer.py:72-98): HIP grounding with edge removal,
        # autograd on the path-count COO + RotatE (HIP backward), Adam
        extra["train_step"] = train_step_line(model, solver, dev)
        del solver
        # config 5: one EM iteration of run_rnnlogic.py on FB15k-237
        extra["em_iteration"] = em_iteration_line(dev)
        extra["em_full_fb"] = recorded_em_full()

    if rank != 0:
        if distributed:
            dist.barrier()
            dist.destroy_process_group()
        return

    E = graph.entity_size
    cores = host_cores()
    threads = args.cpu_threads or cores["usable"]
    (F, T, P), C = algorithmic_work(model, graph, all_rows, threads)
    # ALG_BYTES = 12 F + 12 T + 8 P + 4 B|E| + X
    ground_bytes = 12 * F + 12 * T + 8 * P + 4 * nq * E
    D = model.RotatE.emb_dim if args.feature == "RotatE" else 0
    rotate_flops = 7.0 * nq * E * D
    rotate_bytes = 8.0 * D * E * ((nq + 15) // 16) + 8.0 * D * nq + 4.0 * nq * E
    if ground_ms is None:  # --profile-only with the RotatE overlap: no isolated grounding time
        ground_ms = float("nan")
    # like for like: the counted kernels are the ones the time covers (the
    # bias-row fill that writes SURVEY §8(d)'s 4 B |E| score rows included)
    gt = [gtraffic.get(k) for k in ("fill_rows_kernel", "ground_kernel", "memo_sum_kernel", "score_sum_chunk_kernel",
                                    "score_pna_chunk_kernel", "pack_weights_kernel", "chunk_sum_kernel",
                                    "chunk_fill_kernel")]
    gt = sum(x for x in gt if x) or None
    ground = {"bound": "hbm", "achieved": round(ground_bytes / (ground_ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS,
              "unit": "GB/s", "frac": round(ground_bytes / (ground_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
              "traffic": gt, "traffic_source": "profiles/traffic_bias.json: " + traffic_note.get("bias", "n/a"),
              "kernel": "fill_rows (bias rows) + ground_kernel + scoring (chunk list + memo_sum_kernel + "
                        "score_sum_chunk_kernel)",
              "traffic_over_alg": round(gt / ground_bytes, 3) if gt else None,
              "ms": round(ground_ms, 3),
              "measured": ground_how,
              "alg_bytes": int(ground_bytes), "work": {"F": int(F), "T": int(T), "P": int(P), "C": C}}
    if ground_ms != ground_ms:  # nan
        ground = None
    if args.feature == "RotatE":
        # per launch: n_rot launches of nq / n_rot rows each on the main stream
        ach = rotate_flops / (base_ms * 1e-3) / 1e12
        mode = "direct" if model.RotatE.mode == 0 else "mfma"
        # VALU issue: cycles per 64 terms on one SIMD at the kernel's measured
        # clock (DVFS lowers it under VALU load), against the floor of the
        # kernel's instruction mix
        # (tools/micro/valu_rates.hip: sub,sub,mul,fma + pipelined sqrt + add
        # = 19.1; bf16 MFMA + sqrt + add = 13.1)
        ghz = clock_ghz or 2.4
        cyc = base_ms * 1e-3 * ghz * 1e9 * 1024 / (nq * E * D / 64.0)
        floor = 19.1 if mode == "direct" else 13.1
        roof = {"bound": "valu", "achieved": round(ach, 2), "peak": FP32_PEAK_TFS, "unit": "TFLOP/s",
                "frac": round(ach / FP32_PEAK_TFS, 4), "traffic": traffic.get("rotate_%s_kernel" % mode),
                "traffic_source": "profiles/traffic_rotate.json: " + traffic_note.get("rotate", "n/a"),
                "kernel": "rotate_%s_kernel" % mode,
                "ms": round(base_ms / n_rot, 3), "alg_flops": rotate_flops / n_rot, "launches_per_step": n_rot,
                "valu_issue": {"cycles_per_64_terms": round(cyc, 2), "floor": floor, "frac": round(floor / cyc, 3),
                               "clock_ghz": round(ghz, 3), "clock": "measured in-kernel" if clock_ghz else "nominal"},
                "note": "fp32 compute-bound on the VALU issue port (sub, sub, mul, fma, one quarter-rate sqrt and "
                        "an add per term; the sqrt inside the reduction keeps it off the matrix cores); "
                        "157.3 TF/s is the fp32 peak shared by VALU and MFMA; entity-table bytes %.3g per launch"
                        % rotate_bytes}
        # RotatE's HBM fraction from the counters (the bytes the launch moved,
        # profiles/traffic_rotate.json) over its time; SURVEY §8(d)'s
        # X = 8 D |E| + 8 D B per reference batch charges one entity-table
        # read per 32-row batch (1,514 reads) — a formula, kept beside it
        x_bytes = len(test_set) * 8.0 * D * E + 8.0 * D * nq + 4.0 * nq * E
        tr = traffic.get("rotate_%s_kernel" % mode)
        roof["hbm_view"] = {"bound": "hbm", "achieved": round(tr / (base_ms * 1e-3) / 1e9, 1) if tr else None,
                            "peak": HBM_PEAK_GBS, "unit": "GB/s",
                            "frac": round(tr / (base_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if tr else None,
                            "bytes": tr, "bytes_source": "PMC counters (traffic_source)" if tr else "n/a",
                            "survey_formula_bytes": x_bytes,
                            "note": "survey_formula_bytes charges one entity-table read per reference batch; the "
                                    "kernel reads each XCD's table slab once per launch (HBM fraction = counters)"}
        dominant = roof if not (ground_ms > base_ms) else ground
    else:
        dominant = ground
    out = {
        "metric": METRIC,
        "value": round(n_split * args.steps / elapsed, 1),
        "unit": "queries/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": "synthetic",
        "config": {"workload": "FB15k-237 test split: %d batches, %d queries, sharded over %d rank(s) by the "
                               "reference evaluate()'s DistributedSampler; PredictorPlus(lstm,3,16,sum)"
                               " + %s; rnnlogic_rules.txt (%d rules, L<=3); seeded synthetic train graph%s"
                               % (len(test_set), n_split, world,
                                  "RotatE(D=1000,gamma=9)" if args.feature == "RotatE" else "bias",
                                  model.num_rules, " and RotatE tables" if args.feature == "RotatE" else ""),
                   "batch_size": 32, "parallelism": "dp%d (test batches sharded, KG replicated)" % world,
                   "rows_per_rank": rows_per_rank, "batches_per_rank": len(shard), "shards": shards,
                   "placement": shards["ranks"] if shards else [rank_info(model, dev, local, world, backend)],
                   "process_group": backend if distributed else None},
        "roofline": dominant,
        "kernels_ms": {"rule_encoder+node_weights": round(nodes_ms, 3), "base_score": round(base_ms, 3),
                       "tail_after_base": round(tail_ms, 3), "ground+score_isolated": round(ground_ms, 3)},
        "overlap": {"rotate_chunks": n_rot, "note": "grounding on a side stream beside the RotatE chunks; each "
                    "chunk's scoring pass after its RotatE rows"} if overlapped else None,
        "roofline_grounding": ground,
    }
    out.update(extra)
    if weak is not None:
        out["weak_replicated"] = weak
    if not args.no_cpu_baseline and not args.profile_only and world == 1:
        out["cpu_baseline"] = cpu_baseline(graph.data_path, model, rows, threads, cores)
        with contextlib.redirect_stdout(sys.stderr):
            out["reference_pytorch"] = reference_pytorch_baseline(model, graph, test_set, dev, args.feature)
    print(json.dumps(out), flush=True)
    if distributed:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
