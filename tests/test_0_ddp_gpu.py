"""Multi-process training path on the GPU: TrainerPredictor.train
at world size 2 — DistributedSampler shards + DistributedDataParallel with
find_unused_parameters=True (reference src/trainer.py:52-60) — both ranks on
cuda:0 over a gloo group (CUDA tensors), since the box has one GPU.  The
gradient each rank's optimizer sees must be the mean of the two ranks'
single-process gradients of their own batches.

The file sorts first so the ranks start before this pytest process touches
the GPU (a process that has initialised the GPU must not exec a new one)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

CASE = "umls_lstm_sum_bias"


class _Recorder(object):
    """Optimizer stand-in: step() records every gradient, weights unchanged."""

    def __init__(self, model):
        self.model = model
        self.steps = []

    def step(self):
        self.steps.append({n: p.grad.detach().cpu().clone() for n, p in self.model.named_parameters()
                           if p.grad is not None})

    def zero_grad(self):
        for p in self.model.parameters():
            p.grad = None


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.set_num_threads(2)
    from conftest import Fixture
    from rnnlogic_amd import comm, datasets
    from rnnlogic_amd.data import KnowledgeGraph, TestDataset, TrainDataset, ValidDataset
    from rnnlogic_amd.predictors import PredictorPlus
    from rnnlogic_amd.trainer import TrainerPredictor
    from rnnlogic_amd.utils import set_seed
    comm.init_process_group("gloo", init_method="env://")
    torch.cuda.set_device(0)
    fx = Fixture(CASE)
    set_seed(1)
    graph = KnowledgeGraph(datasets.materialize("umls"))
    train_set, valid_set, test_set = TrainDataset(graph, 32), ValidDataset(graph, 32), TestDataset(graph, 32)
    model = PredictorPlus(graph, type="lstm", num_layers=3, hidden_dim=16, entity_feature="bias", aggregator="sum")
    model.set_rules(datasets.rule_file("umls"))
    model.load_state_dict({k: torch.from_numpy(v) for k, v in fx.sd.items()})
    # each rank's single-process gradients of its first two sampler batches,
    # on the batches train() will draw (make_batches under the same random state)
    import random
    state = random.getstate()
    # make_batches shuffles r2instances in place: restore them with the RNG state
    r2i = [list(x) for x in train_set.r2instances]
    train_set.make_batches()
    sampler = torch.utils.data.DistributedSampler(train_set, world, rank)
    sampler.set_epoch(0)
    idx = list(iter(sampler))[:2]
    model = model.cuda()
    local = _Recorder(model)
    solver = TrainerPredictor(model, train_set, valid_set, test_set, local, gpus=[0] * world)
    for i in idx:
        solver.train_step(model, [x.unsqueeze(0) for x in train_set[i]], 0.2)
    random.setstate(state)
    train_set.r2instances = r2i
    # the same two steps through train(): DDP all-reduces over the gloo group
    rec = _Recorder(model)
    solver.optimizer = rec
    solver.train(batch_per_epoch=2, smoothing=0.2, print_every=10)
    ddp = rec.steps
    torch.save({"ddp": ddp, "local": local.steps, "idx": idx}, os.path.join(out_dir, "rank%d.pt" % rank))
    comm.synchronize()
    torch.distributed.destroy_process_group()


def test_ddp_world2_gradients_are_the_rank_mean(tmp_path):
    if torch.cuda.is_initialized():
        pytest.skip("this process already initialised the GPU (run this file first)")
    if torch.cuda.device_count() < 1:
        pytest.skip("no GPU")
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, start_method="spawn")
    res = [torch.load(os.path.join(str(tmp_path), "rank%d.pt" % r), weights_only=True) for r in range(world)]
    assert res[0]["idx"] != res[1]["idx"]
    for s in range(2):  # the all-reduced gradients are identical on both ranks
        for n in res[0]["ddp"][s]:
            assert torch.equal(res[0]["ddp"][s][n], res[1]["ddp"][s][n]), (s, n)
    for s in range(2):
        g0, g1 = res[0]["ddp"][s], res[1]["ddp"][s]
        assert sorted(g0) == sorted(g1)
        names = sorted(set(res[0]["local"][s]) | set(res[1]["local"][s]))
        for n in names:
            parts = [res[r]["local"][s].get(n) for r in range(world)]
            mean = sum(p for p in parts if p is not None) / world
            for r in range(world):
                got = res[r]["ddp"][s][n]
                err = float((got - mean).abs().max())
                scale = float(mean.abs().max()) + 1e-12
                assert err <= 1e-6 + 1e-5 * scale, (s, n, r, err, scale)
        print("step %d: %d gradients, all-reduced == mean of the ranks' own" % (s, len(names)))
