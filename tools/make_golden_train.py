"""Golden vectors for the training path, made by running the
*reference* Python on CPU in the build container (tools/ref_shims stand in for
torch_scatter / easydict; see tools/make_golden.py).

Per case, the first K steps of TrainerPredictor.train's loop (trainer.py:48-105:
DistributedSampler(world 1, rank 0, epoch 0) batch order, label smoothing 0.2,
loss = -sum(log(softmax + 1e-8) * target)[mask] / sum(target[mask]), Adam
lr 0.005) are replayed on the seeded model.  Stored:
  sd/<name>        initial state_dict (RotatE tables as digests only)
  order            sampler batch order (first K)
  s<k>/h,r,t,etr   the batch of step k
  s<k>/loss        loss of step k
  g/<name>         gradients of step 0 (before the optimizer step)
  gs/<name>/...    for gradients too large to store (the RotatE tables at
                   D = 1000): `rows` (every nonzero row when there are <= 64,
                   else the step's h / t entities + 64 seeded random rows),
                   `vals` (those rows) and `rowabs` (float64 sum of |g| of
                   every row)

The headline case (FB15k-237 lstm/sum + RotatE D = 1000, trainable) uses the
row-wise RotatE.forward of tools/make_golden_eval.py (the reference's own
project() / product() once per row, checked bitwise against the unpatched
forward on the first rows): the unpatched forward holds (B * |E|, 2D) tensors
per step (~40 GB with autograd at B = 32).  The forward values are identical;
the gradients of the h / r rows sum the same per-entity terms in another fp32
order (one row's product per row instead of one per (row, entity) pair).

Usage:  python tools/make_golden_train.py [case ...]
"""
import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
sys.dont_write_bytecode = True
sys.path[:0] = [os.path.join(HERE, "ref_shims"), "/root/reference/src"]

import torch  # noqa: E402
from torch.utils import data as torch_data  # noqa: E402

import data as R_data  # noqa: E402  (reference src/data.py)
import predictors as R_pred  # noqa: E402
import utils as R_utils  # noqa: E402

from rnnlogic_amd import datasets  # noqa: E402
from make_golden import _rotate_dir  # noqa: E402
from make_golden_eval import _rotate_rows  # noqa: E402

OUT = os.path.join(REPO, "tests", "golden")
K = 3
SMOOTHING = 0.2

CASES = {
    "train_umls_lstm_sum_bias": dict(data="umls", model=dict(type="lstm", entity_feature="bias", aggregator="sum")),
    "train_umls_emb_pna_rotate": dict(data="umls", model=dict(type="emb", entity_feature="RotatE", aggregator="pna",
                                                               embedding_path="rotate:200")),
    "train_kinship_lstm_sum_none": dict(data="kinship", model=dict(type="lstm", entity_feature="none",
                                                                   aggregator="sum")),
    "train_kinship_emb_pna_bias": dict(data="kinship", model=dict(type="emb", entity_feature="bias",
                                                                  aggregator="pna")),
    # the headline model (config 4) with edge removal, RotatE trainable
    "train_fb_lstm_sum_rotate": dict(data="FB15k-237", model=dict(type="lstm", entity_feature="RotatE",
                                                                  aggregator="sum", embedding_path="rotate"),
                                     rotate_rows=True),
}
BIG = 1 << 20  # gradients with more elements are stored as sampled rows


def _store_grad(out, n, g, h, t):
    if g.size < BIG:
        out["g/" + n] = g.copy()
        return
    g2 = g.reshape(g.shape[0], -1)
    nz = np.nonzero(np.abs(g2).sum(1))[0]
    if len(nz) <= 64:
        rows = nz
    else:
        rng = np.random.RandomState(7)
        rows = np.unique(np.concatenate([h, t, rng.randint(0, g2.shape[0], 64)]))
    out["gs/%s/rows" % n] = rows.astype(np.int64)
    out["gs/%s/vals" % n] = g2[rows].copy()
    out["gs/%s/rowabs" % n] = np.abs(g2.astype(np.float64)).sum(1)


def run_case(name, spec):
    dpath = datasets.materialize(spec["data"])
    kw = dict(type="lstm", num_layers=3, hidden_dim=16, entity_feature="bias", aggregator="sum", embedding_path=None)
    kw.update(spec["model"])
    if kw.get("embedding_path"):
        kw["embedding_path"] = _rotate_dir(spec["data"], kw["embedding_path"])
    R_utils.set_seed(1)
    graph = R_data.KnowledgeGraph(dpath)
    train_set = R_data.TrainDataset(graph, 32)
    R_data.ValidDataset(graph, 32)
    R_data.TestDataset(graph, 32)
    model = R_pred.PredictorPlus(graph, **kw)
    model.set_rules(datasets.rule_file(spec["data"]))
    if spec.get("rotate_rows"):
        rot = model.RotatE
        # any two rows: a bitwise check of the row-wise form
        h, r = torch.as_tensor([x[0] for x in train_set.batches[0][:2]]), torch.as_tensor(
            [x[1] for x in train_set.batches[0][:2]])
        with torch.no_grad():
            assert torch.equal(rot(h, r), _rotate_rows(rot)(h, r))
        rot.forward = _rotate_rows(rot)
    out = {}
    for k, v in model.state_dict().items():
        if k.startswith("RotatE."):
            out["sha/" + k] = np.array(hashlib.sha256(v.detach().numpy().tobytes()).hexdigest())
        else:
            out["sd/" + k] = v.detach().cpu().numpy().copy()  # the optimizer updates the parameters in place
    optim = torch.optim.Adam(model.parameters(), lr=0.005, weight_decay=0)
    # trainer.py:51-73
    train_set.make_batches()
    sampler = torch_data.DistributedSampler(train_set, 1, 0)
    sampler.set_epoch(0)
    order = list(iter(sampler))[:K]
    out["order"] = np.asarray(order, dtype=np.int64)
    model.train()
    for k, idx in enumerate(order):
        all_h, all_r, all_t, target, etr = train_set[idx]
        target_t = torch.nn.functional.one_hot(all_t, graph.entity_size)
        target = target * SMOOTHING + target_t * (1 - SMOOTHING)
        logits, mask = model(all_h, all_r, etr)
        p = "s%d/" % k
        out[p + "h"], out[p + "r"], out[p + "t"], out[p + "etr"] = (all_h.numpy(), all_r.numpy(), all_t.numpy(),
                                                                    etr.numpy())
        if mask.sum().item() != 0:
            logits = (torch.softmax(logits, dim=1) + 1e-8).log()
            loss = -(logits[mask] * target[mask]).sum() / torch.clamp(target[mask].sum(), min=1)
            loss.backward()
            out[p + "loss"] = np.float64(loss.item())
            if k == 0:
                for n, prm in model.named_parameters():
                    if prm.grad is not None:
                        _store_grad(out, n, prm.grad.detach().numpy(), all_h.numpy(), all_t.numpy())
            optim.step()
            optim.zero_grad()
        else:
            out[p + "loss"] = np.float64("nan")
    path = os.path.join(OUT, name + ".npz")
    np.savez_compressed(path, **out)
    print(name, "->", path, os.path.getsize(path), "losses", [float(out["s%d/loss" % k]) for k in range(K)])


if __name__ == "__main__":
    os.makedirs(OUT, exist_ok=True)
    torch.set_num_threads(int(os.environ.get("THREADS", "8")))
    for n in sys.argv[1:] or list(CASES):
        run_case(n, CASES[n])
