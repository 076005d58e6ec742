"""The run_rnnlogic.py sequence (run_rnnlogic.py:45-91) through rnnlogic_amd,
mirroring tools/make_golden_em.py step for step, so its outputs compare with
tests/golden/em_umls.npz (the reference's own run of the same sequence).

`run(device, em=False)` stops after the generator pre-training / beam search
(pure PyTorch, runs on CPU); `em=True` continues with one EM iteration, which
starts as run_rnnlogic.py:68 does, from TrainerGenerator.sample(), and whose
Predictor runs on the HIP path (GPU only).  `gen_device` (default: `device`)
places the generator: the reference's sample() draws from the CPU RNG in the
fixture, so an EM iteration that must reproduce its rules keeps the generator
on the CPU while the predictor runs on the GPU."""
import json
import os

import numpy as np
import torch

from conftest import GOLDEN


def fixture():
    z = np.load(os.path.join(GOLDEN, "em_umls.npz"), allow_pickle=False)
    return z, json.loads(str(z["cfg"]))


def cpu_model():
    """model name of /proc/cpuinfo (tools/make_golden_em.py stores the fixture's)."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def rule_weight(i):
    return 0.25 * ((i * 37) % 11) - 1.0


def _probe():
    return torch.randint(0, 2 ** 31 - 1, (4,)).numpy()


def run(device, em=False, gen_device=None, stop_after_sample=False):
    from rnnlogic_amd import datasets
    from rnnlogic_amd.data import KnowledgeGraph, RuleDataset, TestDataset, TrainDataset, ValidDataset
    from rnnlogic_amd.generators import Generator
    from rnnlogic_amd.trainer import TrainerGenerator
    from rnnlogic_amd.utils import set_seed

    z, cfg = fixture()
    got = {}
    path = datasets.materialize("umls")
    mined = [[int(x) for x in line.split()] for line in open(datasets.rule_file("umls"))]
    set_seed(cfg["seed"])
    graph = KnowledgeGraph(path)
    train_set = TrainDataset(graph, 32)
    valid_set = ValidDataset(graph, 32)
    test_set = TestDataset(graph, 32)
    dataset = RuleDataset(graph.relation_size, [r + [rule_weight(i)] for i, r in enumerate(mined)])
    gen = Generator(graph, **cfg["gen"])
    got["gen_init"] = {k: v.detach().cpu().numpy().copy() for k, v in gen.state_dict().items()}
    gpu = None if device.type == "cpu" else device.index or 0
    gen_device = device if gen_device is None else gen_device
    solver_g = TrainerGenerator(gen, gpu=None if gen_device.type == "cpu" else gen_device.index or 0)
    got["pre_train/loss"] = _logged(lambda: solver_g.train(dataset, **cfg["pre_train"]))
    got["probe/pre_train"] = _probe()
    got["gen_pre"] = {k: v.detach().cpu().numpy().copy() for k, v in gen.state_dict().items()}
    got["pre/log_prob"] = np.asarray(solver_g.log_probability([list(r) for r in mined]))
    prefixes = json.loads(str(z["pre/next_prefix"]))
    got["pre/next_logp"] = np.asarray([solver_g.next_relation_log_probability(p, 0.2) for p in prefixes])
    got["pre/beam"] = solver_g.beam_search(**cfg["beam"])
    got["probe/beam"] = _probe()
    # run_rnnlogic.py:67-70: the EM iteration starts from the generator's samples
    got["em/sampled"] = solver_g.sample(**cfg["sample"])
    got["probe/sample"] = _probe()
    if not em or stop_after_sample:
        return z, got

    from rnnlogic_amd.predictors import Predictor
    from rnnlogic_amd.trainer import TrainerPredictor
    sampled = json.loads(str(z["em/sampled"]))  # the reference's rules (equal to ours when the test passes)
    prior = [rule[-1] for rule in sampled]
    rules = [rule[0:-1] for rule in sampled]
    predictor = Predictor(graph, entity_feature="bias")
    predictor.set_rules([list(r) for r in rules])
    got["pred_init"] = {k: v.detach().cpu().numpy().copy() for k, v in predictor.state_dict().items()}
    optim = torch.optim.Adam(predictor.parameters(), lr=1e-3, weight_decay=0)
    solver_p = TrainerPredictor(predictor, train_set, valid_set, test_set, optim, gpus=[gpu])
    got["em/train_loss"] = _logged(lambda: solver_p.train(**cfg["predictor_train"]))
    got["probe/em_train"] = _probe()
    got["pred_trained"] = {k: v.detach().cpu().numpy().copy() for k, v in predictor.state_dict().items()}
    got["em/valid_mrr"] = solver_p.evaluate("valid", expectation=True)
    got["em/test_mrr"] = solver_p.evaluate("test", expectation=True)
    likelihood = solver_p.compute_H(print_every=1000)
    got["em/H"] = np.asarray(likelihood)
    posterior = [l + p * cfg["prior_weight"] for l, p in zip(likelihood, prior)]
    got["em/posterior"] = np.asarray(posterior)
    got["probe/em_H"] = _probe()
    for i in range(len(rules)):
        rules[i].append(posterior[i])
    got["m_step/loss"] = _logged(lambda: solver_g.train(RuleDataset(graph.relation_size, rules), **cfg["m_step"]))
    got["probe/m_step"] = _probe()
    got["m_step/log_prob"] = np.asarray(solver_g.log_probability([list(r[:-1]) for r in rules]))
    got["gen_m"] = {k: v.detach().cpu().numpy().copy() for k, v in gen.state_dict().items()}
    return z, got


def _logged(fn):
    """Run fn, return the mean losses it logged ("<step> <total> <loss> ...")."""
    import io
    import logging
    stream = io.StringIO()
    h = logging.StreamHandler(stream)
    root = logging.getLogger()
    old = root.level
    root.addHandler(h)
    root.setLevel(logging.INFO)
    try:
        fn()
    finally:
        root.removeHandler(h)
        root.setLevel(old)
    vals = []
    for line in stream.getvalue().splitlines():
        parts = line.split()
        if len(parts) >= 3 and parts[0].isdigit():
            vals.append(float(parts[2]))
    return np.asarray(vals)


def state(z, prefix):
    return {k[len(prefix) + 1:]: z[k] for k in z.files if k.startswith(prefix + "/")}


def check_beam(got, want, score_tol=1e-5):
    """Same rules per relation; scores within score_tol; an order swap is
    allowed only between rules whose scores lie within score_tol."""
    assert len(got) == len(want)
    for g, w in zip(got, want):
        if g[:-1] != w[:-1]:
            assert abs(g[-1] - w[-1]) <= score_tol, (g, w)
        assert abs(g[-1] - w[-1]) <= score_tol, (g, w)
    assert sorted(tuple(g[:-1]) for g in got) == sorted(tuple(w[:-1]) for w in want)
