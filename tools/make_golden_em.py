"""Golden vectors for the EM loop (run_rnnlogic.py:45-91) on UMLS.

Runs the *reference* Generator / TrainerGenerator / Predictor / TrainerPredictor
(imported from /root/reference/src with the test-only shims of
tools/ref_shims, as tools/make_golden.py does) on CPU, in the order
run_rnnlogic.py calls them, from set_seed(1):

  1. Generator(graph, num_layers=1, embedding_dim=32, hidden_dim=32): seeded
     state_dict;
  2. generator pre-training on a RuleDataset of the UMLS mined rules (weights
     below): logged mean losses, state_dict after, log_probability of every
     rule, next_relation_log_probability of a few prefixes, beam_search;
  3. one EM iteration as run_rnnlogic.py:67-91 runs it: sampled_rules =
     TrainerGenerator.sample(num_rules, max_length) on the CPU (its rules,
     in the reference's own order, and their log-probabilities), prior =
     rule[-1]; Predictor(bias) + Adam, TrainerPredictor train (logged losses)
     / evaluate valid + test / compute_H -> likelihood, posterior =
     likelihood + prior_weight * prior, then the M-step generator.train on
     the posterior-weighted rules (logged losses, final log_probability).
  After each stage the global torch RNG is probed (4 int draws), so a
  drop-in whose DataLoaders consume the RNG differently is caught.

TrainerGenerator.__init__ calls model.cuda(device) even for gpu=None (no GPU
here), so nn.Module.cuda is made the identity while the reference runs.

Output: tests/golden/em_umls.npz.   Usage: python tools/make_golden_em.py
"""
import io
import json
import logging
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as MG  # noqa: E402  (reference import path + shims)

import torch  # noqa: E402

import generators as R_gen  # noqa: E402  (reference src/generators.py)

CFG = dict(seed=1, gen=dict(num_layers=1, embedding_dim=32, hidden_dim=32),
           pre_train=dict(num_epoch=60, lr=1e-3, print_every=20, batch_size=256),
           beam=dict(num_samples=8, max_len=2), sample=dict(num_samples=20, max_len=3), prior_weight=0.001,
           predictor_train=dict(batch_per_epoch=40, smoothing=0.2, print_every=10),
           m_step=dict(num_epoch=30, lr=1e-3, print_every=10, batch_size=256))


def rule_weight(i):
    """Deterministic prior weights for the mined rules (the committed file has
    no H column)."""
    return 0.25 * ((i * 37) % 11) - 1.0


def cpu_model():
    """The CPU the fixture was made on: CPU float results (LSTM GEMMs) are
    bitwise reproducible on the same CPU model only."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def probe():
    return torch.randint(0, 2 ** 31 - 1, (4,)).numpy()


class _Log(object):
    def __enter__(self):
        self.stream = io.StringIO()
        self.h = logging.StreamHandler(self.stream)
        logging.getLogger().addHandler(self.h)
        logging.getLogger().setLevel(logging.INFO)
        return self

    def __exit__(self, *a):
        logging.getLogger().removeHandler(self.h)

    def numbers(self, col):
        out = []
        for line in self.stream.getvalue().splitlines():
            parts = line.split()
            if len(parts) >= 3 and parts[0].isdigit():
                out.append(float(parts[col]))
        return np.asarray(out, np.float64)


def main():
    torch.set_num_threads(8)
    torch.nn.Module.cuda = lambda self, device=None: self
    path = MG.datasets.materialize("umls")
    rule_path = MG.datasets.rule_file("umls")
    mined = [[int(x) for x in line.split()] for line in open(rule_path)]
    out = dict(cfg=np.array(json.dumps(CFG)), cpu=np.array(cpu_model()))

    MG.R_utils.set_seed(CFG["seed"])
    graph = MG.R_data.KnowledgeGraph(path)
    train_set = MG.R_data.TrainDataset(graph, 32)
    valid_set = MG.R_data.ValidDataset(graph, 32)
    test_set = MG.R_data.TestDataset(graph, 32)
    weighted = [r + [rule_weight(i)] for i, r in enumerate(mined)]
    dataset = MG.R_data.RuleDataset(graph.relation_size, [list(r) for r in weighted])

    gen = R_gen.Generator(graph, **CFG["gen"])
    for k, v in gen.state_dict().items():
        out["gen_init/" + k] = v.numpy().copy()
    solver_g = MG.R_trainer.TrainerGenerator(gen, gpu=None)
    with _Log() as lg:
        solver_g.train(dataset, **CFG["pre_train"])
    out["pre_train/loss"] = lg.numbers(2)
    out["probe/pre_train"] = probe()
    for k, v in gen.state_dict().items():
        out["gen_pre/" + k] = v.numpy().copy()
    out["pre/log_prob"] = np.asarray(solver_g.log_probability([list(r) for r in mined]), np.float64)
    prefixes = [[0], [3, 7], [12, 1, 40], [45]]
    out["pre/next_prefix"] = np.array(json.dumps(prefixes))
    out["pre/next_logp"] = np.asarray([solver_g.next_relation_log_probability(p, 0.2) for p in prefixes])
    beam = solver_g.beam_search(**CFG["beam"])
    out["pre/beam"] = np.array(json.dumps(beam))
    out["probe/beam"] = probe()

    # ---- one EM iteration (run_rnnlogic.py:67-91), starting from sample()
    sampled = solver_g.sample(**CFG["sample"])
    out["em/sampled"] = np.array(json.dumps(sampled))
    out["probe/sample"] = probe()
    prior = [rule[-1] for rule in sampled]
    rules = [rule[0:-1] for rule in sampled]
    predictor = MG.R_pred.Predictor(graph, entity_feature="bias")
    predictor.set_rules([list(r) for r in rules])
    for k, v in predictor.state_dict().items():
        out["pred_init/" + k] = v.numpy().copy()
    optim = torch.optim.Adam(predictor.parameters(), lr=1e-3, weight_decay=0)
    solver_p = MG.R_trainer.TrainerPredictor(predictor, train_set, valid_set, test_set, optim, gpus=None)
    with _Log() as lg:
        solver_p.train(**CFG["predictor_train"])
    out["em/train_loss"] = lg.numbers(2)
    out["probe/em_train"] = probe()
    for k, v in predictor.state_dict().items():
        out["pred_trained/" + k] = v.numpy().copy()
    out["em/valid_mrr"] = np.float64(solver_p.evaluate("valid", expectation=True))
    out["em/test_mrr"] = np.float64(solver_p.evaluate("test", expectation=True))
    likelihood = solver_p.compute_H(print_every=1000)
    out["em/H"] = np.asarray(likelihood, np.float64)
    posterior = [l + p * CFG["prior_weight"] for l, p in zip(likelihood, prior)]
    out["em/posterior"] = np.asarray(posterior, np.float64)
    out["probe/em_H"] = probe()
    for i in range(len(rules)):
        rules[i].append(posterior[i])
    dataset = MG.R_data.RuleDataset(graph.relation_size, rules)
    with _Log() as lg:
        solver_g.train(dataset, **CFG["m_step"])
    out["m_step/loss"] = lg.numbers(2)
    out["probe/m_step"] = probe()
    out["m_step/log_prob"] = np.asarray(solver_g.log_probability([list(r[:-1]) for r in rules]), np.float64)
    for k, v in gen.state_dict().items():
        out["gen_m/" + k] = v.numpy().copy()

    dst = os.path.join(MG.OUT, "em_umls.npz")
    np.savez_compressed(dst, **out)
    print("em_umls ->", dst, os.path.getsize(dst))
    print("pre_train losses", out["pre_train/loss"], "em losses", out["em/train_loss"],
          "mrr", out["em/valid_mrr"], out["em/test_mrr"], "m-step", out["m_step/loss"], "beam rules", len(beam))


if __name__ == "__main__":
    main()
