"""A/B of the EM Predictor's training paths on the UMLS EM fixture (GPU box):
the HIP backward (_PredictorLinear, default) against torch autograd on the
grounding COO (Predictor.forward_autograd), each run through the same EM
chain (tests/em_chain.py) and compared with the reference's logged losses,
trained weights and MRRs.  Usage: python tools/em_path_ab.py"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import em_chain  # noqa: E402
from rnnlogic_amd import predictors  # noqa: E402


def run(label):
    z, got = em_chain.run(torch.device("cuda:0"), em=True, gen_device=torch.device("cpu"))
    w = em_chain.state(z, "pred_trained")
    d = np.abs(got["pred_trained"]["rule_weights"] - w["rule_weights"])
    print("%s: train_loss err %s | rule_weights max err %.3g (n > 1e-5: %d) | valid MRR %.6f (ref %.6f) "
          "test MRR %.6f (ref %.6f)" % (label, np.round(got["em/train_loss"] - z["em/train_loss"], 7), d.max(),
                                        int((d > 1e-5).sum()), got["em/valid_mrr"], float(z["em/valid_mrr"]),
                                        got["em/test_mrr"], float(z["em/test_mrr"])), flush=True)


run("hip backward")
orig = predictors.Predictor.forward


def coo_forward(self, all_h, all_r, edges_to_remove):
    if self._needs_grad():
        return self.forward_autograd(all_h, all_r, edges_to_remove)
    return orig(self, all_h, all_r, edges_to_remove)


predictors.Predictor.forward = coo_forward
run("torch autograd on the COO")
