"""RotatE entity-feature scorer, parameter-compatible with the reference's
src/embedding.py (parameters `eemb` (|E|, 2D) and `remb` (2 nrel, D) with the
negated inverse half, embedding.py:7-26).

forward() on a GPU runs the HIP kernel rnnl_rotate_score (rotate.hip): every
(query, entity) distance for a block of 32 query rows is computed from one
pass over the (transposed) entity table.
"""
import json
import os

import numpy as np
import torch

from . import _native


class RotatE(torch.nn.Module):
    def __init__(self, path):
        super(RotatE, self).__init__()
        self.path = path
        with open(os.path.join(path, "config.json"), "r") as fi:
            cfg = json.load(fi)
        self.emb_dim = cfg["hidden_dim"]
        self.gamma = cfg["gamma"]
        self.range = (self.gamma + 2.0) / self.emb_dim
        self.num_entities = cfg["nentity"]
        eemb = np.load(os.path.join(path, "entity_embedding.npy"), allow_pickle=False)
        self.eemb = torch.nn.parameter.Parameter(torch.tensor(eemb))
        remb = torch.tensor(np.load(os.path.join(path, "relation_embedding.npy"), allow_pickle=False))
        self.remb = torch.nn.parameter.Parameter(torch.cat([remb, -remb], dim=0))
        self._t_cache = None

    def _transposed(self):
        """(2D, |E|) copy of eemb for coalesced loads, rebuilt when eemb changes."""
        key = (self.eemb.data_ptr(), self.eemb._version, self.eemb.device)
        if self._t_cache is None or self._t_cache[0] != key:
            t = torch.empty((self.eemb.size(1), self.eemb.size(0)), dtype=torch.float32, device=self.eemb.device)
            _native.call("rnnl_rotate_transpose", self.eemb.data_ptr(), self.eemb.size(0), self.eemb.size(1),
                         t.data_ptr(), torch.cuda.current_stream(self.eemb.device).cuda_stream)
            self._t_cache = (key, t)
        return self._t_cache[1]

    def score_into(self, all_h, all_r, out, accumulate=False):
        """out (B, |E|) (+)= gamma - dist(h o r, e) for every entity (HIP)."""
        if not self.eemb.is_cuda:
            raise RuntimeError("RotatE.forward runs on the HIP path; move the module to a GPU")
        all_h = all_h.to(self.eemb.device, torch.int64).contiguous()
        all_r = all_r.to(self.eemb.device, torch.int64).contiguous()
        eemb = self.eemb.detach().contiguous()
        remb = self.remb.detach().contiguous()
        _native.call("rnnl_rotate_score", eemb.data_ptr(), self._transposed().data_ptr(), remb.data_ptr(),
                     self.emb_dim, float(self.gamma), all_h.data_ptr(), all_r.data_ptr(), all_h.numel(),
                     self.num_entities, out.data_ptr(), 1 if accumulate else 0,
                     torch.cuda.current_stream(self.eemb.device).cuda_stream)
        return out

    def forward(self, all_h, all_r):
        """(B, |E|) = gamma - sum_d |h o r - e| (embedding.py:64-70)."""
        out = torch.empty((all_h.numel(), self.num_entities), dtype=torch.float32, device=self.eemb.device)
        return self.score_into(all_h, all_r, out)
