"""RotatE entity-feature scorer, parameter-compatible with the reference's
src/embedding.py (parameters `eemb` (|E|, 2D) and `remb` (2 nrel, D) with the
negated inverse half, embedding.py:7-26).

forward() on a GPU runs the HIP kernel rnnl_rotate_score (rotate.hip) over
two weight-derived device tables (entity planes, relation cos/sin) that are
built once per weight version.
"""
import ctypes
import json
import os

import numpy as np
import torch

from . import _native


class _RotatEScore(torch.autograd.Function):
    """score = gamma - sum_d |h o r - t| for every (row, entity): forward by the
    HIP scorer (rnnl_rotate_score), backward by rnnl_rotate_param_grads, which
    writes dL/d eemb (tail term + head rows) and dL/d remb in eemb's / remb's
    layouts — no (B, |E|, D) difference tensors, no dense embedding-gather
    gradient, no transposing copy, and none of the torch launches that formed
    h o r for autograd."""

    @staticmethod
    def forward(ctx, eemb, remb, module, all_h, all_r):
        out = torch.empty((all_h.numel(), module.num_entities), dtype=torch.float32, device=eemb.device)
        module.score_into(all_h, all_r, out)
        ctx.module = module
        ctx.save_for_backward(all_h, all_r)
        return out

    @staticmethod
    def backward(ctx, grad):
        all_h, all_r = ctx.saved_tensors
        m = ctx.module
        E, D = m.num_entities, m.emb_dim
        dev = grad.device
        nq = all_h.numel()
        need_e, need_r = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        if not (need_e or need_r):
            return None, None, None, None, None
        planes, rtab = m._device_tables()  # cached for this weight version by the forward
        if m.mode == _native.ROTATE_DIRECT:
            ld = planes.numel() // (2 * D)  # the forward's entity planes [D][2][ld]
        else:
            planes = m.eemb.detach().view(E, 2, D).permute(2, 1, 0).contiguous()
            ld = E
        grad = grad.detach().float().contiguous()
        nb = ctypes.c_size_t()
        _native.call("rnnl_rotate_param_grads_scratch", nq, E, D, int(need_e), ctypes.byref(nb))
        scratch = m._grad_scratch(nb.value)
        d_eemb = torch.empty((E, 2 * D), dtype=torch.float32, device=dev) if need_e else None
        d_remb = torch.empty_like(m.remb, dtype=torch.float32) if need_r else None
        eemb = m.eemb.detach().contiguous()
        _native.call("rnnl_rotate_param_grads", eemb.data_ptr(), planes.data_ptr(), ld, rtab.data_ptr(),
                     float(m.gamma), all_h.data_ptr(), all_r.data_ptr(), nq, E, D, m.remb.size(0), grad.data_ptr(),
                     scratch.data_ptr(), scratch.numel(), d_eemb.data_ptr() if need_e else None,
                     d_remb.data_ptr() if need_r else None, torch.cuda.current_stream(dev).cuda_stream)
        return d_eemb, d_remb, None, None, None


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
        self._tables = None
        self._ws = None
        self._ws_need = {}
        self._args = None  # (key, rnnl_rotate_args) of native_args
        # DIRECT (default) evaluates the reference's arithmetic term by term;
        # mode = ROTATE_MFMA selects the faster expanded bf16x3 MFMA kernel
        # (cancellation-prone when h o r ~= t; include/rnnlogic_hip.h)
        self.mode = _native.ROTATE_DIRECT

    def _device_tables(self):
        """Weight-derived tables (rotate.hip header), rebuilt when eemb/remb or
        the mode change: the mode's entity table and the relation (cos, sin)."""
        dev = self.eemb.device
        key = (self.eemb.data_ptr(), self.eemb._version, self.remb.data_ptr(), self.remb._version, dev,
               int(self.mode))
        if self._tables is None or self._tables[0] != key:
            E, D, R2 = self.num_entities, self.emb_dim, self.remb.size(0)
            eb, rb = ctypes.c_size_t(), ctypes.c_size_t()
            _native.call("rnnl_rotate_table_sizes", E, D, R2, int(self.mode), ctypes.byref(eb), ctypes.byref(rb))
            etab = torch.empty(eb.value // 4, dtype=torch.float32, device=dev)
            rtab = torch.empty(rb.value // 4, dtype=torch.float32, device=dev)
            stream = torch.cuda.current_stream(dev).cuda_stream
            eemb = self.eemb.detach().contiguous()
            remb = self.remb.detach().contiguous()
            _native.call("rnnl_rotate_entity_table", eemb.data_ptr(), E, D, int(self.mode), etab.data_ptr(), stream)
            _native.call("rnnl_rotate_relation_table", remb.data_ptr(), R2, D, float(self.gamma), rtab.data_ptr(),
                         stream)
            self._tables = (key, etab, rtab)
        return self._tables[1], self._tables[2]

    def _workspace(self, nq):
        key = (nq, int(self.mode))
        need = self._ws_need.get(key)
        if need is None:
            need = ctypes.c_size_t()
            _native.call("rnnl_rotate_workspace_size", nq, self.num_entities, self.emb_dim, int(self.mode),
                         ctypes.byref(need))
            self._ws_need[key] = need
        if need.value == 0:
            return None, 0
        if self._ws is None or self._ws.numel() * 4 < need.value or self._ws.device != self.eemb.device:
            self._ws = torch.empty((need.value + 3) // 4, dtype=torch.float32, device=self.eemb.device)
        return self._ws.data_ptr(), need.value

    def _grad_scratch(self, nbytes):
        """Device scratch of rnnl_rotate_param_grads (kept across steps; the
        stream orders its reuse)."""
        g = getattr(self, "_gs", None)
        if g is None or g.numel() < nbytes or g.device != self.eemb.device:
            g = self._gs = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=self.eemb.device)
        return g

    def native_args(self, nq, pieces=1, first_share=0.0):
        """rnnl_rotate_args for a launch over nq rows (the one-call forward,
        rnnl_predictorplus_forward_rotate): the weight tables and workspace
        of score_into, rebuilt only when the weights or the row count change."""
        if not self.eemb.is_cuda:
            raise RuntimeError("RotatE.forward runs on the HIP path; move the module to a GPU")
        if not self.eemb.is_contiguous():
            raise RuntimeError("RotatE.eemb must be contiguous")
        etab, rtab = self._device_tables()
        ws, ws_bytes = self._workspace(nq)
        key = (etab.data_ptr(), rtab.data_ptr(), self.eemb.data_ptr(), ws, ws_bytes, int(self.mode), int(pieces),
               float(first_share))
        a = self._args
        if a is None or a[0] != key:
            args = _native.RotateArgs(self.eemb.data_ptr(), etab.data_ptr(), rtab.data_ptr(), self.emb_dim,
                                      self.num_entities, float(self.gamma), int(self.mode), ws, ws_bytes, int(pieces),
                                      float(first_share))
            self._args = a = (key, args)
        return a[1]

    @_native.on_input_device
    def score_into(self, all_h, all_r, out, accumulate=False, pieces=1, first_share=0.0):
        """out (B, |E|) (+)= gamma - dist(h o r, e) for every entity (HIP);
        accumulate 2: atomic adds (rnnl_rotate_score).  pieces > 1: the same
        scores, bitwise, from that many launches (rnnl_rotate_score_pieces)."""
        if not self.eemb.is_cuda:
            raise RuntimeError("RotatE.forward runs on the HIP path; move the module to a GPU")
        all_h = all_h.to(self.eemb.device, torch.int64).contiguous()
        all_r = all_r.to(self.eemb.device, torch.int64).contiguous()
        eemb = self.eemb.detach().contiguous()
        etab, rtab = self._device_tables()
        ws, ws_bytes = self._workspace(all_h.numel())
        _native.call("rnnl_rotate_score_pieces", eemb.data_ptr(), etab.data_ptr(), rtab.data_ptr(),
                     self.emb_dim, float(self.gamma), all_h.data_ptr(), all_r.data_ptr(), all_h.numel(),
                     self.num_entities, out.data_ptr(), int(accumulate), int(self.mode), ws, ws_bytes,
                     int(pieces), float(first_share), torch.cuda.current_stream(self.eemb.device).cuda_stream)
        return out

    def forward_torch(self, all_h, all_r):
        """Differentiable (B, |E|) scores as torch ops (training path): the
        reference's arithmetic (embedding.py:28-70) without expanding h and r
        to (B * |E|) rows — h o r is formed once per row."""
        pi = 3.141592653589793238462643383279
        D = self.emb_dim
        h = self.eemb.index_select(0, all_h)
        phase = self.remb.index_select(0, all_r) / (self.range / pi)
        re_r, im_r = torch.cos(phase), torch.sin(phase)
        re_h, im_h = h[:, :D], h[:, D:]
        re_hr = re_h * re_r - im_h * im_r
        im_hr = re_h * im_r + im_h * re_r
        re_t, im_t = self.eemb[:, :D], self.eemb[:, D:]
        diff = torch.stack([re_hr.unsqueeze(1) - re_t.unsqueeze(0), im_hr.unsqueeze(1) - im_t.unsqueeze(0)], dim=0)
        return self.gamma - diff.norm(dim=0).sum(dim=-1)

    @_native.on_input_device
    def forward_grad(self, all_h, all_r):
        """Differentiable (B, |E|) scores for training: the HIP scorer forward
        and rnnl_rotate_param_grads (_RotatEScore), which carries the gradient
        to the tail entities, the head rows and the relation phases."""
        all_h = all_h.to(self.eemb.device, torch.int64).contiguous()
        all_r = all_r.to(self.eemb.device, torch.int64).contiguous()
        return _RotatEScore.apply(self.eemb, self.remb, self, all_h, all_r)

    @_native.on_input_device
    def forward(self, all_h, all_r):
        """(B, |E|) = gamma - sum_d |h o r - e| (embedding.py:64-70): the HIP
        kernel; with autograd active (training) the same kernel plus its HIP
        backward (forward_grad)."""
        if torch.is_grad_enabled() and (self.eemb.requires_grad or self.remb.requires_grad):
            return self.forward_grad(all_h, all_r)
        out = torch.empty((all_h.numel(), self.num_entities), dtype=torch.float32, device=self.eemb.device)
        return self.score_into(all_h, all_r, out)
