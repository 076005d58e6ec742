"""Reasoning predictors, API-compatible with the reference's src/predictors.py.

PredictorPlus keeps the reference's constructor, set_rules, encode_rules and
forward signatures and its exact module tree (so state_dict keys/shapes match
and a seeded construction consumes the RNG identically).  Its forward runs on
the HIP path:

    rule embeddings (emb table or LSTM encoder, torch)         predictors.py:201-208, 246-249
      -> per-trie-node aggregates          rnnl_node_weights (HIP)
    base score  bias row / RotatE / -inf   rnnl_fill_rows / rnnl_rotate_score (HIP)
    grounding + aggregation + MLP          rnnl_predictorplus_forward (HIP, one launch)

Predictor (the EM loop's rule-weight model) runs on the same grounding:
score = exact fixed-point sums of count x per-node rule-weight sums
(rnnl_predictor_forward), compute_H from per-node path statistics
(rnnl_predictor_rule_stats).  Training forwards of both run torch autograd on
the exported grounding COO.

There is no CPU fallback: on a CPU tensor forward() raises.
"""
import collections
import ctypes
import logging
import math

import numpy as np
import torch
import torch.nn as nn

from . import _native
from .data import _DeviceHandle
from .embedding import RotatE
from .layers import MLP, FuncToNode, FuncToNodeSum


def _read_rules(input):
    """Rule list/file -> [(head, [body...])] (predictors.py:27-41, 166-182)."""
    rules = []
    if isinstance(input, list):
        for rule in input:
            rules.append((rule[0], list(rule[1:])))
    elif isinstance(input, str):
        with open(input, "r") as fi:
            for line in fi:
                rule = [int(_) for _ in line.strip().split()]
                rules.append((rule[0], rule[1:]))
    else:
        raise ValueError
    return rules


class _NativeRules(object):
    """Per-device rnnl_rules handle (prefix tries of the rule bodies)."""

    def __init__(self, graph, rules, device):
        flat, ptr = [], [0]
        for head, body in rules:
            flat.append(head)
            flat.extend(body)
            ptr.append(len(flat))
        tok = np.ascontiguousarray(flat, dtype=np.int32)
        ptr = np.ascontiguousarray(ptr, dtype=np.int64)
        h = ctypes.c_void_p()
        with torch.cuda.device(device):
            _native.call("rnnl_rules_create", graph.device_graph(device), tok.ctypes.data_as(ctypes.c_void_p),
                         ptr.ctypes.data_as(ctypes.c_void_p), len(rules), ctypes.byref(h))
        self.handle = _DeviceHandle(h, "rnnl_rules_destroy")
        info = (ctypes.c_int32 * 5)()
        _native.call("rnnl_rules_info", h, info)
        self.n_rules, self.n_nodes, self.max_depth = info[0], info[1], info[2]
        self.record_bytes = (info[3], info[4])
        n2r = np.zeros(max(len(rules), 1), dtype=np.int32)
        _native.call("rnnl_rules_node_of_rule", h, n2r.ctypes.data_as(ctypes.c_void_p))
        self.node_of_rule = torch.from_numpy(n2r[:len(rules)].astype(np.int64)).to(torch.device("cuda", device))

    @property
    def ptr(self):
        return self.handle.ptr


class _HipGrounding(object):
    """Grounding plumbing shared by Predictor and PredictorPlus: the per-device
    rules handle (prefix tries), the forward workspace with its overflow retry,
    and the grounding COO export.  Needs self.graph, self.rules,
    self._native_rules, self._ws and self.capacity_scale."""

    def _device_index(self, device):
        return device.index if device.index is not None else torch.cuda.current_device()

    def native_rules(self, device):
        key = self._device_index(device)
        if key not in self._native_rules:
            self._native_rules[key] = _NativeRules(self.graph, self.rules, key)
        return self._native_rules[key]

    def _workspace(self, device, nq, scale):
        g, nr = self.graph.device_graph(device), self.native_rules(device)
        need = ctypes.c_size_t()
        _native.call("rnnl_forward_workspace_size", g, nr.ptr, nq, scale, ctypes.byref(need))
        ws = self._ws.get(device)
        if ws is None or ws.numel() < need.value:
            ws = torch.empty(need.value, dtype=torch.uint8, device=device)
            self._ws[device] = ws
        return ws

    @staticmethod
    def _rows(all_h, all_r, edges_to_remove):
        device = all_h.device
        if device.type != "cuda":
            raise RuntimeError("the predictors run on the HIP path: move inputs and model to a GPU")
        all_h = all_h.to(torch.int64).contiguous()
        all_r = all_r.to(device, torch.int64).contiguous()
        etr = edges_to_remove.to(device, torch.int64).contiguous() if edges_to_remove is not None else None
        return device, all_h, all_r, etr

    def _status(self, ws, stream, totals=None):
        """The launch's status (rnnl_forward_status_flags: one read-back), with
        the grounding's candidate / bucket-entry totals into `totals`
        (int64[2] numpy array, nullable) and its flags kept in self._flags
        (bit 0: the rows hold more than one relation)."""
        rc = _native.lib().rnnl_forward_status_flags(
            ws.data_ptr(), stream, totals.ctypes.data_as(ctypes.c_void_p) if totals is not None else None,
            self._flags.ctypes.data_as(ctypes.c_void_p))
        return rc

    def _check_one_relation(self):
        """The reference forward's one-relation-per-batch assertion
        (predictors.py:54-55, 211-212), from the last launch's flags."""
        assert not (int(self._flags[0]) & _native.FLAG_MIXED), "a batch must hold one relation (predictors.py:54-55)"

    def _launch(self, device, nq, run, totals=None, tolerate_range=False):
        """run(ws, scale) launches onto the workspace; retried with a doubled
        capacity_scale while the launch reports overflow.  Returns (ws, scale).
        `totals` (int64[2] numpy array): filled with the grounding's candidate
        and bucket-entry totals by the same read-back as the status.
        tolerate_range: return on RNNL_ERR_RANGE as well (the caller reads
        the rows' n_cand: -2 marks a row whose path counts reached 2^32)."""
        stream = torch.cuda.current_stream(device).cuda_stream
        while True:
            scale = self.capacity_scale
            ws = self._workspace(device, nq, scale)
            run(ws, scale)
            rc = self._status(ws, stream, totals)
            if rc == _native.RNNL_ERR_OVERFLOW and self.capacity_scale < 64:
                self.capacity_scale *= 2
                logging.info("%s: workspace overflow, capacity_scale -> %d", type(self).__name__,
                             self.capacity_scale)
                continue
            if not (tolerate_range and rc == _native.RNNL_ERR_RANGE):
                _native.check(rc)
            self._ws_touch(ws)
            return ws, scale

    def _ws_touch(self, ws):
        """Count a launch onto workspace `ws`: a grounding saved for a backward
        is stale once its workspace's count moves on."""
        self._ws_uses[ws.data_ptr()] = self._ws_uses.get(ws.data_ptr(), 0) + 1
        return self._ws_uses[ws.data_ptr()]

    @_native.on_input_device
    def ground(self, all_h, all_r, edges_to_remove=None, totals=None, tolerate_range=False):
        """Grounding of every rule of every row into the workspace (HIP
        rnnl_ground).  Returns (ws, scale, n_cand (n,) int32); `totals` and
        `tolerate_range` as in _launch."""
        device, all_h, all_r, etr = self._rows(all_h, all_r, edges_to_remove)
        nq = all_h.numel()
        g, nr = self.graph.device_graph(device), self.native_rules(device)
        stream = torch.cuda.current_stream(device).cuda_stream
        n_cand = torch.empty(nq, dtype=torch.int32, device=device)

        def run(ws, scale):
            _native.call("rnnl_ground", g, nr.ptr, all_h.data_ptr(), all_r.data_ptr(),
                         etr.data_ptr() if etr is not None else None, nq, n_cand.data_ptr(), ws.data_ptr(),
                         ws.numel(), scale, stream)
        ws, scale = self._launch(device, nq, run, totals, tolerate_range)
        return ws, scale, n_cand

    @_native.on_input_device
    def ground_coo(self, all_h, all_r, edges_to_remove=None):
        """The grounding COO (see _ground_coo) with exact int64 counts for
        every row: rows whose path counts reach 2^32 (the grounding kernel's
        u32 sums; RNNL_ERR_RANGE) are grounded again by rnnl_ground_wide, as
        the reference counts in int64 (src/data.py:139-171)."""
        try:
            return self._ground_coo(all_h, all_r, edges_to_remove)
        except _native.NativeError as e:
            if e.code != _native.RNNL_ERR_RANGE:
                raise
        return self._ground_coo_wide(all_h, all_r, edges_to_remove)

    def _ground_coo_wide(self, all_h, all_r, edges_to_remove):
        device, h, r, etr = self._rows(all_h, all_r, edges_to_remove)
        nq, E = h.numel(), self.graph.entity_size
        _, _, n_cand = self.ground(h, r, etr, tolerate_range=True)
        bad = torch.nonzero(n_cand == -2).squeeze(1)
        good = torch.nonzero(n_cand != -2).squeeze(1)
        keys, nodes, counts = [], [], []
        if good.numel():
            row, ent, ce, node, count = self._ground_coo(h[good], r[good], etr[good] if etr is not None else None)
            keys.append(good[row][ce] * E + ent[ce])
            nodes.append(node)
            counts.append(count)
        if bad.numel():
            g, nr = self.graph.device_graph(device), self.native_rules(device)
            stream = torch.cuda.current_stream(device).cuda_stream
            rows32 = bad.to(torch.int32).contiguous()
            sb = ctypes.c_size_t()
            _native.call("rnnl_ground_wide_scratch_bytes", g, rows32.numel(), ctypes.byref(sb))
            scratch = torch.empty(sb.value, dtype=torch.uint8, device=device)
            cursor = torch.zeros(1, dtype=torch.int64, device=device)
            cap = 1 << 16
            while True:
                o_row = torch.empty(cap, dtype=torch.int32, device=device)
                o_ent = torch.empty(cap, dtype=torch.int32, device=device)
                o_node = torch.empty(cap, dtype=torch.int32, device=device)
                o_cnt = torch.empty(cap, dtype=torch.int64, device=device)
                _native.call("rnnl_ground_wide", g, nr.ptr, h.data_ptr(), r.data_ptr(),
                             etr.data_ptr() if etr is not None else None, rows32.data_ptr(), rows32.numel(),
                             scratch.data_ptr(), scratch.numel(), o_row.data_ptr(), o_ent.data_ptr(),
                             o_node.data_ptr(), o_cnt.data_ptr(), cap, cursor.data_ptr(), stream)
                n = int(cursor.item())
                if n <= cap:
                    break
                cap = n
            keys.append(o_row[:n].to(torch.int64) * E + o_ent[:n].to(torch.int64))
            nodes.append(o_node[:n].to(torch.int64))
            counts.append(o_cnt[:n])  # u64 counts < 2^63 (more paths than int64 would hold: as the reference)
        key = torch.cat(keys) if keys else torch.zeros(0, dtype=torch.int64, device=device)
        node = torch.cat(nodes) if nodes else torch.zeros(0, dtype=torch.int64, device=device)
        count = torch.cat(counts) if counts else torch.zeros(0, dtype=torch.int64, device=device)
        # the reference's order: candidates row-major by entity (nonzero), entries by node
        order = torch.argsort(key * max(self.native_rules(device).n_nodes, 1) + node)
        key, node, count = key[order], node[order], count[order]
        cand, ce = torch.unique_consecutive(key, return_inverse=True)
        return cand // E, cand % E, ce, node, count

    def _ground_coo(self, all_h, all_r, edges_to_remove=None):
        """The grounding of every rule of every row as the COO of the
        reference's stacked rule_count matrix (HIP: rnnl_ground + export).

        Returns (row (C,), entity (C,), cand_of_entry (P,), node (P,), count (P,))
        int64 device tensors: candidates in row-major order (= the reference's
        nonzero order, predictors.py:239) and, per candidate, its (trie node,
        path count) entries; node ids index `native_rules(device).node_of_rule`."""
        device = all_h.device
        nq = all_h.numel()
        totals = np.zeros(2, dtype=np.int64)  # (candidates, bucket entries) with the status read-back
        ws, scale, n_cand = self.ground(all_h, all_r, edges_to_remove, totals)
        stream = torch.cuda.current_stream(device).cuda_stream
        nc = n_cand.to(torch.int64)
        cand_off = torch.zeros(nq + 1, dtype=torch.int64, device=device)
        torch.cumsum(nc, 0, out=cand_off[1:])
        C, P = int(totals[0]), int(totals[1])
        ent = torch.empty(max(C, 1), dtype=torch.int32, device=device)
        nent = torch.empty(max(C, 1), dtype=torch.int32, device=device)
        _native.call("rnnl_ground_export_candidates", ws.data_ptr(), nq, scale, n_cand.data_ptr(),
                     cand_off.data_ptr(), ent.data_ptr(), nent.data_ptr(), stream)
        ent, nent = ent[:C].to(torch.int64), nent[:C].to(torch.int64)
        row = torch.repeat_interleave(torch.arange(nq, device=device), nc, output_size=C)  # (no size sync)
        per_row = torch.zeros(nq, dtype=torch.int64, device=device).index_add_(0, row, nent)
        ent_off = torch.zeros(nq + 1, dtype=torch.int64, device=device)
        torch.cumsum(per_row, 0, out=ent_off[1:])
        node = torch.empty(max(P, 1), dtype=torch.int32, device=device)
        count = torch.empty(max(P, 1), dtype=torch.int32, device=device)
        _native.call("rnnl_ground_export_entries", ws.data_ptr(), nq, scale, n_cand.data_ptr(), ent_off.data_ptr(),
                     node.data_ptr(), count.data_ptr(), stream)
        cand_of_entry = torch.repeat_interleave(torch.arange(C, device=device), nent, output_size=P)
        # path counts are u32 in the kernel (< 2^32, carry-checked): reinterpret the int32 bits
        return row, ent, cand_of_entry, node[:P].to(torch.int64), count[:P].to(torch.int64) & 0xFFFFFFFF

    @_native.on_input_device
    def prefetch(self, all_h, all_r, edges_to_remove=None):
        """Ground these rows now, on a side stream, for a forward that will be
        called with the same tensor objects (the training loop's lookahead:
        the grounding does not depend on the weights, so batch k + 1's runs
        while batch k scores, steps back and updates).  Up to prefetch_depth
        groundings are queued, each in its own workspace of a ring; a forward
        whose rows are not the queue's head drops the queue."""
        if self.prefetch_depth <= 0 or not self._prefetch_enabled():
            return
        device, h, r, etr = self._rows(all_h, all_r, edges_to_remove)
        nq = h.numel()
        if nq == 0:
            return
        key = self._device_index(device)
        pf = self._pf.get(key)
        if pf is None:
            pf = self._pf[key] = {"stream": torch.cuda.Stream(device), "ring": {}, "next": 0,
                                  "queue": collections.deque()}
        if len(pf["queue"]) >= self.prefetch_depth:
            return
        g, nr = self.graph.device_graph(device), self.native_rules(device)
        scale = self.capacity_scale
        need = ctypes.c_size_t()
        _native.call("rnnl_forward_workspace_size", g, nr.ptr, nq, scale, ctypes.byref(need))
        # ring of depth + 1 workspaces: the forward in flight keeps one until its backward
        slot = pf["next"] % (self.prefetch_depth + 1)
        pf["next"] += 1
        ws = pf["ring"].get(slot)
        if ws is None or ws.numel() < need.value:
            ws = pf["ring"][slot] = torch.empty(need.value, dtype=torch.uint8, device=device)
        n_cand = torch.empty(nq, dtype=torch.int32, device=device)
        side, main = pf["stream"], torch.cuda.current_stream(device)
        # inputs, and the slot's previous user (its backward is on the current stream already)
        side.wait_stream(main)
        self._prefetch_ground(g, nr, h, r, etr, nq, n_cand, ws, scale, side.cuda_stream)
        # the grounding's status / totals and the one-relation flag, copied to the
        # host behind it: the forward reads them without waiting for the current stream
        # (pinned buffer and event of the ring slot: the slot's previous entry was
        # consumed, or dropped behind the same side stream, before it comes round)
        hdr, ev = self._host_slot(pf, "pf", slot, self.prefetch_depth + 1)
        hb = self._header_bytes()
        with torch.cuda.stream(side):
            hdr[:hb].copy_(ws[:hb], non_blocking=True)  # status, totals and the one-relation flag
            hdr[hb:hb + 8].copy_(r[:1].view(torch.uint8), non_blocking=True)  # the first row's relation
        ev.record(side)
        # the side stream's use of these blocks outlives a dropped queue entry or a
        # grown ring slot: the caching allocator must not hand them out before it ends
        for t in (ws, n_cand, h, r) + ((etr,) if etr is not None else ()):
            t.record_stream(side)
        self._ws_touch(ws)
        pf["queue"].append((all_h, all_r, edges_to_remove, ws, scale, n_cand, ev, (h, r, etr), hdr))

    def _host_slot(self, pf, name, k, n):
        """(pinned header buffer, event) number k % n of a ring kept in pf:
        reused instead of a pinned allocation and an event creation per step."""
        ring = pf.get(name)
        if ring is None or len(ring) != n:
            hb = self._header_bytes() + 8  # + the first row's relation (int64)
            ring = pf[name] = [(torch.empty(hb, dtype=torch.uint8, pin_memory=True), torch.cuda.Event())
                               for _ in range(n)]
        return ring[k % n]

    def _header_bytes(self):
        if getattr(self, "_hdr_bytes", None) is None:
            n = ctypes.c_size_t()
            _native.call("rnnl_forward_header_bytes", ctypes.byref(n))
            self._hdr_bytes = n.value
        return self._hdr_bytes

    def check_deferred(self, keep=0):
        """Raise the scoring pass's own error (an integer range flag) of the
        lookahead forwards, whose status is read late so the host does not
        wait for the scoring: every pending status but the newest `keep`
        (the training step checks the forward before last, which has long
        finished; train() checks them all at its end).  The training steps of
        those forwards have then already run their backward and optimizer
        step on the flagged scores: the error names the forward, and a run
        resumed from a checkpoint written after it should not trust it."""
        q = getattr(self, "_deferred_status", None)
        while q and len(q) > keep:
            dh, ev, n = q.popleft()
            ev.synchronize()
            rc = _native.lib().rnnl_forward_status_host(dh.data_ptr(), None)
            if rc != _native.RNNL_OK:
                q.clear()
                raise _native.NativeError(rc, "%s (scoring pass of lookahead forward #%d, read late: that step's "
                                              "backward and optimizer update have already been applied)" % (
                                                  _native.lib().rnnl_last_error().decode(errors="replace"), n))

    def _prefetched(self, device, all_h, all_r, edges_to_remove, peek=False):
        """The queued grounding of exactly these row tensors, or None.  Entries
        grounded at another capacity_scale (a retry raised it since) and those
        queued before the match (batches that ran without their lookahead) are
        dropped; entries after it are later batches and stay queued.
        peek: leave the match queued."""
        pf = self._pf.get(self._device_index(device))
        if not pf or not pf["queue"]:
            return None
        q = pf["queue"]
        stale = [e for e in q if e[4] != self.capacity_scale]
        if stale:
            self._drop_lookahead(pf, [e for e in q if e[4] == self.capacity_scale], len(stale))
            q = pf["queue"]
        for i, e in enumerate(q):
            if e[0] is all_h and e[1] is all_r and e[2] is edges_to_remove:
                if i:
                    self._drop_lookahead(pf, list(q)[i:], i)
                    q = pf["queue"]
                if peek:
                    return q[0]
                self.prefetch_hits = getattr(self, "prefetch_hits", 0) + 1
                return q.popleft()
        return None  # these rows were not grounded ahead; the queued ones are later batches

    def _drop_lookahead(self, pf, keep, n):
        # the side stream's work on dropped entries still ends before their
        # ring slots come round again (record_stream, the slots' order)
        self.prefetch_dropped += n
        logging.debug(type(self).__name__ + ": %d lookahead groundings dropped (%d so far)", n, self.prefetch_dropped)
        pf["queue"] = collections.deque(keep)

    def _defer_status(self, device, ws):
        """After a scoring pass on a prefetched grounding: its header copied
        behind it into a pinned ring slot, checked two forwards later
        (check_deferred) instead of waiting for the pass now."""
        hb = self._header_bytes()
        main = torch.cuda.current_stream(device)
        self._lookahead_forwards = getattr(self, "_lookahead_forwards", 0) + 1
        dh, dev_ev = self._host_slot(self._pf[self._device_index(device)], "dev", self._lookahead_forwards, 4)
        dh[:hb].copy_(ws[:hb], non_blocking=True)
        dev_ev.record(main)
        if getattr(self, "_deferred_status", None) is None:
            self._deferred_status = collections.deque()
        self._deferred_status.append((dh, dev_ev, self._lookahead_forwards))

    @staticmethod
    def _prefetch_relation(hdr, hb):
        """The first row's relation recorded by prefetch (host read of the
        pinned slot; its event has been waited on)."""
        return int(hdr[hb:hb + 8].view(torch.int64)[0])

    def _reference_nonfinite(self, device, all_r, ridx, rule_vals, row, ce, node, C):
        """Where the reference's dense sums over a relation's rules meet 0 x
        (a non-finite value): it multiplies every rule's path counts, zeros
        included, by the rule's value (Predictor: score += x * w,
        predictors.py:63-64; FuncToNodeSum: (message * weight).sum(1),
        layers.py:70), so a candidate gets NaN in dim d when a rule it is NOT
        reached by has a non-finite value there.  rule_vals: (len(ridx), D).
        Returns (per candidate (C, D), per row (nq, D)) bool: the candidate's
        entry / a non-candidate entity of the row is NaN in the reference."""
        nr = self.native_rules(device)
        bad = (~torch.isfinite(rule_vals.detach())).to(torch.int64)
        D = bad.size(1)
        heads = torch.tensor([h for h, _ in self.rules], dtype=torch.int64, device=device)
        rel_bad = torch.zeros((self.graph.relation_size, D), dtype=torch.int64, device=device).index_add(
            0, heads[ridx], bad)
        node_bad = torch.zeros((max(nr.n_nodes, 1), D), dtype=torch.int64, device=device).index_add(
            0, nr.node_of_rule[ridx], bad)
        key = torch.unique(ce * max(nr.n_nodes, 1) + node)  # distinct (candidate, node) pairs
        reached = torch.zeros((C, D), dtype=torch.int64, device=device).index_add(
            0, key // max(nr.n_nodes, 1), node_bad[key % max(nr.n_nodes, 1)])
        r64 = all_r.to(device, torch.int64)
        return rel_bad[r64[row]] > reached, rel_bad[r64] > 0

    def _needs_grad(self):
        return torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters())


class _RuleGrounder(_HipGrounding):
    """One rule as a one-rule trie under its head relation: the HIP grounding
    behind KnowledgeGraph.grounding (reference data.py:136-147)."""

    def __init__(self, graph, head, body):
        self.graph = graph
        self.rules = [(head, list(body))]
        self._native_rules = {}
        self._ws = {}
        self._ws_uses = {}
        self._flags = np.zeros(1, dtype=np.uint32)
        self.capacity_scale = 1

    @_native.on_input_device
    def counts(self, h, edges_to_remove):
        """(B, |E|) int64 path counts of the rule from each h."""
        device = h.device
        B = h.numel()
        all_r = torch.full((B,), self.rules[0][0], dtype=torch.int64, device=device)
        row, ent, ce, node, count = self.ground_coo(h, all_r, edges_to_remove)
        out = torch.zeros((B, self.graph.entity_size), dtype=torch.int64, device=device)
        # one rule = one trie node, but a hash overflow in the kernel may leave
        # a (candidate, node) pair split over several entries: add them
        return out.index_put_((row[ce], ent[ce]), count, accumulate=True)


class _PredictorLinear(torch.autograd.Function):
    """Predictor.forward under autograd (predictors.py:53-80): the HIP forward
    (rnnl_predictor_forward) and its backward (rnnl_predictor_backward: per
    trie node the sum of count x incoming gradient, shared by the node's
    rules; the bias gradient is the column sum).  The grounding stays in the
    model's workspace between the two; if another launch has reused it by
    the time backward runs, the rows are grounded again (same COO)."""

    @staticmethod
    def forward(ctx, rule_weights, bias, model, all_h, all_r, edges_to_remove):
        score, mask, n_cand, ws, scale, n_total = model._forward_launch(all_h, all_r, edges_to_remove,
                                                                        single_relation=True)
        device = score.device
        ctx.model, ctx.ws, ctx.scale, ctx.n_cand = model, ws, scale, n_cand
        # a batch without any candidate returns `mask + bias` in the reference
        # (predictors.py:67-71): the rule weights are not in its graph, so they
        # get no gradient (None, which Adam skips — a zero gradient would still
        # move them through the moment estimates)
        ctx.no_cand = n_total == 0
        ctx.gen = model._ws_uses.get(ws.data_ptr()) if ws is not None else None
        ctx.rows = model._rows(all_h, all_r, edges_to_remove)[1:]
        ctx.has_bias = bias is not None
        ctx.mark_non_differentiable(mask)
        return score, mask

    @staticmethod
    def backward(ctx, grad_score, grad_mask):
        model = ctx.model
        all_h, all_r, etr = ctx.rows
        device = all_h.device
        nq = all_h.numel()
        gw = gb = None
        if nq and ctx.needs_input_grad[0] and not ctx.no_cand:
            ws, scale, n_cand = ctx.ws, ctx.scale, ctx.n_cand
            if model._ws_uses.get(ws.data_ptr()) != ctx.gen:  # the workspace was reused: ground again
                ws, scale, n_cand = model.ground(all_h, all_r, etr)
            nr = model.native_rules(device)
            _, ld = model.head_roots(device)
            g = grad_score.contiguous().float()
            grad_node = torch.zeros(max(nr.n_nodes, 1), dtype=torch.float64, device=device)
            _native.call("rnnl_predictor_backward", ws.data_ptr(), nq, scale, n_cand.data_ptr(), nr.ptr,
                         all_r.data_ptr(), model.num_entities, g.data_ptr(), ld, grad_node.data_ptr(),
                         torch.cuda.current_stream(device).cuda_stream)
            gw = grad_node.index_select(0, nr.node_of_rule).to(model.rule_weights.dtype)
        if ctx.has_bias and ctx.needs_input_grad[1]:
            gb = grad_score.sum(0)
        return gw, gb, None, None, None, None


class Predictor(_HipGrounding, torch.nn.Module):
    """Rule-weight predictor of the EM loop (reference src/predictors.py:17-119).

    score = sum over the relation's rules of path count x rule weight
    (+ bias).  Eval forwards run the HIP grounding and an exact fixed-point
    per-candidate sum (rnnl_predictor_forward); compute_H reads per-node path
    statistics from the same grounding (rnnl_predictor_rule_stats); training
    forwards are torch autograd on the grounding COO.  No CPU fallback."""

    def __init__(self, graph, entity_feature="bias"):
        super(Predictor, self).__init__()
        self.graph = graph
        self.num_entities = graph.entity_size
        self.num_relations = graph.relation_size
        self.entity_feature = entity_feature
        if entity_feature == "bias":
            self.bias = torch.nn.parameter.Parameter(torch.zeros(self.num_entities))
        self._native_rules = {}
        self._ws = {}
        self._lin_cache = {}
        self._roots = {}
        self._ws_uses = {}  # per workspace pointer: launches onto it so far
        self._flags = np.zeros(1, dtype=np.uint32)  # the last launch's header flags (_status)
        self._pf = {}  # per device: training lookahead (prefetch): side stream, workspace ring, queue
        # groundings launched ahead of the training step that needs them
        # (TrainerPredictor.train; 0 turns the lookahead off)
        self.prefetch_depth = 2
        self.prefetch_dropped = 0  # queued groundings discarded (rows not the queue's head)
        self.capacity_scale = 1

    def set_rules(self, input):
        self.rules = _read_rules(input)
        logging.info("Predictor: read {} rules from {}.".format(len(self.rules),
                                                               "list" if isinstance(input, list) else "file"))
        self.num_rules = len(self.rules)
        self.relation2rules = [[] for _ in range(self.num_relations)]
        for index, rule in enumerate(self.rules):
            self.relation2rules[rule[0]].append([index, rule])
        self.rule_weights = torch.nn.parameter.Parameter(torch.zeros(self.num_rules))
        self._native_rules = {}
        self._lin_cache = {}
        self._roots = {}
        self._pf = {}  # queued lookahead groundings belong to the old rules

    # ------------------------------------------------------------------ native plumbing
    def node_weights(self, device):
        """Per-trie-node sums of the rule weights (HIP, int32 fixed point),
        cached until rule_weights changes."""
        nr = self.native_rules(device)
        key = (self._device_index(device), self.rule_weights.data_ptr(), self.rule_weights._version)
        hit = self._lin_cache.get(device)
        if hit is not None and hit[0] == key:
            return hit[1]
        w = self.rule_weights.detach().float().contiguous()
        nbytes = ctypes.c_size_t()
        _native.call("rnnl_linear_node_weights_size", nr.ptr, ctypes.byref(nbytes))
        out = torch.empty(nbytes.value, dtype=torch.uint8, device=device)
        _native.call("rnnl_linear_node_weights", nr.ptr, w.data_ptr(), self.num_rules, out.data_ptr(),
                     torch.cuda.current_stream(device).cuda_stream)
        self._lin_cache[device] = (key, out, w)
        return out

    def head_roots(self, device):
        key = self._device_index(device)
        if key not in self._roots:
            nr = self.native_rules(device)
            roots = (ctypes.c_int32 * max(self.num_relations, 1))()
            mh = ctypes.c_int32()
            _native.call("rnnl_rules_head_roots", nr.ptr, roots, ctypes.byref(mh))
            self._roots[key] = (list(roots)[:self.num_relations], max(int(mh.value), 1))
        return self._roots[key]

    @_native.on_input_device
    def forward_rows(self, all_h, all_r, edges_to_remove=None, return_ncand=False):
        """Forward for any rows (one or many reference batches, mixed
        relations): (score (n, |E|) f32, mask (n, |E|) bool[, n_cand])."""
        try:
            score, mask, n_cand, _, _, _ = self._forward_launch(all_h, all_r, edges_to_remove)
        except _native.NativeError as e:
            if e.code != _native.RNNL_ERR_RANGE:
                raise
            score, mask, n_cand = self._forward_range_fallback(all_h, all_r, edges_to_remove)
        return (score, mask, n_cand) if return_ncand else (score, mask)

    def _forward_range_fallback(self, all_h, all_r, edges_to_remove):
        """Past the fixed-point kernels' integer ranges (a path count reaching
        2^32, non-finite or huge rule weights): the reference's arithmetic on
        the grounding COO with int64 counts (forward_autograd's torch ops)."""
        logging.info("Predictor: %s; rows recomputed on the grounding COO (int64 counts, torch ops)",
                     _native.lib().rnnl_last_error().decode(errors="replace"))
        with torch.no_grad():
            score, mask = self.forward_autograd(all_h, all_r, edges_to_remove, nonfinite=True)
            row = self.ground_coo(all_h, all_r, edges_to_remove)[0]
            n_cand = torch.bincount(row, minlength=all_h.numel()).to(torch.int32)
        return score, mask, n_cand

    def _prefetch_enabled(self):
        return True

    def _prefetch_ground(self, g, nr, h, r, etr, nq, n_cand, ws, scale, stream):
        _native.call("rnnl_predictor_ground", g, nr.ptr, h.data_ptr(), r.data_ptr(),
                     etr.data_ptr() if etr is not None else None, nq, n_cand.data_ptr(), ws.data_ptr(), ws.numel(),
                     scale, stream)

    def _forward_launch(self, all_h, all_r, edges_to_remove, single_relation=False):
        """rnnl_predictor_forward over the rows -> (score, mask, n_cand, ws,
        scale, candidate total); the workspace keeps the grounding for a
        backward.  With
        `single_relation` the reference's one-relation-per-batch check
        (predictors.py:54-55) is read back with the launch status (no extra
        host sync)."""
        raw = (all_h, all_r, edges_to_remove)
        device, all_h, all_r, etr = self._rows(all_h, all_r, edges_to_remove)
        nq, E = all_h.numel(), self.num_entities
        if nq == 0:  # no rows: empty outputs, no launch
            return (torch.empty((0, E), dtype=torch.float32, device=device),
                    torch.empty((0, E), dtype=torch.bool, device=device),
                    torch.empty(0, dtype=torch.int32, device=device), None, None, 0)
        self.check_deferred(keep=1)
        pre = self._prefetched(device, *raw)
        g, nr = self.graph.device_graph(device), self.native_rules(device)
        node_w = self.node_weights(device)
        stream = torch.cuda.current_stream(device).cuda_stream
        bias_mode = self.entity_feature == "bias"
        feature = _native.FEATURE_ADD if bias_mode else _native.FEATURE_NONE
        score = torch.empty((nq, E), dtype=torch.float32, device=device)
        n_cand = torch.empty(nq, dtype=torch.int32, device=device)
        mask8 = None if bias_mode else torch.empty((nq, E), dtype=torch.uint8, device=device)
        bias = self.bias.detach().float().contiguous() if bias_mode else None

        def fill():
            if bias_mode:
                _native.call("rnnl_fill_rows", bias.data_ptr(), nq, E, score.data_ptr(), stream)
            else:
                _native.call("rnnl_fill_value", float("-inf"), score.numel(), score.data_ptr(), stream)
                mask8.zero_()

        def run(ws, scale):
            fill()
            _native.call("rnnl_predictor_forward", g, nr.ptr, node_w.data_ptr(), feature, all_h.data_ptr(),
                         all_r.data_ptr(), etr.data_ptr() if etr is not None else None, nq, score.data_ptr(),
                         mask8.data_ptr() if mask8 is not None else None, n_cand.data_ptr(), ws.data_ptr(),
                         ws.numel(), scale, stream)
        totals = np.zeros(2, dtype=np.int64)  # (candidates, bucket entries), read with the status
        if pre is not None:  # grounded ahead (prefetch): the scoring half only
            _, _, _, ws, scale, n_cand_pf, ev, _, hdr = pre
            ev.synchronize()  # that grounding and its header copy, not the later side-stream work
            rc = _native.lib().rnnl_forward_status_host(hdr.data_ptr(), totals.ctypes.data_as(ctypes.c_void_p))
            _native.call("rnnl_forward_flags_host", hdr.data_ptr(), self._flags.ctypes.data_as(ctypes.c_void_p))
            if single_relation:
                self._check_one_relation()
            if rc == _native.RNNL_OK:
                fill()
                main = torch.cuda.current_stream(device)
                main.wait_event(ev)
                _native.call("rnnl_predictor_score", g, nr.ptr, node_w.data_ptr(), feature, all_h.data_ptr(),
                             all_r.data_ptr(), nq, score.data_ptr(), mask8.data_ptr() if mask8 is not None else None,
                             n_cand_pf.data_ptr(), ws.data_ptr(), ws.numel(), scale, stream)
                # the scoring pass's range flag: copied behind it, read two forwards
                # later (a ring of 4 pinned buffers / events: at most 2 are pending)
                self._defer_status(device, ws)
                n_cand = n_cand_pf
            else:  # overflow (or another failure): the one-call path, with its retry
                pre = None
        if pre is None:
            ws, scale = self._launch(device, nq, run, totals)
            if single_relation:
                self._check_one_relation()
        mask = torch.ones((nq, E), dtype=torch.bool, device=device) if bias_mode else mask8.bool()
        return score, mask, n_cand, ws, scale, int(totals[0])

    # ------------------------------------------------------------------ reference API
    # every entity is scored (the reference's mask is all True) with the bias feature
    @property
    def mask_all_true(self):
        return self.entity_feature == "bias"

    @_native.on_input_device
    def forward(self, all_h, all_r, edges_to_remove):
        """predictors.py:53-80: one single-relation batch -> (score, mask).
        With autograd (training) the same HIP forward runs inside
        _PredictorLinear, whose backward is rnnl_predictor_backward."""
        try:
            if self._needs_grad():
                bias = self.bias if self.entity_feature == "bias" else None
                score, mask = _PredictorLinear.apply(self.rule_weights, bias, self, all_h, all_r, edges_to_remove)
            else:
                score, mask, _, _, _, _ = self._forward_launch(all_h, all_r, edges_to_remove, single_relation=True)
        except _native.NativeError as e:
            if e.code != _native.RNNL_ERR_RANGE:
                raise
            # past the kernels' integer ranges: torch ops on the int64 grounding COO
            logging.info("Predictor: %s; batch recomputed on the grounding COO",
                         _native.lib().rnnl_last_error().decode(errors="replace"))
            score, mask = self.forward_autograd(all_h, all_r, edges_to_remove, nonfinite=True)
        if self.entity_feature != "bias":
            # early return `mask - float('-inf')` (predictors.py:68-72): +inf where the
            # batch has no candidate at all (mask all False), without a host read
            score = torch.where(mask.any(), score, torch.full_like(score, float("inf")))
        return score, mask

    @_native.on_input_device
    def forward_autograd(self, all_h, all_r, edges_to_remove, nonfinite=False):
        """Differentiable forward (training): the HIP grounding's COO, then
        score = scatter of sum(count x node weight) with node weight = the sum
        of its rules' rule_weights — torch autograd yields the reference's
        gradients (predictors.py:53-80).  nonfinite: reproduce the reference's
        0 x (non-finite weight) NaNs (the range fallback)."""
        device = all_h.device
        nq, E = all_h.numel(), self.num_entities
        row, ent, ce, node, count = self.ground_coo(all_h, all_r, edges_to_remove)
        C = ent.numel()
        if C == 0:
            zero = torch.zeros((nq, E), device=device)
            if self.entity_feature == "bias":
                return zero + self.bias.unsqueeze(0), torch.ones((nq, E), dtype=torch.bool, device=device)
            return zero - float("-inf"), torch.zeros((nq, E), dtype=torch.bool, device=device)
        nr = self.native_rules(device)
        w = self.rule_weights
        node_w = torch.zeros(nr.n_nodes, device=device, dtype=w.dtype).index_add(0, nr.node_of_rule, w)
        val = torch.zeros(C, device=device, dtype=w.dtype).index_add(0, ce, count.to(w.dtype) * node_w.index_select(0, node))
        score = torch.zeros(nq * E, device=device, dtype=w.dtype)
        if nonfinite:
            rels = torch.unique(all_r).tolist()
            ridx = torch.tensor([i for q in rels for i, _ in self.relation2rules[q]], dtype=torch.long, device=device)
            cand_nan, row_nan = self._reference_nonfinite(device, all_r, ridx, w.detach()[ridx].unsqueeze(1), row, ce,
                                                          node, C)
            val = torch.where(cand_nan[:, 0], torch.full_like(val, float("nan")), val)
            score = torch.where(row_nan[:, 0].repeat_interleave(E), torch.full_like(score, float("nan")), score)
        score = score.scatter(0, row * E + ent, val).view(nq, E)
        if self.entity_feature == "bias":
            return score + self.bias.unsqueeze(0), torch.ones((nq, E), dtype=torch.bool, device=device)
        mask = torch.zeros(nq * E, dtype=torch.bool, device=device).index_fill(0, row * E + ent, True).view(nq, E)
        return score.masked_fill(~mask, float("-inf")), mask

    @torch.no_grad()
    @_native.on_input_device
    def compute_H(self, all_h, all_r, all_t, edges_to_remove):
        """Per-rule H scores (predictors.py:82-119): per row, pos = w x count at
        the true tail, neg = w x (sum of counts over candidates) / #candidates;
        softmax over the relation's rules, summed over rows.  Grounding and
        the per-node path statistics run on the HIP path."""
        query_r = all_r[0].item()
        assert (all_r != query_r).sum() == 0
        device = all_h.device
        rules = self.relation2rules[query_r]
        if len(rules) == 0:
            return None, None
        nq = all_h.numel()
        nr = self.native_rules(device)
        roots, ld = self.head_roots(device)
        pos, tot, n_cand = self._rule_stats(all_h, all_r, all_t, edges_to_remove, ld)
        rule_index = torch.tensor([i for i, _ in rules], dtype=torch.long, device=device)
        k = nr.node_of_rule[rule_index] - roots[query_r]
        w = self.rule_weights.detach()[rule_index]
        pos_score = pos[:, k].to(w.dtype) * w
        neg_score = tot[:, k].to(w.dtype) * w / torch.clamp(n_cand.to(w.dtype), min=1).unsqueeze(1)
        return torch.softmax(pos_score - neg_score, dim=-1).sum(0), rule_index

    def _rule_stats(self, all_h, all_r, all_t, edges_to_remove, ld):
        """Per row and trie node of the row's head (local index < ld): the
        path count to the true tail (pos) and the total over the candidates
        (tot), int64, and the rows' candidate counts — rnnl_predictor_rule_stats
        on the grounding, or, for rows whose counts reach 2^32 (the grounding
        kernel's u32 sums), the same sums on the int64 grounding COO
        (rnnl_ground_wide; the reference counts in int64, data.py:139-171)."""
        device = all_h.device
        nq = all_h.numel()
        r64 = all_r.to(device, torch.int64).contiguous()
        t64 = all_t.to(device, torch.int64).contiguous()
        nr = self.native_rules(device)
        pos = torch.zeros((nq, ld), dtype=torch.int64, device=device)
        tot = torch.zeros((nq, ld), dtype=torch.int64, device=device)
        try:
            ws, scale, n_cand = self.ground(all_h, all_r, edges_to_remove)
        except _native.NativeError as e:
            if e.code != _native.RNNL_ERR_RANGE:
                raise
            row, ent, ce, node, count = self.ground_coo(all_h, all_r, edges_to_remove)
            roots = torch.tensor(self.head_roots(device)[0], dtype=torch.int64, device=device)
            rr = row[ce]
            flat = rr * ld + (node - roots[r64[rr]])
            tot.view(-1).index_add_(0, flat, count)
            pos.view(-1).index_add_(0, flat, count * (ent[ce] == t64[rr]).to(torch.int64))
            return pos, tot, torch.bincount(row, minlength=nq).to(torch.int32)
        _native.call("rnnl_predictor_rule_stats", ws.data_ptr(), nq, scale, n_cand.data_ptr(), nr.ptr,
                     r64.data_ptr(), t64.data_ptr(), ld, pos.data_ptr(), tot.data_ptr(),
                     torch.cuda.current_stream(device).cuda_stream)
        return pos, tot, n_cand

    def _rule_table(self, device):
        """Per relation its rules padded to the longest list: (R, Rmax) rule ids
        (-1 pad) and the rules' trie-node index local to the head's root."""
        key = ("rule_table", self._device_index(device))
        hit = self._lin_cache.get(key)
        if hit is not None:
            return hit
        nr = self.native_rules(device)
        roots, ld = self.head_roots(device)
        R = self.num_relations
        rmax = max([len(self.relation2rules[q]) for q in range(R)] + [1])
        idx = np.full((R, rmax), -1, dtype=np.int64)
        for q in range(R):
            ids = [i for i, _ in self.relation2rules[q]]
            idx[q, :len(ids)] = ids
        idx = torch.from_numpy(idx).to(device)
        root = torch.tensor(roots, dtype=torch.int64, device=device).clamp(min=0).unsqueeze(1)
        node = nr.node_of_rule.to(device, torch.int64)[idx.clamp(min=0)] - root
        out = (idx, node.clamp(min=0, max=ld - 1), ld)
        self._lin_cache[key] = out
        return out

    @torch.no_grad()
    @_native.on_input_device
    def compute_H_rows(self, all_h, all_r, all_t, edges_to_remove, chunk=8192):
        """Σ over rows of compute_H's per-row softmax (predictors.py:82-119),
        for rows of any relations in a few launches: the per-row terms are
        independent, so the sum over the reference's batches equals the sum
        over all their rows.  Returns (num_rules,) (rules of relations that
        have none get 0).  `chunk` rows per launch bound the grounding
        workspace (8,192 rows: ~1.9 GB at capacity_scale 1; the result does
        not depend on it)."""
        device = all_h.device
        n = all_h.numel()
        H = torch.zeros(self.num_rules, device=device)
        if n == 0 or self.num_rules == 0:
            return H
        idx, node, ld = self._rule_table(device)
        nr = self.native_rules(device)
        w_all = self.rule_weights.detach()
        for s0 in range(0, n, chunk):
            h, r, t = all_h[s0:s0 + chunk], all_r[s0:s0 + chunk], all_t[s0:s0 + chunk]
            e = edges_to_remove[s0:s0 + chunk] if edges_to_remove is not None else None
            pos, tot, n_cand = self._rule_stats(h, r, t, e, ld)
            r = r.to(device, torch.int64).contiguous()
            ridx, k = idx[r], node[r]  # (m, Rmax)
            valid = ridx >= 0
            w = w_all[ridx.clamp(min=0)]
            pos_score = pos.gather(1, k).to(w.dtype) * w
            neg_score = tot.gather(1, k).to(w.dtype) * w / torch.clamp(n_cand.to(w.dtype), min=1).unsqueeze(1)
            sm = torch.softmax((pos_score - neg_score).masked_fill(~valid, float("-inf")), dim=-1)
            has = valid.any(1, keepdim=True)
            sm = torch.where(valid & has, sm, torch.zeros_like(sm))
            H.index_add_(0, ridx.clamp(min=0).reshape(-1), sm.reshape(-1))
        return H


class _PlusSumTrain(torch.autograd.Function):
    """PredictorPlus.forward under autograd for the SUM aggregator (hidden 16):
    the fused HIP forward (rnnl_predictorplus_forward with the batch's edge
    removal) and the fused backward K2^T (rnnl_predictorplus_backward,
    csrc/backward.hip) instead of torch autograd over the grounding COO —
    reference src/predictors.py:238-271, src/layers.py:9-77 as differentiated
    in src/trainer.py:84-93.

    Inputs: the rule-embedding table `emb` (num_rules x 16: rule_emb, or the
    batch relation's LSTM outputs scattered into a zero table), the rule part's
    weights, and the entity feature: `base` = the bias vector (kind 'bias'),
    the RotatE rows (kind 'rows', whose gradient is grad_score itself) or None
    (kind 'none': -inf outside the candidates, mask from the kernel).  A
    batch without any candidate takes the reference's early return
    (predictors.py:230-237): the rule part is not in the graph, so its
    parameters get no gradient (None, which Adam skips)."""

    @staticmethod
    def forward(ctx, model, raw, all_h, all_r, etr, head, kind, base, emb, add_w, add_b, ln_w, ln_b, s0_w, s0_b,
                s1_w, s1_b, rel_w):
        device = all_h.device
        nq, E = all_h.numel(), model.num_entities
        g, nr = model.graph.device_graph(device), model.native_rules(device)
        emb_d = emb.detach().float().contiguous()
        ws_ = [t.detach().float().contiguous() for t in (add_w, add_b, ln_w, ln_b, s0_w, s0_b, s1_w, s1_b, rel_w)]
        nbytes = ctypes.c_size_t()
        _native.call("rnnl_node_weights_size", nr.ptr, _native.AGG_SUM, ctypes.byref(nbytes))
        node_w = torch.empty(nbytes.value, dtype=torch.uint8, device=device)
        stream = torch.cuda.current_stream(device).cuda_stream
        if head >= 0:  # a one-relation batch reads that head's trie only
            _native.call("rnnl_node_weights_head", nr.ptr, head, emb_d.data_ptr(), 16, _native.AGG_SUM,
                         ws_[0].data_ptr(), node_w.data_ptr(), stream)
        else:
            _native.call("rnnl_node_weights", nr.ptr, emb_d.data_ptr(), 16, _native.AGG_SUM, ws_[0].data_ptr(),
                         node_w.data_ptr(), stream)
        p = _native.PredictorParams()
        p.aggregator = _native.AGG_SUM
        p.feature = _native.FEATURE_NONE if kind == "none" else _native.FEATURE_ADD
        p.node_w = node_w.data_ptr()
        (p.add_w, p.add_b, p.ln_w, p.ln_b, p.s0_w, p.s0_b, p.s1_w, p.s1_b, p.rel_emb) = [t.data_ptr() for t in ws_]
        bias = base.detach().float().contiguous() if kind == "bias" else None
        if bias is not None:
            p.base_row = bias.data_ptr()
        mask8 = None
        totals = np.zeros(2, dtype=np.int64)

        def run(ws, scale):
            if kind == "bias":
                _native.call("rnnl_fill_rows", bias.data_ptr(), nq, E, score.data_ptr(), stream)
            elif kind == "rows":
                score.copy_(base.detach())
            else:
                _native.call("rnnl_fill_value", float("-inf"), score.numel(), score.data_ptr(), stream)
                mask8.zero_()
            _native.call("rnnl_predictorplus_forward", g, nr.ptr, ctypes.byref(p), all_h.data_ptr(),
                         all_r.data_ptr(), etr.data_ptr() if etr is not None else None, nq, score.data_ptr(),
                         mask8.data_ptr() if mask8 is not None else None, n_cand.data_ptr(), None, ws.data_ptr(),
                         ws.numel(), scale, stream)
        score = torch.empty((nq, E), dtype=torch.float32, device=device)
        n_cand = torch.empty(nq, dtype=torch.int32, device=device)
        if kind == "none":
            mask8 = torch.empty((nq, E), dtype=torch.uint8, device=device)
        model.check_deferred(keep=1)
        pre = model._prefetched(device, *raw) if raw is not None else None
        if pre is not None:
            # the node records' range flag (trailer word 2: a non-finite or
            # >= 2^30 aggregate), copied behind rnnl_node_weights*: checked
            # below before the lookahead's scores are used, so that such a
            # batch takes the one-call path and its RNNL_ERR_RANGE fallback
            # (the exact COO path) exactly as without the lookahead
            nflag, nflag_ev = model._node_flag_slot(device)
            nflag.copy_(node_w[nbytes.value - 64 + 8:nbytes.value - 64 + 12], non_blocking=True)
            nflag_ev.record()
        if pre is not None:  # grounded ahead (prefetch): the scoring half only
            _, _, _, ws, scale, n_cand_pf, ev, _, hdr = pre
            ev.synchronize()  # that grounding and its header copy, not the later side-stream work
            rc = _native.lib().rnnl_forward_status_host(hdr.data_ptr(), totals.ctypes.data_as(ctypes.c_void_p))
            if rc == _native.RNNL_OK:
                if kind == "bias":
                    _native.call("rnnl_fill_rows", bias.data_ptr(), nq, E, score.data_ptr(), stream)
                elif kind == "rows":
                    score.copy_(base.detach())
                else:
                    _native.call("rnnl_fill_value", float("-inf"), score.numel(), score.data_ptr(), stream)
                    mask8.zero_()
                torch.cuda.current_stream(device).wait_event(ev)
                _native.call("rnnl_predictorplus_score", g, nr.ptr, ctypes.byref(p), all_h.data_ptr(),
                             all_r.data_ptr(), nq, score.data_ptr(), mask8.data_ptr() if mask8 is not None else None,
                             n_cand_pf.data_ptr(), None, ws.data_ptr(), ws.numel(), scale, 0, 0, stream)
                nflag_ev.synchronize()  # (the node records only: the scoring pass runs on)
                if int(nflag.view(torch.int32)[0]) == 0:
                    # the scoring pass's remaining range flag (a candidate's
                    # counts past the exact int64 sums), read two forwards later
                    model._defer_status(device, ws)
                    n_cand = n_cand_pf
                else:  # out of the records' range: the one-call path raises RNNL_ERR_RANGE
                    pre = None
            else:  # overflow (or another failure): the one-call path, with its retry
                pre = None
        if pre is None:
            ws, scale = model._launch(device, nq, run, totals)
        ctx.no_cand = int(totals[0]) == 0
        ctx.n_total = int(totals[0])
        if ctx.no_cand and kind == "none":
            # the reference's early return `mask - float('-inf')` (predictors.py:236-237): +inf, mask False
            score.fill_(float("inf"))
        mask = mask8.bool() if mask8 is not None else torch.ones((nq, E), dtype=torch.bool, device=device)
        ctx.model, ctx.kind, ctx.head = model, kind, head
        ctx.launch = (ws, scale, n_cand, model._ws_uses.get(ws.data_ptr()), node_w, p, emb_d, ws_, bias)
        ctx.rows = (all_h, all_r, etr)
        ctx.mark_non_differentiable(mask)
        return score, mask

    @staticmethod
    def backward(ctx, grad_score, grad_mask):
        model, kind = ctx.model, ctx.kind
        ws, scale, n_cand, gen, node_w, p, emb_d, ws_, bias = ctx.launch
        all_h, all_r, etr = ctx.rows
        device = all_h.device
        nq, E = all_h.numel(), model.num_entities
        g_base = None
        if kind == "bias" and ctx.needs_input_grad[7]:
            g_base = grad_score.sum(0)
        elif kind == "rows" and ctx.needs_input_grad[7]:
            g_base = grad_score
        if ctx.no_cand or nq == 0:
            return (None,) * 7 + (g_base,) + (None,) * 10
        g, nr = model.graph.device_graph(device), model.native_rules(device)
        stream = torch.cuda.current_stream(device).cuda_stream
        if model._ws_uses.get(ws.data_ptr()) != gen:
            # another launch reused the workspace since the forward: the same
            # rows grounded and scored again rebuild the COO and chunk list
            scratch = torch.empty((nq, E), dtype=torch.float32, device=device)
            _native.call("rnnl_fill_value", 0.0, scratch.numel(), scratch.data_ptr(), stream)
            p2 = _native.PredictorParams.from_buffer_copy(p)
            p2.feature, p2.base_row = _native.FEATURE_ADD, None

            def run(ws2, scale2):
                _native.call("rnnl_predictorplus_forward", g, nr.ptr, ctypes.byref(p2), all_h.data_ptr(),
                             all_r.data_ptr(), etr.data_ptr() if etr is not None else None, nq, scratch.data_ptr(),
                             None, n_cand.data_ptr(), None, ws2.data_ptr(), ws2.numel(), scale2, stream)
            ws, scale = model._launch(device, nq, run)
        gs = grad_score.float().contiguous()
        sb = model._backward_scratch(device)
        nrb = ctypes.c_size_t()
        _native.call("rnnl_predictorplus_backward_rows_size", nq, ctx.n_total, ctypes.byref(nrb))
        rows_sb = torch.empty(max(nrb.value, 4), dtype=torch.uint8, device=device)
        outs = [torch.empty_like(emb_d)] + [torch.empty_like(t) for t in ws_]
        gr = _native.SumGrads()
        gr.emb, gr.emb_ld = outs[0].data_ptr(), 16
        (gr.add_w, gr.add_b, gr.ln_w, gr.ln_b, gr.s0_w, gr.s0_b, gr.s1_w, gr.s1_b, gr.rel_emb) = \
            [t.data_ptr() for t in outs[1:]]
        _native.call("rnnl_predictorplus_backward", g, nr.ptr, ctypes.byref(p), emb_d.data_ptr(), 16,
                     all_r.data_ptr(), nq, gs.data_ptr(), n_cand.data_ptr(), ctx.n_total, ws.data_ptr(), ws.numel(),
                     scale, ctx.head, sb.data_ptr(), sb.numel(), rows_sb.data_ptr(), rows_sb.numel(),
                     ctypes.byref(gr), stream)
        grads = [o if ctx.needs_input_grad[8 + k] else None for k, o in enumerate(outs)]
        return (None,) * 7 + (g_base,) + tuple(grads)


class _PnaStats(torch.autograd.Function):
    """FuncToNode's sufficient statistics (layers.py:89-101) on the HIP
    grounding, under autograd: per candidate (row-major order) the
    count-weighted sums of x and x^2, the min / max of x over the rules
    reaching it, and (not differentiable) its degree, row and entity —
    rnnl_pna_features after rnnl_node_weights(PNA) of the embedding table
    `emb` (num_rules x 16) and rnnl_ground.  Backward:
    rnnl_pna_features_backward (per node count x gradient sums; a
    candidate's min / max gradient to one tied node, as the reference's
    .min(1) / .max(1) route it to one index; int64 fixed point, independent of
    the order of the adds and of how a (node, candidate) pair is split over
    bucket entries: run-to-run bitwise).  The grounding stays in the model's workspace between the two;
    if another launch has reused it by then, the rows are grounded again."""

    @staticmethod
    def forward(ctx, model, emb, all_h, all_r, etr, head):
        device = all_h.device
        nq = all_h.numel()
        nr = model.native_rules(device)
        emb_d = emb.detach().float().contiguous()
        nbytes = ctypes.c_size_t()
        _native.call("rnnl_node_weights_size", nr.ptr, _native.AGG_PNA, ctypes.byref(nbytes))
        node_w = torch.empty(nbytes.value, dtype=torch.uint8, device=device)
        stream = torch.cuda.current_stream(device).cuda_stream
        if head >= 0:  # a one-relation batch: that head's trie only
            _native.call("rnnl_node_weights_head", nr.ptr, head, emb_d.data_ptr(), 16, _native.AGG_PNA, None,
                         node_w.data_ptr(), stream)
        else:
            _native.call("rnnl_node_weights", nr.ptr, emb_d.data_ptr(), 16, _native.AGG_PNA, None, node_w.data_ptr(),
                         stream)
        totals = np.zeros(2, dtype=np.int64)
        ws, scale, n_cand = model.ground(all_h, all_r, etr, totals)
        C = int(totals[0])
        cand_off = torch.zeros(nq + 1, dtype=torch.int64, device=device)
        torch.cumsum(n_cand.to(torch.int64), 0, out=cand_off[1:])
        f32 = dict(dtype=torch.float32, device=device)
        wsum, wsq, mn, mx = [torch.empty((C, 16), **f32) for _ in range(4)]
        deg = torch.empty(C, **f32)
        row = torch.empty(C, dtype=torch.int64, device=device)
        ent = torch.empty(C, dtype=torch.int64, device=device)
        row_scale = torch.zeros(nq, **f32)
        if C:
            lsum = torch.empty(nq, dtype=torch.int64, device=device)
            _native.call("rnnl_pna_features", nr.ptr, node_w.data_ptr(), ws.data_ptr(), nq, scale, n_cand.data_ptr(),
                         cand_off.data_ptr(), C, wsum.data_ptr(), wsq.data_ptr(), mn.data_ptr(), mx.data_ptr(),
                         deg.data_ptr(), row.data_ptr(), ent.data_ptr(), row_scale.data_ptr(), lsum.data_ptr(), stream)
            # the records' / sums' range bits: RNNL_ERR_RANGE -> the caller's COO path
            _native.check(_native.lib().rnnl_forward_status(ws.data_ptr(), stream))
        ctx.model, ctx.head, ctx.C = model, head, C
        ctx.launch = (ws, scale, n_cand, cand_off, model._ws_uses.get(ws.data_ptr()), node_w, emb_d)
        ctx.rows = (all_h, all_r, etr)
        ctx.save_for_backward(mn, mx)
        ctx.mark_non_differentiable(deg, row, ent, row_scale)
        return wsum, wsq, mn, mx, deg, row, ent, row_scale

    @staticmethod
    def backward(ctx, g_wsum, g_wsq, g_mn, g_mx, *_):  # (deg, row, ent, row_scale: no gradient)
        if ctx.C == 0 or not ctx.needs_input_grad[1]:
            return (None,) * 6
        model = ctx.model
        mn, mx = ctx.saved_tensors
        ws, scale, n_cand, cand_off, gen, node_w, emb_d = ctx.launch
        all_h, all_r, etr = ctx.rows
        device = all_h.device
        if model._ws_uses.get(ws.data_ptr()) != gen:  # the workspace was reused: ground again (same COO)
            ws, scale, n_cand = model.ground(all_h, all_r, etr)
        grads = [g.float().contiguous() if g is not None else torch.zeros_like(mn) for g in (g_wsum, g_wsq, g_mn, g_mx)]
        nr = model.native_rules(device)
        d_x = torch.empty((model.num_rules, 16), dtype=torch.float32, device=device)
        sb = model._pna_scratch(device)
        _native.call("rnnl_pna_features_backward", nr.ptr, node_w.data_ptr(), emb_d.data_ptr(), 16, ws.data_ptr(),
                     all_h.numel(), scale, all_r.data_ptr(), n_cand.data_ptr(), cand_off.data_ptr(), ctx.C, mn.data_ptr(),
                     mx.data_ptr(), *[g.data_ptr() for g in grads], ctx.head, sb.data_ptr(), sb.numel(),
                     d_x.data_ptr(), torch.cuda.current_stream(device).cuda_stream)
        return None, d_x, None, None, None, None


class _LstmRules(torch.autograd.Function):
    """PredictorPlus.encode_rules (predictors.py:201-208) for type 'lstm' under
    autograd: the top layer's output at each rule's last token for the rules
    ridx, by rnnl_lstm_train_forward (the inference encoder's recurrence, each
    step's gates and states saved), and its backward through time by
    rnnl_lstm_train_backward — the gate-gradient and layer-input rows, then
    dW = da^T [x | h_prev] and db = sum(da) in a fixed order by
    rnnl_lstm_weight_grads (a library GEMM over K = n T may split K with
    atomics, which made training not bitwise repeatable), and the vocab
    rows' gradient summed per token in position order.  Replaces the library
    LSTM's per-layer / per-step kernels and its host work (~1.6 ms per step)."""

    @staticmethod
    def forward(ctx, module, ridx, tok, csr, vocab_w, *params):
        L, T, n = module.num_layers, tok.size(1), ridx.numel()
        dev = ridx.device
        sizes = [ctypes.c_size_t() for _ in range(4)]
        _native.call("rnnl_lstm_train_sizes", L, 16, T, n, *[ctypes.byref(x) for x in sizes])
        act = torch.empty(sizes[0].value, dtype=torch.float32, device=dev)
        out = torch.empty((n, 16), dtype=torch.float32, device=dev)
        vocab = vocab_w.detach().float().contiguous()
        ps = [p.detach().float().contiguous() for p in params]
        arrs = _LstmRules._ptrs(ps, L)
        ridx = ridx.contiguous()
        _native.call("rnnl_lstm_train_forward", vocab.data_ptr(), *arrs, L, 16, tok.data_ptr(), T, module.padding_index,
                     ridx.data_ptr(), n, out.data_ptr(), act.data_ptr(), torch.cuda.current_stream(dev).cuda_stream)
        ctx.module, ctx.csr, ctx.tok, ctx.sizes = module, csr, tok, [x.value for x in sizes]
        ctx.save_for_backward(ridx, act, vocab, *ps)
        return out

    @staticmethod
    def _ptrs(ps, L):
        arr = lambda k: (ctypes.c_void_p * 3)(*[ps[4 * l + k].data_ptr() for l in range(L)])  # noqa: E731
        return [arr(0), arr(1), arr(2), arr(3)]

    @staticmethod
    def backward(ctx, d_out):
        ridx, act, vocab, *ps = ctx.saved_tensors
        m = ctx.module
        L, T, n = m.num_layers, ctx.tok.size(1), ridx.numel()
        dev = d_out.device
        _, n_da, n_xh, n_dvx = ctx.sizes
        da = torch.empty(n_da, dtype=torch.float32, device=dev)
        xh = torch.empty(n_xh, dtype=torch.float32, device=dev)
        dvx = torch.empty(n_dvx, dtype=torch.float32, device=dev)
        d_vocab = torch.empty_like(vocab)
        tok_id, ptr, pos, n_tok, _ = ctx.csr
        d_out = d_out.detach().float().contiguous()
        _native.call("rnnl_lstm_train_backward", vocab.data_ptr(), *_LstmRules._ptrs(ps, L), L, 16, ctx.tok.data_ptr(),
                     T, m.padding_index, ridx.data_ptr(), n, act.data_ptr(), d_out.data_ptr(), da.data_ptr(),
                     xh.data_ptr(), dvx.data_ptr(), tok_id.data_ptr(), ptr.data_ptr(), pos.data_ptr(), n_tok,
                     d_vocab.data_ptr(), vocab.size(0), torch.cuda.current_stream(dev).cuda_stream)
        rows = n * T
        n_part = ctypes.c_size_t()
        _native.call("rnnl_lstm_weight_grads_scratch", L, rows, ctypes.byref(n_part))
        part = torch.empty(n_part.value, dtype=torch.float32, device=dev)
        wg = torch.empty(L * 64 * 33, dtype=torch.float32, device=dev)
        _native.call("rnnl_lstm_weight_grads", da.data_ptr(), xh.data_ptr(), L, rows, part.data_ptr(), n_part.value,
                     wg.data_ptr(), torch.cuda.current_stream(dev).cuda_stream)
        d_wih = wg[:L * 1024].view(L, 64, 16)
        d_whh = wg[L * 1024:L * 2048].view(L, 64, 16)
        d_b = wg[L * 2048:].view(L, 64)
        grads = []
        for k in range(L):
            grads += [d_wih[k], d_whh[k], d_b[k], d_b[k].clone()]
        return (None, None, None, None, d_vocab) + tuple(grads)


class PredictorPlus(_HipGrounding, torch.nn.Module):
    """Reference src/predictors.py:121-271, forward on the HIP path."""

    def __init__(self, graph, type="emb", num_layers=3, hidden_dim=16, entity_feature="bias", aggregator="sum",
                 embedding_path=None):
        super(PredictorPlus, self).__init__()
        self.graph = graph
        self.type = type
        self.num_layers = num_layers
        self.hidden_dim = hidden_dim
        self.entity_feature = entity_feature
        self.aggregator = aggregator
        self.embedding_path = embedding_path
        self.num_entities = graph.entity_size
        self.num_relations = graph.relation_size
        self.padding_index = graph.relation_size
        # the fused scoring kernels are specialised for the reference's hidden_dim
        # 16; other sizes run the HIP grounding + the aggregation / MLP as torch
        # ops on the grounding COO (forward_coo), on the GPU as well
        self.fused = hidden_dim == 16

        # module creation order == reference (identical RNG consumption under set_seed)
        self.vocab_emb = torch.nn.Embedding(self.num_relations + 1, self.hidden_dim, padding_idx=self.num_relations)
        if self.type == "lstm":
            self.rnn = torch.nn.LSTM(self.hidden_dim, self.hidden_dim, self.num_layers, batch_first=True)
        elif self.type == "gru":
            self.rnn = torch.nn.GRU(self.hidden_dim, self.hidden_dim, self.num_layers, batch_first=True)
        elif self.type == "rnn":
            self.rnn = torch.nn.RNN(self.hidden_dim, self.hidden_dim, self.num_layers, batch_first=True)
        elif self.type == "emb":
            self.rule_emb = None
        else:
            raise NotImplementedError
        if aggregator == "sum":
            self.rule_to_entity = FuncToNodeSum(self.hidden_dim)
        elif aggregator == "pna":
            self.rule_to_entity = FuncToNode(self.hidden_dim)
        else:
            raise NotImplementedError
        self.relation_emb = torch.nn.Embedding(self.num_relations, self.hidden_dim)
        self.score_model = MLP(self.hidden_dim * 2, [128, 1])
        if entity_feature == "bias":
            self.bias = torch.nn.parameter.Parameter(torch.zeros(self.num_entities))
        elif entity_feature == "RotatE":
            self.RotatE = RotatE(embedding_path)
        self._native_rules = {}
        self._node_cache = {}
        self._tok_cache = {}
        self._ws = {}
        self._ws_chunks = {}
        self._side = {}
        self._ws_uses = {}
        self._flags = np.zeros(1, dtype=np.uint32)  # the last launch's header flags (_status)
        self.capacity_scale = 1
        # RotatE base score (_forward_overlap): the grounding and the scoring
        # pass run on a side stream beside the RotatE kernel, both adding into
        # rows zeroed beside the rule encoder
        self.overlap = True
        # persistent workgroups of the side-stream kernels: at most one per CU
        # leaves RotatE its waves (it needs ~6 per SIMD to reach its floor;
        # 88.1 vs 91.1 ms/step at full occupancy).  Round 5: one per two CUs
        # (128 / 128) — the chain still ends well inside RotatE, and half of
        # the CUs keep RotatE's full occupancy: one N = 8 shard (5,261 rows)
        # 11.04-11.16 vs 11.39-11.79 ms, the full split 81.38-81.63 vs
        # 82.00-82.27 (96 / 96: 13.0 / 81.4; 64 / 64: the chain outlasts
        # RotatE, 17.4 / 108 ms; tools/shard_run.py, profiles/r05_overlap_ab.txt)
        # The PNA scoring pass is the chain's long pole beside RotatE: 1.5 per
        # CU since its walks went to four lanes per candidate (125 VGPRs; WN18RR
        # 18.05-18.15 ms at 384 vs 18.13-18.15 at 256, 18.14-18.17 at 512,
        # 20.5-20.7 at 128; the 233-VGPR per-candidate walk: 18.2 at 256,
        # 19.1 at 128, 18.6 at 384 — tools/lines_ab.py)
        self.overlap_ground_wg = 128
        self.overlap_score_wg = 128 if aggregator == "sum" else 384
        # the score rows' zero fill: issued before the rule encoder (beside it)
        # or by the forward call, after the encoder (beside rotate_hr and the
        # grounding's start).  SUM: by the call — FB15k-237 step 80.5-80.8 ->
        # 79.4-79.7 ms, N = 8 shard 11.03-11.21 -> 10.97-11.03 (the encoder
        # runs without the fill's 2.4 GB beside it, the grounding is resident
        # before RotatE starts); PNA (WN18RR) 18.37-18.43 early vs 18.41-18.47
        self.zero_early = aggregator != "sum"
        # without RotatE: the grounding on a side stream beside the rule
        # encoder (_forward_rows_fused)
        self.ground_early = True
        # pna aggregator: RotatE in two launches (rnnl_rotate_score_pieces;
        # bitwise the same scores).  The PNA scoring pass needs ~230 registers
        # per wave and finds no room beside RotatE's waves (6 x 80 per SIMD)
        # until a launch boundary drains them: WN18RR step 20.5 -> 18.4-18.6 ms
        # (round 4, tools/yield_ab.py: first launch over 0.35 / 0.5 / 0.65 /
        # 0.8 of the grid 18.5-18.9 / 18.55 / 18.48 / 18.44 ms).  The sum pass
        # (96 VGPRs) fits beside RotatE; there the boundary only costs its drain.
        self.rotate_yield = True
        self.rotate_share = 0.8  # the first launch's share of RotatE's grid
        # training forwards of the SUM aggregator: the fused HIP forward and
        # backward (_PlusSumTrain); False: torch autograd over the grounding COO
        self.fused_backward = True
        # training lookahead (TrainerPredictor.train calls prefetch on the next
        # batches): their grounding runs on a side stream during this step, and
        # the step reads its status and relation without waiting on the GPU
        self._pf = {}
        self.prefetch_depth = 2
        # the inference rule encoder over the rule trie (rnnl_lstm_encode_trie,
        # bitwise the per-rule rnnl_lstm_encode with 2.6x fewer LSTM steps on
        # FB15k-237); False: one lane row per rule
        self.encoder_trie = True
        self.prefetch_dropped = 0

    # ------------------------------------------------------------------ rules
    def set_rules(self, input):
        self.rules = _read_rules(input)
        logging.info("Predictor+: read {} rules from {}.".format(len(self.rules),
                                                                "list" if isinstance(input, list) else "file"))
        self.num_rules = len(self.rules)
        self.max_length = max([len(rule[1]) for rule in self.rules])
        self.relation2rules = [[] for _ in range(self.num_relations)]
        for index, rule in enumerate(self.rules):
            self.relation2rules[rule[0]].append([index, rule])
        self.rule_features = torch.tensor(
            [[h] + b + [self.padding_index] * (self.max_length - len(b)) for h, b in self.rules], dtype=torch.long)
        self._max_rules_per_relation = max(len(x) for x in self.relation2rules)
        if self.type == "emb":
            self.rule_emb = nn.parameter.Parameter(torch.zeros(self.num_rules, self.hidden_dim))
            nn.init.kaiming_uniform_(self.rule_emb, a=math.sqrt(5), mode="fan_in")
        self._native_rules = {}
        self._node_cache = {}
        self._tok_cache = {}
        # scratch sized by the old rules' trie (encoder state, backward, the
        # parameter block) and groundings of the old rules queued ahead
        self._side = {}
        self._pf = {}
        self.__dict__.pop("_src_lists", None)

    def encode_rules(self, rule_features):
        """LSTM/GRU/RNN output at each rule's last token (predictors.py:201-208)."""
        rule_masks = rule_features != self.num_relations
        output, _ = self.rnn(self.vocab_emb(rule_features))
        idx = (rule_masks.sum(-1) - 1).long()
        return output.gather(1, idx.view(-1, 1, 1).expand(-1, 1, self.hidden_dim)).squeeze(1)

    # ------------------------------------------------------------------ native plumbing
    def _embedding_sources(self):
        if self.type == "emb":
            return [self.rule_emb]
        return [self.vocab_emb.weight] + list(self.rnn.parameters())

    def all_rule_embeddings(self):
        """(num_rules, 16) embeddings of every rule, in rule-id order.  For
        type 'lstm' without autograd this is the fused HIP encoder
        (rnnl_lstm_encode); otherwise the torch modules."""
        if self.type == "emb":
            return self.rule_emb
        device = self.vocab_emb.weight.device
        if self.type == "lstm" and device.type == "cuda" and not self._needs_grad():
            return self._encode_rules_hip(device)
        return self.encode_rules(self.rule_features.to(device))

    def _encode_rules_hip(self, device, add_w=None, node_w=None):
        """The HIP rule encoder's (num_rules, 16) rows; with add_w and node_w
        (trie form only) also node_w's SUM records (rnnl_lstm_encode_trie_sum)."""
        L = self.num_layers
        rnn = self.rnn
        vocab = self.vocab_emb.weight.detach().float().contiguous()
        out = torch.empty((self.num_rules, self.hidden_dim), dtype=torch.float32, device=device)
        stream = torch.cuda.current_stream(device).cuda_stream
        if self.encoder_trie:
            # torch's per-layer parameters in place (no stacked copies)
            ps = []
            for k in range(L):
                for n in ("weight_ih", "weight_hh", "bias_ih", "bias_hh"):
                    t = getattr(rnn, "%s_l%d" % (n, k))
                    # fp32 contiguous parameters are read in place (no copy, no detach)
                    ps.append(t if t.dtype == torch.float32 and t.is_contiguous() else t.detach().float().contiguous())
            arrs = _LstmRules._ptrs(ps, L)
            # one step per rule-trie node: prefixes shared by many rules run once
            nr = self.native_rules(device)
            key = ("trie_state", self._device_index(device))
            st = self._side.get(key)
            if st is None:
                n = ctypes.c_size_t()
                _native.call("rnnl_lstm_encode_trie_scratch", nr.ptr, L, ctypes.byref(n))
                st = self._side[key] = torch.empty(n.value, dtype=torch.uint8, device=device)
            if node_w is not None:
                _native.call("rnnl_lstm_encode_trie_sum", nr.ptr, vocab.data_ptr(), *arrs, L, self.hidden_dim,
                             out.data_ptr(), out.stride(0), st.data_ptr(), st.numel(), add_w.data_ptr(),
                             node_w.data_ptr(), stream)
            else:
                _native.call("rnnl_lstm_encode_trie", nr.ptr, vocab.data_ptr(), *arrs, L, self.hidden_dim,
                             out.data_ptr(), out.stride(0), st.data_ptr(), st.numel(), stream)
            return out
        cat = lambda name: torch.stack([getattr(rnn, "%s_l%d" % (name, k)).detach().float()  # noqa: E731
                                        for k in range(L)]).contiguous()
        w_ih, w_hh, b_ih, b_hh = cat("weight_ih"), cat("weight_hh"), cat("bias_ih"), cat("bias_hh")
        # rule tokens depend only on the rule set: cached across invalidate_cache()
        # (a pageable host->device copy per forward costs 1-20 ms depending on the host)
        key = self._device_index(device)
        tok = self._tok_cache.get(key)
        if tok is None:
            tok = self.rule_features.to(dtype=torch.int32).contiguous().to(device)
            self._tok_cache[key] = tok
        _native.call("rnnl_lstm_encode", vocab.data_ptr(), w_ih.data_ptr(), w_hh.data_ptr(), b_ih.data_ptr(),
                     b_hh.data_ptr(), L, self.hidden_dim, tok.data_ptr(), self.num_rules, tok.size(1),
                     self.padding_index, out.data_ptr(), out.stride(0), stream)
        return out

    def _source_lists(self):
        """(node-weight sources, scoring-parameter sources): the tensors the
        cached node records and parameter block are derived from.  The lists
        are rebuilt when a direct submodule / parameter object or the rule set
        is replaced (a per-batch forward otherwise walks no module tree); the
        caches' keys then read each tensor's storage and version."""
        struct = (tuple(map(id, self._modules.values())), tuple(map(id, self._parameters.values())),
                  id(getattr(self, "rule_emb", None)))
        hit = self.__dict__.get("_src_lists")
        if hit is not None and hit[0] == struct:
            return hit[1], hit[2]
        rte, sm = self.rule_to_entity, self.score_model
        # SUM records carry FuncToNodeSum's Linear weight (rnnl_node_weights)
        node_srcs = self._embedding_sources() + ([rte.add_model.layers[0].weight] if self.aggregator == "sum" else [])
        param_srcs = [rte.add_model.layers[0].weight, rte.add_model.layers[0].bias, rte.layer_norm.weight,
                      rte.layer_norm.bias, sm.layers[0].weight, sm.layers[0].bias, sm.layers[1].weight,
                      sm.layers[1].bias, self.relation_emb.weight]
        if self.entity_feature == "bias":
            param_srcs.append(self.bias)
        self.__dict__["_src_lists"] = (struct, node_srcs, param_srcs)
        return node_srcs, param_srcs

    def node_weights(self, device):
        """Per-trie-node aggregates of the rule embeddings (HIP), cached until a
        source parameter changes (optimizer steps bump `_version`)."""
        nr = self.native_rules(device)
        srcs = self._source_lists()[0]
        key = (self._device_index(device), self.aggregator, tuple([p.data_ptr() for p in srcs]),
               tuple([p._version for p in srcs]))
        hit = self._node_cache.get(device)
        if hit is not None and hit[0] == key:
            return hit[1]
        agg = _native.AGG_SUM if self.aggregator == "sum" else _native.AGG_PNA
        add_w = self.rule_to_entity.add_model.layers[0].weight.detach().float().contiguous() \
            if self.aggregator == "sum" else None
        nbytes = ctypes.c_size_t()
        _native.call("rnnl_node_weights_size", nr.ptr, agg, ctypes.byref(nbytes))
        # the previous table's buffer is rewritten in place (every forward that
        # read it has ended: they end with their status read), so the records'
        # address — and with it the cached parameter block — stays the same
        w = hit[1] if hit is not None and hit[1].numel() == nbytes.value else \
            torch.empty(nbytes.value, dtype=torch.uint8, device=device)
        with torch.no_grad():
            if (self.type == "lstm" and self.aggregator == "sum" and self.encoder_trie and device.type == "cuda"
                    and not self._needs_grad()):
                # the SUM records formed by the trie encoder's launches (rnnl_lstm_encode_trie_sum)
                emb = self._encode_rules_hip(device, add_w, w)
            else:
                emb = self.all_rule_embeddings().detach().float().contiguous()
                _native.call("rnnl_node_weights", nr.ptr, emb.data_ptr(), emb.stride(0), agg,
                             add_w.data_ptr() if add_w is not None else None, w.data_ptr(),
                             torch.cuda.current_stream(device).cuda_stream)
        self._node_cache[device] = (key, w, emb, add_w)
        return w

    def _params(self, device, node_w):
        """The fused kernels' parameter block (rnnl_predictor_params), cached
        while node_w and every source tensor keep their storage and version
        (a per-batch forward then builds nothing)."""
        srcs = self._source_lists()[1]
        key = (node_w.data_ptr(), self.aggregator, self.entity_feature, tuple([t.data_ptr() for t in srcs]),
               tuple([t._version for t in srcs]))
        hit = self._side.get(("params", self._device_index(device)))
        if hit is not None and hit[0] == key:
            return hit[1], hit[2]
        p, keep = self._build_params(node_w)
        self._side[("params", self._device_index(device))] = (key, p, keep)
        return p, keep

    def _build_params(self, node_w):
        rte, sm = self.rule_to_entity, self.score_model
        p = _native.PredictorParams()
        p.aggregator = _native.AGG_SUM if self.aggregator == "sum" else _native.AGG_PNA
        p.feature = _native.FEATURE_ADD if self.entity_feature in ("bias", "RotatE") else _native.FEATURE_NONE
        p.node_w = node_w.data_ptr()
        tensors = [rte.add_model.layers[0].weight, rte.add_model.layers[0].bias, rte.layer_norm.weight,
                   rte.layer_norm.bias, sm.layers[0].weight, sm.layers[0].bias, sm.layers[1].weight,
                   sm.layers[1].bias, self.relation_emb.weight]
        keep = [t.detach().float().contiguous() for t in tensors]
        (p.add_w, p.add_b, p.ln_w, p.ln_b, p.s0_w, p.s0_b, p.s1_w, p.s1_b,
         p.rel_emb) = [t.data_ptr() for t in keep]
        if self.entity_feature == "bias":  # the scoring kernels add bias[t] without reading the filled row
            keep.append(self.bias.detach().float().contiguous())
            p.base_row = keep[-1].data_ptr()
        # packed once per weight version, not per launch (an older A/B build
        # without rnnl_pack_weights packs per launch)
        if self.hidden_dim == 16 and getattr(_native.lib(), "rnnl_pack_weights", None) is not None:
            n = ctypes.c_size_t()
            _native.call("rnnl_pack_weights_floats", ctypes.byref(n))
            packed = torch.empty(n.value, dtype=torch.float32, device=node_w.device)
            _native.call("rnnl_pack_weights", ctypes.byref(p), packed.data_ptr(),
                         torch.cuda.current_stream(node_w.device).cuda_stream)
            keep.append(packed)
            p.packed = packed.data_ptr()
        return p, keep

    def base_score(self, all_h, all_r, out):
        """Entity-feature part of the score (predictors.py:260-269)."""
        stream = torch.cuda.current_stream(out.device).cuda_stream
        nq = all_h.numel()
        if self.entity_feature == "bias":
            b = self.bias.detach().float().contiguous()
            _native.call("rnnl_fill_rows", b.data_ptr(), nq, self.num_entities, out.data_ptr(), stream)
        elif self.entity_feature == "RotatE":
            self.RotatE.score_into(all_h, all_r, out, accumulate=False)
        else:
            _native.call("rnnl_fill_value", float("-inf"), out.numel(), out.data_ptr(), stream)

    def invalidate_cache(self):
        """Drop cached per-node rule aggregates (recomputed on the next forward)."""
        self._node_cache = {}

    @_native.on_input_device
    def forward_rows(self, all_h, all_r, edges_to_remove=None, return_ncand=False, digest=None, events=None,
                     dedupe=False):
        """Forward for any rows (one or many reference batches, mixed relations).

        Returns (score (n, |E|) f32, mask (n, |E|) bool[, n_cand (n,) int32]).
        `events`, if a dict, receives torch.cuda.Events bracketing the node
        aggregate, base-score and grounding kernels (all on the current stream).
        `dedupe` (eval rows only): an eval-mode row's output depends on (h, r)
        alone, so each distinct (h, r) is computed once and its row copied to
        the duplicates — bit-identical output (the FB15k-237 test split has
        22,850 distinct (h, r) among 40,932 rows)."""
        if dedupe and edges_to_remove is None and digest is None and events is None and all_h.numel() > 1:
            key = all_r.to(torch.int64) * self.num_entities + all_h.to(torch.int64)
            uniq, inv = torch.unique(key, return_inverse=True)  # sorted by relation, then head
            if uniq.numel() < key.numel():
                uh, ur = uniq % self.num_entities, uniq // self.num_entities
                score, mask, n_cand = self.forward_rows(uh, ur, None, return_ncand=True)
                score, mask, n_cand = score.index_select(0, inv), mask.index_select(0, inv), n_cand[inv]
                return (score, mask, n_cand) if return_ncand else (score, mask)
        device = all_h.device
        if device.type != "cuda":
            raise RuntimeError("PredictorPlus runs on the HIP path: move inputs and model to a GPU")
        all_h = all_h.to(torch.int64).contiguous()
        all_r = all_r.to(torch.int64).contiguous()
        etr = edges_to_remove.to(device, torch.int64).contiguous() if edges_to_remove is not None else None
        nq = all_h.numel()
        if nq == 0:  # no rows: empty outputs, no launch
            out = (torch.empty((0, self.num_entities), dtype=torch.float32, device=device),
                   torch.empty((0, self.num_entities), dtype=torch.bool, device=device))
            return out + (torch.empty(0, dtype=torch.int32, device=device),) if return_ncand else out
        if not self.fused:
            with torch.no_grad():
                score, mask, n_cand = self.forward_coo(all_h, all_r, etr)
            return (score, mask, n_cand) if return_ncand else (score, mask)
        try:
            return self._forward_rows_fused(device, all_h, all_r, etr, nq, return_ncand, digest, events)
        except _native.NativeError as e:
            if e.code != _native.RNNL_ERR_RANGE or digest is not None:
                raise
        # out of the fused kernels' exact integer ranges (a path count past 2^32,
        # non-finite or huge rule aggregates, feature sums past int64): the
        # reference's fp32 arithmetic on the grounding COO with int64 counts,
        # which propagates infinities and NaNs as the reference does
        logging.info("PredictorPlus: %s; rows recomputed on the grounding COO (int64 counts, fp32 torch ops)",
                     _native.lib().rnnl_last_error().decode(errors="replace"))
        with torch.no_grad():
            score, mask, n_cand = self.forward_coo(all_h, all_r, etr, nonfinite=True)
        return (score, mask, n_cand) if return_ncand else (score, mask)

    def _forward_rows_fused(self, device, all_h, all_r, etr, nq, return_ncand, digest, events):
        g = self.graph.device_graph(device)
        nr = self.native_rules(device)
        rec = (lambda k: events.setdefault(k, torch.cuda.Event(enable_timing=True)).record()) \
            if events is not None else (lambda k: None)
        rec("start")
        score = torch.empty((nq, self.num_entities), dtype=torch.float32, device=device)
        overlap = self.entity_feature == "RotatE" and self.overlap and nq >= 2
        if overlap and self.zero_early:  # zero the rows on a side stream beside the rule encoder
            _native.call("rnnl_forward_rotate_zero", score.data_ptr(), score.numel(),
                         torch.cuda.current_stream(device).cuda_stream)
        early = None
        if not overlap and self.ground_early and events is None and nq >= 2:
            # the grounding reads no rule weights: on a side stream beside the
            # rule encoder and node records, the scoring pass on the current
            # stream after both (the split halves of rnnl_predictorplus_forward)
            main = torch.cuda.current_stream(device)
            side = self._ground_stream(device)
            scale = self.capacity_scale
            ws = self._workspace(device, nq, scale)
            n_cand = torch.empty(nq, dtype=torch.int32, device=device)
            side.wait_stream(main)
            _native.call("rnnl_predictorplus_ground", g, nr.ptr,
                         _native.AGG_SUM if self.aggregator == "sum" else _native.AGG_PNA, all_h.data_ptr(),
                         all_r.data_ptr(), etr.data_ptr() if etr is not None else None, nq, n_cand.data_ptr(),
                         ws.data_ptr(), ws.numel(), scale, 0, side.cuda_stream)
            early = (side, ws, scale)
        node_w = self.node_weights(device)
        params, keep = self._params(device, node_w)
        stream = torch.cuda.current_stream(device).cuda_stream
        none_mode = params.feature == _native.FEATURE_NONE
        if early is None:
            n_cand = torch.empty(nq, dtype=torch.int32, device=device)
        if overlap:
            mask = self._forward_overlap(device, g, nr, params, all_h, all_r, etr, score, n_cand, digest, events)
            del keep
            return (score, mask, n_cand) if return_ncand else (score, mask)
        while True:
            mask8 = torch.zeros((nq, self.num_entities), dtype=torch.uint8, device=device) if none_mode else None
            if early is not None:  # the grounding was enqueued beside the encoder: score after it
                side, ws, scale = early
                early = None
                self.base_score(all_h, all_r, score)
                torch.cuda.current_stream(device).wait_stream(side)
                _native.call("rnnl_predictorplus_score", g, nr.ptr, ctypes.byref(params), all_h.data_ptr(),
                             all_r.data_ptr(), nq, score.data_ptr(), mask8.data_ptr() if mask8 is not None else None,
                             n_cand.data_ptr(), digest.data_ptr() if digest is not None else None, ws.data_ptr(),
                             ws.numel(), scale, 0, 0, stream)
                # a grounding saved for a training backward in this workspace is now stale
                self._ws_touch(ws)
            else:
                scale = self.capacity_scale
                ws = self._workspace(device, nq, scale)
                rec("base")
                self.base_score(all_h, all_r, score)
                rec("ground")
                _native.call("rnnl_predictorplus_forward", g, nr.ptr, ctypes.byref(params), all_h.data_ptr(),
                             all_r.data_ptr(), etr.data_ptr() if etr is not None else None, nq, score.data_ptr(),
                             mask8.data_ptr() if mask8 is not None else None, n_cand.data_ptr(),
                             digest.data_ptr() if digest is not None else None, ws.data_ptr(), ws.numel(), scale,
                             stream)
                self._ws_touch(ws)
            rec("end")
            rc = self._status(ws, stream)
            if rc == _native.RNNL_ERR_OVERFLOW and self.capacity_scale < 64:
                self.capacity_scale *= 2
                logging.info("PredictorPlus: workspace overflow, capacity_scale -> %d", self.capacity_scale)
                continue
            _native.check(rc)
            break
        del keep
        if none_mode:
            mask = mask8.bool()
        else:
            mask = torch.ones((nq, self.num_entities), dtype=torch.bool, device=device)
        return (score, mask, n_cand) if return_ncand else (score, mask)

    def _ground_stream(self, device):
        key = ("ground_stream", self._device_index(device))
        st = self._side.get(key)
        if st is None:
            st = self._side[key] = torch.cuda.Stream(device)
        return st

    def _overlap_workspace(self, device, nq, scale):
        sk = ("need", self._device_index(device), nq, scale)
        need = self._ws_chunks.get(sk)
        if need is None:  # sizes depend on (rows, scale) only: one query per shape
            need = ctypes.c_size_t()
            _native.call("rnnl_forward_workspace_size", self.graph.device_graph(device),
                         self.native_rules(device).ptr, nq, scale, ctypes.byref(need))
            self._ws_chunks[sk] = need
        key = self._device_index(device)
        ws = self._ws_chunks.get(key)
        if ws is None or ws.numel() < need.value:
            ws = torch.empty(need.value, dtype=torch.uint8, device=device)
            self._ws_chunks[key] = ws
        return ws

    def _forward_overlap(self, device, g, nr, params, all_h, all_r, etr, score, n_cand, digest, events):
        """RotatE entity feature: one host call (rnnl_predictorplus_forward_rotate)
        runs the one-stream path's kernels on three streams.  The grounding and
        then the scoring pass run on a side stream beside RotatE on the current
        stream (the grounding does not read the base score; it is latency-bound
        where RotatE is VALU-bound), and are enqueued before RotatE so that
        their persistent workgroups are resident before RotatE's blocks fill
        the chip.  The score rows were zeroed on a second side stream
        (rnnl_forward_rotate_zero, before the rule encoder), and RotatE and the
        scoring pass both add into them atomically: two addends on an exact
        zero round to fl(rotate + out) in either order, so the rows are the
        one-stream path's bit for bit.  Returns the (all-True) mask, filled
        on the current stream behind RotatE."""
        main = torch.cuda.current_stream(device)
        nq = all_h.numel()
        pieces = 2 if self.rotate_yield and params.aggregator == _native.AGG_PNA else 1
        rot = self.RotatE.native_args(nq, pieces, self.rotate_share if pieces > 1 else 0.0)
        mask = torch.empty((nq, self.num_entities), dtype=torch.bool, device=device)
        ev = None
        if events is not None:  # timing: before the launches, after RotatE, after the side stream
            evs = [events.setdefault(k, torch.cuda.Event(enable_timing=True)) for k in ("base", "ground", "end")]
            for e in evs:  # torch creates an event's handle on its first record
                e.record(main)
            ev = (ctypes.c_void_p * 3)(*[e.cuda_event for e in evs])
        zeroed = 1 if self.zero_early else 0
        while True:
            scale = self.capacity_scale
            ws = self._overlap_workspace(device, nq, scale)
            rc = _native.lib().rnnl_predictorplus_forward_rotate(
                g, nr.ptr, ctypes.byref(params), ctypes.byref(rot), all_h.data_ptr(), all_r.data_ptr(),
                etr.data_ptr() if etr is not None else None, nq, score.data_ptr(), mask.data_ptr(), n_cand.data_ptr(),
                digest.data_ptr() if digest is not None else None, ws.data_ptr(), ws.numel(), scale,
                self.overlap_ground_wg, self.overlap_score_wg, zeroed, ev, main.cuda_stream, None,
                self._flags.ctypes.data_as(ctypes.c_void_p))
            if rc == _native.RNNL_ERR_OVERFLOW and self.capacity_scale < 64:
                self.capacity_scale *= 2
                zeroed = 0  # the retried launch starts from zeroed rows again
                logging.info("PredictorPlus: workspace overflow, capacity_scale -> %d", self.capacity_scale)
                continue
            _native.check(rc)
            return mask

    # ------------------------------------------------------------------ autograd (training) path
    @_native.on_input_device
    def forward_autograd(self, all_h, all_r, edges_to_remove, query_r=None):
        """Differentiable forward (training): the HIP grounding's COO, then the
        reference's aggregation / MLP / entity feature as torch ops on it, so
        autograd yields the reference's gradients (predictors.py:210-271,
        layers.py:53-126, embedding.py:45-70)."""
        device = all_h.device
        all_h = all_h.to(torch.int64)
        all_r = all_r.to(torch.int64)
        nq, E = all_h.numel(), self.num_entities
        if self.fused and self.aggregator == "sum" and self.fused_backward and device.type == "cuda":
            try:
                return self._forward_sum_train(all_h, all_r, edges_to_remove, query_r)
            except _native.NativeError as e:
                if e.code != _native.RNNL_ERR_RANGE:
                    raise
                # past the fused kernels' integer ranges: the autograd COO path below
        if self.fused and self.aggregator == "pna" and self.fused_backward and device.type == "cuda":
            try:
                return self._forward_pna_train(all_h, all_r, edges_to_remove, query_r)
            except _native.NativeError as e:
                if e.code != _native.RNNL_ERR_RANGE:
                    raise
        row, ent, ce, node, count = self.ground_coo(all_h, all_r, edges_to_remove)
        if ent.numel() == 0:
            # predictors.py:230-237 early return
            zero = torch.zeros((nq, E), device=device)
            if self.entity_feature == "bias":
                return zero + self.bias.unsqueeze(0), torch.ones((nq, E), dtype=torch.bool, device=device)
            if self.entity_feature == "RotatE":
                return zero + self.RotatE(all_h, all_r), torch.ones((nq, E), dtype=torch.bool, device=device)
            return zero - float("-inf"), torch.zeros((nq, E), dtype=torch.bool, device=device)
        return self._score_coo(all_h, all_r, row, ent, ce, node, count, rels=query_r)

    @_native.on_input_device
    def _forward_sum_train(self, all_h, all_r, edges_to_remove, query_r):
        """forward_autograd for the SUM aggregator through _PlusSumTrain."""
        raw = (all_h, all_r, edges_to_remove)
        device = all_h.device
        etr = edges_to_remove.to(device, torch.int64).contiguous() if edges_to_remove is not None else None
        all_h, all_r = all_h.contiguous(), all_r.contiguous()
        head = int(query_r) if isinstance(query_r, int) else -1
        if self.type == "emb":
            emb = self.rule_emb
        else:
            rels = [head] if head >= 0 else torch.unique(all_r).tolist()
            ridx = self._rule_ids(rels, device)
            x_f = self._encode_rules_padded(ridx, device, rels)
            emb = torch.zeros((self.num_rules, self.hidden_dim), dtype=x_f.dtype, device=device).index_copy(
                0, ridx, x_f)
        if self.entity_feature == "bias":
            kind, base = "bias", self.bias
        elif self.entity_feature == "RotatE":
            kind, base = "rows", self.RotatE(all_h, all_r)
        else:
            kind, base = "none", None
        rte, sm = self.rule_to_entity, self.score_model
        # (autograd runs Function.forward with grad mode off: decide here)
        raw = raw if self._prefetch_enabled() else None
        return _PlusSumTrain.apply(self, raw, all_h, all_r, etr, head, kind, base, emb, rte.add_model.layers[0].weight,
                                   rte.add_model.layers[0].bias, rte.layer_norm.weight, rte.layer_norm.bias,
                                   sm.layers[0].weight, sm.layers[0].bias, sm.layers[1].weight, sm.layers[1].bias,
                                   self.relation_emb.weight)

    @_native.on_input_device
    def _forward_pna_train(self, all_h, all_r, edges_to_remove, query_r):
        """forward_autograd for the PNA aggregator: FuncToNode's statistics
        on the HIP grounding (_PnaStats: one kernel forward, one backward)
        and its dense rest (layers.FuncToNode.finish) and score_model as
        torch layers."""
        device = all_h.device
        nq, E = all_h.numel(), self.num_entities
        etr = edges_to_remove.to(device, torch.int64).contiguous() if edges_to_remove is not None else None
        all_h, all_r = all_h.contiguous(), all_r.contiguous()
        head = int(query_r) if isinstance(query_r, int) else -1
        if self.type == "emb":
            emb = self.rule_emb
        else:
            rels = [head] if head >= 0 else torch.unique(all_r).tolist()
            ridx = self._rule_ids(rels, device)
            x_f = self._encode_rules_padded(ridx, device, rels)
            emb = torch.zeros((self.num_rules, self.hidden_dim), dtype=x_f.dtype, device=device).index_copy(
                0, ridx, x_f)
        wsum, wsq, mn, mx, deg, row, ent, row_scale = _PnaStats.apply(self, emb, all_h, all_r, etr, head)
        if ent.numel() == 0:  # predictors.py:230-237 early return
            zero = torch.zeros((nq, E), device=device)
            if self.entity_feature == "bias":
                return zero + self.bias.unsqueeze(0), torch.ones((nq, E), dtype=torch.bool, device=device)
            if self.entity_feature == "RotatE":
                return zero + self.RotatE(all_h, all_r), torch.ones((nq, E), dtype=torch.bool, device=device)
            return zero - float("-inf"), torch.zeros((nq, E), dtype=torch.bool, device=device)
        out = self.rule_to_entity.finish(wsum, wsq, mn, mx, deg, row, nq, row_scale=row_scale)
        return self._score_tail(all_h, all_r, row, ent, out, head=head)

    def _pna_scratch(self, device):
        key = ("pna_bwd", self._device_index(device))
        sb = self._side.get(key)
        if sb is None:
            n = ctypes.c_size_t()
            _native.call("rnnl_pna_features_backward_scratch", self.native_rules(device).ptr, ctypes.byref(n))
            sb = self._side[key] = torch.empty(n.value, dtype=torch.uint8, device=device)
        return sb

    def _prefetch_enabled(self):
        """The lookahead serves the fused SUM training forward only."""
        return (self.fused and self.aggregator == "sum" and self.fused_backward and self.training and
                torch.is_grad_enabled())

    def _prefetch_ground(self, g, nr, h, r, etr, nq, n_cand, ws, scale, stream):
        _native.call("rnnl_predictorplus_ground", g, nr.ptr, _native.AGG_SUM, h.data_ptr(), r.data_ptr(),
                     etr.data_ptr() if etr is not None else None, nq, n_cand.data_ptr(), ws.data_ptr(), ws.numel(),
                     scale, 0, stream)

    def _node_flag_slot(self, device):
        """(pinned int32, event): the host copy of a node-record table's range
        flag for the lookahead training forward (waited on within the call)."""
        key = ("nflag", self._device_index(device))
        v = self._side.get(key)
        if v is None:
            v = self._side[key] = (torch.zeros(4, dtype=torch.uint8, pin_memory=True), torch.cuda.Event())
        return v

    def _backward_scratch(self, device):
        key = ("bwd", self._device_index(device))
        sb = self._side.get(key)
        if sb is None:
            n = ctypes.c_size_t()
            _native.call("rnnl_predictorplus_backward_size", self.native_rules(device).ptr, self.num_relations,
                         ctypes.byref(n))
            sb = self._side[key] = torch.empty(n.value, dtype=torch.uint8, device=device)
        return sb

    @_native.on_input_device
    def forward_coo(self, all_h, all_r, edges_to_remove=None, nonfinite=False):
        """Rows of any relations through the HIP grounding COO and the torch
        aggregation / MLP (any hidden_dim): (score, mask, n_cand), the
        forward_rows contract — rows without candidates keep their base score
        (bias / RotatE) or -inf with the mask False (entity_feature none).
        nonfinite: the reference's 0 x (non-finite embedding) NaNs (range
        fallback, _reference_nonfinite)."""
        device = all_h.device
        all_h = all_h.to(torch.int64)
        all_r = all_r.to(torch.int64)
        nq, E = all_h.numel(), self.num_entities
        row, ent, ce, node, count = self.ground_coo(all_h, all_r, edges_to_remove)
        n_cand = torch.zeros(nq, dtype=torch.int32, device=device).index_add_(
            0, row, torch.ones_like(row, dtype=torch.int32))
        if ent.numel() == 0:
            if self.entity_feature == "bias":
                return self.bias.detach().float().unsqueeze(0).expand(nq, E).contiguous(), \
                    torch.ones((nq, E), dtype=torch.bool, device=device), n_cand
            if self.entity_feature == "RotatE":
                return self.RotatE(all_h, all_r), torch.ones((nq, E), dtype=torch.bool, device=device), n_cand
            return torch.full((nq, E), float("-inf"), device=device), \
                torch.zeros((nq, E), dtype=torch.bool, device=device), n_cand
        score, mask = self._score_coo(all_h, all_r, row, ent, ce, node, count, nonfinite=nonfinite)
        return score, mask, n_cand

    def _score_coo(self, all_h, all_r, row, ent, ce, node, count, rels=None, nonfinite=False):
        """predictors.py:238-271 on the grounding COO (torch ops).  `rels`: the
        rows' relations when the caller knows them (forward's single-relation
        batch), which saves the host sync of torch.unique."""
        device = all_h.device
        nq, E = all_h.numel(), self.num_entities
        C = ent.numel()
        nr = self.native_rules(device)
        rels = [rels] if isinstance(rels, int) else torch.unique(all_r).tolist()
        ridx = self._rule_ids(rels, device)
        if self.type == "emb":
            x_f = self.rule_emb.index_select(0, ridx)
        else:
            x_f = self._encode_rules_padded(ridx, device, rels)
        nodes = nr.node_of_rule[ridx]
        H = self.hidden_dim
        # gathers of differentiable tables use index_select: its backward is an
        # index_add, where x[idx]'s is the sort-based index_put accumulate
        # (8 ms of a 16.5 ms FB15k-237 training step)
        cnt = count.to(x_f.dtype).unsqueeze(-1)
        node_sum = torch.zeros((nr.n_nodes, H), device=device, dtype=x_f.dtype).index_add(0, nodes, x_f)
        wsum = torch.zeros((C, H), device=device, dtype=x_f.dtype).index_add(0, ce, cnt * node_sum.index_select(0, node))
        cand_nan = None
        if nonfinite:
            cand_nan = self._reference_nonfinite(device, all_r, ridx, x_f, row, ce, node, C)[0]
            wsum = torch.where(cand_nan, torch.full_like(wsum, float("nan")), wsum)
        if self.aggregator == "sum":
            out = self.rule_to_entity.finish(wsum)
        else:
            node_sq = torch.zeros((nr.n_nodes, H), device=device, dtype=x_f.dtype).index_add(0, nodes, x_f * x_f)
            node_n = torch.zeros(nr.n_nodes, device=device, dtype=x_f.dtype).index_add(
                0, nodes, torch.ones_like(nodes, dtype=x_f.dtype))
            idx_n = nodes.unsqueeze(-1).expand(-1, H)
            node_min = torch.full((nr.n_nodes, H), float("inf"), device=device, dtype=x_f.dtype).scatter_reduce(
                0, idx_n, x_f, "amin", include_self=True)
            node_max = torch.full((nr.n_nodes, H), float("-inf"), device=device, dtype=x_f.dtype).scatter_reduce(
                0, idx_n, x_f, "amax", include_self=True)
            wsq = torch.zeros((C, H), device=device, dtype=x_f.dtype).index_add(0, ce, cnt * node_sq.index_select(0, node))
            if cand_nan is not None:
                wsq = torch.where(cand_nan, torch.full_like(wsq, float("nan")), wsq)
            deg = torch.zeros(C, device=device, dtype=x_f.dtype).index_add(0, ce, cnt.squeeze(-1) * node_n.index_select(0, node)) + 1
            idx_c = ce.unsqueeze(-1).expand(-1, H)
            mn = torch.full((C, H), float("inf"), device=device, dtype=x_f.dtype).scatter_reduce(
                0, idx_c, node_min.index_select(0, node), "amin", include_self=True)
            mx = torch.full((C, H), float("-inf"), device=device, dtype=x_f.dtype).scatter_reduce(
                0, idx_c, node_max.index_select(0, node), "amax", include_self=True)
            out = self.rule_to_entity.finish(wsum, wsq, mn, mx, deg, row, nq)
        return self._score_tail(all_h, all_r, row, ent, out)

    def _score_tail(self, all_h, all_r, row, ent, out, head=-1):
        """predictors.py:251-271 from rule_to_entity's output (C, H) of the
        candidates (row, ent): score_model, the scatter into (B, |E|) and the
        entity feature / mask.  head >= 0: every row is of that relation (its
        embedding broadcast: the gradient is a plain sum over the candidates,
        not an index_add's atomics)."""
        device = all_h.device
        nq, E = all_h.numel(), self.num_entities
        if head >= 0:
            rel = self.relation_emb.weight[head].unsqueeze(0).expand(row.numel(), -1)
        else:
            rel = self.relation_emb(all_r).index_select(0, row)  # per row, then per candidate
        output = self.score_model(torch.cat([out, rel], dim=-1)).squeeze(-1)
        score = torch.zeros(nq * E, device=device, dtype=output.dtype).scatter(0, row * E + ent, output).view(nq, E)
        if self.entity_feature == "bias":
            return score + self.bias.unsqueeze(0), torch.ones((nq, E), dtype=torch.bool, device=device)
        if self.entity_feature == "RotatE":
            # RotatE.forward takes its HIP backward only when eemb / remb are trained
            rot = self.RotatE(all_h, all_r)
            return score + rot, torch.ones((nq, E), dtype=torch.bool, device=device)
        mask = torch.zeros(nq * E, dtype=torch.bool, device=device).index_fill(0, row * E + ent, True).view(nq, E)
        return score.masked_fill(~mask, float("-inf")), mask

    def _rule_ids(self, rels, device):
        """Device int64 ids of the rules of relations `rels` (relation order,
        then file order); one relation's list is uploaded once and cached."""
        if len(rels) == 1:
            key = ("rids", self._device_index(device), rels[0])
            hit = self._tok_cache.get(key)
            if hit is None:
                hit = torch.tensor([i for i, _ in self.relation2rules[rels[0]]], dtype=torch.long, device=device)
                self._tok_cache[key] = hit
            return hit
        return torch.tensor([i for q in rels for i, _ in self.relation2rules[q]], dtype=torch.long, device=device)

    def _lstm_hip(self, device):
        """The rule encoder's HIP training path applies: an LSTM of the fused
        kernels' shape (hidden 16, 1-3 layers, rules of <= 7 tokens)."""
        return (self.type == "lstm" and device.type == "cuda" and self.hidden_dim == 16 and
                1 <= self.num_layers <= 3 and self.rule_features.size(1) <= 8 and self.rnn.bias and
                not self.rnn.bidirectional and self.rnn.proj_size == 0)

    def _token_csr(self, rels, device):
        """Per-token positions (row T + t) of the non-pad tokens of the rules of
        `rels` (in _rule_ids order), grouped by token id in position order:
        (tok_id, ptr, pos) on the device — the vocab-row gradient's sum order
        (rnnl_lstm_train_backward).  One relation's lists are cached."""
        key = ("csr", self._device_index(device), tuple(rels))
        hit = self._tok_cache.get(key)
        if hit is not None:
            return hit
        ids = [i for q in rels for i, _ in self.relation2rules[q]]
        tok = self.rule_features.numpy()[ids]
        T = tok.shape[1]
        flat = tok.reshape(-1)
        pos = np.nonzero(flat != self.padding_index)[0]
        order = np.argsort(flat[pos], kind="stable")
        pos = pos[order]
        vals = flat[pos]
        tok_id, counts = np.unique(vals, return_counts=True)
        ptr = np.concatenate([[0], np.cumsum(counts)])
        packed = torch.from_numpy(np.concatenate([tok_id, ptr, pos]).astype(np.int32)).to(device)
        u = tok_id.size
        hit = (packed[:u], packed[u:2 * u + 1], packed[2 * u + 1:], u, T)
        if len(rels) == 1:
            self._tok_cache[key] = hit
        return hit

    def _encode_rules_padded(self, ridx, device, rels=None):
        """encode_rules over the rules `ridx` with autograd (the training
        path).  An LSTM of the fused shape runs the HIP recurrence and its
        backward through time (_LstmRules); otherwise the torch modules.  The
        token table lives on the device (uploaded once), and the
        LSTM input is padded to a fixed row count — the largest per-relation
        rule list, or a multiple of 512 beyond it — so the recurrent kernels
        see one shape, not one per relation (a new RNN shape costs a kernel
        selection on its first use).  The padding rows repeat rule 0; their
        outputs are dropped, so they add nothing to the gradients."""
        if rels is not None and self._lstm_hip(device) and ridx.numel() > 0:
            rnn = self.rnn
            params = []
            for k in range(self.num_layers):
                params += [getattr(rnn, "%s_l%d" % (name, k)) for name in ("weight_ih", "weight_hh", "bias_ih",
                                                                             "bias_hh")]
            key = self._device_index(device)
            tok = self._tok_cache.get(key)
            if tok is None:
                tok = self._tok_cache[key] = self.rule_features.to(dtype=torch.int32).contiguous().to(device)
            return _LstmRules.apply(self, ridx, tok, self._token_csr(rels, device), self.vocab_emb.weight, *params)
        key = ("tok64", self._device_index(device))
        tok = self._tok_cache.get(key)
        if tok is None:
            tok = self.rule_features.to(device)
            self._tok_cache[key] = tok
        n = ridx.numel()
        rows = max(self._max_rules_per_relation, 1)
        if n > rows:
            rows = (n + 511) // 512 * 512
        if rows > n:
            ridx = torch.cat([ridx, ridx.new_zeros(rows - n)])
        return self.encode_rules(tok.index_select(0, ridx))[:n]

    @_native.on_input_device
    def forward(self, all_h, all_r, edges_to_remove):
        """predictors.py:210-271: one single-relation batch -> (score, mask).

        With autograd active (training) the differentiable path runs
        (forward_autograd); otherwise the fused HIP kernels (forward_rows)."""
        if self._needs_grad():
            pre = self._prefetched(all_h.device, all_h, all_r, edges_to_remove, peek=True) \
                if self._prefetch_enabled() and all_h.is_cuda else None
            if pre is not None:
                # grounded ahead: the one-relation flag and the relation from its
                # header copy (its event ended long ago: no wait on this step)
                pre[6].synchronize()
                _native.call("rnnl_forward_flags_host", pre[8].data_ptr(), self._flags.ctypes.data_as(ctypes.c_void_p))
                self._check_one_relation()
                query_r = self._prefetch_relation(pre[8], self._header_bytes())
            else:
                # the reference's single-relation check (predictors.py:211-212) in one host
                # read, which also gives the relation whose rules the autograd path gathers
                query_r, n_other = torch.stack([all_r[0], (all_r != all_r[0]).sum()]).tolist()
                assert n_other == 0
            return self.forward_autograd(all_h, all_r, edges_to_remove, query_r=query_r)
        # eval: the grounding kernel flags rows of another relation in the
        # launch header, read back with the status (no extra reduction or sync)
        self._flags[0] = 0
        score, mask, n_cand = self.forward_rows(all_h, all_r, edges_to_remove, return_ncand=True)
        self._check_one_relation()
        if self.entity_feature not in ("bias", "RotatE"):
            # reference early return `mask - float('-inf')` (predictors.py:236-237): +inf
            # where the batch has no candidate (mask all False), without a host read
            score = torch.where(mask.any(), score, torch.full_like(score, float("inf")))
        return score, mask

    @property
    def mask_all_true(self):
        """Every entity is scored (the reference's mask is all True) with the
        bias and RotatE features (predictors.py:260-266)."""
        return self.entity_feature in ("bias", "RotatE")
