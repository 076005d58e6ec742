"""RuleMiner, API-compatible with the reference's rule-search stage
(miner/rnnlogic.cpp RuleMiner: search :505-589, get_logic_rules, save
:591-610), with the search on the GPU (rnnl_rule_search, csrc/mine.hip).

    miner = RuleMiner(graph)            # graph: rnnlogic_amd.data.KnowledgeGraph
    rules = miner.search(max_length=3)  # [(head, body tuple)] in the reference's order
    miner.save("mined_rules.txt")       # "type head body... H wt prior", as RuleMiner::save

The pool equals the reference's for the same train graph: every relation
path of length <= max_length from h to t of a train triple (h, r, t), the
triple's own edge removed, as the rule r <- path; r <- r dropped; per head in
std::set<Rule> order (length, then body).  max_length <= 3.
"""
import ctypes

import numpy as np
import torch

from . import _native


class RuleMiner(object):

    def __init__(self, graph, device=None):
        self.graph = graph
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        hrt = np.ascontiguousarray(np.asarray(graph.train_facts, dtype=np.int32).reshape(-1, 3))
        self._handle = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            _native.call("rnnl_miner_create", hrt.ctypes.data, len(hrt), graph.entity_size, graph.relation_size,
                         ctypes.byref(self._handle))
        self.rules = []
        self.table_bits = 22

    def __del__(self):
        h = getattr(self, "_handle", None)
        if h is not None and h.value:
            try:
                _native.lib().rnnl_miner_destroy(h)
            except Exception:
                pass

    @staticmethod
    def decode(keys):
        """rule keys (head<<47 | len<<45 | b1<<30 | b2<<15 | b3) -> [(head, body)] in key order."""
        keys = np.sort(np.asarray(keys, dtype=np.uint64))
        m = np.uint64(0x7FFF)
        head = (keys >> np.uint64(47)).astype(np.int64)
        ln = ((keys >> np.uint64(45)) & np.uint64(3)).astype(np.int64)
        b = np.stack([(keys >> np.uint64(30)) & m, (keys >> np.uint64(15)) & m, keys & m], 1).astype(np.int64)
        return [(int(hd), tuple(int(x) for x in b[i, :n])) for i, (hd, n) in enumerate(zip(head, ln))]

    @torch.no_grad()
    def search_keys(self, max_length):
        """Device search; returns the distinct rule keys (numpy uint64, unsorted)."""
        stream = torch.cuda.current_stream(self.device).cuda_stream
        counters = torch.zeros(4, dtype=torch.int64, device=self.device)
        while True:
            cap = 1 << self.table_bits
            table = torch.empty(cap, dtype=torch.int64, device=self.device)
            out = torch.empty(cap, dtype=torch.int64, device=self.device)
            _native.call("rnnl_rule_search", self._handle, int(max_length), table.data_ptr(), cap, out.data_ptr(),
                         cap, counters.data_ptr(), stream)
            c = counters.cpu().tolist()
            if c[1] == 0 and c[2] <= cap // 2:
                return out[:c[2]].cpu().numpy().view(np.uint64)
            self.table_bits += 1  # keep the open-addressing set at most half full
            if self.table_bits > 31:
                raise RuntimeError("rule search: rule set too large")

    def search(self, max_length):
        """RuleMiner::search over all train triples (portion 1)."""
        self.rules = self.decode(self.search_keys(max_length))
        return self.rules

    def get_logic_rules(self):
        """Per head relation, its rules in order (RuleMiner::get_logic_rules)."""
        rel2rules = [[] for _ in range(self.graph.relation_size)]
        for hd, body in self.rules:
            rel2rules[hd].append((hd, body))
        return rel2rules

    def save(self, file_name):
        """RuleMiner::save (rnnlogic.cpp:591-610): 'type head body... H wt prior'
        (H, wt, prior are 0 after a search)."""
        with open(file_name, "w") as fo:
            for hd, body in self.rules:
                fo.write("%d %d%s %f %f %f\n" % (len(body), hd, "".join(" %d" % x for x in body), 0.0, 0.0, 0.0))
        return len(self.rules)
