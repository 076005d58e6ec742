"""Knowledge graph + datasets, API-compatible with the reference's src/data.py.

Names, attributes, batch composition and the order of `random` calls follow
the reference exactly (file:line cited per symbol) so that run_predictorplus
/ run_rnnlogic style drivers see identical batches.  What differs is where
the graph lives: `KnowledgeGraph.device_graph(device)` uploads a vertex-major
CSR once per GPU (rnnl_graph_create) and the PredictorPlus forward grounds
rules there with the HIP kernel instead of the dense one-hot propagation of
the reference (data.py:136-173).
"""
import itertools
import os
import random

import numpy as np
import torch
from torch.utils.data import Dataset

from . import _native


def _read_dict(path):
    e2i, i2e = {}, {}
    with open(path) as fi:
        for line in fi:
            i, name = line.strip().split("\t")
            e2i[name] = int(i)
            i2e[int(i)] = name
    return e2i, i2e


def _read_triples(path, e2i, r2i):
    out = []
    with open(path) as fi:
        for line in fi:
            h, r, t = line.strip().split("\t")
            out.append((e2i[h], r2i[r], e2i[t]))
    return out


class KnowledgeGraph(object):
    """Reference src/data.py:9-173."""

    def __init__(self, data_path):
        self.data_path = data_path
        self.entity2id, self.id2entity = _read_dict(os.path.join(data_path, "entities.dict"))
        self.relation2id, self.id2relation = _read_dict(os.path.join(data_path, "relations.dict"))
        self.entity_size = len(self.entity2id)
        self.relation_size = len(self.relation2id)

        self.train_facts = _read_triples(os.path.join(data_path, "train.txt"), self.entity2id, self.relation2id)
        self.valid_facts = _read_triples(os.path.join(data_path, "valid.txt"), self.entity2id, self.relation2id)
        self.test_facts = _read_triples(os.path.join(data_path, "test.txt"), self.entity2id, self.relation2id)

        E = self.entity_size
        self.hr2o, self.hr2oo, self.hr2ooo = dict(), dict(), dict()
        self.relation2ht2index = [dict() for _ in range(self.relation_size)]
        for h, r, t in self.train_facts:  # data.py:43-71
            k = self.encode_hr(h, r)
            self.hr2o.setdefault(k, []).append(t)
            self.hr2oo.setdefault(k, []).append(t)
            self.hr2ooo.setdefault(k, []).append(t)
            ht = self.encode_ht(h, t)
            assert ht not in self.relation2ht2index[r]
            self.relation2ht2index[r][ht] = len(self.relation2ht2index[r])
        for h, r, t in self.valid_facts:  # data.py:73-87
            k = self.encode_hr(h, r)
            self.hr2oo.setdefault(k, []).append(t)
            self.hr2ooo.setdefault(k, []).append(t)
        for h, r, t in self.test_facts:  # data.py:89-99
            self.hr2ooo.setdefault(self.encode_hr(h, r), []).append(t)

        tr = np.asarray(self.train_facts, dtype=np.int64).reshape(-1, 3)
        self._train = tr
        # relation2adjacency[r] = [LongTensor(2, E_r) rows (tail, head), ones] (data.py:101-104)
        self.relation2adjacency = []
        self.relation2outdegree = []
        for r in range(self.relation_size):
            sel = tr[tr[:, 1] == r]
            index = torch.from_numpy(np.stack([sel[:, 2], sel[:, 0]]).copy())
            self.relation2adjacency.append([index, torch.ones(index.size(1))])
            self.relation2outdegree.append(torch.from_numpy(np.bincount(sel[:, 2], minlength=E).astype(np.int64)))
        self._device_graphs = {}
        self._grounders = {}  # (r, rule body) -> one-rule HIP grounder (grounding())
        print("Data loading | DONE!")

    # data.py:110-122
    def encode_hr(self, h, r):
        return r * self.entity_size + h

    def decode_hr(self, index):
        return index % self.entity_size, index // self.entity_size

    def encode_ht(self, h, t):
        return t * self.entity_size + h

    def decode_ht(self, index):
        return index % self.entity_size, index // self.entity_size

    # ------------------------------------------------------------ device side
    def device_graph(self, device):
        """rnnl_graph handle (vertex-major CSR) on `device`, created once."""
        device = torch.device(device)
        if device.type != "cuda":
            raise RuntimeError("the HIP graph lives on a GPU; got device %s" % device)
        key = device.index if device.index is not None else torch.cuda.current_device()
        if key not in self._device_graphs:
            import ctypes
            hrt = np.ascontiguousarray(self._train, dtype=np.int32)
            h = ctypes.c_void_p()
            with torch.cuda.device(key):
                _native.call("rnnl_graph_create", hrt.ctypes.data_as(ctypes.c_void_p), len(hrt), self.entity_size,
                             self.relation_size, ctypes.byref(h))
            self._device_graphs[key] = _DeviceHandle(h, "rnnl_graph_destroy")
        return self._device_graphs[key].ptr

    # ------------------------------------------------------------ reference API
    def grounding(self, h, r, rule, edges_to_remove):
        """Path counts (B, |E|) int64 of `rule` from each h (data.py:136-147),
        row i's edge edges_to_remove[i] of relation r removed on every hop of
        relation r.

        HIP: the rule becomes a one-rule trie under head r and runs through
        the grounding kernel (rnnl_ground + COO export, the PredictorPlus
        forward's own grounding), the counts are scattered into the dense
        result.  The PredictorPlus / Predictor forwards ground all rules of a
        batch in one launch instead of calling this per rule.  No CPU path."""
        if h.device.type != "cuda":
            raise RuntimeError("KnowledgeGraph.grounding runs on the HIP path: move h to a GPU")
        r = int(r)
        rule = [int(b) for b in rule]
        h = h.to(torch.int64).contiguous()
        if not rule:  # no hop: the one-hot start vectors
            return torch.nn.functional.one_hot(h, self.entity_size)
        key = (r, tuple(rule))
        gr = self._grounders.pop(key, None)
        if gr is None:
            from .predictors import _RuleGrounder
            gr = _RuleGrounder(self, r, rule)
        self._grounders[key] = gr  # most recently used last
        while len(self._grounders) > 64:
            self._grounders.pop(next(iter(self._grounders)))
        with torch.no_grad():
            return gr.counts(h, edges_to_remove)

    def propagate(self, x, relation, edges_to_remove=None):
        """data.py:149-173 with the scatter-sum done by index_add_ (a generic
        scatter over any (|E|, B, D) tensor, on x's device; the grounding
        above and the forwards do not use it)."""
        device = x.device
        node_in = self.relation2adjacency[relation][0][1].to(device)
        node_out = self.relation2adjacency[relation][0][0].to(device)
        message = x[node_in]
        E, B, D = message.size()
        if edges_to_remove is not None:
            message = message.view(-1, D).clone()
            message[edges_to_remove * B + torch.arange(B, device=device)] = 0
            message = message.view(E, B, D)
        out = torch.zeros((x.size(0), B, D), dtype=x.dtype, device=device)
        return out.index_add_(0, node_out, message)


class _DeviceHandle(object):
    """Owns a native handle; destroyed with the Python object."""

    def __init__(self, ptr, destroy):
        self.ptr = ptr
        self._destroy = destroy

    def __del__(self):
        try:
            if self.ptr:
                getattr(_native.lib(), self._destroy)(self.ptr)
        except Exception:
            pass


class TrainDataset(Dataset):
    """Reference src/data.py:175-219."""

    def __init__(self, graph, batch_size):
        self.graph = graph
        self.batch_size = batch_size
        self.r2instances = [[] for _ in range(self.graph.relation_size)]
        for h, r, t in self.graph.train_facts:
            self.r2instances[r].append((h, r, t))
        self.make_batches()

    def make_batches(self):
        for r in range(self.graph.relation_size):
            random.shuffle(self.r2instances[r])
        self.batches = list()
        for r, instances in enumerate(self.r2instances):
            for k in range(0, len(instances), self.batch_size):
                self.batches.append(instances[k:min(k + self.batch_size, len(instances))])
        random.shuffle(self.batches)

    def __len__(self):
        return len(self.batches)

    def __getitem__(self, idx):
        data = self.batches[idx]
        all_h = torch.LongTensor([_[0] for _ in data])
        all_r = torch.LongTensor([_[1] for _ in data])
        all_t = torch.LongTensor([_[2] for _ in data])
        target = torch.zeros(len(data), self.graph.entity_size)
        edges_to_remove = []
        for k, (h, r, t) in enumerate(data):
            target[k][torch.LongTensor(self.graph.hr2o[self.graph.encode_hr(h, r)])] = 1
            edges_to_remove.append(self.graph.relation2ht2index[r][self.graph.encode_ht(h, t)])
        return all_h, all_r, all_t, target, torch.LongTensor(edges_to_remove)


class _DeviceLists(object):
    """A {key: [values]} map (hr2o / hr2oo / hr2ooo, keys r * |E| + h) laid out
    once on the device as a CSR with ascending keys — the input of
    rnnl_multi_hot / rnnl_filter_flags."""

    def __init__(self, lists, device):
        keys = np.fromiter(lists.keys(), dtype=np.int64, count=len(lists))
        order = np.argsort(keys, kind="stable")
        vals_l = list(lists.values())
        lens = np.asarray([len(vals_l[i]) for i in order], dtype=np.int64)
        offs = np.zeros(len(order) + 1, dtype=np.int64)
        np.cumsum(lens, out=offs[1:])
        vals = np.fromiter((t for i in order for t in vals_l[i]), dtype=np.int32, count=int(offs[-1]))
        self.device = device
        self.keys = torch.from_numpy(keys[order]).to(device)
        self.offs = torch.from_numpy(offs).to(device)
        self.vals = torch.from_numpy(vals).to(device)

    def rows(self, fn, row_keys, width, out):
        _native.call(fn, self.keys.data_ptr(), self.offs.data_ptr(), self.vals.data_ptr(), self.keys.numel(),
                     row_keys.data_ptr(), row_keys.numel(), width, out.data_ptr(),
                     torch.cuda.current_stream(self.device).cuda_stream)
        return out


class _RowTable(object):
    """A dataset's batches as one (n, 3) int64 (h, r, t) table on the device
    with per-batch offsets, uploaded once.  It is rebuilt when the batch list
    is another object (make_batches() builds a new list) or has another
    length, and — as a cheap guard against a reshuffle in place, which moves
    nearly every batch — when a batch object differs at one of 17 evenly
    spaced positions (checking all 17,258 FB15k-237 train batches per
    training step cost ~1 ms).  Editing the list in place otherwise (one
    batch replaced at an unchecked position) is NOT supported: assign a new
    list, or call make_batches().  The table keeps references to the list and
    the batches it was built from, so a recycled id cannot alias.  A single
    batch is then a slice of the table (no host->device copy per step) and
    many batches one gather."""

    def __init__(self, device):
        self.device = device
        self._src = None
        self._refs = ()

    def _changed(self, batches):
        n = len(batches)
        if self._src is not batches or len(self._refs) != n:
            return True
        if n == 0:
            return False
        step = max(1, n // 16)
        return any(self._refs[i] is not batches[i] for i in list(range(0, n, step)) + [n - 1])

    def get(self, batches):
        if self._changed(batches):
            lens = np.fromiter((len(b) for b in batches), dtype=np.int64, count=len(batches))
            off = np.zeros(len(batches) + 1, dtype=np.int64)
            np.cumsum(lens, out=off[1:])
            chain = itertools.chain.from_iterable
            flat = np.fromiter(chain(chain(batches)), dtype=np.int64, count=3 * int(off[-1])).reshape(-1, 3)
            self.tab = torch.from_numpy(flat).to(self.device)
            self.lens, self.off = lens, off
            self._src, self._refs = batches, tuple(batches)
        return self.tab, self.lens, self.off

    def batch(self, batches, i):
        tab, _, off = self.get(batches)
        hrt = tab[int(off[i]):int(off[i + 1])]
        return hrt[:, 0].contiguous(), hrt[:, 1].contiguous(), hrt[:, 2].contiguous()

    def rows(self, batches, indices):
        tab, lens, off = self.get(batches)
        idx = np.asarray(list(indices), dtype=np.int64)
        idx = np.where(idx < 0, idx + len(lens), idx)  # Python indexing; `off` has one more entry
        if idx.size and (idx.min() < 0 or idx.max() >= len(lens)):
            raise IndexError("batch index out of range")
        n = lens[idx]
        # positions of the selected batches' rows, in the order of `indices`
        sel = np.repeat(off[idx] - (np.cumsum(n) - n), n) + np.arange(int(n.sum()), dtype=np.int64)
        hrt = tab[torch.from_numpy(sel).to(self.device, non_blocking=True)]
        return hrt[:, 0].contiguous(), hrt[:, 1].contiguous(), hrt[:, 2].contiguous()


class DeviceTrainBatches(object):
    """TrainDataset rows built on the device: item `idx`
    equals `train_set[idx]` — (all_h, all_r, all_t, target, edges_to_remove),
    reference src/data.py:201-219 — as tensors on `device`.  The dense
    multi-hot target comes from rnnl_multi_hot over a CSR of hr2o (keys
    r * |E| + h, built once); the row's own relation-local edge id
    (relation2ht2index) from a sorted key table of all train edges.  Follows
    `train_set.batches` (a device table of its rows, rebuilt when
    make_batches() reshuffles them)."""

    def __init__(self, train_set, device):
        self.train_set = train_set
        self.device = torch.device(device)
        g = train_set.graph
        E = g.entity_size
        self.hr2o = _DeviceLists(g.hr2o, self.device)
        # relation-local edge ids: key (r * |E| + t) * |E| + h -> id, sorted
        ek, ev = [], []
        for r, m in enumerate(g.relation2ht2index):
            if m:
                ht = np.fromiter(m.keys(), dtype=np.int64, count=len(m))
                ek.append(r * E * E + ht)
                ev.append(np.fromiter(m.values(), dtype=np.int64, count=len(m)))
        ek = np.concatenate(ek) if ek else np.zeros(0, np.int64)
        ev = np.concatenate(ev) if ev else np.zeros(0, np.int64)
        o = np.argsort(ek, kind="stable")
        self.edge_keys = torch.from_numpy(ek[o]).to(self.device)
        self.edge_ids = torch.from_numpy(ev[o]).to(self.device)
        self.table = _RowTable(self.device)

    def __len__(self):
        return len(self.train_set)

    @_native.on_self_device
    def __getitem__(self, idx):
        E = self.train_set.graph.entity_size
        tab, lens, off = self.table.get(self.train_set.batches)
        n = len(lens)
        idx = int(idx)
        if idx < 0:  # Python indexing, as train_set[idx]; `off` has n + 1 entries
            idx += n
        if not 0 <= idx < n:
            raise IndexError("DeviceTrainBatches index out of range")
        B = int(lens[idx])
        out = torch.empty((4, B), dtype=torch.int64, device=self.device)  # h, r, t, edges_to_remove
        target = torch.empty((B, E), dtype=torch.float32, device=self.device)
        L = self.hr2o
        _native.call("rnnl_train_batch", tab.data_ptr(), int(off[idx]), B, L.keys.data_ptr(), L.offs.data_ptr(),
                     L.vals.data_ptr(), L.keys.numel(), self.edge_keys.data_ptr(), self.edge_ids.data_ptr(),
                     self.edge_keys.numel(), E, out[0].data_ptr(), out[1].data_ptr(), out[2].data_ptr(),
                     out[3].data_ptr(), target.data_ptr(), torch.cuda.current_stream(self.device).cuda_stream)
        return out[0], out[1], out[2], target, out[3]

    @_native.on_self_device
    def rows(self, idx):
        """(all_h, all_r, all_t, edges_to_remove) of many batches at once
        (their concatenation, in `idx` order), without the dense targets."""
        g = self.train_set.graph
        E = g.entity_size
        all_h, all_r, all_t = self.table.rows(self.train_set.batches, idx)
        ekey = (all_r * E + all_t) * E + all_h
        pos = torch.searchsorted(self.edge_keys, ekey).clamp(max=max(self.edge_keys.numel() - 1, 0))
        return all_h, all_r, all_t, self.edge_ids[pos]


class DeviceEvalBatches(object):
    """ValidDataset / TestDataset rows built on the device:
    item `idx` equals `eval_set[idx]` — (all_h, all_r, all_t, flag), reference
    src/data.py:250-255 / 287-291 — with the filter row from
    rnnl_filter_flags over a CSR of hr2oo / hr2ooo.  `rows(indices)` gives
    the concatenation of many batches with one launch."""

    def __init__(self, eval_set, device):
        self.eval_set = eval_set
        self.device = torch.device(device)
        self.lists = _DeviceLists(getattr(eval_set.graph, eval_set.filter_attr), self.device)
        self.table = _RowTable(self.device)  # the split's rows, gathered per call

    def __len__(self):
        return len(self.eval_set)

    @_native.on_self_device
    def rows(self, indices):
        E = self.eval_set.graph.entity_size
        all_h, all_r, all_t = self.table.rows(self.eval_set.batches, indices)
        flag = torch.empty((all_h.numel(), E), dtype=torch.bool, device=self.device)
        if all_h.numel():
            self.lists.rows("rnnl_filter_flags", (all_r * E + all_h).contiguous(), E, flag.view(torch.uint8))
        return all_h, all_r, all_t, flag

    def __getitem__(self, idx):
        return self.rows([idx])


class _EvalDataset(Dataset):
    facts_attr = None
    filter_attr = None

    def __init__(self, graph, batch_size):
        self.graph = graph
        self.batch_size = batch_size
        r2instances = [[] for _ in range(self.graph.relation_size)]
        for h, r, t in getattr(self.graph, self.facts_attr):
            r2instances[r].append((h, r, t))
        self.batches = list()
        for r, instances in enumerate(r2instances):
            random.shuffle(instances)
            for k in range(0, len(instances), self.batch_size):
                self.batches.append(instances[k:min(k + self.batch_size, len(instances))])

    def __len__(self):
        return len(self.batches)

    def __getitem__(self, idx):
        data = self.batches[idx]
        all_h = torch.LongTensor([_[0] for _ in data])
        all_r = torch.LongTensor([_[1] for _ in data])
        all_t = torch.LongTensor([_[2] for _ in data])
        mask = torch.ones(len(data), self.graph.entity_size).bool()
        filt = getattr(self.graph, self.filter_attr)
        for k, (h, r, t) in enumerate(data):
            mask[k][torch.LongTensor(filt[self.graph.encode_hr(h, r)])] = 0
        return all_h, all_r, all_t, mask


class ValidDataset(_EvalDataset):
    """Reference src/data.py:221-256 (filter: train+valid answers)."""
    facts_attr, filter_attr = "valid_facts", "hr2oo"


class TestDataset(_EvalDataset):
    """Reference src/data.py:258-293 (filter: train+valid+test answers)."""
    facts_attr, filter_attr = "test_facts", "hr2ooo"


class RuleDataset(Dataset):
    """Rule sequences for the LSTM generator (reference src/data.py:295-342).

    Item k is ([head, body..., END], PAD, weight + 1e-5) with END = |R| and
    PAD = |R| + 1; a rule file holds "head body... H" lines, H scaled by 1000.
    Generator side: kept for the EM driver, not on the accelerated path."""

    def __init__(self, num_relations, input):
        self.num_relations = num_relations
        self.ending_idx = num_relations
        self.padding_idx = num_relations + 1
        if isinstance(input, str):
            with open(input, "r") as fi:
                toks = [line.split() for line in fi]
            rules = [[int(x) for x in t[:-1]] + [float(t[-1]) * 1000] for t in toks]
        elif isinstance(input, list):
            rules = input
        else:
            raise ValueError
        self.rules = [[list(x[:-1]) + [self.ending_idx], self.padding_idx, x[-1] + 1e-5] for x in rules]

    def __len__(self):
        return len(self.rules)

    def __getitem__(self, idx):
        return self.rules[idx]

    @staticmethod
    def collate_fn(data):
        seqs = [item[0] for item in data]
        pads = torch.tensor([int(item[-2]) for item in data], dtype=torch.long)
        L = max(len(s) for s in seqs) - 1
        inputs = pads.unsqueeze(1).repeat(1, L)
        target = pads.unsqueeze(1).repeat(1, L)
        for k, s in enumerate(seqs):
            inputs[k, :len(s) - 1] = torch.tensor(s[:-1], dtype=torch.long)
            target[k, :len(s) - 1] = torch.tensor(s[1:], dtype=torch.long)
        weight = torch.tensor([float(item[-1]) for item in data])
        return inputs, target, target != pads.unsqueeze(1), weight


def Iterator(dataloader):
    """Endless iteration over a DataLoader (reference src/data.py:344-347)."""
    while True:
        yield from dataloader
