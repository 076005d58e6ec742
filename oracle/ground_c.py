"""TEST INFRASTRUCTURE ONLY — ctypes front-end of oracle/ground_oracle.c and of
the reference-miner shim oracle/_ref/libref_miner.so.

Builds its own vertex-major CSR from the train triples with NumPy (independent
of the product's builder in rnnlogic_amd/), so a layout bug in the product
cannot hide behind a shared helper.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "libground_oracle.so")
REF_LIB = os.path.join(HERE, "_ref", "libref_miner.so")

_P = ctypes.c_void_p


def build():
    subprocess.run(["make", "-s", "-C", HERE, "oracle"], check=True)
    if os.path.isdir("/root/reference/miner"):
        subprocess.run(["make", "-s", "-C", HERE, "ref"], check=True)


def _lib():
    if not os.path.exists(LIB):
        build()
    lib = ctypes.CDLL(LIB)
    lib.oracle_digests.restype = ctypes.c_int
    lib.oracle_query_candidates.restype = ctypes.c_int
    lib.oracle_query_stats.restype = ctypes.c_int
    lib.oracle_mix64.restype = ctypes.c_uint64
    lib.oracle_mix64.argtypes = [ctypes.c_uint64]
    return lib


def _ptr(a):
    return a.ctypes.data_as(_P) if a is not None else None


class CGraph:
    """Vertex-major CSR (edges of (v, rel) contiguous, file order inside)."""

    def __init__(self, n_entities, n_relations, train):
        train = np.asarray(train, dtype=np.int64).reshape(-1, 3)
        E, R = int(n_entities), int(n_relations)
        key = train[:, 0] * R + train[:, 1]
        order = np.argsort(key, kind="stable")
        self.col = train[order, 2].astype(np.int32)
        counts = np.bincount(key, minlength=E * R)
        self.off = np.zeros(E * R + 1, np.int64)
        np.cumsum(counts, out=self.off[1:])
        self.E, self.R = E, R


class CRules:
    """Rules grouped by head in file order; returns global rule ids."""

    def __init__(self, rules, n_relations):
        heads = np.asarray([hd for hd, _ in rules], dtype=np.int64)
        self.order = np.argsort(heads, kind="stable")  # file order inside each head
        self.rh_ptr = np.zeros(n_relations + 1, np.int32)
        np.cumsum(np.bincount(heads, minlength=n_relations), out=self.rh_ptr[1:])
        # ids must be global rule ids: keep rules in head-sorted order but remember ids
        bodies = [rules[i][1] for i in self.order]
        self.bptr = np.zeros(len(rules) + 1, np.int32)
        np.cumsum([len(b) for b in bodies], out=self.bptr[1:])
        self.body = np.asarray([x for b in bodies for x in b] or [0], dtype=np.int32)
        self.ids = self.order.astype(np.int32)


def mix64(x):
    return int(_lib().oracle_mix64(ctypes.c_uint64(int(x) & 0xFFFFFFFFFFFFFFFF)))


class Oracle:
    def __init__(self, cgraph, rules, n_relations):
        self.g = cgraph
        self.rules = CRules(rules, n_relations)
        self.lib = _lib()

    def _args(self):
        g, r = self.g, self.rules
        return [_ptr(g.off), _ptr(g.col), ctypes.c_int(g.R), ctypes.c_int(g.E), _ptr(r.rh_ptr), _ptr(r.bptr),
                _ptr(r.body), _ptr(r.ids)]

    def candidates(self, h, r, rm_src=-1, rm_dst=-1):
        """Sorted candidates of one query: (t, sum of counts, rule fingerprint)."""
        cap = self.g.E
        t = np.empty(cap, np.int32)
        s = np.empty(cap, np.int64)
        f = np.empty(cap, np.uint64)
        n = self.lib.oracle_query_candidates(*self._args(), int(h), int(r), int(rm_src), int(rm_dst), _ptr(t),
                                             _ptr(s), _ptr(f), ctypes.c_int(cap))
        assert n >= 0
        return t[:n], s[:n], f[:n]

    def digests(self, h, r, rm_src=None, rm_dst=None, threads=None, work=False):
        h = np.ascontiguousarray(h, dtype=np.int32)
        r = np.ascontiguousarray(r, dtype=np.int32)
        rs = np.ascontiguousarray(rm_src, dtype=np.int32) if rm_src is not None else None
        rd = np.ascontiguousarray(rm_dst, dtype=np.int32) if rm_dst is not None else None
        n = len(h)
        d = np.zeros(n, np.uint64)
        c = np.zeros(n, np.int32)
        w = np.zeros((n, 3), np.int64) if work else None
        rc = self.lib.oracle_digests(*self._args(), _ptr(h), _ptr(r), _ptr(rs), _ptr(rd), ctypes.c_int(n),
                                     ctypes.c_int(threads or os.cpu_count() or 1), _ptr(d), _ptr(c), _ptr(w))
        assert rc == 0
        return (d, c, w) if work else (d, c)


    def query_stats(self, h, r, t, rm_src=None, rm_dst=None, weights=None, threads=None):
        """The EM Predictor's integer work per query (oracle_query_stats):
        returns (rq_ptr (n+1,), pos, tot) — for query q and the k-th rule of
        its relation (file order), pos[rq_ptr[q] + k] = paths h -> t and
        tot[...] = paths h -> any entity — and, with `weights` (per global
        rule id), also (cand_ptr (n+1,), cand (entity, sorted per query),
        score = sum_rho count_rho * w_rho in float64)."""
        h = np.ascontiguousarray(h, dtype=np.int32)
        r = np.ascontiguousarray(r, dtype=np.int32)
        t = np.ascontiguousarray(t, dtype=np.int32)
        rs = np.ascontiguousarray(rm_src, dtype=np.int32) if rm_src is not None else None
        rd = np.ascontiguousarray(rm_dst, dtype=np.int32) if rm_dst is not None else None
        n = len(h)
        nrq = np.diff(self.rules.rh_ptr).astype(np.int64)[r]
        rq_ptr = np.zeros(n + 1, np.int64)
        np.cumsum(nrq, out=rq_ptr[1:])
        pos = np.zeros(max(int(rq_ptr[-1]), 1), np.int64)
        tot = np.zeros_like(pos)
        threads = threads or os.cpu_count() or 1
        cand_ptr = out_t = out_s = w = None
        if weights is not None:
            _, nc = self.digests(h, r, rs, rd, threads=threads)
            cand_ptr = np.zeros(n + 1, np.int64)
            np.cumsum(nc.astype(np.int64), out=cand_ptr[1:])
            out_t = np.zeros(max(int(cand_ptr[-1]), 1), np.int32)
            out_s = np.zeros(len(out_t), np.float64)
            w = np.ascontiguousarray(weights, dtype=np.float64)
        rc = self.lib.oracle_query_stats(*self._args(), _ptr(h), _ptr(r), _ptr(rs), _ptr(rd), _ptr(t), ctypes.c_int(n),
                                         ctypes.c_int(threads), _ptr(w), _ptr(rq_ptr), _ptr(pos), _ptr(tot),
                                         _ptr(cand_ptr), _ptr(out_t), _ptr(out_s))
        assert rc == 0
        if weights is None:
            return rq_ptr, pos, tot
        return rq_ptr, pos, tot, cand_ptr, out_t[:cand_ptr[-1]], out_s[:cand_ptr[-1]]


class RefMiner:
    """The reference's own C++ path counter (miner/rnnlogic.cpp), via oracle/_ref."""

    def __init__(self, data_path):
        if not os.path.exists(REF_LIB):
            build()
        self.lib = ctypes.CDLL(REF_LIB)
        self.lib.ref_kg_load.restype = _P
        self.lib.ref_out_test_timed.restype = ctypes.c_double
        import sys
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            self.kg = self.lib.ref_kg_load(data_path.encode())
        finally:
            os.dup2(saved, 1)
            os.close(saved)

    def rule_destination(self, e, body, rm=(-1, -1, -1), cap=1 << 20):
        b = np.asarray(body, dtype=np.int32)
        d = np.empty(cap, np.int32)
        c = np.empty(cap, np.int32)
        n = self.lib.ref_rule_destination(_P(self.kg), int(e), _ptr(b), len(b), int(rm[0]), int(rm[1]),
                                          int(rm[2]), _ptr(d), _ptr(c), cap)
        assert n >= 0
        return d[:n], c[:n]

    def out_test_timed(self, rules, threads, sample):
        flat = []
        for hd, body in rules:
            flat += [hd, len(body)] + list(body)
        f = np.asarray(flat, dtype=np.int32)
        n = ctypes.c_longlong(0)
        # the miner prints progress on stdout: send it to stderr for the call
        import sys
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            sec = self.lib.ref_out_test_timed(_P(self.kg), _ptr(f), len(rules), int(threads), int(sample),
                                              ctypes.byref(n))
        finally:
            os.dup2(saved, 1)
            os.close(saved)
        return sec, n.value

    def rule_search(self, max_length, threads=1, cap=1 << 26):
        """RuleMiner::search (rnnlogic.cpp:505-589) over all train triples:
        (rules [(head, body tuple)] in the reference's order, seconds)."""
        out = np.empty(cap, np.int32)
        sec = ctypes.c_double(0.0)
        self.lib.ref_rule_search.restype = ctypes.c_longlong
        import sys
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            n = self.lib.ref_rule_search(_P(self.kg), int(max_length), int(threads), _ptr(out),
                                         ctypes.c_longlong(cap), ctypes.byref(sec))
        finally:
            os.dup2(saved, 1)
            os.close(saved)
        assert n >= 0, "cap too small"
        rules, k = [], 0
        while k < n:
            hd, ln = int(out[k]), int(out[k + 1])
            rules.append((hd, tuple(int(x) for x in out[k + 2:k + 2 + ln])))
            k += 2 + ln
        return rules, sec.value

    def close(self):
        self.lib.ref_kg_free(_P(self.kg))
