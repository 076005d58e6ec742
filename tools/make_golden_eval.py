"""Per-query reference ranks for evaluate() parity (SURVEY §8c vector (5)/(a14)).

Runs the *reference* PredictorPlus (imported from /root/reference/src with the
test-only shims, exactly as tools/make_golden.py does) over the test split of a
case and records, per query row, the reference's filtered rank bounds
(trainer.py:191-203):

    L = #(flagged scores > s_t) + 1,  H = #(flagged scores >= s_t) + 2
    (or L = 1, H = |E| + 1 when t is not a candidate)

plus s_t and `near`, the number of flagged competitors whose score lies within
`TOL` = 1e-4 of s_t.  So that the test can hold a rank difference to the score
error it actually measures (not to a fixed 1e-4 window), each row also has:
  near_w (n, len(WINDOWS))  flagged competitors with |s_e - s_t| <= w for each
                            w in WINDOWS (w = 0: exact ties);
  probe_ent / probe_score   (n, NPROBE) entities and reference scores: the
                            NCLOSE flagged competitors closest to s_t (ties
                            first) and NRAND seeded random entities, -1 / nan
                            padded — where the HIP score error is measured, and
                            an exact flip count for rows whose window holds no
                            more competitors than the probes.
The metrics of the reference's own formula over these rows (world size 1, no
sampler padding) are stored beside them.  Weights are the seeded state_dict of
the same case in tests/golden/<case>.npz (checked equal here).

RotatE cases: the reference's RotatE.forward (embedding.py:64-70) evaluates
project() and product() once per (query, entity) pair — 3.5 s per query at
D = 1000 on FB15k-237 here.  With --rotate-rows the forward is evaluated row
by row: the reference's project() / product() once per row on its (h, r)
(the per-pair values are that row's, repeated), the difference to every
entity, diff()'s norm of the (re, im) pair taken over a trailing size-2 axis
instead of a leading one (10x faster; the same torch norm of the same two
values), the sum over dims, and gamma minus that.  Before use, this is checked
to equal the unpatched forward bitwise on the first CHECK_ROWS rows.
`--verify` re-runs the whole unpatched reference model (rules part and
RotatE.forward as shipped) on test batch 0 and on the first batch of another
relation (64 rows at B = 32), requires every stored record of those rows —
(L, H), s_t, the windows' counts, the probe entities and their scores — to be
bitwise what the unpatched reference gives, and records the verified batches
and rows in the fixture (`rotate_verified_batches`, `rotate_verified_rows`).

Output: tests/golden/eval_<case>.npz.  Long runs: FB15k-237 full test split
(40,932 rows) takes ~25 min on 8 cores; rows are split over worker processes.

Usage: python tools/make_golden_eval.py <case> [--batches N] [--workers W] [--rotate-rows] [--verify]
"""
import argparse
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as MG  # noqa: E402  (sets up the reference import path + shims)

import torch  # noqa: E402

TOL = 1e-4
WINDOWS = (0.0, 1e-6, 2e-6, 5e-6, 1e-5, 2e-5, 5e-5, 1e-4)
# NCLOSE: --nclose (passed to the spawned workers through the environment)
NCLOSE, NRAND = int(os.environ.get("RNNL_GOLDEN_NCLOSE", "12")), 4
NPROBE = NCLOSE + NRAND
_STATE = {}


def _build(name):
    spec = MG.CASES[name]
    dpath = MG.datasets.materialize(spec["data"])
    rules = MG.datasets.rule_file(spec["data"])
    kw = dict(type="lstm", num_layers=3, hidden_dim=16, entity_feature="bias", aggregator="sum", embedding_path=None)
    kw.update(spec["model"])
    if kw.get("embedding_path"):
        kw["embedding_path"] = MG._rotate_dir(spec["data"], kw["embedding_path"])
    MG.R_utils.set_seed(1)
    graph = MG.R_data.KnowledgeGraph(dpath)
    MG.R_data.TrainDataset(graph, 32)
    MG.R_data.ValidDataset(graph, 32)
    test_set = MG.R_data.TestDataset(graph, 32)
    model = MG.R_pred.PredictorPlus(graph, **kw)
    model.set_rules(rules)
    model.eval()
    return graph, test_set, model


CHECK_ROWS = 32  # one full reference batch (3 before round 5; --verify covers 64 rows)


def _rotate_rows(rot):
    """The reference RotatE.forward(all_h, all_r) evaluated row by row with
    the reference's own product / project / diff (see the module docstring)."""
    def forward(all_h, all_r):
        out = []
        for b in range(all_h.numel()):
            h_emb = rot.eemb.index_select(0, all_h[b:b + 1])
            r_emb = rot.project(rot.remb.index_select(0, all_r[b:b + 1]))
            e_emb = rot.product(h_emb, r_emb)
            re_d, im_d = torch.chunk(e_emb - rot.eemb, 2, dim=-1)
            dist = torch.stack([re_d, im_d], dim=-1).norm(dim=-1).sum(dim=-1)
            out.append(rot.gamma - dist)
        return torch.stack(out)
    return forward


def batch_records(score, mask, all_h, all_r, all_t, flag, E, rng, windows=WINDOWS):
    """Per row of one batch: (h, r, t, L, H, near, s_t, near_w, probe_ent,
    probe_score) from the reference's scores and mask (see the module doc)."""
    out = []
    for k in range(all_t.numel()):
        t = int(all_t[k])
        pe = np.full(NPROBE, -1, np.int64)
        ps = np.full(NPROBE, np.nan, np.float32)
        nw = np.zeros(len(windows), np.int64)
        if bool(mask[k, t]):
            val = score[k, t]
            fl = flag[k]
            s = score[k][fl]
            L = int((s > val).sum()) + 1
            H = int((s >= val).sum()) + 2
            near = int(((s - val).abs() <= TOL).sum())
            st = float(val)
            d = (s - val).abs().double().numpy()
            nw[:] = [int((d <= w).sum()) for w in windows]
            ids = torch.nonzero(fl).squeeze(1).numpy()
            close = ids[np.argsort(d, kind="stable")[:NCLOSE]]
            pe[:len(close)] = close
        else:
            L, H, near, st = 1, E + 1, 0, float("nan")
        pe[NCLOSE:] = rng.randint(0, E, NRAND)
        ok = pe >= 0
        ps[ok] = score[k][torch.from_numpy(pe[ok])].numpy()
        out.append((int(all_h[k]), int(all_r[k]), t, L, H, near, st, nw, pe, ps))
    return out


def _ranks_of_batch(i):
    graph, test_set, model = _STATE["g"], _STATE["t"], _STATE["m"]
    all_h, all_r, all_t, flag = test_set[i]
    with torch.no_grad():
        score, mask = model(all_h, all_r, None)
    return i, batch_records(score, mask, all_h, all_r, all_t, flag, graph.entity_size, np.random.RandomState(1000 + i))


def _init_worker(case, rotate_rows):
    graph, test_set, model = _build(case)
    if rotate_rows:
        model.RotatE.forward = _rotate_rows(model.RotatE)
    _STATE.update(g=graph, t=test_set, m=model)


def _cached(cache, i):
    """Rows of batch i from a resumable per-batch cache (None if absent)."""
    if not cache:
        return None
    f = os.path.join(cache, "b%05d.npz" % i)
    if not os.path.exists(f):
        return None
    z = np.load(f)
    return i, [(int(a[0]), int(a[1]), int(a[2]), int(a[3]), int(a[4]), int(a[5]), np.float32(s), nw, pe, ps)
               for a, s, nw, pe, ps in zip(z["a"], z["s"], z["nw"], z["pe"], z["ps"])]


def _store(cache, i, out):
    if not cache:
        return
    rows = out[1]
    tmp = os.path.join(cache, "b%05d.tmp.npz" % i)
    np.savez(tmp, a=np.asarray([r[:6] for r in rows], np.int64), s=np.asarray([r[6] for r in rows], np.float32),
             nw=np.stack([r[7] for r in rows]), pe=np.stack([r[8] for r in rows]), ps=np.stack([r[9] for r in rows]))
    os.replace(tmp, os.path.join(cache, "b%05d.npz" % i))


def _worker(args):
    idx, threads, cache = args
    torch.set_num_threads(threads)
    res = []
    t0 = time.time()
    for j, i in enumerate(idx):
        got = _cached(cache, i)
        if got is None:
            got = _ranks_of_batch(i)
            _store(cache, i, got)
        res.append(got)
        if j % 50 == 0:
            print("  worker %d: %d/%d batches, %.0f s" % (os.getpid(), j, len(idx), time.time() - t0), flush=True)
    return res


def metrics(rows, expectation=True):
    """The reference formula (trainer.py:207-238) over [h, r, t, L, H] rows."""
    q = {}
    for h, r, t, L, H in rows:
        q[(h, r, t)] = (L, H)
    hit1 = hit3 = hit10 = mr = mrr = 0.0
    for L, H in q.values():
        for rank in range(L, H):
            w = 1.0 / (H - L)
            hit1 += w if rank <= 1 else 0.0
            hit3 += w if rank <= 3 else 0.0
            hit10 += w if rank <= 10 else 0.0
            mr += rank * w
            mrr += w / rank
    n = len(rows)
    return dict(Hit1=hit1 / n, Hit3=hit3 / n, Hit10=hit10 / n, MR=mr / n, MRR=mrr / n)


def verify(case, path):
    """--verify: the unpatched reference on two batches of two relations
    against the stored rows (see the module docstring); adds the verified
    batch / row lists to the fixture at `path`."""
    graph, test_set, model = _build(case)
    z = dict(np.load(path))
    ptr = z["batch_ptr"]
    r0 = int(test_set[0][1][0])
    other = next(i for i in range(1, len(test_set)) if int(test_set[i][1][0]) != r0)
    done = []
    for i in (0, other):
        t0 = time.time()
        _, got = _ranks_of_batch_with(graph, test_set, model, i)
        lo, hi = int(ptr[i]), int(ptr[i + 1])
        assert len(got) == hi - lo
        for k, row in enumerate(got):
            j = lo + k
            assert tuple(row[:6]) == tuple(int(x) for x in z["rows"][j]), (i, k, row[:6], z["rows"][j])
            assert np.float32(row[6]).tobytes() == np.float32(z["s_t"][j]).tobytes(), (i, k)
            assert np.array_equal(row[7], z["near_w"][j]), (i, k)
            assert np.array_equal(row[8].astype(np.int32), z["probe_ent"][j]), (i, k)
            assert np.array_equal(row[9].view(np.uint32), np.asarray(z["probe_score"][j], np.float32).view(np.uint32)), (i, k)
        done.append((i, lo, hi))
        print("batch %d (relation %d, rows %d..%d): unpatched reference == stored rows bitwise (%.0f s)" % (
            i, int(test_set[i][1][0]), lo, hi, time.time() - t0), flush=True)
    z["rotate_verified_batches"] = np.asarray([d[0] for d in done], np.int64)
    z["rotate_verified_rows"] = np.concatenate([np.arange(d[1], d[2]) for d in done]).astype(np.int64)
    np.savez_compressed(path, **z)
    print("%s: %d rows verified against the unpatched reference -> %s" % (case, len(z["rotate_verified_rows"]), path))


def _ranks_of_batch_with(graph, test_set, model, i):
    _STATE.update(g=graph, t=test_set, m=model)
    return _ranks_of_batch(i)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("case")
    ap.add_argument("--batches", type=int, default=0, help="prefix of test batches (0 = all)")
    ap.add_argument("--workers", type=int, default=4)
    ap.add_argument("--threads", type=int, default=2)
    ap.add_argument("--rotate-rows", action="store_true", help="row-wise RotatE from the reference's methods")
    ap.add_argument("--cache", default="", help="directory of per-batch results (resumable long runs)")
    ap.add_argument("--out", default="", help="output path (default tests/golden/eval_<case>.npz)")
    ap.add_argument("--nclose", type=int, default=NCLOSE,
                    help="closest flagged competitors kept as probes (more: more rows accounted exactly)")
    ap.add_argument("--verify", action="store_true",
                    help="check an existing fixture's rows against the unpatched reference on two batches")
    a = ap.parse_args()
    if a.verify:
        verify(a.case, a.out or os.path.join(MG.OUT, "eval_%s.npz" % a.case))
        return
    if a.nclose != NCLOSE:  # the module constant of this process and of the workers it spawns
        os.environ["RNNL_GOLDEN_NCLOSE"] = str(a.nclose)
        globals().update(NCLOSE=a.nclose, NPROBE=a.nclose + NRAND)
    if a.cache:
        os.makedirs(a.cache, exist_ok=True)
    graph, test_set, model = _build(a.case)
    if a.rotate_rows:
        rot = model.RotatE
        h, r = test_set[0][0][:CHECK_ROWS], test_set[0][1][:CHECK_ROWS]
        t0 = time.time()
        with torch.no_grad():
            want = rot(h, r)
            got = _rotate_rows(rot)(h, r)
        assert torch.equal(want, got), float((want - got).abs().max())
        print("row-wise RotatE == reference RotatE.forward bitwise on %d rows (%.0f s)" % (CHECK_ROWS,
                                                                                          time.time() - t0))
        rot.forward = _rotate_rows(rot)
    fx = np.load(os.path.join(MG.OUT, a.case + ".npz"))
    for k, v in model.state_dict().items():
        if "sd/" + k in fx.files:
            assert np.array_equal(v.detach().numpy(), fx["sd/" + k]), k
    _STATE.update(g=graph, t=test_set, m=model)
    nb = len(test_set) if a.batches <= 0 else min(a.batches, len(test_set))
    order = list(range(nb))
    chunks = [order[w::a.workers] for w in range(a.workers)]
    t0 = time.time()
    import multiprocessing as mp
    if a.workers == 1:
        parts = [_worker((order, a.threads, a.cache))]
    else:
        # spawn: the parent has run torch ops (an OpenMP pool does not survive fork)
        with mp.get_context("spawn").Pool(a.workers, _init_worker, (a.case, a.rotate_rows)) as pool:
            parts = pool.map(_worker, [(c, a.threads, a.cache) for c in chunks])
    res = dict(x for p in parts for x in p)
    rows = [row for i in range(nb) for row in res[i]]
    arr = np.asarray([r[:6] for r in rows], dtype=np.int64)
    st = np.asarray([r[6] for r in rows], dtype=np.float32)
    m = metrics(arr[:, :5].tolist())
    out = dict(batches=np.int64(nb), rows=arr, s_t=st, tol=np.float64(TOL),
               batch_ptr=np.cumsum([0] + [len(res[i]) for i in range(nb)]).astype(np.int64),
               windows=np.asarray(WINDOWS, np.float64), near_w=np.stack([r[7] for r in rows]),
               probe_ent=np.stack([r[8] for r in rows]).astype(np.int32),
               probe_score=np.stack([r[9] for r in rows]))
    for k, v in m.items():
        out["metric/" + k] = np.float64(v)
    path = a.out or os.path.join(MG.OUT, "eval_%s.npz" % a.case)
    np.savez_compressed(path, **out)
    print("%s: %d batches, %d rows in %.0f s -> %s (%d B); MRR %.6f, rows with near-ties %d" % (
        a.case, nb, len(rows), time.time() - t0, path, os.path.getsize(path), m["MRR"], int((arr[:, 5] > 0).sum())))


if __name__ == "__main__":
    main()
