"""CPU checks of the rank-parity accounting (tests/rank_parity.py) on
synthetic scores: a perturbation of at most eps moves each row's (L, H)
only within its 2-eps window, the exact accounting reproduces every move it
claims, and |dMRR| stays within the per-row bound, which is checked against
a brute-force maximum over the window."""
import numpy as np

import rank_parity

WINDOWS = np.asarray((0.0, 1e-6, 2e-6, 5e-6, 1e-5, 2e-5, 5e-5, 1e-4), np.float64)


def _bounds(s, t, flag):
    val = s[t]
    c = s[flag]
    return int((c > val).sum()) + 1, int((c >= val).sum()) + 2


def _records(ref, flags, tgt, rng, nclose=12, nrand=4):
    n, E = ref.shape
    rows, near_w, pe, ps = [], [], [], []
    for k in range(n):
        t = tgt[k]
        L, H = _bounds(ref[k], t, flags[k])
        d = np.abs(ref[k][flags[k]].astype(np.float64) - float(ref[k, t]))
        near_w.append([int((d <= w).sum()) for w in WINDOWS])
        ids = np.nonzero(flags[k])[0]
        close = ids[np.argsort(d, kind="stable")[:nclose]]
        e = np.full(nclose + nrand, -1, np.int64)
        e[:len(close)] = close
        e[nclose:] = rng.randint(0, E, nrand)
        pe.append(e)
        ps.append(np.where(e >= 0, ref[k][np.maximum(e, 0)], np.nan))
        rows.append((k, 0, t, L, H))
    return np.asarray(rows, np.int64), np.asarray(near_w), np.asarray(pe), np.asarray(ps, np.float64)


def test_rank_parity_accounting_on_perturbed_scores():
    rng = np.random.RandomState(0)
    n, E = 400, 300
    # coarse scores: many exact ties and near-ties around each target
    ref = (rng.randint(0, 2000, size=(n, E)) * 1e-6).astype(np.float32)
    flags = rng.rand(n, E) < 0.9
    tgt = rng.randint(0, E, n)
    flags[np.arange(n), tgt] = True
    want, near_w, pe, ps = _records(ref, flags, tgt, rng)
    eps = 4e-6
    hip = (ref.astype(np.float64) + rng.uniform(-eps, eps, size=ref.shape)).astype(np.float32)
    LH = np.asarray([_bounds(hip[k], tgt[k], flags[k]) for k in range(n)])
    hip_p = np.where(pe >= 0, hip[np.arange(n)[:, None], np.maximum(pe, 0)], np.nan).astype(np.float64)
    hip_t = hip[np.arange(n), tgt].astype(np.float64)
    ref_t = ref[np.arange(n), tgt].astype(np.float64)
    ptr = np.arange(0, n + 1, 32)
    ptr[-1] = n
    rep = rank_parity.check(want, LH[:, 0], LH[:, 1], hip_t, np.nan_to_num(hip_p), np.ones(n, bool), ref_t,
                            np.nan_to_num(ps), pe, near_w, WINDOWS, ptr, eps_max=1e-5)
    assert rep["moved"] > 0 and rep["exact"] > 0
    # the observed change equals the metric's
    harm = rank_parity.harmonic(E + 10)
    d = rank_parity.rr(LH[:, 0], LH[:, 1], harm) - rank_parity.rr(want[:, 3], want[:, 4], harm)
    assert abs(d.sum() / n - rep["d_mrr"]) <= 1e-15
    assert abs(rep["d_mrr"]) <= rep["mrr_bound"]


def test_window_bound_is_the_brute_force_maximum():
    harm = rank_parity.harmonic(200)
    for L, H, a in ((1, 2, 3), (5, 9, 2), (2, 40, 7), (17, 18, 1)):
        best = 0.0
        for L2 in range(max(1, L - a), L + a + 1):
            for H2 in range(max(L2 + 1, H - a), H + a + 1):
                best = max(best, abs(rank_parity.rr(L2, H2, harm) - rank_parity.rr(L, H, harm)))
        lo = max(1, L - a)
        up = rank_parity.rr(lo, max(lo + 1, H - a), harm) - rank_parity.rr(L, H, harm)
        down = rank_parity.rr(L, H, harm) - rank_parity.rr(L + a, H + a, harm)
        assert abs(max(up, down) - best) <= 1e-15, (L, H, a, max(up, down), best)
