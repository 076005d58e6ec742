"""Per-query rank parity held to the measured score error (shared by
tests/test_gpu_eval.py and tests/test_gpu_flow.py).

A fixture row (tools/make_golden_eval.py `row_record`) holds the reference's
filtered rank bounds (L, H) (trainer.py:191-203), the number of flagged
competitors within each stored window of the target's score (`near_w`), and
probe entities with their reference scores (the NCLOSE flagged competitors
closest to the target, then random entities).  Given the HIP scores at the
targets and probes:

* eps per reference batch = max |HIP - reference| over its targets and probes;
* a competitor can change sides only if |s_e - s_t| <= 2 eps, so a row's
  (L, H) may move by at most `allowed` = the competitors within the smallest
  stored window >= 2 eps;
* where that window holds no more competitors than the close probes, the move
  is accounted exactly (dL / dH = probe competitors that moved above / to
  at-or-above the target minus those that moved below);
* MRR: rows accounted exactly contribute their exact reciprocal-rank change;
  the others at most the largest change any (L', H') inside their window
  allows — the sum of the two (over the metric's unique (h, r, t)) bounds
  |dMRR|.
"""
import numpy as np


def harmonic(n):
    """Prefix harmonic numbers H(0..n) in float64."""
    h = np.zeros(n + 1, dtype=np.float64)
    h[1:] = np.cumsum(1.0 / np.arange(1, n + 1, dtype=np.float64))
    return h


def rr(L, H, harm):
    """Expected reciprocal rank over ranks L .. H-1 (trainer.py:222-233)."""
    L = np.asarray(L, np.int64)
    H = np.asarray(H, np.int64)
    return (harm[H - 1] - harm[L - 1]) / (H - L)


def last_occurrence(hrt):
    """Indices of the rows the metric keeps: the last row of each (h, r, t)
    (the reference's dict, trainer.py:204-210)."""
    a = np.asarray(hrt, np.int64)
    hi = int(a.max()) + 1
    key = (a[::-1, 0] * hi + a[::-1, 1]) * hi + a[::-1, 2]
    _, first_rev = np.unique(key, return_index=True)
    return len(a) - 1 - first_rev


def check(want, L, H, hip_t, hip_p, hit, ref_t, ref_p, pe, near_w, windows, batch_ptr, eps_max, nclose=12):
    """Assert the rank parity above; returns a report dict.

    want: (n, >= 5) int rows h, r, t, L, H of the reference; L, H: the HIP
    path's bounds; hip_t / ref_t: target scores (ref nan where the target is
    no candidate); hip_p / ref_p / pe: probe scores and entities (-1 pad)."""
    n = len(want)
    valid_p = pe >= 0
    # the target is a candidate in both or in neither (exact mask parity)
    assert np.array_equal(hit, ~np.isnan(ref_t))
    # equal scores (including the -inf of non-candidates without an entity
    # feature on both sides) are no error; an inf on one side only is
    with np.errstate(invalid="ignore"):
        d = np.where(hip_p == ref_p, 0.0, np.abs(hip_p - ref_p))
    err = np.where(valid_p, d, 0.0).max(1)
    err = np.maximum(err, np.where(hit, np.abs(hip_t - np.nan_to_num(ref_t)), 0.0))
    eps = np.zeros(n)
    for b in range(len(batch_ptr) - 1):
        if batch_ptr[b + 1] > batch_ptr[b]:
            eps[batch_ptr[b]:batch_ptr[b + 1]] = err[batch_ptr[b]:batch_ptr[b + 1]].max()
    assert eps.max() <= eps_max, "score error %g above %g" % (eps.max(), eps_max)
    wi = np.searchsorted(windows, 2 * eps)  # smallest stored window >= 2 eps
    assert (wi < len(windows)).all()
    allowed = near_w[np.arange(n), wi]
    dL, dH = L - want[:, 3], H - want[:, 4]
    moved = (dL != 0) | (dH != 0)
    bad = np.nonzero((np.abs(dL) > allowed) | (np.abs(dH) > allowed))[0]
    assert len(bad) == 0, (bad[:10], L[bad[:10]], H[bad[:10]], want[bad[:10]], allowed[bad[:10]])
    # exact accounting where the window's competitors are all close probes
    close = valid_p[:, :nclose]
    exact = hit & (allowed <= nclose)
    above_h = (hip_p[:, :nclose] > hip_t[:, None]) & close
    above_r = (ref_p[:, :nclose] > ref_t[:, None]) & close
    atleast_h = (hip_p[:, :nclose] >= hip_t[:, None]) & close
    atleast_r = (ref_p[:, :nclose] >= ref_t[:, None]) & close
    exp_dL = above_h.sum(1) - above_r.sum(1)
    exp_dH = atleast_h.sum(1) - atleast_r.sum(1)
    ex = np.nonzero(exact)[0]
    mism = ex[(dL[ex] != exp_dL[ex]) | (dH[ex] != exp_dH[ex])]
    assert len(mism) == 0, (mism[:10], dL[mism[:10]], exp_dL[mism[:10]], dH[mism[:10]], exp_dH[mism[:10]])
    # MRR bound over the rows the metric keeps
    keep = last_occurrence(want[:, :3])
    harm = harmonic(int(max(H.max(), want[:, 4].max()) + allowed.max() + 2))
    Lr, Hr = want[:, 3].astype(np.int64), want[:, 4].astype(np.int64)
    d_rr = rr(L, H, harm) - rr(Lr, Hr, harm)
    km = keep[moved[keep]]
    k_ex = km[exact[km]]
    k_bd = km[~exact[km]]
    a = allowed[k_bd].astype(np.int64)
    lo_L = np.maximum(1, Lr[k_bd] - a)
    up = rr(lo_L, np.maximum(lo_L + 1, Hr[k_bd] - a), harm) - rr(Lr[k_bd], Hr[k_bd], harm)
    down = rr(Lr[k_bd], Hr[k_bd], harm) - rr(Lr[k_bd] + a, Hr[k_bd] + a, harm)
    bound_rows = np.maximum(up, down)
    observed = float(d_rr[keep].sum()) / n
    bound = (abs(float(d_rr[k_ex].sum())) + float(bound_rows.sum())) / n
    assert abs(observed) <= bound + 1e-15, (observed, bound)
    return dict(n=n, eps_max=float(eps.max()), eps_median=float(np.median(eps)), moved=int(moved.sum()),
                exact=int(moved[ex].sum()), bounded=int(moved.sum() - moved[ex].sum()), d_mrr=observed,
                mrr_bound=bound, bound_exact_part=abs(float(d_rr[k_ex].sum())) / n,
                bound_window_part=float(bound_rows.sum()) / n)


def describe(rep):
    ratio = rep["mrr_bound"] / abs(rep["d_mrr"]) if rep["d_mrr"] else float("inf") if rep["mrr_bound"] else 1.0
    return ("%d rows, score error max %.3g (median %.3g); %d rows with differing (L, H), all within their window "
            "(%d accounted exactly, %d bounded); MRR delta %.3g, per-row bound %.3g (exact %.3g + window %.3g; "
            "bound / |delta| %.3g)" % (rep["n"], rep["eps_max"], rep["eps_median"], rep["moved"], rep["exact"],
                                      rep["bounded"], rep["d_mrr"], rep["mrr_bound"], rep["bound_exact_part"],
                                      rep["bound_window_part"], ratio))
