"""A/B timing of rnnl_rotate_score across the compile variants built by
tools/build_variants.sh rotate.hip (rnnlogic_amd/_build/variants/*.so), at the bench
workload's shape (FB15k-237 test split: 40,932 queries x 14,541 entities x
D = 1000).  Prints one line per variant: mean ms per launch (HIP events) and
the max |diff| against the main library's RNNL_ROTATE_DIRECT result.

Usage: python tools/bench_rotate.py [--nq N] [--reps K] [variant ...]
"""
import argparse
import ctypes
import glob
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from rnnlogic_amd import _native  # noqa: E402


def load(path):
    L = ctypes.CDLL(path)
    for name, res, args in _native.SIGNATURES:
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    return L


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nq", type=int, default=40932)
    ap.add_argument("--E", type=int, default=14541)
    ap.add_argument("--D", type=int, default=1000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--scale", type=float, default=0.011)
    ap.add_argument("variants", nargs="*")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator(device="cpu").manual_seed(0)
    E, D, R2, nq = a.E, a.D, 474, a.nq
    eemb = ((torch.rand(E, 2 * D, generator=g) * 2 - 1) * a.scale).to(dev)
    remb = ((torch.rand(R2, D, generator=g) * 2 - 1) * 0.011).to(dev)
    h = torch.randint(0, E, (nq,), generator=g).to(dev)
    r = torch.randint(0, R2, (nq,), generator=g).to(dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    tabs = {}
    for mode in (_native.ROTATE_DIRECT, _native.ROTATE_MFMA):
        eb, rb = ctypes.c_size_t(), ctypes.c_size_t()
        _native.call("rnnl_rotate_table_sizes", E, D, R2, mode, ctypes.byref(eb), ctypes.byref(rb))
        etab = torch.empty(eb.value // 4, device=dev)
        _native.call("rnnl_rotate_entity_table", eemb.data_ptr(), E, D, mode, etab.data_ptr(), st)
        tabs[mode] = etab
    rtab = torch.empty(rb.value // 4, device=dev)
    _native.call("rnnl_rotate_relation_table", remb.data_ptr(), R2, D, 9.0, rtab.data_ptr(), st)
    wsb = ctypes.c_size_t()
    _native.call("rnnl_rotate_workspace_size", nq, E, D, _native.ROTATE_DIRECT, ctypes.byref(wsb))
    ws = torch.empty(wsb.value // 2 + 1024, device=dev)  # 2x: variants may pad the query groups differently
    out = torch.empty(nq, E, device=dev)
    ref = torch.empty(nq, E, device=dev)

    def run(L, mode, dst, reps):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
        L.rnnl_rotate_score(eemb.data_ptr(), tabs[mode].data_ptr(), rtab.data_ptr(), D, 9.0, h.data_ptr(),
                            r.data_ptr(), nq, E, dst.data_ptr(), 0, mode, ws.data_ptr(), ws.numel() * 4, st)  # warmup
        ev[0].record()
        for i in range(reps):
            rc = L.rnnl_rotate_score(eemb.data_ptr(), tabs[mode].data_ptr(), rtab.data_ptr(), D, 9.0, h.data_ptr(),
                                     r.data_ptr(), nq, E, dst.data_ptr(), 0, mode, ws.data_ptr(), ws.numel() * 4, st)
            assert rc == 0, L.rnnl_last_error()
            ev[i + 1].record()
        torch.cuda.synchronize()
        return [ev[i].elapsed_time(ev[i + 1]) for i in range(reps)]

    main_lib = _native.lib()
    # float64 restatement of embedding.py:45-70 on the first 32 rows
    import numpy as np
    n64 = 32
    E64 = eemb.double().cpu().numpy()
    div = np.float32((9.0 + 2.0) / D / np.pi)
    ph = (remb.cpu().numpy()[r[:n64].cpu().numpy()] / div).astype(np.float64)
    hh = E64[h[:n64].cpu().numpy()]
    re = hh[:, :D] * np.cos(ph) - hh[:, D:] * np.sin(ph)
    im = hh[:, :D] * np.sin(ph) + hh[:, D:] * np.cos(ph)
    want = np.empty((n64, E))
    for i in range(n64):
        want[i] = 9.0 - np.sqrt((re[i][None, :] - E64[:, :D]) ** 2 + (im[i][None, :] - E64[:, D:]) ** 2).sum(1)
    t = run(main_lib, _native.ROTATE_DIRECT, ref, a.reps)
    print("main/direct %8.2f ms  (%s)  vs f64 %.3g" % (sum(t) / len(t), " ".join("%.2f" % x for x in t),
                                                      np.abs(ref[:n64].cpu().numpy() - want).max()), flush=True)
    t = run(main_lib, _native.ROTATE_MFMA, out, a.reps)
    print("main/mfma   %8.2f ms  maxdiff %.3g  vs f64 %.3g" % (sum(t) / len(t), (out - ref).abs().max().item(),
                                                                np.abs(out[:n64].cpu().numpy() - want).max()), flush=True)
    paths = sorted(glob.glob(os.path.join(REPO, "rnnlogic_amd", "_build", "variants", "*.so")))
    for p in paths:
        name = os.path.basename(p)[:-3]
        if a.variants and name not in a.variants:
            continue
        L = load(p)
        out.zero_()
        t = run(L, _native.ROTATE_MFMA if name.startswith('mfma') else _native.ROTATE_DIRECT, out, a.reps)
        print("%-20s %8.2f ms  maxdiff %.3g" % (name, sum(t) / len(t), (out - ref).abs().max().item()), flush=True)


if __name__ == "__main__":
    main()
