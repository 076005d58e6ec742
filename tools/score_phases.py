"""Phase clocks of the SUM chunk scoring kernel (score_sum_chunk_kernel,
rnnl_debug_profile slots 16-23) over per-batch PredictorPlus.forward calls —
where a small launch's scoring time goes (diagnostic; GPU box).
Needs a library built with -DRNNL_SCORE_PROF=1 for ground.hip (tools/build_variants.sh ground.hip prof "-DRNNL_SCORE_PROF=1", then RNNL_LIB=rnnlogic_amd/_build/variants/prof.so).
Usage: python tools/score_phases.py [N_BATCHES [FEATURE]]"""
import contextlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from rnnlogic_amd import _native  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 200
FEATURE = sys.argv[2] if len(sys.argv) > 2 else "RotatE"
dev = torch.device("cuda:0")
with contextlib.redirect_stdout(sys.stderr):
    graph, test_set, model, rows = bench.build_workload(FEATURE)
model = model.to(dev).eval()
batches = test_set.batches[:N]
hs = [torch.tensor([x[0] for x in b], device=dev) for b in batches]
rs = [torch.tensor([x[1] for x in b], device=dev) for b in batches]
with torch.no_grad():
    for k in range(3):
        model(hs[k], rs[k], None)
    torch.cuda.synchronize()
    prof = torch.zeros(25, dtype=torch.int64, device=dev)
    _native.call("rnnl_debug_profile", prof.data_ptr())
    for h, r in zip(hs, rs):
        model(h, r, None)
    torch.cuda.synchronize()
    _native.call("rnnl_debug_profile", None)
p = prof.cpu().tolist()
waves = max(p[21], 1)
MHZ = p[19] / max(p[24] / 100.0, 1e-9)  # s_memtime ticks per us, vs s_memrealtime (100 MHz)
print("s_memtime clock: %.0f MHz" % MHZ)
print("calls %d: active waves/call %.0f, chunks/wave %.2f" % (len(batches), p[21] / len(batches), p[20] / waves))
for name, v in zip(["setup", "classify", "flush", "total"], p[16:20]):
    print("  %-9s %8.2f us per active wave" % (name, v / waves / MHZ))
print("  max total %.2f us, max flush %.2f us (any wave of any call)" % (p[22] / MHZ, p[23] / MHZ))
