cat > /tmp/ob.py <<'PY'
import os, sys, time, contextlib, torch
sys.path.insert(0, os.getcwd())
import bench
dev = torch.device("cuda:0")
with contextlib.redirect_stdout(sys.stderr):
    graph, test_set, model, rows = bench.build_workload("RotatE")
model = model.to(dev).eval()
h = torch.from_numpy(rows[:, 0]).to(dev); r = torch.from_numpy(rows[:, 1]).to(dev)
def step():
    model.invalidate_cache()
    with torch.no_grad():
        return model.forward_rows(h, r, None)
for rep in range(3):
    for flag in (False, True):
        model.overlap_begin = flag
        print("begin=%s %.3f ms" % (flag, bench.time_forward(step, 10) * 1e3), flush=True)
PY
timeout -k 10 400 python3 /tmp/ob.py 2>/dev/null
for v in eall e2 e4 e8 eall e4; do V=$v RNNL_LIB=rnnlogic_amd/_build/variants/$v.so timeout -k 10 200 python3 tools/enc_tmp.py 2>/dev/null; done
