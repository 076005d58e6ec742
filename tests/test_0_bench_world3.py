"""bench.py's N > 1 path on the GPU box: three ranks launched
by torch.distributed.run as the driver launches the scaling bench, both on
cuda:0 (RNNL_BENCH_ONE_DEVICE=1) over gloo (RNNL_BENCH_BACKEND=gloo; RCCL
refuses two ranks on one device).  Checks the one JSON line: the ranks'
batches are the reference evaluate()'s DistributedSampler shards — their
union is the whole test split, the surplus the sampler's padding (1,514
batches over 3 ranks: 505 each, one repeated) — and
`value` counts the split's 40,932 queries once (value x ms_per_step = 40,932
x 1000).  A rehearsal of the sharding and the timing contract, not a
measurement (both ranks share one GPU).

The file sorts first: the bench ranks start before this pytest process
initialises the GPU."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_bench_world3_shards_and_value():
    if torch.cuda.is_initialized():
        pytest.skip("this process already initialised the GPU (run this file first)")
    env = dict(os.environ, RNNL_BENCH_ONE_DEVICE="1", RNNL_BENCH_BACKEND="gloo", OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "3",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(REPO, "bench.py"),
           "--gpus", "3", "--steps", "2", "--warmup", "1", "--no-cpu-baseline"]
    out = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=420)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [x for x in out.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, out.stdout  # rank 0 prints one JSON line
    d = json.loads(lines[0])
    assert d["n_gpus"] == 3 and d["steps"] == 2 and d["scaling"] == "strong"
    sh = d["config"]["shards"]
    assert sh["union_is_split"]
    assert sh["batches_per_rank"] == [505, 505, 505] and sh["padding_batches"] == 1
    assert sh["rows_counted"] == 40932 and sh["rows_total_with_padding"] > 40932
    assert abs(d["value"] * d["ms_per_step"] / 1e3 - 40932) <= 40932 * 1e-3
    assert d["weak_replicated"]["rows_per_rank"] == 40932
