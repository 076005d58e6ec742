"""bench.py over RCCL on the GPU box: one rank launched by
torch.distributed.run as the driver launches the scaling bench, with the
`nccl` backend (RCCL on ROCm) — the one-GPU box cannot hold two RCCL ranks,
but one rank runs RCCL's communicator through the same init, barriers,
all-reduce (MAX over the ranks' times) and all-gathers (rows and batch
indices per rank) as the N-GPU run.  Checks the JSON line: the process group
is RCCL's, the single shard is the whole split, and `value` counts the
split's queries once.

The file sorts first: the bench rank starts before this pytest process
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


def test_bench_rccl_one_rank():
    if torch.cuda.is_initialized():
        pytest.skip("this process already initialised the GPU (run this file first)")
    env = dict(os.environ, OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(REPO, "bench.py"),
           "--gpus", "1", "--steps", "2", "--warmup", "1", "--profile-only"]
    out = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=420)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [x for x in out.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, out.stdout
    d = json.loads(lines[0])
    assert d["config"]["process_group"] == "nccl"
    sh = d["config"]["shards"]
    assert sh["union_is_split"] and sh["batches_per_rank"] == [1514] and sh["padding_batches"] == 0
    assert d["config"]["rows_per_rank"] == [40932]
    assert abs(d["value"] * d["ms_per_step"] / 1e3 - 40932) <= 40932 * 1e-3
