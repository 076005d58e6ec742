"""Process-group helpers, API-compatible with the reference's src/comm.py
(get_rank, get_world_size, get_group, init_process_group, get_cpu_count,
synchronize, reduce, stack, cat).

One process per GPU.  backend "nccl" is RCCL on ROCm (xGMI between the GPUs of
a node); a gloo group is kept beside it for CPU tensors, as in the reference
(comm.py:50-65).  reduce/stack/cat take a tensor or a nested dict/list/tuple of
tensors and return the same structure: every leaf of one dtype travels in one
flat buffer, so a call costs one collective per dtype (cat: two, the second
after a size exchange), not one per leaf.  bool leaves travel as uint8 (RCCL
has no bool) and come back as bool, as in the reference (comm.py:162-172).
`dst` (reduce) leaves the result on that rank only (dist.reduce); stack and
cat accept `dst` and return the gathered result on every rank.
"""
import multiprocessing
import os

import torch
from torch import distributed as dist

cpu_group = None
gpu_group = None


def get_rank():
    """comm.py:13-22: rank of this process, 0 without a process group."""
    if dist.is_initialized():
        return dist.get_rank()
    return int(os.environ.get("RANK", 0))


def get_world_size():
    """comm.py:25-34: number of processes, 1 without a process group."""
    if dist.is_initialized():
        return dist.get_world_size()
    return int(os.environ.get("WORLD_SIZE", 1))


def get_group(device):
    """comm.py:37-47: the process group for tensors on `device`."""
    group = cpu_group if device.type == "cpu" else gpu_group
    if group is None:
        raise ValueError("%s group is not initialized. Use comm.init_process_group() to initialize it"
                         % device.type.upper())
    return group


def init_process_group(backend, init_method=None, **kwargs):
    """comm.py:50-65: WORLD on `backend`; for nccl (RCCL) also a gloo group for
    CPU tensors."""
    global cpu_group, gpu_group
    dist.init_process_group(backend, init_method, **kwargs)
    gpu_group = dist.group.WORLD
    cpu_group = dist.new_group(backend="gloo") if backend == "nccl" else gpu_group


def get_cpu_count():
    return multiprocessing.cpu_count()


def synchronize():
    """Barrier over all processes (no-op for one process)."""
    if get_world_size() > 1:
        dist.barrier()


# ---------------------------------------------------------------- structures
def _leaves(obj, out):
    if isinstance(obj, torch.Tensor):
        out.append(obj)
    elif isinstance(obj, dict):
        for v in obj.values():
            _leaves(v, out)
    elif isinstance(obj, (list, tuple)):
        for v in obj:
            _leaves(v, out)
    else:
        raise ValueError("Unknown type `%s`" % type(obj))
    return out


def _rebuild(obj, it):
    if isinstance(obj, torch.Tensor):
        return next(it)
    if isinstance(obj, dict):
        return type(obj)((k, _rebuild(v, it)) for k, v in obj.items())
    if isinstance(obj, (list, tuple)):
        return type(obj)(_rebuild(v, it) for v in obj)
    raise ValueError("Unknown type `%s`" % type(obj))


def _by_dtype(leaves):
    groups = {}
    for i, t in enumerate(leaves):
        groups.setdefault(t.dtype, []).append(i)
    return groups


_OPS = {"sum": dist.ReduceOp.SUM, "mean": dist.ReduceOp.SUM, "min": dist.ReduceOp.MIN,
        "max": dist.ReduceOp.MAX, "product": dist.ReduceOp.PRODUCT}


def _wire(t):
    """The tensor as sent: bool -> uint8 (no bool in RCCL)."""
    return t.to(torch.uint8) if t.dtype == torch.bool else t


def reduce(obj, op="sum", dst=None):
    """Reduce every tensor of `obj` over the ranks (comm.py:136-175); op is
    "sum", "mean", "min", "max" or "product".  With dst the result is valid
    on that rank only."""
    if op not in _OPS:
        raise ValueError("Unknown reduction `%s`" % op)
    world = get_world_size()
    if world == 1:
        return obj
    leaves = _leaves(obj, [])
    result = [None] * len(leaves)
    for dtype, idx in _by_dtype(leaves).items():
        flat = torch.cat([_wire(leaves[i]).reshape(-1) for i in idx])
        group = get_group(flat.device)
        if dst is None:
            dist.all_reduce(flat, op=_OPS[op], group=group)
        else:
            dist.reduce(flat, dst=dst, op=_OPS[op], group=group)
        if op == "mean":
            flat = flat / world
        for i, part in zip(idx, flat.split([leaves[i].numel() for i in idx])):
            result[i] = part.view(leaves[i].shape).to(dtype)
    return _rebuild(obj, iter(result))


def stack(obj, dst=None):
    """All-gather every tensor of `obj` and stack along a new dim 0
    (comm.py:178-211); every rank must pass equal shapes.  `dst` is accepted
    for the reference's signature only: the result is returned on every rank
    (the reference's reduce leaves it valid on dst alone, so this is a
    superset)."""
    world = get_world_size()
    if world == 1:
        return _rebuild(obj, iter([t.unsqueeze(0) for t in _leaves(obj, [])]))
    leaves = _leaves(obj, [])
    result = [None] * len(leaves)
    for dtype, idx in _by_dtype(leaves).items():
        flat = torch.cat([_wire(leaves[i]).reshape(-1) for i in idx])
        parts = [torch.empty_like(flat) for _ in range(world)]
        dist.all_gather(parts, flat, group=get_group(flat.device))
        gathered = torch.stack(parts)
        for i, part in zip(idx, gathered.split([leaves[i].numel() for i in idx], dim=1)):
            result[i] = part.reshape((world,) + tuple(leaves[i].shape)).to(dtype)
    return _rebuild(obj, iter(result))


def cat(obj, dst=None):
    """All-gather every tensor of `obj` and concatenate along dim 0
    (comm.py:214-256); dim 0 may differ across ranks (sizes are exchanged
    first, payloads padded to the largest rank).  `dst` is accepted for the
    reference's signature only: the result is returned on every rank."""
    world = get_world_size()
    if world == 1:
        return obj
    leaves = _leaves(obj, [])
    result = [None] * len(leaves)
    for dtype, idx in _by_dtype(leaves).items():
        device = leaves[idx[0]].device
        group = get_group(device)
        sizes = torch.tensor([leaves[i].numel() for i in idx], dtype=torch.long, device=device)
        all_sizes = [torch.empty_like(sizes) for _ in range(world)]
        dist.all_gather(all_sizes, sizes, group=group)
        all_sizes = torch.stack(all_sizes).cpu()          # (world, n_leaves)
        totals = all_sizes.sum(1)
        cap = int(totals.max())
        flat = torch.cat([_wire(leaves[i]).reshape(-1) for i in idx])
        padded = torch.zeros(cap, dtype=flat.dtype, device=device)
        padded[:flat.numel()] = flat
        gathered = [torch.empty_like(padded) for _ in range(world)]
        dist.all_gather(gathered, padded, group=group)
        pieces = [[] for _ in idx]
        for w in range(world):
            parts = gathered[w][:int(totals[w])].split(all_sizes[w].tolist())
            for j, part in enumerate(parts):
                pieces[j].append(part)
        for j, i in enumerate(idx):
            tail = tuple(leaves[i].shape[1:])
            result[i] = torch.cat(pieces[j]).view((-1,) + tail).to(dtype)
    return _rebuild(obj, iter(result))
