"""Test-only stand-in for the third-party torch_scatter package (not installed
in this container).  The reference uses only the sum reduction
(src/data.py:161,171), which index_add_ computes exactly for integer inputs."""
import torch


def scatter(src, index, dim=0, out=None, dim_size=None, reduce="sum"):
    assert reduce in ("sum", "add") and dim == 0
    if dim_size is None:
        dim_size = int(index.max()) + 1 if index.numel() else 0
    res = torch.zeros((dim_size,) + tuple(src.shape[1:]), dtype=src.dtype, device=src.device)
    return res.index_add_(0, index, src)


def scatter_add(src, index, dim=0, out=None, dim_size=None):
    return scatter(src, index, dim, out, dim_size)


def _unsupported(*a, **k):
    raise NotImplementedError("not used by the reference hot path")


scatter_min = scatter_max = scatter_mean = _unsupported
