"""Rule->entity aggregators and the MLP, parameter-compatible with the
reference's src/layers.py (same module tree, so state_dict keys and shapes
match and checkpoints interchange).

On the GPU the eval forward of these modules is fused into the HIP kernel
(rnnlogic_amd/csrc/ground.hip, score_candidate); the torch forwards below
serve the autograd (training) path, where they consume the kernel's
candidate/rule count lists.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F


class MLP(nn.Module):
    """Reference src/layers.py:9-51: Linear layers with `activation` between
    them (none after the last), optional BatchNorm / dropout / shortcut."""

    def __init__(self, input_dim, hidden_dims, short_cut=False, batch_norm=False, activation="relu", dropout=0):
        super(MLP, self).__init__()
        self.dims = [input_dim] + list(hidden_dims)
        self.short_cut = short_cut
        self.activation = getattr(F, activation) if isinstance(activation, str) else activation
        self.dropout = nn.Dropout(dropout) if dropout else None
        self.layers = nn.ModuleList(nn.Linear(a, b) for a, b in zip(self.dims[:-1], self.dims[1:]))
        self.batch_norms = (nn.ModuleList(nn.BatchNorm1d(d) for d in self.dims[1:-1]) if batch_norm else None)

    def forward(self, input):
        x = input
        last = len(self.layers) - 1
        for i, layer in enumerate(self.layers):
            y = layer(x)
            if i < last:
                if self.batch_norms:
                    y = self.batch_norms[i](y.flatten(0, -2)).view_as(y)
                y = self.activation(y)
                if self.dropout:
                    y = self.dropout(y)
            if self.short_cut and y.shape == x.shape:
                y = y + x
            x = y
        return x


class FuncToNodeSum(nn.Module):
    """Reference src/layers.py:53-77: relu(LN(Linear(sum_rho A[rho, c] x_rho)))."""

    def __init__(self, vector_dim):
        super(FuncToNodeSum, self).__init__()
        self.vector_dim = vector_dim
        self.layer_norm = nn.LayerNorm(self.vector_dim)
        self.add_model = MLP(self.vector_dim, [self.vector_dim])
        self.eps = 1e-6

    def forward(self, A_fn, x_f, b_n):
        # (R_q, C)^T @ (R_q, H) == sum over rules of count * embedding
        return self.finish(A_fn.t().matmul(x_f))

    def finish(self, features):
        """relu(LN(Linear(features))) on the count-weighted sums (C, H)."""
        return torch.relu(self.layer_norm(self.add_model(features)))


class FuncToNode(nn.Module):
    """Reference src/layers.py:79-126: PNA aggregation — mean/min/max/std of
    the rule embeddings weighted by path counts, scaled by {1, s, 1/s} with
    s = log(degree) / (per-query mean of log(degree))."""

    def __init__(self, vector_dim):
        super(FuncToNode, self).__init__()
        self.vector_dim = vector_dim
        self.layer_norm = nn.LayerNorm(self.vector_dim)
        self.add_model = MLP(self.vector_dim * 12, [self.vector_dim])
        self.eps = 1e-6

    def forward(self, A_fn, x_f, b_n):
        At = A_fn.t()                                  # (C, R_q)
        deg = At.sum(1) + 1                            # (C,)
        active = (At != 0).unsqueeze(-1)               # (C, R_q, 1)
        xb = x_f.unsqueeze(0)
        mn = torch.where(active, xb, torch.full_like(xb, float("inf"))).min(1)[0]
        mx = torch.where(active, xb, torch.full_like(xb, float("-inf"))).max(1)[0]
        return self.finish(At.matmul(x_f), At.matmul(x_f * x_f), mn, mx, deg, b_n, int(b_n.max().item()) + 1)

    def finish(self, wsum, wsq, mn, mx, deg, b_n, n_batch, row_scale=None):
        """The PNA block from its sufficient statistics per candidate:
        count-weighted sums of x and x^2 (C, H), unweighted min/max over the
        candidate's rules (C, H), degree = 1 + sum of counts (C,), and the
        candidate's batch row b_n (C,).  row_scale (n_batch,): the rows' mean
        log-degree when the caller has it (the HIP statistics' order-free sum;
        else the per-row index_add below)."""
        eps = self.eps
        deg = deg.unsqueeze(-1)
        mean = wsum / deg.clamp(min=eps)
        sq_mean = wsq / deg.clamp(min=eps)
        std = (sq_mean - mean * mean).clamp(min=eps).sqrt()
        feats = torch.cat([mean, mn, mx, std], -1)     # (C, 4H)
        s = deg.log()
        if row_scale is None:
            s_sum = torch.zeros(n_batch, device=s.device, dtype=s.dtype).index_add(0, b_n, s.squeeze(-1))
            s_cnt = torch.zeros(n_batch, device=s.device, dtype=s.dtype).index_add(
                0, b_n, torch.ones_like(s.squeeze(-1)))
            row_scale = s_sum / s_cnt.clamp(min=eps)
        s = s / row_scale[b_n].unsqueeze(-1).clamp(min=eps)
        scales = torch.cat([torch.ones_like(s), s, 1 / s.clamp(min=eps)], -1)  # (C, 3)
        upd = (feats.unsqueeze(-1) * scales.unsqueeze(-2)).flatten(-2)
        return torch.relu(self.layer_norm(self.add_model(upd)))
