"""MLP building blocks (mirror of reference models/helpers.py).

``GenericMLP`` keeps the reference's ``layers`` Sequential indexing
(conv/linear, [norm], activation, [dropout], ..., out conv, [norm], [act]) so
state-dict keys such as ``mlp_heads.center_head.layers.0.weight`` load
unchanged (reference models/helpers.py:45-112).
"""
import copy

import torch
import torch.nn as nn

from .gemm import rows_linear

NORM_DICT = {
    "bn1d": nn.BatchNorm1d,
    "id": nn.Identity,
    "ln": nn.LayerNorm,
}

ACTIVATION_DICT = {
    "relu": nn.ReLU,
    "gelu": nn.GELU,
}


class GenericMLP(nn.Module):
    def __init__(self, input_dim, hidden_dims, output_dim, norm_fn_name=None, activation="relu",
                 use_conv=False, dropout=None, hidden_use_bias=False, output_use_bias=True,
                 output_use_activation=False, output_use_norm=False, weight_init_name=None):
        super().__init__()
        act = ACTIVATION_DICT[activation]
        if norm_fn_name == "ln" and use_conv:
            norm = lambda c: nn.GroupNorm(1, c)  # noqa: E731  (reference: LayerNorm over conv channels)
        elif norm_fn_name is not None:
            norm = NORM_DICT[norm_fn_name]
        else:
            norm = None
        if dropout is not None and not isinstance(dropout, list):
            dropout = [dropout] * len(hidden_dims)

        def proj(cin, cout, bias):
            return nn.Conv1d(cin, cout, 1, bias=bias) if use_conv else nn.Linear(cin, cout, bias=bias)

        mods = []
        cin = input_dim
        for i, h in enumerate(hidden_dims):
            mods.append(proj(cin, h, hidden_use_bias))
            if norm is not None:
                mods.append(norm(h))
            mods.append(act())
            if dropout is not None:
                mods.append(nn.Dropout(p=dropout[i]))
            cin = h
        mods.append(proj(cin, output_dim, output_use_bias))
        if output_use_norm:
            mods.append(norm(output_dim))
        if output_use_activation:
            mods.append(act())
        self.layers = nn.Sequential(*mods)
        if weight_init_name is not None:
            for p in self.parameters():
                if p.dim() > 1:
                    nn.init.xavier_uniform_(p)

    def forward(self, x):
        """Reference layout: (B, C, N) for conv MLPs, (..., C) for linear ones."""
        if isinstance(self.layers[0], nn.Conv1d):
            B, C, N = x.shape
            y = self.rows(x.transpose(1, 2).reshape(B * N, C))
            return y.view(B, N, -1).transpose(1, 2)
        return self.layers(x)

    def rows(self, x):
        """Channels-last evaluation on (R, Cin) rows -> (R, Cout): each 1x1 conv is one
        GEMM, BatchNorm1d statistics over the R rows (== over (B, N) positions).  Training
        under bf16 autocast: BatchNorm + ReLU (+ Dropout) run as one HIP row pass each way
        (heads.bn_relu_rows)."""
        from . import heads
        from . import resnorm as rn
        mods = list(self.layers)
        i = 0
        while i < len(mods):
            m = mods[i]
            if isinstance(m, nn.Conv1d) and i + 2 < len(mods) and isinstance(mods[i + 1], nn.ReLU) \
                    and isinstance(mods[i + 2], nn.Conv1d) and x.is_cuda:
                # conv + ReLU + conv (the query projection): the ReLU is the first GEMM's
                # epilogue forward and the second GEMM's input-gradient epilogue backward
                m2 = mods[i + 2]
                w1 = m.weight.view(m.weight.shape[0], m.weight.shape[1])
                w2 = m2.weight.view(m2.weight.shape[0], m2.weight.shape[1])
                xb = x.to(torch.bfloat16) if torch.is_autocast_enabled("cuda") else x
                if rn.ffn_weights_ok(xb, w1, w2):
                    x = rn.ffn_weights(xb, w1, m.bias, w2, m2.bias)
                    i += 3
                    continue
            if isinstance(m, nn.ReLU) and x.is_cuda and x.dtype == torch.bfloat16 and \
                    x.shape[-1] % 8 == 0:
                x = rn.relu_rows(x)
                i += 1
                continue
            if isinstance(m, nn.Conv1d):
                x = rows_linear(x, m.weight.view(m.weight.shape[0], m.weight.shape[1]), m.bias)
            elif isinstance(m, nn.GroupNorm):
                raise NotImplementedError("GroupNorm MLPs are not on the reference path")
            elif isinstance(m, (nn.BatchNorm1d, nn.SyncBatchNorm)) and i + 1 < len(mods):
                drop = mods[i + 2] if i + 2 < len(mods) and isinstance(mods[i + 2], nn.Dropout) else None
                if heads.bn_relu_rows_ok(x, m, mods[i + 1], drop):
                    x = heads.bn_relu_rows(x, m, drop)
                    i += 3 if drop is not None else 2
                    continue
                from .pointnet2_modules import batch_norm_rows
                x = batch_norm_rows(m, x) if isinstance(m, nn.SyncBatchNorm) else m(x)
            else:
                x = m(x)
            i += 1
        return x


def get_clones(module, n):
    return nn.ModuleList([copy.deepcopy(module) for _ in range(n)])
