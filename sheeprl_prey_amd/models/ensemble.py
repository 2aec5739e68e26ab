"""Batched ensembles of identical MLPs (SAC twin-Q / DroQ / SAC-AE critics).

The reference keeps ``n`` separate critic modules and runs them one after the other
(``sac/agent.py:256-263``: ``torch.cat([qf(obs, act) for qf in qfs], -1)``), i.e. n x L small
GEMMs per evaluation.  Here the n members' weights are stacked, ``[n, out, in]``: the first layer
(whose input is shared by all members) is ONE GEMM against the members' concatenated weights, the
deeper layers are one batched GEMM (``baddbmm``) each, so a twin-Q evaluation costs L launches
instead of n x L and each launch has n x more work for the matrix cores.

Because member i's parameters only ever receive gradients from member i's output, a single
optimiser over the stacked parameters with loss ``sum_i loss_i`` is exactly the reference's
per-critic updates (``droq/droq.py:95-110`` updates critic i with only loss_i; Adam is elementwise).
"""
from __future__ import annotations

import math
from typing import Callable, Optional, Sequence

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch import Tensor

_ACTS = {
    "relu": F.relu,
    "tanh": torch.tanh,
    "elu": F.elu,
    "silu": F.silu,
    "identity": lambda x: x,
    None: lambda x: x,
}


def _act_name(act) -> Optional[str]:
    if act is None:
        return None
    if isinstance(act, str):
        name = act.split(".")[-1].lower()
    else:
        name = getattr(act, "__name__", type(act).__name__).lower()
    return {"relu": "relu", "tanh": "tanh", "elu": "elu", "silu": "silu", "identity": "identity"}.get(name, name)


class EnsembleLinear(nn.Module):
    """``n`` independent ``nn.Linear(in_features, out_features)`` layers with stacked weights."""

    def __init__(self, n: int, in_features: int, out_features: int, bias: bool = True):
        super().__init__()
        self.n, self.in_features, self.out_features = n, in_features, out_features
        self.weight = nn.Parameter(torch.empty(n, out_features, in_features))
        self.bias = nn.Parameter(torch.empty(n, out_features)) if bias else None
        self.reset_parameters()

    def reset_parameters(self) -> None:
        # per member exactly nn.Linear's default init (kaiming_uniform(a=sqrt 5) == U(+-1/sqrt(fan_in)))
        bound = 1.0 / math.sqrt(self.in_features) if self.in_features > 0 else 0.0
        with torch.no_grad():
            self.weight.uniform_(-bound, bound)
            if self.bias is not None:
                self.bias.uniform_(-bound, bound)

    def forward(self, x: Tensor) -> Tensor:
        """``x``: ``[B, in]`` (shared input) or ``[n, B, in]`` -> ``[n, B, out]``."""
        if x.dim() == 2:
            w = self.weight.reshape(self.n * self.out_features, self.in_features)
            b = self.bias.reshape(-1) if self.bias is not None else None
            y = F.linear(x, w, b)  # [B, n*out]: one GEMM for all members
            return y.view(x.shape[0], self.n, self.out_features).transpose(0, 1)
        if self.bias is not None:
            return torch.baddbmm(self.bias.unsqueeze(1), x, self.weight.transpose(1, 2))
        return torch.bmm(x, self.weight.transpose(1, 2))

    def extra_repr(self) -> str:
        return f"n={self.n}, in_features={self.in_features}, out_features={self.out_features}"


class EnsembleLayerNorm(nn.Module):
    """Per-member LayerNorm over the last dim (affine params ``[n, H]``)."""

    def __init__(self, n: int, normalized_shape: int, eps: float = 1e-5):
        super().__init__()
        self.eps = eps
        self.normalized_shape = (normalized_shape,)
        self.weight = nn.Parameter(torch.ones(n, normalized_shape))
        self.bias = nn.Parameter(torch.zeros(n, normalized_shape))

    def forward(self, x: Tensor) -> Tensor:  # [n, B, H]
        y = F.layer_norm(x, self.normalized_shape, None, None, self.eps)
        return torch.addcmul(self.bias.unsqueeze(1), y, self.weight.unsqueeze(1))


class EnsembleMLP(nn.Module):
    """``n`` MLPs ``in -> hidden... -> out`` evaluated together; per hidden layer the reference
    ``miniblock`` order Linear -> Dropout -> LayerNorm -> activation (``models/models.py``)."""

    def __init__(
        self,
        n: int,
        input_dim: int,
        hidden_sizes: Sequence[int],
        output_dim: Optional[int] = 1,
        activation="relu",
        dropout: float = 0.0,
        layer_norm: bool = False,
    ):
        super().__init__()
        self.n = n
        self.input_dim = input_dim
        self.dropout = float(dropout)
        self.act_name = _act_name(activation)
        self._act: Callable = _ACTS[self.act_name]
        self.layers = nn.ModuleList()
        self.norms = nn.ModuleList() if layer_norm else None
        d = input_dim
        for h in hidden_sizes:
            self.layers.append(EnsembleLinear(n, d, h))
            if layer_norm:
                self.norms.append(EnsembleLayerNorm(n, h))
            d = h
        self.head = EnsembleLinear(n, d, output_dim) if output_dim is not None else None
        self.output_dim = output_dim if output_dim is not None else d

    def hidden(self, x: Tensor) -> Tensor:
        """Every member's last hidden layer, ``[n, B, hidden]`` (the head's input)."""
        for i, layer in enumerate(self.layers):
            x = layer(x)
            if self.dropout > 0:
                x = F.dropout(x, self.dropout, self.training)
            if self.norms is not None:
                x = self.norms[i](x)
            x = self._act(x)
        return x

    def forward(self, x: Tensor) -> Tensor:
        """``x``: ``[B, in]`` or ``[n, B, in]`` -> ``[n, B, out]``."""
        for i, layer in enumerate(self.layers):
            x = layer(x)
            if self.dropout > 0:
                x = F.dropout(x, self.dropout, self.training)
            if self.norms is not None:
                x = self.norms[i](x)
            x = self._act(x)
        if self.head is not None:
            x = self.head(x)
        return x

    @torch.no_grad()
    def member_(self, i: int, module: nn.Module) -> None:
        """Copy member ``i``'s weights from a reference-layout critic (an ``MLP`` of Linear /
        LayerNorm layers, in order) - used to import per-critic state."""
        lins = [m for m in module.modules() if isinstance(m, nn.Linear)]
        lns = [m for m in module.modules() if isinstance(m, nn.LayerNorm)]
        mine = list(self.layers) + ([self.head] if self.head is not None else [])
        assert len(lins) == len(mine), "member layout mismatch"
        for src, dst in zip(lins, mine):
            dst.weight[i].copy_(src.weight)
            dst.bias[i].copy_(src.bias)
        if self.norms is not None:
            for src, dst in zip(lns, self.norms):
                dst.weight[i].copy_(src.weight)
                dst.bias[i].copy_(src.bias)


def orthogonal_init_(module: nn.Module) -> None:
    """SAC-AE ``weight_init`` (``sac_ae/utils.py:67-82``) for ensemble linears: orthogonal per member,
    zero bias."""
    for m in module.modules():
        if isinstance(m, EnsembleLinear):
            with torch.no_grad():
                for i in range(m.n):
                    nn.init.orthogonal_(m.weight.data[i])
                if m.bias is not None:
                    m.bias.zero_()
