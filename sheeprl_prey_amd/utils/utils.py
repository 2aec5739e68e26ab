"""Misc helpers (reference: ``sheeprl/utils/utils.py``).

``gae`` and ``compute_lambda_values`` dispatch to the HIP scan kernels on GPU tensors
(``sheeprl_prey_amd.ops``); the eager code here is their CPU path and test oracle.
"""
from __future__ import annotations

import copy
import os
from typing import Any, Dict, Optional, Sequence, Tuple

import numpy as np
import torch
from torch import Tensor


class dotdict(dict):
    """Attribute-access dict that stays picklable (reference ``utils.py:13-32``)."""

    __getattr__ = dict.get
    __setattr__ = dict.__setitem__
    __delattr__ = dict.__delitem__

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        for k, v in list(self.items()):
            if isinstance(v, dict) and not isinstance(v, dotdict):
                self[k] = dotdict(v)
            elif isinstance(v, list):
                self[k] = [dotdict(x) if isinstance(x, dict) and not isinstance(x, dotdict) else x for x in v]

    def __getstate__(self):
        return dict(self)

    def __setstate__(self, state):
        self.update(state)

    def __deepcopy__(self, memo=None):
        return dotdict(copy.deepcopy(dict(self), memo=memo))

    def as_dict(self) -> Dict[str, Any]:
        def conv(x):
            if isinstance(x, dict):
                return {k: conv(v) for k, v in x.items()}
            if isinstance(x, list):
                return [conv(v) for v in x]
            return x

        return conv(self)


@torch.no_grad()
def gae(
    rewards: Tensor,
    values: Tensor,
    dones: Tensor,
    next_value: Tensor,
    num_steps: int,
    gamma: float,
    gae_lambda: float,
) -> Tuple[Tensor, Tensor]:
    """Generalised advantage estimation over a [T, N, 1] rollout (reference ``utils.py:35-72``).

    ``dones[t]`` marks that the step *after* t starts a new episode.  GPU tensors run the
    fused reverse-scan HIP kernel (one launch, one lane per env)."""
    if rewards.is_cuda:
        from sheeprl_prey_amd.ops import gae_scan

        return gae_scan(rewards, values, dones, next_value, gamma, gae_lambda)
    lastgaelam = 0
    nextvalues = next_value
    not_dones = torch.logical_not(dones)
    nextnonterminal = not_dones[-1]
    advantages = torch.zeros_like(rewards)
    for t in reversed(range(num_steps)):
        if t < num_steps - 1:
            nextnonterminal = not_dones[t]
            nextvalues = values[t + 1]
        delta = rewards[t] + nextvalues * nextnonterminal * gamma - values[t]
        advantages[t] = lastgaelam = delta + nextnonterminal * lastgaelam * gamma * gae_lambda
    returns = advantages + values
    return returns, advantages


def normalize_tensor(tensor: Tensor, eps: float = 1e-8, mask: Optional[Tensor] = None) -> Tensor:
    if mask is None:  # no boolean indexing: keeps the op free of host syncs (graph-capturable)
        return (tensor - tensor.mean()) / (tensor.std() + eps)
    return (tensor - tensor[mask].mean()) / (tensor[mask].std() + eps)


def polynomial_decay(
    current_step: int, *, initial: float = 1.0, final: float = 0.0, max_decay_steps: int = 100, power: float = 1.0
) -> float:
    if current_step > max_decay_steps or initial == final:
        return final
    return (initial - final) * ((1 - current_step / max_decay_steps) ** power) + final


def symlog(x: Tensor) -> Tensor:
    return torch.sign(x) * torch.log1p(torch.abs(x))


def symexp(x: Tensor) -> Tensor:
    return torch.sign(x) * (torch.exp(torch.abs(x)) - 1)


def init_weights(m: torch.nn.Module) -> None:
    """Kaiming-uniform init, zero bias (reference ``utils/utils.py:75-89``): convolutions with the
    ReLU gain, linears with the default (leaky-ReLU a=0) gain."""
    if isinstance(m, (torch.nn.Conv2d, torch.nn.ConvTranspose2d)):
        torch.nn.init.kaiming_uniform_(m.weight, nonlinearity="relu")
        if m.bias is not None:
            m.bias.data.zero_()
    elif isinstance(m, torch.nn.Linear):
        torch.nn.init.kaiming_uniform_(m.weight)
        if m.bias is not None:
            m.bias.data.zero_()


def print_config(cfg: Dict[str, Any], fields: Sequence[str] = ("algo", "buffer", "checkpoint", "env", "fabric", "metric"), rank: int = 0) -> None:
    """Pretty-print the composed config on rank 0 (reference ``utils.py:128-157``)."""
    if rank != 0:
        return
    try:
        import rich.syntax
        import rich.tree
        import yaml

        tree = rich.tree.Tree("CONFIG", style="dim", guide_style="dim")
        queue = [f for f in fields if f in cfg] + [k for k in cfg if k not in fields and k not in ("hydra", "_choices_")]
        for field in queue:
            branch = tree.add(field, style="dim", guide_style="dim")
            section = cfg[field]
            if isinstance(section, dict):
                content = yaml.safe_dump(dotdict(section).as_dict(), sort_keys=False)
            else:
                content = str(section)
            branch.add(rich.syntax.Syntax(content, "yaml"))
        rich.print(tree)
    except Exception:  # pragma: no cover - printing must never break a run
        print(cfg)


def unwrap(module: torch.nn.Module) -> torch.nn.Module:
    return getattr(module, "module", module)


def save_configs(cfg: Dict[str, Any], log_dir: str) -> None:
    import yaml

    os.makedirs(os.path.join(log_dir, ".hydra"), exist_ok=True)
    plain = dotdict(cfg).as_dict() if isinstance(cfg, dict) else cfg
    with open(os.path.join(log_dir, ".hydra", "config.yaml"), "w") as f:
        yaml.safe_dump(plain, f, sort_keys=False)


def np_seed_everything(seed: int) -> None:
    import random

    random.seed(seed)
    np.random.seed(seed % (2**32))
    torch.manual_seed(seed)
