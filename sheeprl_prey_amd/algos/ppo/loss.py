"""PPO losses (reference: ``sheeprl/algos/ppo/loss.py:6-72``)."""
from __future__ import annotations

import torch
import torch.nn.functional as F
from torch import Tensor


def _reduce(x: Tensor, reduction: str) -> Tensor:
    reduction = reduction.lower()
    if reduction == "none":
        return x
    if reduction == "mean":
        return x.mean()
    if reduction == "sum":
        return x.sum()
    raise ValueError(f"Unrecognized reduction: {reduction}")


def policy_loss(new_logprobs: Tensor, logprobs: Tensor, advantages: Tensor, clip_coef: float, reduction: str = "mean") -> Tensor:
    """Clipped surrogate objective (PPO eq. 7)."""
    ratio = (new_logprobs - logprobs).exp()
    pg1 = advantages * ratio
    pg2 = advantages * torch.clamp(ratio, 1 - clip_coef, 1 + clip_coef)
    return _reduce(-torch.min(pg1, pg2), reduction)


def value_loss(new_values: Tensor, old_values: Tensor, returns: Tensor, clip_coef: float, clip_vloss: bool,
               reduction: str = "mean") -> Tensor:
    pred = new_values if not clip_vloss else old_values + torch.clamp(new_values - old_values, -clip_coef, clip_coef)
    return F.mse_loss(pred, returns, reduction=reduction)


def entropy_loss(entropy: Tensor, reduction: str = "mean") -> Tensor:
    return _reduce(-entropy, reduction)
