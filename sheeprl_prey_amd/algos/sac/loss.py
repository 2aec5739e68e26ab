"""SAC losses (reference ``sheeprl/algos/sac/loss.py:10-26``; "Soft Actor-Critic Algorithms and
Applications", arXiv:1812.05905)."""
from __future__ import annotations

from typing import Union

import torch
from torch import Tensor


def policy_loss(alpha: Union[float, Tensor], logprobs: Tensor, qf_values: Tensor) -> Tensor:
    """Eq. 7."""
    return ((alpha * logprobs) - qf_values).mean()


def critic_loss(qf_values: Tensor, next_qf_value: Tensor, num_critics: int) -> Tensor:
    """Eq. 5, summed over critics: ``sum_i mean((Q_i - y)^2)`` - for the ``[B, n]`` ensemble output
    this is ``n * mean((Q - y)^2)`` computed in one reduction."""
    return (qf_values - next_qf_value).pow(2).mean() * num_critics


def entropy_loss(log_alpha: Tensor, logprobs: Tensor, target_entropy: Tensor) -> Tensor:
    """Eq. 17."""
    return (-log_alpha * (logprobs + target_entropy)).mean()
