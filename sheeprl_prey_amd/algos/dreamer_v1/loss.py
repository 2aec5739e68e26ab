"""DreamerV1 losses (reference: ``sheeprl/algos/dreamer_v1/loss.py:9-94``)."""
from __future__ import annotations

from typing import Dict, Optional, Tuple

import torch
import torch.nn.functional as F
from torch import Tensor

from sheeprl_prey_amd.algos.dreamer_v2.loss import normal_nll


def diag_normal_kl(m1: Tensor, s1: Tensor, m2: Tensor, s2: Tensor) -> Tensor:
    """KL(N(m1, s1) || N(m2, s2)) summed over the last dim (diagonal Gaussians)."""
    var_ratio = (s1 / s2).pow(2)
    t1 = ((m1 - m2) / s2).pow(2)
    return (0.5 * (var_ratio + t1 - 1 - var_ratio.log())).sum(-1)


def critic_loss(qv_mean: Tensor, lambda_values: Tensor, discount: Tensor) -> Tensor:
    """-mean(discount * log N(lambda | qv, 1))."""
    return torch.mean(discount * normal_nll(qv_mean, lambda_values, 1))


def actor_loss(lambda_values: Tensor) -> Tensor:
    return -torch.mean(lambda_values)


def reconstruction_loss(
    recon: Dict[str, Tensor], observations: Dict[str, Tensor], reward_mean: Tensor, rewards: Tensor,
    post_mean: Tensor, post_std: Tensor, prior_mean: Tensor, prior_std: Tensor, kl_free_nats: float = 3.0,
    kl_regularizer: float = 1.0, continue_logits: Optional[Tensor] = None, continue_targets: Optional[Tensor] = None,
    continue_scale_factor: float = 10.0,
) -> Tuple[Tensor, Tensor, Tensor, Tensor, Tensor, Tensor]:
    observation_loss = sum(normal_nll(recon[k], observations[k], recon[k].dim() - 2).mean() for k in recon)
    reward_loss = normal_nll(reward_mean, rewards, 1).mean()
    kl = diag_normal_kl(post_mean, post_std, prior_mean, prior_std).mean()
    state_loss = torch.clamp(kl, min=kl_free_nats)
    if continue_logits is not None and continue_targets is not None:
        # the reference adds +log p (a sign slip that also breaks its scalar backward); the NLL is used here
        continue_loss = continue_scale_factor * F.binary_cross_entropy_with_logits(
            continue_logits, continue_targets, reduction="none").sum(-1).mean()
    else:
        continue_loss = torch.zeros((), device=rewards.device)
    total = kl_regularizer * state_loss + observation_loss + reward_loss + continue_loss
    return total, kl, state_loss, reward_loss, observation_loss, continue_loss
