"""DreamerV2 world-model loss (reference: ``sheeprl/algos/dreamer_v2/loss.py:10-105``).

Unit-variance Gaussian NLLs are written in closed form (``0.5*(x-mu)^2 + 0.5*log(2*pi)`` summed
over the event dims - the exact value of ``Independent(Normal(mu, 1)).log_prob``); the balanced
categorical KL is the fused ``kl_balance`` kernel with ``dyn=alpha, rep=1-alpha`` (both terms are
the same KL value, the kernel routes alpha of the gradient to the prior and 1-alpha to the
posterior)."""
from __future__ import annotations

import math
from typing import Dict, Optional, Tuple

import torch
import torch.nn.functional as F
from torch import Tensor

from sheeprl_prey_amd import ops

HALF_LOG_2PI = 0.5 * math.log(2 * math.pi)


def normal_nll(mean: Tensor, target: Tensor, event_dims: int) -> Tensor:
    """-log N(target | mean, 1) summed over the last ``event_dims`` dims."""
    nll = 0.5 * (target - mean).pow(2) + HALF_LOG_2PI
    return nll.sum(dim=tuple(range(-event_dims, 0))) if event_dims > 0 else nll


def balanced_kl(posteriors_logits: Tensor, priors_logits: Tensor, groups: int, classes: int, alpha: float,
                free_nats: float, free_avg: bool) -> Tuple[Tensor, Tensor]:
    """(kl_loss, kl[T,B]) with DreamerV2 KL balancing."""
    if free_avg:
        per, kl = ops.kl_balance(posteriors_logits, priors_logits, groups, classes, alpha, 1.0 - alpha, 0.0)
        m = kl.mean()
        free = m.new_full((), float(free_nats))  # fill kernel: capturable (no host->device copy)
        return torch.where(m > free, per.mean(), free), kl
    per, kl = ops.kl_balance(posteriors_logits, priors_logits, groups, classes, alpha, 1.0 - alpha, free_nats)
    return per.mean(), kl


def reconstruction_loss(
    recon: Dict[str, Tensor],
    observations: Dict[str, Tensor],
    reward_mean: Tensor,
    rewards: Tensor,
    priors_logits: Tensor,
    posteriors_logits: Tensor,
    groups: int,
    classes: int,
    kl_balancing_alpha: float = 0.8,
    kl_free_nats: float = 0.0,
    kl_free_avg: bool = True,
    kl_regularizer: float = 1.0,
    continue_logits: Optional[Tensor] = None,
    continue_targets: Optional[Tensor] = None,
    discount_scale_factor: float = 1.0,
) -> Tuple[Tensor, Tensor, Tensor, Tensor, Tensor, Tensor]:
    observation_loss = sum(normal_nll(recon[k], observations[k], recon[k].dim() - 2).mean() for k in recon)
    reward_loss = normal_nll(reward_mean, rewards, 1).mean()
    kl_loss, kl = balanced_kl(posteriors_logits, priors_logits, groups, classes, kl_balancing_alpha, kl_free_nats,
                              kl_free_avg)
    if continue_logits is not None and continue_targets is not None:
        continue_loss = discount_scale_factor * F.binary_cross_entropy_with_logits(
            continue_logits, continue_targets, reduction="none").sum(-1).mean()
    else:
        continue_loss = torch.zeros((), device=rewards.device)
    total = kl_regularizer * kl_loss + observation_loss + reward_loss + continue_loss
    return total, kl, kl_loss, reward_loss, observation_loss, continue_loss
