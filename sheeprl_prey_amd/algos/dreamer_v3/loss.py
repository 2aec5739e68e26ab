"""DreamerV3 world-model loss (reference: ``sheeprl/algos/dreamer_v3/loss.py:11-110``).

KL balancing, two-hot reward NLL and the categorical KL run as fused HIP kernels."""
from __future__ import annotations

from typing import Dict, Optional, Tuple

import torch
import torch.nn.functional as F
from torch import Tensor

from sheeprl_prey_amd import ops


def reconstruction_loss(
    obs_losses: Tensor,
    reward_logits: Tensor,
    rewards: Tensor,
    priors_logits: Tensor,
    posteriors_logits: Tensor,
    groups: int,
    classes: int,
    kl_dynamic: float = 0.5,
    kl_representation: float = 0.1,
    kl_free_nats: float = 1.0,
    kl_regularizer: float = 1.0,
    continue_logits: Optional[Tensor] = None,
    continue_targets: Optional[Tensor] = None,
    continue_scale_factor: float = 1.0,
    entropies: Optional[list] = None,
) -> Tuple[Tensor, Tensor, Tensor, Tensor, Tensor, Tensor]:
    """Eq. 5 of the DreamerV3 paper.  ``obs_losses`` is the per-(t,b) observation NLL already
    summed over keys.  Returns (total, kl, kl_loss, reward_loss, observation_loss, continue_loss).
    ``entropies``: receives the per-(t,b) posterior and prior entropies (``ops.kl_balance``)."""
    reward_loss = ops.twohot_nll(reward_logits, rewards)
    kl_loss, kl = ops.kl_balance(posteriors_logits, priors_logits, groups, classes, kl_dynamic, kl_representation, kl_free_nats,
                                 entropies=entropies)
    if continue_logits is not None and continue_targets is not None:
        continue_loss = continue_scale_factor * F.binary_cross_entropy_with_logits(
            continue_logits, continue_targets, reduction="none").sum(-1)
    else:
        continue_loss = torch.zeros_like(reward_loss)
    total = (kl_regularizer * kl_loss + obs_losses + reward_loss + continue_loss).mean()
    # the five logged means as one reduction (they are metrics: no gradient flows through them)
    with torch.no_grad():
        parts = [kl, kl_loss, reward_loss, obs_losses, continue_loss]
        if len({tuple(p.shape) for p in parts}) == 1:
            m = torch.stack(parts).flatten(1).mean(1)
            return total, m[0], m[1], m[2], m[3], m[4]
    return total, kl.mean(), kl_loss.mean(), reward_loss.mean(), obs_losses.mean(), continue_loss.mean()
