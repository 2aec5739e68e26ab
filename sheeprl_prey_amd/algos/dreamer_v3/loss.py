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
    dones: Optional[Tensor] = None,
) -> Tuple[Tensor, Tensor, Tensor, Tensor, Tensor, Tensor]:
    """Eq. 5 of the DreamerV3 paper.  ``obs_losses`` is the per-(t,b) observation NLL already
    summed over keys.  Returns (total, kl, kl_loss, reward_loss, observation_loss, continue_loss) -
    the last five as means (logged metrics).  ``entropies``: receives the per-(t,b) posterior and
    prior entropies (``ops.kl_balance``).  ``dones``: when given (GPU), the continue targets are
    ``1 - dones`` and the assembly runs as one fused kernel each way."""
    reward_loss = ops.twohot_nll(reward_logits, rewards)
    kl_loss, kl = ops.kl_balance(posteriors_logits, priors_logits, groups, classes, kl_dynamic, kl_representation, kl_free_nats,
                                 entropies=entropies)
    if (dones is not None and ops._native(reward_loss) and all(
            t.dtype == torch.float32 for t in (kl_loss, obs_losses, reward_loss, kl, dones))
            and (continue_logits is None or continue_logits.numel() == reward_loss.numel())):
        # continue BCE + weighted sum + mean + the five metric means: one kernel each way (wm_loss.hip)
        return _WMLoss.apply(kl_loss, obs_losses, reward_loss, continue_logits, dones, kl, float(kl_regularizer),
                             float(continue_scale_factor))
    if continue_targets is None and dones is not None:
        continue_targets = 1 - dones
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


class _WMLoss(torch.autograd.Function):
    """Fused world-model loss assembly (``ops/csrc/wm_loss.hip``): per-row terms in, (total, metric
    means) out; backward: the per-row gradients of the total."""

    @staticmethod
    def forward(ctx, kl_loss, obs, rew, logits, dones, kl, kl_reg, scale):
        ctx.set_materialize_grads(False)  # unused outputs: None, not a zero-filled tensor (one fill launch each)
        C = ops._ext()
        R = kl_loss.numel()
        lg = logits.detach().contiguous().view(-1) if logits is not None else None
        dn = dones.detach().contiguous().view(-1).float() if logits is not None else None
        total, means = C.wm_loss_fwd(kl_loss.contiguous().view(-1), obs.contiguous().view(-1), rew.contiguous().view(-1),
                                     lg, dn, kl.detach().contiguous().view(-1), kl_reg, scale)
        ctx.save_for_backward(lg, dn)
        ctx.cfg = (R, kl_reg, scale, kl_loss.shape, obs.shape, rew.shape, None if logits is None else logits.shape)
        m = means.unbind(0)
        ctx.mark_non_differentiable(*m)
        return (total, *m)

    @staticmethod
    def backward(ctx, g, *_):
        if g is None:
            return (None,) * 8
        lg, dn = ctx.saved_tensors
        R, kl_reg, scale, s_kll, s_obs, s_rew, s_lg = ctx.cfg
        d_kll, d_obs, d_rew, d_lg = ops._ext().wm_loss_bwd(lg, dn, g.contiguous().view(1), R, kl_reg, scale)
        return (d_kll.view(s_kll), d_obs.view(s_obs), d_rew.view(s_rew), None if d_lg is None else d_lg.view(s_lg),
                None, None, None, None)
