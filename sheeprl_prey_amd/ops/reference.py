"""Eager PyTorch implementations of every fused op.

They are (1) the CPU execution path and (2) the fp32 oracles the HIP kernels are tested
against.  Each mirrors the reference's eager math:
``LayerNormGRUCell`` (models.py:362-402), ``RSSM._uniform_mix`` + ``compute_stochastic_state``
(dreamer_v3/agent.py:390-437), ``TwoHotEncodingDistribution`` (distribution.py:224-270),
the KL balancing of ``dreamer_v3/loss.py:65-110``, ``compute_lambda_values``
(dreamer_v3/utils.py:44-55) and ``gae`` (utils.py:35-72).
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch
import torch.nn.functional as F
from torch import Tensor

ACTS = {"none": 0, "identity": 0, "silu": 1, "elu": 2, "relu": 3, "tanh": 4}


def act_fn(z: Tensor, act: str) -> Tensor:
    if act == "silu":
        return F.silu(z)
    if act == "elu":
        return F.elu(z)
    if act == "relu":
        return F.relu(z)
    if act == "tanh":
        return torch.tanh(z)
    return z


def ln_act(x: Tensor, weight: Optional[Tensor], bias: Optional[Tensor], eps: float, act: str) -> Tensor:
    y = F.layer_norm(x, x.shape[-1:], weight, bias, eps)
    return act_fn(y, act)


def ln_act_nchw(x: Tensor, weight: Optional[Tensor], bias: Optional[Tensor], eps: float, act: str) -> Tensor:
    y = F.layer_norm(x.permute(0, 2, 3, 1), x.shape[1:2], weight, bias, eps).permute(0, 3, 1, 2)
    return act_fn(y, act)


def ln_gru(x: Tensor, h: Tensor, weight: Tensor, bias: Tensor, eps: float) -> Tensor:
    z = F.layer_norm(x, x.shape[-1:], weight, bias, eps)
    reset, cand, update = torch.chunk(z, 3, -1)
    reset = torch.sigmoid(reset)
    cand = torch.tanh(reset * cand)
    update = torch.sigmoid(update - 1)
    return update * cand + (1 - update) * h


def unimix_logits(logits: Tensor, classes: int, unimix: float) -> Tensor:
    if unimix <= 0.0:
        return logits
    shape = logits.shape
    lg = logits.reshape(*shape[:-1], -1, classes)
    probs = lg.softmax(-1)
    probs = (1 - unimix) * probs + unimix / classes
    eps = torch.finfo(probs.dtype).eps
    return torch.log(probs.clamp(min=eps, max=1 - eps)).reshape(shape)


def unimix_sample(
    logits: Tensor, classes: int, unimix: float, uniform: Optional[Tensor] = None, sample: bool = True,
    forced: Optional[Tensor] = None,
) -> Tuple[Tensor, Tensor]:
    """Returns (mixed_logits, one_hot_straight_through_sample or mode).  ``forced`` (one-hot, logits' shape):
    the sample to take instead of drawing one (teacher forcing of an oracle run, straight-through grads
    still through these logits' probabilities)."""
    mixed = unimix_logits(logits, classes, unimix)
    shape = mixed.shape
    m = mixed.reshape(-1, classes)
    probs = m.softmax(-1)
    if sample and forced is not None:
        st = forced.reshape(-1, classes).to(probs) + probs - probs.detach()
    elif sample:
        if uniform is None:
            idx = torch.multinomial(probs.detach(), 1).squeeze(-1)
        else:
            cdf = probs.detach().cumsum(-1)
            u = uniform.reshape(-1, 1) * cdf[:, -1:]
            idx = (cdf < u).sum(-1).clamp(max=classes - 1)
        onehot = F.one_hot(idx, classes).to(probs)
        st = onehot + probs - probs.detach()
    else:
        st = F.one_hot(probs.argmax(-1), classes).to(probs)
    return mixed, st.reshape(shape)


def twohot_bins(num_bins: int, low: float, high: float, device=None) -> Tensor:
    return torch.linspace(low, high, num_bins, device=device)


def symlog(x: Tensor) -> Tensor:
    return torch.sign(x) * torch.log1p(torch.abs(x))


def symexp(x: Tensor) -> Tensor:
    return torch.sign(x) * (torch.exp(torch.abs(x)) - 1)


def twohot_nll(logits: Tensor, target: Tensor, bins: Tensor) -> Tensor:
    """-log_prob of the two-hot encoded symlog(target); logits [..., K], target [...] -> [...]."""
    x = symlog(target).unsqueeze(-1)
    K = bins.numel()
    below = (bins <= x).to(torch.int32).sum(-1, keepdim=True) - 1
    above = K - (bins > x).to(torch.int32).sum(-1, keepdim=True)
    below = below.clamp(0, K - 1).long()
    above = above.clamp(0, K - 1).long()
    equal = below == above
    d_below = torch.where(equal, torch.ones_like(x), (bins[below] - x).abs())
    d_above = torch.where(equal, torch.ones_like(x), (bins[above] - x).abs())
    total = d_below + d_above
    w_below = d_above / total
    w_above = d_below / total
    tgt = F.one_hot(below.squeeze(-1), K) * w_below + F.one_hot(above.squeeze(-1), K) * w_above
    logp = logits - torch.logsumexp(logits, -1, keepdim=True)
    return -(tgt * logp).sum(-1)


def twohot_mean(logits: Tensor, bins: Tensor) -> Tensor:
    return symexp((logits.softmax(-1) * bins).sum(-1))


def kl_balance(
    post: Tensor, prior: Tensor, groups: int, classes: int, dyn: float, rep: float, free_nats: float
) -> Tuple[Tensor, Tensor]:
    """Returns (loss, kl) per row; gradients follow the reference's stop-gradient routing."""
    a = post.reshape(-1, groups, classes)
    b = prior.reshape(-1, groups, classes)

    def kl(p_logits, q_logits):
        lp = p_logits.log_softmax(-1)
        lq = q_logits.log_softmax(-1)
        return (lp.exp() * (lp - lq)).sum(-1).sum(-1)

    free = torch.tensor(free_nats, device=post.device, dtype=post.dtype)
    dyn_kl = kl(a.detach(), b)
    rep_kl = kl(a, b.detach())
    loss = dyn * torch.maximum(dyn_kl, free) + rep * torch.maximum(rep_kl, free)
    return loss.reshape(post.shape[:-1]), dyn_kl.detach().reshape(post.shape[:-1])


def lambda_returns(rewards: Tensor, values: Tensor, continues: Tensor, lmbda: float) -> Tensor:
    vals = [values[-1:]]
    interm = rewards + continues * values * (1 - lmbda)
    for t in reversed(range(len(continues))):
        vals.append(interm[t : t + 1] + continues[t : t + 1] * lmbda * vals[-1])
    return torch.cat(list(reversed(vals))[:-1])


@torch.no_grad()
def gae(rewards, values, dones, next_value, gamma, lam):
    T = rewards.shape[0]
    not_dones = 1.0 - dones.float()
    adv = torch.zeros_like(rewards)
    last = torch.zeros_like(rewards[0])
    nnt = not_dones[-1]
    nv = next_value.reshape(rewards[0].shape)
    for t in reversed(range(T)):
        if t < T - 1:
            nnt = not_dones[t]
            nv = values[t + 1]
        delta = rewards[t] + nv * nnt * gamma - values[t]
        last = delta + nnt * last * gamma * lam
        adv[t] = last
    return adv + values, adv


def squashed_gaussian(mean: Tensor, log_std: Tensor, eps: Tensor, scale: Tensor, bias: Tensor, mode: int, lo: float,
                      hi: float):
    """Eager oracle of the tanh-squashed Gaussian head (reference ``sac/agent.py:100-138``,
    ``sac_ae/agent.py:283-320``): returns (action, logp[..., 1])."""
    if mode == 0:
        ls = torch.clamp(log_std, lo, hi)
    else:
        ls = lo + 0.5 * (hi - lo) * (torch.tanh(log_std) + 1)
    std = ls.exp()
    x = mean + std * eps
    y = torch.tanh(x)
    action = y * scale + bias
    logp = -0.5 * eps.pow(2) - ls - 0.5 * math.log(2 * math.pi)
    logp = logp - torch.log(scale * (1 - y.pow(2)) + 1e-6)
    return action, logp.sum(-1, keepdim=True)


# ---------------------------------------------------------------- truncated normal (K16)
_SQRT2 = math.sqrt(2.0)
_LOG_INV_SQRT_2PI = -0.5 * math.log(2.0 * math.pi)


def truncnorm_terms(loc: Tensor, scale: Tensor, lo: Tensor, hi: Tensor) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    """Standardised bounds (alpha, beta), Phi(alpha) and the mass Z = max(Phi(beta) - Phi(alpha), eps)."""
    alpha = (lo - loc) / scale
    beta = (hi - loc) / scale
    cdf_a = 0.5 * (1.0 + torch.erf(alpha / _SQRT2))
    cdf_b = 0.5 * (1.0 + torch.erf(beta / _SQRT2))
    Z = (cdf_b - cdf_a).clamp_min(torch.finfo(loc.dtype).eps)
    return alpha, beta, cdf_a, Z


def truncnorm_rsample(loc: Tensor, scale: Tensor, lo: Tensor, hi: Tensor, u: Tensor) -> Tensor:
    """Inverse-CDF sample loc + scale * Phi^-1(Phi(alpha) + u Z) (reference distribution.py:97-112, 139-140)."""
    _, _, cdf_a, Z = truncnorm_terms(loc, scale, lo, hi)
    return loc + scale * (_SQRT2 * torch.erfinv(2.0 * (cdf_a + u * Z) - 1.0))


def truncnorm_log_prob(value: Tensor, loc: Tensor, scale: Tensor, lo: Tensor, hi: Tensor) -> Tensor:
    """-log sqrt(2 pi) - log Z - z^2 / 2 - log scale (reference distribution.py:102-105, 142-143)."""
    _, _, _, Z = truncnorm_terms(loc, scale, lo, hi)
    z = (value - loc) / scale
    return _LOG_INV_SQRT_2PI - Z.log() - 0.5 * z * z - scale.log()
