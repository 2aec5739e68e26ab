"""DreamerV3 utilities (reference: ``sheeprl/algos/dreamer_v3/utils.py:16-207``)."""
from __future__ import annotations

import os
from typing import Any, Dict

import numpy as np
import torch
from torch import Tensor

from sheeprl_prey_amd import ops
from sheeprl_prey_amd.utils.env import make_env


def _ranks(n: int, q: float):
    pos = q * (n - 1)
    lo = int(np.floor(pos))
    return lo, min(lo + 1, n - 1), pos - lo


def quantile(x: Tensor, q: float) -> Tensor:
    """``torch.quantile(x, q)`` (linear interpolation) built from a sort with host-constant
    indices, so it is hipGraph-capturable."""
    flat = x.reshape(-1)
    n = flat.numel()
    s, _ = torch.sort(flat)
    pos = q * (n - 1)
    lo = int(np.floor(pos))
    hi = min(lo + 1, n - 1)
    frac = pos - lo
    return s[lo] + (s[hi] - s[lo]) * frac


class Moments(torch.nn.Module):
    """Percentile EMA used to normalise the returns; percentiles over ALL ranks (all-gather)."""

    def __init__(self, runner, decay: float = 0.99, max_: float = 1e8, percentile_low: float = 0.05,
                 percentile_high: float = 0.95) -> None:
        super().__init__()
        self._runner = runner
        self._decay = decay
        self._max = float(max_)
        self._percentile_low = percentile_low
        self._percentile_high = percentile_high
        self.register_buffer("low", torch.zeros((), dtype=torch.float32))
        self.register_buffer("high", torch.zeros((), dtype=torch.float32))
        self.register_buffer("_invscale", torch.zeros((), dtype=torch.float32), persistent=False)

    def gather(self, x: Tensor) -> Tensor:
        return self._runner.all_gather(x.detach()) if self._runner is not None else x.detach()

    def update(self, gathered: Tensor):
        if ops._native(gathered) and gathered.dtype == torch.float32:
            # one radix-select launch (moments.hip): both percentiles, the EMA and the scale, in place
            g = gathered.detach().reshape(-1).contiguous()
            l0, l1, fl = _ranks(g.numel(), self._percentile_low)
            h0, h1, fh = _ranks(g.numel(), self._percentile_high)
            ops._ext().moments_update(g, [l0, l1, h0, h1], [fl, fh], float(self._decay), float(self._max), self.low,
                                      self.high, self._invscale)
            return self.low.detach(), self._invscale.detach()
        low = quantile(gathered, self._percentile_low)
        high = quantile(gathered, self._percentile_high)
        # in place: the buffers stay the same tensors across hipGraph replays
        self.low.mul_(self._decay).add_((1 - self._decay) * low)
        self.high.mul_(self._decay).add_((1 - self._decay) * high)
        invscale = torch.clamp(self.high - self.low, min=1.0 / self._max)
        return self.low.detach(), invscale.detach()

    def forward(self, x: Tensor):
        return self.update(self.gather(x))


def compute_lambda_values(rewards: Tensor, values: Tensor, continues: Tensor, lmbda: float = 0.95) -> Tensor:
    """DreamerV3 lambda returns; one HIP reverse-scan kernel on GPU."""
    return ops.lambda_returns(rewards, values, continues, lmbda)


@torch.no_grad()
def test(player, runner, cfg: Dict[str, Any], log_dir: str, test_name: str = "", sample_actions: bool = False,
         render: bool = False, obs_offset: float = 0.0) -> float:
    """One greedy (or sampled) episode; logs ``Test/cumulative_reward``."""
    env = make_env(cfg, cfg.seed, 0, log_dir, "test" + (f"_{test_name}" if test_name != "" else ""))()
    done = False
    cumulative_rew = 0.0
    device = runner.device
    next_obs = env.reset(seed=cfg.seed)[0]
    player.num_envs = 1
    player.init_states()
    while not done:
        pre = {}
        for k, v in next_obs.items():
            t = torch.as_tensor(np.asarray(v), device=device).view(1, 1, *np.asarray(v).shape).float()
            if k in cfg.cnn_keys.encoder:
                pre[k] = t / 255 + obs_offset
            elif k in cfg.mlp_keys.encoder:
                pre[k] = t
        mask = {k: v for k, v in pre.items() if k.startswith("mask")} or None
        real_actions = player.get_greedy_action(pre, sample_actions, mask)
        if player.actor.is_continuous:
            real_actions = torch.cat(real_actions, -1).cpu().numpy()
        else:
            real_actions = np.array([a.cpu().argmax(dim=-1).numpy() for a in real_actions])
        next_obs, reward, done, truncated, _ = env.step(real_actions.reshape(env.action_space.shape))
        if render:
            env.render()
        done = done or truncated or cfg.dry_run
        cumulative_rew += float(reward)
    runner.print("Test - Reward:", cumulative_rew)
    if runner.logger is not None:
        runner.logger.log_metrics({"Test/cumulative_reward": cumulative_rew}, 0)
    env.close()
    return cumulative_rew
