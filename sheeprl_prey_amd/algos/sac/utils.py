"""SAC greedy test episode (reference ``sheeprl/algos/sac/utils.py:10-36``)."""
from __future__ import annotations

from typing import Any, Dict

import numpy as np
import torch

from sheeprl_prey_amd.utils.env import make_env

AGGREGATOR_KEYS = {"Rewards/rew_avg", "Game/ep_len_avg", "Loss/value_loss", "Loss/policy_loss", "Loss/alpha_loss"}


def obs_to_tensor(o: Dict[str, Any], mlp_keys, device, n: int = 1) -> torch.Tensor:
    return torch.cat([torch.as_tensor(np.asarray(o[k]), dtype=torch.float32).reshape(n, -1) for k in mlp_keys],
                     dim=-1).to(device)


@torch.no_grad()
def test(actor, runner, cfg: Dict[str, Any], log_dir: str) -> float:
    env = make_env(cfg, cfg.seed, 0, log_dir, "test", vector_env_idx=0)()
    actor.eval()
    done = False
    cumulative_rew = 0.0
    o = env.reset(seed=cfg.seed)[0]
    while not done:
        obs = obs_to_tensor(o, cfg.mlp_keys.encoder, runner.device)
        action = actor.get_greedy_actions(obs)
        o, reward, terminated, truncated, _ = env.step(action.cpu().numpy().reshape(env.action_space.shape))
        done = terminated or truncated or cfg.dry_run
        cumulative_rew += float(reward)
    runner.print("Test - Reward:", cumulative_rew)
    if runner.logger is not None:
        runner.logger.log_metrics({"Test/cumulative_reward": cumulative_rew}, 0)
    env.close()
    actor.train()
    return cumulative_rew
