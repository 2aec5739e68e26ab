"""Recurrent PPO greedy test episode (reference ``sheeprl/algos/ppo_recurrent/utils.py:13-66``)."""
from __future__ import annotations

from typing import Any, Dict

import numpy as np
import torch

from sheeprl_prey_amd.utils.env import make_env


@torch.no_grad()
def test(agent, runner, cfg: Dict[str, Any], log_dir: str) -> float:
    env = make_env(cfg, None, 0, log_dir, "test", vector_env_idx=0)()
    agent.eval()
    dev = runner.device

    def to_obs(o):
        out = {k: torch.as_tensor(np.asarray(o[k]), dtype=torch.float32, device=dev).view(1, 1, -1, *np.asarray(o[k]).shape[-2:]) / 255
               for k in cfg.cnn_keys.encoder}
        out.update({k: torch.as_tensor(np.asarray(o[k]), dtype=torch.float32, device=dev).view(1, 1, -1)
                    for k in cfg.mlp_keys.encoder})
        return out

    done = False
    cumulative_rew = 0.0
    obs = to_obs(env.reset(seed=cfg.seed)[0])
    state = (torch.zeros(1, 1, agent.rnn_hidden_size, device=dev), torch.zeros(1, 1, agent.rnn_hidden_size, device=dev))
    actions = torch.zeros(1, 1, sum(agent.actions_dim), device=dev)
    while not done:
        acts, state = agent.get_greedy_actions(obs, state, actions)
        if agent.is_continuous:
            real = torch.cat(acts, -1)
        else:
            real = torch.cat([a.argmax(-1) for a in acts], -1)
        actions = torch.cat(acts, -1).view(1, 1, -1)
        o, reward, terminated, truncated, _ = env.step(real.cpu().numpy().reshape(env.action_space.shape))
        done = terminated or truncated or cfg.dry_run
        cumulative_rew += float(reward)
        obs = to_obs(o)
    runner.print("Test - Reward:", cumulative_rew)
    if runner.logger is not None:
        runner.logger.log_metrics({"Test/cumulative_reward": cumulative_rew}, 0)
    env.close()
    agent.train()
    return cumulative_rew
