"""PPO greedy test episode (reference: ``sheeprl/algos/ppo/utils.py:10-52``)."""
from __future__ import annotations

from typing import Any, Dict

import numpy as np
import torch

from sheeprl_prey_amd.utils.env import make_env


@torch.no_grad()
def test(agent, runner, cfg: Dict[str, Any], log_dir: str) -> float:
    env = make_env(cfg, None, 0, log_dir, "test", vector_env_idx=0)()
    agent.eval()
    done = False
    cumulative_rew = 0.0
    o = env.reset(seed=cfg.seed)[0]
    obs = {}
    keys = list(cfg.cnn_keys.encoder) + list(cfg.mlp_keys.encoder)
    while not done:
        obs = {}
        for k in keys:
            t = torch.as_tensor(np.asarray(o[k]), device=runner.device).unsqueeze(0)
            if k in cfg.cnn_keys.encoder:  # stacked frames x channels -> channels, as the training loop
                t = t.view(1, -1, *t.shape[-2:])
            obs[k] = t.float() / 255 - 0.5 if k in cfg.cnn_keys.encoder else t.float()
        actions = agent.get_greedy_actions(obs)
        if agent.is_continuous:
            act = torch.cat(actions, dim=-1).view(-1).cpu().numpy()
        else:
            act = np.array([a.argmax(dim=-1).item() for a in actions])
            if len(act) == 1:
                act = act[0]
        o, reward, terminated, truncated, _ = env.step(act)
        done = terminated or truncated or cfg.dry_run
        cumulative_rew += float(reward)
    runner.print("Test - Reward:", cumulative_rew)
    if runner.logger is not None:
        runner.logger.log_metrics({"Test/cumulative_reward": cumulative_rew}, 0)
    env.close()
    agent.train()
    return cumulative_rew
