"""Evaluation / visualisation of trained agents (the fork's ``eval.py`` and ``visulize.py``, which
hard-code one DreamerV3 prey checkpoint and call ``test``/``test_vis``).

    python -m sheeprl_prey_amd.evaluate checkpoint_path=<run>/version_0/checkpoint/ckpt_X_0.ckpt \
        [episodes=5] [sample_actions=True] [render=True] [device=cuda] [env.env_type=test ...]
    sheeprl-eval checkpoint_path=...

The run's saved ``.hydra/config.yaml`` is reloaded (any further ``a.b=value`` arguments override
it), the models are rebuilt for the run's algorithm, weights are loaded with
``torch.load(weights_only=True)`` and ``episodes`` test episodes are played; with ``render=True``
every episode's ``rgb_array`` frames are written as an animated GIF next to the checkpoint (the
fork's visualiser opens a matplotlib window instead).  Returns the per-episode returns.
"""
from __future__ import annotations

import os
import pathlib
import sys
from typing import Any, Dict, List, Optional

import numpy as np
import torch
import yaml

from sheeprl_prey_amd.config.compose import parse_override
from sheeprl_prey_amd.utils.utils import dotdict

_EVAL_KEYS = ("checkpoint_path", "episodes", "sample_actions", "render", "device", "seed", "video_dir")


def _load_run_config(ckpt: pathlib.Path) -> dotdict:
    for cand in (ckpt.parent.parent.parent / ".hydra" / "config.yaml", ckpt.parent.parent / ".hydra" / "config.yaml"):
        if cand.exists():
            with open(cand) as f:
                return dotdict(yaml.safe_load(f))
    raise FileNotFoundError(f"No .hydra/config.yaml found for checkpoint {ckpt}")


def _set(cfg: Dict[str, Any], key: str, value: Any) -> None:
    node = cfg
    parts = key.split(".")
    for p in parts[:-1]:
        node = node.setdefault(p, dotdict({}))
    node[parts[-1]] = value


class _EvalRunner:
    """The minimal runner surface the players / test helpers need (single process, no collectives)."""

    def __init__(self, device: str):
        self.device = torch.device(device)
        self.world_size = 1
        self.global_rank = 0
        self.is_global_zero = True
        self.logger = None

    def setup_module(self, m):
        return m.to(self.device)

    def print(self, *a, **k):
        print(*a, **k)


def _build_player(cfg, state, runner, obs_space, action_space):
    from sheeprl_prey_amd.algos.common import action_info

    is_continuous, _, actions_dim = action_info(action_space)
    algo = cfg.algo.name
    if algo in ("dreamer_v3",):
        from sheeprl_prey_amd.algos.dreamer_v3.agent import PlayerDV3, build_models

        wm, actor, _, _ = build_models(runner, actions_dim, is_continuous, cfg, obs_space, state["world_model"],
                                       state["actor"], state["critic"], state["target_critic"])
        return PlayerDV3(wm.encoder, wm.rssm, actor, actions_dim, cfg.algo.player.expl_amount, 1,
                         cfg.algo.world_model.stochastic_size, cfg.algo.world_model.recurrent_model.recurrent_state_size,
                         runner.device, discrete_size=cfg.algo.world_model.discrete_size), 0.0
    if algo in ("dreamer_v2", "p2e_dv2"):
        from sheeprl_prey_amd.algos.dreamer_v2.agent import PlayerDV2

        if algo == "dreamer_v2":
            from sheeprl_prey_amd.algos.dreamer_v2.agent import build_models

            wm, actor, _, _ = build_models(runner, actions_dim, is_continuous, cfg, obs_space, state["world_model"],
                                           state["actor"], state["critic"], state["target_critic"])
        else:
            from sheeprl_prey_amd.algos.p2e_dv2.agent import build_models

            wm, actor, *_ = build_models(runner, actions_dim, is_continuous, cfg, obs_space, state["world_model"],
                                         state["actor_task"], state["critic_task"], state["target_critic_task"],
                                         state["actor_exploration"], state["critic_exploration"],
                                         state["target_critic_exploration"])
        return PlayerDV2(wm.encoder, wm.rssm.recurrent_model, wm.rssm.representation_model, actor, actions_dim,
                         cfg.algo.player.expl_amount, 1, cfg.algo.world_model.stochastic_size,
                         cfg.algo.world_model.recurrent_model.recurrent_state_size, runner.device,
                         discrete_size=cfg.algo.world_model.discrete_size), -0.5
    if algo in ("dreamer_v1", "p2e_dv1"):
        from sheeprl_prey_amd.algos.dreamer_v1.agent import PlayerDV1

        if algo == "dreamer_v1":
            from sheeprl_prey_amd.algos.dreamer_v1.agent import build_models

            wm, actor, _ = build_models(runner, actions_dim, is_continuous, cfg, obs_space, state["world_model"],
                                        state["actor"], state["critic"])
        else:
            from sheeprl_prey_amd.algos.p2e_dv1.agent import build_models

            wm, actor, *_ = build_models(runner, actions_dim, is_continuous, cfg, obs_space, state["world_model"],
                                         state["actor_task"], state["critic_task"], state["actor_exploration"],
                                         state["critic_exploration"])
        return PlayerDV1(wm.encoder, wm.rssm.recurrent_model, wm.rssm.representation_model, actor, actions_dim,
                         cfg.algo.player.expl_amount, 1, cfg.algo.world_model.stochastic_size,
                         cfg.algo.world_model.recurrent_model.recurrent_state_size, runner.device,
                         min_std=cfg.algo.world_model.min_std), -0.5
    raise ValueError(f"evaluation is implemented for the Dreamer family (got algo `{algo}`); the model-free "
                     "agents run their greedy `test` at the end of training")


@torch.no_grad()
def evaluate(checkpoint_path: str, overrides: Optional[List[str]] = None, episodes: int = 1,
             sample_actions: bool = True, render: bool = False, device: str = "cpu", seed: Optional[int] = None,
             video_dir: Optional[str] = None) -> List[float]:
    from sheeprl_prey_amd.utils.env import make_env

    ckpt = pathlib.Path(checkpoint_path)
    cfg = _load_run_config(ckpt)
    for o in overrides or []:
        ov = parse_override(o)
        _set(cfg, ov.key, ov.value)
    cfg.env.num_envs = 1
    cfg.env.capture_video = False
    cfg.dry_run = False
    if seed is not None:
        cfg.seed = seed
    if render:
        cfg.env.wrapper["render_mode"] = "rgb_array"
    runner = _EvalRunner(device)
    state = torch.load(str(ckpt), map_location="cpu", weights_only=True)
    env = make_env(cfg, cfg.seed, 0, None, "eval")()
    player, offset = _build_player(cfg, state, runner, env.observation_space, env.action_space)
    returns: List[float] = []
    out_dir = video_dir or str(ckpt.parent / "eval_videos")
    for ep in range(episodes):
        o, _ = env.reset(seed=int(cfg.seed) + ep)
        player.num_envs = 1
        player.init_states()
        frames = []
        done, total = False, 0.0
        while not done:
            pre = {}
            for k, v in o.items():
                t = torch.as_tensor(np.asarray(v), device=runner.device).view(1, 1, *np.asarray(v).shape).float()
                if k in cfg.cnn_keys.encoder:
                    pre[k] = t / 255 + offset
                elif k in cfg.mlp_keys.encoder:
                    pre[k] = t
            acts = player.get_greedy_action(pre, sample_actions, None)
            if player.actor.is_continuous:
                a = torch.cat(acts, -1).cpu().numpy()
            else:
                a = np.array([x.cpu().argmax(dim=-1).numpy() for x in acts])
            o, r, term, trunc, _ = env.step(a.reshape(env.action_space.shape))
            total += float(r)
            done = bool(term or trunc)
            if render:
                f = env.render()
                if f is not None:
                    frames.append(np.asarray(f))
        returns.append(total)
        print(f"Episode {ep}: return {total:.3f}")
        if render and frames:
            from PIL import Image

            os.makedirs(out_dir, exist_ok=True)
            imgs = [Image.fromarray(f) for f in frames]
            path = os.path.join(out_dir, f"{cfg.env.id}_ep{ep}.gif")
            imgs[0].save(path, save_all=True, append_images=imgs[1:], duration=33, loop=0)
            print("saved", path)
    env.close()
    print(f"Mean return over {episodes} episode(s): {float(np.mean(returns)):.3f}")
    return returns


def evaluate_from_cli(argv: List[str]) -> List[float]:
    kw: Dict[str, Any] = {}
    rest = []
    for a in argv:
        key = a.split("=", 1)[0]
        if key in _EVAL_KEYS:
            kw[key] = parse_override(a).value
        else:
            rest.append(a)
    if "checkpoint_path" not in kw:
        raise ValueError("usage: sheeprl-eval checkpoint_path=<ckpt> [episodes=N] [render=True] [a.b=value ...]")
    kw["checkpoint_path"] = str(kw["checkpoint_path"])
    return evaluate(overrides=rest, **kw)


if __name__ == "__main__":
    evaluate_from_cli(sys.argv[1:])
