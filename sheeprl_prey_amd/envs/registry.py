"""``make(id)`` - the gymnasium.make role: id -> env instance (+ TimeLimit from the spec)."""
from __future__ import annotations

import importlib
from typing import Any, Callable, Dict, Optional, Union

from sheeprl_prey_amd.envs.core import EnvSpec, TimeLimit

_REGISTRY: Dict[str, EnvSpec] = {}


def register(id: str, entry_point: Union[str, Callable[..., Any]], max_episode_steps: Optional[int] = None, **kwargs) -> None:
    _REGISTRY[id] = EnvSpec(id, entry_point, max_episode_steps, kwargs)


def spec(id: str) -> EnvSpec:
    if id not in _REGISTRY:
        raise KeyError(f"No registered env with id: {id}. Registered: {sorted(_REGISTRY)}")
    return _REGISTRY[id]


def registered_ids():
    return sorted(_REGISTRY)


def _load(entry_point):
    if callable(entry_point):
        return entry_point
    mod, _, attr = entry_point.partition(":")
    return getattr(importlib.import_module(mod), attr)


def make(id: str, render_mode: Optional[str] = None, max_episode_steps: Optional[int] = None, **kwargs):
    if id in ("LunarLander-v2", "LunarLanderContinuous-v2", "BipedalWalker-v3", "CarRacing-v2"):
        from sheeprl_prey_amd.utils.imports import _IS_BOX2D_AVAILABLE

        if not _IS_BOX2D_AVAILABLE:
            raise ModuleNotFoundError(
                f"'{id}' needs the Box2D physics engine, which is not installed in this image. "
                "Use e.g. `env.id=Pendulum-v1` or `env.id=MountainCarContinuous-v0` for continuous control."
            )
    sp = spec(id)
    params = dict(sp.kwargs)
    params.update(kwargs)
    if render_mode is not None and render_mode != "None":
        params["render_mode"] = render_mode
    env = _load(sp.entry_point)(**params)
    env.spec = sp
    steps = max_episode_steps if max_episode_steps is not None else sp.max_episode_steps
    if steps:
        env = TimeLimit(env, steps)
    return env


register("CartPole-v0", "sheeprl_prey_amd.envs.classic:CartPoleEnv", max_episode_steps=200)
register("CartPole-v1", "sheeprl_prey_amd.envs.classic:CartPoleEnv", max_episode_steps=500)
register("Pendulum-v1", "sheeprl_prey_amd.envs.classic:PendulumEnv", max_episode_steps=200)
register("MountainCar-v0", "sheeprl_prey_amd.envs.classic:MountainCarEnv", max_episode_steps=200)
register("MountainCarContinuous-v0", "sheeprl_prey_amd.envs.classic:MountainCarContinuousEnv", max_episode_steps=999)
register("prey_d_1", "sheeprl_prey_amd.envs.prey.env:PreyEnv", max_episode_steps=None)
# dm_control walker_walk-shaped synthetic control (24-dim state, 6-dim action): bench.py --algo sac
register("walker_walk_synthetic", "sheeprl_prey_amd.envs.synthetic:SyntheticControl", max_episode_steps=1000,
         obs_dim=24, act_dim=6)
