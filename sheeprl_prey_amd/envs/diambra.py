"""DIAMBRA Arena adapter (reference ``sheeprl/envs/diambra.py:16-134``): one player, flattened
observation dict (Discrete / MultiDiscrete entries become int Boxes), frame shape applied by the
engine (``increase_performance``) or by DIAMBRA's wrappers."""
from __future__ import annotations

import warnings
from typing import Any, Dict, Optional, Tuple, Union

import numpy as np

from sheeprl_prey_amd.envs import spaces
from sheeprl_prey_amd.envs._gate import require
from sheeprl_prey_amd.envs.core import Env


class DiambraWrapper(Env):
    def __init__(self, id: str, action_space: str = "discrete", screen_size: Union[int, Tuple[int, int]] = 64,
                 grayscale: bool = False, repeat_action: int = 1, rank: int = 0,
                 diambra_settings: Optional[Dict[str, Any]] = None, diambra_wrappers: Optional[Dict[str, Any]] = None,
                 render_mode: str = "rgb_array", log_level: int = 0, increase_performance: bool = True) -> None:
        require("diambra", "Install `diambra` and `diambra-arena` to use `env=diambra`.")
        arena = require("diambra.arena", "Install `diambra-arena` to use `env=diambra`.")
        settings_in = dict(diambra_settings or {})
        wrappers_in = dict(diambra_wrappers or {})
        if isinstance(screen_size, int):
            screen_size = (screen_size,) * 2
        for k in ("frame_shape", "n_players"):
            if settings_in.pop(k, None) is not None:
                warnings.warn(f"The DIAMBRA {k} setting is disabled")
        role = settings_in.pop("role", None)
        space_type = getattr(arena.SpaceTypes, action_space.split(".")[-1].upper())
        settings = arena.EnvironmentSettings(**settings_in, game_id=id, action_space=space_type, n_players=1,
                                             role=getattr(arena.Roles, role.split(".")[-1]) if role else None,
                                             render_mode=render_mode)
        if repeat_action > 1:
            if getattr(settings, "step_ratio", 1) > 1:
                warnings.warn(f"step_ratio parameter modified to 1 because the sticky action is active ({repeat_action})")
            settings.step_ratio = 1
        for k in ("frame_shape", "stack_frames", "dilation", "flatten"):
            if wrappers_in.pop(k, None) is not None:
                warnings.warn(f"The DIAMBRA {k} wrapper is disabled")
        wrappers = arena.WrappersSettings(**wrappers_in, flatten=True, repeat_action=repeat_action)
        if increase_performance:
            settings.frame_shape = tuple(screen_size) + (int(grayscale),)
        else:
            wrappers.frame_shape = tuple(screen_size) + (int(grayscale),)
        self._env = arena.make(id, settings, wrappers, rank=rank, render_mode=render_mode, log_level=log_level)
        self.action_space = spaces.from_external(self._env.action_space)
        obs = {}
        for k, s in self._env.observation_space.spaces.items():
            kind = type(s).__name__
            if kind == "Discrete":
                obs[k] = spaces.Box(0, s.n - 1, (1,), np.int32)
            elif kind == "MultiDiscrete":
                nvec = np.asarray(s.nvec)
                obs[k] = spaces.Box(np.zeros_like(nvec), nvec - 1, (len(nvec),), np.int32)
            elif kind == "Box":
                obs[k] = spaces.from_external(s)
            else:
                raise RuntimeError(f"Invalid observation space, got: {kind}")
        self.observation_space = spaces.Dict(obs)
        self.render_mode = render_mode

    def _convert_obs(self, obs: Dict[str, Any]) -> Dict[str, np.ndarray]:
        return {k: np.asarray(v).reshape(self.observation_space[k].shape) for k, v in obs.items()}

    def step(self, action: Any):
        obs, reward, done, truncated, infos = self._env.step(action)
        infos["env_domain"] = "DIAMBRA"
        return self._convert_obs(obs), reward, done or infos.get("env_done", False), truncated, infos

    def reset(self, *, seed: Optional[int] = None, options: Optional[Dict[str, Any]] = None):
        obs, infos = self._env.reset(seed=seed, options=options)
        infos["env_domain"] = "DIAMBRA"
        return self._convert_obs(obs), infos

    def render(self, mode: str = "rgb_array", **kwargs):
        return self._env.render()

    def close(self) -> None:
        self._env.close()
