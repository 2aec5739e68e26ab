"""Crafter adapter (reference ``sheeprl/envs/crafter.py:14-60``): ``rgb`` observation,
``Discrete`` actions; ``id`` is ``reward`` or ``nonreward``."""
from __future__ import annotations

from typing import Any, Dict, Optional, Tuple, Union

import numpy as np

from sheeprl_prey_amd.envs import spaces
from sheeprl_prey_amd.envs._gate import require
from sheeprl_prey_amd.envs.core import Env


class CrafterWrapper(Env):
    def __init__(self, id: str, screen_size: Union[int, Tuple[int, int]] = 64, seed: Optional[int] = None) -> None:
        crafter = require("crafter", "Install `crafter` to use `env=crafter`.")
        assert id in {"reward", "nonreward"}
        if isinstance(screen_size, int):
            screen_size = (screen_size,) * 2
        self._env = crafter.Env(size=screen_size, seed=seed, reward=(id == "reward"))
        os_ = self._env.observation_space
        self.observation_space = spaces.Dict({"rgb": spaces.Box(os_.low, os_.high, os_.shape, os_.dtype)})
        self.action_space = spaces.Discrete(self._env.action_space.n)
        self.reward_range = self._env.reward_range or (-np.inf, np.inf)
        self.observation_space.seed(seed)
        self.action_space.seed(seed)
        self.render_mode = "rgb_array"

    def step(self, action: Any):
        obs, reward, done, info = self._env.step(action)
        return {"rgb": obs}, reward, done, False, info

    def reset(self, *, seed: Optional[int] = None, options: Optional[Dict[str, Any]] = None):
        return {"rgb": self._env.reset()}, {}

    def render(self):
        return self._env.render()
