"""Fake environments for tests (reference: ``sheeprl/envs/dummy.py:7-103``).

uint8 3x64x64 observations; continuous / discrete / multi-discrete actions; fixed lengths."""
from __future__ import annotations

from typing import List, Tuple

import numpy as np

from sheeprl_prey_amd.envs import spaces
from sheeprl_prey_amd.envs.core import Env


class _DummyBase(Env):
    def __init__(self, size: Tuple[int, int, int], n_steps: int, random_obs: bool):
        self.observation_space = spaces.Box(0, 256, shape=size, dtype=np.uint8)
        self.reward_range = (-np.inf, np.inf)
        self._current_step = 0
        self._n_steps = n_steps
        self._random_obs = random_obs

    def step(self, action):
        done = self._current_step == self._n_steps
        self._current_step += 1
        if self._random_obs:
            obs = np.random.randint(0, 256, self.observation_space.shape, dtype=np.uint8)
        else:
            obs = np.zeros(self.observation_space.shape, dtype=np.uint8)
        return obs, 0.0, done, False, {}

    def reset(self, seed=None, options=None):
        self._current_step = 0
        return np.zeros(self.observation_space.shape, dtype=np.uint8), {}

    def render(self, *args, **kwargs):
        return None

    def seed(self, seed=None):
        pass


class ContinuousDummyEnv(_DummyBase):
    def __init__(self, action_dim: int = 2, size: Tuple[int, int, int] = (3, 64, 64), n_steps: int = 128):
        super().__init__(size, n_steps, random_obs=False)
        self.action_space = spaces.Box(-1.0, 1.0, shape=(action_dim,))


class DiscreteDummyEnv(_DummyBase):
    def __init__(self, action_dim: int = 2, size: Tuple[int, int, int] = (3, 64, 64), n_steps: int = 4):
        super().__init__(size, n_steps, random_obs=True)
        self.action_space = spaces.Discrete(action_dim)


class MultiDiscreteDummyEnv(_DummyBase):
    def __init__(self, action_dims: List[int] = (2, 2), size: Tuple[int, int, int] = (3, 64, 64), n_steps: int = 128):
        super().__init__(size, n_steps, random_obs=False)
        self.action_space = spaces.MultiDiscrete(list(action_dims))
