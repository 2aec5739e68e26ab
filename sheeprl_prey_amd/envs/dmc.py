"""DeepMind Control Suite adapter (reference ``sheeprl/envs/dmc.py:1-242``, after dmc2gym).

Observations: ``rgb`` (CHW uint8 render of ``camera_id``) and/or ``state`` (all task observations
flattened); actions are normalised to [-1, 1] and rescaled to the task's bounds."""
from __future__ import annotations

from typing import Any, Dict, Optional, Tuple

import numpy as np

from sheeprl_prey_amd.envs import spaces
from sheeprl_prey_amd.envs._gate import require
from sheeprl_prey_amd.envs.core import Env


def _spec_bounds(specs_list) -> Tuple[np.ndarray, np.ndarray]:
    lows, highs = [], []
    for s in specs_list:
        dim = int(np.prod(s.shape))
        if hasattr(s, "minimum"):
            lows.append(np.zeros(dim, np.float32) + s.minimum)
            highs.append(np.zeros(dim, np.float32) + s.maximum)
        else:
            lows.append(np.full(dim, -np.inf, np.float32))
            highs.append(np.full(dim, np.inf, np.float32))
    return np.concatenate(lows).astype(np.float32), np.concatenate(highs).astype(np.float32)


def _flatten_obs(obs: Dict[str, Any]) -> np.ndarray:
    return np.concatenate([np.array([v]) if np.isscalar(v) else np.asarray(v).ravel() for v in obs.values()], 0)


class DMCWrapper(Env):
    def __init__(self, id: str, from_pixels: bool = False, from_vectors: bool = False, height: int = 84,
                 width: int = 84, camera_id: int = 0, task_kwargs: Optional[Dict[str, Any]] = None,
                 environment_kwargs: Optional[Dict[str, Any]] = None, channels_first: bool = True,
                 visualize_reward: bool = False, seed: Optional[int] = None):
        suite = require("dm_control.suite", "Install dm_control + MuJoCo to use `env=dmc`.")
        if not from_pixels and not from_vectors:
            raise ValueError("'from_pixels' and 'from_vectors' cannot both be False")
        domain_name, task_name = id.split("_", 1)
        task_kwargs = dict(task_kwargs or {})
        if seed is not None:
            task_kwargs["random"] = seed
        self._from_pixels, self._from_vectors = from_pixels, from_vectors
        self._height, self._width, self._camera_id = height, width, camera_id
        self._channels_first = channels_first
        self._env = suite.load(domain_name=domain_name, task_name=task_name, task_kwargs=task_kwargs,
                               visualize_reward=visualize_reward, environment_kwargs=environment_kwargs)
        lo, hi = _spec_bounds([self._env.action_spec()])
        self._true_low, self._true_high = lo, hi
        self.action_space = spaces.Box(-1.0, 1.0, lo.shape, np.float32)
        rlo, rhi = _spec_bounds([self._env.reward_spec()])
        self.reward_range = (float(rlo[0]), float(rhi[0]))
        slo, shi = _spec_bounds(self._env.observation_spec().values())
        state_space = spaces.Box(slo, shi, slo.shape, np.float64)
        shape = (3, height, width) if channels_first else (height, width, 3)
        rgb_space = spaces.Box(0, 255, shape, np.uint8)
        if from_pixels and from_vectors:
            self.observation_space = spaces.Dict({"rgb": rgb_space, "state": state_space})
        elif from_vectors:
            self.observation_space = state_space
        else:
            self.observation_space = rgb_space
        self.state_space = state_space
        self.render_mode = "rgb_array"
        self.current_state = None
        self.action_space.seed(seed)

    def _get_obs(self, ts):
        rgb = None
        if self._from_pixels:
            rgb = self.render()
            if self._channels_first:
                rgb = rgb.transpose(2, 0, 1).copy()
        if self._from_vectors:
            vec = _flatten_obs(ts.observation)
            return {"rgb": rgb, "state": vec} if self._from_pixels else vec
        return rgb

    def step(self, action):
        a = np.asarray(action, dtype=np.float64)
        a = (a + 1.0) / 2.0 * (self._true_high - self._true_low) + self._true_low
        ts = self._env.step(a.astype(np.float32))
        self.current_state = _flatten_obs(ts.observation)
        info = {"discount": ts.discount, "internal_state": self._env.physics.get_state().copy()}
        return self._get_obs(ts), ts.reward or 0.0, ts.last(), False, info

    def reset(self, seed: Optional[int] = None, options: Optional[Dict[str, Any]] = None):
        ts = self._env.reset()
        self.current_state = _flatten_obs(ts.observation)
        return self._get_obs(ts), {}

    def render(self, camera_id: Optional[int] = None) -> np.ndarray:
        return self._env.physics.render(height=self._height, width=self._width,
                                        camera_id=self._camera_id if camera_id is None else camera_id)

    def close(self) -> None:
        self._env.close()
