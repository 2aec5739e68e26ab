"""Env / Wrapper base classes with the gymnasium 0.29 step/reset contract:
``reset(seed=None, options=None) -> (obs, info)``,
``step(action) -> (obs, reward, terminated, truncated, info)``."""
from __future__ import annotations

from typing import Any, Callable, Dict, Optional, SupportsFloat, Tuple

import numpy as np

from sheeprl_prey_amd.envs import spaces


class EnvSpec:
    def __init__(self, id: str, entry_point: Any = None, max_episode_steps: Optional[int] = None, kwargs=None):
        self.id = id
        self.entry_point = entry_point
        self.max_episode_steps = max_episode_steps
        self.kwargs = kwargs or {}

    def __repr__(self):
        return f"EnvSpec({self.id})"


class Env:
    metadata: Dict[str, Any] = {"render_modes": []}
    render_mode: Optional[str] = None
    reward_range = (-float("inf"), float("inf"))
    spec: Optional[EnvSpec] = None
    action_space: spaces.Space
    observation_space: spaces.Space
    _np_random: Optional[np.random.Generator] = None

    @property
    def np_random(self) -> np.random.Generator:
        if self._np_random is None:
            self._np_random = np.random.default_rng()
        return self._np_random

    @np_random.setter
    def np_random(self, value):
        self._np_random = value

    def reset(self, *, seed: Optional[int] = None, options: Optional[Dict[str, Any]] = None) -> Tuple[Any, Dict[str, Any]]:
        if seed is not None:
            self._np_random = np.random.default_rng(seed)
        return None, {}

    def step(self, action) -> Tuple[Any, SupportsFloat, bool, bool, Dict[str, Any]]:
        raise NotImplementedError

    def render(self):
        return None

    def close(self) -> None:
        pass

    @property
    def unwrapped(self) -> "Env":
        return self

    def __enter__(self):
        return self

    def __exit__(self, *args):
        self.close()
        return False

    def __str__(self):
        return f"<{type(self).__name__}{'<' + self.spec.id + '>' if self.spec else ''}>"


class Wrapper(Env):
    def __init__(self, env: Env):
        self.env = env
        self._action_space: Optional[spaces.Space] = None
        self._observation_space: Optional[spaces.Space] = None
        self._metadata = None

    def __getattr__(self, name: str):
        if name.startswith("_"):
            raise AttributeError(f"accessing private attribute '{name}' is prohibited")
        return getattr(self.env, name)

    @property
    def spec(self):
        return self.env.spec

    @property
    def action_space(self):
        return self._action_space if self._action_space is not None else self.env.action_space

    @action_space.setter
    def action_space(self, space):
        self._action_space = space

    @property
    def observation_space(self):
        return self._observation_space if self._observation_space is not None else self.env.observation_space

    @observation_space.setter
    def observation_space(self, space):
        self._observation_space = space

    @property
    def metadata(self):
        return self._metadata if self._metadata is not None else self.env.metadata

    @metadata.setter
    def metadata(self, value):
        self._metadata = value

    @property
    def render_mode(self):
        return self.env.render_mode

    @property
    def reward_range(self):
        return self.env.reward_range

    @property
    def np_random(self):
        return self.env.np_random

    def step(self, action):
        return self.env.step(action)

    def reset(self, *, seed: Optional[int] = None, options: Optional[Dict[str, Any]] = None):
        return self.env.reset(seed=seed, options=options)

    def render(self):
        return self.env.render()

    def close(self):
        return self.env.close()

    @property
    def unwrapped(self) -> Env:
        return self.env.unwrapped

    def __str__(self):
        return f"<{type(self).__name__}{self.env}>"


class ObservationWrapper(Wrapper):
    def reset(self, *, seed=None, options=None):
        obs, info = self.env.reset(seed=seed, options=options)
        return self.observation(obs), info

    def step(self, action):
        obs, r, term, trunc, info = self.env.step(action)
        return self.observation(obs), r, term, trunc, info

    def observation(self, observation):
        raise NotImplementedError


class RewardWrapper(Wrapper):
    def step(self, action):
        obs, r, term, trunc, info = self.env.step(action)
        return obs, self.reward(r), term, trunc, info

    def reward(self, reward):
        raise NotImplementedError


class ActionWrapper(Wrapper):
    def step(self, action):
        return self.env.step(self.action(action))

    def action(self, action):
        raise NotImplementedError


class TransformObservation(ObservationWrapper):
    def __init__(self, env: Env, f: Callable[[Any], Any]):
        super().__init__(env)
        self.f = f

    def observation(self, observation):
        return self.f(observation)


class TimeLimit(Wrapper):
    def __init__(self, env: Env, max_episode_steps: int):
        super().__init__(env)
        self._max_episode_steps = max_episode_steps
        self._elapsed_steps = 0

    def step(self, action):
        obs, r, term, trunc, info = self.env.step(action)
        self._elapsed_steps += 1
        if self._elapsed_steps >= self._max_episode_steps:
            trunc = True
        return obs, r, term, trunc, info

    def reset(self, *, seed=None, options=None):
        self._elapsed_steps = 0
        return self.env.reset(seed=seed, options=options)


class RecordEpisodeStatistics(Wrapper):
    """Adds ``info["episode"] = {"r", "l", "t"}`` at episode end (gymnasium semantics)."""

    def __init__(self, env: Env, deque_size: int = 100):
        super().__init__(env)
        import time
        from collections import deque

        self._time = time.perf_counter
        self.episode_return = 0.0
        self.episode_length = 0
        self.episode_start = self._time()
        self.return_queue = deque(maxlen=deque_size)
        self.length_queue = deque(maxlen=deque_size)

    def reset(self, *, seed=None, options=None):
        obs, info = self.env.reset(seed=seed, options=options)
        self.episode_return = 0.0
        self.episode_length = 0
        self.episode_start = self._time()
        return obs, info

    def step(self, action):
        obs, r, term, trunc, info = self.env.step(action)
        self.episode_return += float(np.asarray(r).sum())
        self.episode_length += 1
        if term or trunc:
            info = dict(info)
            info["episode"] = {
                "r": np.array([self.episode_return], dtype=np.float32),
                "l": np.array([self.episode_length], dtype=np.int32),
                "t": np.array([round(self._time() - self.episode_start, 6)], dtype=np.float32),
            }
            self.return_queue.append(self.episode_return)
            self.length_queue.append(self.episode_length)
        return obs, r, term, trunc, info


class PixelObservationWrapper(ObservationWrapper):
    """Replace/augment the observation with ``env.render()`` (render_mode rgb_array)."""

    def __init__(self, env: Env, pixels_only: bool = True, pixel_keys=("pixels",), state_key: str = "state"):
        super().__init__(env)
        self._pixels_only = pixels_only
        self._pixel_key = pixel_keys[0]
        self._state_key = state_key
        frame = self._render_frame(reset=True)
        space = {}
        if not pixels_only:
            space[state_key] = env.observation_space
        space[self._pixel_key] = spaces.Box(0, 255, frame.shape, np.uint8)
        self.observation_space = spaces.Dict(space)

    def _render_frame(self, reset: bool = False):
        if reset:
            self.env.reset()
        frame = self.env.render()
        if frame is None:
            raise RuntimeError("PixelObservationWrapper requires render_mode='rgb_array'")
        return np.asarray(frame, dtype=np.uint8)

    def observation(self, observation):
        out = {}
        if not self._pixels_only:
            out[self._state_key] = observation
        out[self._pixel_key] = self._render_frame()
        return out
