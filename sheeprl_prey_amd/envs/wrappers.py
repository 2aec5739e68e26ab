"""Environment wrappers (reference: ``sheeprl/envs/wrappers.py:11-253``) + a video recorder."""
from __future__ import annotations

import copy
import os
import time
import warnings
from collections import deque
from typing import Any, Callable, Dict, List, Optional, Sequence, SupportsFloat, Tuple, Union

import numpy as np

from sheeprl_prey_amd.envs import spaces
from sheeprl_prey_amd.envs.core import Env, ObservationWrapper, Wrapper


class MaskVelocityWrapper(ObservationWrapper):
    """Zero the velocity terms of the observation (partially-observable MDP)."""

    velocity_indices = {
        "CartPole-v0": np.array([1, 3]),
        "CartPole-v1": np.array([1, 3]),
        "MountainCar-v0": np.array([1]),
        "MountainCarContinuous-v0": np.array([1]),
        "Pendulum-v1": np.array([2]),
        "LunarLander-v2": np.array([2, 3, 5]),
        "LunarLanderContinuous-v2": np.array([2, 3, 5]),
    }

    def __init__(self, env: Env):
        super().__init__(env)
        spec = env.unwrapped.spec or getattr(env, "spec", None)
        if spec is None:
            raise NotImplementedError("Velocity masking requires an env with a registered spec")
        self.mask = np.ones_like(env.observation_space.sample())
        try:
            self.mask[self.velocity_indices[spec.id]] = 0.0
        except KeyError as e:
            raise NotImplementedError(f"Velocity masking not implemented for {spec.id}") from e

    def observation(self, observation: np.ndarray) -> np.ndarray:
        return observation * self.mask


class ActionRepeat(Wrapper):
    def __init__(self, env: Env, amount: int = 1):
        super().__init__(env)
        if amount <= 0:
            raise ValueError("`amount` should be a positive integer")
        self._amount = amount

    @property
    def action_repeat(self) -> int:
        return self._amount

    def step(self, action):
        done = truncated = False
        total = 0.0
        i = 0
        obs, info = None, {}
        while i < self._amount and not (done or truncated):
            obs, reward, done, truncated, info = self.env.step(action)
            total += reward
            i += 1
        return obs, total, done, truncated, info


class RestartOnException(Wrapper):
    """Rebuild a crashed env (at most ``maxfails`` within ``window`` seconds); flags
    ``info["restart_on_exception"]`` so the caller can patch its buffers."""

    def __init__(self, env_fn: Callable[..., Env], exceptions=(Exception,), window: float = 300, maxfails: int = 2,
                 wait: float = 20):
        if not isinstance(exceptions, (tuple, list)):
            exceptions = [exceptions]
        self._env_fn = env_fn
        self._exceptions = tuple(exceptions)
        self._window = window
        self._maxfails = maxfails
        self._wait = wait
        self._last = time.time()
        self._fails = 0
        super().__init__(self._env_fn())

    def _restart(self, what: str, e: BaseException):
        if time.time() > self._last + self._window:
            self._last = time.time()
            self._fails = 1
        else:
            self._fails += 1
        if self._fails > self._maxfails:
            raise RuntimeError(f"The env crashed too many times: {self._fails}")
        warnings.warn(f"{what} - Restarting env after crash with {type(e).__name__}: {e}")
        time.sleep(self._wait)
        self.env = self._env_fn()
        new_obs, info = self.env.reset()
        info = dict(info)
        info["restart_on_exception"] = True
        return new_obs, info

    def step(self, action):
        try:
            return self.env.step(action)
        except self._exceptions as e:
            obs, info = self._restart("STEP", e)
            return obs, 0.0, False, False, info

    def reset(self, *, seed: Optional[int] = None, options: Optional[Dict[str, Any]] = None):
        try:
            return self.env.reset(seed=seed, options=options)
        except self._exceptions as e:
            return self._restart("RESET", e)


class FrameStack(Wrapper):
    """Stack the last ``num_stack`` frames (with ``dilation``) of every cnn key."""

    def __init__(self, env: Env, num_stack: int, cnn_keys: Sequence[str], dilation: int = 1) -> None:
        super().__init__(env)
        if num_stack <= 0:
            raise ValueError(f"Invalid value for num_stack, expected a value greater than zero, got {num_stack}")
        if not isinstance(env.observation_space, spaces.Dict):
            raise RuntimeError(f"Expected an observation space of type spaces.Dict, got: {type(env.observation_space)}")
        self._num_stack = num_stack
        self._cnn_keys: List[str] = []
        self._dilation = dilation
        self.observation_space = copy.deepcopy(self.env.observation_space)
        for k, v in self.env.observation_space.spaces.items():
            if cnn_keys and len(v.shape) == 3:
                self._cnn_keys.append(k)
                self.observation_space[k] = spaces.Box(
                    np.repeat(v.low[None, ...], num_stack, axis=0), np.repeat(v.high[None, ...], num_stack, axis=0),
                    (num_stack, *v.shape), v.dtype,
                )
        if not self._cnn_keys:
            raise RuntimeError("Specify at least one valid cnn key to be stacked")
        self._frames = {k: deque(maxlen=num_stack * dilation) for k in self._cnn_keys}

    def _get_obs(self, key):
        subset = list(self._frames[key])[self._dilation - 1 :: self._dilation]
        assert len(subset) == self._num_stack
        return np.stack(subset, axis=0)

    def step(self, action):
        obs, reward, done, truncated, infos = self.env.step(action)
        for k in self._cnn_keys:
            self._frames[k].append(obs[k])
            if (
                infos.get("env_domain") == "DIAMBRA"
                and {"round_done", "stage_done", "game_done"} <= set(infos.keys())
                and (infos["round_done"] or infos["stage_done"] or infos["game_done"])
                and not (done or truncated)
            ):
                for _ in range(self._num_stack * self._dilation - 1):
                    self._frames[k].append(obs[k])
            obs[k] = self._get_obs(k)
        return obs, reward, done, truncated, infos

    def reset(self, *, seed: Optional[int] = None, options: Optional[Dict[str, Any]] = None, **kwargs):
        obs, infos = self.env.reset(seed=seed, options=options)
        for k in self._cnn_keys:
            self._frames[k].clear()
            for _ in range(self._num_stack * self._dilation):
                self._frames[k].append(obs[k])
            obs[k] = self._get_obs(k)
        return obs, infos


class RewardAsObservationWrapper(Wrapper):
    """Adds the last reward to the observation dict under ``reward`` (Box(1,))."""

    def __init__(self, env: Env) -> None:
        super().__init__(env)
        rr = getattr(self.env, "reward_range", None) or (-np.inf, np.inf)
        reward_space = spaces.Box(*rr, (1,), np.float32)
        if isinstance(self.env.observation_space, spaces.Dict):
            self.observation_space = spaces.Dict({"reward": reward_space, **dict(self.env.observation_space.items())})
        else:
            self.observation_space = spaces.Dict({"obs": self.env.observation_space, "reward": reward_space})

    def _convert_obs(self, obs: Any, reward) -> Dict[str, Any]:
        reward_obs = (np.array(reward) if not isinstance(reward, np.ndarray) else reward).reshape(-1).astype(np.float32)
        if isinstance(obs, dict):
            obs["reward"] = reward_obs
            return obs
        return {"obs": obs, "reward": reward_obs}

    def step(self, action):
        obs, reward, done, truncated, infos = self.env.step(action)
        return self._convert_obs(obs, copy.deepcopy(reward)), reward, done, truncated, infos

    def reset(self, *, seed=None, options=None):
        obs, infos = self.env.reset(seed=seed, options=options)
        return self._convert_obs(obs, 0), infos


class GrayscaleRenderWrapper(Wrapper):
    def render(self):
        frame = super().render()
        if isinstance(frame, np.ndarray):
            if frame.ndim == 2:
                frame = frame[..., None]
            if frame.ndim == 3 and frame.shape[-1] == 1:
                frame = frame.repeat(3, axis=-1)
        return frame


class RecordVideo(Wrapper):
    """Record ``env.render()`` frames of every ``episode_trigger(ep)`` episode to an animated GIF
    (Pillow) or an ``.npy`` stack when Pillow is unavailable."""

    def __init__(self, env: Env, video_folder: str, episode_trigger: Optional[Callable[[int], bool]] = None, fps: int = 30,
                 name_prefix: str = "rl-video", **_ignored):
        super().__init__(env)
        self.video_folder = os.path.abspath(video_folder)
        os.makedirs(self.video_folder, exist_ok=True)
        self.episode_trigger = episode_trigger or (lambda ep: int(round(ep ** (1.0 / 3))) ** 3 == ep)
        self.frames_per_sec = fps
        self.name_prefix = name_prefix
        self.episode_id = 0
        self._frames: List[np.ndarray] = []
        self._recording = False

    def reset(self, *, seed=None, options=None):
        obs, info = self.env.reset(seed=seed, options=options)
        self._recording = self.episode_trigger(self.episode_id)
        self._frames = []
        self._capture()
        return obs, info

    def _capture(self):
        if self._recording:
            f = self.env.render()
            if isinstance(f, np.ndarray):
                self._frames.append(f)

    def step(self, action):
        obs, r, te, tr, info = self.env.step(action)
        self._capture()
        if te or tr:
            self._flush()
            self.episode_id += 1
        return obs, r, te, tr, info

    def _flush(self):
        if not self._recording or not self._frames:
            return
        path = os.path.join(self.video_folder, f"{self.name_prefix}-episode-{self.episode_id}")
        try:
            from PIL import Image

            imgs = [Image.fromarray(f.astype(np.uint8)) for f in self._frames]
            imgs[0].save(path + ".gif", save_all=True, append_images=imgs[1:], duration=int(1000 / self.frames_per_sec), loop=0)
        except Exception:
            np.save(path + ".npy", np.stack(self._frames))
        self._frames = []
        self._recording = False

    def close(self):
        self._flush()
        return super().close()
